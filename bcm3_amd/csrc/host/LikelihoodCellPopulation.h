// LikelihoodCellPopulation.h -- likelihood type "cell_population" (CellPopulationLikelihood,
// src/cellpop/CellPopulationLikelihood.h) on the MI355X: the experiment description of
// Experiment::Load / PostInitialize (src/cellpop/Experiment.cpp:145-237, 404-633) is built here on
// the host; the cells are simulated by libbcm3hip's cell-population context (bcm3hip_open_cellpop:
// the per-model ODE kernel compiled with hipRTC, generation-by-generation division).
//
// Supported (the reference's options this path uses): one or more <experiment>s (their
// log-likelihoods summed in order, CellPopulationLikelihood.cpp:82-101), each with model_file, data_file
// (netCDF classic, or a JSON sidecar with the netCDF group's variables), num_cells, max_cells,
// divide_cells, entry_time, synchronization_time_offset, trailing_simulation_time,
// simulate_past_chromatid_separation_time,
// solver_* settings (solver_type CVODE or DP5); <set_parameter>; <cell_variability
// distribution="diagonal_gaussian">; <treatment_trajectory type="pulses">; <data> of type
// "time_course_population_average" or "time_course" (the default type; single cells matched to
// the simulated cells, observed lineages through "cell_id" / "parent"; synchronize= any of the reference's points, on stored
// integration points) with the normal / additive_normal /
// proportional_normal / additive_proportional_normal / student_t4 error models, stdev /
// proportional_stdev / offset / scale / stdev_relative_to_scale / weight / relative_to_time_average /
// missing_simulation_time_stdev, and the cellpop.use_only_cell_ix option; <data type="time_points">
// (DataLikelihoodTimePoints: cells matched at every time point, ";"-separated species columns, "+"
// sums, 2-D or 3-D data, value_relative_to_timepoint_ix, use_only_nondivided; normal / student_t4).
// Not built: the duration likelihood (the reference's reads past its matrix), DP5 with treatment
// trajectories, non-sampled parameters.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "LikelihoodGPU.h"
#include "SBMLModel.h"

namespace bcm3 {

struct Json;

class LikelihoodCellPopulation : public LikelihoodGPUBase {
public:
    LikelihoodCellPopulation(size_t sampling_threads, size_t evaluation_threads);
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override;

    const std::string& GetGeneratedCode() const { return derivative_body; }
    const bcm3hip_cellpop_model& GetDeviceModel() const { return model; }
    // every experiment's device model, in <experiment> order
    std::vector<const bcm3hip_cellpop_model*> GetDeviceModels() const;

private:
    struct DataLikelihood {
        std::string data_name, species_name;
        int32_t species_ix = -1;
        std::vector<double> times;
        std::vector<double> observed;  // [R][T]
        int32_t R = 0;
        bcm3hip_value_ref stdev{}, offset{}, scale{}, proportional_stdev{};
        double weight = 1.0;
        int32_t error_model = 0;
        int32_t relative_to_time_average = 0;
        int32_t kind = BCM3HIP_CP_DATA_POPULATION_AVERAGE, stdev_relative_to_scale = 0;
        int32_t sync = BCM3HIP_CP_SYNC_NONE;  // synchronize (BCM3HIP_CP_SYNC_*)
        bcm3hip_value_ref missing_stdev{};
        std::vector<int32_t> entry;
        // time points (DataLikelihoodTimePoints): observed [R][T][MK]; column l sums the species
        // term_species[term_offset[l] .. term_offset[l+1]); the species registered for simulation in
        // first-use order (species_order), their entries per time point (term_entry[k][T])
        int32_t L = 0, MK = 0, relative_ix = -1, only_nondivided = 0;
        std::vector<int32_t> term_offset, term_species, species_order, term_entry;
        std::vector<bcm3hip_value_ref> col_ref;  // [3L] stdev, offset, scale
        // observed lineage (time courses): roots in data order, children ascending (CSR)
        std::vector<int32_t> roots, child_off, child_ix;
    };
    bool LoadExperiment(const XmlNode& ex, const OptionsMap& vm);
    bool LoadTimePoints(const XmlNode& dn, DataLikelihood& d, const Json& group, const OptionsMap& vm) const;
    bool ParseRef(const std::string& s, bcm3hip_value_ref& r) const;

    SBMLModel sbml;
    std::string name, derivative_body;
    std::map<std::string, double> forced;
    double rtol = 0, atol = 0, hmin = 0;
    int32_t max_steps = 10000, num_cells = 1, max_cells = 20;
    int32_t solver = BCM3HIP_CP_SOLVER_CVODE;  // solver_type
    double hmax = 0.0;                         // solver_max_timestep (DP5's max_dt)
    bool divide_cells = true;
    double trailing = 0, past_cs = 0;
    bcm3hip_value_ref entry_time{}, sync_offset{};
    struct VarVariable {
        std::string species, parameter;
        bool entry_time = false, negate = false, only_initial = false;
        int32_t apply = 0;
        bcm3hip_value_ref scale{};
    };
    std::vector<std::vector<VarVariable>> variabilities;
    // per variability: full_gaussian (VariabilityDescription.cpp:184-212) and its covariance references
    // b<j+1>_<i+1>, j < i, in the reference's order
    std::vector<int> variability_full;
    std::vector<std::vector<bcm3hip_value_ref>> variability_cov;
    std::vector<int32_t> full_groups;
    std::vector<bcm3hip_value_ref> covariance;
    std::vector<DataLikelihood> data;

    // flat device model and its arrays
    std::vector<int32_t> transforms, output_species, output_sync, reset_index;
    std::vector<double> y_init, constant_init, output_times, reset_value, sobol;
    std::vector<bcm3hip_value_ref> scales;
    std::vector<bcm3hip_variability_action> actions;
    std::vector<bcm3hip_cellpop_data> data_flat;
    // <treatment_trajectory type="pulses">: constant-species index, pulse start times per trajectory
    std::vector<int32_t> treat_species, treat_offset{0};
    std::vector<double> treat_times;
    std::vector<std::string> treat_names;
    bcm3hip_cellpop_model model{};
    bool host_only = false;
    // the second and later <experiment>s (host-side descriptions; one device context sums them)
    std::vector<std::unique_ptr<LikelihoodCellPopulation>> more_experiments;
};

// boost::random::sobol (Joe & Kuo 2008 direction numbers, first point skipped) through
// uniform_01<double>: points x dims, row-major (VariabilityPseudoRandomIterator::Initialize)
std::vector<double> SobolPoints(size_t points, size_t dims);

}  // namespace bcm3
