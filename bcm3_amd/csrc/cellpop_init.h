// cellpop_init.h -- one new cell's parameters and initial state: Cell::Initialize (Cell.cpp:150-191)
// with CellPopulation::AddNewCell's initial conditions (CellPopulation.cpp:36-104): the model's initial
// amounts or the parent's end state with the daughter resets (Cell::SetInitialConditionsFromOtherCell,
// Cell.cpp:119-148), then the variabilities (VariabilityDescription::GetPseudorandomVector: diagonal
// gaussian QuantileNormal(sobol) * exp(scale), full gaussian L z; ApplyVariability*). Shared by
// cp_init_kernel (cellpop_kernels.hip, the generation launches and the initial cells) and the per-model
// cell kernel's work queue (cellpop_solver.h CP_QUEUE, the daughters as their mothers end), so both
// compute the same bits from one source.
#pragma once
#include "cellpop_static.h"
#include "pk_math.h"

namespace bcm3hip {

__device__ inline double cp_transform(int32_t tf, double x)
{
    // VariableSet::TransformVariable (src/sampler/VariableSet.cpp:97-124)
    switch (tf) {
    case BCM3HIP_TF_LOG: return exp(x);
    case BCM3HIP_TF_LOG10: return exp(x * 2.3025850929940459);  // bcm3::fastpow10
    case BCM3HIP_TF_LOGIT:
        if (x > 0) {
            const double z = exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            const double z = exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

__device__ inline double cp_ref(const bcm3hip_value_ref& r, const double* values, const int32_t* transforms, double none)
{
    if (r.kind == BCM3HIP_REF_VARIABLE) return cp_transform(transforms[r.index], values[r.index]);
    if (r.kind == BCM3HIP_REF_FIXED) return r.value;
    return none;
}

__device__ inline double cp_apply(int32_t kind, double x, double v)
{
    switch (kind) {
    case BCM3HIP_APPLY_ADDITIVE: return x + v;
    case BCM3HIP_APPLY_ADDITIVE_LOG: return x + exp(v);
    case BCM3HIP_APPLY_ADDITIVE_LOG2: return x + pow(2.0, v);
    case BCM3HIP_APPLY_MULTIPLICATIVE: return x * v;
    case BCM3HIP_APPLY_MULTIPLICATIVE_LOG: return x * exp(v);
    case BCM3HIP_APPLY_MULTIPLICATIVE_LOG2: return x * pow(2.0, v);
    default: return v;  // replace
    }
}



// the cell of item `it` into params[slot] / y0[slot] / creation[slot] (sync_off[slot] when given)
__device__ inline void cp_init_cell(const CpStatic& m, const CpInitItem& it, const double* values, double* params,
                                    double* y0, double* creation, const double* end_y, const double* achieved,
                                    double* sync_off)
{
    const double* v = values + (size_t)it.eval * m.d;
    // Experiment::EvaluateLogProbability's time_offset: the sampled value, before any cell
    // variability (Experiment.cpp:267-272)
    if (sync_off) sync_off[it.slot] = cp_ref(m.sync_offset, v, m.transforms, 0.0);
    double* prm = params + (size_t)it.slot * m.d;
    double* y = y0 + (size_t)it.slot * m.NS;
    for (int i = 0; i < m.d; i++) prm[i] = cp_transform(m.transforms[i], v[i]);
    if (it.parent < 0) {
        for (int i = 0; i < m.NS; i++) y[i] = m.y_init[i];
        creation[it.slot] = cp_ref(m.entry_time, v, m.transforms, 0.0);
    } else {
        const double* pe = end_y + (size_t)it.parent * m.NS;
        for (int i = 0; i < m.NS; i++) y[i] = pe[i];
        for (int r = 0; r < m.n_reset; r++) y[m.reset_index[r]] = m.reset_value[r];
        creation[it.slot] = achieved[it.parent];
    }
    if (m.sobol_dims == 0) return;
    // pseudorandom vector, diagonal gaussian (VariabilityDescription.cpp:60-67)
    // (the work queue's build sizes these by the model's Sobol dimensions, CP_INIT_DMAX: no scratch)
#ifdef CP_INIT_DMAX
    constexpr int DMAX = CP_INIT_DMAX;
#else
    constexpr int DMAX = 32;
#endif
    double pr[DMAX];
    const double* sob = m.sobol + (size_t)it.sobol_ix * m.sobol_dims;
    for (int k = 0; k < m.sobol_dims && k < DMAX; k++)
        pr[k] = quantile_normal(sob[k], 0.0, 1.0) * exp(cp_ref(m.scales[k], v, m.transforms, 0.0));
    // full gaussian groups (VariabilityDescription.cpp:69-128): z = QuantileNormal(sobol) and
    // L(i, j) = exp(scale_i) * prod_{k < i, k <= j} (k == j ? cos : sin)(cov(k, i) * pi), j <= i; the
    // vector is L z (Eigen's MatrixXd * VectorXd, summed over j in order)
    const bcm3hip_value_ref* cov = m.covariance;
    for (int g = 0; g < m.n_full; g++) {
        const int g0 = m.full_groups[2 * g], D = m.full_groups[2 * g + 1];
        double z[DMAX];
        for (int i = 0; i < D; i++) z[i] = quantile_normal(sob[g0 + i], 0.0, 1.0);
        for (int i = 0; i < D; i++) {
            const double exp_scale = exp(cp_ref(m.scales[g0 + i], v, m.transforms, 0.0));
            double acc = 0.0;
            for (int j = 0; j < D; j++) {
                double lij = 0.0;
                if (j <= i) {
                    lij = exp_scale;
                    for (int k = 0; k < i; k++) {
                        if (k <= j) {
                            const double cv = cp_ref(cov[(i - 1) * i / 2 + k], v, m.transforms, 0.0) * 3.14159265358979323846;  // M_PI
                            lij *= (k == j) ? cos(cv) : sin(cv);
                        }
                    }
                }
                acc = (j == 0) ? lij * z[0] : acc + lij * z[j];
            }
            pr[g0 + i] = acc;
        }
        cov += D * (D - 1) / 2;
    }
    for (int a = 0; a < m.n_actions; a++) {
        const bcm3hip_variability_action act = m.actions[a];
        if (act.only_initial_cells && !it.is_initial) continue;
        const double r = act.negate ? -pr[act.dim] : pr[act.dim];
        if (act.target_kind == 0)
            prm[act.target_index] = cp_apply(act.apply, prm[act.target_index], r);
        else
            y[act.target_index] = cp_apply(act.apply, y[act.target_index], r);
    }
}

}  // namespace bcm3hip
