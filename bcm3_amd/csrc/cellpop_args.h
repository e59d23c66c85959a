// cellpop_args.h -- argument block of cp_solve_kernel (cellpop_solver.h), shared by the run-time
// compiled kernel and the host launcher (cellpop_rt.cpp), so both see one layout.
#pragma once
#include <stdint.h>

namespace cpk {

// one stored integration point (ODESolverCVODE's CVodeTimepoint, .cpp:375-401): cvode_time, tn, h,
// hu, q, then the Nordsieck rows zn[0..qmax] of the nstore species the data read. One definition
// for the kernel (CP_REC, cellpop_solver.h, with qmax = QMAX) and the host that sizes the store.
constexpr int cp_record_doubles(int qmax, int nstore) { return 5 + (qmax + 1) * (nstore > 0 ? nstore : 1); }
constexpr int CP_STORE_QMAX = 5;  // = QMAX of bdf_lane.h (static_assert in cellpop_solver.h)

struct CpSolveArgs {
    const int32_t* work;          // [n_work] cell slots of this launch
    int32_t n_work;
    int32_t M;                    // output entries (sorted simulation time points) = CP_M
    const double* output_times;   // [M] experiment times
    const int32_t* output_species;  // [M] ODE species index or -1
    const double* params;         // [slot][NP] cell-specific transformed variables
    const double* y0;             // [slot][NS]
    const double* creation;       // [slot]
    const double* constant_species;  // [NC]
    double end_time;              // Experiment target time
    double rtol, atol, hmin;
    int32_t max_steps;
    int32_t divide_cells;
    double past_cs;               // simulate_past_chromatid_separation_time
    int32_t ev[7];                // event species (simulated-species index applied to the ODE state), -1 = none
    const double* treat_times;    // pulse start times of the treatment trajectories, concatenated (CP_NTREAT)
    const int32_t* treat_offset;  // [CP_NTREAT + 1]
    // outputs
    double* out_values;           // [slot][M]
    double* end_y;                // [slot][NS]
    double* sim_end;              // [slot] cell time
    double* achieved;             // [slot] experiment time
    int32_t* flags;               // [slot] bit0 ok, bit1 divided, bit2 died, bit3 entered mitosis
    double* event_times;          // [slot][5]
    int32_t* nsteps;              // [slot]
    // stored integration points (CP_STORED builds, synchronised data): per work item of the launch
    // store_cap records of CP_REC doubles (ODESolverCVODE's CVodeTimepoint: time, tn, h, hu, q,
    // zn[0..q] of the stored species -- needed only during the cell's own solve, whose evaluation
    // passes read them back before it ends); the sync pass of every output entry; the
    // synchronisation offset per slot
    double* store;
    int32_t store_cap;
    const int32_t* output_sync;   // [M] BCM3HIP_CP_SYNC_*
    const double* sync_offset;    // [slot]
    double hmax;                  // DP5's max_dt (solver_max_timestep)
    const void* pow_tables;       // xm::GlibcPow (libm_exact.h): glibc's pow for DP5's step-size factor
};

// The cell work queue of CP_QUEUE builds (cellpop_solver.h cp_queue_kernel, cellpop_rt.cpp): the
// reference simulates a mother's daughters from a queue as soon as it divides (Experiment.cpp:691-782);
// here every wavefront of one persistent launch takes the next cells from the queue and enqueues the
// daughters of the cells it ends. Items are indexed by queue position (qi); the FIFO numbering of the
// reference is restored afterwards (cp_number_kernel), so every sum runs in the reference's cell order.
struct CpQueueItem {
    int32_t slot, eval, parent, sobol_ix, is_initial;  // = bcm3hip::CpInitItem (slot = qi)
};
struct CpQueueArgs {
    CpQueueItem* items;      // [cap]
    int32_t* ready;          // [cap] 1 once the item is written (initial cells: preset)
    int32_t* counters;       // [6] head (next item to take), tail (items reserved), outstanding (items
                             //     not finished), error (a bounded wait ran out)
    int32_t* child_qi;       // [cap][2] queue indices of the daughters (-1)
    int32_t* ncells_eval;    // [n] cells of each evaluation (initial cells + daughters enqueued)
    int32_t* failed_eval;    // [n] a cell failed or a limit was hit: the evaluation is -inf
    double* creation;        // [cap] the cells' creation times (written by the queue's initialisation)
    const double* values;    // [n][d]
    int32_t cap, n0, max_cells, sobol_points, sobol_dims;
    int64_t idle_limit;      // wall-clock ticks a wavefront may find nothing ready before the launch fails
};

}  // namespace cpk
