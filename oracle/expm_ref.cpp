// expm_ref.cpp -- TEST INFRASTRUCTURE (oracle/_ref/libexpmref.so): the matrix exponential and the
// dose-to-dose solve of the pharmaco_single path computed by the reference's own vendored Eigen
// (dependencies/eigen-3.4-rc1: MatrixBase::exp from unsupported/Eigen/MatrixFunctions,
// Eigen::MatrixXd products), compiled from those headers where they lie under /root/reference.
// The loop is a restatement of PharmacokineticModel::Solve (src/pharmaco/PharmacokineticModel.cpp:
// 111-177) on Eigen types; only oracle/expm_pk.py loads this library.
#include <cmath>
#include <thread>
#include <vector>

#include <Eigen/Dense>
#include <unsupported/Eigen/MatrixFunctions>

using Mat = Eigen::MatrixXd;
using Vec = Eigen::VectorXd;

extern "C" {

// out = exp(A), both n x n column-major
int eigen_expm(int n, const double* a, double* out)
{
    Eigen::Map<const Mat> A(a, n, n);
    Mat tmp1 = A;
    Mat tmp2 = tmp1.exp();
    Eigen::Map<Mat>(out, n, n) = tmp2;
    return 0;
}

// central[n_obs]: compartment 1 at the observation times; returns 1 if the state stayed finite
int eigen_pk_solve(int n, const double* a, int n_treat, const double* treat_times, const double* treat_doses,
                   int n_obs, const double* obs_times, double* central)
{
    Eigen::Map<const Mat> A(a, n, n);
    Mat tmp1(n, n), tmp2(n, n);
    Vec y = Vec::Zero(n), tmp_y(n);
    const double simulate_until = obs_times[n_obs - 1];
    int tti = 0, oti = 0;
    double t = 0.0;
    while (tti < n_treat && t < simulate_until) {
        const double target = (tti < n_treat - 1) ? treat_times[tti + 1] : simulate_until;
        y(0) += treat_doses[tti] * 1.0;
        while (oti < n_obs && obs_times[oti] <= target) {
            tmp1.noalias() = A * (obs_times[oti] - t);
            tmp2.noalias() = tmp1.exp();
            tmp_y = tmp2 * y;
            central[oti] = tmp_y(1);
            oti++;
        }
        tmp1.noalias() = A * (target - t);
        tmp2.noalias() = tmp1.exp();
        Vec next = tmp2 * y;
        for (int i = 0; i < n; i++)
            if (std::isnan(next(i))) return 0;
        y = next;
        t = target;
        tti++;
    }
    return 1;
}

// The reference's fan-out for the CPU baseline (bench.py): n_jobs solves (one evaluation's patient
// each) split over nthreads std::threads like TaskManager's one-task-per-chain workers. a_all is
// [n_jobs][n*n] column-major, job_patient[n_jobs] selects the patient's dose / observation time
// ranges (treat_off / obs_off, [P+1]); each job's doses (already scaled by its bioavailability)
// start at doses_all + dose_off[job], and its n_obs(patient) outputs at central_all + central_off[job].
// Returns the number of solves that stayed finite.
int eigen_pk_solve_batch(int nthreads, int n_jobs, int n, const double* a_all, const int* job_patient,
                         const int* treat_off, const double* treat_times, const double* doses_all,
                         const long long* dose_off, const int* obs_off, const double* obs_times,
                         const long long* central_off, double* central_all)
{
    std::vector<int> ok(n_jobs, 0);
    auto work = [&](int t) {
        for (int j = t; j < n_jobs; j += nthreads) {
            const int p = job_patient[j];
            ok[j] = eigen_pk_solve(n, a_all + (size_t)j * n * n, treat_off[p + 1] - treat_off[p],
                                   treat_times + treat_off[p], doses_all + dose_off[j],
                                   obs_off[p + 1] - obs_off[p], obs_times + obs_off[p],
                                   central_all + central_off[j]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    int n_ok = 0;
    for (int v : ok) n_ok += v;
    return n_ok;
}
}
