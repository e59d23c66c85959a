// expm_ref.cpp -- TEST INFRASTRUCTURE (oracle/_ref/libexpmref.so): the matrix exponential and the
// dose-to-dose solve of the pharmaco_single path computed by the reference's own vendored Eigen
// (dependencies/eigen-3.4-rc1: MatrixBase::exp from unsupported/Eigen/MatrixFunctions,
// Eigen::MatrixXd products), compiled from those headers where they lie under /root/reference.
// The loop is a restatement of PharmacokineticModel::Solve (src/pharmaco/PharmacokineticModel.cpp:
// 111-177) on Eigen types; only oracle/expm_pk.py loads this library.
#include <cmath>

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
}
