// oracle/mixture_ref.cpp -- TEST INFRASTRUCTURE (checker only; never linked into the product).
//
// The reference's mixture test likelihoods over the reference's own vendored Eigen
// (dependencies/eigen-3.4-rc1, included where it lies by oracle/Makefile -> _ref/libmixref.so):
//   dmvnormal  src/stats/mvn.cpp:9-33     Eigen::LLT, log-det from L's diagonal, L.solveInPlace
//   dmvt       src/stats/mvt.cpp:119-157  same factorisation; p = 1 through LogPdfT
//   LogPdfT    src/utils/ProbabilityDistributions.cpp:159-180 (the (x - mu) * sigma form;
//              boost::math::beta and log1p replaced by the lgamma form and std::log1p: Boost
//              is absent, so that constant's last bits are unpinned)
//   logsum     src/utils/MathFunctions.h:67-82
//   TestLikelihoodMultimodalGaussians::EvaluateLogProbability (TestLikelihoodMultimodalGaussians.cpp:36-42)
//   TestLikelihoodTruncatedT::EvaluateLogProbability          (TestLikelihoodTruncatedT.cpp:81-90)
// The statements are restated (not copied) in the order the reference evaluates them.
#include <Eigen/Dense>
#include <cmath>
#include <limits>

typedef Eigen::VectorXd VectorReal;
typedef Eigen::MatrixXd MatrixReal;

static double logsum(double loga, double logb)
{
    if (logb > loga) std::swap(loga, logb);
    if (loga == -std::numeric_limits<double>::infinity()) return loga;
    const double diff = logb - loga;
    if (diff < -500) return loga;
    return loga + std::log1p(std::exp(diff));
}

static double log_pdf_normal(double x, double mu, double sigma)
{
    const double two_sigma_sq = 2.0 * sigma * sigma;
    const double d = x - mu;
    return -std::log(sigma) - 0.91893853320467274178032973640562 - d * d / two_sigma_sq;
}

static double log_pdf_t(double x, double mu, double sigma, double nu)
{
    if (nu > 1e10) return log_pdf_normal(x, mu, sigma);
    const double xn = (x - mu) * sigma;
    const double basem1 = xn * xn / nu;
    if (basem1 == std::numeric_limits<double>::infinity()) return -std::numeric_limits<double>::infinity();
    const double result = -0.5 * (nu + 1.0) * std::log1p(basem1);
    const double beta = std::exp(std::lgamma(nu / 2.0) + std::lgamma(0.5) - std::lgamma(nu / 2.0 + 0.5));
    const double logC = -std::log(sigma * std::sqrt(nu) * beta);
    return logC + result;
}

static double dmvnormal_log(const VectorReal& x, const VectorReal& mu, const MatrixReal& sigma)
{
    const int p = (int)mu.size();
    Eigen::LLT<MatrixReal> llt;
    llt.compute(sigma);
    double det = 0.0;
    for (int i = 0; i < p; i++) det += std::log(llt.matrixL()(i, i));
    const double logC = -det - 0.5 * p * std::log(2.0 * M_PI);
    VectorReal v = x - mu;
    llt.matrixL().solveInPlace(v);
    return logC - 0.5 * v.dot(v);
}

static double dmvt_log(const VectorReal& x, const VectorReal& mu, const MatrixReal& sigma, double nu)
{
    const int p = (int)mu.size();
    if (p == 1) return log_pdf_t(x(0), mu(0), sigma(0, 0), nu);
    Eigen::LLT<MatrixReal> llt;
    llt.compute(sigma);
    double det = 0.0;
    for (int i = 0; i < p; i++) det += std::log(llt.matrixL()(i, i));
    const double logC = std::lgamma(0.5 * (p + nu)) - (std::lgamma(0.5 * nu) + det + 0.5 * p * std::log(M_PI * nu));
    VectorReal v = x - mu;
    llt.matrixL().solveInPlace(v);
    return logC - 0.5 * (p + nu) * std::log1p(v.dot(v) / nu);
}

static MatrixReal mat(int d, const double* rowmajor)
{
    MatrixReal m(d, d);
    for (int i = 0; i < d; i++)
        for (int j = 0; j < d; j++) m(i, j) = rowmajor[i * d + j];
    return m;
}

extern "C" {

double mixref_dmvnormal(int d, const double* x, const double* mu, const double* sigma)
{
    return dmvnormal_log(Eigen::Map<const VectorReal>(x, d), Eigen::Map<const VectorReal>(mu, d), mat(d, sigma));
}

double mixref_dmvt(int d, const double* x, const double* mu, const double* sigma, double nu)
{
    return dmvt_log(Eigen::Map<const VectorReal>(x, d), Eigen::Map<const VectorReal>(mu, d), mat(d, sigma), nu);
}

// kind 1: TestLikelihoodMultimodalGaussians (K = 2, d = 2, its fixed components, weights 0.5)
// kind 2: TestLikelihoodTruncatedT (weights as given in the XML; normalised here as Initialize does)
void mixref_eval(int kind, int d, int K, const double* weights, const double* means, const double* covs,
                 const double* nus, long n, const double* x, double* logp)
{
    VectorReal w(K);
    for (int k = 0; k < K; k++) w(k) = weights[k];
    if (kind == 2) w.array() /= w.sum();
    for (long e = 0; e < n; e++) {
        const Eigen::Map<const VectorReal> xv(x + e * d, d);
        if (kind == 1) {
            const double logp1 = std::log(0.5) + dmvnormal_log(xv, Eigen::Map<const VectorReal>(means, d), mat(d, covs));
            const double logp2 =
                std::log(0.5) + dmvnormal_log(xv, Eigen::Map<const VectorReal>(means + d, d), mat(d, covs + d * d));
            logp[e] = logsum(logp1, logp2);
        } else {
            double lp = -std::numeric_limits<double>::infinity();
            for (int k = 0; k < K; k++) {
                const double thislogp =
                    dmvt_log(xv, Eigen::Map<const VectorReal>(means + k * d, d), mat(d, covs + k * d * d), nus[k]);
                lp = logsum(lp, thislogp + std::log(w(k)));
            }
            logp[e] = lp;
        }
    }
}

}  // extern "C"
