// GMM.h -- the proposal adaptation of the device sampler, on the host:
//   * bcm3::GMM (src/stats/GMM.h, GMM.cpp): Set, Fit (k-means++ initialisation + EM with the
//     ESS-regularised covariance estimate), LogPdf, CalculateResponsibilities;
//   * Proposal::Initialize's history thinning (src/sampler/Proposal.cpp:92-129);
//   * ProposalGaussianMixture::InitializeImpl (src/sampler/ProposalGaussianMixture.cpp:125-254):
//     effective sample size from autocorrelations, GMMs with 1, 2, 3, 4, 5, 8, 13 components,
//     selection by (adjusted) AIC, fallback to the prior's moments;
//   * ProposalGlobalCovariance::InitializeImpl (src/sampler/ProposalGlobalCovariance.cpp:64-104).
// Eigen- and Boost-free: small row-major matrices, Cholesky (Eigen::LLT), a symmetric eigensolver
// (Householder tridiagonalisation + implicit QL, eigenvalues ascending as
// Eigen::SelfAdjointEigenSolver returns them). Random numbers come from a counter-based stream
// keyed by (seed, adaptation, chain), like every other random number of the device sampler (the
// reference's per-thread ranlux48 streams are clock-seeded).
// The device proposal kernels (proposal_kernels.hip) consume the fitted mixtures as Cholesky
// factors, means, weights and log normalisers.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace bcm3 {

using Real = double;

// dense row-major matrix
struct Mat {
    int rows = 0, cols = 0;
    std::vector<Real> a;
    Mat() = default;
    Mat(int r, int c, Real v = 0.0) : rows(r), cols(c), a((size_t)r * c, v) {}
    Real& operator()(int i, int j) { return a[(size_t)i * cols + j]; }
    Real operator()(int i, int j) const { return a[(size_t)i * cols + j]; }
    const Real* row(int i) const { return a.data() + (size_t)i * cols; }
};

// splitmix64 stream of (seed, key): the host counterpart of csrc/ctr_rng.h
class CtrRng {
public:
    CtrRng(uint64_t seed, uint64_t key);
    uint64_t Next();
    Real GetReal();                            // [0, 1), 53 bits (RNG::GetReal)
    unsigned GetUnsignedInt(unsigned max);     // uniform in [0, max] (RNG::GetUnsignedInt(max))
    unsigned Sample(const std::vector<Real>& probabilities);  // RNG::Sample (RNG.cpp:41-56)

private:
    uint64_t base_, n_;
};

// Eigen::LLT: lower-triangular L with A = L L^T; false if A is not positive definite
bool Cholesky(const Mat& A, Mat& L);
// symmetric eigendecomposition: eigenvalues ascending, eigenvectors in the columns of V
void SymmetricEigen(const Mat& A, std::vector<Real>& eval, Mat& V);
// MathFunctions.h:67-82
Real LogSum(Real loga, Real logb);

class GMM {
public:
    bool Set(const std::vector<std::vector<Real>>& means, const std::vector<Mat>& covariances,
             const std::vector<Real>& weights);
    bool Fit(const Mat& samples, size_t num_samples, size_t num_components, CtrRng& rng, Real ess_factor);

    Real LogPdf(const Real* x) const;
    std::vector<Real> CalculateResponsibilities(const Real* x) const;

    size_t GetNumComponents() const { return comps.size(); }
    const std::vector<Real>& GetWeights() const { return weights; }
    const std::vector<Real>& GetMean(size_t k) const { return comps[k].mean; }
    const Mat& GetCovariance(size_t k) const { return comps[k].cov; }
    const Mat& GetCholesky(size_t k) const { return comps[k].L; }
    Real GetLogC(size_t k) const { return comps[k].logC; }
    Real GetLogLikelihood() const { return full_logl; }
    Real GetAIC() const { return aic; }

private:
    struct Component {
        std::vector<Real> mean;
        Mat cov, L;
        Real logC = 0.0;
    };
    bool KMeanspp(const Mat& samples, size_t n, size_t K, CtrRng& rng, Mat& resp);
    void CalculateMeanCovariance(const Mat& samples, size_t n, const Mat& resp, int col, std::vector<Real>& mean,
                                 Mat& cov, Real ess_factor) const;
    void EM_maximization(const Mat& samples, size_t n, const Mat& resp, Real ess_factor);
    bool EM_expectation(const Mat& samples, size_t n, Mat& resp, Real& logl);
    Real LogPdfMVN(const Real* x, const Component& c) const;

    std::vector<Real> weights;
    std::vector<Component> comps;
    Real full_logl = 0.0 / 0.0;
    Real aic = 0.0 / 0.0;
};

// one chain's adapted proposal: K components, arrays sized for kmax (unused slots: weight 0,
// mean 0, identity factor)
struct ProposalFit {
    int ncomp = 0;
    bool fitted = false;  // false: the prior-moments fallback
    std::vector<Real> weights, means, chol, logc;
};

// Proposal::Initialize's reduction of the history to max_samples rows (Proposal.cpp:92-121)
Mat ThinHistory(const Mat& history, size_t max_samples, CtrRng& rng);
// ProposalGaussianMixture::InitializeImpl (ProposalGaussianMixture.cpp:125-254)
bool FitGaussianMixtureProposal(const Mat& history, bool select_with_adjusted_aic, CtrRng& rng,
                                const Real* prior_mean, const Real* prior_var, int kmax, ProposalFit& out);
// ProposalGlobalCovariance::InitializeImpl (ProposalGlobalCovariance.cpp:64-104)
bool FitGlobalCovarianceProposal(const Mat& history, const Real* prior_var, ProposalFit& out);

}  // namespace bcm3
