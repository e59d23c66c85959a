// capi_proposal.cpp -- include/bcm3.h's proposal-adaptation entry points on top of GMM.cpp:
// SamplerPTChain::AdaptProposal (src/sampler/SamplerPTChain.cpp:120-178) for every chain of a
// rank, one std::thread per host core (the reference runs AsyncDoAdaptProposal as TaskManager
// tasks, one per chain).
#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../../include/bcm3.h"
#include "GMM.h"
#include "log.h"

extern "C" {

int bcm3_adapt_proposals(int kind, int adjusted_aic, int C, int H, int d, int kmax, const float* history,
                         const int64_t* counts, const uint8_t* active, size_t max_history_samples,
                         const double* prior_mean, const double* prior_var, uint64_t seed, uint64_t adaptation,
                         int64_t chain0, int nthreads, int32_t* ncomp, double* weights, double* means, double* chol,
                         double* logc, int32_t* fitted)
{
    if (C < 0 || H <= 0 || d <= 0 || kmax <= 0 || (kind != BCM3_PROPOSAL_GLOBAL_COVARIANCE &&
                                                   kind != BCM3_PROPOSAL_GAUSSIAN_MIXTURE))
        return -1;
    if (C > 0 && (!history || !counts || !prior_mean || !prior_var || !ncomp || !weights || !means || !chol ||
                  !logc))
        return -1;
    if (nthreads < 1) nthreads = 1;
    std::atomic<int> failed{0};
    auto work = [&](int t) {
        for (int c = t; c < C; c += nthreads) {
            if (active && !active[c]) continue;
            // SampleHistory::GetHistory: the first min(stored, H) ring slots, in slot order
            const int n = (int)std::min<int64_t>(counts[c], H);
            bcm3::Mat h(n, d);
            const float* src = history + (size_t)c * H * d;
            for (size_t i = 0; i < (size_t)n * d; i++) h.a[i] = (double)src[i];
            bcm3::CtrRng rng(seed, ((uint64_t)(chain0 + c) << 20) ^ adaptation);
            h = bcm3::ThinHistory(h, max_history_samples, rng);
            bcm3::ProposalFit fit;
            const bool ok = (kind == BCM3_PROPOSAL_GAUSSIAN_MIXTURE)
                                ? bcm3::FitGaussianMixtureProposal(h, adjusted_aic != 0, rng, prior_mean, prior_var,
                                                                   kmax, fit)
                                : bcm3::FitGlobalCovarianceProposal(h, prior_var, fit);
            if (!ok) {
                failed++;
                continue;
            }
            const int K = (kind == BCM3_PROPOSAL_GAUSSIAN_MIXTURE) ? kmax : 1;
            ncomp[c] = fit.ncomp;
            if (fitted) fitted[c] = fit.fitted ? 1 : 0;
            for (int k = 0; k < kmax; k++) {
                const bool have = k < K;
                weights[(size_t)c * kmax + k] = have ? fit.weights[k] : 0.0;
                logc[(size_t)c * kmax + k] = have ? fit.logc[k] : fit.logc[0];
                for (int i = 0; i < d; i++) means[((size_t)c * kmax + k) * d + i] = have ? fit.means[(size_t)k * d + i] : 0.0;
                for (int i = 0; i < d * d; i++)
                    chol[((size_t)c * kmax + k) * d * d + i] =
                        have ? fit.chol[(size_t)k * d * d + i] : ((i % (d + 1) == 0) ? 1.0 : 0.0);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (failed) {
        LOGERROR("proposal adaptation failed for %d chain(s) (Creation of GMM failed)", (int)failed);
        return -2;
    }
    return 0;
}

int bcm3_gmm_eval(int K, int d, const double* weights, const double* means, const double* covariances, int n,
                  const double* x, double* logpdf, double* resp, double* chol_out, double* logc_out)
{
    if (K <= 0 || d <= 0 || n < 0 || !weights || !means || !covariances || (n > 0 && !x)) return -1;
    std::vector<std::vector<double>> mu(K);
    std::vector<bcm3::Mat> cov(K, bcm3::Mat(d, d));
    for (int k = 0; k < K; k++) {
        mu[k].assign(means + (size_t)k * d, means + (size_t)(k + 1) * d);
        std::copy(covariances + (size_t)k * d * d, covariances + (size_t)(k + 1) * d * d, cov[k].a.begin());
    }
    bcm3::GMM g;
    if (!g.Set(mu, cov, std::vector<double>(weights, weights + K))) {
        LOGERROR("GMM::Set: a covariance is not positive definite");
        return -2;
    }
    for (int i = 0; i < n; i++) {
        if (logpdf) logpdf[i] = g.LogPdf(x + (size_t)i * d);
        if (resp) {
            const std::vector<double> r = g.CalculateResponsibilities(x + (size_t)i * d);
            std::copy(r.begin(), r.end(), resp + (size_t)i * K);
        }
    }
    for (int k = 0; k < K; k++) {
        if (chol_out) std::copy(g.GetCholesky(k).a.begin(), g.GetCholesky(k).a.end(), chol_out + (size_t)k * d * d);
        if (logc_out) logc_out[k] = g.GetLogC(k);
    }
    return 0;
}

}  // extern "C"
