// SamplerPTDevice.h -- the PT-MH sampler loop of one rank in C++ (SamplerPT::Initialize / Run /
// DoExchangeMove / DoMutateMove, src/sampler/SamplerPT.cpp:97-319, with SamplerPTChain's
// MutateMove / ExchangeMove / AdaptProposal, src/sampler/SamplerPTChain.cpp:120-381), driving the
// MI355X kernels through include/bcm3hip.h. The rank owns a contiguous slice of the temperature
// ladder; all chain state stays in HBM; one batched likelihood launch per mutate step
// (bcm3::Likelihood::EvaluateLogProbabilityBatchDevice); the PT swap of slice-boundary pairs goes
// over a Transport (RCCL between processes, or an in-process transport for tests).
// Counter-based random numbers make a run independent of the number of ranks: the same seed gives
// the same chains on 1, 2, 4 or 8 GPUs, and the same chains as bcm3_amd.sampler.PTMHDevice.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "Likelihood.h"
#include "Prior.h"

namespace bcm3 {

// moves of one {values[d], llh, lprior, lpp, T} record per message between ranks
class Transport {
public:
    virtual ~Transport() = default;
    // sends[i] -> send_peer[i], recvs[j] <- recv_peer[j]; count doubles each; device buffers on
    // `stream`; messages between one pair of ranks match in posting order
    virtual bool Exchange(int n_send, const double* const* sends, const int* send_peer, int n_recv,
                          double* const* recvs, const int* recv_peer, size_t count, void* stream) = 0;
};

std::unique_ptr<Transport> MakeRcclTransport(const void* nccl_id, int rank, int world);

// between OS processes on one host (e.g. several ranks sharing one GPU, which RCCL refuses):
// host-staged records over Unix domain sockets under `dir` (SocketTransport.cpp)
std::unique_ptr<Transport> MakeSocketTransport(const std::string& dir, int rank, int world);

// in-process transport between the ranks of one process (one host thread per rank): host-staged
// mailboxes, for tests of the sharded exchange on one GPU
class LocalGroup;
std::shared_ptr<LocalGroup> MakeLocalGroup(int world);
std::unique_ptr<Transport> MakeLocalTransport(std::shared_ptr<LocalGroup> group, int rank);

struct PTMHConfig {
    int64_t num_chains = 256;  // over all ranks (ptmhsampler.num_chains)
    int rank = 0, world = 1;
    double temperature_power = 3.0, temperature_max = 1.0;
    uint64_t seed = 0;
    double learning_rate = 1.0;
    int exploration_steps = 1;
    int proposal = 1;  // 0 global_covariance, 1 gaussian_mixture, 2 gaussian_mixture_adjustedAIC, 3 random_walk
    double t_dof = 0.0;
    int kmax = 0;  // 0: 13 for the mixtures, 1 otherwise
    int adapt_proposal_samples = 2000, adapt_proposal_times = 2;
    int max_history_size = 2000, adapt_proposal_max_history_samples = 2000, use_every_nth = 1;
    int swapping_scheme = 0;  // 0 deterministic_even_odd, 1 stochastic_even_odd, 2 stochastic_random
    double exchange_probability = 0.5;
    int initial_position_tries = 100;
    int nan_check_every = 100;
    int host_threads = 0;  // proposal adaptation threads, 0 = hardware concurrency (max 16)
    // speculative iteration pairs: iteration r's likelihood launch also evaluates every proposal
    // iteration r + 1 can make (own / exchange partner's state, accepted or not), so the pair needs
    // one launch; bit-identical results. Used when the likelihood supports counted device batches
    // (the PopPK kernel), one rank, deterministic_even_odd, one exploration step, adaptive proposals.
    int speculate = 1;
};

struct PTMHCounters {
    int64_t attempted_mutate = 0, accepted_mutate = 0, attempted_exchange = 0, accepted_exchange = 0;
    int64_t samples_done = 0, adaptations_done = 0, iterations = 0, rounds = 0;
    // likelihood launches and the trajectories they evaluated, speculative candidates included
    // (committed evaluations = attempted_mutate)
    int64_t likelihood_launches = 0, evaluated_entries = 0;
};

class SamplerPTDevice {
public:
    SamplerPTDevice();
    ~SamplerPTDevice();
    bool Initialize(std::shared_ptr<Likelihood> ll, const std::vector<Marginal>& prior, const PTMHConfig& cfg,
                    std::unique_ptr<Transport> transport, void* stream);
    // SamplerPT::Run's loop body (SamplerPT.cpp:191-248) n times; `last` marks the final sample
    bool Iterate(int64_t n, bool last_at_end);
    // num_samples * use_every_nth iterations with the NaN check every nan_check_every
    bool Run(int64_t num_samples);
    bool AdaptProposal();
    // diagnostics: the last speculative launch's entries in dispatch order (source ids as in
    // bcm3hip_spec::batch_src, BDF steps); returns the entry count, -1 without speculation
    int64_t SpeculativeBatch(int32_t* src, int32_t* steps, int32_t* unused);
    // SampleHandlerNetCDF (SampleHandlerNetCDF.cpp:24-110): every emitted sample goes to `filename`,
    // staged in HBM and written every `flush_every` samples; call on every rank before the first
    // iteration. netCDF-4 (the reference's format) when libnetcdf can be loaded -- for a sharded
    // ladder rank 0 then receives the other ranks' staged rows over the transport at each flush and
    // writes the whole ladder --, else netCDF classic (NetCDFClassic.h), the ranks of a sharded ladder
    // sharing the file and each writing its own temperature columns
    bool SetOutput(const std::string& filename, int64_t num_samples, int flush_every);
    bool FlushOutput();
    // ptmhsampler.output_proposal_adaptation (SamplerPTChain.cpp:149-166): after every adaptation
    // the highest-temperature chain's proposal -- group adapt<k>/block1 with variable_indices,
    // gmm_weights and cluster<i>_mean / _covariance (ProposalGaussianMixture::WriteToFile :109-123)
    // or covariance (ProposalGlobalCovariance::WriteToFile :52-61), and from the second
    // adaptation on the history it was fitted to -- rewritten into `filename` (NetCDFBundler
    // layout in the classic format). Only the rank holding that chain writes.
    bool SetAdaptationOutput(const std::string& filename);
    bool CheckNaN();  // synchronises; false (and an error) if a likelihood returned NaN
    bool Synchronize();
    bool GetState(double* values, double* llh, double* lprior, double* lpp);
    bool GetProposalComponents(int32_t* ncomp);
    PTMHCounters GetCounters();
    void* Stream() const { return stream_; }
    int64_t NumLocalChains() const { return C_; }
    int NumVariables() const { return d_; }

private:
    struct Impl;
    std::unique_ptr<Impl> p_;
    void* stream_ = nullptr;
    int64_t C_ = 0;
    int d_ = 0;
};

// the reference's temperature ladder (SamplerPT.cpp:83-93)
std::vector<double> TemperatureLadder(int64_t num_chains, double power, double tmax);
// the counter-based uniforms of bcm3_amd.pt (exchange acceptance, move choice, random pair)
double ExchangeUniform(uint64_t seed, uint64_t rnd, uint64_t pair);

}  // namespace bcm3
