// SamplerPTDevice.cpp -- see SamplerPTDevice.h. The iteration restates SamplerPT::Run
// (src/sampler/SamplerPT.cpp:174-260) exactly as bcm3_amd/sampler.py's PTMHDevice does, so the
// two produce the same chains bit for bit (tests/test_ptmh_native_gpu.py).
#include "SamplerPTDevice.h"

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <limits>
#include <map>
#include <mutex>
#include <thread>

#include "../../../include/bcm3.h"
#include "../../../include/bcm3hip.h"
#include "GMM.h"
#include "NetCDFClassic.h"
#include "log.h"

namespace bcm3 {

static const double kInf = std::numeric_limits<double>::infinity();

// ---------------------------------------------------------------------------------------------
// counter-based host uniforms (bcm3_amd/pt.py)

static uint64_t SplitMix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double ExchangeUniform(uint64_t seed, uint64_t rnd, uint64_t pair)
{
    const uint64_t z = SplitMix64(SplitMix64(seed) ^ (rnd * 0x100000001B3ull) ^ (pair * 0xC2B2AE3D27D4EB4Full));
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

static const uint64_t kMoveSalt = 0x6D6F76655F747970ull;
static const uint64_t kPairSalt = 0x706169725F696478ull;

static double MoveUniform(uint64_t seed, uint64_t iteration) { return ExchangeUniform(seed ^ kMoveSalt, iteration, 0); }

static int64_t RandomPair(uint64_t seed, uint64_t rnd, int64_t Ctot)
{
    // rng.GetUnsignedInt(chains.size() - 2) (SamplerPT.cpp:301)
    return std::min((int64_t)(ExchangeUniform(seed ^ kPairSalt, rnd, 0) * (double)(Ctot - 1)), Ctot - 2);
}

std::vector<double> TemperatureLadder(int64_t num_chains, double power, double tmax)
{
    // SamplerPT::LoadSettings (SamplerPT.cpp:83-93): T0 = 0, Ti = Tmax (i / (C - 1))^power
    std::vector<double> t(num_chains, 0.0);
    for (int64_t i = 1; i < num_chains - 1; i++) t[i] = tmax * std::pow((double)i / (double)(num_chains - 1), power);
    if (num_chains > 1) t[num_chains - 1] = tmax;
    return t;
}

// SamplerPT::Initialize history size / subsampling (SamplerPT.cpp:113-123)
static void HistoryGeometry(int64_t adapt_samples, int64_t every_nth, int64_t exploration_steps, int64_t Ctot,
                            int64_t max_history, bool deterministic, int& size, int& sub)
{
    int64_t expected = adapt_samples * every_nth;
    if (Ctot > 1 && deterministic) expected *= exploration_steps + 1;
    int64_t s = 1, n = expected;
    if (n > max_history) {
        s = (expected + max_history - 1) / max_history;
        n = expected / s;
    }
    size = (int)std::max<int64_t>(n, 1);
    sub = (int)s;
}

// the chains of this rank in a pair of an exchange round (bcm3_amd.sampler.exchange_participants)
static std::vector<std::vector<uint8_t>> ExchangeParticipants(int64_t C, int64_t g0, int64_t Ctot, int world, int start,
                                                              bool& all_once)
{
    std::vector<std::vector<uint8_t>> out;
    all_once = false;
    if (Ctot < 2) return out;
    std::vector<uint8_t> local(C, 0), extra(C, 0);
    for (int64_t i = 0; i + 1 < C; i++)
        if (((g0 + i - start) % 2 + 2) % 2 == 0) local[i] = local[i + 1] = 1;
    if (world == 1) {
        if ((Ctot - 1 - start) % 2 == 0) extra[C - 1] = extra[0] = 1;
    } else {
        if (((g0 + C - 1 - start) % 2 + 2) % 2 == 0) extra[C - 1] = 1;
        if (((((g0 - 1) % Ctot + Ctot) % Ctot - start) % 2 + 2) % 2 == 0) extra[0] = 1;
    }
    bool exclusive = true;
    for (int64_t i = 0; i < C; i++) exclusive &= (local[i] != extra[i]);
    if (exclusive) {
        all_once = true;
        return out;
    }
    bool any_local = false, any_extra = false;
    for (int64_t i = 0; i < C; i++) {
        any_local |= local[i] != 0;
        any_extra |= extra[i] != 0;
    }
    if (any_local) out.push_back(local);
    if (any_extra) out.push_back(extra);
    return out;
}

// ---------------------------------------------------------------------------------------------
// transports

namespace {

class RcclTransport : public Transport {
public:
    explicit RcclTransport(void* comm) : comm_(comm) {}
    ~RcclTransport() override { bcm3hip_nccl_comm_destroy(comm_); }
    bool Exchange(int n_send, const double* const* sends, const int* send_peer, int n_recv, double* const* recvs,
                  const int* recv_peer, size_t count, void* stream) override
    {
        return bcm3hip_nccl_exchange(comm_, n_send, sends, send_peer, n_recv, recvs, recv_peer, count, stream) == 0;
    }

private:
    void* comm_;
};

}  // namespace

std::unique_ptr<Transport> MakeRcclTransport(const void* nccl_id, int rank, int world)
{
    void* comm = nullptr;
    if (bcm3hip_nccl_comm_init(nccl_id, rank, world, &comm) != 0) {
        LOGERROR("ncclCommInitRank failed (rank %d of %d)", rank, world);
        return nullptr;
    }
    return std::unique_ptr<Transport>(new RcclTransport(comm));
}

class LocalGroup {
public:
    explicit LocalGroup(int world) : world(world) {}
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::pair<int, int>, std::deque<std::vector<double>>> box;  // (src, dst) -> messages
};

std::shared_ptr<LocalGroup> MakeLocalGroup(int world) { return std::make_shared<LocalGroup>(world); }

namespace {

class LocalTransport : public Transport {
public:
    LocalTransport(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}
    bool Exchange(int n_send, const double* const* sends, const int* send_peer, int n_recv, double* const* recvs,
                  const int* recv_peer, size_t count, void* stream) override
    {
        if (bcm3hip_stream_synchronize(stream) != 0) return false;
        for (int i = 0; i < n_send; i++) {
            std::vector<double> msg(count);
            if (bcm3hip_memcpy_async(msg.data(), sends[i], count * sizeof(double), BCM3HIP_D2H, stream) != 0 ||
                bcm3hip_stream_synchronize(stream) != 0)
                return false;
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->box[{rank_, send_peer[i]}].push_back(std::move(msg));
            g_->cv.notify_all();
        }
        for (int j = 0; j < n_recv; j++) {
            std::vector<double> msg;
            {
                std::unique_lock<std::mutex> lk(g_->mu);
                auto& q = g_->box[{recv_peer[j], rank_}];
                if (!g_->cv.wait_for(lk, std::chrono::seconds(120), [&] { return !q.empty(); })) return false;
                msg = std::move(q.front());
                q.pop_front();
            }
            if (bcm3hip_memcpy_async(recvs[j], msg.data(), count * sizeof(double), BCM3HIP_H2D, stream) != 0 ||
                bcm3hip_stream_synchronize(stream) != 0)
                return false;
        }
        return true;
    }

private:
    std::shared_ptr<LocalGroup> g_;
    int rank_;
};

}  // namespace

std::unique_ptr<Transport> MakeLocalTransport(std::shared_ptr<LocalGroup> group, int rank)
{
    if (!group || rank < 0 || rank >= group->world) return nullptr;
    return std::unique_ptr<Transport>(new LocalTransport(std::move(group), rank));
}

// ---------------------------------------------------------------------------------------------
// device buffers

namespace {

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    bool alloc(size_t count)
    {
        n = count;
        return bcm3hip_malloc((void**)&p, std::max<size_t>(count, 1) * sizeof(T)) == 0;
    }
    ~DevBuf() { bcm3hip_free(p); }
};

template <class T>
bool Upload(DevBuf<T>& b, const std::vector<T>& h, void* s)
{
    return bcm3hip_memcpy_async(b.p, h.data(), h.size() * sizeof(T), BCM3HIP_H2D, s) == 0;
}
template <class T>
bool Download(std::vector<T>& h, const DevBuf<T>& b, void* s)
{
    h.resize(b.n);
    return bcm3hip_memcpy_async(h.data(), b.p, b.n * sizeof(T), BCM3HIP_D2H, s) == 0 && bcm3hip_stream_synchronize(s) == 0;
}

}  // namespace

struct SamplerPTDevice::Impl {
    PTMHConfig cfg;
    std::shared_ptr<Likelihood> ll;
    std::unique_ptr<Transport> transport;
    void* stream = nullptr;
    bool own_stream = false;
    int64_t C = 0, Ctot = 0, g0 = 0;
    int d = 0, kmax = 1, H = 1, sub = 1;
    bool adaptive = true, adjusted = false;
    int kind = 1;  // BCM3HIP_PROPOSAL_*
    std::vector<double> temps_host, prior_mean, prior_var;
    double target = 0.234;

    DevBuf<int32_t> pkind;
    DevBuf<double> p0, p1, p2, lower, upper, rw_scale, temps, zeros;
    DevBuf<double> values, prop, lprior, lprior_prop, llh, llh_prop, lpp, log_mh;
    DevBuf<int32_t> status, nan_flag;
    DevBuf<uint64_t> acc_mutate, acc_exchange;
    // proposal state
    DevBuf<int32_t> ncomp, selected;
    DevBuf<double> weights, mean, chol, logc, scale, ema, work;
    bcm3hip_proposal P{};
    // history
    DevBuf<float> hist;
    DevBuf<int64_t> hcount;
    // exchange masks per start (0 / 1): null = every chain once
    std::vector<std::unique_ptr<DevBuf<uint8_t>>> masks[2];
    bool mask_all[2] = {false, false};
    DevBuf<uint8_t> pair_mask;
    // boundary records
    DevBuf<double> send_last, send_first, recv_next, recv_prev;

    PTMHCounters cnt;
    int64_t iter = 0, round = 0;

    // speculative iteration pairs (bcm3hip_ptmh_spec_*): candidate / batch buffers, per round parity
    // the exchange partner and the first chain of each chain's pair, accept flags of both moves
    bool spec_on = false;
    bool spec_tail_on = true;  // BCM3_NO_SPEC_TAIL (read once, SetupSpeculation): the three separate launches
    DevBuf<double> sp_cand_x, sp_cand_lp, sp_cand_lmh, sp_cand_llh, sp_cand_sc, sp_batch_x, sp_batch_llh;
    DevBuf<int32_t> sp_cand_sel, sp_cand_upd, sp_cand_steps, sp_steps_hint, sp_steps_prop, sp_batch_status,
        sp_batch_steps, sp_batch_src, sp_batch_n, sp_err;
    DevBuf<int32_t> sp_pos;    // batch position of each entry (bcm3hip_spec::batch_pos)
    DevBuf<float> sp_xs;       // the batch's scaled single-precision coordinates (bcm3hip_spec::batch_xs)
    DevBuf<int64_t> sp_total;  // entries of all speculative batches (bcm3hip_spec::batch_total)
    DevBuf<uint8_t> sp_cand_active, acc_mut, acc_mut2, acc_exc;
    DevBuf<int32_t> partner[2], pair_first[2];
    DevBuf<double> sp_send_last, sp_send_first, sp_remote;  // boundary rows [state | proposal] of a sharded ladder
    DevBuf<uint8_t> cross_acc;
    DevBuf<int32_t> sp_pred;
    DevBuf<double> sp_inv_scale;  // 1 / prior sd per variable (the predictor's distance)
    bool cross_round[2] = {false, false};  // do the slice-boundary pairs exchange in rounds of this parity
    bcm3hip_spec S{};
    int64_t spec_pairs = 0;
    int spec_first_round = 0;  // the device's SIMDs: batch positions p and p + this share a SIMD

    // sample output: [flush][values C*d | lprior C | llh C] staged on the device
    std::unique_ptr<SampleFileWriter> out;
    DevBuf<double> out_buf;
    // a sharded ladder writing the reference's netCDF-4 file: every rank stages its samples, rank 0
    // receives the other ranks' staged rows over the transport at each flush and writes all columns
    bool out_on = false, out_gather = false;
    DevBuf<double> out_recv;
    int64_t out_samples = 0, out_first = 0, out_pending = 0, emitted = 0;
    int out_flush = 64;
    bool out_overflow_logged = false;
    std::string adapt_file;
    BundleFile adapt_out;

    bool Emit()
    {
        // SamplerPT::EmitSample (SamplerPT.cpp:321-330): every chain, weight 1
        const int64_t six = emitted++;
        if (!out_on) return true;
        if (six >= out_samples) {
            if (!out_overflow_logged) LOGWARNING("More samples than the output file holds (%lld); later samples are not stored", (long long)out_samples);
            out_overflow_logged = true;
            return true;
        }
        if (out_pending == 0) out_first = six;
        double* slot = out_buf.p + out_pending * C * (d + 2);
        if (bcm3hip_memcpy_async(slot, values.p, C * d * sizeof(double), BCM3HIP_D2D, stream) != 0 ||
            bcm3hip_memcpy_async(slot + C * d, lprior.p, C * sizeof(double), BCM3HIP_D2D, stream) != 0 ||
            bcm3hip_memcpy_async(slot + C * (d + 1), llh.p, C * sizeof(double), BCM3HIP_D2D, stream) != 0)
            return false;
        out_pending++;
        if (out_pending == out_flush || six + 1 == out_samples) return Flush();
        return true;
    }

    bool Flush()
    {
        if (!out_on || out_pending == 0) return true;
        if (out_gather) return FlushGather();
        std::vector<double> h((size_t)(out_pending * C * (d + 2)));
        if (bcm3hip_memcpy_async(h.data(), out_buf.p, h.size() * sizeof(double), BCM3HIP_D2H, stream) != 0 ||
            bcm3hip_stream_synchronize(stream) != 0)
            return false;
        const std::vector<double> w(C, 1.0);
        for (int64_t k = 0; k < out_pending; k++) {
            const double* r = &h[(size_t)(k * C * (d + 2))];
            if (!out->Write((size_t)(out_first + k), 0, (size_t)C, r, r + C * d, r + C * (d + 1), w.data())) {
                LOGERROR("Writing sample %lld to the output file failed", (long long)(out_first + k));
                return false;
            }
        }
        out_pending = 0;
        return true;
    }

    // all ranks flush together (Emit runs in lockstep on every rank): ranks > 0 send their staged
    // [pending][values C*d | lprior C | llh C] block to rank 0, which assembles each sample's rows of
    // the whole ladder (rank r holds temperatures r*C .. r*C + C - 1) and writes them at once
    bool FlushGather()
    {
        const size_t cnt = (size_t)(out_pending * C * (d + 2));
        const int world = cfg.world, rank = cfg.rank;
        if (rank != 0) {
            const double* sp = out_buf.p;
            const int peer = 0;
            if (!transport || !transport->Exchange(1, &sp, &peer, 0, nullptr, nullptr, cnt, stream)) {
                LOGERROR("Sending sample rows to rank 0 failed (rank %d)", rank);
                return false;
            }
            out_pending = 0;
            return bcm3hip_stream_synchronize(stream) == 0;
        }
        std::vector<double*> recvs((size_t)(world - 1));
        std::vector<int> peers((size_t)(world - 1));
        for (int r = 1; r < world; r++) {
            recvs[(size_t)(r - 1)] = out_recv.p + (size_t)(r - 1) * cnt;
            peers[(size_t)(r - 1)] = r;
        }
        if (!transport || !transport->Exchange(0, nullptr, nullptr, world - 1, recvs.data(), peers.data(), cnt, stream)) {
            LOGERROR("Receiving the other ranks' sample rows failed");
            return false;
        }
        std::vector<double> h((size_t)world * cnt);
        if (bcm3hip_memcpy_async(h.data(), out_buf.p, cnt * sizeof(double), BCM3HIP_D2H, stream) != 0 ||
            (world > 1 && bcm3hip_memcpy_async(h.data() + cnt, out_recv.p, (size_t)(world - 1) * cnt * sizeof(double),
                                               BCM3HIP_D2H, stream) != 0) ||
            bcm3hip_stream_synchronize(stream) != 0)
            return false;
        const size_t Cw = (size_t)(C * world), dd = (size_t)d;
        std::vector<double> vals(Cw * dd), lp(Cw), ll(Cw);
        const std::vector<double> w(Cw, 1.0);
        for (int64_t k = 0; k < out_pending; k++) {
            for (int r = 0; r < world; r++) {
                const double* b = &h[(size_t)r * cnt + (size_t)(k * C * (d + 2))];
                std::copy(b, b + C * d, vals.begin() + (size_t)r * C * dd);
                std::copy(b + C * d, b + C * (d + 1), lp.begin() + (size_t)r * C);
                std::copy(b + C * (d + 1), b + C * (d + 2), ll.begin() + (size_t)r * C);
            }
            if (!out->Write((size_t)(out_first + k), 0, Cw, vals.data(), lp.data(), ll.data(), w.data())) {
                LOGERROR("Writing sample %lld to the output file failed", (long long)(out_first + k));
                return false;
            }
        }
        out_pending = 0;
        return true;
    }

    bool Launch(int rc, const char* what)
    {
        if (rc != 0) LOGERROR("%s failed: %s (%d)", what, bcm3hip_error_string(rc), rc);
        return rc == 0;
    }

    bool Eval(double* x, double* out)
    {
        cnt.likelihood_launches++;
        cnt.evaluated_entries += C;
        if (!ll->EvaluateLogProbabilityBatchDevice((size_t)C, x, out, status.p, stream)) {
            LOGERROR("EvaluateLogProbabilityBatchDevice failed");
            return false;
        }
        return true;
    }

    bool ProposeInit(uint64_t it)
    {
        if (adaptive)
            return Launch(bcm3hip_ptmh_propose_adaptive((int)C, d, pkind.p, p0.p, p1.p, p2.p, zeros.p, values.p, prop.p,
                                                        lprior_prop.p, log_mh.p, &P, g0, cfg.seed, it, stream),
                          "ptmh_propose_adaptive");
        return Launch(bcm3hip_ptmh_propose((int)C, d, pkind.p, p0.p, p1.p, rw_scale.p, zeros.p, values.p, prop.p,
                                           lprior_prop.p, g0, cfg.seed, it, stream),
                      "ptmh_propose");
    }

    // DeviceProposal.reset_from_prior + _reset_scales(initial=True)
    bool InitProposal()
    {
        std::vector<int32_t> nc(C, 1), sel(C, -1);
        std::vector<double> w(C * kmax, 0.0), mu(C * kmax * d, 0.0), L(C * kmax * d * d, 0.0), lc(C * kmax);
        double det = 0.0;
        std::vector<double> sd(d);
        for (int j = 0; j < d; j++) sd[j] = std::sqrt(prior_var[j]);
        for (int j = 0; j < d; j++) det += std::log(sd[j]);
        const double logc_prior = -det - 0.5 * d * std::log(2.0 * M_PI);
        const double logc_id = -0.0 - 0.5 * d * std::log(2.0 * M_PI);
        for (int64_t c = 0; c < C; c++) {
            w[c * kmax] = 1.0;
            for (int j = 0; j < d; j++) mu[(c * kmax) * d + j] = prior_mean[j];
            for (int k = 0; k < kmax; k++)
                for (int j = 0; j < d; j++) L[((c * kmax + k) * d + j) * d + j] = (k == 0) ? sd[j] : 1.0;
            for (int k = 0; k < kmax; k++) lc[c * kmax + k] = (k == 0) ? logc_prior : logc_id;
        }
        const bool gmm = kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE;
        std::vector<double> sc(C * kmax, gmm ? 2.38 / std::sqrt((double)d) : 1.0);
        std::vector<double> em(C * kmax, gmm ? target : 0.23);
        return Upload(ncomp, nc, stream) && Upload(selected, sel, stream) && Upload(weights, w, stream) &&
               Upload(mean, mu, stream) && Upload(chol, L, stream) && Upload(logc, lc, stream) &&
               Upload(scale, sc, stream) && Upload(ema, em, stream) &&
               bcm3hip_memset_async(work.p, 0, work.n * sizeof(double), stream) == 0;
    }

    bool InitialPositions()
    {
        // SamplerPTChain::Initialize / FindStartingPosition (SamplerPTChain.cpp:188-214), as
        // PTMHDevice._initial_positions: prior draws on counter streams INIT_ITER, INIT_ITER - 1, ...
        const uint64_t INIT_ITER = (1ull << 63) - 1;
        std::vector<double> v(C * d, 0.0), q(C, -kInf), l(C, -kInf), pv, pq, pl;
        std::vector<char> bad(C, 1);
        std::vector<int32_t> hint(C, 0), ps;  // the speculative pairs' dispatch-order hints
        bool any = true;
        for (int k = 0; k < cfg.initial_position_tries && any; k++) {
            if (!Upload(values, v, stream) || !ProposeInit(INIT_ITER - (uint64_t)k)) return false;
            if (spec_on) {
                // the same evaluation through the counted entry point, for the solves' step counts
                const std::vector<int32_t> nC(1, (int32_t)C);
                cnt.likelihood_launches++;
                cnt.evaluated_entries += C;
                if (!Upload(sp_batch_n, nC, stream) ||
                    !ll->EvaluateLogProbabilityBatchDeviceCounted((size_t)C, sp_batch_n.p, prop.p, llh_prop.p,
                                                                  status.p, sp_steps_prop.p, stream) ||
                    !Download(ps, sp_steps_prop, stream))
                    return false;
            } else if (!Eval(prop.p, llh_prop.p)) {
                return false;
            }
            if (!Download(pv, prop, stream) || !Download(pq, lprior_prop, stream) || !Download(pl, llh_prop, stream))
                return false;
            any = false;
            for (int64_t c = 0; c < C; c++) {
                const double nl = pl[c] * cfg.learning_rate;
                if (std::isnan(nl)) {
                    LOGERROR("Likelihood evaluation returned NaN while finding starting positions");
                    return false;
                }
                if (bad[c]) {
                    std::copy(pv.begin() + c * d, pv.begin() + (c + 1) * d, v.begin() + c * d);
                    q[c] = pq[c];
                    l[c] = nl;
                    if (spec_on) hint[c] = ps[c];
                }
                bad[c] = !(q[c] + temps_host[c] * l[c] > -kInf);
                any |= bad[c] != 0;
            }
        }
        if (any) {
            LOGERROR("Could not find starting position with power posterior != inf after %d tries",
                     cfg.initial_position_tries);
            return false;
        }
        std::vector<double> pp(C);
        for (int64_t c = 0; c < C; c++) pp[c] = (temps_host[c] == 0.0) ? q[c] : q[c] + temps_host[c] * l[c];
        // (the counted evaluations above used batch_n: reset, so the first pair predicts from hints)
        return Upload(values, v, stream) && Upload(lprior, q, stream) && Upload(llh, l, stream) &&
               Upload(lpp, pp, stream) &&
               (!spec_on || (Upload(sp_steps_hint, hint, stream) &&
                             bcm3hip_memset_async(sp_batch_n.p, 0, sizeof(int32_t), stream) == 0));
    }

    bool HistoryAdd(const uint8_t* mask)
    {
        return Launch(bcm3hip_history_add((int)C, d, H, sub, temps.p, values.p, mask, hist.p, hcount.p, stream),
                      "history_add");
    }

    bool Mutate()
    {
        // DoMutateMove (SamplerPT.cpp:308-319): every chain's proposal in one likelihood launch
        if (adaptive) {
            if (!Launch(bcm3hip_ptmh_propose_adaptive((int)C, d, pkind.p, p0.p, p1.p, p2.p, temps.p, values.p, prop.p,
                                                      lprior_prop.p, log_mh.p, &P, g0, cfg.seed, (uint64_t)iter,
                                                      stream),
                        "ptmh_propose_adaptive") ||
                !Eval(prop.p, llh_prop.p) ||
                !Launch(bcm3hip_ptmh_accept_adaptive((int)C, d, temps.p, prop.p, lprior_prop.p, llh_prop.p, log_mh.p,
                                                     cfg.learning_rate, values.p, lprior.p, llh.p, lpp.p, nullptr,
                                                     acc_mutate.p, nan_flag.p, &P, g0, cfg.seed, (uint64_t)iter,
                                                     stream),
                        "ptmh_accept_adaptive") ||
                !HistoryAdd(nullptr))  // SamplerPTChain.cpp:309
                return false;
        } else {
            if (!Launch(bcm3hip_ptmh_propose((int)C, d, pkind.p, p0.p, p1.p, rw_scale.p, temps.p, values.p, prop.p,
                                             lprior_prop.p, g0, cfg.seed, (uint64_t)iter, stream),
                        "ptmh_propose") ||
                !Eval(prop.p, llh_prop.p) ||
                !Launch(bcm3hip_ptmh_accept((int)C, d, temps.p, prop.p, lprior_prop.p, llh_prop.p, cfg.learning_rate,
                                            values.p, lprior.p, llh.p, lpp.p, nullptr, acc_mutate.p, nan_flag.p, g0,
                                            cfg.seed, (uint64_t)iter, stream),
                        "ptmh_accept"))
                return false;
        }
        cnt.attempted_mutate += C;
        iter++;
        return true;
    }

    // ranks' neighbours on the ring
    int Next() const { return (cfg.rank + 1) % cfg.world; }
    int Prev() const { return (cfg.rank - 1 + cfg.world) % cfg.world; }

    bool Cross(bool do_next, bool do_prev, int64_t gp, uint8_t* acc_out = nullptr)
    {
        const size_t n = (size_t)d + 4;
        if (!Launch(bcm3hip_pt_pack_boundary((int)C, d, temps.p, values.p, llh.p, lprior.p, lpp.p,
                                             do_next ? send_last.p : nullptr, do_prev ? send_first.p : nullptr,
                                             stream),
                    "pt_pack_boundary"))
            return false;
        // PTExchange._cross's order: send(last -> next), recv(prev), send(first -> prev), recv(next)
        const double* sends[2];
        int speer[2], rpeer[2], ns = 0, nr = 0;
        double* recvs[2];
        if (do_next) {
            sends[ns] = send_last.p;
            speer[ns++] = Next();
        }
        if (do_prev) {
            sends[ns] = send_first.p;
            speer[ns++] = Prev();
            recvs[nr] = recv_prev.p;
            rpeer[nr++] = Prev();
        }
        if (do_next) {
            recvs[nr] = recv_next.p;
            rpeer[nr++] = Next();
        }
        if (!transport || !transport->Exchange(ns, sends, speer, nr, recvs, rpeer, n, stream)) {
            LOGERROR("PT swap transport failed (rank %d)", cfg.rank);
            return false;
        }
        return Launch(bcm3hip_pt_cross_accept((int)C, d, g0, gp, do_next, do_prev, temps.p, values.p, llh.p,
                                              lprior.p, lpp.p, recv_next.p, recv_prev.p, acc_out,
                                              do_next ? acc_exchange.p : nullptr, cfg.seed, (uint64_t)round, stream),
                      "pt_cross_accept");
    }

    bool Exchange(uint8_t* acc_mask = nullptr, uint8_t* cross_out = nullptr)
    {
        // DoExchangeMove (SamplerPT.cpp:277-298): pairs inside the slice on the GPU, the two
        // slice-boundary pairs over the transport (sampler.sharded_exchange_round)
        if (Ctot < 2) return true;
        const int start = (int)(round % 2);
        const bool wrap_local = cfg.world == 1 && (Ctot - 1 - start) % 2 == 0;
        if (!Launch(bcm3hip_pt_exchange_local((int)C, d, g0, start, wrap_local ? 1 : 0, temps.p, values.p, llh.p,
                                              lprior.p, lpp.p, acc_mask, acc_exchange.p, cfg.seed, (uint64_t)round,
                                              stream),
                    "pt_exchange_local"))
            return false;
        int64_t attempted = wrap_local ? 1 : 0;
        for (int64_t i = 0; i + 1 < C; i++)
            if (((g0 + i - start) % 2 + 2) % 2 == 0) attempted++;
        if (cfg.world > 1 && ((g0 + C - 1 - start) % 2 + 2) % 2 == 0) {
            if (!Cross(true, true, (int64_t)Prev() * C + C - 1, cross_out)) return false;
            attempted++;
        }
        cnt.attempted_exchange += attempted;
        if (adaptive) {
            // ExchangeMove adds both chains of every pair to their histories (SamplerPTChain.cpp:374-379)
            if (mask_all[start]) {
                if (!HistoryAdd(nullptr)) return false;
            } else {
                for (auto& m : masks[start])
                    if (!HistoryAdd(m->p)) return false;
            }
        }
        round++;
        return true;
    }

    bool ExchangeRandom()
    {
        // stochastic_random (SamplerPT.cpp:300-305)
        const int64_t ci = RandomPair(cfg.seed, (uint64_t)round, Ctot);
        const int64_t l1 = ci - g0, l2 = ci + 1 - g0;
        if (0 <= l1 && l2 < C) {
            if (!Launch(bcm3hip_pt_exchange_pair((int)C, d, (int)l1, (int)l2, ci, temps.p, values.p, llh.p, lprior.p,
                                                 lpp.p, nullptr, acc_exchange.p, cfg.seed, (uint64_t)round, stream),
                        "pt_exchange_pair"))
                return false;
            cnt.attempted_exchange++;
        } else if (cfg.world > 1 && (l1 == C - 1 || l2 == 0)) {
            if (l1 == C - 1) {
                if (!Cross(true, false, 0)) return false;
                cnt.attempted_exchange++;
            } else if (!Cross(false, true, ci)) {
                return false;
            }
        }
        if (adaptive) {
            std::vector<uint8_t> m(C, 0);
            bool any = false;
            for (int64_t i : {l1, l2})
                if (0 <= i && i < C) {
                    m[i] = 1;
                    any = true;
                }
            if (any && (!Upload(pair_mask, m, stream) || !HistoryAdd(pair_mask.p))) return false;
        }
        round++;
        return true;
    }

    bool IterationOnce(bool last)
    {
        // SamplerPT::Run (SamplerPT.cpp:191-248)
        bool ok;
        if (Ctot < 2) {
            ok = Mutate();
        } else if (cfg.swapping_scheme == 0) {
            ok = Exchange();
            for (int s = 0; ok && s < cfg.exploration_steps; s++) ok = Mutate();
        } else if (MoveUniform(cfg.seed, (uint64_t)cnt.samples_done) < cfg.exchange_probability) {
            ok = (cfg.swapping_scheme == 1) ? Exchange() : ExchangeRandom();
        } else {
            ok = Mutate();
        }
        return ok && PostIteration(last);
    }

    // does the end of iteration si (0-based sample index) adapt the proposals (SamplerPT.cpp:229-248)
    bool AdaptDue(int64_t si, bool last) const
    {
        if (!adaptive || (si + 1) % cfg.use_every_nth != 0) return false;
        const int64_t sample_ix = si / cfg.use_every_nth;
        return cfg.adapt_proposal_samples > 0 && (sample_ix + 1) % cfg.adapt_proposal_samples == 0 && !last &&
               cnt.adaptations_done < cfg.adapt_proposal_times;
    }

    // the end of SamplerPT::Run's loop body: sample emission, proposal adaptation when due
    bool PostIteration(bool last)
    {
        const int64_t si = cnt.samples_done++;
        cnt.iterations++;
        if ((si + 1) % cfg.use_every_nth == 0 && !Emit()) return false;
        if (AdaptDue(si, last)) return Adapt();
        return true;
    }

    // can the next two iterations run as a speculative pair (the first must not adapt: the second's
    // proposals are made before it ends)
    bool PairPossible() const { return spec_on && !AdaptDue(cnt.samples_done, false); }

    // Two DeterministicEvenOdd iterations r, r+1 with ONE likelihood launch (include/bcm3hip.h
    // "speculative iteration pairs"): exchange r, propose r, the candidates of r+1 (every state
    // exchange r+1 can leave in each slot), one launch over r's proposals and the candidates, accept
    // r; exchange r+1, select the candidate that happened, accept r+1. The same kernels' arithmetic
    // on the same counter-based random numbers as two IterationOnce calls.
    // an exchange round of a pair and its dispatch-order tracking: on one rank whose pairs cover every
    // chain once, the exchange, the tracking and the history adds in one launch (spec_exchange)
    bool PairExchange()
    {
        const int st = (int)(round % 2);
        if (cfg.world == 1 && mask_all[st] && Ctot >= 2) {
            const bool wrap_local = (Ctot - 1 - st) % 2 == 0;
            int64_t attempted = wrap_local ? 1 : 0;
            for (int64_t i = 0; i + 1 < C; i++)
                if (((g0 + i - st) % 2 + 2) % 2 == 0) attempted++;
            if (!Launch(bcm3hip_ptmh_spec_exchange((int)C, d, g0, st, wrap_local ? 1 : 0, temps.p, values.p, llh.p,
                                                   lprior.p, lpp.p, acc_exc.p, acc_exchange.p, cfg.seed,
                                                   (uint64_t)round, partner[st].p, pair_first[st].p, &S, H, sub,
                                                   adaptive ? hist.p : nullptr, hcount.p, stream),
                        "ptmh_spec_exchange"))
                return false;
            cnt.attempted_exchange += attempted;
            round++;
            return true;
        }
        return Exchange(acc_exc.p, cross_acc.p) &&
               Launch(bcm3hip_ptmh_spec_track((int)C, nullptr, partner[st].p, pair_first[st].p, acc_exc.p, &S, stream),
                      "ptmh_spec_track");
    }

    // can the rest of a pair after its likelihood launch run as one spec_tail launch: a single rank
    // whose exchange pairs cover every chain in round r + 1 (PairExchange's one-launch case), and no
    // sample output copied between the two iterations (Emit after iteration r)
    bool TailFusable() const
    {
        const int st = (int)(round % 2);
        return cfg.world == 1 && mask_all[st] && Ctot >= 2 && C <= 4096 && S.batch_pos &&
               !(out_on && (cnt.samples_done + 1) % cfg.use_every_nth == 0) && spec_tail_on;
    }

    bool IterationPair(bool last)
    {
        if (!PairExchange()) return false;
        const int nxt = (int)(round % 2);  // start parity of exchange round r + 1
        if (!Launch(bcm3hip_ptmh_propose_adaptive((int)C, d, pkind.p, p0.p, p1.p, p2.p, temps.p, values.p, prop.p,
                                                  lprior_prop.p, log_mh.p, &P, g0, cfg.seed, (uint64_t)iter, stream),
                    "ptmh_propose_adaptive"))
            return false;
        if (cross_round[nxt]) {
            // a sharded ladder whose boundary pairs exchange in round r + 1: the neighbours' boundary
            // chains' (state, proposal) rows, for the candidates that start from them
            const size_t row = (size_t)d * sizeof(double);
            if (bcm3hip_memcpy_async(sp_send_last.p, values.p + (C - 1) * d, row, BCM3HIP_D2D, stream) != 0 ||
                bcm3hip_memcpy_async(sp_send_last.p + d, prop.p + (C - 1) * d, row, BCM3HIP_D2D, stream) != 0 ||
                bcm3hip_memcpy_async(sp_send_first.p, values.p, row, BCM3HIP_D2D, stream) != 0 ||
                bcm3hip_memcpy_async(sp_send_first.p + d, prop.p, row, BCM3HIP_D2D, stream) != 0)
                return false;
            const double* sends[2] = {sp_send_last.p, sp_send_first.p};
            const int speer[2] = {Next(), Prev()};
            double* recvs[2] = {sp_remote.p + 2 * d, sp_remote.p};  // from prev -> PREV slot, from next -> NEXT slot
            const int rpeer[2] = {Prev(), Next()};
            if (!transport || !transport->Exchange(2, sends, speer, 2, recvs, rpeer, (size_t)(2 * d), stream)) {
                LOGERROR("speculative boundary rows: transport failed (rank %d)", cfg.rank);
                return false;
            }
        }
        if (!Launch(bcm3hip_ptmh_spec_candidates((int)C, d, pkind.p, p0.p, p1.p, p2.p, temps.p, values.p, prop.p,
                                                 partner[nxt].p, sp_remote.p, &P, &S, g0, cfg.seed, (uint64_t)iter + 1,
                                                 stream),
                    "ptmh_spec_candidates") ||
            !Launch(bcm3hip_ptmh_spec_batch((int)C, d, prop.p, partner[nxt].p, sp_inv_scale.p, spec_first_round, &S,
                                            stream),
                    "ptmh_spec_batch"))
            return false;
        cnt.likelihood_launches++;  // its entries are summed on the device (sp_total)
        if (!ll->EvaluateLogProbabilityBatchDeviceCounted((size_t)C * (1 + BCM3HIP_SPEC_SLOTS), S.batch_n, S.batch_x,
                                                          S.batch_llh, S.batch_status, S.batch_steps, stream)) {
            LOGERROR("EvaluateLogProbabilityBatchDeviceCounted failed");
            return false;
        }
        if (TailFusable()) {
            // accept r, the exchange round of r + 1 and accept r + 1 in one launch (spec_tail: the three
            // launches below in one workgroup); the host's bookkeeping in the same order
            const int st = (int)(round % 2);
            const bool wrap_local = (Ctot - 1 - st) % 2 == 0;
            int64_t attempted = wrap_local ? 1 : 0;
            for (int64_t i = 0; i + 1 < C; i++)
                if (((g0 + i - st) % 2 + 2) % 2 == 0) attempted++;
            if (!Launch(bcm3hip_ptmh_spec_tail((int)C, d, g0, st, wrap_local ? 1 : 0, temps.p, partner[st].p,
                                               pair_first[st].p, acc_mut.p, acc_mut2.p, acc_exc.p, cross_acc.p,
                                               sp_remote.p, acc_mutate.p, acc_exchange.p, &S, prop.p, lprior_prop.p,
                                               log_mh.p, llh_prop.p, cfg.learning_rate, values.p, lprior.p, llh.p, lpp.p,
                                               nan_flag.p, &P, cfg.seed, (uint64_t)iter, (uint64_t)round, H, sub, hist.p,
                                               hcount.p, sp_err.p, stream),
                        "ptmh_spec_tail"))
                return false;
            cnt.attempted_mutate += C;
            iter++;
            if (!PostIteration(false)) return false;  // (no device work: TailFusable)
            cnt.attempted_exchange += attempted;
            round++;
            cnt.attempted_mutate += C;
            iter++;
            spec_pairs++;
            return PostIteration(last);
        }
        // the batch's results to their chains, accept r, its dispatch-order tracking and the history
        // add in one launch (spec_commit reads the batch through S.batch_pos: no spec_scatter launch)
        if (!Launch(bcm3hip_ptmh_spec_commit((int)C, d, 0, temps.p, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                             &S, prop.p, lprior_prop.p, log_mh.p, llh_prop.p, cfg.learning_rate,
                                             values.p, lprior.p, llh.p, lpp.p, acc_mut.p, acc_mutate.p, nan_flag.p, &P,
                                             g0, cfg.seed, (uint64_t)iter, H, sub, hist.p, hcount.p, sp_err.p, stream),
                    "ptmh_spec_commit"))
            return false;
        cnt.attempted_mutate += C;
        iter++;
        if (!PostIteration(false)) return false;
        // iteration r + 1
        if (!PairExchange()) return false;
        // select the candidate that happened, accept r + 1, tracking, history: one launch (the accept
        // flags of r + 1 go to acc_mut2, select reads r's from acc_mut)
        if (!Launch(bcm3hip_ptmh_spec_commit((int)C, d, 1, temps.p, partner[nxt].p, pair_first[nxt].p, acc_mut.p,
                                             acc_exc.p, cross_acc.p, sp_remote.p, &S, prop.p, lprior_prop.p, log_mh.p,
                                             llh_prop.p, cfg.learning_rate, values.p, lprior.p, llh.p, lpp.p, acc_mut2.p,
                                             acc_mutate.p, nan_flag.p, &P, g0, cfg.seed, (uint64_t)iter, H, sub, hist.p,
                                             hcount.p, sp_err.p, stream),
                    "ptmh_spec_commit"))
            return false;
        cnt.attempted_mutate += C;
        iter++;
        spec_pairs++;
        return PostIteration(last);
    }

    // n iterations: speculative pairs where possible, single iterations otherwise
    bool Iterations(int64_t n, bool last_at_end, int64_t nan_every)
    {
        int64_t since_check = 0;
        for (int64_t i = 0; i < n;) {
            int64_t k;
            if (i + 2 <= n && PairPossible()) {
                if (!IterationPair(last_at_end && i + 2 == n)) return false;
                k = 2;
            } else {
                if (!IterationOnce(last_at_end && i + 1 == n)) return false;
                k = 1;
            }
            i += k;
            since_check += k;
            if (nan_every > 0 && since_check >= nan_every) {
                since_check = 0;
                if (!CheckNaN()) return false;
            }
        }
        return true;
    }

    bool SetupSpeculation()
    {
        spec_tail_on = getenv("BCM3_NO_SPEC_TAIL") == nullptr;
        spec_on = cfg.speculate != 0 && adaptive && (cfg.world == 1 || transport) && cfg.swapping_scheme == 0 &&
                  cfg.exploration_steps == 1 && Ctot >= 2 && d <= 64 && C * (1 + BCM3HIP_SPEC_SLOTS) <= 4096 &&
                  ll->SupportsCountedBatch();
        if (!spec_on) return true;
        spec_first_round = bcm3hip_current_device_simds();
        const int64_t K = BCM3HIP_SPEC_SLOTS, N = C * (1 + K);
        bool ok = sp_cand_x.alloc(C * K * d) && sp_cand_lp.alloc(C * K) && sp_cand_lmh.alloc(C * K) &&
                  sp_cand_llh.alloc(C * K) && sp_cand_sc.alloc(C * K) && sp_cand_sel.alloc(C * K) &&
                  sp_cand_upd.alloc(C * K) && sp_cand_steps.alloc(C * K) && sp_cand_active.alloc(C * K) &&
                  sp_steps_hint.alloc(C) && sp_steps_prop.alloc(C) && sp_batch_x.alloc(N * d) &&
                  sp_batch_llh.alloc(N) && sp_batch_status.alloc(N) && sp_batch_steps.alloc(N) &&
                  sp_batch_src.alloc(N) && sp_batch_n.alloc(1) && sp_err.alloc(1) && acc_mut.alloc(C) &&
                  acc_mut2.alloc(C) &&
                  acc_exc.alloc(C) && sp_send_last.alloc(2 * d) && sp_send_first.alloc(2 * d) &&
                  sp_remote.alloc(4 * d) && cross_acc.alloc(2) && sp_pred.alloc(N) && sp_inv_scale.alloc(d) &&
                  sp_total.alloc(1) && sp_pos.alloc(N) && sp_xs.alloc(N * d);
        for (int st = 0; st < 2 && ok; st++) ok = partner[st].alloc(C) && pair_first[st].alloc(C);
        if (!ok) {
            LOGERROR("SamplerPTDevice: speculative buffers could not be allocated");
            return false;
        }
        // exchange pairs of a round with start parity st (pt_exchange_kernel: first chains i with
        // (g0 + i - st) even, i + 1 < C, then the wrap pair (C-1, 0) on one rank)
        for (int st = 0; st < 2; st++) {
            std::vector<int32_t> pa(C, -1), pf(C, -1);
            const int par = (int)(((g0 - st) % 2 + 2) % 2);
            for (int64_t i = par; i + 1 < C; i += 2) {
                pa[i] = (int32_t)(i + 1);
                pa[i + 1] = (int32_t)i;
                pf[i] = pf[i + 1] = (int32_t)i;
            }
            if (cfg.world == 1 && (Ctot - 1 - st) % 2 == 0) {
                pa[C - 1] = 0;
                pa[0] = (int32_t)(C - 1);
                pf[C - 1] = pf[0] = (int32_t)(C - 1);
            }
            // sharded: the slice-boundary pairs over the transport (Exchange: both cross pairs of a
            // rank exchange in the same rounds, C being even)
            cross_round[st] = cfg.world > 1 && ((g0 + C - 1 - st) % 2 + 2) % 2 == 0;
            if (cross_round[st]) {
                pa[C - 1] = BCM3HIP_SPEC_REMOTE_NEXT;
                pa[0] = BCM3HIP_SPEC_REMOTE_PREV;
            }
            if (!Upload(partner[st], pa, stream) || !Upload(pair_first[st], pf, stream)) return false;
        }
        std::vector<double> isc(d);
        for (int j = 0; j < d; j++)
            isc[j] = (prior_var[j] > 0.0 && std::isfinite(prior_var[j])) ? 1.0 / std::sqrt(prior_var[j]) : 1.0;
        if (!Upload(sp_inv_scale, isc, stream) ||
            bcm3hip_memset_async(sp_batch_n.p, 0, sizeof(int32_t), stream) != 0 ||
            bcm3hip_memset_async(sp_steps_hint.p, 0, C * sizeof(int32_t), stream) != 0 ||
            bcm3hip_memset_async(sp_batch_steps.p, 0, N * sizeof(int32_t), stream) != 0 ||
            bcm3hip_memset_async(sp_cand_steps.p, 0, C * K * sizeof(int32_t), stream) != 0 ||
            bcm3hip_memset_async(sp_err.p, 0, sizeof(int32_t), stream) != 0 ||
            bcm3hip_memset_async(sp_total.p, 0, sizeof(int64_t), stream) != 0)
            return false;
        S.cand_x = sp_cand_x.p;
        S.cand_lp = sp_cand_lp.p;
        S.cand_lmh = sp_cand_lmh.p;
        S.cand_llh = sp_cand_llh.p;
        S.cand_sel = sp_cand_sel.p;
        S.cand_upd = sp_cand_upd.p;
        S.cand_sc = sp_cand_sc.p;
        S.cand_active = sp_cand_active.p;
        S.cand_steps = sp_cand_steps.p;
        S.steps_hint = sp_steps_hint.p;
        S.steps_prop = sp_steps_prop.p;
        S.batch_x = sp_batch_x.p;
        S.batch_llh = sp_batch_llh.p;
        S.batch_status = sp_batch_status.p;
        S.batch_steps = sp_batch_steps.p;
        S.batch_src = sp_batch_src.p;
        S.batch_n = sp_batch_n.p;
        S.pred_steps = sp_pred.p;
        S.batch_total = sp_total.p;
        S.batch_pos = sp_pos.p;
        S.batch_xs = sp_xs.p;
        return true;
    }

    bool CheckNaN()
    {
        std::vector<int32_t> f;
        if (!Download(f, nan_flag, stream)) return false;
        if (f[0] != 0) {
            LOGERROR("Likelihood evaluation returned NaN (Sampler::EvaluateLikelihood, fatal)");
            return false;
        }
        if (spec_on) {
            if (!Download(f, sp_err, stream)) return false;
            if (f[0] != 0) {
                LOGERROR("Speculative iteration: the candidate that happened was not evaluated (internal error)");
                return false;
            }
        }
        return true;
    }

    bool Adapt()
    {
        // SamplerPTChain::AdaptProposal for every chain of the rank (T == 0 excepted), then the
        // history reset (SampleHistory::Reset)
        if (!CheckNaN()) return false;
        std::vector<float> h;
        std::vector<int64_t> counts2;
        if (!Download(h, hist, stream) || !Download(counts2, hcount, stream)) return false;
        std::vector<int64_t> counts(C);
        std::vector<uint8_t> active(C);
        for (int64_t c = 0; c < C; c++) {
            counts[c] = counts2[2 * c];
            active[c] = temps_host[c] != 0.0;
        }
        std::vector<int32_t> nc(C), fit(C);
        std::vector<double> w(C * kmax), mu(C * kmax * d), L(C * kmax * d * d), lc(C * kmax);
        int nthreads = cfg.host_threads > 0 ? cfg.host_threads
                                            : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
        if (bcm3_adapt_proposals(kind, adjusted ? 1 : 0, (int)C, H, d, kmax, h.data(), counts.data(), active.data(),
                                 (size_t)cfg.adapt_proposal_max_history_samples, prior_mean.data(), prior_var.data(),
                                 cfg.seed, (uint64_t)cnt.adaptations_done, g0, nthreads, nc.data(), w.data(),
                                 mu.data(), L.data(), lc.data(), fit.data()) != 0)
            return false;
        // merge into the device state: adapted chains get the fit and a fresh proposal's scales
        std::vector<int32_t> dnc, dsel;
        std::vector<double> dw, dmu, dL, dlc, dsc, dem;
        if (!Download(dnc, ncomp, stream) || !Download(dsel, selected, stream) || !Download(dw, weights, stream) ||
            !Download(dmu, mean, stream) || !Download(dL, chol, stream) || !Download(dlc, logc, stream) ||
            !Download(dsc, scale, stream) || !Download(dem, ema, stream))
            return false;
        const bool gmm = kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE;
        const double s0 = gmm ? 2.38 / std::sqrt((double)d) : 1.0, e0 = gmm ? target : 0.23;
        for (int64_t c = 0; c < C; c++) {
            if (!active[c]) continue;
            dnc[c] = nc[c];
            dsel[c] = -1;
            std::copy(w.begin() + c * kmax, w.begin() + (c + 1) * kmax, dw.begin() + c * kmax);
            std::copy(mu.begin() + c * kmax * d, mu.begin() + (c + 1) * kmax * d, dmu.begin() + c * kmax * d);
            std::copy(L.begin() + c * kmax * d * d, L.begin() + (c + 1) * kmax * d * d, dL.begin() + c * kmax * d * d);
            std::copy(lc.begin() + c * kmax, lc.begin() + (c + 1) * kmax, dlc.begin() + c * kmax);
            std::fill(dsc.begin() + c * kmax, dsc.begin() + (c + 1) * kmax, s0);
            std::fill(dem.begin() + c * kmax, dem.begin() + (c + 1) * kmax, e0);
        }
        if (!Upload(ncomp, dnc, stream) || !Upload(selected, dsel, stream) || !Upload(weights, dw, stream) ||
            !Upload(mean, dmu, stream) || !Upload(chol, dL, stream) || !Upload(logc, dlc, stream) ||
            !Upload(scale, dsc, stream) || !Upload(ema, dem, stream) ||
            bcm3hip_memset_async(hcount.p, 0, hcount.n * sizeof(int64_t), stream) != 0)
            return false;
        // SamplerPTChain::AdaptProposal names the fit adapt<adaptation_iteration>: adapt0 is the
        // initial proposal (written by SetAdaptationOutput), so the k-th fit is adapt<k+1>, and every
        // fit carries the history it was fitted to (SamplerPTChain.cpp:149-166)
        if (!adapt_file.empty() && g0 + C == Ctot &&
            !WriteAdaptation(cnt.adaptations_done + 1, C - 1, nc, w, mu, L, &h, counts))
            return false;
        cnt.adaptations_done++;
        return bcm3hip_stream_synchronize(stream) == 0;
    }

    // adapt<index>/block1 of sampler_adaptation.nc for chain c's proposal; h == nullptr: no history
    // group (adapt0, the proposal before any fit)
    bool WriteAdaptation(int64_t index, int64_t c, const std::vector<int32_t>& nc, const std::vector<double>& w,
                         const std::vector<double>& mu, const std::vector<double>& L, const std::vector<float>* h,
                         const std::vector<int64_t>& counts)
    {
        const std::string g = "adapt" + std::to_string(index) + "/block1";
        std::vector<int32_t> ix(d);
        for (int j = 0; j < d; j++) ix[j] = j;
        adapt_out.AddVector(g, "variable_indices", ix);
        // covariance of component k = L_k L_k^T (the Cholesky factor the proposal state holds)
        auto cov = [&](int k) {
            std::vector<double> S((size_t)d * d, 0.0);
            const double* Lk = &L[(size_t)((c * kmax + k) * d * d)];
            for (int i = 0; i < d; i++)
                for (int j = 0; j < d; j++) {
                    double s = 0.0;
                    for (int m = 0; m <= std::min(i, j); m++) s += Lk[i * d + m] * Lk[j * d + m];
                    S[(size_t)i * d + j] = s;
                }
            return S;
        };
        if (kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
            const int K = nc[c];
            adapt_out.AddVector(g, "gmm_weights", std::vector<double>(w.begin() + c * kmax, w.begin() + c * kmax + K));
            for (int k = 0; k < K; k++) {
                const double* m = &mu[(size_t)((c * kmax + k) * d)];
                adapt_out.AddVector(g, "cluster" + std::to_string(k) + "_mean", std::vector<double>(m, m + d));
                adapt_out.AddMatrix(g, "cluster" + std::to_string(k) + "_covariance", d, d, cov(k));
            }
        } else {
            adapt_out.AddMatrix(g, "covariance", d, d, cov(0));
        }
        if (h) {
            // the history this adaptation was fitted to (rows as stored in the device ring)
            const int64_t rows = std::min<int64_t>(counts[c], H);
            std::vector<double> hist((size_t)(rows * d));
            for (int64_t r = 0; r < rows; r++)
                for (int j = 0; j < d; j++) hist[(size_t)(r * d + j)] = (*h)[(size_t)((c * H + r) * d + j)];
            adapt_out.AddMatrix(g, "history", (size_t)rows, (size_t)d, hist);
        }
        if (!adapt_out.Write(adapt_file)) {
            LOGERROR("Writing %s failed", adapt_file.c_str());
            return false;
        }
        return true;
    }
};

SamplerPTDevice::SamplerPTDevice() : p_(new Impl) {}

SamplerPTDevice::~SamplerPTDevice()
{
    if (p_ && p_->out_on && !p_->Flush()) LOGERROR("Flushing the sample output failed");
    if (p_ && p_->stream) bcm3hip_stream_synchronize(p_->stream);
    if (p_ && p_->own_stream) bcm3hip_stream_destroy(p_->stream);
}

bool SamplerPTDevice::Initialize(std::shared_ptr<Likelihood> ll, const std::vector<Marginal>& prior,
                                 const PTMHConfig& cfg, std::unique_ptr<Transport> transport, void* stream)
{
    Impl& s = *p_;
    s.cfg = cfg;
    s.ll = std::move(ll);
    s.transport = std::move(transport);
    s.d = (int)prior.size();
    s.Ctot = cfg.num_chains;
    if (!s.ll || s.d == 0 || s.Ctot < 1 || cfg.world < 1 || cfg.rank < 0 || cfg.rank >= cfg.world ||
        s.Ctot % cfg.world != 0 || s.ll->GetNumVariables() != (size_t)s.d) {
        LOGERROR("SamplerPTDevice: inconsistent configuration (chains %lld, ranks %d, variables %d / %zu)",
                 (long long)s.Ctot, cfg.world, s.d, s.ll ? s.ll->GetNumVariables() : (size_t)0);
        return false;
    }
    s.C = s.Ctot / cfg.world;
    if (cfg.world > 1 && (s.C % 2 != 0 || !s.transport)) {
        LOGERROR("SamplerPTDevice: a sharded ladder needs an even number of chains per rank and a transport");
        return false;
    }
    s.g0 = cfg.rank * s.C;
    C_ = s.C;
    d_ = s.d;
    if (cfg.use_every_nth < 1 || cfg.exploration_steps < 0 || cfg.initial_position_tries < 1 ||
        cfg.adapt_proposal_samples < 0 || cfg.adapt_proposal_times < 0 || cfg.max_history_size < 1 ||
        !(cfg.exchange_probability >= 0.0 && cfg.exchange_probability <= 1.0)) {
        LOGERROR("SamplerPTDevice: out-of-range setting (use_every_nth %d, exploration_steps %d, "
                 "initial_position_tries %d, adapt_proposal_samples %lld, adapt_proposal_times %lld, "
                 "max_history_size %lld, exchange_probability %g)",
                 (int)cfg.use_every_nth, (int)cfg.exploration_steps, (int)cfg.initial_position_tries,
                 (long long)cfg.adapt_proposal_samples, (long long)cfg.adapt_proposal_times,
                 (long long)cfg.max_history_size, cfg.exchange_probability);
        return false;
    }
    if (cfg.proposal < 0 || cfg.proposal > 3 || cfg.swapping_scheme < 0 || cfg.swapping_scheme > 2) {
        LOGERROR("SamplerPTDevice: unknown proposal type or swapping scheme");
        return false;
    }
    s.adaptive = cfg.proposal != 3;
    s.adjusted = cfg.proposal == 2;
    s.kind = (cfg.proposal == 0) ? BCM3HIP_PROPOSAL_GLOBAL_COVARIANCE : BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE;
    s.kmax = cfg.kmax > 0 ? cfg.kmax : (s.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE ? 13 : 1);
    if (s.kind == BCM3HIP_PROPOSAL_GLOBAL_COVARIANCE) s.kmax = 1;
    if (s.kmax > BCM3HIP_PROPOSAL_KMAX) return false;
    if (!s.adaptive) {
        for (auto& m : prior)
            if (m.kind != BCM3HIP_PRIOR_UNIFORM && m.kind != BCM3HIP_PRIOR_NORMAL) {
                LOGERROR("the random-walk proposal kernel supports uniform and normal priors only");
                return false;
            }
    }
    // Proposal::Initialize (Proposal.cpp:45-53)
    s.target = (s.d == 1) ? 0.44 : (s.d == 2) ? 0.35 : (s.d == 3) ? 0.3 : 0.234;
    const auto ladder = TemperatureLadder(s.Ctot, cfg.temperature_power, cfg.temperature_max);
    s.temps_host.assign(ladder.begin() + s.g0, ladder.begin() + s.g0 + s.C);

    if (stream) {
        s.stream = stream;
    } else {
        if (bcm3hip_stream_create(&s.stream) != 0) return false;
        s.own_stream = true;
    }
    stream_ = s.stream;
    const int64_t C = s.C, d = s.d, K = s.kmax;
    HistoryGeometry(cfg.adapt_proposal_samples, cfg.use_every_nth, cfg.exploration_steps, s.Ctot,
                    cfg.max_history_size, cfg.swapping_scheme == 0, s.H, s.sub);
    bool ok = s.pkind.alloc(d) && s.p0.alloc(d) && s.p1.alloc(d) && s.p2.alloc(d) && s.lower.alloc(d) &&
              s.upper.alloc(d) && s.rw_scale.alloc(d) && s.temps.alloc(C) && s.zeros.alloc(C) &&
              s.values.alloc(C * d) && s.prop.alloc(C * d) && s.lprior.alloc(C) && s.lprior_prop.alloc(C) &&
              s.llh.alloc(C) && s.llh_prop.alloc(C) && s.lpp.alloc(C) && s.log_mh.alloc(C) && s.status.alloc(C) &&
              s.nan_flag.alloc(1) && s.acc_mutate.alloc(1) && s.acc_exchange.alloc(1) && s.ncomp.alloc(C) &&
              s.selected.alloc(C) && s.weights.alloc(C * K) && s.mean.alloc(C * K * d) &&
              s.chol.alloc(C * K * d * d) && s.logc.alloc(C * K) && s.scale.alloc(C * K) && s.ema.alloc(C * K) &&
              s.work.alloc(C * (2 * K + 2 * d)) && s.hist.alloc(C * (int64_t)s.H * d) && s.hcount.alloc(2 * C) &&
              s.pair_mask.alloc(C) && s.send_last.alloc(d + 4) && s.send_first.alloc(d + 4) &&
              s.recv_next.alloc(d + 4) && s.recv_prev.alloc(d + 4);
    if (!ok) {
        LOGERROR("SamplerPTDevice: device allocation failed");
        return false;
    }
    std::vector<int32_t> kinds(d);
    std::vector<double> a0(d), a1(d), a2(d), lo(d), hi(d), rw(d);
    s.prior_mean.resize(d);
    s.prior_var.resize(d);
    for (int j = 0; j < d; j++) {
        kinds[j] = prior[j].kind;
        a0[j] = prior[j].p0;
        a1[j] = prior[j].p1;
        a2[j] = prior[j].p2;
        lo[j] = prior[j].lower;
        hi[j] = prior[j].upper;
        s.prior_mean[j] = prior[j].mean;
        s.prior_var[j] = prior[j].var;
        rw[j] = 0.05 * std::sqrt(prior[j].var);  // DevicePrior.scale
    }
    ok = Upload(s.pkind, kinds, s.stream) && Upload(s.p0, a0, s.stream) && Upload(s.p1, a1, s.stream) &&
         Upload(s.p2, a2, s.stream) && Upload(s.lower, lo, s.stream) && Upload(s.upper, hi, s.stream) &&
         Upload(s.rw_scale, rw, s.stream) && Upload(s.temps, s.temps_host, s.stream) &&
         bcm3hip_memset_async(s.zeros.p, 0, C * sizeof(double), s.stream) == 0 &&
         bcm3hip_memset_async(s.log_mh.p, 0, C * sizeof(double), s.stream) == 0 &&
         bcm3hip_memset_async(s.nan_flag.p, 0, sizeof(int32_t), s.stream) == 0 &&
         bcm3hip_memset_async(s.acc_mutate.p, 0, sizeof(uint64_t), s.stream) == 0 &&
         bcm3hip_memset_async(s.acc_exchange.p, 0, sizeof(uint64_t), s.stream) == 0 &&
         bcm3hip_memset_async(s.hist.p, 0, s.hist.n * sizeof(float), s.stream) == 0 &&
         bcm3hip_memset_async(s.hcount.p, 0, s.hcount.n * sizeof(int64_t), s.stream) == 0;
    if (!ok) return false;
    s.P.kind = s.kind;
    s.P.kmax = (int32_t)K;
    s.P.t_dof = cfg.t_dof;
    s.P.target_acceptance = s.target;
    s.P.scaling_learning_rate = 0.05;
    s.P.scaling_ema_period = 1000.0;
    s.P.lower = s.lower.p;
    s.P.upper = s.upper.p;
    s.P.ncomp = s.ncomp.p;
    s.P.weights = s.weights.p;
    s.P.mean = s.mean.p;
    s.P.chol = s.chol.p;
    s.P.logc = s.logc.p;
    s.P.scale = s.scale.p;
    s.P.ema = s.ema.p;
    s.P.selected = s.selected.p;
    s.P.work = s.work.p;
    if (!s.InitProposal()) return false;
    for (int start = 0; start < 2; start++) {
        auto m = ExchangeParticipants(C, s.g0, s.Ctot, cfg.world, start, s.mask_all[start]);
        for (auto& v : m) {
            s.masks[start].emplace_back(new DevBuf<uint8_t>());
            if (!s.masks[start].back()->alloc(C) || !Upload(*s.masks[start].back(), v, s.stream)) return false;
        }
    }
    if (!s.SetupSpeculation()) return false;
    return s.InitialPositions() && bcm3hip_stream_synchronize(s.stream) == 0;
}

bool SamplerPTDevice::Iterate(int64_t n, bool last_at_end) { return p_->Iterations(n, last_at_end, 0); }

bool SamplerPTDevice::Run(int64_t num_samples)
{
    const int64_t total = num_samples * p_->cfg.use_every_nth;
    return p_->Iterations(total, true, p_->cfg.nan_check_every) && p_->CheckNaN() && FlushOutput();
}

bool SamplerPTDevice::AdaptProposal() { return p_->Adapt(); }

int64_t SamplerPTDevice::SpeculativeBatch(int32_t* src, int32_t* steps, int32_t* hint_of_src)
{
    Impl& s = *p_;
    if (!s.spec_on) return -1;
    std::vector<int32_t> n, bs, bt, cand_active;
    if (!Download(n, s.sp_batch_n, s.stream) || !Download(bs, s.sp_batch_src, s.stream) ||
        !Download(bt, s.sp_batch_steps, s.stream))
        return -1;
    for (int32_t i = 0; i < n[0]; i++) {
        if (src) src[i] = bs[i];
        if (steps) steps[i] = bt[i];
    }
    (void)hint_of_src;
    return n[0];
}

bool SamplerPTDevice::SetOutput(const std::string& filename, int64_t num_samples, int flush_every)
{
    Impl& s = *p_;
    const VariableSet* vs = s.ll ? s.ll->GetVariableSet() : nullptr;
    if (!vs || num_samples < 1 || s.emitted != 0 || s.out_on) {
        LOGERROR("SetOutput: needs an initialised sampler before its first sample, once");
        return false;
    }
    std::vector<std::string> names(vs->GetVariableNames());
    std::vector<int32_t> tr(names.size());
    for (size_t i = 0; i < names.size(); i++) tr[i] = (int32_t)vs->GetVariableTransform(i);
    // a sharded ladder: the reference's netCDF-4 file (SampleHandlerNetCDF.cpp:24-110) written by rank 0
    // from every rank's rows when libnetcdf can be loaded; otherwise the shared netCDF classic file,
    // each rank writing its own temperature columns
    // Rank 0 decides (only its libnetcdf matters: it alone writes the gathered file) and tells every
    // other rank over the transport, together with whether its writer opened, so the ranks never
    // disagree on the mode nor wait at a flush for rows a failed rank 0 will not take.
    const std::vector<double> ladder = TemperatureLadder(s.Ctot, s.cfg.temperature_power, s.cfg.temperature_max);
    std::unique_ptr<SampleFileWriter> w;
    bool gather = false;
    auto open_writer = [&](bool all) {
        w = std::make_unique<SampleFileWriter>();
        return all ? w->Initialize(filename, (size_t)num_samples, names, tr, ladder, 0, (size_t)s.Ctot)
                   : w->Initialize(filename, (size_t)num_samples, names, tr, ladder, (size_t)s.g0, (size_t)s.C);
    };
    if (s.cfg.world > 1 && s.transport) {
        double code = 0.0;  // rank 0's decision: 1 gather, 0 every rank its own columns, -1 rank 0 failed
        if (s.cfg.rank == 0) {
            gather = NcNetCDF4WriteAvailable(nullptr);
            code = open_writer(gather) ? (gather ? 1.0 : 0.0) : -1.0;
        }
        DevBuf<double> msg;
        if (!msg.alloc(1)) return false;
        std::vector<const double*> sends;
        std::vector<int> speer;
        double* recv = msg.p;
        const int from0 = 0;
        bool ok;
        if (s.cfg.rank == 0) {
            ok = bcm3hip_memcpy_async(msg.p, &code, sizeof(double), BCM3HIP_H2D, s.stream) == 0;
            for (int r = 1; r < s.cfg.world; r++) {
                sends.push_back(msg.p);
                speer.push_back(r);
            }
            ok = ok && s.transport->Exchange((int)sends.size(), sends.data(), speer.data(), 0, nullptr, nullptr, 1,
                                             s.stream) &&
                 bcm3hip_stream_synchronize(s.stream) == 0;
        } else {
            ok = s.transport->Exchange(0, nullptr, nullptr, 1, &recv, &from0, 1, s.stream) &&
                 bcm3hip_memcpy_async(&code, msg.p, sizeof(double), BCM3HIP_D2H, s.stream) == 0 &&
                 bcm3hip_stream_synchronize(s.stream) == 0;
        }
        if (!ok || code < 0.0) {
            LOGERROR("SetOutput: %s", ok ? "rank 0 could not open the sample file" : "the transport failed");
            return false;
        }
        gather = code > 0.0;
        if (!gather && s.cfg.rank != 0 && !open_writer(false)) return false;
    } else if (!open_writer(false)) {
        return false;
    }
    s.out_flush = std::max(1, flush_every);
    if (!s.out_buf.alloc((size_t)(s.out_flush * s.C * (s.d + 2)))) return false;
    if (gather && s.cfg.rank == 0 &&
        !s.out_recv.alloc((size_t)((s.cfg.world - 1) * s.out_flush * s.C * (s.d + 2))))
        return false;
    s.out = std::move(w);
    s.out_on = true;
    s.out_gather = gather;
    s.out_samples = num_samples;
    s.out_pending = 0;
    return true;
}

bool SamplerPTDevice::SetAdaptationOutput(const std::string& filename)
{
    if (filename.empty() || !p_->adaptive) {
        LOGERROR("SetAdaptationOutput: needs a file name and an adaptive proposal");
        return false;
    }
    Impl& s = *p_;
    s.adapt_file = filename;
    if (s.cnt.adaptations_done > 0 || s.g0 + s.C != s.Ctot) return true;
    // adapt0: the hottest chain's initial proposal (SamplerPTChain::Initialize -> AdaptProposal(0) with
    // an empty history: the prior-moment proposal InitProposal uploaded), no history group
    std::vector<int32_t> dnc;
    std::vector<double> dw, dmu, dL;
    if (!Download(dnc, s.ncomp, s.stream) || !Download(dw, s.weights, s.stream) || !Download(dmu, s.mean, s.stream) ||
        !Download(dL, s.chol, s.stream))
        return false;
    return s.WriteAdaptation(0, s.C - 1, dnc, dw, dmu, dL, nullptr, std::vector<int64_t>());
}

bool SamplerPTDevice::FlushOutput() { return p_->Flush() && (!p_->out || p_->out->Sync()); }
bool SamplerPTDevice::CheckNaN() { return p_->CheckNaN(); }
bool SamplerPTDevice::Synchronize() { return bcm3hip_stream_synchronize(p_->stream) == 0; }

bool SamplerPTDevice::GetState(double* values, double* llh, double* lprior, double* lpp)
{
    Impl& s = *p_;
    auto get = [&](double* out, const DevBuf<double>& b) {
        return !out || bcm3hip_memcpy_async(out, b.p, b.n * sizeof(double), BCM3HIP_D2H, s.stream) == 0;
    };
    return get(values, s.values) && get(llh, s.llh) && get(lprior, s.lprior) && get(lpp, s.lpp) &&
           bcm3hip_stream_synchronize(s.stream) == 0;
}

bool SamplerPTDevice::GetProposalComponents(int32_t* nc)
{
    return nc && bcm3hip_memcpy_async(nc, p_->ncomp.p, p_->C * sizeof(int32_t), BCM3HIP_D2H, p_->stream) == 0 &&
           bcm3hip_stream_synchronize(p_->stream) == 0;
}

PTMHCounters SamplerPTDevice::GetCounters()
{
    Impl& s = *p_;
    PTMHCounters c = s.cnt;
    uint64_t a = 0, b = 0;
    if (bcm3hip_memcpy_async(&a, s.acc_mutate.p, sizeof(a), BCM3HIP_D2H, s.stream) == 0 &&
        bcm3hip_memcpy_async(&b, s.acc_exchange.p, sizeof(b), BCM3HIP_D2H, s.stream) == 0 &&
        bcm3hip_stream_synchronize(s.stream) == 0) {
        c.accepted_mutate = (int64_t)a;
        c.accepted_exchange = (int64_t)b;
    }
    c.rounds = s.round;
    if (s.spec_on) {
        int64_t t = 0;
        if (bcm3hip_memcpy_async(&t, s.sp_total.p, sizeof(t), BCM3HIP_D2H, s.stream) == 0 &&
            bcm3hip_stream_synchronize(s.stream) == 0)
            c.evaluated_entries += t;
    }
    return c;
}

}  // namespace bcm3
