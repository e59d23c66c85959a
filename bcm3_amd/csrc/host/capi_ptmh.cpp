// capi_ptmh.cpp -- include/bcm3.h's sampler entry points (bcm3_ptmh_*) on SamplerPTDevice.
#include <cstring>
#include <memory>

#include "../../../include/bcm3.h"
#include "../../../include/bcm3hip.h"
#include "Config.h"
#include "Likelihood.h"
#include "Prior.h"
#include "SamplerPTDevice.h"
#include "log.h"

#include "capi_internal.h"

struct bcm3_ptmh {
    bcm3::SamplerPTDevice s;
};

struct bcm3_ptmh_group {
    std::shared_ptr<bcm3::LocalGroup> g;
};

extern "C" {

void bcm3_ptmh_config_default(bcm3_ptmh_config* c)
{
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    const bcm3::PTMHConfig d;
    c->num_chains = d.num_chains;
    c->rank = 0;
    c->world = 1;
    c->temperature_power = d.temperature_power;
    c->temperature_max = d.temperature_max;
    c->seed = 0;
    c->learning_rate = d.learning_rate;
    c->exploration_steps = d.exploration_steps;
    c->proposal = BCM3_PTMH_GAUSSIAN_MIXTURE;
    c->t_dof = 0.0;
    c->kmax = 0;
    c->adapt_proposal_samples = d.adapt_proposal_samples;
    c->adapt_proposal_times = d.adapt_proposal_times;
    c->max_history_size = d.max_history_size;
    c->adapt_proposal_max_history_samples = d.adapt_proposal_max_history_samples;
    c->use_every_nth = d.use_every_nth;
    c->swapping_scheme = BCM3_PTMH_DETERMINISTIC_EVEN_ODD;
    c->exchange_probability = d.exchange_probability;
    c->initial_position_tries = d.initial_position_tries;
    c->nan_check_every = d.nan_check_every;
    c->host_threads = 0;
    c->speculate = d.speculate;
    c->transport = BCM3_PTMH_TRANSPORT_NONE;
}

static bool CopyString(char* dst, size_t cap, const std::string& src, const char* what)
{
    if (src.size() + 1 > cap) {
        LOGERROR("config: %s is longer than %zu characters", what, cap - 1);
        return false;
    }
    std::memcpy(dst, src.c_str(), src.size() + 1);
    return true;
}

int bcm3_run_config_from_file(const char* path, bcm3_run_config* out)
{
    if (!path || !out) return -1;
    bcm3::RunConfig rc;
    if (!bcm3::LoadRunConfig(path, rc)) return -2;
    bcm3_run_config r;
    std::memset(&r, 0, sizeof(r));
    bcm3_ptmh_config_default(&r.ptmh);
    const bcm3::PTMHConfig& p = rc.ptmh;
    r.ptmh.num_chains = p.num_chains;
    r.ptmh.temperature_power = p.temperature_power;
    r.ptmh.temperature_max = p.temperature_max;
    r.ptmh.seed = p.seed;
    r.ptmh.learning_rate = p.learning_rate;
    r.ptmh.exploration_steps = p.exploration_steps;
    r.ptmh.proposal = p.proposal;
    r.ptmh.t_dof = p.t_dof;
    r.ptmh.adapt_proposal_samples = p.adapt_proposal_samples;
    r.ptmh.adapt_proposal_times = p.adapt_proposal_times;
    r.ptmh.max_history_size = p.max_history_size;
    r.ptmh.adapt_proposal_max_history_samples = p.adapt_proposal_max_history_samples;
    r.ptmh.use_every_nth = p.use_every_nth;
    r.ptmh.swapping_scheme = p.swapping_scheme;
    r.ptmh.exchange_probability = p.exchange_probability;
    r.ptmh.initial_position_tries = p.initial_position_tries;
    r.ptmh.host_threads = p.host_threads;
    r.num_samples = rc.num_samples;
    r.output_proposal_adaptation = rc.output_proposal_adaptation ? 1 : 0;
    r.sampling_threads = rc.sampling_threads;
    r.evaluation_threads = rc.evaluation_threads;
    if (!CopyString(r.sampler_type, sizeof(r.sampler_type), rc.sampler_type, "sampler.type") ||
        !CopyString(r.prior, sizeof(r.prior), rc.prior, "prior") ||
        !CopyString(r.likelihood, sizeof(r.likelihood), rc.likelihood, "likelihood") ||
        !CopyString(r.output_folder, sizeof(r.output_folder), rc.output_folder, "output.folder") ||
        !CopyString(r.likelihood_options, sizeof(r.likelihood_options), rc.likelihood_options, "likelihood options"))
        return -2;
    *out = r;
    return 0;
}

int bcm3_ptmh_config_from_file(const char* path, bcm3_ptmh_config* cfg)
{
    if (!path || !cfg) return -1;
    bcm3_run_config r;
    const int rc = bcm3_run_config_from_file(path, &r);
    if (rc != 0) return rc;
    *cfg = r.ptmh;
    return 0;
}

int bcm3_ptmh_nccl_unique_id(void* id) { return bcm3hip_nccl_get_unique_id(id) == 0 ? 0 : -2; }

int bcm3_ptmh_group_create(int world, bcm3_ptmh_group** out)
{
    if (world < 1 || !out) return -1;
    *out = new bcm3_ptmh_group{bcm3::MakeLocalGroup(world)};
    return 0;
}

void bcm3_ptmh_group_destroy(bcm3_ptmh_group* g) { delete g; }

int bcm3_ptmh_create(bcm3_likelihood* ll, const char* prior_xml, const bcm3_ptmh_config* c, void* stream,
                     bcm3_ptmh** out)
{
    if (!ll || !prior_xml || !c || !out) return -1;
    *out = nullptr;
    std::vector<bcm3::Marginal> prior;
    if (!bcm3::LoadPriorMarginals(prior_xml, prior)) return -2;
    bcm3::PTMHConfig cfg;
    cfg.num_chains = c->num_chains;
    cfg.rank = c->rank;
    cfg.world = c->world;
    cfg.temperature_power = c->temperature_power;
    cfg.temperature_max = c->temperature_max;
    cfg.seed = c->seed;
    cfg.learning_rate = c->learning_rate;
    cfg.exploration_steps = c->exploration_steps;
    cfg.proposal = c->proposal;
    cfg.t_dof = c->t_dof;
    cfg.kmax = c->kmax;
    cfg.adapt_proposal_samples = c->adapt_proposal_samples;
    cfg.adapt_proposal_times = c->adapt_proposal_times;
    cfg.max_history_size = c->max_history_size;
    cfg.adapt_proposal_max_history_samples = c->adapt_proposal_max_history_samples;
    cfg.use_every_nth = c->use_every_nth;
    cfg.swapping_scheme = c->swapping_scheme;
    cfg.exchange_probability = c->exchange_probability;
    cfg.initial_position_tries = c->initial_position_tries;
    cfg.nan_check_every = c->nan_check_every;
    cfg.host_threads = c->host_threads;
    cfg.speculate = c->speculate;
    std::unique_ptr<bcm3::Transport> tr;
    if (c->world > 1) {
        if (c->transport == BCM3_PTMH_TRANSPORT_RCCL) {
            tr = bcm3::MakeRcclTransport(c->nccl_id, c->rank, c->world);
        } else if (c->transport == BCM3_PTMH_TRANSPORT_LOCAL && c->group) {
            tr = bcm3::MakeLocalTransport(c->group->g, c->rank);
        } else if (c->transport == BCM3_PTMH_TRANSPORT_SOCKET) {
            tr = bcm3::MakeSocketTransport(std::string(c->socket_dir, strnlen(c->socket_dir, sizeof(c->socket_dir))),
                                           c->rank, c->world);
        }
        if (!tr) {
            LOGERROR("bcm3_ptmh_create: %d ranks need a transport", c->world);
            return -3;
        }
    }
    auto h = std::make_unique<bcm3_ptmh>();
    if (!h->s.Initialize(ll->ll, prior, cfg, std::move(tr), stream)) return -4;
    *out = h.release();
    return 0;
}

int bcm3_ptmh_iterate(bcm3_ptmh* h, int64_t n, int last_at_end)
{
    return (h && h->s.Iterate(n, last_at_end != 0)) ? 0 : -2;
}

int bcm3_ptmh_run(bcm3_ptmh* h, int64_t num_samples) { return (h && h->s.Run(num_samples)) ? 0 : -2; }

int64_t bcm3_ptmh_spec_batch_info(bcm3_ptmh* h, int32_t* src, int32_t* steps)
{
    return h ? h->s.SpeculativeBatch(src, steps, nullptr) : -1;
}

int bcm3_ptmh_adapt(bcm3_ptmh* h) { return (h && h->s.AdaptProposal()) ? 0 : -2; }

int bcm3_ptmh_synchronize(bcm3_ptmh* h) { return (h && h->s.Synchronize() && h->s.CheckNaN()) ? 0 : -2; }

int bcm3_ptmh_num_chains(const bcm3_ptmh* h) { return h ? (int)h->s.NumLocalChains() : -1; }

int bcm3_ptmh_get_state(bcm3_ptmh* h, double* values, double* llh, double* lprior, double* lpp)
{
    return (h && h->s.GetState(values, llh, lprior, lpp)) ? 0 : -2;
}

int bcm3_ptmh_set_output(bcm3_ptmh* h, const char* filename, int64_t num_samples, int32_t flush_every)
{
    if (!h || !filename) return -1;
    return h->s.SetOutput(filename, num_samples, flush_every) ? 0 : -2;
}

int bcm3_ptmh_flush_output(bcm3_ptmh* h) { return (h && h->s.FlushOutput()) ? 0 : -2; }

int bcm3_ptmh_set_adaptation_output(bcm3_ptmh* h, const char* filename)
{
    if (!h || !filename) return -1;
    return h->s.SetAdaptationOutput(filename) ? 0 : -2;
}

int bcm3_ptmh_get_components(bcm3_ptmh* h, int32_t* ncomp) { return (h && h->s.GetProposalComponents(ncomp)) ? 0 : -2; }

int bcm3_ptmh_get_counters(bcm3_ptmh* h, int64_t* out)
{
    if (!h || !out) return -1;
    const bcm3::PTMHCounters c = h->s.GetCounters();
    const int64_t v[BCM3_PTMH_NUM_COUNTERS] = {c.attempted_mutate,   c.accepted_mutate, c.attempted_exchange,
                                               c.accepted_exchange,  c.samples_done,    c.adaptations_done,
                                               c.iterations,         c.rounds,
                                               c.likelihood_launches, c.evaluated_entries};
    std::memcpy(out, v, sizeof(v));
    return 0;
}

void* bcm3_ptmh_stream(const bcm3_ptmh* h) { return h ? h->s.Stream() : nullptr; }

void bcm3_ptmh_destroy(bcm3_ptmh* h) { delete h; }

}  // extern "C"
