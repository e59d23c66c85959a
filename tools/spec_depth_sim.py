"""Deeper speculation, simulated before building it (VERDICT r03 "next" 3).

The C3 headline runs speculative iteration PAIRS: one likelihood launch evaluates iteration r's
proposals and every candidate proposal of r+1. This script asks whether a THIRD
level pays: one launch over r's proposals, the candidates of r+1 and those of r+2 (three committed
iterations per launch), either
  (a) with every level-2 candidate, or only those of the most probable level-1 outcomes plus a
      fallback launch for the chains whose actual state was not covered, or
  (b) with a kernel variant limited to 128 VGPRs (4 wavefronts per SIMD instead of 2), so the
      larger batch has SIMD slots.

Model (all inputs measured and committed):
  * a trajectory's BDF step count: the reference CVODE's counts of 8,192 C3 prior draws
    (tests/golden/c3_golden_llh.npz; the sampler's batches have the same mean, 985 vs 995 steps,
    profiles/r03k_spec_sim.txt);
  * time per step alone on a SIMD: calibrated so that the plain 256-trajectory launch takes the
    measured 1.479 ms (the model then gives 1.58 ms for the pairs' ~1,295 entries, measured 1.58-1.61);
    sharing a SIMD with a second wavefront costs +16..51 % per step (profiles/r03j_placement.txt:
    BCM3HIP_OPT_PLACEMENT_LOG, hardware HW_ID of every trajectory);
    k wavefronts on a SIMD: alone x (1 + 0.40 (k - 1)) (the measured 2-wave factor, extrapolated
    linearly -- optimistic for k > 2, since one SIMD issues one instruction per cycle for all
    its waves and each wave issues every ~6 cycles alone);
  * dispatch: 1,024 SIMDs, a wavefront placed on the least loaded SIMD with a free slot, longest
    predicted solve first (the kNN predictor's rank correlation 0.84 is modelled as the true
    length times log-normal noise of sd 0.25);
  * candidates per chain: level 1 as the sampler measures it (1,295 entries for 256 chains:
    ~4.06 per chain); level 2: for each of the chain's r+1 states (its level-1 candidate
    accepted or not) and its r+2 exchange partner's states -- 2 x 4.06 own + 2 x 4.06 partner
    states, ~16 per chain before EMA variants; pruned: the level-2 candidates of the level-1
    outcome that happened with probability p_hit per chain (mutate acceptance 0.47 from the bench,
    exchange acceptance 0.85 from the sampler's counters, r03 bench lines), plus one fallback launch
    of the missed chains' actual proposals when any chain misses.
Each configuration is simulated over 60 launches; committed evaluations per second of kernel
time is the figure of merit (iteration overheads outside the launch are ~8 % either way).

    python tools/spec_depth_sim.py        (CPU only; writes nothing)
"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NSIMD = 1024
SHARE = 0.40        # per extra co-resident wavefront


def makespan(steps, slots, rng, t_alone, noise=0.25, vgpr_slow=1.0):
    """event simulation of one launch: wavefronts ordered by predicted length; up to 2 x NSIMD
    entries use the sampler's SIMD-aware layout (the 2R - M longest alone, the others paired), more
    entries fill every slot longest first and the rest start as slots free up; a wavefront on a
    SIMD with k residents advances at 1 / (t_alone vgpr_slow (1 + SHARE (k - 1))) steps per ms"""
    n = len(steps)
    pred = steps * np.exp(rng.normal(0.0, noise, n))
    rem_sorted = steps[np.argsort(-pred)].astype(float)
    res = np.full((NSIMD, slots), np.inf)
    if n <= 2 * NSIMD and slots >= 2:
        alone = max(0, min(n, 2 * NSIMD - n))
        res[:alone, 0] = rem_sorted[:alone]
        rest = rem_sorted[alone:]
        pairs = (len(rest) + 1) // 2
        res[alone:alone + pairs, 0] = rest[:pairs]
        res[alone:alone + len(rest) - pairs, 1] = rest[pairs:]
        queue = np.array([])
    else:
        first = min(n, NSIMD * slots)
        k = 0
        for r in range(slots):
            take = min(NSIMD, first - k)
            if take <= 0:
                break
            res[:take, r] = rem_sorted[k:k + take]
            k += take
        queue = rem_sorted[first:]
    qi, t = 0, 0.0
    per = t_alone * vgpr_slow
    while True:
        occ = np.isfinite(res)
        kk = occ.sum(axis=1)
        if kk.sum() == 0:
            return t
        rate = np.where(kk > 0, 1.0 / (per * (1.0 + SHARE * np.maximum(kk - 1, 0))), 0.0)
        mn = np.min(res, axis=1)
        dt = np.where(kk > 0, mn / np.where(rate > 0, rate, 1.0), np.inf)
        best = dt.min()
        t += best
        res = res - (rate * best)[:, None]
        res[res <= 1e-9] = np.inf
        if qi < len(queue):
            free = np.argwhere(~np.isfinite(res))
            for s, r in free:
                if qi >= len(queue):
                    break
                res[s, r] = queue[qi]
                qi += 1


def main():
    rng = np.random.default_rng(4)
    z = np.load(os.path.join(ROOT, "tests", "golden", "c3_golden_llh.npz"))
    pool = z["nst"][z["ok"].astype(bool)].astype(float)
    C = 256
    L1 = 4.06  # level-1 candidates per chain (sampler: 1,295 entries for 256 chains)
    p_acc, p_exc = 0.47, 0.85
    reps = 60

    # per-step time calibrated so that the plain 256-trajectory launch takes the measured 1.479 ms
    # (profiles/r03k_spec_sim.txt; its slowest trajectory sets it)
    t_alone = 1.479 / np.mean([np.max(rng.choice(pool, C)) for _ in range(2000)])

    def sim(n_entries, slots, vgpr_slow=1.0):
        return np.mean([makespan(rng.choice(pool, int(n_entries)), slots, rng, t_alone, vgpr_slow=vgpr_slow)
                        for _ in range(reps)])

    plain = sim(C, 2)
    pairs = sim(C * (1 + L1), 2)
    L2_full = 2 * L1 + 2 * L1
    triple_full = sim(C * (1 + L1 + L2_full), 2)
    triple_full_4w = sim(C * (1 + L1 + L2_full), 4, vgpr_slow=1.10)
    # pruned: level-2 candidates of the single most probable level-1 outcome per chain (own reject,
    # the exchange accepted): covers a chain with probability p_hit
    p_hit = (1 - p_acc) * p_exc + (1 - p_exc) * (1 - p_acc)
    L2_pruned = 4.0
    miss_all = 1.0 - p_hit ** C
    triple_pruned = sim(C * (1 + L1 + L2_pruned), 2)
    fallback = sim(max(1, C * (1 - p_hit)), 2)
    triple_pruned_eff = triple_pruned + miss_all * fallback
    rows = [("plain (one launch per iteration)", C, plain, 1),
            ("pairs (built, r03)", C * (1 + L1), pairs, 2),
            ("triples, every level-2 candidate, 2 waves/SIMD", C * (1 + L1 + L2_full), triple_full, 3),
            ("triples, every level-2 candidate, <=128 VGPR (4 waves/SIMD, +10 % per step)", C * (1 + L1 + L2_full),
             triple_full_4w, 3),
            (f"triples, pruned to the likeliest outcome (p_hit {p_hit:.2f}/chain) + fallback "
             f"(needed in {100 * miss_all:.0f} % of launches)", C * (1 + L1 + L2_pruned), triple_pruned_eff, 3)]
    print(f"step-count pool: {len(pool)} C3 prior draws, mean {pool.mean():.0f}, p99 {np.percentile(pool, 99):.0f}, "
          f"max {pool.max():.0f}; {NSIMD} SIMDs, {t_alone * 1e3:.3f} us/step alone (calibrated: plain launch "
          f"1.479 ms as measured), +{SHARE:.2f} per co-resident wave")
    print("measured for reference (profiles/r03k_spec_sim.txt, r03z): plain 1.479 ms, pairs 1.58-1.61 ms")
    print(f"{'configuration':90s} {'entries':>8s} {'launch ms':>10s} {'iters':>6s} {'committed evals/s':>18s} {'vs pairs':>9s}")
    base = C * 2 / (pairs * 1e-3)
    for name, n, ms, it in rows:
        rate = C * it / (ms * 1e-3)
        print(f"{name:90s} {n:8.0f} {ms:10.3f} {it:6d} {rate:18.0f} {rate / base:9.2f}")


if __name__ == "__main__":
    main()
