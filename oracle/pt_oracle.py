"""TEST INFRASTRUCTURE ONLY -- sequential CPU restatement of the reference's even/odd exchange.

Follows SamplerPT::DoExchangeMove (src/sampler/SamplerPT.cpp:277-298: start index alternates
0,1,0,... because previous_swap_even starts false, :30; pair (ci, ci+1), ix2 == C -> 0) and
SamplerPTChain::ExchangeMove (src/sampler/SamplerPTChain.cpp:328-381) in one process, one pair
after the other, exactly as the reference loops. The only substitution is the acceptance uniform:
the reference draws sampler->rng.GetReal() (ranlux48) in pair order; here it is the
counter-based uniform of bcm3_amd.pt.exchange_uniform(seed, round, ci), the same number the
sharded GPU implementation uses, so decisions can be compared bit for bit.
"""
import math


def exchange_round(chains, temps, rnd, seed, uniform):
    """chains: list of dicts {values(list), llh, lprior, lpp}; mutated in place.
    Returns list of (ci, ix2, accepted)."""
    C = len(chains)
    start = rnd % 2
    out = []
    ci = start
    while ci < C:
        ix2 = ci + 1
        if ix2 == C:
            ix2 = 0
        c1, c2 = chains[ci], chains[ix2]
        t1, t2 = temps[ci], temps[ix2]
        p1 = c2["lprior"] if t1 == 0.0 else t1 * c2["llh"] + c2["lprior"]
        p2 = c1["lprior"] if t2 == 0.0 else t2 * c1["llh"] + c1["lprior"]
        x = (p1 + p2) - (c1["lpp"] + c2["lpp"])
        # tp = std::min((Real)1.0, exp(x)) == (exp(x) < 1 ? exp(x) : 1): a NaN x gives 1
        if math.isnan(x) or x >= 0.0:
            tp = 1.0
        else:
            tp = math.exp(x)
            tp = tp if tp < 1.0 else 1.0
        alpha = uniform(seed, rnd, ci)
        acc = alpha < tp
        if acc:
            for k in ("values", "llh", "lprior"):
                c1[k], c2[k] = c2[k], c1[k]
            c1["lpp"], c2["lpp"] = p1, p2
        out.append((ci, ix2, acc))
        ci += 2
    return out


def exchange_single(chains, temps, ci, rnd, seed, uniform):
    """stochastic_random (SamplerPT.cpp:300-305): ExchangeMove of the pair (ci, ci + 1) only."""
    c1, c2 = chains[ci], chains[ci + 1]
    t1, t2 = temps[ci], temps[ci + 1]
    p1 = c2["lprior"] if t1 == 0.0 else t1 * c2["llh"] + c2["lprior"]
    p2 = c1["lprior"] if t2 == 0.0 else t2 * c1["llh"] + c1["lprior"]
    x = (p1 + p2) - (c1["lpp"] + c2["lpp"])
    if math.isnan(x) or x >= 0.0:
        tp = 1.0
    else:
        tp = math.exp(x)
        tp = tp if tp < 1.0 else 1.0
    acc = uniform(seed, rnd, ci) < tp
    if acc:
        for k in ("values", "llh", "lprior"):
            c1[k], c2[k] = c2[k], c1[k]
        c1["lpp"], c2["lpp"] = p1, p2
    return acc
