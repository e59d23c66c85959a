"""TEST INFRASTRUCTURE ONLY -- numpy restatement of bcm3_amd/csrc/pt_kernels.hip (same counter-based
random numbers), itself a restatement of SamplerPTChain::MutateMove / TestSample / ExchangeMove
(src/sampler/SamplerPTChain.cpp:217-381, 465-481) and SamplerPT::DoExchangeMove
(src/sampler/SamplerPT.cpp:277-298)."""
import math

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _u(x):
    return np.asarray(x, dtype=np.uint64)


def splitmix64(x):
    with np.errstate(over="ignore"):
        x = _u(x) + np.uint64(0x9E3779B97F4A7C15)
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rng_key(seed, it, chain, slot):
    with np.errstate(over="ignore"):
        return splitmix64(splitmix64(_u(seed)) ^ (_u(it) * np.uint64(0x100000001B3)) ^
                          (_u(chain) * np.uint64(0xC2B2AE3D27D4EB4F)) ^ (_u(slot) * np.uint64(0x165667B19E3779F9)))


def u01(z):
    return (_u(z) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal01(seed, it, chain, slot):
    u1 = 1.0 - u01(rng_key(seed, it, chain, 2 * slot))
    u2 = u01(rng_key(seed, it, chain, 2 * slot + 1))
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(6.283185307179586 * u2)


def propose(kind, p0, p1, scale, temps, values, chain0, seed, it):
    C, d = values.shape
    prop = np.empty_like(values)
    lp = np.zeros(C)
    for c in range(C):
        gc = chain0 + c
        for i in range(d):
            if temps[c] == 0.0:
                if kind[i] == 0:
                    x = p0[i] + float(u01(rng_key(seed, it, gc, 0x8000 + i))) * (p1[i] - p0[i])
                else:
                    x = p0[i] + p1[i] * float(normal01(seed, it, gc, 0x2000 + i))
            else:
                x = values[c, i] + scale[i] * float(normal01(seed, it, gc, i))
            prop[c, i] = x
            if kind[i] == 0:
                l = -math.inf if (x < p0[i] or x > p1[i]) else -math.log(p1[i] - p0[i])
            else:
                s = p1[i]
                dx = x - p0[i]
                l = math.log(1.0 / math.sqrt(2.0 * s * s * 3.141592653589793)) - dx * dx * (1.0 / (2.0 * s * s))
            lp[c] += l
    return prop, lp


def accept(temps, prop, lprior_prop, llh_prop, lr, values, lprior, llh, lpp, chain0, seed, it):
    """In place; returns the accept mask."""
    C = len(temps)
    acc = np.zeros(C, dtype=bool)
    for c in range(C):
        T = temps[c]
        nl = llh_prop[c] * lr
        nq = lprior_prop[c]
        if math.isnan(nl):  # Sampler.cpp:172-178: fatal; the kernel flags it and keeps the chain
            a, npp = False, 0.0
        elif T == 0.0:
            a = True
            npp = nq if nl == -math.inf else nq + T * nl
        else:
            npp = nq + T * nl
            a = False
            if npp > -math.inf:
                with np.errstate(invalid="ignore", over="ignore"):
                    tp = np.exp(npp - lpp[c])
                tp = tp if tp < 1.0 else 1.0
                a = float(u01(rng_key(seed, it, chain0 + c, 0xC000))) < tp
        if a:
            values[c] = prop[c]
            lprior[c], llh[c], lpp[c] = nq, nl, npp
        acc[c] = a
    return acc
