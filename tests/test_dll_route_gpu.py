"""The reference's zero-change route to the GPU: single-vector EvaluateLogProbability calls from
many sampling threads at once (TaskManager, README.md:77 re-entrancy) -- through libbcm3.so and
through the LikelihoodDLL plugin libbcm3_dll.so -- are combined into batched launches, with each
result equal to the batched evaluation of its own vector and inside the parity envelope of the
oracle (the reference's CVODE restated bit for bit, tests/parity.py)."""
import ctypes as C
import os
import threading

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIK = os.path.join(H.GOLDEN, "c3_likelihood.xml")
PRI = os.path.join(H.GOLDEN, "c3_prior.xml")


def _draws(n, seed):
    prob = H.c3_problem(1)
    lo = np.array([v.lower for v in prob.variables])
    hi = np.array([v.upper for v in prob.variables])
    return H.draws(lo, hi, n, seed)


def _assert_matches_oracle(x, got):
    import oracle as O
    import parity
    prob = H.c3_problem(1)
    r = O.Oracle("restated").popk_eval(prob, x, nthreads=8, want_traj=False)
    ref = r["logp"]
    mism = np.isfinite(got) != np.isfinite(ref)
    assert np.all(r["stats"][mism, 0, 0] >= 0.99 * prob.max_steps)
    err = parity.llh_err(got[~mism], ref[~mism])
    parity.log_summary({"llh_t1": float(np.mean(err <= parity.LLH_T1)), "llh_max": float(err.max())}, n=int(err.size))
    assert np.mean(err <= parity.LLH_T1) >= parity.llh_min_fraction(err.size) and np.all(err <= parity.LLH_T2)


def _threads(fn, nt, x):
    out = np.full(len(x), np.nan)
    errs = []

    def work(t):
        try:
            for i in range(t, len(x), nt):
                out[i] = fn(x[i])
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(nt)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    return out


def test_concurrent_single_evaluations_are_combined():
    from bcm3_amd import _hip
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(LIK, PRI, device=0)
    x = _draws(256, 3)
    want, _ = ll.evaluate_batch(x)
    ll.set_option(_hip.OPT_TIMING_LOG, 1)
    got = _threads(ll.evaluate, 64, x)
    _, launches, _ = ll.kernel_time_log()
    ll.set_option(_hip.OPT_TIMING_LOG, 0)
    assert np.array_equal(got, want)  # per-item results do not depend on the batch
    assert launches < len(x) // 2, launches  # requests were combined into batched launches
    _assert_matches_oracle(x, got)


def test_dll_plugin_route_many_threads():
    os.environ["BCM3_LIKELIHOOD_XML"] = LIK
    os.environ["BCM3_PRIOR_XML"] = PRI
    os.environ["BCM3_DEVICE"] = "0"
    from bcm3_amd import _hip
    from bcm3_amd.likelihood import Likelihood
    _hip.lib()
    dll = C.CDLL(os.path.join(ROOT, "bcm3_amd", "lib", "libbcm3_dll.so"))
    dll.initialize_likelihood.restype = C.c_bool
    dll.initialize_likelihood.argtypes = [C.c_size_t, C.c_void_p]
    dll.evaluate_log_probability.restype = C.c_bool
    dll.evaluate_log_probability.argtypes = [C.c_size_t, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
    ref = Likelihood(LIK, PRI, device=0)
    names = ref.variable_names
    arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
    assert dll.initialize_likelihood(len(names), arr)
    x = _draws(192, 5)
    want, _ = ref.evaluate_batch(x)

    def one(v):
        v = np.ascontiguousarray(v)
        out = C.c_double()
        assert dll.evaluate_log_probability(len(v), v.ctypes.data, arr, C.byref(out))
        return out.value

    got = _threads(one, 48, x)
    assert np.array_equal(got, want)
    _assert_matches_oracle(x, got)
