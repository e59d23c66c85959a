"""The mixture test likelihoods (multimodal_gaussians, truncated_t) and dummy, CPU side.

* The checker (oracle/_ref/libmixref.so: dmvnormal / dmvt restated over the reference's vendored
  Eigen LLT, oracle/mixture_ref.cpp) against the reference's own golden values
  (tests/stats/mvn.cpp:17-44, tests/stats/mvt.cpp:5-44; BOOST_CHECK_CLOSE's tolerance is in percent).
* libbcm3's host parsing of the reference's example files (examples/multimodal_gaussians,
  examples/truncated_t, copied as data into tests/golden/) and the reference's failure modes
  (TestLikelihoodTruncatedT.cpp:20-79, VectorUtils.h:39-67, VectorUtils.cpp:204-219).
* The examples' config files through the config reader.
No likelihood is evaluated here (backend=none)."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import helpers as H
from bcm3_amd import ptmh

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle", "_ref", "libmixref.so")


def mixref():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libmixref.so not built (needs /root/reference's Eigen)")
    L = C.CDLL(REF)
    dp = C.POINTER(C.c_double)
    L.mixref_dmvnormal.argtypes = [C.c_int, dp, dp, dp]
    L.mixref_dmvnormal.restype = C.c_double
    L.mixref_dmvt.argtypes = [C.c_int, dp, dp, dp, C.c_double]
    L.mixref_dmvt.restype = C.c_double
    L.mixref_eval.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                              C.c_long, C.c_void_p, C.c_void_p]
    return L


def _p(a):
    a = np.ascontiguousarray(a, np.float64)
    return a.ctypes.data_as(C.POINTER(C.c_double)), a


SIG = np.array([[234.0, 42.0], [42.0, 786.0]])
MU = np.ones(2) * 1.2e3
X = np.array([1000.0, 1050.0])
# (function, x, mu, sigma, expected log density) -- tests/stats/mvn.cpp:17-44, tests/stats/mvt.cpp:17-44
GOLDEN = [
    ("n", np.zeros(2), np.zeros(2), np.eye(2), -1.837877066409345),
    ("n", np.ones(2), np.zeros(2), np.eye(2), -2.837877066409345),
    ("n", -np.ones(2), np.zeros(2), np.eye(2), -2.837877066409345),
    ("n", MU, MU, SIG, -7.894197416778156),
    ("n", X, MU, SIG, -101.726542607819),
    ("t", np.zeros(2), np.zeros(2), np.eye(2), -1.837877066409345),
    ("t", np.ones(2), np.zeros(2), np.eye(2), -3.015529894583591),
    ("t", -np.ones(2), np.zeros(2), np.eye(2), -3.015529894583591),
    ("t", MU, MU, SIG, -7.894197416778155),
    ("t", X, MU, SIG, -20.67449435172604),
]
GOLDEN_PDF = [(0, 0.1591549430918953), (1, 0.05854983152431917), (3, 0.0003729010642586194),
              (4, 6.617956105689106e-45), (6, 0.04901985324897605), (8, 0.0003729010642586194),
              (9, 1.04998038728666e-09)]


@pytest.mark.parametrize("i", range(len(GOLDEN)))
def test_checker_golden_log_densities(i):
    L = mixref()
    f, x, mu, sig, want = GOLDEN[i]
    (px, _), (pm, _), (ps, _) = _p(x), _p(mu), _p(sig)
    got = L.mixref_dmvnormal(2, px, pm, ps) if f == "n" else L.mixref_dmvt(2, px, pm, ps, 5.0)
    assert abs(got - want) <= 1e-14 * abs(want), (got, want)


@pytest.mark.parametrize("i,want", GOLDEN_PDF)
def test_checker_golden_densities(i, want):
    L = mixref()
    f, x, mu, sig, _ = GOLDEN[i]
    (px, _), (pm, _), (ps, _) = _p(x), _p(mu), _p(sig)
    got = math.exp(L.mixref_dmvnormal(2, px, pm, ps) if f == "n" else L.mixref_dmvt(2, px, pm, ps, 5.0))
    assert abs(got - want) <= 1e-14 * want, (got, want)


def test_checker_dmvt_1d_is_logpdft():
    # tests/stats/mvt.cpp:5-15: dmvt with p = 1 is LogPdfT(x, mu, sigma(0,0), nu); LogPdfT
    # (ProbabilityDistributions.cpp:159-180) scales by multiplying with sigma
    L = mixref()
    for x, mu, s, nu in ((0.0, 0.0, 1.0, 5.0), (1.0, 0.0, 1.0, 5.0), (-1.0, 0.0, 1.0, 5.0), (0.7, 0.2, 2.5, 3.0)):
        (px, _), (pm, _), (ps, _) = _p([x]), _p([mu]), _p([[s]])
        got = L.mixref_dmvt(1, px, pm, ps, nu)
        xn = (x - mu) * s
        beta = math.exp(math.lgamma(nu / 2) + math.lgamma(0.5) - math.lgamma(nu / 2 + 0.5))
        want = -math.log(s * math.sqrt(nu) * beta) - 0.5 * (nu + 1) * math.log1p(xn * xn / nu)
        assert abs(got - want) <= 1e-14 * (1 + abs(want))


def _lik(name, tmp_path=None, text=None, prior=None):
    from bcm3_amd.likelihood import Likelihood
    if text is not None:
        p = tmp_path / "likelihood.xml"
        p.write_text(text)
        lik = str(p)
    else:
        lik = os.path.join(H.GOLDEN, f"{name}_likelihood.xml")
    pri = prior or os.path.join(H.GOLDEN, f"{name}_prior.xml")
    return Likelihood(lik, pri, options="backend=none")


def test_examples_load():
    for name, d in (("multimodal_gaussians", 2), ("truncated_t", 3)):
        ll = _lik(name)
        assert ll.d == d
        ll.close()


TT = ('<bcm_likelihood type="truncated_t" num_clusters="{k}" dimensions="{d}" nus="{nus}" mu1="{mu1}" '
      'sigma1="{s1}" {more} weights="{w}"/>')


def _tt(**kw):
    f = dict(k=1, d=3, nus="3.0", mu1="0.5;2.0;0.0", s1="1,0,0;0,1,0;0,0,1", more="", w="1")
    f.update(kw)
    return TT.format(**f)


@pytest.mark.parametrize("kw,msg", [
    (dict(s1="1,0;0,1,0;0,0,1"), "Inconsistent matrix"),
    (dict(s1="1,0;0,1"), "Inconsistent dimension for sigma0"),
    (dict(mu1="0.5;2.0"), "Inconsistent dimension for mu0"),
    (dict(mu1="0.5; 2.0;0"), "Could not cast value"),        # lexical_cast: no surrounding spaces
    (dict(mu1="0.5;2.0;0;"), "Could not cast value"),        # keep_empty_tokens: a trailing ';' is an empty token
    (dict(nus="3;4"), "Inconsistent number of nus"),
    (dict(w="0.5;0.5"), "Inconsistent number of weights"),
    (dict(d=2), "Incorrect number of variables"),
    (dict(k=2), "mu2"),
])
def test_truncated_t_rejects_what_the_reference_rejects(tmp_path, capfd, kw, msg):
    with pytest.raises(Exception):
        _lik("truncated_t", tmp_path, _tt(**kw))
    assert msg in capfd.readouterr().err


def test_multimodal_gaussians_needs_two_variables(tmp_path, capfd):
    with pytest.raises(Exception):
        _lik("multimodal_gaussians", prior=os.path.join(H.GOLDEN, "truncated_t_prior.xml"))
    assert "Inconsistent prior and likelihood (3 variables and 2 dimensions)" in capfd.readouterr().err


def test_dummy_loads(tmp_path):
    ll = _lik("dummy", tmp_path, '<bcm_likelihood type="dummy"/>', prior=os.path.join(H.GOLDEN, "banana_prior.xml"))
    assert ll.d == 2
    ll.close()


def test_example_configs():
    c = ptmh.load_config(os.path.join(H.GOLDEN, "multimodal_gaussians_config_gmm.txt"))
    p = c["ptmh"]
    assert c["num_samples"] == 16000 and p["use_every_nth"] == 5 and p["num_chains"] == 2
    assert p["proposal"] == ptmh.PROPOSALS["gaussian_mixture"] and p["adapt_proposal_samples"] == 4000
    c = ptmh.load_config(os.path.join(H.GOLDEN, "truncated_t_config_gmm_t.txt"))
    p = c["ptmh"]
    assert c["num_samples"] == 12000 and p["num_chains"] == 1 and p["exploration_steps"] == 2
    assert p["t_dof"] == 5.0 and p["adapt_proposal_times"] == 2
