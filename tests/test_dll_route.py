"""The reference's `type="dll"` likelihood (LikelihoodDLL, src/likelihoods/LikelihoodDLL.cpp:34-116)
in the host factory: a user plugin .so (tests/plugins/gauss_plugin.c, built by build()) loaded by
dll_filename_base, initialised with the variable names, evaluated single and batched on host
threads; NaN or false is an error. CPU only -- the plugin is the user's host code."""
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PLUGIN = os.path.join(ROOT, "tests", "plugins", "build", "gauss_plugin")


def _files(tmp_path, include_build_dir=False, base=PLUGIN):
    lik = tmp_path / "likelihood.xml"
    lik.write_text(f'<bcm_likelihood type="dll" dll_filename_base="{base}" '
                   f'include_build_dir="{"true" if include_build_dir else "false"}"/>\n')
    pri = tmp_path / "prior.xml"
    pri.write_text('<prior>\n <variable name="a" distribution="uniform" lower="-5" upper="5"/>\n'
                   ' <variable name="b" distribution="normal" mu="0" sigma="2" repeat="2"/>\n</prior>\n')
    return str(lik), str(pri)


def _want(x):
    z = np.asarray(x) - np.arange(len(x))
    return float(np.sum(-0.5 * z * z / 4.0))


def test_dll_type_single_and_batch(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(*_files(tmp_path))
    assert ll.variable_names == ["a", "b_0", "b_1"]
    x = np.array([0.3, 1.7, -2.0])
    assert abs(ll.evaluate(x) - _want(x)) < 1e-12
    X = np.random.default_rng(0).normal(size=(333, 3))
    lp, st = ll.evaluate_batch(X)
    np.testing.assert_allclose(lp, [_want(r) for r in X], rtol=1e-14)
    assert (st == 0).all()
    with pytest.raises(RuntimeError):
        ll.evaluate(np.array([2e6, 0.0, 0.0]))  # the plugin returns NaN: fatal


def test_dll_type_build_dir_prefix(tmp_path, monkeypatch):
    """include_build_dir (default true) prefixes "build/" to the relative path, as the reference."""
    from bcm3_amd.likelihood import Likelihood
    monkeypatch.chdir(os.path.join(ROOT, "tests", "plugins"))
    ll = Likelihood(*_files(tmp_path, include_build_dir=True, base="gauss_plugin"))
    assert abs(ll.evaluate(np.zeros(3)) - _want(np.zeros(3))) < 1e-12
    with pytest.raises(RuntimeError):
        Likelihood(*_files(tmp_path, include_build_dir=True, base="no_such_plugin"))
