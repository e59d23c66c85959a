"""The device's libm (bcm3_amd/csrc/libm_exact.h) against the host's glibc, which the oracle and
the reference's CPU build call (DESIGN.md §3 "bit-exact arithmetic").

libm_exact.h is plain IEEE double arithmetic with explicit fma, so compiled for the host it
computes what the GPU computes. exp / log / pow(x, 1/k) must be correctly rounded (checked
against quad precision, libquadmath); log1p is glibc's fdlibm algorithm and must match the host's
glibc bit for bit; erf / erfc likewise except where glibc's own exp (inside them) is not correctly
rounded. The agreement fractions with glibc are asserted too: they are what bounds the GPU's
bit-exact fraction against the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "libm", "libm_check.cpp")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("libm") / "libm_check")
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-mfma", "-o", exe, SRC,
                    os.path.join(ROOT, "bcm3_amd", "csrc", "libm_tables.cpp"), "-lquadmath"], check=True)
    return exe


def run(exe, fn, n=400000, seed=3):
    out = subprocess.run([exe, fn, str(n), str(seed)], check=True, capture_output=True, text=True).stdout.split()
    n, agree_glibc, agree_cr, glibc_cr = map(int, out)
    return agree_glibc / n, agree_cr / n, glibc_cr / n


@pytest.mark.parametrize("fn", ["exp", "log", "pow"])
def test_correctly_rounded(checker, fn):
    ag, ac, gc = run(checker, fn)
    assert ac == 1.0, (fn, ac)
    # glibc itself is correctly rounded on all but ~0.1 % of arguments, and exactly there we differ
    assert ag == gc and ag > 0.998, (fn, ag, gc)


def test_log1p_is_glibc(checker):
    ag, _, _ = run(checker, "log1p")
    assert ag == 1.0


@pytest.mark.parametrize("fn", ["erf", "erfc"])
def test_erf_is_glibc(checker, fn):
    ag, _, _ = run(checker, fn)
    assert ag > 0.9995, (fn, ag)


def test_pow_is_glibc(checker):
    """xm::pow_glibc with the tables of the loaded libm: glibc's pow bit for bit, including the
    arguments where glibc is not correctly rounded"""
    ag, _, gc = run(checker, "powglibc", n=1000000)
    assert ag == 1.0, ag
    assert gc < 1.0  # the check sees the non-correctly-rounded cases


def test_device_root_is_glibc(checker):
    """the checked root of bdf_lane.h's BCM3_ROOT_HYBRID / BCM3_ROOT_CALL variants: the correctly
    rounded root where it is certainly glibc's result, glibc's algorithm near rounding midpoints --
    glibc's pow bit for bit"""
    ag, _, _ = run(checker, "powhybrid", n=2000000)
    assert ag == 1.0, ag


def test_exp_is_glibc(checker):
    """xm::exp_glibc (the device's exp with the uploaded tables) is glibc's exp bit for bit over the
    range of its main path"""
    ag, _, gc = run(checker, "expglibc", n=1000000)
    assert ag == 1.0, ag


def test_pow_computed_tables_fallback(checker):
    """without the libm's tables the same algorithm on host-computed tables: correctly rounded on
    all but a small fraction of the roots (the fallback)"""
    _, ac, _ = run(checker, "powcomputed", n=400000)
    assert ac > 0.99, ac
