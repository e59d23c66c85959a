"""CPU tests of the C-ABI boundary: the libraries load and export every symbol the public
headers declare (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")

LIBS = {
    "bcm3hip.h": os.path.join(ROOT, "bcm3_amd", "lib", "libbcm3hip.so"),
    "bcm3.h": os.path.join(ROOT, "bcm3_amd", "lib", "libbcm3.so"),
    "bcm3_dll.h": os.path.join(ROOT, "bcm3_amd", "lib", "libbcm3_dll.so"),
}


def declared_functions(header):
    src = open(os.path.join(INCLUDE, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//.*", "", src)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(bcm3\w*|initialize_likelihood|evaluate_log_probability)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.mark.parametrize("header", sorted(LIBS))
def test_library_exports_every_declared_symbol(header):
    path = LIBS[header]
    if not os.path.exists(path):
        pytest.fail(f"{path} not built; run __graft_entry__.build()")
    names = declared_functions(header)
    assert names, header
    lib = ctypes.CDLL(path)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_error_strings_without_gpu():
    lib = ctypes.CDLL(LIBS["bcm3hip.h"])
    lib.bcm3hip_error_string.restype = ctypes.c_char_p
    assert lib.bcm3hip_error_string(0) == b"success"
    assert lib.bcm3hip_error_string(-4) == b"invalid model description"


def test_dll_plugin_initialises_against_prior(monkeypatch):
    """LikelihoodDLL contract: initialize_likelihood checks the names; without a GPU the
    evaluation fails (no CPU fallback)."""
    golden = os.path.join(ROOT, "tests", "golden")
    monkeypatch.setenv("BCM3_LIKELIHOOD_XML", os.path.join(golden, "banana_likelihood.xml"))
    monkeypatch.setenv("BCM3_PRIOR_XML", os.path.join(golden, "banana_prior.xml"))
    monkeypatch.setenv("BCM3_OPTIONS", "backend=none")
    import bcm3_amd.likelihood as L
    L.lib()  # loads torch + libbcm3hip + libbcm3 first
    lib = ctypes.CDLL(LIBS["bcm3_dll.h"])
    lib.initialize_likelihood.restype = ctypes.c_bool
    lib.initialize_likelihood.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_char_p)]
    lib.evaluate_log_probability.restype = ctypes.c_bool
    lib.evaluate_log_probability.argtypes = [ctypes.c_size_t, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double)]
    names = (ctypes.c_char_p * 2)(b"x1", b"x2")
    assert lib.initialize_likelihood(2, names)
    bad = (ctypes.c_char_p * 2)(b"x1", b"y")
    assert not lib.initialize_likelihood(2, bad)
    assert lib.initialize_likelihood(2, names)
    v = (ctypes.c_double * 2)(0.5, 1.0)
    out = ctypes.c_double()
    assert not lib.evaluate_log_probability(2, v, names, ctypes.byref(out))
