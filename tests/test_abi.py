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
}


def declared_functions(header):
    src = open(os.path.join(INCLUDE, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//.*", "", src)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(bcm3\w*)\s*\(", src, flags=re.M)
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
