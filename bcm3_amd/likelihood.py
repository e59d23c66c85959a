"""Python front-end of the host library libbcm3.so (include/bcm3.h).

Mirrors how the reference's bcminf wires a likelihood (src/bcminf/main.cpp:47-121):
VariableSet from prior.xml, LikelihoodFactory::CreateLikelihood from likelihood.xml, then
EvaluateLogProbability -- plus the batched / device-resident entry points the MI355X fan-out uses.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import _hip

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libbcm3.so")
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    _hip.lib()  # loads torch first (one HIP runtime per process), then libbcm3hip.so
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libbcm3.so not built at {LIB_PATH}; run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    vp, sz = C.c_void_p, C.c_size_t
    L.bcm3_likelihood_create.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(vp)]
    L.bcm3_likelihood_create_ex.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(vp)]
    L.bcm3_likelihood_popk_model.argtypes = [vp, C.POINTER(_hip.PopPKModel)]
    L.bcm3_likelihood_expm_pk_model.argtypes = [vp, C.POINTER(_hip.ExpmPKModel)]
    L.bcm3_likelihood_destroy.argtypes = [vp]
    L.bcm3_likelihood_destroy.restype = None
    L.bcm3_likelihood_num_variables.argtypes = [vp]
    L.bcm3_likelihood_variable_name.argtypes = [vp, C.c_int, C.c_char_p, sz]
    L.bcm3_likelihood_variable_transform.argtypes = [vp, C.c_int]
    L.bcm3_likelihood_set_learning_rate.argtypes = [vp, C.c_double]
    L.bcm3_likelihood_evaluate.argtypes = [vp, sz, vp, vp]
    L.bcm3_likelihood_evaluate_batch.argtypes = [vp, sz, vp, vp, vp]
    L.bcm3_likelihood_evaluate_batch_device.argtypes = [vp, sz, vp, vp, vp, vp]
    L.bcm3_likelihood_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_float)]
    L.bcm3_likelihood_set_option.argtypes = [vp, C.c_int, C.c_int64]
    L.bcm3_likelihood_kernel_time_log.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                                  C.POINTER(C.c_double)]
    L.bcm3_last_error.restype = C.c_char_p
    L.bcm3_likelihood_generated_code.argtypes = [vp, C.c_char_p, sz]
    L.bcm3_likelihood_cellpop_cells.argtypes = [vp, sz, C.POINTER(C.c_int32), vp, vp, vp]
    i32, i64, u64 = C.c_int, C.c_int64, C.c_uint64
    L.bcm3_adapt_proposals.argtypes = [i32, i32, i32, i32, i32, i32, vp, vp, vp, sz, vp, vp, u64, u64, i64, i32, vp,
                                       vp, vp, vp, vp, vp]
    L.bcm3_gmm_eval.argtypes = [i32, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp]
    _lib = L
    return L


def _err(what: str, code: int):
    raise RuntimeError(f"{what} failed ({code}): {lib().bcm3_last_error().decode()}")


class Likelihood:
    """bcm3::Likelihood created from the reference's prior.xml + likelihood.xml."""

    def __init__(self, likelihood_xml: str, prior_xml: str, device: int = -1, options: Optional[str] = None):
        L = lib()
        h = C.c_void_p()
        if options is None:
            r = L.bcm3_likelihood_create(likelihood_xml.encode(), prior_xml.encode(), device, C.byref(h))
        else:
            opts = options + ("" if device < 0 else f";device={device}")
            r = L.bcm3_likelihood_create_ex(likelihood_xml.encode(), prior_xml.encode(), opts.encode(), C.byref(h))
        if r != 0:
            _err("bcm3_likelihood_create", r)
        self.h = h
        self.d = L.bcm3_likelihood_num_variables(h)

    @property
    def variable_names(self):
        buf = C.create_string_buffer(512)
        return [(lib().bcm3_likelihood_variable_name(self.h, i, buf, 512), buf.value.decode())[1]
                for i in range(self.d)]

    @property
    def variable_transforms(self):
        return [lib().bcm3_likelihood_variable_transform(self.h, i) for i in range(self.d)]

    def popk_model(self) -> _hip.PopPKModel:
        m = _hip.PopPKModel()
        r = lib().bcm3_likelihood_popk_model(self.h, C.byref(m))
        if r != 0:
            _err("bcm3_likelihood_popk_model", r)
        return m

    def expm_pk_model(self) -> _hip.ExpmPKModel:
        """bcm3_likelihood_expm_pk_model (pharmaco_single): treatment schedule, observations and
        variable indices as the device sees them; the array pointers stay valid while self lives."""
        m = _hip.ExpmPKModel()
        r = lib().bcm3_likelihood_expm_pk_model(self.h, C.byref(m))
        if r != 0:
            _err("bcm3_likelihood_expm_pk_model", r)
        return m

    def generated_code(self) -> str:
        """cell_population: the generated_derivative body this likelihood compiled (SBMLModel::GenerateCode)."""
        n = lib().bcm3_likelihood_generated_code(self.h, None, 0)
        if n < 0:
            _err("bcm3_likelihood_generated_code", n)
        buf = C.create_string_buffer(n + 1)
        lib().bcm3_likelihood_generated_code(self.h, buf, n + 1)
        return buf.value.decode()

    def cellpop_cells(self, item: int, M: int, NS: int):
        """cell_population: per-cell records, data values [cells][M] and end states [cells][NS] of
        item `item` of the last batch (bcm3hip_cellpop_cells)."""
        rec_t = np.dtype([("creation", "f8"), ("sim_end", "f8"), ("achieved", "f8"), ("flags", "i4"), ("nsteps", "i4")])
        count = C.c_int32()
        r = lib().bcm3_likelihood_cellpop_cells(self.h, item, C.byref(count), None, None, None)
        if r != 0:
            _err("bcm3_likelihood_cellpop_cells", r)
        n = count.value
        rec = np.zeros(n, dtype=rec_t)
        vals = np.empty((n, M))
        endy = np.empty((n, NS))
        r = lib().bcm3_likelihood_cellpop_cells(self.h, item, C.byref(count), rec.ctypes.data, vals.ctypes.data,
                                                endy.ctypes.data)
        if r != 0:
            _err("bcm3_likelihood_cellpop_cells", r)
        return rec, vals, endy

    def set_learning_rate(self, lr: float):
        if lib().bcm3_likelihood_set_learning_rate(self.h, lr) != 0:
            _err("set_learning_rate", -1)

    def evaluate(self, values, threadix: int = 0) -> float:
        v = np.ascontiguousarray(values, dtype=np.float64)
        out = C.c_double()
        r = lib().bcm3_likelihood_evaluate(self.h, threadix, v.ctypes.data, C.addressof(out))
        if r != 0:
            _err("EvaluateLogProbability", r)
        return out.value

    def evaluate_batch(self, values):
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.d)
        n = v.shape[0]
        logp = np.empty(n)
        status = np.empty(n, dtype=np.int32)
        r = lib().bcm3_likelihood_evaluate_batch(self.h, n, v.ctypes.data, logp.ctypes.data, status.ctypes.data)
        if r != 0:
            _err("EvaluateLogProbabilityBatch", r)
        return logp, status

    def evaluate_batch_device(self, n: int, values_ptr: int, logp_ptr: int, status_ptr: Optional[int] = None,
                              stream: Optional[int] = None):
        r = lib().bcm3_likelihood_evaluate_batch_device(self.h, n, values_ptr, logp_ptr, status_ptr, stream)
        if r != 0:
            _err("EvaluateLogProbabilityBatchDevice", r)

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        r = lib().bcm3_likelihood_last_kernel_ms(self.h, C.byref(ms))
        if r != 0:
            _err("last_kernel_ms", r)
        return float(ms.value)

    def kernel_time_log(self):
        """(total_ms, launches, max_ms) since the previous call; needs set_option(OPT_TIMING_LOG, 1)."""
        tot, n, mx = C.c_double(), C.c_int64(), C.c_double()
        r = lib().bcm3_likelihood_kernel_time_log(self.h, C.byref(tot), C.byref(n), C.byref(mx))
        if r != 0:
            _err("kernel_time_log", r)
        return tot.value, n.value, mx.value

    def set_option(self, option: int, value: int):
        if lib().bcm3_likelihood_set_option(self.h, option, int(value)) != 0:
            _err("set_option", -1)

    def close(self):
        if getattr(self, "h", None):
            lib().bcm3_likelihood_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
