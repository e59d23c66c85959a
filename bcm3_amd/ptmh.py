"""The C++ PT-MH sampler loop (libbcm3.so bcm3_ptmh_*, csrc/host/SamplerPTDevice.cpp) from Python.

SamplerPT::Initialize / Run (src/sampler/SamplerPT.cpp:97-260) run by C++ host code over the
HIP C-ABI: chain state in HBM, one batched likelihood launch per mutate step, proposal adaptation
on host threads, the PT swap between ranks over RCCL. This module only configures it and reads
results back; nothing of the iteration runs in Python or torch. bcm3_amd.sampler.PTMHDevice is
the same loop written in Python over the same kernels (the two agree bit for bit,
tests/test_ptmh_native_gpu.py).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _hip
from .likelihood import Likelihood, lib as host_lib

PROPOSALS = {"global_covariance": 0, "gaussian_mixture": 1, "gaussian_mixture_adjustedAIC": 2, "random_walk": 3}
SCHEMES = {"deterministic_even_odd": 0, "stochastic_even_odd": 1, "stochastic_random": 2}
TRANSPORT_NONE, TRANSPORT_RCCL, TRANSPORT_LOCAL, TRANSPORT_SOCKET = 0, 1, 2, 3
COUNTERS = ("attempted_mutate", "accepted_mutate", "attempted_exchange", "accepted_exchange", "samples_done",
            "adaptations_done", "iterations", "rounds", "likelihood_launches", "evaluated_entries")


class PTMHConfig(C.Structure):
    _fields_ = [
        ("num_chains", C.c_int64), ("rank", C.c_int32), ("world", C.c_int32),
        ("temperature_power", C.c_double), ("temperature_max", C.c_double), ("seed", C.c_uint64),
        ("learning_rate", C.c_double), ("exploration_steps", C.c_int32), ("proposal", C.c_int32),
        ("t_dof", C.c_double), ("kmax", C.c_int32), ("adapt_proposal_samples", C.c_int32),
        ("adapt_proposal_times", C.c_int32), ("max_history_size", C.c_int32),
        ("adapt_proposal_max_history_samples", C.c_int32), ("use_every_nth", C.c_int32),
        ("swapping_scheme", C.c_int32), ("exchange_probability", C.c_double),
        ("initial_position_tries", C.c_int32), ("nan_check_every", C.c_int32), ("host_threads", C.c_int32),
        ("speculate", C.c_int32),
        ("transport", C.c_int32), ("nccl_id", C.c_uint8 * 128), ("group", C.c_void_p),
        ("socket_dir", C.c_char * 256),
    ]


class RunConfig(C.Structure):
    """bcm3_run_config (include/bcm3.h): bcminf's config.txt as the PT-MH path reads it."""
    _fields_ = [
        ("ptmh", PTMHConfig), ("num_samples", C.c_int64), ("output_proposal_adaptation", C.c_int32),
        ("pad_", C.c_int32), ("sampling_threads", C.c_int64), ("evaluation_threads", C.c_int64),
        ("sampler_type", C.c_char * 64), ("prior", C.c_char * 1024), ("likelihood", C.c_char * 1024),
        ("output_folder", C.c_char * 1024), ("likelihood_options", C.c_char * 2048),
    ]


_bound = False


def _lib():
    global _bound
    L = host_lib()
    if not _bound:
        vp = C.c_void_p
        L.bcm3_ptmh_config_default.argtypes = [C.POINTER(PTMHConfig)]
        L.bcm3_ptmh_config_default.restype = None
        L.bcm3_run_config_from_file.argtypes = [C.c_char_p, C.POINTER(RunConfig)]
        L.bcm3_ptmh_config_from_file.argtypes = [C.c_char_p, C.POINTER(PTMHConfig)]
        L.bcm3_ptmh_nccl_unique_id.argtypes = [vp]
        L.bcm3_ptmh_group_create.argtypes = [C.c_int, C.POINTER(vp)]
        L.bcm3_ptmh_group_destroy.argtypes = [vp]
        L.bcm3_ptmh_group_destroy.restype = None
        L.bcm3_ptmh_create.argtypes = [vp, C.c_char_p, C.POINTER(PTMHConfig), vp, C.POINTER(vp)]
        L.bcm3_ptmh_iterate.argtypes = [vp, C.c_int64, C.c_int]
        L.bcm3_ptmh_run.argtypes = [vp, C.c_int64]
        L.bcm3_ptmh_adapt.argtypes = [vp]
        L.bcm3_ptmh_spec_batch_info.argtypes = [vp, vp, vp]
        L.bcm3_ptmh_spec_batch_info.restype = C.c_int64
        L.bcm3_ptmh_synchronize.argtypes = [vp]
        L.bcm3_ptmh_num_chains.argtypes = [vp]
        L.bcm3_ptmh_get_state.argtypes = [vp, vp, vp, vp, vp]
        L.bcm3_ptmh_get_components.argtypes = [vp, vp]
        L.bcm3_ptmh_get_counters.argtypes = [vp, vp]
        L.bcm3_ptmh_stream.argtypes = [vp]
        L.bcm3_ptmh_stream.restype = vp
        L.bcm3_ptmh_destroy.argtypes = [vp]
        L.bcm3_ptmh_destroy.restype = None
        L.bcm3_ptmh_set_output.argtypes = [vp, C.c_char_p, C.c_int64, C.c_int32]
        L.bcm3_ptmh_flush_output.argtypes = [vp]
        L.bcm3_ptmh_set_adaptation_output.argtypes = [vp, C.c_char_p]
        L.bcm3_samples_open.argtypes = [C.c_char_p, C.c_int64, C.c_int32, C.POINTER(C.c_char_p), vp, C.c_int32, vp,
                                        C.c_int32, C.c_int32, C.POINTER(vp)]
        L.bcm3_samples_write.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp]
        L.bcm3_samples_sync.argtypes = [vp]
        L.bcm3_samples_close.argtypes = [vp]
        L.bcm3_samples_close.restype = None
        _bound = True
    return L


def _check(r: int, what: str):
    if r != 0:
        msg = host_lib().bcm3_last_error()
        raise RuntimeError(f"{what} failed ({r}): {msg.decode() if msg else ''}")


def load_config(path: str) -> dict:
    """config.txt through bcm3_run_config_from_file: {"ptmh": {field: value}, "num_samples": ...,
    "prior": ..., ...}; raises RuntimeError with the reader's message on a file the reference
    would reject."""
    rc = RunConfig()
    _check(_lib().bcm3_run_config_from_file(path.encode(), C.byref(rc)), "bcm3_run_config_from_file")
    ptmh = {k: getattr(rc.ptmh, k) for k, _ in PTMHConfig._fields_ if k not in ("nccl_id", "group", "socket_dir")}
    out = {"ptmh": ptmh}
    for k, _ in RunConfig._fields_:
        if k in ("ptmh", "pad_"):
            continue
        v = getattr(rc, k)
        out[k] = v.decode() if isinstance(v, bytes) else v
    return out


def nccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    _check(_lib().bcm3_ptmh_nccl_unique_id(buf), "bcm3_ptmh_nccl_unique_id")
    return bytes(buf)


class LocalGroup:
    """In-process ranks (one host thread each) exchanging through host-staged mailboxes."""

    def __init__(self, world: int):
        h = C.c_void_p()
        _check(_lib().bcm3_ptmh_group_create(world, C.byref(h)), "bcm3_ptmh_group_create")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            _lib().bcm3_ptmh_group_destroy(self.h)
            self.h = None


class PTMHNative:
    """One rank of the C++ sampler (bcm3_ptmh_create)."""

    def __init__(self, likelihood: Likelihood, prior_xml: str, num_chains: int, rank: int = 0, world: int = 1,
                 seed: int = 0, proposal: str = "gaussian_mixture", swapping_scheme: str = "deterministic_even_odd",
                 stream: Optional[int] = None, transport: int = TRANSPORT_NONE, nccl_id: Optional[bytes] = None,
                 group: Optional[LocalGroup] = None, socket_dir: Optional[str] = None, **options):
        _hip.lib()
        L = _lib()
        cfg = PTMHConfig()
        L.bcm3_ptmh_config_default(C.byref(cfg))
        cfg.num_chains, cfg.rank, cfg.world = int(num_chains), int(rank), int(world)
        cfg.seed = int(seed) & ((1 << 64) - 1)
        cfg.proposal = PROPOSALS[proposal]
        cfg.swapping_scheme = SCHEMES[swapping_scheme]
        cfg.transport = int(transport)
        if nccl_id is not None:
            cfg.nccl_id[:] = list(nccl_id[:128])
        self.group = group
        if group is not None:
            cfg.group = group.h
        if socket_dir is not None:
            cfg.socket_dir = socket_dir.encode()
        for k, v in options.items():
            if k not in dict(PTMHConfig._fields_):
                raise ValueError(f"unknown sampler option {k}")
            setattr(cfg, k, v)
        self.ll = likelihood  # keeps the likelihood alive
        h = C.c_void_p()
        _check(L.bcm3_ptmh_create(likelihood.h, prior_xml.encode(), C.byref(cfg), stream, C.byref(h)),
               "bcm3_ptmh_create")
        self.h = h
        self.d = likelihood.d
        self.C = L.bcm3_ptmh_num_chains(h)

    def set_output(self, filename: str, num_samples: int, flush_every: int = 64):
        """SampleHandlerNetCDF (bcm3_ptmh_set_output): the reference's output.nc schema, netCDF-4 when
        libnetcdf can be loaded (a sharded ladder: rank 0 writes every rank's rows, received over the
        transport), netCDF classic otherwise (SampleFile); every rank calls it before the first
        iteration."""
        _check(_lib().bcm3_ptmh_set_output(self.h, filename.encode(), num_samples, flush_every), "bcm3_ptmh_set_output")

    def set_adaptation_output(self, filename: str):
        """ptmhsampler.output_proposal_adaptation: the highest-temperature chain's fitted proposal
        after every adaptation (bcm3_ptmh_set_adaptation_output)."""
        _check(_lib().bcm3_ptmh_set_adaptation_output(self.h, filename.encode()), "bcm3_ptmh_set_adaptation_output")

    def flush_output(self):
        _check(_lib().bcm3_ptmh_flush_output(self.h), "bcm3_ptmh_flush_output")

    def iterate(self, n: int, last_at_end: bool = False):
        _check(_lib().bcm3_ptmh_iterate(self.h, int(n), int(last_at_end)), "bcm3_ptmh_iterate")

    def run(self, num_samples: int):
        _check(_lib().bcm3_ptmh_run(self.h, int(num_samples)), "bcm3_ptmh_run")

    def spec_batch_info(self):
        """(src, steps) of the last speculative launch in dispatch order, or None"""
        src = np.zeros(7 * self.C, dtype=np.int32)
        steps = np.zeros(7 * self.C, dtype=np.int32)
        n = _lib().bcm3_ptmh_spec_batch_info(self.h, src.ctypes.data, steps.ctypes.data)
        return None if n < 0 else (src[:n], steps[:n])

    def adapt(self):
        _check(_lib().bcm3_ptmh_adapt(self.h), "bcm3_ptmh_adapt")

    def synchronize(self):
        _check(_lib().bcm3_ptmh_synchronize(self.h), "bcm3_ptmh_synchronize")

    @property
    def stream(self) -> int:
        return _lib().bcm3_ptmh_stream(self.h)

    def state(self):
        v = np.empty((self.C, self.d))
        llh, lprior, lpp = np.empty(self.C), np.empty(self.C), np.empty(self.C)
        _check(_lib().bcm3_ptmh_get_state(self.h, v.ctypes.data, llh.ctypes.data, lprior.ctypes.data, lpp.ctypes.data),
               "bcm3_ptmh_get_state")
        return dict(values=v, llh=llh, lprior=lprior, lpp=lpp)

    def components(self):
        nc = np.empty(self.C, dtype=np.int32)
        _check(_lib().bcm3_ptmh_get_components(self.h, nc.ctypes.data), "bcm3_ptmh_get_components")
        return nc

    def counters(self):
        out = np.empty(len(COUNTERS), dtype=np.int64)
        _check(_lib().bcm3_ptmh_get_counters(self.h, out.ctypes.data), "bcm3_ptmh_get_counters")
        return dict(zip(COUNTERS, out.tolist()))

    def close(self):
        if getattr(self, "h", None):
            _lib().bcm3_ptmh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_data_file(path: str) -> dict:
    """A data or output file as libbcm3's loaders read it (bcm3_data_file_json): netCDF classic,
    netCDF-4 through a run-time loaded libnetcdf, or the JSON sidecar -> {group: {variable:
    {"dims": [...], "data": nested lists}}}, fill values as None."""
    import json
    L = _lib()
    L.bcm3_data_file_json.argtypes = [C.c_char_p, C.c_char_p, C.c_int64]
    L.bcm3_data_file_json.restype = C.c_int64
    n = L.bcm3_data_file_json(path.encode(), None, 0)
    if n < 0:
        raise RuntimeError(f"bcm3_data_file_json failed ({n}): {host_lib().bcm3_last_error().decode()}")
    buf = C.create_string_buffer(n + 1)
    L.bcm3_data_file_json(path.encode(), buf, n + 1)
    return json.loads(buf.value.decode())


class SampleFile:
    """bcm3_samples_*: the reference's output.nc (SampleHandlerNetCDF.cpp:24-110) as a netCDF
    classic file written by libbcm3 (group members "samples.<name>"); a process writes the
    temperature columns [first, first + own)."""

    def __init__(self, filename: str, num_samples: int, names, transforms, temperatures, first: int = 0,
                 own: Optional[int] = None):
        L = _lib()
        temps = np.ascontiguousarray(temperatures, dtype=np.float64)
        tr = np.ascontiguousarray(transforms, dtype=np.int32)
        own = len(temps) - first if own is None else own
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        self.d = len(names)
        self.h = C.c_void_p()
        _check(L.bcm3_samples_open(filename.encode(), num_samples, self.d, arr, tr.ctypes.data, len(temps),
                                   temps.ctypes.data, first, own, C.byref(self.h)), "bcm3_samples_open")

    def write(self, sample_ix: int, t0: int, values, lprior, llh, weight=None):
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.d)
        nt = v.shape[0]
        lp = np.ascontiguousarray(lprior, dtype=np.float64).reshape(nt)
        ll = np.ascontiguousarray(llh, dtype=np.float64).reshape(nt)
        w = np.ones(nt) if weight is None else np.ascontiguousarray(weight, dtype=np.float64).reshape(nt)
        _check(_lib().bcm3_samples_write(self.h, sample_ix, t0, nt, v.ctypes.data, lp.ctypes.data, ll.ctypes.data,
                                         w.ctypes.data), "bcm3_samples_write")

    def close(self):
        if self.h:
            _lib().bcm3_samples_close(self.h)
            self.h = None

    def __del__(self):
        self.close()
