"""ctypes binding of libbcm3hip.so (include/bcm3hip.h).

The product path: every evaluation goes through the HIP kernels in ``bcm3_amd/csrc``. There is
no CPU fallback -- if the library is missing or no GPU is present, opening a context raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# BCM3HIP_LIB overrides the library (profiling builds, tools/phase_probe.py only)
LIB_PATH = os.environ.get("BCM3HIP_LIB") or os.path.join(_HERE, "lib", "libbcm3hip.so")

PK_TYPES = {"one": 0, "two": 1, "one_biphasic": 2, "two_biphasic": 3, "one_transit": 4, "two_transit": 5}
ANALYTIC_BANANA, ANALYTIC_CIRCULAR, ANALYTIC_DUMMY = 1, 2, 3
MIXTURE_NORMAL, MIXTURE_T = 1, 2
OPT_LANES_PER_WAVE, OPT_BLOCK_WAVES, OPT_TIMING_LOG, OPT_UNI_SOLVER, OPT_BLOCK_LDS = 1, 2, 3, 4, 5
OPT_PLACEMENT_LOG = 6
PRIOR_UNIFORM, PRIOR_NORMAL = 0, 1
PROPOSAL_GLOBAL_COVARIANCE, PROPOSAL_GAUSSIAN_MIXTURE = 0, 1
PROPOSAL_KMAX = 16


class PopPKModel(C.Structure):
    """bcm3hip_popk_model"""
    _fields_ = [
        ("pk_type", C.c_int32), ("N", C.c_int32), ("num_pk_params", C.c_int32),
        ("num_pk_pop_params", C.c_int32), ("d", C.c_int32), ("P", C.c_int32), ("T", C.c_int32),
        ("sd_ix", C.c_int32), ("n_transit_ix", C.c_int32), ("transit_time_ix", C.c_int32),
        ("biphasic_time_ix", C.c_int32), ("absorption2_ix", C.c_int32), ("max_steps", C.c_int32),
        ("param_map", C.c_int32),
        ("rtol", C.c_double), ("atol", C.c_double), ("MW", C.c_double), ("fixed_vod", C.c_double),
        ("fixed_kf", C.c_double), ("fixed_kb", C.c_double),
        ("transforms", C.c_void_p), ("time", C.c_void_p), ("observed", C.c_void_p), ("dose", C.c_void_p),
        ("dosing_interval", C.c_void_p), ("dose_after_dose_change", C.c_void_p),
        ("dose_change_time", C.c_void_p), ("intermittent", C.c_void_p), ("skipped_days", C.c_void_p),
        ("simulate_until", C.c_void_p),
    ]


class ExpmPKModel(C.Structure):
    """bcm3hip_expm_pk_model"""
    _fields_ = [(k, C.c_int32) for k in (
        "d", "n_transit", "peripheral", "biphasic", "metabolite", "additive_sd_ix", "proportional_sd_ix",
        "absorption_ix", "clearance_ix", "vod_ix", "excretion_ix", "pf_ix", "pb_ix", "mtt_ix", "direct_ix",
        "metab_conv_ix", "n_treat", "n_obs")] + \
        [("MW", C.c_double)] + \
        [(k, C.c_void_p) for k in ("transforms", "treat_times", "treat_doses", "obs_times", "obs_conc")] + \
        [("param_map", C.c_int32), ("P", C.c_int32), ("sigma_ix", C.c_int32 * 5)] + \
        [(k, C.c_void_p) for k in ("patient_ix", "treat_offset", "obs_offset")]


# pharmaco_single's defaults for the population fields of bcm3hip_expm_pk_model
EXPM_PK_SINGLE_DEFAULTS = {"param_map": 1, "P": 1, "sigma_ix": [-1] * 5, "patient_ix": None,
                           "treat_offset": None, "obs_offset": None}


class AnalyticModel(C.Structure):
    """bcm3hip_analytic_model"""
    _fields_ = [("kind", C.c_int32), ("d", C.c_int32), ("p0", C.c_double), ("p1", C.c_double),
                ("p2", C.c_double)]


class MixtureModel(C.Structure):
    """bcm3hip_mixture_model"""
    _fields_ = [("kind", C.c_int32), ("d", C.c_int32), ("K", C.c_int32), ("log_weights", C.c_void_p),
                ("means", C.c_void_p), ("covariances", C.c_void_p), ("nus", C.c_void_p)]


class TrajStats(C.Structure):
    """bcm3hip_traj_stats"""
    _fields_ = [(k, C.c_int32) for k in ("nst", "nfe", "nni", "nsetups", "nje", "netf", "ncfn", "nreinit")]


class Proposal(C.Structure):
    """bcm3hip_proposal (device pointers)"""
    _fields_ = [("kind", C.c_int32), ("kmax", C.c_int32), ("t_dof", C.c_double),
                ("target_acceptance", C.c_double), ("scaling_learning_rate", C.c_double),
                ("scaling_ema_period", C.c_double)] + \
               [(k, C.c_void_p) for k in ("lower", "upper", "ncomp", "weights", "mean", "chol", "logc", "scale",
                                          "ema", "selected", "work")]


STATS_DTYPE = np.dtype([(k, np.int32) for k in ("nst", "nfe", "nni", "nsetups", "nje", "netf", "ncfn", "nreinit")])

_lib = None


def lib() -> C.CDLL:
    """Load libbcm3hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libbcm3hip.so not built at {LIB_PATH}; run __graft_entry__.build()")
    # PyTorch-ROCm ships its own libamdhip64 (same SONAME libamdhip64.so.7). Loading torch first
    # makes the dynamic loader bind this library to torch's copy, so the process has ONE HIP
    # runtime and torch tensors / torch.distributed streams can be handed to our kernels.
    # (Two runtimes in one process make the second initialisation fail.)
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, i64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_int64
    L.bcm3hip_device_count.restype = C.c_int
    L.bcm3hip_error_string.argtypes = [C.c_int]
    L.bcm3hip_error_string.restype = C.c_char_p
    L.bcm3hip_open_popk.argtypes = [C.c_int, C.POINTER(PopPKModel), C.POINTER(vp)]
    L.bcm3hip_open_analytic.argtypes = [C.c_int, C.POINTER(AnalyticModel), C.POINTER(vp)]
    L.bcm3hip_open_expm_pk.argtypes = [C.c_int, C.POINTER(ExpmPKModel), C.POINTER(vp)]
    L.bcm3hip_open_mixture.argtypes = [C.c_int, C.POINTER(MixtureModel), C.POINTER(vp)]
    L.bcm3hip_close.argtypes = [vp]
    L.bcm3hip_set_option.argtypes = [vp, C.c_int, i64]
    L.bcm3hip_num_variables.argtypes = [vp]
    u64 = C.c_uint64
    L.bcm3hip_ptmh_propose.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, i64, u64, u64, vp]
    L.bcm3hip_ptmh_accept.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, C.c_double, vp, vp, vp, vp, vp, vp, vp,
                                      i64, u64, u64, vp]
    L.bcm3hip_pt_exchange_local.argtypes = [C.c_int, C.c_int, i64, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp,
                                            u64, u64, vp]
    L.bcm3hip_ptmh_propose_adaptive.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                                C.POINTER(Proposal), i64, u64, u64, vp]
    L.bcm3hip_ptmh_accept_adaptive.argtypes = [C.c_int, C.c_int, vp, vp, vp, vp, vp, C.c_double, vp, vp, vp, vp,
                                               vp, vp, vp, C.POINTER(Proposal), i64, u64, u64, vp]
    L.bcm3hip_pt_exchange_pair.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, i64, vp, vp, vp, vp, vp, vp, vp,
                                           u64, u64, vp]
    L.bcm3hip_history_add.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp]
    L.bcm3hip_gmm_eval.argtypes = [C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    L.bcm3hip_kernel_time_log.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(i64), C.POINTER(C.c_double)]
    L.bcm3hip_eval_batch.argtypes = [vp, sz, sz, vp, vp, vp]
    L.bcm3hip_eval_batch_device.argtypes = [vp, sz, vp, vp, vp, vp]
    L.bcm3hip_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_float)]
    if hasattr(L, "bcm3hip_placement_log"):  # (absent from libraries built before it: tools/variant_timing.py)
        L.bcm3hip_placement_log.argtypes = [vp, i64, vp]
        L.bcm3hip_placement_log.restype = i64
    if hasattr(L, "bcm3hip_assign_cells"):
        L.bcm3hip_assign_cells.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp]
        L.bcm3hip_assign_cells.restype = C.c_int
    L.bcm3hip_eval_batch_detail.argtypes = [vp, sz, sz, vp, vp, vp, vp, vp, vp]
    for f in ("bcm3hip_open_popk", "bcm3hip_open_analytic", "bcm3hip_open_mixture", "bcm3hip_open_expm_pk", "bcm3hip_close", "bcm3hip_set_option",
              "bcm3hip_num_variables", "bcm3hip_eval_batch", "bcm3hip_eval_batch_device",
              "bcm3hip_last_kernel_ms", "bcm3hip_eval_batch_detail"):
        getattr(L, f).restype = C.c_int
    _lib = L
    return L


def check(code: int, what: str = "bcm3hip"):
    if code != 0:
        msg = lib().bcm3hip_error_string(code).decode()
        raise RuntimeError(f"{what} failed: {msg} ({code})")


def assign_cells(lik):
    """The time-course likelihood's observed-to-simulated cell matching alone, on lik's device
    (bcm3hip_assign_cells). lik: CUDA float64 tensor [problems, observed cells, simulated cells] of
    cell log-likelihoods. Returns numpy (match [problems, R], sum [problems], ok [problems])."""
    import torch
    lik = lik.contiguous()
    P, R, S = lik.shape
    match = torch.empty((P, R), dtype=torch.int32, device=lik.device)
    total = torch.empty(P, dtype=torch.float64, device=lik.device)
    ok = torch.empty(P, dtype=torch.int32, device=lik.device)
    stream = torch.cuda.current_stream(lik.device).cuda_stream
    check(lib().bcm3hip_assign_cells(P, R, S, lik.data_ptr(), match.data_ptr(), total.data_ptr(), ok.data_ptr(),
                                     stream), "bcm3hip_assign_cells")
    torch.cuda.synchronize(lik.device)
    return match.cpu().numpy(), total.cpu().numpy(), ok.cpu().numpy()


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


class Context:
    """One GPU likelihood context (not thread-safe; one per host thread / GPU)."""

    def __init__(self, handle, d: int, P: int = 1, N: int = 0, T: int = 0, keep=None):
        self.h = handle
        self.d, self.P, self.N, self.T = d, P, N, T
        self._keep = keep

    @classmethod
    def popk(cls, model_fields: dict, device: int = 0) -> "Context":
        """model_fields: the bcm3hip_popk_model fields; arrays as numpy arrays."""
        m = PopPKModel()
        keep = []
        arrays = {"transforms": np.int32, "time": np.float64, "observed": np.float64, "dose": np.float64,
                  "dosing_interval": np.float64, "dose_after_dose_change": np.float64,
                  "dose_change_time": np.float64, "intermittent": np.int32, "skipped_days": np.uint8,
                  "simulate_until": np.int32}
        for name, _ in PopPKModel._fields_:
            v = model_fields.get(name, 0) if name == "param_map" else model_fields[name]
            if name in arrays:
                a = np.ascontiguousarray(v, dtype=arrays[name])
                keep.append(a)
                setattr(m, name, a.ctypes.data)
            else:
                setattr(m, name, v)
        h = C.c_void_p()
        check(lib().bcm3hip_open_popk(device, C.byref(m), C.byref(h)), "bcm3hip_open_popk")
        return cls(h, int(m.d), int(m.P), int(m.N), int(m.T))

    @classmethod
    def from_popk_model(cls, m: "PopPKModel", device: int = 0) -> "Context":
        """A second context on a model description some other owner keeps alive (e.g.
        bcm3.Likelihood.popk_model(), whose arrays live as long as that likelihood)."""
        h = C.c_void_p()
        check(lib().bcm3hip_open_popk(device, C.byref(m), C.byref(h)), "bcm3hip_open_popk")
        return cls(h, int(m.d), int(m.P), int(m.N), int(m.T))

    @classmethod
    def analytic(cls, kind: int, d: int, p0: float, p1: float, p2: float = 0.0, device: int = 0) -> "Context":
        m = AnalyticModel(kind, d, p0, p1, p2)
        h = C.c_void_p()
        check(lib().bcm3hip_open_analytic(device, C.byref(m), C.byref(h)), "bcm3hip_open_analytic")
        return cls(h, d)

    @classmethod
    def mixture(cls, kind: int, log_weights, means, covariances, nus=None, device: int = 0) -> "Context":
        """bcm3hip_open_mixture: means [K][d], covariances [K][d][d] (lower triangles used)."""
        lw = np.ascontiguousarray(log_weights, np.float64)
        mu = np.ascontiguousarray(means, np.float64)
        cov = np.ascontiguousarray(covariances, np.float64)
        K, d = mu.shape
        assert lw.shape == (K,) and cov.shape == (K, d, d)
        nu = None if nus is None else np.ascontiguousarray(nus, np.float64)
        m = MixtureModel(kind, d, K, lw.ctypes.data, mu.ctypes.data, cov.ctypes.data,
                         None if nu is None else nu.ctypes.data)
        h = C.c_void_p()
        check(lib().bcm3hip_open_mixture(device, C.byref(m), C.byref(h)), "bcm3hip_open_mixture")
        return cls(h, d)

    @classmethod
    def expm_pk(cls, fields: dict, device: int = 0) -> "Context":
        """bcm3hip_open_expm_pk from a dict of bcm3hip_expm_pk_model fields (arrays as sequences)."""
        m = ExpmPKModel()
        keep = []
        arrays = {"transforms": np.int32, "treat_times": np.float64, "treat_doses": np.float64,
                  "obs_times": np.float64, "obs_conc": np.float64, "patient_ix": np.int32,
                  "treat_offset": np.int32, "obs_offset": np.int32}
        for name, _ in ExpmPKModel._fields_:
            v = fields[name] if name in fields else EXPM_PK_SINGLE_DEFAULTS[name]
            if name == "sigma_ix":
                m.sigma_ix = (C.c_int32 * 5)(*v)
            elif name in arrays and v is None:
                setattr(m, name, None)
            elif name in arrays:
                a = np.ascontiguousarray(v, dtype=arrays[name])
                keep.append(a)
                setattr(m, name, a.ctypes.data)
            else:
                setattr(m, name, v)
        h = C.c_void_p()
        check(lib().bcm3hip_open_expm_pk(device, C.byref(m), C.byref(h)), "bcm3hip_open_expm_pk")
        return cls(h, int(m.d))

    def set_option(self, opt: int, value: int):
        check(lib().bcm3hip_set_option(self.h, opt, int(value)), "bcm3hip_set_option")

    def eval(self, values: np.ndarray, detail: bool = False):
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, self.d)
        n = v.shape[0]
        logp = np.empty(n)
        status = np.empty(n, dtype=np.int32)
        if not detail:
            check(lib().bcm3hip_eval_batch(self.h, n, self.d, _ptr(v), _ptr(logp), _ptr(status)), "eval_batch")
            return logp, status
        pllh = np.empty(n * self.P)
        traj = np.empty(n * self.P * self.N * self.T)
        stats = np.empty(n * self.P, dtype=STATS_DTYPE)
        check(lib().bcm3hip_eval_batch_detail(self.h, n, self.d, _ptr(v), _ptr(logp), _ptr(status), _ptr(pllh),
                                              _ptr(traj), _ptr(stats)), "eval_batch_detail")
        return dict(logp=logp, status=status, patient_llh=pllh.reshape(n, self.P),
                    traj=traj.reshape(n, self.P, self.N, self.T), stats=stats.reshape(n, self.P))

    def eval_device(self, n: int, values_ptr: int, logp_ptr: int, status_ptr: Optional[int] = None,
                    stream: Optional[int] = None):
        check(lib().bcm3hip_eval_batch_device(self.h, n, values_ptr, logp_ptr, status_ptr, stream),
              "eval_batch_device")

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        check(lib().bcm3hip_last_kernel_ms(self.h, C.byref(ms)), "last_kernel_ms")
        return float(ms.value)

    def placement_log(self, n_max: int):
        """(n, 4) uint64 rows of the last PopPK launch with OPT_PLACEMENT_LOG on: HW_ID in the low 32 bits
        of word 0 with the trajectory's shader-clock cycles in its high 32 bits, XCC_ID, wall clock
        (100 MHz) at start and at end of each trajectory (include/bcm3hip.h)."""
        import numpy as np
        out = np.zeros((n_max, 4), dtype=np.uint64)
        m = lib().bcm3hip_placement_log(self.h, n_max, out.ctypes.data)
        if m < 0:
            check(int(m), "placement_log")
        return out[:m]

    def kernel_time_log(self):
        """(total_ms, launches, max_ms) of the launches logged since the last call (OPT_TIMING_LOG)."""
        tot, n, mx = C.c_double(), C.c_int64(), C.c_double()
        check(lib().bcm3hip_kernel_time_log(self.h, C.byref(tot), C.byref(n), C.byref(mx)), "kernel_time_log")
        return tot.value, n.value, mx.value

    def close(self):
        if self.h:
            lib().bcm3hip_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _u64(x: int) -> int:
    return int(x) & ((1 << 64) - 1)


def ptmh_propose(C, d, kind, p0, p1, scale, temps, values, prop, lprior_prop, chain0, seed, it, stream=None):
    """bcm3hip_ptmh_propose on device pointers (ints)."""
    check(lib().bcm3hip_ptmh_propose(C, d, kind, p0, p1, scale, temps, values, prop, lprior_prop, chain0,
                                     _u64(seed), _u64(it), stream), "ptmh_propose")


def ptmh_accept(C, d, temps, prop, lprior_prop, llh_prop, learning_rate, values, lprior, llh, lpp, accept_out,
                accepted, chain0, seed, it, stream=None, nan_llh=None):
    """bcm3hip_ptmh_accept on device pointers (ints; accept_out / accepted / nan_llh may be None)."""
    check(lib().bcm3hip_ptmh_accept(C, d, temps, prop, lprior_prop, llh_prop, learning_rate, values, lprior, llh, lpp,
                                    accept_out, accepted, nan_llh, chain0, _u64(seed), _u64(it), stream),
          "ptmh_accept")


def pt_exchange_local(C, d, g0, start, wrap_local, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, rnd,
                      stream=None):
    """bcm3hip_pt_exchange_local on device pointers (ints; acc_mask / accepted may be None)."""
    check(lib().bcm3hip_pt_exchange_local(C, d, g0, start, int(wrap_local), temps, values, llh, lprior, lpp,
                                          acc_mask, accepted, _u64(seed), _u64(rnd), stream), "pt_exchange_local")


def ptmh_propose_adaptive(C, d, kind, p0, p1, p2, temps, values, prop, lprior_prop, log_mh, proposal: Proposal,
                          chain0, seed, it, stream=None):
    """bcm3hip_ptmh_propose_adaptive on device pointers (ints) and a Proposal of device pointers."""
    check(lib().bcm3hip_ptmh_propose_adaptive(C, d, kind, p0, p1, p2, temps, values, prop, lprior_prop, log_mh,
                                              C_byref(proposal), chain0, _u64(seed), _u64(it), stream),
          "ptmh_propose_adaptive")


def ptmh_accept_adaptive(C, d, temps, prop, lprior_prop, llh_prop, log_mh, learning_rate, values, lprior, llh, lpp,
                         accept_out, accepted, proposal: Proposal, chain0, seed, it, stream=None, nan_llh=None):
    """bcm3hip_ptmh_accept_adaptive on device pointers (ints; accept_out / accepted / nan_llh may be None)."""
    check(lib().bcm3hip_ptmh_accept_adaptive(C, d, temps, prop, lprior_prop, llh_prop, log_mh, learning_rate, values,
                                             lprior, llh, lpp, accept_out, accepted, nan_llh, C_byref(proposal),
                                             chain0, _u64(seed), _u64(it), stream), "ptmh_accept_adaptive")


def pt_exchange_pair(C, d, i1, i2, g1, temps, values, llh, lprior, lpp, acc_out, accepted, seed, rnd, stream=None):
    """bcm3hip_pt_exchange_pair on device pointers (ints; acc_out / accepted may be None)."""
    check(lib().bcm3hip_pt_exchange_pair(C, d, i1, i2, g1, temps, values, llh, lprior, lpp, acc_out, accepted,
                                         _u64(seed), _u64(rnd), stream), "pt_exchange_pair")


def history_add(C, d, H, subsampling, temps, values, mask, history, counters, stream=None):
    """bcm3hip_history_add on device pointers (ints; mask may be None)."""
    check(lib().bcm3hip_history_add(C, d, H, subsampling, temps, values, mask, history, counters, stream),
          "history_add")


C_byref = C.byref


def gmm_eval(n, d, K, x, mean, chol, logc, weights, logpdf, resp, stream=None):
    """bcm3hip_gmm_eval on device pointers (ints; logpdf / resp may be None)."""
    check(lib().bcm3hip_gmm_eval(n, d, K, x, mean, chol, logc, weights, logpdf, resp, stream), "gmm_eval")
