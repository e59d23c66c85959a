#!/usr/bin/env python3
"""Headline benchmark: PopPK ODE log-likelihood evaluations/s in the PT-MH loop.

BASELINE.json metric "log-likelihood evals/sec (whole node), PopPK ODE @256 chains; HBM-roofline %"
on configs[2] (PopPK ODE likelihood, 256 chains x 1 trajectory each, batched BDF on 1 MI355X) and,
with --gpus N, configs[4] (256 chains per GPU, ladder sharded over N ranks, PT swap over RCCL).

One step = one DeterministicEvenOdd PT-MH iteration of every chain on the rank
(SamplerPT.cpp:203-212): exchange round, then a mutate move whose C likelihood evaluations
run as ONE batched launch of the HIP BDF kernel (bcm3_likelihood_evaluate_batch_device).
Everything stays in HBM; no host buffers inside the timed region.

python bench.py --gpus N --steps K --warmup W
    N > 1 without a torch.distributed environment: bench.py starts
    `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child process (before
    any GPU call) and exits with its code; under torch.distributed.run WORLD_SIZE must equal N.
    Default: 256 chains per GPU ("scaling": "weak"; N=1 is C3, N=8 is C5's 2,048 chains).
    --total-chains C fixes the ladder size over all GPUs instead ("scaling": "strong",
    SURVEY.md §8(e): C=2048 at 1/2/4/8 GPUs).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(ROOT, "tests", "golden")
LIK_XML = os.path.join(GOLDEN, "c3_likelihood.xml")
PRIOR_XML = os.path.join(GOLDEN, "c3_prior.xml")
PROFILES = os.path.join(ROOT, "profiles")

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X spec, half the 157.3 TF FP32 vector rate


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chains", type=int, default=256, help="tempered chains per GPU (weak scaling)")
    ap.add_argument("--total-chains", type=int, default=0,
                    help="tempered chains over all GPUs (strong scaling; must divide by the GPU count)")
    ap.add_argument("--lanes-per-wave", type=int, default=0, help="0 = auto")
    ap.add_argument("--proposal", default="gaussian_mixture",
                    help="ptmhsampler.proposal_type: gaussian_mixture (reference default) | global_covariance | "
                         "random_walk")
    ap.add_argument("--seed", type=int, default=20251016)
    ap.add_argument("--loop", default="native", choices=("native", "python"),
                    help="native: the C++ sampler (bcm3_ptmh_*); python: bcm3_amd.sampler.PTMHDevice")
    ap.add_argument("--speculate", type=int, default=1,
                    help="C++ loop: 1 = speculative iteration pairs (one likelihood launch per two iterations, "
                         "bit-identical chains), 0 = one launch per iteration")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--throughput-batch", type=int, default=16384,
                    help="extra: evals/s of one large batch (0 = skip); not the headline value")
    ap.add_argument("--issue-probe", type=int, default=1,
                    help="measure cycles per BDF step on a plain 256-proposal launch after the timed region "
                         "(0 = skip, so a kernel trace holds only the sampler's launches)")
    ap.add_argument("--extras", type=int, default=1, help="extra: P=64 and circular workloads (0 = skip)")
    ap.add_argument("--strong-chains", type=int, default=2048,
                    help="also time this fixed ladder size over all GPUs in the same run (the strong-scaling "
                         "companion of the weak headline, C5 = 2,048; 0 = skip)")
    ap.add_argument("--strong-steps", type=int, default=30, help="timed iterations of the strong-scaling run")
    return ap.parse_args()


def algorithmic_bytes_per_eval(m) -> int:
    """HBM bytes one likelihood evaluation must move at minimum: the parameter
    vector in, the observations of every patient in, logp out. Output times / doses are shared
    by every lane of a launch and counted once per launch, not per eval."""
    return 8 * m.d + 8 * m.P * m.T + 8


def flops_per_eval() -> float:
    """F_alg: mean FP64 operations of one C3 evaluation, frozen by op-counting the CPU
    restatement (tests/golden/c3_falg.json, tests/golden/make_falg.py)."""
    with open(os.path.join(GOLDEN, "c3_falg.json")) as f:
        return float(json.load(f)["flops_per_eval_mean"])


CLOCK_GHZ = 2.4  # MI355X peak engine clock (MI355X_MICROARCH.md)


def issue_rate(ll, x_dev, device):
    """Cycles per BDF step of the slowest trajectory of one launch (the launch lasts as long as its
    slowest trajectory): the kernel's duration on these proposals times the clock, over that
    trajectory's step count (solver statistics from a second, detail launch of the same inputs)."""
    import numpy as np
    from bcm3_amd import _hip
    x = x_dev.detach().cpu().numpy()
    ctx = _hip.Context.from_popk_model(ll.popk_model(), device.index or 0)
    try:
        ctx.eval(x)
        times = []
        for _ in range(3):
            ctx.eval(x)
            times.append(ctx.last_kernel_ms())
        ms = min(times)
        st = ctx.eval(x, detail=True)["stats"]
    finally:
        ctx.close()
    nst = st["nst"].reshape(len(x), -1).sum(axis=1)
    smax = int(nst.max())
    return {"kernel_ms": ms, "steps_slowest": smax, "steps_mean": float(nst.mean()),
            "cycles_per_step_slowest": ms * 1e-3 * CLOCK_GHZ * 1e9 / max(1, smax), "clock_ghz": CLOCK_GHZ,
            "issue_bound": issue_bound_from_profiles(len(x), float(nst.mean())),
            "note": "launch time is set by the slowest trajectory; issue_bound compares the measured "
                    "cycles per step with 4 cycles per issued instruction (DESIGN.md §7)"}


class NativeLoop:
    """The C++ sampler (libbcm3.so bcm3_ptmh_*): the timed iterations run without Python; the PT
    swap between ranks goes over RCCL (unique id broadcast over torch.distributed)."""

    def __init__(self, ll, num_chains, rank, world, args, dist):
        from bcm3_amd.ptmh import TRANSPORT_RCCL, PTMHNative, nccl_unique_id
        kw = {}
        if world > 1:
            obj = [nccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            kw = dict(transport=TRANSPORT_RCCL, nccl_id=obj[0])
        self.s = PTMHNative(ll, PRIOR_XML, num_chains, rank=rank, world=world, seed=args.seed,
                            proposal=args.proposal, speculate=args.speculate, **kw)
        self.exploration_steps = 1

    def run(self, n):
        if n > 0:
            self.s.iterate(n)

    def sync(self):
        self.s.synchronize()

    def acceptance(self):
        c = self.s.counters()
        return c["accepted_mutate"] / max(1, c["attempted_mutate"])

    def launch_counters(self):
        """(likelihood launches, trajectories they evaluated -- speculative candidates included)"""
        c = self.s.counters()
        return c["likelihood_launches"], c["evaluated_entries"]

    def values(self):
        import torch
        return torch.tensor(self.s.state()["values"])


class PythonLoop:
    """bcm3_amd.sampler.PTMHDevice (the same iteration written in Python over the same kernels)."""

    def __init__(self, ll, num_chains, rank, world, args, device):
        from bcm3_amd.pt import temperature_ladder
        from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior
        self.loop = PTMHDevice(ll, DevicePrior(load_prior(PRIOR_XML), device), temperature_ladder(num_chains),
                               rank=rank, world=world, seed=args.seed, device=device, proposal=args.proposal)
        self.exploration_steps = self.loop.exploration_steps

    def run(self, n):
        for _ in range(n):
            self.loop.iteration()

    def sync(self):
        self.loop.check_nan()

    def acceptance(self):
        return float(self.loop.accepted_mutate) / max(1, self.loop.attempted_mutate)

    def launch_counters(self):
        return None

    def values(self):
        return self.loop.prop


def spawn_ranks(args) -> int:
    """--gpus N > 1 outside torch.distributed: run this script under torch.distributed.run as a
    CHILD process (never an exec: nothing here has touched the GPU yet) and return its exit code."""
    import socket
    import subprocess
    import torch
    have = torch.cuda.device_count()  # does not initialise the GPU on this image
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {have} visible", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def traffic_from_profiles(tag: str, n: int):
    """HBM bytes per launch from the newest committed PMC summary (tools/pmc_traffic.py,
    profiles/<round tag>_traffic_<tag>.json), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(PROFILES, f"*_traffic_{tag}.json")), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
            if int(t.get("n", -1)) == n:
                return float(t["bytes_per_launch"])
        except (OSError, ValueError, KeyError):
            continue
    return None


def issue_bound_from_profiles(n: int, steps_mean: float):
    """The instruction-issue bound of the BDF kernel from the newest committed SQ counters
    (profiles/<tag>_traffic_c3_<n>.json: SQ_INSTS_VALU / SALU per launch, SQ_WAVE_CYCLES in quad
    cycles; profiles/<tag>_pmc_sq2.json: SQ_INSTS_BRANCH, SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY). A wavefront
    issues at most one instruction per 4 cycles (one issue slot per SIMD every 4 cycles, a wave64
    VALU instruction occupies its SIMD for 4), so 4 x instructions per step is the fastest one
    trajectory can step; the measured cycles per step are SQ_WAVE_CYCLES over the same waves."""
    import glob
    for path in sorted(glob.glob(os.path.join(PROFILES, f"*_traffic_c3_{n}.json")), reverse=True):
        try:
            with open(path) as f:
                t = json.load(f)
            sq = t["sq_per_launch"]
            tag = os.path.basename(path).split("_traffic_")[0]
            with open(os.path.join(PROFILES, f"{tag}_pmc_sq2.json")) as f:
                sq2 = json.load(f)
        except (OSError, ValueError, KeyError):
            continue
        waves = float(sq["SQ_WAVES"])
        per_step = lambda c: c / waves / steps_mean  # noqa: E731
        instr = per_step(sq["SQ_INSTS_VALU"] + sq["SQ_INSTS_SALU"] + sq2["SQ_INSTS_BRANCH"])
        measured = 4.0 * per_step(sq["SQ_WAVE_CYCLES"])
        return {"profile": os.path.basename(path), "valu_per_step": per_step(sq["SQ_INSTS_VALU"]),
                "salu_per_step": per_step(sq["SQ_INSTS_SALU"]), "branch_per_step": per_step(sq2["SQ_INSTS_BRANCH"]),
                "issue_bound_cycles_per_step": 4.0 * instr, "measured_cycles_per_step_mean": measured,
                "frac_of_issue_bound": 4.0 * instr / measured,
                "wait_share": sq2["SQ_WAIT_ANY"] / (sq2["SQ_WAIT_ANY"] + sq2["SQ_ACTIVE_INST_ANY"])}
    return None


def host_cores() -> int:
    """CPU threads this process may use: the box's share (OMP_NUM_THREADS is set to it on the GPU
    box), else the cgroup quota, else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return n


def cpu_baseline(budget_s: float, seed: int):
    """The reference CPU path on this box's host cores: the vendored CVODE 5.3.0 of the reference
    (compiled from its sources into oracle/_ref, with the restated PopPK glue) evaluating prior
    draws of the same C3 problem on a thread per core, like the reference's TaskManager fan-out."""
    sys.path[:0] = [os.path.join(ROOT, "oracle"), GOLDEN, os.path.join(ROOT, "tests")]
    import numpy as np
    import oracle as O
    import helpers as H
    kind = "reference"
    try:
        orc = O.Oracle("ref")
    except FileNotFoundError:
        orc, kind = O.Oracle("restated"), "port"
    prob = H.c3_problem(1)
    cores = host_cores()
    rng = np.random.default_rng(seed)
    lo = np.array([v.lower for v in prob.variables])
    hi = np.array([v.upper for v in prob.variables])
    batch = 256 * max(1, cores // 4)
    n = 0
    t0 = time.perf_counter()
    while True:
        x = lo + rng.random((batch, prob.d)) * (hi - lo)
        orc.popk_eval(prob, x, nthreads=cores, want_traj=False)
        n += batch
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": n / el, "unit": "log-likelihood evals/sec", "cores": cores, "kind": kind,
            "sample": f"{n} uniform prior draws of the C3 PopPK problem in batches of {batch}, "
                      f"{cores} threads, {el:.1f} s ({'oracle/_ref/libbcm3ref.so: reference CVODE 5.3.0 sources' if kind == 'reference' else 'oracle/liboracle.so restatement'})"}


def p64_cpu_baseline(budget_s: float, seed: int):
    """The reference CVODE (oracle/_ref) on the P=64 population variant, a thread per host core."""
    sys.path[:0] = [os.path.join(ROOT, "oracle"), GOLDEN, os.path.join(ROOT, "tests")]
    import numpy as np
    import oracle as O
    import helpers as H
    kind = "reference"
    try:
        orc = O.Oracle("ref")
    except FileNotFoundError:
        orc, kind = O.Oracle("restated"), "port"
    prob = H.c3_problem(64)
    cores = host_cores()
    rng = np.random.default_rng(seed)
    lo = np.array([v.lower for v in prob.variables])
    hi = np.array([v.upper for v in prob.variables])
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        x = lo + rng.random((cores, prob.d)) * (hi - lo)
        orc.popk_eval(prob, x, nthreads=cores, want_traj=False, full_patients=False)
        n += cores
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "log-likelihood evals/sec", "cores": cores, "kind": kind,
            "sample": f"{n} uniform prior draws of the P=64 problem (64 trajectories each), {cores} threads, {el:.1f} s"}


def _rate(ll, n, x, device, reps=3):
    import torch
    from bcm3_amd import _hip
    out = torch.empty(n, dtype=torch.float64, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
    torch.cuda.synchronize()
    ll.set_option(_hip.OPT_TIMING_LOG, 1)
    for _ in range(reps):
        ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
    tt, nl, _ = ll.kernel_time_log()
    ll.set_option(_hip.OPT_TIMING_LOG, 0)
    return tt / nl


def expm_cpu_baseline(budget_s: float, seed: int):
    """The reference CPU path of the matrix-exponential PK likelihoods: PharmacokineticModel::Solve
    on the reference's vendored Eigen (oracle/_ref/libexpmref.so, MatrixBase::exp) over uniform
    prior draws (the matrix set-up and the observation model, a few % of an evaluation, run
    untimed in Python): one thread, and the same solves on a thread per host core
    (eigen_pk_solve_batch, TaskManager's one task per chain)."""
    import ctypes as C
    sys.path[:0] = [os.path.join(ROOT, "oracle"), GOLDEN]
    import json
    import numpy as np
    import expm_pk as X
    import make_pharmaco_fixtures as S
    import make_pharmaco_population_fixtures as PF
    lib = X.ref_lib()
    with open(os.path.join(GOLDEN, "pharmaco_pkdata.json")) as f:
        pk = json.load(f)
    dp = C.POINTER(C.c_double)
    out = {}
    for tag, m, v in (("pharmaco_single_256chains", S.model_fields("all", "B2", pk), S.draws(4096, seed)),
                      ("pharmaco_population_256chains", PF.model_fields("all", pk), PF.draws("all", 4096, seed))):
        P = m.get("P", 1)
        toff = m.get("treat_offset") or [0, m["n_treat"]]
        ooff = m.get("obs_offset") or [0, m["n_obs"]]
        arr = lambda k, j, off: np.ascontiguousarray(m[k][off[j]:off[j + 1]], dtype=np.float64)  # noqa: E731
        pats = [(arr("treat_times", j, toff), arr("treat_doses", j, toff), arr("obs_times", j, ooff)) for j in range(P)]
        t_solve, n = 0.0, 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget_s and n < len(v):
            for j, (tt, td, ot) in enumerate(pats):
                A, _, _, _, ba = X.construct_matrix(m, v[n], j)
                a = np.asfortranarray(A)
                tdb = td * ba
                cen = np.empty(len(ot))
                t1 = time.perf_counter()
                lib.eigen_pk_solve(A.shape[0], a.ctypes.data_as(dp), len(tt), tt.ctypes.data_as(dp),
                                   tdb.ctypes.data_as(dp), len(ot), ot.ctypes.data_as(dp), cen.ctypes.data_as(dp))
                t_solve += time.perf_counter() - t1
            n += 1
        # the same draws' solves on every host core at once
        cores = host_cores()
        mats, jp, doses, doff, coff = [], [], [], [], []
        nd = len(v)
        tot_d = tot_c = 0
        for e in range(nd):
            for j, (tt, td, ot) in enumerate(pats):
                A, _, _, _, ba = X.construct_matrix(m, v[e], j)
                mats.append(np.asfortranarray(A).ravel(order="F"))
                jp.append(j)
                doses.append(td * ba)
                doff.append(tot_d)
                coff.append(tot_c)
                tot_d += len(td)
                tot_c += len(ot)
        a_all = np.ascontiguousarray(np.concatenate(mats))
        jp = np.array(jp, dtype=np.int32)
        d_all = np.ascontiguousarray(np.concatenate(doses))
        doff = np.array(doff, dtype=np.int64)
        coff = np.array(coff, dtype=np.int64)
        tofs = np.array(toff, dtype=np.int32)
        oofs = np.array(ooff, dtype=np.int32)
        tt_all = np.ascontiguousarray(m["treat_times"], dtype=np.float64)
        ot_all = np.ascontiguousarray(m["obs_times"], dtype=np.float64)
        cen = np.empty(tot_c)
        nA = X.construct_matrix(m, v[0], 0)[0].shape[0]
        reps, t1 = 0, time.perf_counter()
        while reps < 1 or time.perf_counter() - t1 < 1.0:  # repeat the batch for >= 1 s
            lib.eigen_pk_solve_batch(cores, len(jp), nA, a_all.ctypes.data, jp.ctypes.data, tofs.ctypes.data,
                                     tt_all.ctypes.data, d_all.ctypes.data, doff.ctypes.data, oofs.ctypes.data,
                                     ot_all.ctypes.data, coff.ctypes.data, cen.ctypes.data)
            reps += 1
        t_mt = (time.perf_counter() - t1) / reps
        out[tag] = {"value": nd / t_mt, "unit": "log-likelihood evals/sec", "cores": cores, "kind": "reference",
                    "evals_per_s_1thread": n / t_solve,
                    "sample": f"{nd} prior draws x {P} patient solve(s) on {cores} threads, {t_mt:.3f} s per pass "
                              f"({reps} passes); "
                              f"1 thread: {n} draws, {t_solve:.1f} s of Eigen solves"}
    return out


def cellpop_workload(device, gen, n=64):
    """Config C4 (BASELINE.json configs[3]): the cell-population likelihood (synthetic cell-cycle SBML
    model, 15 ODE species, 500 initial heterogeneous cells dividing over 20 h, ~1,500 cell
    trajectories per evaluation), 64 chains' proposals per launch -- the whole batch (the device-side cell
    work queue: init, solve, division bookkeeping and the reference's numbering in one persistent
    launch, then the data likelihood) timed with HIP events."""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.sampler import DevicePrior, load_prior
    lik, pri = os.path.join(GOLDEN, "cellpop_likelihood.xml"), os.path.join(GOLDEN, "cellpop_prior.xml")
    ll = Likelihood(lik, pri, device=device.index or 0)
    x = DevicePrior(load_prior(pri), device).sample(n, gen).contiguous()
    ms = _rate(ll, n, x, device, reps=2)
    cells = steps = 0
    for i in range(n):
        rec, _, _ = ll.cellpop_cells(i, 21, 15)
        cells += len(rec)
        steps += int(rec["nsteps"].sum())
    # evaluations that fail (-inf: too many cells, a solver failure) stop enqueueing cells
    # (cellpop_rt.cpp), so the all-draws rate mixes full and truncated evaluations:
    # the same launch size over finite draws only gives the full-evaluation rate
    import numpy as np
    import torch
    lp, _ = ll.evaluate_batch(x.detach().cpu().numpy())
    fin = np.flatnonzero(np.isfinite(lp))
    finite = {"finite_draws": int(fin.size), "of": n}
    if fin.size:
        xf = x[torch.as_tensor(fin[np.arange(n) % fin.size], device=x.device)].contiguous()
        ms_f = _rate(ll, n, xf, device, reps=2)
        finite.update(kernel_ms=ms_f, evals_per_s=n / (ms_f * 1e-3),
                      note="the same launch size over the finite draws of this batch, repeated in order")
    ll.close()
    # FP64 roofline: F_alg per cell BDF step from the operation-count model over the reference CVODE's
    # own per-cell counters (tests/golden/make_c4_falg.py), times the cell steps this launch took
    with open(os.path.join(GOLDEN, "c4_falg.json")) as fh:
        falg = json.load(fh)
    tf = falg["flops_per_cell_step"] * steps / (ms * 1e-3) / 1e12
    roof = {"bound": "fp64-vector (latency-limited chains)", "achieved": tf, "peak": FP64_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": tf / FP64_VECTOR_PEAK_TFLOPS,
            "flops_per_cell_step": falg["flops_per_cell_step"], "cell_steps_per_launch": steps,
            "method": falg["method"]}
    return {"chains": n, "kernel_ms": ms, "evals_per_s": n / (ms * 1e-3), "finite_only": finite,
            "cells_per_eval": cells / n, "roofline": roof,
            "cell_trajectories_per_s": cells / (ms * 1e-3), "bdf_steps_per_cell": steps / max(1, cells),
            "cell_bdf_steps_per_s": steps / (ms * 1e-3), "cells_per_wavefront": 4,
            "note": "throughput-bound (every SIMD busy); four cells per wavefront, one 16-lane row each, "
                    "from a device-side work queue in one persistent launch (DESIGN.md §4 'cell population')",
            "draws": x.detach().cpu().numpy()}


def cellpop_cpu_baseline(draws, budget_s: float):
    """The reference CPU path of C4: each evaluation's cells integrated by the reference's vendored
    CVODE 5.3.0 + PartialPivLU (oracle/_ref/libcellpopref.so) in the reference's sequential order,
    one evaluation per host thread (the sampling threads of TaskManager)."""
    import concurrent.futures as cf
    sys.path[:0] = [os.path.join(ROOT, "oracle")]
    import cellpop as CP
    prob = CP.load_problem(os.path.join(GOLDEN, "cellpop_likelihood.xml"), os.path.join(GOLDEN, "cellpop_prior.xml"))
    e = prob["experiments"][0]
    cores = host_cores()
    done = 0
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(cores) as pool:
        while time.perf_counter() - t0 < budget_s and done < len(draws):
            batch = draws[done:done + cores]
            list(pool.map(lambda v: CP.simulate_experiment(e, prob, v), batch))
            done += len(batch)
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "log-likelihood evals/sec", "cores": cores, "kind": "reference",
            "sample": f"{done} of the GPU line's prior draws, one evaluation per thread on {cores} threads, {el:.1f} s "
                      "(reference CVODE 5.3.0 + PartialPivLUExtended per cell, experiment logic restated)",
            "threading": "one evaluation per host thread, cells in the reference's FIFO order; the reference itself "
                         "runs one evaluation per sampling thread AND evaluation_threads auxiliary threads per "
                         "experiment (Experiment.cpp:691-782), which splits an evaluation's cells across cores -- "
                         "lower latency per evaluation, the same cores for the same total work, so at most this "
                         "throughput when every core is busy"}


def circular_in_sampler(device, seed, steps=400, warmup=40):
    """Config C2 in the sampler: the C++ PT-MH loop (bcm3_ptmh_iterate) over the
    circular-ridge likelihood, 256 chains on this GPU -- the config where the sampler loop itself, not
    the likelihood, is the cost. Rate = chains x iterations / wall time, timed like the headline
    (synchronize on both sides)."""
    import torch
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative
    lik, pri = os.path.join(GOLDEN, "circular_likelihood.xml"), os.path.join(GOLDEN, "circular_prior.xml")
    ll = Likelihood(lik, pri, device=device.index or 0)
    s = PTMHNative(ll, pri, 256, seed=seed)
    try:
        s.iterate(warmup)
        s.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.iterate(steps)
        s.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        c = s.counters()
    finally:
        s.close()
        ll.close()
    return {"chains": 256, "iterations": steps, "evals_per_s": 256 * steps / dt, "ms_per_iteration": dt / steps * 1e3,
            "likelihood_launches_per_iteration": c["likelihood_launches"] / max(1, c["iterations"]),
            "sampler_loop": "C++ host loop (libbcm3.so bcm3_ptmh_iterate), every kernel of the iteration on the GPU",
            "data": "synthetic; chains start at prior draws"}


def circular_cpu_baseline(budget_s: float, seed: int):
    """The C2 likelihood on the host cores: TestLikelihoodCircular::EvaluateLogProbability restated in C
    (oracle/liboracle.so orc_circular_eval, TestLikelihoodCircular.cpp:42-53) over uniform draws, one
    batch per thread. The likelihood alone: the reference's loop adds its proposals, accepts and
    exchanges on top of this, so this is an upper bound of its rate (the reference sampler needs Boost,
    absent here)."""
    import concurrent.futures as cf
    import ctypes
    sys.path[:0] = [os.path.join(ROOT, "oracle")]
    import numpy as np
    import oracle as O
    orc = O.Oracle("restated")
    cores = host_cores()
    per = 1 << 16
    rng = np.random.default_rng(seed)
    xs = [rng.uniform(-6.0, 6.0, size=(per, 2)) for _ in range(cores)]
    outs = [np.empty(per) for _ in range(cores)]
    fn = orc.lib.orc_circular_eval

    def one(k):
        fn(per, 2, 2.0, 3.5, 0.1, xs[k].ctypes.data, outs[k].ctypes.data)

    n, t0 = 0, time.perf_counter()
    with cf.ThreadPoolExecutor(cores) as pool:
        while time.perf_counter() - t0 < budget_s:
            list(pool.map(one, range(cores)))
            n += per * cores
    el = time.perf_counter() - t0
    return {"value": n / el, "unit": "log-likelihood evals/sec", "cores": cores, "kind": "port",
            "sample": f"{n} uniform draws in [-6, 6]^2 of the circular ridge (dimension 2, offset 3.5, radius 2, "
                      f"width 0.1), {cores} threads, {el:.1f} s; the likelihood alone (no proposals / accepts)"}


def extra_workloads(device, seed):
    """Secondary lines (not the headline): the P=64 population variant of C3 (256 chains x 64
    patient trajectories per launch) and config C2 (circular ridge, 256 chains)."""
    import torch
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.sampler import DevicePrior, load_prior
    out = {}
    gen = torch.Generator(device=device)
    gen.manual_seed(seed + 2)
    for name, tag, n in (("p64", "popk_p64_256chains", 256), ("circular", "circular_256chains", 256)):
        lik, pri = os.path.join(GOLDEN, f"{name}_likelihood.xml"), os.path.join(GOLDEN, f"{name}_prior.xml")
        ll = Likelihood(lik, pri, device=device.index or 0)
        x = DevicePrior(load_prior(pri), device).sample(n, gen).contiguous()
        ms = _rate(ll, n, x, device)
        rec = {"chains": n, "kernel_ms": ms, "evals_per_s": n / (ms * 1e-3)}
        if name == "p64":
            rec["trajectories_per_s"] = 64 * n / (ms * 1e-3)
        out[tag] = rec
        ll.close()
    out["circular_256chains"]["in_sampler"] = circular_in_sampler(device, seed)
    out.update(expm_workloads(device, gen))
    out["cellpop_c4_64chains"] = cellpop_workload(device, gen)
    return out


def expm_workloads(device, gen):
    """Secondary lines for the matrix-exponential PK likelihoods (expm_pk_kernel.hip): pharmaco_single
    (patient B2, all options: 8 compartments) and pharmaco_population (2 patients, peripheral + 3
    transit compartments, every random effect, bioavailability), 256 chains each."""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.sampler import DevicePrior, load_prior
    out = {}
    for tag, name, patients in (("pharmaco_single_256chains", "pharmaco_single", 1),
                                ("pharmaco_population_256chains", "pharmaco_population", 2)):
        lik = os.path.join(GOLDEN, f"{name}_likelihood.xml")
        pri = os.path.join(GOLDEN, "pharmaco_prior.xml" if patients == 1 else "pharmaco_population_prior.xml")
        ll = Likelihood(lik, pri, device=device.index or 0)
        n = 256
        x = DevicePrior(load_prior(pri), device).sample(n, gen).contiguous()
        ms = _rate(ll, n, x, device)
        out[tag] = {"chains": n, "patients": patients, "kernel_ms": ms, "evals_per_s": n / (ms * 1e-3)}
        ll.close()
    return out


def strong_run(ll, args, rank, world, device, dist):
    import torch
    cg = args.strong_chains
    loop = NativeLoop(ll, cg, rank, world, args, dist)
    try:
        return _strong_timed(loop, cg, args, world, device, dist)
    finally:
        loop.s.close()


def _strong_timed(loop, cg, args, world, device, dist):
    import torch
    loop.run(args.warmup)
    loop.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop.run(args.strong_steps)
    loop.sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    evals = cg * args.strong_steps * loop.exploration_steps
    return {"scaling": "strong", "global_chains": cg, "chains_per_gpu": cg // world, "n_gpus": world,
            "steps": args.strong_steps, "value": evals / dt, "unit": "log-likelihood evals/sec",
            "ms_per_step": dt / args.strong_steps * 1e3,
            "config": "C5" if cg == 2048 else "custom",
            "note": "the same ladder size at every GPU count: speedup(N) = value(N) / value(1); DESIGN.md §6 "
                    "gives the physical bound (one GPU already runs 2,048 chains near its chip-filling rate)"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)
    if args.total_chains and args.total_chains % world:
        print(f"bench.py: --total-chains {args.total_chains} does not divide over {world} GPUs", file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)  # RCCL on ROCm

    from bcm3_amd import _hip
    from bcm3_amd.likelihood import Likelihood

    ll = Likelihood(LIK_XML, PRIOR_XML, device=local)
    if args.lanes_per_wave:
        ll.set_option(_hip.OPT_LANES_PER_WAVE, args.lanes_per_wave)
    m = ll.popk_model()
    C = args.total_chains // world if args.total_chains else args.chains
    loop_kind = args.loop
    if args.loop == "native":
        # the C++ sampler is the measured loop; if its RCCL communicator cannot be set up this run
        # fails (never a silent switch to the Python loop, which is only run with --loop python)
        err = None
        try:
            loop = NativeLoop(ll, C * world, rank, world, args, dist if world > 1 else None)
        except RuntimeError as e:
            if world == 1:
                raise
            err = e
            print(f"bench.py rank {rank}: C++ sampler setup failed: {e}", file=sys.stderr, flush=True)
        if world > 1:
            ok = torch.tensor([0 if err else 1], device=device)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0:
                print(f"bench.py rank {rank}: the C++ sampler is unavailable on some rank; no fallback "
                      "(rerun with --loop python to time the Python loop)", file=sys.stderr, flush=True)
                dist.destroy_process_group()
                sys.exit(3)
    else:
        loop = PythonLoop(ll, C * world, rank, world, args, device)

    loop.run(args.warmup)
    loop.sync()
    torch.cuda.synchronize()
    ll.set_option(_hip.OPT_TIMING_LOG, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    lc0 = loop.launch_counters()
    t0 = time.perf_counter()
    loop.run(args.steps)
    loop.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lc1 = loop.launch_counters()
    # trajectories per likelihood launch, speculative candidates included (the headline
    # counts committed evaluations only; this is the solve work the GPU actually does)
    evaluated_per_launch = ((lc1[1] - lc0[1]) / max(1, lc1[0] - lc0[0])) if lc0 and lc1 else None
    k_total, k_launches, k_max = ll.kernel_time_log()
    ll.set_option(_hip.OPT_TIMING_LOG, 0)
    k_avg = k_total / max(1, k_launches)
    rank_k_ms = [k_avg]
    if world > 1:
        t = torch.tensor([dt, k_avg], dtype=torch.float64, device=device)
        allk = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(world)]
        dist.all_gather(allk, t[1:2].clone())
        rank_k_ms = [float(a) for a in allk]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, k_avg = float(t[0]), float(t[1])
    nan_flag = False  # loop.sync() raises on a NaN log-likelihood (Sampler.cpp:172-178)

    evals = C * world * args.steps * loop.exploration_steps
    value = evals / dt
    # committed evaluations per likelihood launch on this rank: C for one launch per iteration, 2C when
    # the C++ sampler runs speculative iteration pairs (one launch for two iterations; the launch also
    # evaluates the candidates that did not happen, which are not counted anywhere)
    per_launch = C * args.steps * loop.exploration_steps / max(1, k_launches)
    b_eval = algorithmic_bytes_per_eval(m)
    achieved_gbs = b_eval * per_launch / (k_avg * 1e-3) / 1e9
    tb = traffic_from_profiles("c3_256", C)
    f_alg = flops_per_eval()
    achieved_tf = f_alg * per_launch / (k_avg * 1e-3) / 1e12  # the kernel's own rate, like achieved_gbs
    issue = issue_rate(ll, loop.values(), device) if rank == 0 and args.issue_probe else None

    extra = {}
    if rank == 0 and args.throughput_batch > 0:
        # extra (not the headline): one large batch of proposals, to show the chip-filling rate
        n = args.throughput_batch
        gen = torch.Generator(device=device)
        gen.manual_seed(args.seed + 1)
        from bcm3_amd.sampler import DevicePrior, load_prior
        x = DevicePrior(load_prior(PRIOR_XML), device).sample(n, gen).contiguous()
        out = torch.empty(n, dtype=torch.float64, device=device)
        stream = torch.cuda.current_stream(device).cuda_stream
        ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
        torch.cuda.synchronize()
        ll.set_option(_hip.OPT_TIMING_LOG, 1)
        reps = 3
        for _ in range(reps):
            ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
        tt, nl, _ = ll.kernel_time_log()
        ll.set_option(_hip.OPT_TIMING_LOG, 0)
        extra["throughput_batch"] = {"n": n, "kernel_ms": tt / nl, "evals_per_s": n / (tt / nl * 1e-3)}

    if args.strong_chains and not args.total_chains and loop_kind == "native" and args.strong_chains % world == 0:
        # the fixed-size ladder north_star's strong scaling is about (C5: 2,048
        # chains over all GPUs), timed in the same run with the same barrier / max-over-ranks rule, so a
        # SCALE curve carries strong-scaling values next to the weak headline. The weak run's sampler
        # (and its RCCL communicator) is released first; a failure here is reported in the line and
        # never costs the headline
        acc_weak = loop.acceptance()
        loop.s.close()
        try:
            extra["strong_scaling"] = strong_run(ll, args, rank, world, device, dist if world > 1 else None)
        except Exception as ex:  # noqa: BLE001 -- reported, the weak headline stands
            extra["strong_scaling"] = {"error": f"{type(ex).__name__}: {ex}"}
            print(f"bench.py rank {rank}: strong-scaling run failed: {ex}", file=sys.stderr, flush=True)
        loop.acceptance = lambda: acc_weak  # (the headline's acceptance, read below)

    if rank == 0 and args.extras:
        extra.update(extra_workloads(device, args.seed))

    if world > 1:
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return

    cpu = None
    if world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args.cpu_seconds, args.seed)
        if args.extras:
            for tag, rec in expm_cpu_baseline(2.0, args.seed).items():
                if tag in extra:
                    extra[tag]["cpu_baseline"] = rec
            if "popk_p64_256chains" in extra:
                extra["popk_p64_256chains"]["cpu_baseline"] = p64_cpu_baseline(6.0, args.seed)
            if "circular_256chains" in extra:
                extra["circular_256chains"]["cpu_baseline"] = circular_cpu_baseline(2.0, args.seed)
            if "cellpop_c4_64chains" in extra:
                extra["cellpop_c4_64chains"]["cpu_baseline"] = cellpop_cpu_baseline(extra["cellpop_c4_64chains"]["draws"], 8.0)
    for rec in extra.values():
        if isinstance(rec, dict):
            rec.pop("draws", None)

    acc_mut = loop.acceptance()
    line = {
        "metric": "log-likelihood evals/sec (whole node), PopPK ODE @256 chains; HBM-roofline %",
        "value": value,
        "unit": "log-likelihood evals/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.total_chains else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (C3 PopPK data simulated from fixed true parameters; chains start at prior draws)",
        "config": {
            "workload": "PopPK ODE likelihood (pop_pk_trajectory, two-compartment lapatinib, 1 patient x 16 "
                        f"observations, 14 q24h doses, CVODE-BDF rtol 1e-6), {C * world} tempered chains over "
                        f"{world} GPU(s) ({C} per GPU); step = one PT-MH iteration (even/odd exchange + "
                        "mutate with one batched eval)",
            "config": ("C3" if C * world == 256 and world == 1 else
                       "C5" if C * world == 2048 else "custom"),
            "chains_per_gpu": C,
            "global_chains": C * world,
            "kernel_ms_per_rank": rank_k_ms,
            "lanes_per_wave": args.lanes_per_wave or "auto",
            "parallelism": f"chains sharded over {world} rank(s); PT swap = RCCL neighbour send/recv",
            "proposal": args.proposal,
            "sampler_loop": ("C++ host loop (libbcm3.so bcm3_ptmh_iterate), speculative iteration pairs"
                             if loop_kind == "native" and k_launches < args.steps else
                             "C++ host loop (libbcm3.so bcm3_ptmh_iterate)" if loop_kind == "native"
                             else "Python loop (bcm3_amd.sampler.PTMHDevice)"),
        },
        "roofline": {
            # the kernel is bound by one wavefront's FP64 instruction issue and dependent latency
            # (DESIGN.md §4, §7): achieved = F_alg (op-counted in the CPU restatement,
            # tests/golden/c3_falg.json) x committed evaluations per launch / the launch's average
            # duration; frac_of_issue_bound from the committed SQ counters; the HBM view follows
            "bound": "fp64-issue",
            "achieved": achieved_tf,
            "peak": FP64_VECTOR_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved_tf / FP64_VECTOR_PEAK_TFLOPS,
            "traffic": tb,
            "frac_of_issue_bound": ((issue or {}).get("issue_bound") or {}).get("frac_of_issue_bound"),
            "kernel": "popk_traj_kernel<TWO>",
            "kernel_ms_avg": k_avg,
            "committed_evals_per_launch": per_launch,
            "evaluated_trajectories_per_launch": evaluated_per_launch,
            "launches_per_step": k_launches / max(1, args.steps),
            "flops_per_eval": f_alg,
            "hbm": {"achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_eval": b_eval, "traffic_bytes_per_launch": tb},
            "issue": issue,
            "note": "traffic: PMC FETCH_SIZE + WRITE_SIZE bytes per launch (mostly code and constant fetch); "
                    "evaluated_trajectories_per_launch - committed_evals_per_launch are speculative candidates "
                    "that did not happen (DESIGN.md §4)",
        },
        "nan_llh_detected": nan_flag,
        "cpu_baseline": cpu,
        "kernel_share_of_step": k_avg * k_launches / max(1, args.steps) / (dt / args.steps * 1e3),
        "mutate_acceptance": acc_mut,
        **extra,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
