"""TEST INFRASTRUCTURE (oracle). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
this module; the product path never imports it.

CPU oracle of the reference's cell-population likelihood (likelihood type "cell_population"):
  CellPopulationLikelihood::Initialize / EvaluateLogProbability  src/cellpop/CellPopulationLikelihood.cpp:19-101
  Experiment::Load / PostInitialize / Initialize                  src/cellpop/Experiment.cpp:145-237, 404-633
  Experiment::EvaluateLogProbability / Simulate / SimulateCell    src/cellpop/Experiment.cpp:239-372, 635-782
  CellPopulation::AddNewCell / CountCellsAtTime                   src/cellpop/CellPopulation.cpp:36-121
  Cell::SetInitialConditionsFromOtherCell / Initialize            src/cellpop/Cell.cpp:79-191
  VariabilityDescription(+Variable)::GetPseudorandomVector / Apply* (diagonal_gaussian)
                                                                  src/cellpop/VariabilityDescription*.cpp
  VariabilityPseudoRandomIterator (Sobol)                          src/cellpop/VariabilityPseudoRandomIterator.cpp
  DataLikelihoodTimeCoursePopulationAverage                       src/cellpop/DataLikelihoodTimeCoursePopulationAverage.cpp
  DataLikelihoodTimeCourseBase / DataLikelihoodBase (Normal / t4 error models)
Each cell is integrated by oracle/_ref/libcellpopref.so (the reference's vendored CVODE + its
PartialPivLU, see oracle/cellpop_ref.cpp) on the generated derivative (oracle/sbml_codegen.py)
compiled for the host. The experiment logic runs here in Python in the reference's sequential
order (the single-thread FIFO of ParallelSimulation: cells in index order, children appended).

Restated without a pin (the reference gets them from Boost, absent here):
  * the Sobol sequence: boost::random::sobol (Joe & Kuo 2008 direction numbers, the first point
    skipped) through boost::random::uniform_01 (= x / 2^64) -- restated in sobol_points();
  * QuantileNormal = boost::math::quantile(normal) -- scipy.special.ndtri.
"""
import ctypes as C
import hashlib
import json
import math
import os
import subprocess
import xml.etree.ElementTree as ET

import numpy as np

import sbml_codegen as SG

HERE = os.path.dirname(os.path.abspath(__file__))
NAN = float("nan")
FLT_EPS = float(np.finfo(np.float32).eps)


class CellIn(C.Structure):
    _fields_ = [("N", C.c_int), ("rhs", C.c_void_p), ("constant_species", C.c_void_p), ("parameters", C.c_void_p),
                ("non_sampled_parameters", C.c_void_p), ("y0", C.c_void_p), ("creation_time", C.c_double),
                ("end_time", C.c_double), ("M", C.c_int), ("output_times", C.c_void_p), ("output_species", C.c_void_p),
                ("rtol", C.c_double), ("atol", C.c_double), ("hmin", C.c_double), ("hmax", C.c_double),
                ("max_steps", C.c_int), ("divide_cells", C.c_int), ("simulate_past_chromatid_separation_time", C.c_double),
                ("ev_replicating", C.c_int), ("ev_replicated", C.c_int), ("ev_pcna", C.c_int),
                ("ev_nuclear_envelope", C.c_int), ("ev_chromatid_separation", C.c_int), ("ev_cytokinesis", C.c_int),
                ("ev_apoptosis", C.c_int), ("n_constant", C.c_int), ("n_treat", C.c_int), ("treat_cs", C.c_void_p),
                ("treat_off", C.c_void_p), ("treat_times", C.c_void_p), ("stored", C.c_int),
                ("output_sync", C.c_void_p), ("sync_offset", C.c_double), ("solver", C.c_int)]


# ESynchronizeCellTrajectory (Experiment.h:21-27) of the synchronize attribute
# (DataLikelihoodTimeCourse.cpp:27-41, DataLikelihoodTimePoints.cpp:29-43)
SYNC_NONE = 4
_SYNC = {"": SYNC_NONE, "none": SYNC_NONE, "DNA_replication_start": 0, "PCNA_gfp_increase": 1, "mitosis": 2,
         "nuclear_envelope_breakdown": 2, "anaphase": 3, "anaphase_onset": 3}


class CellOut(C.Structure):
    _fields_ = [("ok", C.c_int), ("divided", C.c_int), ("died", C.c_int), ("sim_end", C.c_double),
                ("achieved_time", C.c_double), ("event_times", C.c_double * 5), ("nsteps", C.c_long),
                ("nsetups", C.c_long), ("nje", C.c_long), ("nni", C.c_long), ("netf", C.c_long), ("nfe", C.c_long)]


_libs = {}


def ref_lib(variant=""):
    """variant "" = the reference's flags; "nofma" = FMA contraction off (the build-to-build spread)"""
    if variant not in _libs:
        L = C.CDLL(os.path.join(HERE, "_ref", f"libcellpopref{'_' + variant if variant else ''}.so"))
        L.cp_simulate_cell.argtypes = [C.POINTER(CellIn), C.POINTER(CellOut), C.c_void_p, C.c_void_p]
        L.cp_simulate_cell.restype = C.c_int
        _libs[variant] = L
    return _libs[variant]


def compile_derivative(body: str, variant: str = "") -> C.CDLL:
    """The generated derivative for the host, with the reference's flags for generated code
    (SolverCodeGenerator.cpp:326: -O3 -march=native; x86-64-v3 here so it runs on any host)."""
    src = SG.host_translation_unit(body)
    h = hashlib.sha1((src + variant).encode()).hexdigest()[:16]
    d = os.path.join(HERE, "_ref", "codegen")
    os.makedirs(d, exist_ok=True)
    so = os.path.join(d, f"deriv_{h}.so")
    if not os.path.exists(so):
        cpp = os.path.join(d, f"deriv_{h}.cpp")
        with open(cpp, "w") as f:
            f.write(src)
        tmp = so + f".{os.getpid()}.tmp"
        flags = ["-ffp-contract=off"] if variant == "nofma" else []
        subprocess.run(["g++", "-O3", "-march=x86-64-v3", *flags, "-fPIC", "-shared", "-o", tmp, cpp], check=True)
        os.replace(tmp, so)
    return C.CDLL(so)


# ---- Sobol (boost::random::sobol, restated) --------------------------------------------------
# Joe & Kuo (2008) new-joe-kuo-6.21201: dimension d >= 2 -> (s, a, m_1..m_s); dimension 1 is the
# van der Corput sequence.
_JOE_KUO = [(1, 0, [1]), (2, 1, [1, 3]), (3, 1, [1, 3, 1]), (3, 2, [1, 1, 1]), (4, 1, [1, 1, 3, 3]),
            (4, 4, [1, 3, 5, 13]), (5, 2, [1, 1, 5, 5, 17]), (5, 4, [1, 1, 5, 5, 5]), (5, 7, [1, 1, 7, 11, 19]),
            (5, 11, [1, 1, 5, 1, 1]), (5, 13, [1, 1, 1, 3, 11]), (5, 14, [1, 3, 5, 5, 31])]


def _directions(dim, bits=64):
    if dim == 0:
        return [1 << (bits - 1 - k) for k in range(bits)]
    s, a, m = _JOE_KUO[dim - 1]
    m = list(m)
    for k in range(s, bits):
        v = m[k - s] ^ (m[k - s] << s)
        for j in range(1, s):
            if (a >> (s - 1 - j)) & 1:
                v ^= m[k - j] << j
        m.append(v)
    return [(m[k] << (bits - 1 - k)) & ((1 << bits) - 1) for k in range(bits)]


def sobol_points(n, dims):
    """n points of boost::random::sobol(dims) through uniform_01<double>: Gray-code order, the
    state XOR-ed with the direction of the lowest zero bit of the point counter before each point
    (so the first point is 0.5 in every dimension), value = state * 2^-64."""
    out = np.empty((n, dims))
    if dims == 0:
        return out
    v = [_directions(d) for d in range(dims)]
    state = [0] * dims
    for i in range(n):
        c = 0
        x = i
        while x & 1:
            x >>= 1
            c += 1
        for d in range(dims):
            state[d] ^= v[d][c]
            out[i, d] = float(state[d]) * 2.0 ** -64
    return out


def quantile_normal(p):
    from scipy.special import ndtri
    return float(ndtri(p))


# ---- problem set-up ---------------------------------------------------------------------------
def fastpow10(x):
    return math.exp(x * 2.3025850929940459)


def transform(tf, x):
    if tf == "log10":
        return fastpow10(x)
    return x


def _bool(s, default):
    if s is None:
        return default
    return s.strip().lower() in ("1", "true")


def load_problem(likelihood_xml, prior_xml, num_cells=None, max_cells=None, variant="", use_only_cell_ix="-1"):
    """use_only_cell_ix: the reference's cellpop.use_only_cell_ix option (CellPopulationLikelihood.cpp:116)"""
    root = ET.parse(prior_xml).getroot()
    variables, transforms = [], []
    for v in root.iter("variable"):
        for _ in range(int(v.get("repeat", "1"))):
            variables.append(v.get("name"))
            transforms.append("log10" if _bool(v.get("logspace"), False) else "none")
    base = os.path.dirname(os.path.abspath(likelihood_xml))
    lik = ET.parse(likelihood_xml).getroot()
    assert lik.get("type") == "cell_population"
    exps = []
    for ex in lik.iter("experiment"):
        exps.append(_load_experiment(ex, base, variables, num_cells, max_cells, variant, use_only_cell_ix))
    return dict(variables=variables, transforms=transforms, experiments=exps, variant=variant)


def _ref_value(s, variables):
    """ValueReference / DataLikelihoodBase::ParseString: sampled variable index, else a number."""
    if s in variables:
        return ("var", variables.index(s))
    return ("fixed", float(s))


def _load_experiment(ex, base, variables, num_cells, max_cells, variant="", use_only_cell_ix="-1"):
    model = SG.SBMLModel(os.path.join(base, ex.get("model_file")))
    e = dict(name=ex.get("name"), model=model)
    e["rtol"] = float(ex.get("solver_relative_tolerance", 4 * FLT_EPS))
    e["atol"] = float(ex.get("solver_absolute_tolerance", 4 * FLT_EPS))
    e["hmin"] = float(ex.get("solver_min_timestep", 1e-8))
    e["hmax"] = float(ex.get("solver_max_timestep", "inf"))
    e["max_steps"] = int(ex.get("solver_max_steps", 10000))
    # Cell::AllocateSolver (Cell.cpp:57-66): CVODE or DP5 (ODESolverDP5, restated in cellpop_ref.cpp)
    e["solver"] = {"CVODE": 0, "DP5": 1}[ex.get("solver_type", "CVODE")]
    e["num_cells"] = int(num_cells if num_cells is not None else ex.get("num_cells", 1))
    e["max_cells"] = int(max_cells if max_cells is not None else ex.get("max_cells", 20))
    e["divide_cells"] = _bool(ex.get("divide_cells"), True)
    e["trailing"] = float(ex.get("trailing_simulation_time", 0.0))
    e["past_cs"] = float(ex.get("simulate_past_chromatid_separation_time", 0.0))
    forced = {}
    for sp in ex.iter("set_parameter"):
        forced[sp.get("parameter_name")] = float(sp.get("value"))
    e["forced"] = forced
    # treatment trajectories (Experiment.cpp:571-584; TreatmentTrajectoryPulses::Load): in document
    # order, the constant species index and the sorted pulse start times
    treats = []
    for tt in ex.iter("treatment_trajectory"):
        assert tt.get("type") == "pulses", tt.get("type")
        ci = model.constant_index(tt.get("species_name"))
        assert ci is not None, tt.get("species_name")
        treats.append((ci, sorted(float(x) for x in tt.get("times").split(","))))
    e["treatments"] = treats
    # variabilities (VariabilityDescription::Load, VariabilityDescription.cpp:170-212)
    vds, vfull = [], []
    for cv in ex.iter("cell_variability"):
        assert cv.get("distribution") in ("diagonal_gaussian", "full_gaussian"), cv.get("distribution")
        vv = []
        for v in cv.iter("variable"):
            entry_time = v.get("entry_time", "") != ""
            vv.append(dict(species=v.get("initial_condition_species", ""), parameter=v.get("model_parameter", ""),
                           entry_time=entry_time, apply=v.get("apply"), scale=_ref_value(v.get("scale"), variables),
                           negate=_bool(v.get("negate"), False),
                           only_initial=_bool(v.get("only_initial_cells"), entry_time)))
        vds.append(vv)
        cov = None
        if cv.get("distribution") == "full_gaussian":
            b = cv.get("covar_base_name")
            cov = [_ref_value(f"{b}{j + 1}_{i + 1}", variables) for i in range(len(vv)) for j in range(i)]
        vfull.append(cov)
    e["variabilities"] = vds
    e["variability_cov"] = vfull
    # data file (JSON sidecar with the netCDF group's variables)
    with open(os.path.join(base, ex.get("data_file"))) as f:
        data = json.load(f)[e["name"]]
    dls = []
    timepoints = []  # Experiment::simulation_timepoints: (dl index, time, time_ix, species_ix)
    tp_sync = []     # their synchronisation point
    for dl in ex.iter("data"):
        sync = _SYNC[dl.get("synchronize", "")] if kind_of(dl) != "time_course_population_average" else SYNC_NONE
        kind = dl.get("type", "time_course")  # DataLikelihoodBase::Create (DataLikelihoodBase.cpp:22)
        assert kind in ("time_course_population_average", "time_course", "time_points"), kind
        var = data[dl.get("data_name")]
        if kind == "time_points":
            d = _load_time_points(dl, data, var, model, variables, e["max_cells"], use_only_cell_ix)
            # AddSimulationTimepoints once per species, at its first use (.cpp:139-188)
            for six in d["species_order"]:
                for ti, t in enumerate(d["times"]):
                    timepoints.append((len(dls), t, ti, six))
                    tp_sync.append(sync)
            _full_duration(timepoints, tp_sync, len(dls), d["times"], sync)
            dls.append(d)
            continue
        tdim = var["dims"][0]
        times = [float(t) for t in data[tdim]["data"]]
        obs = np.array(var["data"], dtype=float)
        if kind == "time_course":
            # DataLikelihoodTimeCourse::Load (DataLikelihoodTimeCourse.cpp:43-130): cells x time
            # points; a third (marker) dimension is read, of which one species uses column 0
            if obs.ndim == 1:
                assert use_only_cell_ix == "-1"
                obs = obs[None, :]
            else:
                if obs.ndim == 3:
                    obs = obs[:, :, 0]
                obs = obs.T
                if use_only_cell_ix != "-1":
                    obs = obs[[int(t) for t in use_only_cell_ix.split(",")]]
            assert e["max_cells"] == obs.shape[0], "max_cells must equal the observed cells (.cpp:174-183)"
            lineage = _load_lineage(data, obs.shape[0], use_only_cell_ix)
        else:
            if obs.ndim == 1:
                obs = obs[:, None]
            obs = obs.T  # replicates x timepoints
        sname = dl.get("species_name").strip()
        six = model.ode_index(sname)
        if six is None:
            six = len(model.ode) + model.constant_index(sname)
        em = dl.get("error_model", "normal")
        msd = dl.get("missing_simulation_time_stdev", "")
        d = dict(kind=kind, times=times, observed=obs, species=six, weight=float(dl.get("weight", 1.0)),
                 stdev=_ref_value(dl.get("stdev"), variables),
                 offset=_ref_value(dl.get("offset"), variables) if dl.get("offset") else None,
                 scale=_ref_value(dl.get("scale"), variables) if dl.get("scale") else None,
                 stdev_relative_to_scale=_bool(dl.get("stdev_relative_to_scale"), False),
                 error_model={"normal": "normal", "additive_normal": "normal", "student_t4": "t4", "t4": "t4",
                              "proportional_normal": "proportional",
                              "additive_proportional_normal": "additive_proportional"}[em],
                 proportional_stdev=(_ref_value(dl.get("proportional_stdev"), variables)
                                     if dl.get("proportional_stdev") else None),
                 # DataLikelihoodTimeCourseBase: missing_simulation_time_stdev, fixed 300 by default
                 missing_stdev=_ref_value(msd, variables) if msd else ("fixed", 300.0),
                 relative_to_time_average=_bool(dl.get("relative_to_time_average"), False),
                 lineage=lineage if kind == "time_course" else None)
        for ti, t in enumerate(times):
            timepoints.append((len(dls), t, ti, six))
            tp_sync.append(sync)
        _full_duration(timepoints, tp_sync, len(dls), times, sync)
        dls.append(d)
    # bubble sort by time (stable), Experiment.cpp:593-600
    order = sorted(range(len(timepoints)), key=lambda k: timepoints[k][1])
    e["data"] = dls
    e["timepoints"] = [timepoints[k] for k in order]
    e["timepoint_sync"] = [tp_sync[k] for k in order]
    # any synchronised entry: every cell stores its integration points (Experiment.cpp:119-121)
    e["stored"] = any(x != SYNC_NONE for x in e["timepoint_sync"])
    e["output_times"] = sorted(t[1] for t in timepoints)
    e["entry_time"] = _ref_value(ex.get("entry_time"), variables)
    # synchronization_time_offset (Experiment.cpp:172-185): a variable, or a number that the
    # reference writes to fixed_entry_time (replacing a constant entry time), the offset staying 0
    e["sync_offset"] = ("fixed", 0.0)
    so = ex.get("synchronization_time_offset", "")
    if so:
        if so in variables:
            e["sync_offset"] = ("var", variables.index(so))
        else:
            v = float(so)
            if e["entry_time"][0] == "fixed":
                e["entry_time"] = ("fixed", v)
    # derivative code (SBMLModel::GenerateCode) for the host copy
    e["derivative_body"] = model.generate_derivative(variables, forced)
    e["deriv_lib"] = compile_derivative(e["derivative_body"], variant)
    # event species: SIMULATED-species indices (Cell.cpp:44-50)
    def sim_ix(name):
        for i, s in enumerate(model.simulated):
            if model.species[s]["name"] == name:
                return i
        return -1
    e["events"] = [sim_ix(n) for n in ("replicating_DNA", "replicated_DNA", "PCNA_gfp", "nuclear_envelope",
                                       "chromatid_separation", "cytokinesis", "apoptosis")]
    e["reset"] = [(model.ode_index(n), v) for n, v in (("cytokinesis", 0.0), ("nuclear_envelope", 1.0), ("G1S_break", 1.0),
                                                       ("G2_break", 1.0), ("spindle_components", 0.0),
                                                       ("assembled_spindle", 0.0), ("chromatid_separation", 0.0))]
    dims = sum(len(v) for v in vds)
    e["sobol"] = sobol_points(e["num_cells"] * 100, dims) if dims else None
    e["y_init"] = np.array([model.species[s]["initial"] for s in model.ode])
    e["constant_init"] = np.array([model.species[s]["initial"] for s in model.constant])
    return e


INT_MIN = -2147483648


def _load_lineage(data, ncells, use_only_cell_ix):
    """observed lineage of a time course (DataLikelihoodTimeCourse.cpp:132-167): "parent" holds the
    parent's "cell_id" (INT_MIN: none); returns (roots in data order, children per cell ascending)
    or None without a "parent" variable"""
    if "parent" not in data:
        return None
    ids, par = data["cell_id"]["data"], data["parent"]["data"]
    pick = list(range(ncells)) if use_only_cell_ix == "-1" else [int(t) for t in use_only_cell_ix.split(",")]
    idp = [int(ids[p]) for p in pick]
    children = [[] for _ in pick]
    roots = []
    for j, p in enumerate(pick):
        pv = int(par[p])
        if pv != INT_MIN:
            children[idp.index(pv)].append(j)  # ValueError: "Could not find cell ... for parent"
        else:
            roots.append(j)
    return roots, children


def kind_of(dl):
    return dl.get("type", "time_course")


def _full_duration(timepoints, tp_sync, dli, times, sync):
    """a synchronised time course / time points also simulates its full duration, for negative
    time points (DataLikelihoodTimeCourse.cpp:192-199, DataLikelihoodTimePoints.cpp:190-197): an
    entry without species"""
    if sync != SYNC_NONE and times:
        full_duration = times[-1] - times[0]
        if full_duration > times[-1]:
            timepoints.append((dli, full_duration, -1, -1))
            tp_sync.append(sync)


def _load_time_points(dl, data, var, model, variables, max_cells, use_only_cell_ix):
    """DataLikelihoodTimePoints::Load (DataLikelihoodTimePoints.cpp:19-201) and the per-column
    references of DataLikelihoodBase::PostInitialize (DataLikelihoodBase.cpp:77-127)"""
    times = [float(t) for t in data[var["dims"][0]]["data"]]
    obs = np.array(var["data"], dtype=float)
    assert obs.ndim in (2, 3), "Need 2 or 3 dimensional data"
    if obs.ndim == 2:
        if use_only_cell_ix != "-1":
            obs = obs[:, [int(t) for t in use_only_cell_ix.split(",")]]
        obs = obs[:, :, None]
    else:
        assert use_only_cell_ix == "-1", "Not implemented yet"
    obs = obs.transpose(1, 0, 2)  # cells x time points x markers
    assert max_cells >= obs.shape[0]
    sname = dl.get("species_name")
    cols = [c.strip() for c in sname.split(";")] if ";" in sname else [sname]
    species_map = {}  # species index -> columns it adds to, in order
    order = []
    for l, col in enumerate(cols):
        assert "/" not in col, "Division currently not supported for time points data"
        for t in ([x.strip() for x in col.split("+")] if "+" in col else [col]):
            six = model.ode_index(t)
            assert six is not None, t
            if six not in species_map:
                species_map[six] = []
                order.append(six)
            species_map[six].append(l)
    assert len(cols) <= obs.shape[2]

    def refs(attr, none):
        s = dl.get(attr, "")
        toks = s.split(";") if s else []
        out = []
        for l in range(len(cols)):
            if len(toks) == 1:
                out.append(_ref_value(toks[0], variables))
            elif l < len(toks):
                out.append(_ref_value(toks[l], variables))
            elif toks:
                out.append(("fixed", math.nan))  # GetCurrent*: "Out of bounds" -> NaN
            else:
                out.append(("fixed", none))
        return out

    em = dl.get("error_model", "normal")
    rel = dl.get("value_relative_to_timepoint_ix")
    return dict(kind="time_points", times=times, observed=obs, columns=len(cols), species_map=species_map,
                species_order=order, species=order[0], weight=float(dl.get("weight", 1.0)),
                stdevs=refs("stdev", 1.0), offsets=refs("offset", 0.0), scales=refs("scale", 1.0),
                stdev_relative_to_scale=_bool(dl.get("stdev_relative_to_scale"), False),
                error_model={"normal": "normal", "additive_normal": "normal", "student_t4": "t4", "t4": "t4"}[em],
                relative_ix=int(rel) if rel is not None else None,
                only_nondivided=_bool(dl.get("use_only_nondivided"), False))


def notify_time_points(e, dli, values):
    """cell_trajectories of time-points data likelihood dli from the cells' values at the sorted
    simulation time points (values[cell][entry]): Experiment.cpp:298-311 calls NotifySimulatedValue
    for every time point in order and every cell with a non-NaN value; DataLikelihoodTimePoints::
    NotifySimulatedValue (.cpp:345-370) skips daughters under use_only_nondivided and adds the value
    to every column the species belongs to. Returns traj[max_cells][T][columns]."""
    d = e["data"][dli]
    traj = np.full((e["max_cells"], len(d["times"]), d["columns"]), np.nan)
    for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
        if tdl != dli or ti < 0:
            continue
        for c in range(len(values)):
            x = values[c][k]
            if x != x or (d["only_nondivided"] and c >= e["num_cells"]):
                continue
            for l in d["species_map"][six]:
                v = traj[c, ti, l]
                traj[c, ti, l] = x if math.isnan(v) else v + x
    return traj


def _timepoints_logp(d, traj, tv):
    """DataLikelihoodTimePoints::Evaluate (DataLikelihoodTimePoints.cpp:210-343): at every time point
    the observed cells with a finite marker against the simulated cells with a value, matched by the
    vendored hungarian2 routine (oracle/hungarian.py) over (observed, simulated) edges in row order;
    traj[cell][ti][column]."""
    import hungarian as HG
    L = d["columns"]
    scales = [_refval(r, tv) for r in d["scales"]]
    offsets = [_refval(r, tv) for r in d["offsets"]]
    stdevs = [_refval(r, tv) * (scales[l] if d["stdev_relative_to_scale"] else 1.0) for l, r in enumerate(d["stdevs"])]
    rel = d["relative_ix"]
    obs = d["observed"]
    logp = 0.0
    for ti in range(len(d["times"])):
        rows = [i for i in range(obs.shape[0]) if np.isfinite(obs[i, ti]).any()]
        if not rows:
            continue
        sims = [j for j in range(traj.shape[0])
                if not math.isnan(traj[j, ti, 0]) and (rel is None or not math.isnan(traj[j, rel, 0]))]
        if len(sims) < len(rows):
            return -math.inf
        lik = np.full((len(rows), len(sims)), -math.inf)
        edges = []
        for a, i in enumerate(rows):
            for b, j in enumerate(sims):
                cl = 0.0
                for l in range(L):
                    x = traj[j, ti, l]
                    if rel is not None:
                        x += offsets[l]
                        x /= traj[j, rel, l]
                        x *= scales[l]
                    else:
                        x *= scales[l]
                        x += offsets[l]
                    y = obs[i, ti, l]
                    if math.isnan(y):
                        continue
                    cl += _log_pdf_tnu4(y, x, stdevs[l]) if d["error_model"] == "t4" else _log_pdf_normal(y, x, stdevs[l])
                lik[a, b] = cl
                edges.append((a, b, -cl))
        match = HG.min_weight_perfect_matching(len(rows), len(sims), edges)
        if len(match) != len(rows):
            return -math.inf
        for a in range(len(rows)):
            logp += lik[a, match[a]]
    return logp * d["weight"]


def _apply(kind, x, value):
    # VariabilityDescriptionVariable::Apply
    if kind == "additive":
        return x + value
    if kind == "additive_log":
        return x + math.exp(value)
    if kind == "additive_log2":
        return x + math.pow(2.0, value)
    if kind == "multiplicative":
        return x * value
    if kind == "multiplicative_log":
        return x * math.exp(value)
    if kind == "multiplicative_log2":
        return x * math.pow(2.0, value)
    if kind == "replace":
        return value
    raise ValueError(kind)


def _refval(ref, tv):
    return tv[ref[1]] if ref[0] == "var" else ref[1]


def _cell_init(e, prob, tv, y, sobol_ix, is_initial):
    """Cell::Initialize: variability on parameters and initial conditions."""
    params = np.array(tv, dtype=float)
    y = np.array(y, dtype=float)
    k = 0
    for g, vv in enumerate(e["variabilities"]):
        cov = e.get("variability_cov", [None] * len(e["variabilities"]))[g]
        if cov is None:
            # VariabilityDescription::GetPseudorandomVector (diagonal, VariabilityDescription.cpp:58-67)
            pr = []
            for v in vv:
                scale = _refval(v["scale"], tv)
                pr.append(quantile_normal(e["sobol"][sobol_ix, k]) * math.exp(scale))
                k += 1
        else:
            # full gaussian (:69-128): spherical Cholesky factor L from exp(scale_i) and cov(k, i) * pi,
            # then L z with z = QuantileNormal(sobol), summed over j in order
            D = len(vv)
            L = [[0.0] * D for _ in range(D)]
            for i in range(D):
                exp_scale = math.exp(_refval(vv[i]["scale"], tv))
                for j in range(i + 1):
                    x = exp_scale
                    for kk in range(i):
                        if kk <= j:
                            cvv = _refval(cov[(i - 1) * i // 2 + kk], tv) * math.pi
                            x *= math.cos(cvv) if kk == j else math.sin(cvv)
                    L[i][j] = x
            z = [quantile_normal(e["sobol"][sobol_ix, k + i]) for i in range(D)]
            pr = []
            for i in range(D):
                acc = L[i][0] * z[0]
                for j in range(1, D):
                    acc = acc + L[i][j] * z[j]
                pr.append(acc)
            k += D
        for i, name in enumerate(prob["variables"]):
            for v, r in zip(vv, pr):
                if v["parameter"] and v["parameter"] == name and (not v["only_initial"] or is_initial):
                    params[i] = _apply(v["apply"], params[i], -r if v["negate"] else r)
        for i, s in enumerate(e["model"].ode):
            name = e["model"].species[s]["name"]
            for v, r in zip(vv, pr):
                if v["species"] and v["species"] == name and (not v["only_initial"] or is_initial):
                    y[i] = _apply(v["apply"], y[i], -r if v["negate"] else r)
    return params, y


def simulate_experiment(e, prob, values):
    """Experiment::EvaluateLogProbability for one parameter vector: per-cell records, population
    averages, logp."""
    tv = [transform(tf, x) for tf, x in zip(prob["transforms"], values)]
    model = e["model"]
    N = len(model.ode)
    out_times = np.array(e["output_times"], dtype=float)
    M = len(out_times)
    # per sorted output index: the species the data likelihoods read there
    out_species = np.full(M, -1, dtype=np.int32)
    for k, tp in enumerate(e["timepoints"]):
        out_species[k] = tp[3]
    end_time = (e["timepoints"][-1][1] if e["timepoints"] else 0.0) + e["trailing"]
    entry_time = _refval(e["entry_time"], tv)
    lib = ref_lib(prob.get("variant", ""))
    rhs = C.cast(e["deriv_lib"].generated_derivative, C.c_void_p).value
    const = np.ascontiguousarray(e["constant_init"], dtype=float)
    treats = e.get("treatments", [])
    t_cs = np.array([t[0] for t in treats] or [0], dtype=np.int32)
    t_off = np.array([0] + list(np.cumsum([len(t[1]) for t in treats])), dtype=np.int32)
    t_times = np.array([x for t in treats for x in t[1]] or [0.0], dtype=float)
    out_sync = np.array(e.get("timepoint_sync", [SYNC_NONE] * M), dtype=np.int32)
    sync_offset = _refval(e.get("sync_offset", ("fixed", 0.0)), tv)
    cells = []  # dicts
    fail = False

    def add_cell(creation, parent, child_ix, is_initial):
        if len(cells) == e["max_cells"]:
            return None
        ix = len(cells)
        if parent is None:
            y = e["y_init"].copy()
            sidx = ix
        else:
            y = parent["end_y"].copy()
            for r, v in e["reset"]:
                y[r] = v
            sidx = e["num_cells"] + parent["sobol_ix"] * 2 + child_ix
            if e["sobol"] is not None and sidx >= e["sobol"].shape[0]:
                return None
        params, y = (_cell_init(e, prob, tv, y, sidx, is_initial) if e["sobol"] is not None
                     else (np.array(tv, dtype=float), y))
        c = dict(index=ix, creation=creation, sobol_ix=sidx, params=params, y0=y, parent=parent["index"] if parent else -1)
        cells.append(c)
        return c

    n0 = e["num_cells"]
    if n0 > 1:
        for i in range(n0):
            add_cell(entry_time, None, -1, True)
    else:
        add_cell(entry_time, None, -1, False)
    if entry_time < -7.0 * 24.0 * 60.0 * 60.0:
        return dict(ok=False, logp=-math.inf, cells=cells)
    i = 0
    while i < len(cells):  # FIFO: ParallelSimulation with one thread
        c = cells[i]
        cin = CellIn()
        cin.N = N
        cin.rhs = rhs
        cin.constant_species = const.ctypes.data
        prm = np.ascontiguousarray(c["params"])
        y0 = np.ascontiguousarray(c["y0"])
        cin.parameters = prm.ctypes.data
        cin.non_sampled_parameters = None
        cin.y0 = y0.ctypes.data
        cin.creation_time = c["creation"]
        cin.end_time = end_time
        cin.M = M
        cin.output_times = out_times.ctypes.data
        cin.output_species = out_species.ctypes.data
        cin.rtol, cin.atol, cin.hmin, cin.hmax = e["rtol"], e["atol"], e["hmin"], e["hmax"]
        cin.max_steps = e["max_steps"]
        cin.divide_cells = 1 if e["divide_cells"] else 0
        cin.simulate_past_chromatid_separation_time = e["past_cs"]
        (cin.ev_replicating, cin.ev_replicated, cin.ev_pcna, cin.ev_nuclear_envelope, cin.ev_chromatid_separation,
         cin.ev_cytokinesis, cin.ev_apoptosis) = e["events"]
        cin.n_constant = len(const)
        cin.n_treat = len(treats)
        cin.treat_cs = t_cs.ctypes.data
        cin.treat_off = t_off.ctypes.data
        cin.treat_times = t_times.ctypes.data
        cin.stored = 1 if e.get("stored") else 0
        cin.output_sync = out_sync.ctypes.data
        cin.sync_offset = sync_offset
        cin.solver = e.get("solver", 0)
        cout = CellOut()
        vals = np.empty(M)
        end_y = np.empty(N)
        lib.cp_simulate_cell(C.byref(cin), C.byref(cout), vals.ctypes.data, end_y.ctypes.data)
        c.update(ok=bool(cout.ok), divided=bool(cout.divided), died=bool(cout.died), sim_end=cout.sim_end,
                 achieved=cout.achieved_time, events=list(cout.event_times), values=vals, end_y=end_y,
                 nsteps=cout.nsteps, stats=dict(nsetups=cout.nsetups, nje=cout.nje, nni=cout.nni, netf=cout.netf,
                                                 nfe=cout.nfe))
        if not cout.ok:
            fail = True
            break
        if e["divide_cells"] and c["divided"] and c["achieved"] < end_time:
            c1 = add_cell(c["achieved"], c, 0, False)
            c2 = add_cell(c["achieved"], c, 1, False)
            if c1 is None or c2 is None:
                fail = True
                break
        i += 1
    if fail:
        return dict(ok=False, logp=-math.inf, cells=cells)
    # population averages / cell trajectories (Experiment.cpp:298-311 + NotifySimulatedValue)
    avgs = [np.zeros((len(d["times"]), 1)) for d in e["data"]]
    trajs = [np.full((e["max_cells"], len(d["times"])) + ((d["columns"],) if d["kind"] == "time_points" else ()), np.nan)
             for d in e["data"]]
    for k, (dli, t, ti, six) in enumerate(e["timepoints"]):
        if ti < 0:
            continue
        # CountCellsAtTime(st.time + time_offset, ...) (Experiment.cpp:285, 301)
        alive = [c for c in cells if 0.0 <= (t + sync_offset) - c["creation"] <= c["sim_end"]]
        pop = len(alive)
        d = e["data"][dli]
        for c in cells:
            x = c["values"][k]
            if x == x:
                if d["kind"] == "time_points":
                    continue
                if d["kind"] == "time_course_population_average":
                    avgs[dli][ti, 0] += x / pop
                trajs[dli][c["index"], ti] = x
    for dli, d in enumerate(e["data"]):
        if d["kind"] == "time_points" and cells:
            trajs[dli] = notify_time_points(e, dli, np.array([c["values"] for c in cells]))
    # Experiment::EvaluateLogProbability (Experiment.cpp:346-355): a data likelihood whose Evaluate
    # returns false ends the sum there, and the experiment keeps what it had (it still succeeds)
    logp = 0.0
    roots = [c["parent"] < 0 for c in cells]
    # NotifyParents (DataLikelihoodTimeCourse.cpp:411-429): each cell's first daughter, -1 = none
    sim_child = [-1] * len(cells)
    for c in cells:
        if c["parent"] >= 0 and sim_child[c["parent"]] < 0:
            sim_child[c["parent"]] = c["index"]
    for dli, d in enumerate(e["data"]):
        if d["kind"] == "time_course":
            ok, lp = _timecourse_logp(d, trajs[dli], roots, tv, sim_child)
            if not ok:
                break
            logp += lp
        elif d["kind"] == "time_points":
            logp += _timepoints_logp(d, trajs[dli], tv)
        else:
            logp += _popavg_logp(d, avgs[dli], tv)
    return dict(ok=True, logp=logp, cells=cells, population_average=[a[:, 0] for a in avgs],
                cell_trajectories=trajs)


def _data_stdev(d, tv, scale):
    """DataLikelihoodBase::GetCurrentSTDev (DataLikelihoodBase.cpp:130-156)"""
    s = _refval(d["stdev"], tv)
    return s * scale if d.get("stdev_relative_to_scale") else s


def _log_pdf_normal(x, mu, sigma):
    # bcm3::LogPdfNormal (src/utils/ProbabilityDistributions.cpp:129-138)
    two_sigma_sq = 2.0 * sigma * sigma
    dd = x - mu
    return -math.log(sigma) - 0.91893853320467274178032973640562 - dd * dd / two_sigma_sq


def _log_pdf_tnu4(x, mu, sigma):
    # bcm3::LogPdfTnu4 (ProbabilityDistributions.cpp:216-224)
    xn = (x - mu) / sigma
    return -0.9808292530117262 - 2.5 * math.log1p(0.25 * xn * xn) - math.log(sigma)


def _timecourse_logp(d, traj, roots, tv, sim_child=None):
    """DataLikelihoodTimeCourse::Evaluate (DataLikelihoodTimeCourse.cpp:230-365) for one species and
    no observed lineage: the likelihood of every observed cell against every simulated initial cell
    (CalculateCellLikelihood, :431-497; missing simulated values: CalculateMissingValueLikelihood,
    :566-588), then the observed-to-simulated assignment of the vendored hungarian2 routine
    (oracle/hungarian.py). Returns (Evaluate's result, logp)."""
    import hungarian as HG
    offset = _refval(d["offset"], tv) if d["offset"] else 0.0
    scale = _refval(d["scale"], tv) if d["scale"] else 1.0
    stdev = _data_stdev(d, tv, scale)
    pstd = _refval(d["proportional_stdev"], tv) if d["proportional_stdev"] else 0.0
    msd = _refval(d["missing_stdev"], tv)
    em = d["error_model"]
    times = d["times"]
    T = len(times)
    x = traj * scale  # (.cpp:236-241): col *= scale; col += offset
    x = x + offset
    obs = d["observed"]
    R = obs.shape[0]
    nsim = len(roots)
    n = max(R, nsim)

    def missing(j, k):
        first = times[T - 1]
        for m in range(T):
            if not math.isnan(x[j, m]):
                first = times[m]
                break
        last = times[0]
        for m in range(T - 1, -1, -1):
            if not math.isnan(x[j, m]):
                last = times[m]
                break
        off = min(abs(times[k] - first), abs(times[k] - last))
        return _log_pdf_tnu4(off, 0.0, msd) if em == "t4" else _log_pdf_normal(off, 0.0, msd)

    def cell(i, j):
        lp = 0.0
        mls = -math.log(stdev)
        inv2 = 1.0 / (2.0 * stdev * stdev)
        for k in range(T):
            y = obs[i, k]
            if math.isnan(y):
                continue
            xv = x[j, k]
            if math.isnan(xv):
                lp += missing(j, k)
            elif em == "normal":
                dd = y - xv
                lp += mls - 0.91893853320467274178032973640562 - dd * dd * inv2
            elif em == "t4":
                lp += _log_pdf_tnu4(y, xv, stdev)
            else:
                # (.cpp:274-285): sigma from the scaled trajectory, Eigen's vectorised log and
                # inverse (the device and this checker use the scalar log: see the test's tolerance)
                sigma = np.float64(pstd * max(xv, 0.0))
                if em == "additive_proportional":
                    sigma += stdev
                dd = y - xv
                with np.errstate(all="ignore"):  # IEEE: sigma = 0 gives inf - inf = NaN
                    lp += float(-np.log(sigma) - 0.91893853320467274178032973640562
                                - dd * dd * (np.float64(1.0) / (2.0 * (sigma * sigma))))
        return lp

    lineage = d.get("lineage")
    if lineage is not None:
        # CalculateCellLikelihood's recursion over the observed lineage (.cpp:431-563)
        obs_roots, obs_children = lineage

        def rec(o, s):
            lp = 0.0
            if s is None:
                for k in range(T):
                    if not math.isnan(obs[o, k]):
                        lp += _log_pdf_tnu4(times[k], 0.0, msd) if em == "t4" else _log_pdf_normal(times[k], 0.0, msd)
                for ch in obs_children[o]:
                    lp += rec(ch, None)
                return lp
            lp = cell(o, s)
            if lp == -math.inf:
                return lp
            if obs_children[o]:
                d0 = sim_child[s] if sim_child is not None else -1
                if d0 >= 0:
                    m = [[rec(ch, d0), rec(ch, d0 + 1)] for ch in obs_children[o]]
                    if sum(1 for a, _ in m if a > -math.inf) == 0 or sum(1 for _, b in m if b > -math.inf) == 0:
                        return -math.inf
                    if len(m) == 1:
                        lp += m[0][0] if m[0][0] > m[0][1] else m[0][1]
                    # two or more observed children: the reference's #if TODO block adds nothing
                else:
                    for ch in obs_children[o]:
                        lp = rec(ch, None)  # assigned, not added (.cpp:555-557)
            return lp

        R = len(obs_roots)
        n = max(R, nsim)
        row_cell = obs_roots
    else:
        def rec(o, s):
            return cell(o, s)
        row_cell = list(range(R))
    L = np.full((n, n), 0.0)
    edges = []
    for i in range(R):
        finite = 0
        for j in range(nsim):
            if roots[j]:
                L[i, j] = rec(row_cell[i], j)
                if math.isnan(L[i, j]):
                    return False, -math.inf
                if L[i, j] > -math.inf:
                    finite += 1
            else:
                L[i, j] = -math.inf
            edges.append((i, j, -L[i, j]))
        if finite < R:
            return True, -math.inf
    match = HG.min_weight_perfect_matching(n, nsim, edges)
    if len(match) != R:
        return True, -math.inf
    lp = 0.0
    for i in range(R):
        lp += L[i, match[i]]
    return True, lp * d["weight"]


def _popavg_logp(d, avg, tv):
    """DataLikelihoodTimeCoursePopulationAverage::Evaluate (one species)."""
    offset = _refval(d["offset"], tv) if d["offset"] else 0.0
    scale = _refval(d["scale"], tv) if d["scale"] else 1.0
    stdev = _data_stdev(d, tv, scale)
    a = avg.copy()
    if d["relative_to_time_average"]:
        # DataLikelihoodTimeCoursePopulationAverage.cpp:106-113 (the time mean summed in time order;
        # Eigen's vectorised colwise mean may round the last bit differently)
        a += offset
        tm = 0.0
        for i in range(a.shape[0]):
            tm += a[i, 0]
        tm /= a.shape[0]
        a = np.log(a / tm)
        a *= scale
    else:
        a *= scale
        a += offset
    minus_log_sigma = -math.log(stdev)
    inv2 = 1.0 / (2.0 * stdev * stdev)
    logp = 0.0
    obs = d["observed"]
    times = d["times"]
    for i in range(len(times)):
        x = a[i].sum()
        if math.isnan(x):
            raise NotImplementedError("missing-simulation penalty")
        for j in range(obs.shape[0]):
            o = obs[j, i]
            if not math.isnan(o):
                if d["error_model"] == "normal":
                    dd = x - o  # EvaluateValue(observed_data, x): d = observed - simulated with the arguments swapped
                    logp += minus_log_sigma - 0.91893853320467274178032973640562 - dd * dd * inv2
                elif d["error_model"] in ("proportional", "additive_proportional"):
                    # DataLikelihoodTimeCourseBase.cpp:280-286 with the swapped arguments: the data
                    # value is "simulated", LogPdfNormal(x, o, sigma) (ProbabilityDistributions.cpp:129-138)
                    ps = _refval(d["proportional_stdev"], tv) if d["proportional_stdev"] else 0.0
                    sigma = ps * max(o, 0.0)
                    if d["error_model"] == "additive_proportional":
                        sigma = stdev + sigma
                    two_sigma_sq = 2.0 * sigma * sigma
                    dd = x - o
                    logp += -math.log(sigma) - 0.91893853320467274178032973640562 - dd * dd / two_sigma_sq
                else:
                    z = (o - x) / stdev
                    logp += -0.9808292530117262 - 2.5 * math.log1p(0.25 * z * z) - math.log(stdev)
    return logp * d["weight"]


def simulate(prob, values, nthreads=1):
    """Every draw's experiments in order; nthreads > 1 runs draws on a thread pool (the per-cell
    CVODE solves run in C without the GIL), one evaluation per thread like the reference's
    sampling threads. Results do not depend on nthreads."""
    values = np.atleast_2d(np.asarray(values, dtype=float))
    if nthreads > 1 and len(values) > 1:
        import concurrent.futures as cf
        with cf.ThreadPoolExecutor(nthreads) as pool:
            parts = list(pool.map(lambda v: simulate(prob, v[None, :]), values))
        return dict(logp=np.concatenate([p["logp"] for p in parts]),
                    population_average=[p["population_average"][0] for p in parts],
                    num_cells=[p["num_cells"][0] for p in parts], detail=[p["detail"][0] for p in parts])
    res = []
    for v in values:
        logp = 0.0
        avgs, ncells = [], []
        for e in prob["experiments"]:
            r = simulate_experiment(e, prob, v)
            logp += r["logp"]
            avgs.append(r.get("population_average", [None])[0])
            ncells.append(len(r["cells"]))
        res.append(dict(logp=logp, avg=avgs[0], ncells=ncells[0], detail=r))
    return dict(logp=np.array([r["logp"] for r in res]), population_average=[r["avg"] for r in res],
                num_cells=[r["ncells"] for r in res], detail=[r["detail"] for r in res])
