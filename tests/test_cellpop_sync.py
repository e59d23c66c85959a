"""CPU tests of synchronised cell-population data (time courses / time points with
synchronize="...", the experiment's synchronization_time_offset): the oracle's stored-integration-
point mode and the product's loader and kernel build.

Reference: Experiment.cpp:95-121 (AddSimulationTimepoints), 172-185 (the offset), 265-292 (the
evaluation passes); Cell.cpp:152, 232-252 (SolveStoreIntegrationPoints), 280-327
(GetInterpolatedSpeciesValue), 463-538 (events, division on the interpolant); ODESolverCVODE.cpp:
176-242 (the interpolation iterator), 264-320 (threshold crossings), 375-401 (the records);
DataLikelihoodTimeCourse.cpp:27-41, 190-199; DataLikelihoodTimePoints.cpp:29-43, 186-197.
Parity of the synchronised values is pinned by the reference's own CVODE (oracle/_ref/
libcellpopref*.so run in the stored mode by oracle/cellpop_ref.cpp), not by a reference fixture:
the reference ships none for this path."""
import ctypes
import math
import os

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP

SYNC_DATA = os.path.join(CH.GOLDEN, "cellpop_sync_data.json")
POP = '<data type="time_course_population_average" data_name="pcna_mean" species_name="PCNA_gfp" stdev="stdev"/>'


def _tc(sync, data_name="pcna_sync"):
    return f'<data data_name="{data_name}" species_name="PCNA_gfp" stdev="stdev" synchronize="{sync}"/>'


def _tp(sync, data_name="pcna_sync"):
    return f'<data type="time_points" data_name="{data_name}" species_name="PCNA_gfp" stdev="stdev" synchronize="{sync}"/>'


# name -> (data elements, likelihood kwargs, cellpop.use_only_cell_ix)
CASES = {
    # population average (unsynchronised, read through the stored points too) + a course aligned at
    # the start of DNA replication
    "replication": (POP + _tc("DNA_replication_start"), dict(experiment_attrs=' divide_cells="false"'), None),
    # the offset as a sampled variable (k_D's value, hours)
    "pcna_offset": (_tc("PCNA_gfp_increase"),
                    dict(experiment_attrs=' divide_cells="false" synchronization_time_offset="k_D"'), None),
    # time points aligned at replication start, simulated 10 h past the last time point
    "time_points": (_tp("DNA_replication_start"), dict(experiment_attrs=' divide_cells="false" trailing_simulation_time="10"'),
                    None),
    # dividing cells in the stored mode: division times and daughters' states on the interpolant
    "division": (_tp("anaphase", "pcna_neg"), dict(num_cells=4, max_cells=32, experiment_attrs=' trailing_simulation_time="8"'),
                 "2,7,11"),
    # a treatment trajectory in the stored mode: the records of the stop-time returns and restarts
    "treatment": (POP + _tc("DNA_replication_start"),
                  dict(experiment_attrs=' divide_cells="false"',
                       extra='\n    <treatment_trajectory type="pulses" species_name="mitogen" times="13,-1"/>'), None),
    # a population average next to synchronised time points with a sampled offset and dividing cells:
    # the population is counted at data time + offset (Experiment.cpp:285, 301), where the values are read
    "pop_offset": (POP + _tp("anaphase", "pcna_neg"),
                   dict(num_cells=4, max_cells=32,
                        experiment_attrs=' trailing_simulation_time="8" synchronization_time_offset="k_D"'), "2,7,11"),
    # two synchronisation points and an unsynchronised course in one experiment (three passes)
    "mixed": (POP + _tc("PCNA_gfp_increase") + _tc("mitosis").replace('stdev="stdev"', 'stdev="0.2" error_model="t4"'),
              dict(experiment_attrs=' divide_cells="false"'), None),
}


def sync_likelihood(directory, name):
    import make_cellpop_fixtures as F
    data_xml, kw, _ = CASES[name]
    kw = dict(kw)
    kw.setdefault("num_cells", 16)
    kw.setdefault("max_cells", 16)
    path = os.path.join(str(directory), f"sync_{name}.xml")
    with open(path, "w") as f:
        f.write(F.likelihood_text(data_file=SYNC_DATA, model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"),
                                  data_xml=data_xml, **kw))
    return path


def only(name):
    return CASES[name][2] or "-1"


def test_stored_mode_and_full_duration_entry(tmp_path):
    """any synchronised entry turns the stored mode on; a course with negative time points adds its
    full duration (last - first) as an entry without species, sorted with the others"""
    e = CP.load_problem(sync_likelihood(tmp_path, "replication"), CH.PRIOR)["experiments"][0]
    assert e["stored"]
    tps, sync = e["timepoints"], e["timepoint_sync"]
    assert [t[1] for t in tps] == sorted(t[1] for t in tps)
    full = [(t, s) for t, s in zip(tps, sync) if t[3] < 0]
    assert full == [((1, 10.0, -1, -1), 0)]  # 4 - (-6), synchronised like its course
    assert sum(1 for s in sync if s == CP.SYNC_NONE) == 21  # the population average's 0..20 h
    plain = CP.load_problem(os.path.join(CH.GOLDEN, "cellpop_likelihood.xml"), CH.PRIOR)["experiments"][0]
    assert not plain["stored"]


def test_offset_number_replaces_a_constant_entry_time(tmp_path):
    """Experiment.cpp:172-181: a numeric synchronization_time_offset is written to fixed_entry_time"""
    import make_cellpop_fixtures as F
    path = os.path.join(str(tmp_path), "num.xml")
    with open(path, "w") as f:
        f.write(F.likelihood_text(num_cells=16, max_cells=16, data_file=SYNC_DATA,
                                  model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"), data_xml=_tc("mitosis"),
                                  experiment_attrs=' divide_cells="false" synchronization_time_offset="2.5"'))
    e = CP.load_problem(path, CH.PRIOR)["experiments"][0]
    assert e["entry_time"] == ("fixed", 2.5) and e["sync_offset"] == ("fixed", 0.0)
    e = CP.load_problem(sync_likelihood(tmp_path, "pcna_offset"), CH.PRIOR)["experiments"][0]
    assert e["sync_offset"] == ("var", 0)


@pytest.fixture(scope="module")
def replication(tmp_path_factory):
    d = tmp_path_factory.mktemp("sync")
    return CP.load_problem(sync_likelihood(d, "replication"), CH.PRIOR)


def test_event_times_are_bisections_of_the_interpolant(replication):
    """stored mode: the replication-start time is a real crossing inside the step that found it (the
    non-stored mode only walks to one end of the step), and the synchronised values follow it"""
    r = CP.simulate(replication, CH.draws(1, 3))
    cells = r["detail"][0]["cells"]
    e = replication["experiments"][0]
    ks = [k for k, s in enumerate(e["timepoint_sync"]) if s == 0 and e["timepoints"][k][3] >= 0]
    for c in cells:
        t_rep = c["events"][0]
        assert 0.0 < t_rep < c["sim_end"]
        for k in ks:
            ct = e["timepoints"][k][1] + t_rep
            assert math.isnan(c["values"][k]) == (not (0.0 <= ct <= c["sim_end"]))
    # the same cells without synchronised data: the replication time is the crossing's other end
    plain = CP.load_problem(os.path.join(CH.GOLDEN, "cellpop_likelihood.xml"), CH.PRIOR, num_cells=16, max_cells=16)
    rp = CP.simulate(plain, CH.draws(1, 3))
    assert rp["detail"][0]["cells"][0]["events"][0] != cells[0]["events"][0]


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_builds_agree(tmp_path, name):
    """the reference built with and without FMA contraction: the stored mode's own spread stays
    within 1e-5 (1 + |logp|) (measured: up to 2.1e-6, pop_offset draw 0; the GPU tests allow 10x the
    spread per draw, cellpop_helpers.logp_bar) and the -inf pattern is the same"""
    path = sync_likelihood(tmp_path, name)
    x = CH.draws(3, 5)
    a = CP.simulate(CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only(name)), x)["logp"]
    b = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma", use_only_cell_ix=only(name)), x)["logp"]
    assert ((a == -math.inf) == (b == -math.inf)).all()
    fin = np.isfinite(a)
    assert fin.any(), name
    assert (np.abs(a[fin] - b[fin]) <= 1e-5 * (1 + np.abs(a[fin]))).all()


@pytest.mark.parametrize("name", list(CASES))
def test_loader_builds_the_stored_kernel(tmp_path, name):
    """the product loads every case and compiles its stored-integration-point cell kernel (hipRTC,
    no device needed; the code object lands in the cache the GPU runs load)"""
    from bcm3_amd import likelihood
    opts = "backend=none" + (f";cellpop.use_only_cell_ix={CASES[name][2]}" if CASES[name][2] else "")
    ll = likelihood.Likelihood(sync_likelihood(tmp_path, name), CH.PRIOR, options=opts)
    L = likelihood.lib()
    L.bcm3_likelihood_cellpop_precompile.argtypes = [ctypes.c_void_p]
    assert L.bcm3_likelihood_cellpop_precompile(ll.h) == 0
    ll.close()


def test_loader_refuses_unknown_synchronisation(tmp_path):
    from bcm3_amd import likelihood
    import make_cellpop_fixtures as F
    for data_xml, attrs in ((_tc("bogus"), ' divide_cells="false"'),
                            (_tc("mitosis"), ' divide_cells="false" synchronization_time_offset="no_such_variable"'),
                            # a sampled offset without synchronised data (the reference's exact-time lookups
                            # at data time + offset miss, Cell.cpp:328-335)
                            (POP, ' divide_cells="false" synchronization_time_offset="k_D"')):
        path = os.path.join(str(tmp_path), "bad.xml")
        with open(path, "w") as f:
            f.write(F.likelihood_text(num_cells=16, max_cells=16, data_file=SYNC_DATA,
                                      model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"), data_xml=data_xml,
                                      experiment_attrs=attrs))
        with pytest.raises(RuntimeError):
            likelihood.Likelihood(path, CH.PRIOR, options="backend=none")


def test_unsynchronised_kernel_still_builds():
    """the stored mode is compiled out of the plain kernel (CP_STORED 0), which must still build"""
    from bcm3_amd import likelihood
    ll = likelihood.Likelihood(os.path.join(CH.GOLDEN, "cellpop_likelihood.xml"), CH.PRIOR, options="backend=none")
    L = likelihood.lib()
    L.bcm3_likelihood_cellpop_precompile.argtypes = [ctypes.c_void_p]
    assert L.bcm3_likelihood_cellpop_precompile(ll.h) == 0
    ll.close()
