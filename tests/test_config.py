"""config.txt (bcminf's configuration file) through libbcm3's reader, bcm3_run_config_from_file
(csrc/host/Config.cpp): the reference's own example files (examples/banana/config.txt,
examples/multimodal_circular_ridge/config.txt, copied as data into tests/golden/) and the
boost::program_options rules the reader restates (SamplerPT.cpp:147-171, Sampler.cpp:142-149,
main.cpp:293-343). CPU only: no likelihood is evaluated."""
import os

import pytest

import helpers as H
from bcm3_amd import ptmh


def _write(tmp_path, text, name="config.txt"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_banana_example_config():
    c = ptmh.load_config(os.path.join(H.GOLDEN, "banana_config.txt"))
    p = c["ptmh"]
    # the file's settings
    assert c["num_samples"] == 8000 and p["use_every_nth"] == 5
    assert p["num_chains"] == 6 and p["exploration_steps"] == 1 and p["max_history_size"] == 5000
    assert p["proposal"] == ptmh.PROPOSALS["gaussian_mixture"]
    assert p["swapping_scheme"] == ptmh.SCHEMES["deterministic_even_odd"]
    assert p["adapt_proposal_times"] == 1 and p["adapt_proposal_samples"] == 2000
    assert p["adapt_proposal_max_history_samples"] == 5000
    assert p["temperature_power"] == 3.0 and c["output_proposal_adaptation"] == 1
    assert c["output_folder"] == "output_t6_n5_e1"
    # the registered defaults for everything the file omits (SamplerPT.cpp:149-170, main.cpp:294-307)
    assert p["temperature_max"] == 1.0 and p["exchange_probability"] == 0.5 and p["t_dof"] == 0.0
    assert p["initial_position_tries"] == 100 and p["learning_rate"] == 1.0
    assert c["sampler_type"] == "ptmh" and c["prior"] == "prior.xml" and c["likelihood"] == "likelihood.xml"
    assert c["sampling_threads"] == 0 and c["evaluation_threads"] == 1 and c["likelihood_options"] == ""
    # rngseed = 0 (the default) -> a time-based seed (Sampler.cpp:91-94)
    assert p["seed"] != 0


def test_circular_example_config_fails_like_the_reference():
    # proposal_type=parametric_mixture: SamplerPTChain::CreateProposalInstance logs "Unknown proposal
    # type" and the chain's Initialize fails (SamplerPTChain.cpp:428-444)
    with pytest.raises(RuntimeError, match="Unknown proposal type \"parametric_mixture\""):
        ptmh.load_config(os.path.join(H.GOLDEN, "circular_config.txt"))


def test_defaults_of_an_empty_file(tmp_path):
    c = ptmh.load_config(_write(tmp_path, "# nothing but a comment\n\n"))
    p = c["ptmh"]
    assert c["num_samples"] == 2500 and p["use_every_nth"] == 1 and p["num_chains"] == 6
    assert p["adapt_proposal_samples"] == 2000 and p["adapt_proposal_times"] == 2
    assert p["max_history_size"] == 2000 and p["adapt_proposal_max_history_samples"] == 2000
    assert p["proposal"] == ptmh.PROPOSALS["gaussian_mixture"] and c["output_proposal_adaptation"] == 0
    assert c["output_folder"] == "output"


def test_every_setting(tmp_path):
    text = """prior = p.xml   # trailing comment
likelihood=l.xml
learning_rate=0.25
sampling_threads=3
[sampler]
num_samples=10
use_every_nth=2
rngseed=12345
[ptmhsampler]
num_chains=16
blocking_strategy=one_block
proposal_type=gaussian_mixture_adjustedAIC
proposal_transform_to_unbounded=off
adapt_proposal_samples=40
adapt_proposal_times=3
max_history_size=100
adapt_proposal_max_history_samples=80
stop_proposal_scaling=9
swapping_scheme=stochastic_random
exchange_probability=0.3
num_exploration_steps=2
temperature_schedule_power=2.5
temperature_schedule_max=0.5
output_proposal_adaptation=yes
proposal_t_dof=5
initial_position_tries=7
[pk]
patient=B2
[output]
folder=out
"""
    c = ptmh.load_config(_write(tmp_path, text))
    p = c["ptmh"]
    assert (c["prior"], c["likelihood"], c["output_folder"]) == ("p.xml", "l.xml", "out")
    assert p["learning_rate"] == 0.25 and p["host_threads"] == 3 and c["sampling_threads"] == 3
    assert c["num_samples"] == 10 and p["use_every_nth"] == 2 and p["seed"] == 12345
    assert p["num_chains"] == 16 and p["proposal"] == ptmh.PROPOSALS["gaussian_mixture_adjustedAIC"]
    assert p["adapt_proposal_samples"] == 40 and p["adapt_proposal_times"] == 3
    assert p["max_history_size"] == 100 and p["adapt_proposal_max_history_samples"] == 80
    assert p["swapping_scheme"] == ptmh.SCHEMES["stochastic_random"] and p["exchange_probability"] == 0.3
    assert p["exploration_steps"] == 2 and p["temperature_power"] == 2.5 and p["temperature_max"] == 0.5
    assert c["output_proposal_adaptation"] == 1 and p["t_dof"] == 5.0 and p["initial_position_tries"] == 7
    assert c["likelihood_options"] == "pk.patient=B2"


@pytest.mark.parametrize("text,msg", [
    ("[ptmhsampler]\nnum_chain=6\n", "unrecognised option 'ptmhsampler.num_chain'"),
    ("[sampler]\nnum_samples=5\nnum_samples=6\n", "cannot be specified more than once"),
    ("[sampler]\nnum_samples=many\n", "is invalid"),
    ("[sampler]\nnum_samples=-3\n", "is invalid"),
    ("[ptmhsampler]\noutput_proposal_adaptation=maybe\n", "is invalid"),
    ("[ptmhsampler]\nswapping_scheme=round_robin\n", "Unknown swapping scheme"),
    ("[sampler]\ntype=is\n", "importance sampling"),
    ("[ptmhsampler]\nblocking_strategy=Turek\n", "only one_block"),
    ("[ptmhsampler]\nproposal_type=clustered_covariance\n", "not built here"),
    ("[ptmhsampler]\nproposal_transform_to_unbounded=true\n", "proposal_transform_to_unbounded"),
    ("just some words\n", "invalid syntax"),
])
def test_rejected_files(tmp_path, text, msg):
    with pytest.raises(RuntimeError, match=msg):
        ptmh.load_config(_write(tmp_path, text))


def test_missing_file(tmp_path):
    with pytest.raises(RuntimeError, match="Could not open config file"):
        ptmh.load_config(str(tmp_path / "nope.txt"))
