"""bench.py's contract without GPUs (CPU): --gpus N asks torch.distributed.run for N ranks only when
N GPUs are visible, and fails loudly otherwise (exit 2, no fallback); the default single-GPU run
fails instead of measuring anything on the CPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=600, cwd=ROOT)


@pytest.fixture(scope="module")
def no_gpu():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")


def test_more_gpus_than_visible_fails_loudly(no_gpu):
    r = _run("--gpus", "2", "--steps", "1", "--warmup", "0")
    assert r.returncode == 2
    assert "--gpus 2 needs 2 GPUs, 0 visible" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line


def test_no_cpu_fallback(no_gpu):
    r = _run("--steps", "1", "--warmup", "0")
    assert r.returncode != 0
    assert r.stdout.strip() == ""
