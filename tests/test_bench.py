"""bench.py's multi-rank contract: --gpus N starts N ranks (or, under an external
torch.distributed.run, checks WORLD_SIZE), refuses a run it cannot honour, and the ranks
the communicator saw are reported in the line."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, env=e,
                          timeout=timeout, cwd=ROOT)


def test_world_size_mismatch_refused():
    r = run(["--gpus", "2"], env={"WORLD_SIZE": "4"}, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_too_few_gpus_refused():
    """RCCL needs one GPU per rank: asking for more than are visible fails before any rank
    starts (on this CPU container none are)."""
    import torch
    n = torch.cuda.device_count() + 1
    r = run(["--gpus", str(n)], timeout=120)
    assert r.returncode != 0
    assert "GPUs" in r.stderr


@pytest.mark.gpu
def test_two_ranks_host_transport_match_one():
    """Two ranks on one GPU through the library's host transport (gloo): the launcher starts
    them, the communicator reports 2, and the Newton step's residuals equal one rank's."""
    common = ["--config", "global4", "--state", "synthetic", "--steps", "1", "--warmup", "0",
              "--no-cpu", "--newton-seq", "0"]
    r1 = run(["--gpus", "1", *common], timeout=300)
    assert r1.returncode == 0, r1.stderr[-2000:]
    one = json.loads(r1.stdout.strip().splitlines()[-1])
    r2 = run(["--gpus", "2", "--transport", "host", *common], timeout=300)
    assert r2.returncode == 0, r2.stderr[-2000:]
    two = json.loads([ln for ln in r2.stdout.splitlines() if ln.startswith("{")][-1])
    assert two["n_gpus"] == 2 and two["ranks_seen"] == 2
    assert two["config"]["transport"] == "host"
    assert two["comm"]["per_fgmres_step"]["batches"] > 0
    f0, f1 = one["newton"]["norm_f0"], one["newton"]["norm_f1"]
    assert abs(two["newton"]["norm_f0"] - f0) <= 1e-12 * f0
    # both solves reach the tolerance; the decompositions' preconditioners differ, so the
    # updates agree to the solve tolerance, amplified by the (diverging, far from a
    # solution) step's nonlinearity in ||F1||
    assert one["newton"]["converged"] and two["newton"]["converged"]
    assert two["newton"]["explicit_rel_res"] <= 2e-8
    assert abs(two["newton"]["norm_f1"] - f1) <= 1e-6 * f1 + 1e-8 * f0
