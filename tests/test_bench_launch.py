"""bench.py --gpus N: how the ranks are launched (CPU, no GPU touched).

The driver runs `python bench.py --gpus N` as well as `torch.distributed.run ... bench.py
--gpus N`; the first form must start N ranks itself (before any GPU call), the second must
agree with --gpus.  SURVEY.md §8e."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_single_rank_runs_in_process():
    assert bench.launch_plan(1, {}, ["--gpus", "1"]) is None
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, []) is None


def test_multi_gpu_launches_n_ranks():
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "1"]
    cmd = bench.launch_plan(8, {}, argv)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    port = [a for a in cmd if a.startswith("--master-port=")]
    assert len(port) == 1 and int(port[0].split("=")[1]) > 0
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == argv


def test_launched_rank_must_match_gpus():
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, []) is None
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 8"):
        bench.launch_plan(8, {"WORLD_SIZE": "2"}, [])
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, [])


def test_backend_label_names_what_ran():
    assert "RCCL" in bench.backend_label(8, "nccl", False)
    lab = bench.backend_label(2, "gloo", True)
    assert "gloo" in lab and "RCCL" not in lab and "same-device" in lab
    assert bench.backend_label(1, "nccl", False).startswith("dp1")


def test_parent_starts_ranks_and_relays_failure():
    """End to end on this GPU-less host: the parent launches 2 ranks through
    torch.distributed.run; each rank sees WORLD_SIZE=2 and stops loudly (no GPU), and the
    parent exits with the launcher's non-zero code."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-extras"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "2 ranks but only 0 visible GPU" in p.stderr + p.stdout


def test_c2_full_parity_reads_and_removes_the_oracle_file(tmp_path):
    """bench.c2_full_parity: per-instance relative errors of every column, counters exactly,
    and the oracle file's directory removed afterwards (CPU tensors stand in for the GPU's)."""
    import numpy as np
    import torch

    from practice_path_planning_for_formula_student_driverless_amd import distributed as D

    B, N, MO = 3, 5, 2
    rng = np.random.default_rng(1)
    orc = {f: rng.normal(size=(B, N)) for f in D.RESULT_F64}
    orc["evals"] = rng.integers(1, 9, size=(B, MO)).astype(np.int32)
    orc["accepts"] = orc["evals"] - 1
    d = tmp_path / "orc"
    d.mkdir()
    path = str(d / "c2_oracle.npz")
    np.savez(path, **orc)
    _, res = D.alloc_result_block(B, N, MO)
    for f in D.RESULT_F64:
        res[f].copy_(torch.from_numpy(orc[f]))
    res["evals"].copy_(torch.from_numpy(orc["evals"]))
    res["kappa"][1, 2] += 1e-6 * float(np.max(np.abs(orc["kappa"][1])))
    out = bench.c2_full_parity(res, path)
    assert out["instances"] == B and out["evals_equal"] and out["instances_within_tolerance"]
    assert 0 < out["kappa_max_rel"] <= 1.1e-6 and out["x_max_rel"] == 0.0
    assert not d.exists()
