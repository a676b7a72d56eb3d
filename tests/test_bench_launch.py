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
