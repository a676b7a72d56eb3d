#!/usr/bin/env python3
"""Benchmark: PGD outer-iterations/s of the batched raceline optimizer on MI355X.

Workload (BASELINE.json configs[1] = SURVEY.md §8d C2): competition_map1 closed,
N=2000 resample, B=1024 α-seeds per GPU, min-curvature optimiser, default cfg
(14 outer iterations).  One *step* = one launch optimising the whole batch from
inputs already resident in HBM; for N>1 the step also gathers per-instance
summaries to rank 0 with RCCL over xGMI (the only collective).  Weak scaling:
every rank optimises its own 1024 seeds.

value = (instances x 14 outer iterations, all ranks) / (max over ranks of the
timed K steps).  Also reported (rank 0): C3/C4/C5, the PCIe-inclusive C2 rate,
the drop-in B=1 latency per bundled track next to the reference's own CPU time,
lap-time Δ statistics over instances against the CPU oracle, and the CPU
baseline (the reference compiled from its sources, oracle/_ref, on one pinned
core; the C restatement beside it).  The CPU work runs in a child process
started before any GPU call (`--cpu-leg`), pinned away from the GPU host thread.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu] [--no-extras]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

# HIP hardware queues of this process: the operator's setting is kept (the GPU box exports
# HIP's default, 4); only when nothing is set does the bench ask for 16.  The value is
# recorded in the JSON line (`hip_hw_queues`): the C4 line's concurrent plans are scheduled
# onto that many streams (run_c4).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from practice_path_planning_for_formula_student_driverless_amd import abi, raceline  # noqa: E402
from practice_path_planning_for_formula_student_driverless_amd import distributed as D  # noqa: E402

# MI355X fp64 vector peak (AMD spec, FMA counted as 2 flops; equal to the fp64 dense
# matrix peak).  The path is fp64 VALU arithmetic; most of its operations are plain
# add/mul (-ffp-contract=off keeps the reference's roundings), for which the same pipe
# peaks at half that rate.
FP64_PEAK_TFLOPS = 78.6
FP64_NONFMA_TFLOPS = 39.3
HBM_PEAK_GBS = 8000.0
PKG = os.path.join(REPO, "practice_path_planning_for_formula_student_driverless_amd")
C4_ITEMS = 7 * 512
C3_BATCH = 4096
C3_SAMPLE = 128            # C3 instances whose laps the CPU oracle recomputes (strided over the batch)
C2_BATCH = 1024            # C2 instances per GPU (the default --batch); all of rank 0's are checked
DROPIN_CASES = ["track_" + t for t in D.C4_TRACKS] + ["cmap1_n2000"]


def source_sha() -> str:
    """Hash of the kernel sources: a PMC summary is used only if measured on this code."""
    h = hashlib.sha256()
    # (build.py too: its per-source compiler flags change the code)
    files = sorted(glob.glob(os.path.join(PKG, "csrc", "*"))) + [os.path.join(REPO, "include", "rl_abi.h"),
                                                                 os.path.join(PKG, "build.py")]
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def read_pmc(tag: str):
    """The committed rocprofv3 PMC summary for `tag` (profiles/pmc_traffic.json, written by
    scripts/pmc_summary.py --commit), or None when it was measured on other kernel sources."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p)).get(tag)
    except Exception:
        return None
    if not d or d.get("source_sha") != source_sha():
        return None
    return d


def load_problem(name: str):
    import oracle_lib as O   # fixture loader (npz, no pickle); the oracle itself is not touched here

    case = O.load_case(name)
    return case, O.case_problem(case), O.case_cfg(case)


def flops_per_outer(N: int, E_k: float, Eseg: int, mintime: bool = False) -> float:
    """Algorithmic fp64 flops per outer iteration, SURVEY.md §8d's per-unit figure:
    34 (min-curv) / 36 (min-time) per sample per evaluation, plus the reference's
    2·(Ei+Eo) ray tests per sample at 12 flops + 1 reciprocal each (the kernel culls
    most ray tests exactly, so it executes fewer: see executed_fp64_TFLOPs_pmc)."""
    per_eval = 36.0 if mintime else 34.0
    return N * (per_eval * E_k + 2 * Eseg * 13)


def bytes_per_outer(N: int, E_k: float, Eseg: int) -> float:
    """SURVEY.md §8d streaming model (8-B words, each array once per evaluation pass)."""
    return N * (80 * E_k + 224) + 32 * Eseg


# ============================================================ CPU leg (child process)
def _cpu_info() -> dict:
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}


def _ref_bench_available() -> bool:
    """oracle/_ref/ref_bench_o3: the reference's own main.cpp built from its sources with
    its README's flags (oracle/Makefile `ref`, built in the build container)."""
    import oracle_lib as O

    return os.path.exists(O.REF_BENCH)


def _lap_worker(job):
    """Pool worker (CPU only): min-time laps of (case, cfg dict, seed) jobs with the C oracle."""
    import oracle_lib as O

    out = []
    cache = {}
    for name, cfgd, seed in job:
        if name not in cache:
            cache[name] = O.case_problem(O.load_case(name))
        c = abi.RlCfg.from_dict(cfgd)
        _, mt = O.run_oracle(cache[name], [c], seeds=[seed], B=1, modes=(False, True))
        out.append(float(mt.lap[0]))
    return out


def _c2_worker(seeds):
    """Pool worker (CPU only): C2's min-curvature results for a list of seeds with the C
    oracle (every column and counter; the full-size parity check of the headline batch)."""
    import oracle_lib as O

    _, prob, cfg = load_problem("cmap1_n2000")
    if not seeds:
        return None
    mc, _ = O.run_oracle(prob, cfg, seeds=list(seeds), B=len(seeds), modes=(True, False))
    return {f: getattr(mc, f) for f in C2_PARITY_COLS}


C2_PARITY_COLS = ("x", "y", "heading", "kappa", "alpha_total", "alpha_last", "evals", "accepts")
ALLCORE_CORES = 16      # the host CPU share of one GPU on the box (its operator's worker-pool size)


def reference_multicore(prob, cfg, cores, work: str, MO: int, budget_s: float = 6.0) -> dict:
    """The reference's compute_min_curvature_raceline on C2's problem, one independent
    instance stream per core (the instance-parallel CPU form of the batch), `len(cores)`
    processes pinned one per core, run together for ~budget_s.  Context, not the target."""
    import oracle_lib as O

    path = os.path.join(work, "problem_mc.bin")
    O.write_problem_bin(prob, cfg, path)
    procs = []
    for c in cores:
        procs.append(subprocess.Popen([O.REF_BENCH, path, "mincurv", str(budget_s), "2"], stdout=subprocess.PIPE,
                                      text=True, preexec_fn=(lambda c=c: os.sched_setaffinity(0, {c}))))
    rates, calls = [], 0
    for p in procs:
        out, _ = p.communicate(timeout=600)
        r = json.loads(out.strip().splitlines()[-1])
        calls += int(r["calls"])
        rates.append(int(r["calls"]) * MO / float(r["seconds"]))
    return {"value": round(sum(rates), 1), "unit": "PGD outer-iters/s", "cores": len(cores), "kind": "reference",
            "per_core_min": round(min(rates), 1), "per_core_max": round(max(rates), 1), "calls": calls,
            "note": f"context only: {len(cores)} concurrent ref_bench_o3 processes, one pinned per core (this GPU's "
                    f"host CPU share on the box), each ~{budget_s:.0f} s of C2 calls; the reference itself is "
                    f"single-threaded"}


def cpu_multicore_leg() -> dict:
    """Context only (SURVEY §8d optional): the reference instance-parallel on
    this GPU's host CPU share -- one ref_bench process per core, each pinned, on C2's
    problem.  Run by the CPU-leg child only when the parent says so, after every GPU leg
    (it saturates 16 cores, which must not overlap any rank's GPU timing)."""
    import tempfile

    cores = sorted(os.sched_getaffinity(0))
    if not _ref_bench_available() or len(cores) <= 3:
        return {}
    case, prob, cfg = load_problem("cmap1_n2000")
    work = tempfile.mkdtemp(prefix="rl_cpu_mc_")
    try:
        return {"reference_multicore": reference_multicore(prob, cfg, cores[2:2 + ALLCORE_CORES], work,
                                                           int(cfg.max_outer_iters))}
    finally:
        import shutil

        shutil.rmtree(work, ignore_errors=True)


def cpu_leg(budget_s: float) -> dict:
    """Everything the bench needs from the CPU, computed without touching the GPU:
    the baseline on one pinned core, the reference's per-track drop-in times, and the
    oracle laps the GPU laps are compared with (process pool on the other cores)."""
    import multiprocessing as mp

    import oracle_lib as O

    import tempfile

    cores = sorted(os.sched_getaffinity(0))
    os.sched_setaffinity(0, {cores[0]})
    info = _cpu_info()
    res = {"cpu": info}
    case, prob, cfg = load_problem("cmap1_n2000")
    MO = int(cfg.max_outer_iters)
    have_ref = _ref_bench_available()
    work = tempfile.mkdtemp(prefix="rl_cpu_leg_")
    # ---- baseline: C2 min-curvature at N=2000 on one core, the reference as its README builds it
    if have_ref:
        r = O.run_ref_bench(prob, cfg, False, budget_s, 3, work)
        n, dt = int(r["calls"]), float(r["seconds"])
        c3case, p3, cfg3 = load_problem("cmap1_n2000_vp20")
        rt = O.run_ref_bench(p3, cfg3, True, budget_s / 3, 2, work)
        res["reference"] = {"value": n * MO / dt, "unit": "PGD outer-iters/s", "cores": 1, "kind": "reference",
                            "build": O.ref_bench_build(),
                            "sample": f"{n} calls of the reference's compute_min_curvature_raceline (main.cpp:683-764; "
                                      f"oracle/_ref/ref_bench_o3 = /root/reference/src/main.cpp built with its README's "
                                      f"g++ -std=c++17 -O3) on C2's problem (competition_map1, N={prob.N}, alpha=0 "
                                      f"start), {MO} outer each, {dt:.1f} s, one thread pinned to core {cores[0]}",
                            "ms_per_call_median": float(np.median(r["ms"])),
                            "x0_equals_reference_fixture": r["x0"] == float(case["mc_x"][0]),
                            "mintime_c3_problem": {
                                "value": int(rt["calls"]) * int(cfg3.max_outer_iters) / float(rt["seconds"]),
                                "unit": "PGD outer-iters/s", "calls": int(rt["calls"]),
                                "ms_per_call_median": float(np.median(rt["ms"])),
                                "lap_equals_reference_fixture": rt["lap"] == float(c3case["mt_lap"]),
                                "sample": "compute_min_time_raceline (main.cpp:905-1052) on C3's problem "
                                          "(competition_map1, N=2000, max_vpass_iters=20), same build and core"}}
    n, t0 = 0, time.perf_counter()
    seeds = np.arange(256, dtype=np.uint64)
    while n < len(seeds) and (n == 0 or time.perf_counter() - t0 < budget_s / 2):
        O.run_oracle(prob, cfg, seeds=seeds, B=len(seeds), modes=(True, False), b_range=(n, n + 1))
        n += 1
    dt = time.perf_counter() - t0
    res["port"] = {"value": n * MO / dt, "unit": "PGD outer-iters/s", "cores": 1, "kind": "port",
                   "sample": f"{n} C2 instances (seeds 0..{n - 1}) through the C restatement of main.cpp:683-1052 "
                             f"(oracle/raceline_oracle.c), {dt:.1f} s, one thread pinned to core {cores[0]}"}
    # ---- the drop-in use (one instance per call, ref:1347 / 1397): the reference per track
    # (median of 3 calls, same build and core)
    if have_ref:
        per = {}
        for name in DROPIN_CASES:
            _, p, c = load_problem(name)
            ts = [float(np.median(O.run_ref_bench(p, c, mt, 0.0, 3, work)["ms"])) for mt in (False, True)]
            per[name] = {"N": p.N, "mincurv_ms": round(ts[0], 2), "mintime_ms": round(ts[1], 2)}
        res["reference_per_track"] = per
    # ---- oracle laps for the lap-Δ statistics (C3 sample, the whole C4 grid)
    c3case, _, cfg3 = load_problem("cmap1_n2000_vp20")
    c3_seeds = list(range(0, C3_BATCH, C3_BATCH // C3_SAMPLE))
    jobs = [("cmap1_n2000_vp20", cfg3.to_dict(), s) for s in c3_seeds]
    base = O.case_cfg(O.load_case("track_training_map"))
    cfgs = D.c4_cfgs(base)
    c4_jobs = [("track_" + D.C4_TRACKS[t], cfgs[k].to_dict(), 0) for t, k in D.c4_items()]
    workers = max(1, min(15, len(cores) - 2))
    pool_cores = set(cores[2:2 + workers]) or {cores[-1]}
    os.sched_setaffinity(0, pool_cores)
    t0 = time.perf_counter()
    chunks = lambda js, n: [js[i::n] for i in range(n)]   # noqa: E731
    with mp.get_context("spawn").Pool(workers) as pool:
        r3 = pool.map(_lap_worker, chunks(jobs, workers))
        r4 = pool.map(_lap_worker, chunks(c4_jobs, workers))
        # the whole C2 batch of rank 0 (seeds 0..B-1) through the oracle, for the bench's
        # full-size parity check; saved for the parent (our own file, no pickle in it)
        nb = C2_BATCH
        parts = [p for p in pool.map(_c2_worker, [list(range(nb))[i::workers] for i in range(workers)]) if p]
        full = {f: np.empty((nb,) + parts[0][f].shape[1:], dtype=parts[0][f].dtype) for f in C2_PARITY_COLS}
        for i, p in enumerate(parts):
            for f in C2_PARITY_COLS:
                full[f][i::workers] = p[f]
        npz_dir = tempfile.mkdtemp(prefix="rl_c2_oracle_")
        res["c2_oracle_npz"] = os.path.join(npz_dir, "c2_oracle.npz")
        np.savez(res["c2_oracle_npz"], **full)
    unchunk = lambda rs, n, total: [rs[i % n][i // n] for i in range(total)]   # noqa: E731
    res["c3_oracle_laps"] = {"seeds": c3_seeds, "laps": unchunk(r3, workers, len(jobs))}
    res["c4_oracle_laps"] = unchunk(r4, workers, len(c4_jobs))
    res["oracle_pool"] = {"workers": workers, "seconds": round(time.perf_counter() - t0, 1)}
    # ---- open-mode line: the first seeds through the oracle
    oprob, ocfg = open_problem()
    omc, omt = O.run_oracle(oprob, ocfg, seeds=list(range(OPEN_CHECK)), B=OPEN_CHECK)
    res["open_oracle"] = {"x": omc.x.tolist(), "evals": omc.evals.tolist(), "lap": omt.lap.tolist(),
                          "mt_evals": omt.evals.tolist()}
    import shutil

    shutil.rmtree(work, ignore_errors=True)
    return res


def open_problem():
    """C2's track as an open path (is_closed_track = false: DiffOpsOpen ref:560-579, open
    normals/heading ref:581-620): the open-mode throughput line."""
    case, prob, cfg = load_problem("cmap1_n2000")
    return abi.Problem(center=prob.center, L=prob.L, inner_seg=raceline.edges_for(case["inner_ring"], False),
                       outer_seg=raceline.edges_for(case["outer_ring"], False),
                       veh_width=prob.veh_width, closed=False), cfg


def run_open(local, B: int = 1024):
    """Open-mode throughput: C2's problem with closed = false, B seeds, both optimisers."""
    prob, cfg = open_problem()
    MO = int(cfg.max_outer_iters)
    plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B,
                         modes=abi.RL_MODE_MINCURV | abi.RL_MODE_MINTIME, device=local)
    plan.run()
    ms = {1: [], 2: []}
    for _ in range(3):
        plan.run()
        for i in (1, 2):
            ms[i].append(plan.kernel_ms(i))
    mc, mt = plan.fetch()
    plan.close()
    k1, k2 = float(np.median(ms[1])), float(np.median(ms[2]))
    res = {"N": prob.N, "instances": B, "kernel_ms_mincurv": round(k1, 3), "kernel_ms_mintime": round(k2, 3),
           "outer_iters_per_s_mincurv": round(B * MO / (k1 * 1e-3), 1),
           "outer_iters_per_s_mintime": round(B * MO / (k2 * 1e-3), 1),
           "kernels": "rl_optimize_kernel<8,256,open,mincurv> / <8,256,open,mintime>"}
    gpu = {"x": mc.x[:OPEN_CHECK].tolist(), "evals": mc.evals[:OPEN_CHECK].tolist(),
           "lap": mt.lap[:OPEN_CHECK].tolist(), "mt_evals": mt.evals[:OPEN_CHECK].tolist()}
    return res, gpu


OPEN_CHECK = 8     # seeds of the open-mode line checked against the oracle (CPU leg)
HOST_CORES: set = set()   # the process's host cores at start (before the CPU leg pins it)


def start_cpu_leg(budget_s: float):
    """The CPU leg as a child process (before the parent touches the GPU).  The parent
    then keeps to the cores the child does not use first."""
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-leg", "--cpu-budget", str(budget_s)]
    proc = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    cores = sorted(os.sched_getaffinity(0))
    if len(cores) > 1:
        os.sched_setaffinity(0, {cores[1]})
    return proc


def read_cpu_leg(proc):
    """The CPU leg's first line (baseline, laps, per-track reference times); None if the
    child failed.  The child then waits for finish_cpu_leg."""
    line = proc.stdout.readline()
    if not line.strip():
        finish_cpu_leg(proc, False)
        return None
    return json.loads(line)


def finish_cpu_leg(proc, multicore: bool):
    """Tell the waiting child whether to run the multicore context leg (after every GPU
    leg), and return its result ({} when skipped or failed)."""
    try:
        out, err = proc.communicate(input="go\n" if multicore else "stop\n", timeout=900)
    except (BrokenPipeError, OSError):
        out, err = proc.communicate(timeout=900)
    if proc.returncode != 0:
        sys.stderr.write(err[-4000:])
        return {}
    lines = out.strip().splitlines()
    return json.loads(lines[-1]) if lines else {}


def c2_full_parity(res, npz_path) -> dict:
    """Every column and counter of rank 0's timed C2 batch against the CPU oracle on the same
    seeds (1e-4 x column max per instance; counters exactly).  Deletes the oracle file."""
    import shutil

    try:
        orc = np.load(npz_path)
        out = {"instances": int(orc["x"].shape[0]), "tolerance": "1e-4 x column max (+1e-9) per instance"}
        worst = 0.0
        for f in ("x", "y", "heading", "kappa", "alpha_total", "alpha_last"):
            g = res[f].cpu().numpy() if f in res else None
            if g is None:
                continue
            o = orc[f]
            rel = np.max(np.abs(g - o), axis=1) / (np.max(np.abs(o), axis=1) + 1e-300)
            out[f + "_max_rel"] = float(rel.max())
            worst = max(worst, float(rel.max()))
        ev = res["evals"].cpu().numpy()
        out["evals_equal"] = bool(np.array_equal(ev, orc["evals"]))
        out["instances_within_tolerance"] = worst <= 1e-4
        return out
    finally:
        shutil.rmtree(os.path.dirname(npz_path), ignore_errors=True)


def lap_delta(gpu, oracle) -> dict:
    d = np.abs(np.asarray(gpu, dtype=np.float64) - np.asarray(oracle, dtype=np.float64))
    rel = d / np.abs(np.asarray(oracle, dtype=np.float64))
    return {"n": int(d.size), "max_abs_s": float(d.max()), "mean_abs_s": float(d.mean()),
            "max_rel": float(rel.max()), "tolerance_rel": 1e-4}


# ============================================================== GPU legs
def run_c3(rank, local, stream, reps: int = 3):
    """C3: N=2000, max_vpass_iters=20, 4096 seeds per GPU, min-curv + min-time."""
    c3, p3, cfg3 = load_problem("cmap1_n2000_vp20")
    MO = int(cfg3.max_outer_iters)
    pl3 = raceline.Plan(p3, cfg3, seeds=np.arange(rank * C3_BATCH, (rank + 1) * C3_BATCH, dtype=np.uint64),
                        B=C3_BATCH, modes=abi.RL_MODE_MINCURV | abi.RL_MODE_MINTIME, device=local)
    pl3.run(stream.cuda_stream)
    stream.synchronize()
    walls, kmc, kmt = [], [], []
    for _ in range(reps):
        t1 = time.perf_counter()
        pl3.run(stream.cuda_stream)          # inputs resident; results stay in HBM (fetched below)
        stream.synchronize()
        walls.append(time.perf_counter() - t1)
        kmc.append(pl3.kernel_ms(1))
        kmt.append(pl3.kernel_ms(2))
    mc3, mt3 = pl3.fetch()
    pl3.close()
    t3 = float(np.mean(walls))
    return {"instances": C3_BATCH, "reps": reps, "wall_ms_mean": round(t3 * 1e3, 2),
            "wall_ms_min": round(min(walls) * 1e3, 2), "outer_iters_per_s": round(2 * C3_BATCH * MO / t3, 1),
            "kernel_ms_mincurv": round(float(np.mean(kmc)), 3), "kernel_ms_mintime": round(float(np.mean(kmt)), 3),
            "lap_seed0_s": float(mt3.lap[0]), "lap_ref_s": float(c3["mt_lap"]),
            "lap_seed0_delta_vs_reference_s": float(abs(mt3.lap[0] - float(c3["mt_lap"]))),
            "lap_mean_over_seeds_s": float(np.mean(mt3.lap)),
            "vpass_sweeps_mean": float(np.mean(mt3.vpass_sweeps))}, mt3.lap


def run_c4(world, rank, local, dev, dist):
    """C4: 7 bundled tracks x 512 (mu, P_max_W, lambda_smooth) points, min-curv + min-time.
    Items are sharded track-major over ranks; one plan per (track, mode), all run by one
    rl_plan_run_group: per mode one launch per K of one-wave plans, the launches concurrent;
    laps gathered to rank 0 in item order.  (scripts/c4_group.py at the box's 4 hardware
    queues: 13.3 ms grouped against 16.4 ms with every plan on its own stream, bit-exact;
    profiles/r06/c4_group.log.)"""
    import torch

    groups = D.c4_shard(world, rank)
    base = load_problem("track_training_map")[2]
    cfgs = D.c4_cfgs(base)
    plans, mt_plans, meta = [], [], []
    # instances of all concurrent plans: both modes of every group run at once
    n_flight = 2 * sum(len(ks) for ks in groups.values())
    shapes = {}
    for t, ks in groups.items():
        case, prob, _ = load_problem("track_" + D.C4_TRACKS[t])
        for mode in (abi.RL_MODE_MINCURV, abi.RL_MODE_MINTIME):
            pl = raceline.Plan(prob, [cfgs[k] for k in ks], B=len(ks), modes=mode, device=local)
            # the plans run concurrently: every one takes the shape of the whole rank's load
            # (ADVICE r4), not a latency shape meant to spread its own few instances over the GPU
            pl.set_shape_batch(n_flight)
            shapes.setdefault(D.C4_TRACKS[t], {})["mincurv" if mode == abi.RL_MODE_MINCURV else "mintime"] = \
                "x".join(map(str, pl.shape(mode)))
            plans.append(pl)
            if mode == abi.RL_MODE_MINTIME:
                mt_plans.append(pl)
        meta.append((t, ks, prob))
    stream = torch.cuda.Stream(device=dev)
    launches = set()        # the group launches: one per (mode, K) of one-wave plans
    for pl in plans:
        m = abi.RL_MODE_MINCURV if pl.modes & abi.RL_MODE_MINCURV else abi.RL_MODE_MINTIME
        launches.add((m, *pl.shape(m)))

    def launch():
        raceline.Plan.run_group(plans, stream.cuda_stream)
        stream.synchronize()

    launch()
    if dist is not None:
        dist.barrier()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        launch()
    dt = (time.perf_counter() - t0) / reps
    n_inst = sum(len(ks) for _, ks, _ in meta)
    laps = np.concatenate([pl.fetch()[1].lap for pl in mt_plans])
    for pl in plans:
        pl.close()
    if dist is not None:
        allst = D.gather_stats([dt, float(n_inst)], world, rank, device=dev)
        laps = D.gather_ragged(laps, world, rank, C4_ITEMS, device=dev)
        if rank != 0:
            return None, None
        dt, n_inst = float(allst[:, 0].max()), int(allst[:, 1].sum())
    return {"instances": int(n_inst), "modes": "min-curv + min-time", "ms": round(dt * 1e3, 3),
            "rank0_plan_shapes_KxT": shapes, "shape_batch": n_flight,
            "schedule": f"rl_plan_run_group: {len(plans)} plans in {len(launches)} launches (one per mode and K "
                        f"of one-wave plans), concurrent",
            "tracks_per_s": round(n_inst / dt, 1), "outer_iters_per_s": round(2 * 14 * n_inst / dt, 1),
            "lap_min_s": float(laps.min()), "lap_max_s": float(laps.max())}, laps


def run_c5(world, rank, local, dev, dist):
    """C5: synthetic oval N=10000 (streaming kernel, HBM-bound), 1024 seeds per rank, min-curv."""
    case, prob, cfg = load_problem("oval_n10000")
    B = 1024
    seeds = D.seed_block(world, rank, B)
    s = int(seeds[0])
    plan = raceline.Plan(prob, cfg, seeds=seeds, B=B, modes=abi.RL_MODE_MINCURV, device=local)
    plan.run()
    mc, _ = plan.fetch()
    if dist is not None:
        dist.barrier()
    ms = []
    for _ in range(3):
        plan.run()
        ms.append(plan.kernel_ms(1))
    k_ms = float(np.mean(ms))
    E_k = float(mc.evals.mean())
    Eseg = prob.inner_seg.shape[0] + prob.outer_seg.shape[0]
    model = B * 14 * bytes_per_outer(prob.N, E_k, Eseg)
    rel = float(np.max(np.abs(mc.x[0] - case["mc_x"])) / np.max(np.abs(case["mc_x"]))) if s == 0 else 0.0
    plan.close()
    if dist is not None:
        arr = D.gather_stats([k_ms, rel], world, rank, device=dev)
        if rank != 0:
            return None
        k_ms, rel = float(arr[:, 0].max()), float(arr[:, 1].max())
    pmc = read_pmc("c5_mincurv")
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": "rl_stream_kernel<closed,mincurv>",
            "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
            "achieved": round(pmc["hbm_bytes_per_launch"] / (k_ms * 1e-3) / 1e9, 1) if pmc else None,
            "frac": round(pmc["hbm_bytes_per_launch"] / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if pmc else None,
            "basis": "measured HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE x1, separate --pmc passes, "
                     "profiles/pmc_traffic.json at these kernel sources) / kernel time",
            "counter_calibration": "x2 / x1 measured at this kernel's own 8-B/lane streaming width on a 2 GiB array, "
                                   "through plain and buffer-resource loads (scripts/fetch_calib.hip; "
                                   "profiles/r06/fetch_calib.json: read8 2.000, read8buf 2.000, write8 1.000); the "
                                   "stencil passes' i-1/i+1 neighbour pattern counts 1.872 (plain) / 1.886 (buffer), "
                                   "so frac_range gives the fraction with x1.886 and x2 (ADVICE r5)",
            "frac_range": ([round((1.886 * pmc["fetch_bytes_raw"] + pmc["write_bytes"]) / (k_ms * 1e-3) / 1e9
                                  / HBM_PEAK_GBS, 4),
                            round(pmc["hbm_bytes_per_launch"] / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)]
                           if pmc else None),
            "pmc_profile": pmc.get("profile") if pmc else None,
            "model_GBps_aside": round(model / (k_ms * 1e-3) / 1e9, 1),
            "model_note": "SURVEY §8d one-pass-per-evaluation streaming bytes; batched backtracking reads the state "
                          "once per 4 trial steps, so this model is not a roofline for this kernel"}
    out = {"instances": world * B, "N": prob.N, "kernel_ms": round(k_ms, 3),
           "outer_iters_per_s": round(world * B * 14 / (k_ms * 1e-3), 1), "evals_per_outer": E_k,
           "roofline": roof, "seed0_vs_reference_max_rel_err": rel}
    if rank == 0:
        out["mintime"] = run_c5_mintime(local, prob, cfg, case, B)
    return out


def run_c5_mintime(local, prob, cfg, case, B):
    """compute_min_time_raceline (ref:905-1052) at C5's size: the N=10000 oval, B seeds,
    through the streaming kernel's min-time instantiation (rank 0's own seeds)."""
    plan = raceline.Plan(prob, cfg, seeds=np.arange(B, dtype=np.uint64), B=B, modes=abi.RL_MODE_MINTIME,
                         device=local)
    plan.run()
    ms = []
    for _ in range(3):
        plan.run()
        ms.append(plan.kernel_ms(2))
    _, mt = plan.fetch()
    plan.close()
    k_ms = float(np.mean(ms))
    lap_ref = float(case["mt_lap"])
    return {"instances": B, "kernel_ms": round(k_ms, 3), "outer_iters_per_s": round(B * 14 / (k_ms * 1e-3), 1),
            "evals_per_outer": float(mt.evals.mean()), "vpass_sweeps_mean": float(mt.vpass_sweeps.mean()),
            "kernel": "rl_stream_kernel<closed,mintime>", "lap_seed0_s": float(mt.lap[0]),
            "lap_seed0_vs_reference_rel": abs(float(mt.lap[0]) - lap_ref) / lap_ref}


def run_dropin(local):
    """The reference's own use: one instance per call (pipeline::compute_raceline_and_save
    ref:1347 and compute_mintime_and_save ref:1397), host buffers in and out (PCIe
    included), for the 7 bundled tracks and competition_map1 at N=2000."""
    import ctypes as C

    lib = abi.load_library()
    out = {}
    for name in DROPIN_CASES:
        case, prob, cfg = load_problem(name)
        raceline.optimize_batch(prob, cfg, None, 1)            # warm-up (module load, first launch)
        t = {"mincurv": [], "mintime": []}
        k = {"mincurv": [], "mintime": []}
        for _ in range(5):
            for mode in ("mincurv", "mintime"):
                t0 = time.perf_counter()
                raceline.optimize_batch(prob, cfg, None, 1, mincurv=mode == "mincurv", mintime=mode == "mintime")
                t[mode].append(1e3 * (time.perf_counter() - t0))
                run, kmc, kmt, cm = C.c_float(), C.c_float(), C.c_float(), C.c_float()
                lib.rl_last_call_times(C.byref(run), C.byref(kmc), C.byref(kmt), C.byref(cm))
                k[mode].append((run.value, kmc.value if mode == "mincurv" else kmt.value, cm.value))
        # both optimisers in one call (the ABI runs them concurrently on two streams when one
        # kernel leaves the GPU idle): what a host that needs both pays per track
        tb, kb = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            raceline.optimize_batch(prob, cfg, None, 1)
            tb.append(1e3 * (time.perf_counter() - t0))
            run, cm = C.c_float(), C.c_float()
            lib.rl_last_call_times(C.byref(run), None, None, C.byref(cm))
            kb.append(run.value)
        med = lambda v: round(float(np.median(v)), 3)   # noqa: E731
        out[name] = {"N": prob.N, "mincurv_ms": med(t["mincurv"]), "mintime_ms": med(t["mintime"]),
                     "both_modes_one_call_ms": med(tb), "both_modes_run_bracket_ms": med(kb),
                     "shape_KxT": {m: "x".join(map(str, abi.kernel_shape(prob.N, 1, mode)))
                                   for m, mode in (("mincurv", abi.RL_MODE_MINCURV), ("mintime", abi.RL_MODE_MINTIME))}}
        for mode in ("mincurv", "mintime"):
            # the optimiser kernel alone (its own start/end events)
            out[name][mode + "_kernel_ms"] = med([m for _, m, _ in k[mode]])
            # inside the C call, outside the run bracket: uploads, launch, downloads, host copies
            out[name][mode + "_abi_overhead_ms"] = med([c - r for r, _, c in k[mode]])
            # the Python wrapper's own share (numpy output allocation, ctypes marshalling)
            out[name][mode + "_python_ms"] = med([w - c for w, (_, _, c) in zip(t[mode], k[mode])])
    return out


def run_c2_pcie(prob, cfg, B, MO, rank, reps: int = 5):
    """C2 through the synchronous host-buffer entry point rl_optimize (the drop-in use):
    upload, kernel, download of all result columns into fresh numpy arrays (PCIe and the
    host copies included; the arrays' buffers recycled by abi.HOST_POOL once the caller
    drops them, with a pool-off sub-leg beside it).  The download overlaps the kernel (rl_last_call_download: groups
    of finished instances copied out while later ones compute); the C side copies the
    results out with up to 8 host threads, so this leg runs after the CPU leg, with the
    process's host cores."""
    import ctypes as C

    lib = abi.load_library()
    seeds = np.arange(rank * B, (rank + 1) * B, dtype=np.uint64)
    prev = os.sched_getaffinity(0)
    cores = sorted(HOST_CORES)[:ALLCORE_CORES] if HOST_CORES else sorted(prev)
    os.sched_setaffinity(0, set(cores))
    try:
        for _ in range(4):           # warm-up: the cached plan, pinned staging, flags, host pool, clocks
            raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
        pool = abi.HOST_POOL
        h0, m0 = pool.hits, pool.misses

        def fresh_calls():
            ts, ks = [], []
            for _ in range(reps):
                t0 = time.perf_counter()
                out = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
                ts.append(time.perf_counter() - t0)
                del out              # the caller keeps its results: freeing them is not part of the call
                run, kmc, cm = C.c_float(), C.c_float(), C.c_float()
                lib.rl_last_call_times(C.byref(run), C.byref(kmc), None, C.byref(cm))
                g, sg = C.c_int32(), C.c_int32()
                lib.rl_last_call_download(C.byref(g), C.byref(sg))
                ks.append((run.value, kmc.value, cm.value, g.value, sg.value))
            return ts, ks

        ts, ks = fresh_calls()
        pool_hits, pool_misses = pool.hits - h0, pool.misses - m0
        # the same calls into output arrays the caller keeps (pages already present)
        keep = raceline.optimize_batch(prob, cfg, seeds, B, mintime=False)
        tr, kr = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            raceline.optimize_batch(prob, cfg, seeds, B, mintime=False, out=keep)
            tr.append(time.perf_counter() - t0)
            run, kmc, cm = C.c_float(), C.c_float(), C.c_float()
            lib.rl_last_call_times(C.byref(run), C.byref(kmc), None, C.byref(cm))
            kr.append((kmc.value, cm.value))
        del keep
        # last, fresh outputs with the host pool off: every call's arrays newly mapped by numpy
        # and unmapped after it (the round-5 wrapper's behaviour)
        cap = pool.cap
        pool.cap = 0
        try:
            tn, kn = fresh_calls()
        finally:
            pool.cap = cap
    finally:
        os.sched_setaffinity(0, prev)
    t = float(np.median(ts))
    reused = {"call_ms_median": round(float(np.median(tr)) * 1e3, 2),
              "outer_iters_per_s": round(B * MO / float(np.median(tr)), 1),
              "kernel_ms_median": round(float(np.median([k for k, _ in kr])), 3),
              "abi_call_ms_median": round(float(np.median([c for _, c in kr])), 3),
              "note": "output arrays allocated once and passed to every call (optimize_batch(out=...)): "
                      "no page faults in the copies, and the next kernel is not slowed (DESIGN §3g)"}
    no_pool = {"call_ms_median": round(float(np.median(tn)) * 1e3, 2),
               "outer_iters_per_s": round(B * MO / float(np.median(tn)), 1),
               "kernel_ms_median": round(float(np.median([k[1] for k in kn])), 3),
               "note": "RL_HOST_POOL_MB=0: fresh arrays mapped by numpy every call and unmapped after it"}
    return {"call_ms_median": round(t * 1e3, 2), "outer_iters_per_s": round(B * MO / t, 1),
            "reused_outputs": reused, "host_pool_off": no_pool,
            "host_pool": {"hits": int(pool_hits), "misses": int(pool_misses), "cap_mb": round(pool.cap / 2**20)},
            "call_ms_all": [round(x * 1e3, 2) for x in ts],
            "run_bracket_ms_median": round(float(np.median([k[0] for k in ks])), 3),
            "kernel_ms_median": round(float(np.median([k[1] for k in ks])), 3),
            "abi_call_ms_median": round(float(np.median([k[2] for k in ks])), 3),
            # the Python wrapper's share: fresh numpy output arrays and ctypes marshalling
            "python_wrapper_ms_median": round(float(np.median([1e3 * w - k[2] for w, k in zip(ts, ks)])), 3),
            "download_groups": int(ks[-1][3]), "download_groups_signalled_min": int(min(k[4] for k in ks)),
            "host_cores": len(cores),
            "bytes_down": int(B * prob.N * 6 * 8 + B * MO * 8),
            "note": "fresh numpy outputs per call (freed after it), their buffers recycled by the library's "
                    "host pool (abi.HostPool); kernel_ms is the optimiser in this call pattern (DESIGN §3g); the "
                    "download of each group of 64 finished instances overlaps the later instances' compute"}


def run_step6(world, rank):
    """step 6 (compute_geom_and_save) for competition_map1 at
    samples=2000 on the GPU (rl_geom) vs the CPU oracle on the same inputs; the rows
    formatted as <base>_with_geom.csv are compared with the reference's own file."""
    import oracle_lib as O

    if rank != 0:
        return None
    case = O.load_geom_case("cmap1_n2000")
    gp, cfg = O.geom_problem(case), O.geom_cfg(case)
    raceline.compute_geom(gp, cfg)                       # warm-up (module load, first launch)
    walls, kms = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        rows, kms_i = raceline.compute_geom(gp, cfg, return_ms=True)
        walls.append(time.perf_counter() - t0)
        kms.append(kms_i)
    return {"rows": int(rows.shape[0]), "segments": int(gp.inner_seg.shape[0] + gp.outer_seg.shape[0]),
            "kernel_ms": round(float(np.median(kms)), 4), "wall_ms_incl_transfers": round(1e3 * float(np.median(walls)), 3),
            "csv_bytes_equal_reference": raceline.format_geom_csv(rows).encode() == case["_csv"]}


def run_lapeval(world, rank, racelines):
    """batched lap evaluations (heading/kappa + v-pass, h = L/N) of the
    C2 run's 1024 optimised racelines (rank 0's), GPU, checked on a sample against the oracle."""
    import oracle_lib as O

    if rank != 0:
        return None
    case, prob, cfg = load_problem("cmap1_n2000")
    P = np.ascontiguousarray(racelines)
    B, N = P.shape[0], P.shape[1]
    Ls = np.full(B, float(prob.L))
    raceline.lap_eval(P[:8], Ls[:8], True, cfg)                        # warm-up
    t0 = time.perf_counter()
    ev, kms = raceline.lap_eval(P, Ls, True, cfg, return_ms=True)
    wall = time.perf_counter() - t0
    for b in (0, B // 2, B - 1):
        orc = O.run_oracle_lap_eval(P[b], float(prob.L), True, cfg)
        assert abs(orc.lap[0] - ev.lap[b]) <= 1e-9 * orc.lap[0]
    return {"paths": B, "N": N, "kernel_ms": round(kms, 3), "wall_ms_incl_transfers": round(1e3 * wall, 2),
            "laps_per_s_kernel": round(B / (kms * 1e-3), 1), "lap_min_s": float(ev.lap.min()),
            "lap_max_s": float(ev.lap.max())}


def run_format(world, rank, mc_x, mc_y, mc_k, mc_al, case, cfg):
    """the _raceline_with_geom.csv tables (7 columns, N+1 rows) of the
    C2 run's 1024 instances formatted on the GPU in one pass (rl_format_csv), checked on
    a sample against glibc "%.9f" (the oracle's snprintf loop)."""
    import oracle_lib as O

    if rank != 0:
        return None
    B, N = mc_x.shape
    L, s0 = float(case["L"]) if "L" in case else 0.0, float(case["s0"]) if "s0" in case else 0.0
    s = (s0 + L * (np.arange(N) / float(N))) - s0
    T = np.zeros((B, N + 1, 7))
    T[:, :N, 0] = s
    T[:, :N, 1], T[:, :N, 2], T[:, :N, 4], T[:, :N, 5] = mc_x, mc_y, mc_k, mc_al
    T[:, :N, 3] = np.arctan2(np.gradient(mc_y, axis=1), np.gradient(mc_x, axis=1))     # a heading-like column
    T[:, :N, 6] = np.minimum(cfg.v_cap_mps, np.sqrt(cfg.a_lat_max / np.maximum(np.abs(mc_k), cfg.kappa_eps)))
    T[:, N] = T[:, 0]
    T[:, N, 0] = L
    T = T.reshape(-1, 7)
    raceline.format_table(T[:100])                                      # warm-up
    t0 = time.perf_counter()
    text = raceline.format_table(T)
    gpu_s = time.perf_counter() - t0
    k = 20000
    cpu_text = O.oracle_format_rows(T[:k])
    return {"rows": int(T.shape[0]), "numbers": int(T.size), "bytes": len(text),
            "gpu_wall_ms_incl_transfers": round(1e3 * gpu_s, 2), "gpu_MB_per_s": round(len(text) / gpu_s / 1e6, 1),
            "bytes_equal_on_sample": text[: len(cpu_text)] == cpu_text, "sample_rows": k}


def run_result_gather(res_buf, res, world, rank, dev, dist, backend, same_device, B, N, MO, reps: int = 3):
    """SURVEY §8e's final gather at its real size, outside the timed C2 steps: every rank's
    whole min-curvature result block (x, y, κ, α_last, α_total, heading: [B][N] float64
    each, and evals [B][MO] int32; one contiguous buffer the plan writes into) gathered to
    rank 0 with one collective per rank -- RCCL over xGMI under the nccl backend, host
    copies under gloo.  Timed between barriers + device syncs, `reps` times; the max over
    ranks of the median is reported.  Rank 0 then checks block 0 against its own buffer and
    every block's per-instance summary against the summary rows its rank sent in the timed
    steps (bit for bit)."""
    import torch

    nbytes = int(res_buf.numel())
    ts, blocks = [], None
    for _ in range(reps):
        blocks = None
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        blocks = D.gather_result_blocks(res_buf, world, rank)
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    st = D.gather_stats([float(np.median(ts)), float(min(ts))], world, rank, device=dev if backend == "nccl" else None)
    mine = D.instance_summary(res["evals"], res["x"], res["alpha_last"]).cpu()
    sums = D.gather_rows(mine.to(dev) if backend == "nccl" else mine, world, rank)
    if rank != 0:
        return None
    sums = sums.cpu().numpy().reshape(world, B, 3)
    ok0 = bool(torch.equal(blocks[0].to(res_buf.device), res_buf))
    ok = []
    for r, blk in enumerate(blocks):
        v = D.result_views(blk.to(dev), B, N, MO)
        ok.append(bool(np.array_equal(D.instance_summary(v["evals"], v["x"], v["alpha_last"]).cpu().numpy(), sums[r])))
    t_med, t_min = float(st[:, 0].max()), float(st[:, 1].max())
    where = "same-device rehearsal" if same_device else "one rank per GPU"
    return {"bytes_per_rank": nbytes, "bytes_total": nbytes * world, "instances_gathered": world * B,
            "arrays": list(D.RESULT_F64) + ["evals"], "reps": reps,
            "ms": round(t_med * 1e3, 3), "ms_min": round(t_min * 1e3, 3),
            "GBps_per_rank": round(nbytes / t_med / 1e9, 2),
            "rank0_ingress_GBps": round(nbytes * (world - 1) / t_med / 1e9, 2),
            "backend": ("RCCL (torch.distributed nccl gather) over xGMI, device to device" if backend == "nccl"
                        else f"torch.distributed {backend} gather of host copies (device->host included)") + f"; {where}",
            "rank0_block_equals_own": ok0, "blocks_equal_step_summaries": all(ok),
            "note": "outside the timed C2 steps; max over ranks of each rank's median gather time"}


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_plan(gpus: int, env, argv) -> list | None:
    """How `bench.py --gpus N` runs (decided before anything touches the GPU).

    * WORLD_SIZE unset, N == 1: this process is the single rank (None).
    * WORLD_SIZE unset, N > 1: this process only launches N fresh ranks, one per GPU, with
      torch.distributed.run on 127.0.0.1 (the command is returned; the parent relays rank
      0's JSON line and the exit code).
    * WORLD_SIZE set (launched by torch.distributed.run): it must equal N, else SystemExit.
    """
    if gpus < 1:
        raise SystemExit(f"bench: --gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench: WORLD_SIZE={ws} but --gpus {gpus}: launch one rank per GPU "
                             f"(--nproc-per-node {gpus}) or pass --gpus {ws}")
        return None
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)


def backend_label(world: int, backend: str, same_device: bool) -> str:
    """The `parallelism` string: what actually ran (backend and device placement)."""
    if world == 1:
        return "dp1: one GPU, no collective"
    coll = "RCCL (torch.distributed nccl) over xGMI" if backend == "nccl" else f"torch.distributed {backend}"
    where = (f"{world} ranks on one GPU (same-device rehearsal)" if same_device
             else f"instances sharded over {world} GPUs, one rank per GPU")
    return (f"dp{world}: {where}; per-step {coll} gather of per-instance summaries to rank 0, then one "
            f"{coll} gather of every rank's whole result block (result_gather, outside the timed steps)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="only the timed C2 steps")
    ap.add_argument("--cpu-leg", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()
    if args.cpu_leg:
        print(json.dumps(cpu_leg(args.cpu_budget)), flush=True)
        if sys.stdin.readline().strip() == "go":
            print(json.dumps(cpu_multicore_leg()), flush=True)
        return
    cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:
        # N ranks as child processes (this parent has not touched the GPU and never does);
        # rank 0's JSON line reaches stdout through the inherited descriptor
        rc = subprocess.run(cmd, env={**os.environ, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}).returncode
        sys.exit(rc)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU leg (rank 0, any world size) starts before this process touches the GPU; the
    # other ranks keep off its pinned core
    HOST_CORES.update(os.sched_getaffinity(0))
    cpu_proc = start_cpu_leg(args.cpu_budget) if (rank == 0 and not args.no_cpu and not args.no_extras) else None
    if rank != 0 and len(HOST_CORES) > 2:
        os.sched_setaffinity(0, set(HOST_CORES) - {min(HOST_CORES)})
    # rehearsal on a one-GPU box only: every rank on cuda:0, gloo instead of RCCL
    same_device = os.environ.get("RL_BENCH_SAME_DEVICE") == "1"
    if same_device:
        local = 0
    backend = os.environ.get("RL_BENCH_BACKEND", "nccl")
    import torch

    if world > 1 and not same_device and torch.cuda.device_count() < world:
        raise SystemExit(f"bench: {world} ranks but only {torch.cuda.device_count()} visible GPU(s)")

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    lib = abi.load_library()
    if lib.rl_device_count() < 1:
        raise SystemExit("bench: no HIP device visible")

    case, prob, cfg = load_problem("cmap1_n2000")
    B = args.batch
    N = prob.N
    MO = int(cfg.max_outer_iters)
    seeds = D.seed_block(world, rank, B)
    plan = raceline.Plan(prob, cfg, seeds=seeds, B=B, modes=abi.RL_MODE_MINCURV, device=local)

    # results straight into views of one contiguous device block per rank (zero-copy for
    # the result gather: one RCCL collective per rank)
    res_buf, res = D.alloc_result_block(B, N, MO, device=dev)
    plan.bind_device_outputs(abi.RL_MODE_MINCURV, {k: v.data_ptr() for k, v in res.items()})

    stream = torch.cuda.Stream(device=dev)
    gathered = {}

    def step():
        plan.run(stream.cuda_stream)
        if world > 1:
            with torch.cuda.stream(stream):
                rows = D.gather_rows(D.instance_summary(res["evals"], res["x"], res["alpha_last"]), world, rank)
                if rank == 0:
                    gathered["summary"] = rows

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if args.steps <= 50:
            stream.synchronize()
            kernel_ms.append(plan.kernel_ms(1))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    total_outer = world * B * MO * args.steps
    result_gather = run_result_gather(res_buf, res, world, rank, dev, dist, backend, same_device, B, N, MO) \
        if world > 1 else None
    value = total_outer / elapsed
    tracks_per_s = world * B * args.steps / elapsed

    extras = {}
    if not args.no_extras:
        c4, c4_laps = run_c4(world, rank, local, dev, dist)
        c5 = run_c5(world, rank, local, dev, dist)
        if rank == 0:
            c3, c3_laps = run_c3(rank, local, stream)
            extras["c3_mintime_plus_mincurv"] = c3
            extras["c4_sweep_7tracks_x_512"] = c4
            extras["c5_oval_n10000"] = c5
            extras["open_mode_n2000"], open_gpu = run_open(local)
            extras["step6_geom_cmap1_n2000"] = run_step6(world, rank)
            xh, yh = res["x"].cpu().numpy(), res["y"].cpu().numpy()
            extras["lap_eval_1024_racelines_n2000"] = run_lapeval(world, rank, np.stack([xh, yh], axis=2))
            extras["csv_format_1024_instances"] = run_format(world, rank, xh, yh, res["kappa"].cpu().numpy(),
                                                              res["alpha_last"].cpu().numpy(), case, cfg)
    if rank != 0:
        plan.close()
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    # ---- parity of this run (outside the timed region) ----
    summary_check = None
    if world > 1:
        allsum = gathered["summary"].cpu().numpy()                    # [world*B, 3], rank-major
        mine = D.instance_summary(res["evals"], res["x"], res["alpha_last"]).cpu().numpy()
        summary_check = {"instances_gathered": int(allsum.shape[0]),
                         "rank0_rows_equal": bool(np.array_equal(allsum[:B], mine)),
                         "seed0_x_sum_vs_reference": float(abs(allsum[0, 1] - float(np.sum(case["mc_x"]))))}
    evals = res["evals"].cpu().numpy()
    E_k = float(evals.mean())
    x0 = res["x"][0].cpu().numpy()
    al0 = res["alpha_last"][0].cpu().numpy()
    k0 = res["kappa"][0].cpu().numpy()
    parity = {
        "seed0_vs_reference_max_rel_err": float(max(
            np.max(np.abs(x0 - case["mc_x"])) / np.max(np.abs(case["mc_x"])),
            np.max(np.abs(al0 - case["mc_alpha_last"])) / np.max(np.abs(case["mc_alpha_last"])),
            np.max(np.abs(k0 - case["mc_kappa"])) / np.max(np.abs(case["mc_kappa"])))),
        "tolerance": "1e-4 x column max (+1e-9)",
    }

    # ---- roofline of the dominant kernel (HIP events on the launch stream) ----
    Eseg = prob.inner_seg.shape[0] + prob.outer_seg.shape[0]
    k_ms = float(np.mean(kernel_ms)) if kernel_ms else plan.kernel_ms(1)
    fl_launch = B * MO * flops_per_outer(N, E_k, Eseg)
    achieved_tf = fl_launch / (k_ms * 1e-3) / 1e12
    pmc = read_pmc("c2_mincurv")
    roofline = {
        "bound": "fp64-valu", "achieved": round(achieved_tf, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved_tf / FP64_PEAK_TFLOPS, 4),
        "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
        "kernel": "rl_optimize_kernel<8,256,closed,mincurv>", "kernel_ms": round(k_ms, 3),
        "flops_per_launch_algorithmic": fl_launch,
        "algorithmic_model": f"SURVEY §8d: N*(34*E_k + 26*(Ei+Eo)) per outer, N={N}, E_k={E_k:.2f}, "
                             f"Ei+Eo={Eseg}, x {B}x{MO} outers (the corridor term counts the reference's "
                             f"every-segment ray tests; the kernel culls most of them exactly)",
        "peak_note": "78.6 TF = MI355X fp64 vector peak with FMA counted as 2 flops; the path's operations are "
                     "mostly plain add/mul (-ffp-contract=off keeps the reference's roundings), whose ceiling on "
                     "the same pipe is 39.3 TF",
        "frac_of_nonfma_ceiling": round(achieved_tf / FP64_NONFMA_TFLOPS, 4),
        "evals_per_outer": round(E_k, 2),
    }
    if pmc:
        # north_star's achieved-HBM fraction, measured: PMC bytes per launch / this kernel time
        hbm_gbs = pmc["hbm_bytes_per_launch"] / (k_ms * 1e-3) / 1e9
        roofline["hbm_GBps_measured"] = round(hbm_gbs, 1)
        roofline["hbm_frac_measured"] = round(hbm_gbs / HBM_PEAK_GBS, 4)
    # SURVEY §8d's streaming byte model beside the flop roofline (its achieved/8 TB/s exceeds
    # 1 at C2: the per-evaluation state lives in VGPRs/LDS and never reaches HBM)
    model_b = B * MO * bytes_per_outer(N, E_k, Eseg)
    model_gbs = model_b / (k_ms * 1e-3) / 1e9
    roofline["byte_model"] = {
        "bytes_per_launch": model_b, "achieved_GBps": round(model_gbs, 1), "peak_GBps": HBM_PEAK_GBS,
        "frac": round(model_gbs / HBM_PEAK_GBS, 3),
        "model": f"SURVEY §8d: N*(80*E_k + 224) + 32*(Ei+Eo) bytes per outer, x {B}x{MO} outers",
        "note": "frac > 1: on-chip residency -- the state stays in VGPRs/LDS across evaluations, so the HBM "
                "roofline does not bind; the measured HBM traffic is `traffic`"}
    if pmc:
        ex = pmc.get("fp64_flops_per_launch")
        if ex:
            roofline["executed_fp64_TFLOPs_pmc"] = round(ex / (k_ms * 1e-3) / 1e12, 3)
            roofline["executed_frac"] = round(ex / (k_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4)
        for key in ("valu_fp64_share", "hbm_GBps_note"):
            if pmc.get(key) is not None:
                roofline[key + "_pmc"] = pmc[key]
        roofline["pmc_profile"] = pmc.get("profile")
    roofline["pmc_source_sha"] = source_sha() if pmc else None

    cpu, cpu_res = None, None
    if cpu_proc is not None:
        cpu_res = read_cpu_leg(cpu_proc)
    # the drop-in legs (host buffers, host copy threads) once the CPU leg has left the host
    # cores: the reference's caller has them to itself
    if not args.no_extras:
        extras["c2_pcie_inclusive"] = run_c2_pcie(prob, cfg, B, MO, rank)
        extras["dropin_b1_latency"] = run_dropin(local)
    if cpu_proc is not None:
        mc = finish_cpu_leg(cpu_proc, cpu_res is not None)
        if cpu_res is not None:
            cpu_res.update(mc)
    if cpu_res is not None:
        cpu = dict(cpu_res.get("reference") or cpu_res["port"])
        cpu["cpu_model"] = cpu_res["cpu"]["model"]
        cpu["host_nproc"] = cpu_res["cpu"]["nproc"]
        cpu["port_restatement"] = cpu_res["port"] if cpu_res.get("reference") else None
        cpu["reference_multicore_context"] = cpu_res.get("reference_multicore")
        if "c3_mintime_plus_mincurv" in extras:
            c3o = cpu_res["c3_oracle_laps"]
            extras["c3_mintime_plus_mincurv"]["lap_delta_vs_oracle"] = {
                **lap_delta(c3_laps[c3o["seeds"]], c3o["laps"]),
                "sample": f"{len(c3o['seeds'])} seeds strided over the {C3_BATCH}-instance batch (seeds "
                          f"{c3o['seeds'][0]}..{c3o['seeds'][-1]} step {C3_BATCH // C3_SAMPLE})"}
        if "c4_sweep_7tracks_x_512" in extras and c4_laps is not None:
            extras["c4_sweep_7tracks_x_512"]["lap_delta_vs_oracle"] = {
                **lap_delta(c4_laps, cpu_res["c4_oracle_laps"]), "sample": "all 3584 (track, sweep point) instances"}
        if "dropin_b1_latency" in extras and cpu_res.get("reference_per_track"):
            for name, v in extras["dropin_b1_latency"].items():
                r = cpu_res["reference_per_track"].get(name)
                if r:
                    v["reference_cpu_mincurv_ms"] = r["mincurv_ms"]
                    v["reference_cpu_mintime_ms"] = r["mintime_ms"]
        if "open_mode_n2000" in extras and cpu_res.get("open_oracle"):
            oo = cpu_res["open_oracle"]
            gx, ox = np.array(open_gpu["x"]), np.array(oo["x"])
            extras["open_mode_n2000"]["vs_oracle"] = {
                "seeds": list(range(OPEN_CHECK)),
                "x_max_abs": float(np.max(np.abs(gx - ox))), "x_tol": 1e-4 * float(np.max(np.abs(ox))) + 1e-9,
                "lap_max_rel": float(np.max(np.abs(np.array(open_gpu["lap"]) - np.array(oo["lap"])) / np.abs(oo["lap"]))),
                "evals_equal": open_gpu["evals"] == oo["evals"] and open_gpu["mt_evals"] == oo["mt_evals"]}
        extras["cpu_oracle_pool"] = cpu_res.get("oracle_pool")
        if cpu_res.get("c2_oracle_npz") and B == C2_BATCH:
            parity["c2_all_instances_vs_oracle"] = c2_full_parity(res, cpu_res["c2_oracle_npz"])

    out = {
        "metric": "PGD outer-iters/sec (N=2000 samples, closed, competition_map1, 1024 alpha-seeds/GPU, min-curv)",
        "value": round(value, 1),
        "unit": "PGD outer-iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "competition_map1 cones from the reference repo -> reference steps 1-6 (fixture); synthetic alpha-seeds",
        "config": {"workload": "C2: competition_map1 closed, N=2000, B=1024 alpha-seeds per GPU, min-curvature, "
                               "14 outer iterations, default cfg::Config", "N": N, "batch_per_gpu": B,
                   "global_batch": world * B, "parallelism": backend_label(world, backend, same_device),
                   "backend": backend if world > 1 else None},
        "tracks_per_s": round(tracks_per_s, 2),
        "hip_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        "roofline": roofline,
        "cpu_baseline": cpu,
        "parity": parity if summary_check is None else {**parity, "gather": summary_check},
        **({"result_gather": result_gather} if result_gather is not None else {}),
        **extras,
    }
    print(json.dumps(out), flush=True)
    plan.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
