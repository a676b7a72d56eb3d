"""Multi-GPU plumbing for batched raceline optimisation.

Instances (α-seeds, cfg sweep points, tracks) are independent, so the batch is
sharded across ranks with no data-path collective (weak scaling); a single
instance is never split.  The only collective is the final gather of results
to rank 0 over RCCL (torch.distributed backend "nccl" on ROCm) — or gloo on CPU
for the tests.  One process per GPU, launched by torch.distributed.run.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [start, end) of `total` items for `rank` (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_to_root(tensors: Dict[str, "object"], world: int, rank: int, group=None):
    """dist.gather every tensor of `tensors` to rank 0.  Shapes must match across
    ranks (pad shards to the same size).  Returns {name: [tensor per rank]} on rank 0,
    None elsewhere.  With the nccl backend this is RCCL over xGMI, device to device."""
    import torch
    import torch.distributed as dist

    out = {} if rank == 0 else None
    host = dist.get_backend(group) == "gloo"      # gloo gathers host tensors (CPU tests, rehearsal)
    for name, t in tensors.items():
        if host and t.is_cuda:
            t = t.cpu()
        lst = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
        dist.gather(t, lst, dst=0, group=group)
        if rank == 0:
            out[name] = lst
    return out


def seed_block(world: int, rank: int, B: int) -> np.ndarray:
    """Weak scaling: rank r optimises seeds [r*B, (r+1)*B) (rank 0 / seed 0 = the reference)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return np.arange(rank * B, (rank + 1) * B, dtype=np.uint64)


def instance_summary(evals, x, alpha_last):
    """Per-instance summary rows [B, 3] = (Σ evaluations, Σ x, Σ α_last): what every rank
    sends to rank 0 each step (a gather of per-instance summaries); the full
    SoA results are gathered once after the timed steps (gather_result_blocks).  torch
    tensors in, float64 tensor out."""
    import torch

    return torch.stack([evals.sum(1, dtype=torch.float64), x.sum(1), alpha_last.sum(1)], dim=1)


def gather_rows(t, world: int, rank: int, group=None):
    """Gather equal-shape row blocks to rank 0 in rank order: the concatenation on rank 0,
    None elsewhere."""
    import torch

    got = gather_to_root({"t": t}, world, rank, group)
    return torch.cat(got["t"]) if rank == 0 else None


def gather_stats(values: Sequence[float], world: int, rank: int, device=None, group=None):
    """Gather one row of float64 values per rank to rank 0: a numpy [world, len(values)]
    array on rank 0 (row r = rank r's values), None elsewhere.  The bench reduces the rows
    (max of the per-rank times, sum of the instance counts)."""
    import torch

    t = torch.tensor([list(values)], dtype=torch.float64, device=device)
    rows = gather_rows(t, world, rank, group)
    return rows.cpu().numpy() if rank == 0 else None


# --------------------------------------------------------- result block (SURVEY §8e gather)
# One rank's min-curvature results as ONE contiguous byte buffer, so the final gather is a
# single collective per rank: six [B][N] float64 columns, then the [B][MO] int32
# evaluations.  The plan writes its outputs straight into views of the buffer
# (rl_plan_bind_device_outputs), so gathering needs no packing copy.
RESULT_F64 = ("x", "y", "kappa", "alpha_last", "alpha_total", "heading")


def result_layout(B: int, N: int, MO: int) -> Dict[str, Tuple[int, int, str, Tuple[int, int]]]:
    """{name: (byte offset, bytes, dtype name, shape)} of a result block."""
    out, off = {}, 0
    for name in RESULT_F64:
        n = B * N * 8
        out[name] = (off, n, "float64", (B, N))
        off += n
    out["evals"] = (off, B * MO * 4, "int32", (B, MO))
    return out


def result_block_bytes(B: int, N: int, MO: int) -> int:
    return sum(v[1] for v in result_layout(B, N, MO).values())


def result_views(buf, B: int, N: int, MO: int) -> Dict[str, "object"]:
    """Typed views (torch) of a uint8 result block: {name: tensor of its dtype and shape}."""
    import torch

    dt = {"float64": torch.float64, "int32": torch.int32}
    return {name: buf[o:o + n].view(dt[d]).view(*shape) for name, (o, n, d, shape) in result_layout(B, N, MO).items()}


def alloc_result_block(B: int, N: int, MO: int, device=None):
    """A zeroed uint8 result block on `device` and its typed views."""
    import torch

    buf = torch.zeros(result_block_bytes(B, N, MO), dtype=torch.uint8, device=device)
    return buf, result_views(buf, B, N, MO)


def gather_result_blocks(buf, world: int, rank: int, group=None):
    """dist.gather of every rank's result block to rank 0 (RCCL over xGMI with the nccl
    backend, device to device; gloo gathers host copies).  Returns the list of blocks in
    rank order on rank 0, None elsewhere."""
    got = gather_to_root({"r": buf}, world, rank, group)
    return got["r"] if rank == 0 else None


def gather_ragged(a: np.ndarray, world: int, rank: int, total: int, device=None, group=None):
    """Gather 1-D float64 shards of different lengths (at most ceil(total/world) each) to
    rank 0 in rank order.  Returns the concatenation (numpy) on rank 0, None elsewhere."""
    import torch

    per = pad_to(total, world)
    a = np.asarray(a, dtype=np.float64).ravel()
    if a.size > per:
        raise ValueError("shard larger than ceil(total/world)")
    buf = torch.zeros(per + 1, dtype=torch.float64, device=device)
    buf[0] = float(a.size)
    buf[1:1 + a.size] = torch.from_numpy(a).to(buf.device)
    got = gather_to_root({"b": buf}, world, rank, group)
    if rank != 0:
        return None
    parts = [g.cpu().numpy() for g in got["b"]]
    return np.concatenate([p[1:1 + int(p[0])] for p in parts])


# ----------------------------------------------------------------- C4 sweep
C4_TRACKS = ["training_map", "competition_map1", "competition_map2", "competition_map3",
             "competition_map_testday1", "competition_map_testday2", "competition_map_testday3"]


def c4_grid() -> List[Tuple[float, float, float]]:
    """mu in linspace(0.9,1.5,8), P_max_W in linspace(40kW,120kW,8),
    lambda_smooth in logspace(4e-4, 6.4e-3, 8) -> 512 points (mu-major)."""
    mus = np.linspace(0.9, 1.5, 8)
    Ps = np.linspace(40000.0, 120000.0, 8)
    lams = np.geomspace(4e-4, 6.4e-3, 8)
    return [(float(m), float(P), float(l)) for m in mus for P in Ps for l in lams]


def c4_cfgs(base: abi.RlCfg) -> List[abi.RlCfg]:
    """512 cfgs; a_total_max = 9.81*mu recomputed per point (ref:102 quirk)."""
    out = []
    for mu, P, lam in c4_grid():
        c = abi.RlCfg.from_dict(base.to_dict())
        abi.set_mu(c, mu)
        c.P_max_W = P
        c.lambda_smooth = lam
        out.append(c)
    return out


def c4_items(n_tracks: int = 7, n_points: int = 512) -> List[Tuple[int, int]]:
    """Track-major (track, sweep point) items: 7 x 512 = 3584."""
    return [(t, k) for t in range(n_tracks) for k in range(n_points)]


def c4_shard(world: int, rank: int, n_tracks: int = 7, n_points: int = 512) -> Dict[int, List[int]]:
    """Rank's share of the C4 items grouped by track: {track: [sweep point indices]}."""
    items = c4_items(n_tracks, n_points)
    s, e = shard_range(len(items), world, rank)
    groups: Dict[int, List[int]] = {}
    for t, k in items[s:e]:
        groups.setdefault(t, []).append(k)
    return groups


def pad_to(n: int, world: int) -> int:
    return int(math.ceil(n / world))
