"""Host-side mirror of the reference's raceline interface, over the C-ABI.

Reference (``ref`` = /root/reference/src/main.cpp):

* :func:`compute_min_curvature_raceline` — ``raceline_min_curv::compute_min_curvature_raceline``
  (ref:683-764): same arguments (center, innerE, outerE, veh_width, L, closed),
  same :class:`MinCurvResult` fields (raceline, heading, curvature,
  alpha_total, alpha_last; ref:677-681).
* :func:`compute_min_time_raceline` — ``raceline_min_time::compute_min_time_raceline``
  (ref:905-1052), :class:`MinTimeResult` adds v, ax, lap_time (ref:897-903).
* :func:`ring_edges` / :func:`polyline_edges` — ``edges::ringEdges`` / ``polylineEdges`` (ref:251-260).
* :func:`compute_raceline_and_save` / :func:`compute_mintime_and_save` — the
  pipeline callers and their CSV writers (ref:1337-1438), same file names,
  headers and ``precision(9)`` fixed formatting.
* ``cfg`` — :func:`default_cfg` holds ``cfg::Config``'s hot-path knobs (ref:77-113).

Beyond the reference: :func:`optimize_batch` and :class:`Plan` run B
instances (α-seeds, cfg sweeps) in one launch; that is the product.

Every compute call goes through ``librl.so`` (HIP, gfx950).  With no GPU the
calls raise :class:`RacelineError` (RL_ENODEV): there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import abi
from .abi import GeomProblem, Outputs, Problem, RlCfg, default_cfg, set_mu  # noqa: F401


class RacelineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rl error {code}: {msg}")
        self.code = code


def _lib():
    return abi.load_library()


def _check(rc: int) -> None:
    if rc != 0:
        raise RacelineError(rc, _lib().rl_last_error().decode(errors="replace"))


# ------------------------------------------------------------------ geometry
def ring_edges(ring: np.ndarray) -> np.ndarray:
    """edges::ringEdges (ref:251-255): n segments, the last one closing the ring."""
    ring = np.ascontiguousarray(ring, dtype=np.float64).reshape(-1, 2)
    n = len(ring)
    if n == 0:
        return np.zeros((0, 4))
    return np.concatenate([ring, np.roll(ring, -1, axis=0)], axis=1)


def polyline_edges(ring: np.ndarray) -> np.ndarray:
    """edges::polylineEdges (ref:256-260): n-1 segments."""
    ring = np.ascontiguousarray(ring, dtype=np.float64).reshape(-1, 2)
    if len(ring) < 2:
        return np.zeros((0, 4))
    return np.concatenate([ring[:-1], ring[1:]], axis=1)


def edges_for(ring: np.ndarray, closed: bool) -> np.ndarray:
    return ring_edges(ring) if closed else polyline_edges(ring)


# ------------------------------------------------------------------ results
@dataclass
class MinCurvResult:
    """raceline_min_curv::Result (ref:677-681)."""

    raceline: np.ndarray      # [N,2]
    heading: np.ndarray
    curvature: np.ndarray
    alpha_total: np.ndarray
    alpha_last: np.ndarray
    evals: Optional[np.ndarray] = None


@dataclass
class MinTimeResult(MinCurvResult):
    """raceline_min_time::Result (ref:897-903)."""

    v: Optional[np.ndarray] = None
    ax: Optional[np.ndarray] = None
    lap_time: float = 0.0
    vpass_sweeps: Optional[np.ndarray] = None


# ------------------------------------------------------------------ batch API
def _check_batch(B: int, ncfg: int, seeds) -> None:
    """The C side reads exactly B seeds and B (or 1) cfgs (rl_abi.h): a shorter array
    would be read past its end, so a mismatch is an error here."""
    if B < 0:
        raise ValueError(f"B must be >= 0, got {B}")
    if ncfg not in (1, B):
        raise ValueError(f"cfgs: need 1 or B={B} entries, got {ncfg}")
    if seeds is not None and len(seeds) != B:
        raise ValueError(f"seeds: need exactly B={B} entries, got {len(seeds)}")


def optimize_batch(prob: Problem, cfgs, seeds=None, B: Optional[int] = None,
                   mincurv: bool = True, mintime: bool = True, devices: Optional[Sequence[int]] = None,
                   out=None):
    """Optimise B instances (seed b / cfg b) of one problem on the GPU.

    cfgs: one RlCfg (broadcast) or a list of B.  seeds: None (all zero — the
    reference exactly) or B uint64 seeds.  devices: None (the current device) or a
    list of device indices: contiguous instance blocks, one per device
    (rl_optimize_multi).  out: None (fresh output arrays from abi.HOST_POOL, which
    recycles the buffers of earlier results the caller has dropped) or the
    (Outputs|None, Outputs|None) of an earlier call of the same shape, written in place
    (a caller that keeps its buffers, as the C ABI's callers own theirs).  Returns
    (Outputs|None, Outputs|None).
    """
    cfg_arr, ncfg = abi.cfg_array(cfgs)
    if B is None:
        B = ncfg if ncfg > 1 else (len(seeds) if seeds is not None else 1)
    _check_batch(B, ncfg, seeds)
    mo = int(cfg_arr[0].max_outer_iters)
    seeds_a = abi.seed_array(seeds)
    if out is not None:
        out_mc, out_mt = out
        for o, want, mt in ((out_mc, mincurv, False), (out_mt, mintime, True)):
            if (o is not None) != want:
                raise ValueError("out: one Outputs per requested mode (None for the others)")
            if o is not None and (o.x.shape != (B, prob.N) or o.evals.shape != (B, mo) or (mt and o.lap is None)
                                  or not all(getattr(o, f).flags.c_contiguous for f in abi.OUT_F64)):
                raise ValueError("out: Outputs of a different shape or mode")
    else:
        # every element is written by the call (no zeroing of memory about to be overwritten);
        # buffers recycled from arrays of earlier calls that the caller has dropped
        out_mc = Outputs.alloc(B, prob.N, mo, False, zero=False, pool=abi.HOST_POOL) if mincurv else None
        out_mt = Outputs.alloc(B, prob.N, mo, True, zero=False, pool=abi.HOST_POOL) if mintime else None
    c_mc = out_mc.as_c() if out_mc else None
    c_mt = out_mt.as_c() if out_mt else None
    p = prob.as_c()
    if devices is None:
        _check(_lib().rl_optimize(C.byref(p), cfg_arr, ncfg, abi.u64ptr(seeds_a), B,
                                  C.byref(c_mc) if c_mc else None, C.byref(c_mt) if c_mt else None))
    else:
        devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
        _check(_lib().rl_optimize_multi(C.byref(p), cfg_arr, ncfg, abi.u64ptr(seeds_a), B,
                                        devs.ctypes.data_as(C.POINTER(C.c_int32)), len(devs),
                                        C.byref(c_mc) if c_mc else None, C.byref(c_mt) if c_mt else None))
    return out_mc, out_mt


class Plan:
    """Device-resident batch (rl_plan_*): inputs uploaded once, run() enqueues
    the optimisation on a HIP stream, fetch() copies results to the host."""

    def __init__(self, prob: Problem, cfgs, seeds=None, B: Optional[int] = None, modes: int = abi.RL_MODE_MINCURV,
                 device: int = 0):
        cfg_arr, ncfg = abi.cfg_array(cfgs)
        if B is None:
            B = ncfg if ncfg > 1 else (len(seeds) if seeds is not None else 1)
        _check_batch(B, ncfg, seeds)
        self.B, self.N, self.modes = B, prob.N, modes
        self.max_outer = int(cfg_arr[0].max_outer_iters)
        self._keep = (prob, cfg_arr)
        seeds_a = abi.seed_array(seeds)
        h = C.c_void_p()
        p = prob.as_c()
        _check(_lib().rl_plan_create(C.byref(h), device, C.byref(p), cfg_arr, ncfg, abi.u64ptr(seeds_a), B, modes))
        self._h = h

    def run(self, stream_ptr: int = 0) -> None:
        _check(_lib().rl_plan_run(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))

    @staticmethod
    def run_group(plans: Sequence["Plan"], stream_ptr: int = 0) -> None:
        """rl_plan_run_group: run the plans (one device) in as few kernel launches as their
        shapes allow -- a sweep of small plans as a few large grids -- with results equal to
        each plan's own run().  `stream_ptr` (0: the first plan's stream) waits for all."""
        if not plans or any(getattr(pl, "_h", None) is None for pl in plans):
            raise ValueError("run_group: no plans, or a closed plan")
        hs = (C.c_void_p * len(plans))(*[pl._h.value for pl in plans])
        _check(_lib().rl_plan_run_group(hs, len(plans), C.c_void_p(stream_ptr) if stream_ptr else None))

    def set_shape_batch(self, shape_B: int) -> None:
        """Choose the kernel shape for a batch of shape_B instances (0 = this plan's B):
        rl_plan_set_shape_batch.  Concurrent plans on one device pass the total in flight."""
        _check(_lib().rl_plan_set_shape_batch(self._h, int(shape_B)))

    def shape(self, mode: int) -> tuple:
        """(K, T) of the kernel rl_plan_run launches for `mode` (K = 0: streaming kernel)."""
        k, t = C.c_int32(), C.c_int32()
        _check(_lib().rl_plan_shape(self._h, int(mode), C.byref(k), C.byref(t)))
        return k.value, t.value

    def kernel_ms(self, idx: int) -> float:
        ms = C.c_float()
        _check(_lib().rl_plan_kernel_ms(self._h, idx, C.byref(ms)))
        return float(ms.value)

    def fetch(self):
        out_mc = Outputs.alloc(self.B, self.N, self.max_outer, False) if self.modes & abi.RL_MODE_MINCURV else None
        out_mt = Outputs.alloc(self.B, self.N, self.max_outer, True) if self.modes & abi.RL_MODE_MINTIME else None
        c_mc = out_mc.as_c() if out_mc else None
        c_mt = out_mt.as_c() if out_mt else None
        _check(_lib().rl_plan_fetch(self._h, C.byref(c_mc) if c_mc else None, C.byref(c_mt) if c_mt else None))
        return out_mc, out_mt

    def device_outputs(self, which: int) -> abi.RlOut:
        d = abi.RlOut()
        _check(_lib().rl_plan_device_outputs(self._h, which, C.byref(d)))
        return d

    def bind_device_outputs(self, which: int, ptrs: dict) -> None:
        """Use caller-owned device buffers (name -> device pointer int, e.g. a
        torch tensor's data_ptr()) as result storage for mode `which`."""
        d = abi.RlOut()
        for name, ptr in ptrs.items():
            typ = C.POINTER(C.c_int32) if name in ("evals", "accepts", "vpass_sweeps") else C.POINTER(C.c_double)
            setattr(d, name, C.cast(C.c_void_p(ptr), typ))
        _check(_lib().rl_plan_bind_device_outputs(self._h, which, C.byref(d)))

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib().rl_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --------------------------------------------------- reference-shaped calls
def _single(center, innerE, outerE, veh_width, L, closed, cfg, mincurv):
    cfg = cfg if cfg is not None else default_cfg()
    prob = Problem(center=center, L=L, inner_seg=innerE, outer_seg=outerE, veh_width=veh_width, closed=closed)
    if prob.N == 0:                       # ref:689 / 912: N==0 -> empty Result
        z = np.zeros(0)
        if mincurv:
            return MinCurvResult(np.zeros((0, 2)), z, z, z, z)
        return MinTimeResult(np.zeros((0, 2)), z, z, z, z, v=z, ax=z, lap_time=0.0)
    mc, mt = optimize_batch(prob, cfg, None, 1, mincurv=mincurv, mintime=not mincurv)
    o = mc if mincurv else mt
    res = dict(raceline=np.stack([o.x[0], o.y[0]], axis=1), heading=o.heading[0], curvature=o.kappa[0],
               alpha_total=o.alpha_total[0], alpha_last=o.alpha_last[0], evals=o.evals[0])
    if mincurv:
        return MinCurvResult(**res)
    return MinTimeResult(**res, v=o.v[0], ax=o.ax[0], lap_time=float(o.lap[0]), vpass_sweeps=o.vpass_sweeps[0])


def compute_min_curvature_raceline(center, innerE, outerE, veh_width: float, L: float, closed: bool,
                                   cfg: Optional[RlCfg] = None) -> MinCurvResult:
    """raceline_min_curv::compute_min_curvature_raceline (ref:683)."""
    return _single(center, innerE, outerE, veh_width, L, closed, cfg, True)


def compute_min_time_raceline(center, innerE, outerE, veh_width: float, L: float, closed: bool,
                              cfg: Optional[RlCfg] = None) -> MinTimeResult:
    """raceline_min_time::compute_min_time_raceline (ref:905)."""
    return _single(center, innerE, outerE, veh_width, L, closed, cfg, False)


# ------------------------------------------------------------- CSV writers
def _f9(x: float) -> str:
    """std::fixed + precision(9) (ref:1354)."""
    return f"{x:.9f}"


def _vkappa(kappa: float, cfg: RlCfg) -> float:
    """v_kappa column (ref:1369-1370): min(v_cap, sqrt(a_lat_max / max(|k|, kappa_eps)))."""
    k = abs(float(kappa))
    denom = cfg.kappa_eps if k < cfg.kappa_eps else k          # std::max(|k|, eps)
    v = float(np.sqrt(cfg.a_lat_max / denom))
    return cfg.v_cap_mps if v > cfg.v_cap_mps else v


def _s_rel(s0: float, L: float, k: int, n: int) -> float:
    """si - s0 with si = s0 + L*(k/max(1,n)) (ref:1367-1368), same roundings."""
    return (s0 + L * (float(k) / float(max(1, n)))) - s0


def write_raceline_csvs(base: str, res: MinCurvResult, L: float, cfg: Optional[RlCfg] = None,
                        emit_closed_duplicate: bool = True, s0: float = 0.0) -> None:
    """Writers of pipeline::compute_raceline_and_save (ref:1351-1382)."""
    cfg = cfg if cfg is not None else default_cfg()
    P = res.raceline
    with open(base + "_raceline.csv", "w") as f:
        for x, y in P:
            f.write(f"{_f9(x)},{_f9(y)}\n")
        if emit_closed_duplicate and len(P):
            f.write(f"{_f9(P[0, 0])},{_f9(P[0, 1])}\n")
    with open(base + "_raceline_with_geom.csv", "w") as f:
        f.write("s,x,y,heading_rad,curvature,alpha_last,v_kappa_mps\n")
        n = len(P)
        for k in range(n):
            s = _s_rel(s0, L, k, n)
            f.write(",".join(_f9(v) for v in (s, P[k, 0], P[k, 1], res.heading[k], res.curvature[k],
                                                 res.alpha_last[k], _vkappa(res.curvature[k], cfg))) + "\n")
        if emit_closed_duplicate and n:
            f.write(",".join(_f9(v) for v in (L, P[0, 0], P[0, 1], res.heading[0], res.curvature[0],
                                                 res.alpha_last[0], _vkappa(res.curvature[0], cfg))) + "\n")


def write_mintime_csvs(base: str, res: MinTimeResult, L: float, emit_closed_duplicate: bool = True,
                       s0: float = 0.0) -> None:
    """Writers of pipeline::compute_mintime_and_save (ref:1400-1436)."""
    P = res.raceline
    with open(base + "_mintime_raceline.csv", "w") as f:
        for x, y in P:
            f.write(f"{_f9(x)},{_f9(y)}\n")
        if emit_closed_duplicate and len(P):
            f.write(f"{_f9(P[0, 0])},{_f9(P[0, 1])}\n")
    with open(base + "_mintime_with_geom.csv", "w") as f:
        f.write("s,x,y,heading_rad,curvature,alpha_last,v_mps,ax_mps2\n")
        n = len(P)
        for k in range(n):
            s = _s_rel(s0, L, k, n)
            f.write(",".join(_f9(v) for v in (s, P[k, 0], P[k, 1], res.heading[k], res.curvature[k],
                                                 res.alpha_last[k], res.v[k], res.ax[k])) + "\n")
        if emit_closed_duplicate and n:
            f.write(",".join(_f9(v) for v in (L, P[0, 0], P[0, 1], res.heading[0], res.curvature[0],
                                                 res.alpha_last[0], res.v[0], res.ax[0])) + "\n")


def compute_raceline_and_save(base: str, center_for_opt, s0: float, L: float, closed: bool, inner_from_mids,
                              outer_from_mids, cfg: Optional[RlCfg] = None) -> MinCurvResult:
    """pipeline::compute_raceline_and_save (ref:1337-1383)."""
    cfg = cfg if cfg is not None else default_cfg()
    res = compute_min_curvature_raceline(center_for_opt, edges_for(inner_from_mids, closed),
                                         edges_for(outer_from_mids, closed), cfg.veh_width_m, L, closed, cfg)
    write_raceline_csvs(base, res, L, cfg, s0=s0)
    return res


def compute_mintime_and_save(base: str, center_for_opt, s0: float, L: float, closed: bool, inner_from_mids,
                             outer_from_mids, cfg: Optional[RlCfg] = None, debug_dump: bool = True,
                             device: int = 0) -> MinTimeResult:
    """pipeline::compute_mintime_and_save (ref:1385-1593).  debug_dump (cfg::debug_dump,
    on by default in the reference, ref:117) adds the centreline / min-curvature lap
    evaluations and <base>_debug_compare_paths.csv (debug_dump())."""
    import sys
    cfg = cfg if cfg is not None else default_cfg()
    res = compute_min_time_raceline(center_for_opt, edges_for(inner_from_mids, closed),
                                    edges_for(outer_from_mids, closed), cfg.veh_width_m, L, closed, cfg)
    write_mintime_csvs(base, res, L, s0=s0)
    sys.stderr.write(f"[mintime] Estimated laptime: {res.lap_time:.3f} s\n")
    if debug_dump:
        debug_dump_block(base, center_for_opt, s0, L, closed, res, cfg, device)
    return res


# --------------------------------------------------- lap evaluation (§8f row 2)
def lap_eval(paths, L, closed: bool, cfg: Optional[RlCfg] = None, device: int = 0, return_ms: bool = False):
    """B lap evaluations on the GPU (rl_lap_eval): heading/curvature with h = L[b]/N and
    velocity_profile_forward_backward on path b (ref:1045-1048, 1466-1478).
    paths [B, N, 2]; returns min-time Outputs (heading, kappa, v, ax, lap, sweeps)."""
    P = np.ascontiguousarray(paths, dtype=np.float64)
    if P.ndim == 2:
        P = P[None]
    B, N = P.shape[0], P.shape[1]
    Ls = np.ascontiguousarray(np.broadcast_to(np.asarray(L, dtype=np.float64), (B,)))
    cfg = cfg if cfg is not None else default_cfg()
    out = Outputs.alloc(B, N, 0, True)         # max_outer_iters = 0: vpass_sweeps [B][1]
    o = out.as_c()
    o.evals = None
    o.accepts = None
    arr, n = abi.cfg_array(cfg)
    ms = C.c_float(0.0)
    rc = _lib().rl_lap_eval(abi.dptr(P), abi.dptr(Ls), N, B, 1 if closed else 0, arr, n, int(device), C.byref(o),
                            C.byref(ms))
    _check(rc)
    out.x, out.y = P[:, :, 0].copy(), P[:, :, 1].copy()
    return (out, float(ms.value)) if return_ms else out


_LIBM = None


def _hypot(a: float, b: float) -> float:
    """glibc hypot (what std::hypot resolves to in the reference build)."""
    global _LIBM
    if _LIBM is None:
        _LIBM = C.CDLL("libm.so.6")
        _LIBM.hypot.restype = C.c_double
        _LIBM.hypot.argtypes = [C.c_double, C.c_double]
    return _LIBM.hypot(a, b)


def path_length(P, closed: bool) -> float:
    """The debug dump's path_length lambda (ref:1443-1448)."""
    P = np.asarray(P, dtype=np.float64)
    n = len(P)
    if n <= 1:
        return 0.0
    tot = 0.0
    for i in range(n - 1):
        tot += _hypot(P[i + 1, 0] - P[i, 0], P[i + 1, 1] - P[i, 1])
    if closed and n >= 2:
        tot += _hypot(P[0, 0] - P[n - 1, 0], P[0, 1] - P[n - 1, 1])
    return tot


def normals_from_points(P, closed: bool) -> np.ndarray:
    """normals_from_points_generic (ref:581-593) restated on the host."""
    P = np.asarray(P, dtype=np.float64)
    N = len(P)
    n = np.zeros((N, 2))
    for i in range(N):
        if N == 1:
            tx, ty = 1.0, 0.0
        elif closed:
            ip, im = (i + 1) % N, (i - 1 + N) % N
            tx, ty = (P[ip, 0] - P[im, 0]) * 0.5, (P[ip, 1] - P[im, 1]) * 0.5
        elif i == 0:
            tx, ty = P[1, 0] - P[0, 0], P[1, 1] - P[0, 1]
        elif i == N - 1:
            tx, ty = P[N - 1, 0] - P[N - 2, 0], P[N - 1, 1] - P[N - 2, 1]
        else:
            tx, ty = (P[i + 1, 0] - P[i - 1, 0]) * 0.5, (P[i + 1, 1] - P[i - 1, 1]) * 0.5
        if float(np.sqrt(tx * tx + ty * ty)) < 1e-15:
            tx, ty = 1.0, 0.0
        vx, vy = -ty, tx
        nn = float(np.sqrt(vx * vx + vy * vy))
        if not (nn < 1e-15):
            n[i] = (vx / nn, vy / nn)
    return n


DEBUG_HEADER = ("s,cx,cy,mt_x,mt_y,mc_x,mc_y,d_mt_signed_m,d_mc_signed_m,"
                "d_mt_abs_m,d_mc_abs_m,kappa_mt,v_mt,ax_mt,alat_mt,alat_ratio,"
                "gamma,a_acc_cap,a_brk_cap,a_power_cap\n")


def debug_compare_rows(center, s0: float, L: float, res_mt: "MinTimeResult", mc_path, cfg: RlCfg,
                       closed: bool) -> np.ndarray:
    """Rows of <base>_debug_compare_paths.csv (ref:1490-1561), same operations in the
    same order, libstdc++ min/max/clamp forms."""
    smax = lambda a, b: b if a < b else a          # noqa: E731  std::max
    smin = lambda a, b: b if b < a else a          # noqa: E731  std::min
    nan = float("nan")
    center = np.asarray(center, dtype=np.float64)
    Pmt = np.asarray(res_mt.raceline, dtype=np.float64)
    mc = np.asarray(mc_path, dtype=np.float64).reshape(-1, 2) if mc_path is not None else np.zeros((0, 2))
    nc = normals_from_points(center, closed)
    N = min(len(Pmt), len(center))
    rows = np.zeros((N, 20))
    c = cfg
    for k in range(N):
        si = s0 + L * (float(k) / float(max(1, N)))
        cx, cy = center[k]
        mx, my = Pmt[k]
        if len(mc) > k:
            ccx, ccy = mc[k]
        else:
            ccx = ccy = nan
        dmt = (mx - cx) * nc[k, 0] + (my - cy) * nc[k, 1]
        dmc = (ccx - cx) * nc[k, 0] + (ccy - cy) * nc[k, 1] if np.isfinite(ccx) else nan
        admt = abs(dmt)
        admc = abs(dmc) if np.isfinite(dmc) else nan
        kap = float(res_mt.curvature[k]) if k < len(res_mt.curvature) else 0.0
        v = float(res_mt.v[k]) if k < len(res_mt.v) else 0.0
        ax = float(res_mt.ax[k]) if k < len(res_mt.ax) else 0.0
        alat = v * v * abs(kap)
        alat_ratio = smin(1.0, alat / c.a_total_max) if c.a_total_max > 1e-9 else 0.0
        vkappa = float(np.sqrt(c.a_lat_max / smax(abs(kap), c.kappa_eps)))
        x = (vkappa - v) / smax(1e-6, vkappa)
        pen = 0.0 if x < 0 else (1.0 if x > 1 else x)
        gamma = 1.0 + c.w_time_gain * pen
        alatloc = v * v * abs(kap)
        a_res = float(np.sqrt(smax(0.0, c.a_total_max * c.a_total_max - alatloc * alatloc)))
        Fd = 0.5 * c.rho_air * c.Cd * c.A_front_m2 * v * v
        Fr = c.mass_kg * 9.81 * c.c_rr
        a_power = (c.P_max_W / (c.mass_kg * v) - (Fd + Fr) / c.mass_kg) if (c.P_max_W > 0 and v > 1e-6) else 1e9
        m3 = a_res                                     # std::min({a_res, acc_cap, a_power})
        if c.a_long_acc_cap < m3:
            m3 = c.a_long_acc_cap
        if a_power < m3:
            m3 = a_power
        a_acc = smax(0.0, m3)
        a_brk = smax(0.0, smin(a_res, c.a_long_brake_cap) + (Fd + Fr) / c.mass_kg)
        a_pow = smax(0.0, a_power)
        rows[k] = (si - s0, cx, cy, mx, my, ccx, ccy, dmt, dmc, admt, admc, kap, v, ax, alat, alat_ratio,
                   gamma, a_acc, a_brk, a_pow)
    return rows


def format_debug_compare_csv(rows: np.ndarray) -> str:
    out = [DEBUG_HEADER]
    for r in np.asarray(rows, dtype=np.float64).reshape(-1, 20):
        out.append(",".join(_f9(v) for v in r) + "\n")
    return "".join(out)


def debug_dump_block(base: str, center_for_opt, s0: float, L: float, closed: bool, res_mt: "MinTimeResult",
               cfg: RlCfg, device: int = 0, debug_offset_warn_m: float = 0.04, log=None) -> dict:
    """The cfg::debug_dump block of compute_mintime_and_save (ref:1441-1593): centreline
    and min-curvature laps with the same dynamics (two GPU lap evaluations), and
    <base>_debug_compare_paths.csv.  The min-curvature path is re-read from
    <base>_raceline.csv as the reference does (ref:1452-1459)."""
    import sys
    log = log if log is not None else sys.stderr
    center = np.asarray(center_for_opt, dtype=np.float64).reshape(-1, 2)
    mc = load_csv_xy(base + "_raceline.csv") if os.path.exists(base + "_raceline.csv") else np.zeros((0, 2))
    if len(mc) and closed and len(mc) >= 2 and abs(mc[0, 0] - mc[-1, 0]) <= 1e-12 and abs(mc[0, 1] - mc[-1, 1]) <= 1e-12:
        mc = mc[:-1]
    Nc = len(center)
    laps = {}
    if Nc:
        paths, Ls = [center], [L]
        if len(mc) == Nc:
            paths.append(mc)
            Ls.append(path_length(mc, closed))
        ev = lap_eval(np.stack(paths), np.array(Ls), closed, cfg, device)
        laps["center"] = float(ev.lap[0])
        if len(paths) == 2:
            laps["mincurv"] = float(ev.lap[1])
        elif len(mc):
            laps["mincurv"] = float(lap_eval(mc, [path_length(mc, closed)], closed, cfg, device).lap[0])
    lap_c = laps.get("center", 0.0)
    if "mincurv" in laps:
        log.write(f"[debug] centerline lap ≈ {lap_c:.3f} s,  min-curv lap ≈ {laps['mincurv']:.3f} s,  "
                  f"min-time lap ≈ {res_mt.lap_time:.3f} s\n")
    else:
        log.write(f"[debug] centerline lap ≈ {lap_c:.3f} s,  (min-curv not found),  min-time lap ≈ {res_mt.lap_time:.3f} s\n")
    rows = debug_compare_rows(center, s0, L, res_mt, mc if len(mc) else None, cfg, closed)
    with open(base + "_debug_compare_paths.csv", "w") as f:
        f.write(format_debug_compare_csv(rows))
    N = len(rows)
    admt, admc = rows[:, 9], rows[:, 10]
    stats = {"laps": laps, "mean_abs_mt": float(np.sum(admt) / max(1, N)) if N else 0.0,
             "max_abs_mt": float(np.max(admt)) if N else 0.0,
             "near_cnt": int(np.sum(admt < debug_offset_warn_m))}
    log.write(f"[debug] min-time vs center: mean|offset|={stats['mean_abs_mt']:.3f} m, "
              f"max={stats['max_abs_mt']:.3f} m, within {debug_offset_warn_m:.3f} m : {stats['near_cnt']}/{N}\n")
    if "mincurv" in laps and laps["mincurv"] > 0:
        log.write(f"[debug] lap gain vs min-curv: {(laps['mincurv'] - res_mt.lap_time) / laps['mincurv'] * 100.0:.3f} %\n")
    return stats


# ------------------------------------------------------- step 6: geometry
GEOM_HEADER = "s,x,y,heading_rad,curvature,dist_to_inner,dist_to_outer,width,v_kappa_mps\n"


def format_geom_csv(rows: np.ndarray) -> str:
    """<base>_with_geom.csv text of pipeline::compute_geom_and_save (ref:1300-1334):
    header, then every row with std::fixed / precision(9)."""
    out = [GEOM_HEADER]
    for r in np.asarray(rows, dtype=np.float64).reshape(-1, 9):
        out.append(",".join(_f9(v) for v in r) + "\n")
    return "".join(out)


def corridor(prob: Problem, cfg: Optional[RlCfg] = None, device: int = 0):
    """The optimisers' first corridor (ref:692-711) of the path prob.center on the GPU
    (rl_corridor): normals, then lo/hi per sample with guard = veh_width/2 + margin."""
    cfg = cfg if cfg is not None else default_cfg()
    N = prob.N
    lo, hi = np.zeros(max(N, 1)), np.zeros(max(N, 1))
    p = prob.as_c()
    _check(_lib().rl_corridor(C.byref(p), C.byref(cfg), int(device), abi.dptr(lo), abi.dptr(hi)))
    return lo[:N], hi[:N]


def compute_geom(gp: GeomProblem, cfg: Optional[RlCfg] = None, device: int = 0, return_ms: bool = False):
    """Rows of pipeline::compute_geom_and_save (ref:1295-1335) on the GPU (rl_geom):
    [Kmax + emit_closed_duplicate, 9] = s_rel, x, y, heading, curvature, d_in, d_out,
    width, v_kappa.  Fails loudly without a device (no CPU path)."""
    lib = _lib()
    cfg = cfg if cfg is not None else default_cfg()
    rows = np.zeros((max(gp.rows, 1), 9))
    g = gp.as_c()
    ms = C.c_float(0.0)
    n = lib.rl_geom(C.byref(g), C.byref(cfg), int(device), rows.ctypes.data_as(C.POINTER(C.c_double)),
                    C.byref(ms))
    if n < 0:
        raise RacelineError(n, lib.rl_last_error().decode())
    rows = rows[:n]
    return (rows, float(ms.value)) if return_ms else rows


def compute_geom_and_save(base: str, gp: GeomProblem, cfg: Optional[RlCfg] = None, device: int = 0) -> np.ndarray:
    """pipeline::compute_geom_and_save (ref:1288-1335): writes <base>_with_geom.csv."""
    rows = compute_geom(gp, cfg, device)
    with open(base + "_with_geom.csv", "w") as f:
        f.write(format_geom_csv(rows))
    return rows


# ------------------------------------------------- CSV number format (§8f row 3)
def format_table(table, device: int = 0, return_offsets: bool = False):
    """glibc "%.9f" CSV rows ("v,...,v\\n") of a [rows, cols] table, formatted on the GPU
    (rl_format_csv); byte-identical to the reference's std::fixed/precision(9) output."""
    T = np.ascontiguousarray(table, dtype=np.float64)
    if T.ndim == 1:
        T = T[:, None]
    rows, cols = T.shape
    cap = rows * cols * 22
    buf = C.create_string_buffer(max(cap, 1))
    n = C.c_int64(0)
    offs = np.zeros(rows + 1, dtype=np.int64)
    rc = _lib().rl_format_csv(abi.dptr(T), rows, cols, int(device), C.cast(buf, C.c_void_p), cap, C.byref(n),
                              offs.ctypes.data_as(C.POINTER(C.c_int64)))
    _check(rc)
    text = buf.raw[: n.value]
    return (text, offs) if return_offsets else text


def write_batch_raceline_with_geom(bases, mc: Outputs, L: float, cfg: Optional[RlCfg] = None, s0: float = 0.0,
                                   emit_closed_duplicate: bool = True, device: int = 0) -> None:
    """<base_b>_raceline_with_geom.csv (ref:1362-1381) for all B instances of a batch in
    one GPU formatting pass (rows split by the returned offsets)."""
    cfg = cfg if cfg is not None else default_cfg()
    B, N = mc.x.shape
    s = np.array([_s_rel(s0, L, k, N) for k in range(N)])
    vk = lambda kap: np.array([_vkappa(k, cfg) for k in kap])          # noqa: E731
    per = N + (1 if (emit_closed_duplicate and N) else 0)
    T = np.zeros((B, per, 7))
    for b in range(B):
        T[b, :N] = np.stack([s, mc.x[b], mc.y[b], mc.heading[b], mc.kappa[b], mc.alpha_last[b], vk(mc.kappa[b])], 1)
        if per > N:
            T[b, N] = (L, *T[b, 0, 1:])
    text, offs = format_table(T.reshape(B * per, 7), device, return_offsets=True)
    head = b"s,x,y,heading_rad,curvature,alpha_last,v_kappa_mps\n"
    for b, base in enumerate(bases):
        with open(base + "_raceline_with_geom.csv", "wb") as f:
            f.write(head + text[offs[b * per]: offs[(b + 1) * per]])


def load_csv_xy(path: str) -> np.ndarray:
    """io::loadCSV_XY (ref:267-279): x,y per line; ',' ';' tab or space."""
    pts = []
    with open(path) as f:
        for line in f:
            if not line.strip():
                continue
            parts = line.replace(";", " ").replace("\t", " ").replace(",", " ").split()
            if len(parts) >= 2:
                try:
                    pts.append((float(parts[0]), float(parts[1])))
                except ValueError:
                    continue
    return np.array(pts, dtype=np.float64).reshape(-1, 2)


def seeds_range(B: int, first: int = 0) -> np.ndarray:
    """Seeds first..first+B-1 (seed 0 = the reference's α≡0 start)."""
    return np.arange(first, first + B, dtype=np.uint64)


__all__ = ["RacelineError", "MinCurvResult", "MinTimeResult", "Plan", "Problem", "RlCfg", "Outputs",
           "default_cfg", "set_mu", "ring_edges", "polyline_edges", "edges_for", "optimize_batch",
           "compute_min_curvature_raceline", "compute_min_time_raceline", "compute_raceline_and_save",
           "compute_mintime_and_save", "write_raceline_csvs", "write_mintime_csvs", "load_csv_xy",
           "seeds_range"]
