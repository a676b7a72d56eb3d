"""ctypes mirror of ``include/rl_abi.h`` (the C-ABI drop-in boundary).

The structs here are byte-for-byte the C structs of ``rl_abi.h``; the loader
binds ``librl.so`` (HIP kernels for gfx950 + the C-ABI).  There is no CPU
fallback: if the library is missing, :func:`load_library` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref
from dataclasses import dataclass, fields
from typing import Optional

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "_lib", "librl.so")
# experiment builds only (scripts/build_variants.py): RL_LIB names another librl.so to load
if os.environ.get("RL_LIB"):
    LIB_PATH = os.path.abspath(os.environ["RL_LIB"])

RL_OK = 0
RL_EINVAL = -1
RL_ENODEV = -2
RL_EHIP = -3
RL_ENOMEM = -4
RL_ETOOBIG = -5

RL_MODE_MINCURV = 1
RL_MODE_MINTIME = 2
RL_SEED_SIGMA = 0.25


class RlCfg(C.Structure):
    """``rl_cfg`` — hot-path subset of ``cfg::Config`` (main.cpp:47-119)."""

    _fields_ = [
        ("veh_width_m", C.c_double),
        ("safety_margin_m", C.c_double),
        ("lambda_smooth", C.c_double),
        ("max_outer_iters", C.c_int32),
        ("max_inner_iters", C.c_int32),
        ("step_init", C.c_double),
        ("step_min", C.c_double),
        ("armijo_c", C.c_double),
        ("kappa_eps", C.c_double),
        ("v_cap_mps", C.c_double),
        ("mass_kg", C.c_double),
        ("Cd", C.c_double),
        ("A_front_m2", C.c_double),
        ("rho_air", C.c_double),
        ("c_rr", C.c_double),
        ("P_max_W", C.c_double),
        ("mu", C.c_double),
        ("a_total_max", C.c_double),
        ("a_lat_max", C.c_double),
        ("a_long_acc_cap", C.c_double),
        ("a_long_brake_cap", C.c_double),
        ("w_time_gain", C.c_double),
        ("time_gamma_power", C.c_double),
        ("time_weight_use_inv_v", C.c_int32),
        ("max_vpass_iters", C.c_int32),
        ("inv_v_gain", C.c_double),
        ("use_total_ge_lat", C.c_int32),
        ("_pad0", C.c_int32),
    ]

    def to_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_ if not n.startswith("_")}

    @classmethod
    def from_dict(cls, d: dict) -> "RlCfg":
        c = cls()
        for n, t in cls._fields_:
            if n in d:
                setattr(c, n, d[n])
        return c


class RlProblem(C.Structure):
    _fields_ = [
        ("center_xy", C.POINTER(C.c_double)),
        ("N", C.c_int32),
        ("closed", C.c_int32),
        ("L", C.c_double),
        ("inner_seg", C.POINTER(C.c_double)),
        ("Ei", C.c_int32),
        ("Eo", C.c_int32),
        ("outer_seg", C.POINTER(C.c_double)),
        ("veh_width", C.c_double),
    ]


class RlOut(C.Structure):
    _fields_ = [
        ("x", C.POINTER(C.c_double)),
        ("y", C.POINTER(C.c_double)),
        ("heading", C.POINTER(C.c_double)),
        ("kappa", C.POINTER(C.c_double)),
        ("alpha_total", C.POINTER(C.c_double)),
        ("alpha_last", C.POINTER(C.c_double)),
        ("v", C.POINTER(C.c_double)),
        ("ax", C.POINTER(C.c_double)),
        ("lap", C.POINTER(C.c_double)),
        ("evals", C.POINTER(C.c_int32)),
        ("accepts", C.POINTER(C.c_int32)),
        ("vpass_sweeps", C.POINTER(C.c_int32)),
    ]


OUT_F64 = ("x", "y", "heading", "kappa", "alpha_total", "alpha_last")
OUT_F64_MT = OUT_F64 + ("v", "ax")


def default_cfg() -> RlCfg:
    """cfg::Config defaults (main.cpp:77-113), computed in Python so the
    product path needs no oracle.  a_total_max = mu*9.81 (main.cpp:102)."""
    c = RlCfg()
    c.veh_width_m = 1.0
    c.safety_margin_m = 0.05
    c.lambda_smooth = 1.6e-3
    c.max_outer_iters = 14
    c.max_inner_iters = 120
    c.step_init = 0.65
    c.step_min = 1e-6
    c.armijo_c = 1e-5
    c.kappa_eps = 1e-6
    c.v_cap_mps = 27.0
    c.mass_kg = 255.0
    c.Cd = 0.30
    c.A_front_m2 = 1.00
    c.rho_air = 1.225
    c.c_rr = 0.015
    c.P_max_W = 80000.0
    c.mu = 1.17
    c.a_total_max = 1.17 * 9.81
    c.a_lat_max = 11.0
    c.a_long_acc_cap = 8.0
    c.a_long_brake_cap = 11.0
    c.w_time_gain = 1.0
    c.time_gamma_power = 2.0
    c.time_weight_use_inv_v = 0
    c.inv_v_gain = 0.1
    c.max_vpass_iters = 6
    c.use_total_ge_lat = 1
    return c


def set_mu(c: RlCfg, mu: float) -> None:
    """Sweep helper: a recompiled reference would evaluate a_total_max=mu*9.81 (main.cpp:102)."""
    c.mu = mu
    c.a_total_max = mu * 9.81


def dptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_double))


def iptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_int32))


@dataclass
class Problem:
    """Inputs of compute_*_raceline (main.cpp:683-686): centerline [N,2], L,
    ring segments [E,4], veh_width (initial corridor only), closed."""

    center: np.ndarray
    L: float
    inner_seg: np.ndarray
    outer_seg: np.ndarray
    veh_width: float = 1.0
    closed: bool = True

    def __post_init__(self):
        self.center = np.ascontiguousarray(self.center, dtype=np.float64).reshape(-1, 2)
        self.inner_seg = np.ascontiguousarray(self.inner_seg, dtype=np.float64).reshape(-1, 4)
        self.outer_seg = np.ascontiguousarray(self.outer_seg, dtype=np.float64).reshape(-1, 4)

    @property
    def N(self) -> int:
        return int(self.center.shape[0])

    def as_c(self) -> RlProblem:
        p = RlProblem()
        p.center_xy = dptr(self.center)
        p.N = self.N
        p.closed = 1 if self.closed else 0
        p.L = float(self.L)
        p.inner_seg = dptr(self.inner_seg)
        p.Ei = int(self.inner_seg.shape[0])
        p.outer_seg = dptr(self.outer_seg)
        p.Eo = int(self.outer_seg.shape[0])
        p.veh_width = float(self.veh_width)
        return p


class HostPool:
    """Recycling allocator for the host result arrays of ``optimize_batch``.

    A caller of the drop-in that takes fresh arrays from every call and drops them after
    use makes the OS fault in ~100 MB of new pages per C2-sized call and unmap the old
    ones, and the next call's kernel runs slower behind that churn.  Arrays
    from this pool are views of a buffer the pool keeps mapped: when the last view of an
    array dies, its buffer returns to the pool (``weakref.finalize`` on the ctypes object
    the views are built on) and the next request of the same byte size gets it back, pages
    already resident.  An array is handed out again only after every view of it is gone, so
    results a caller keeps are never overwritten.  At most ``cap_bytes`` of free buffers
    are kept (``RL_HOST_POOL_MB``, default 1024; 0 disables the pool): a returned buffer
    that does not fit evicts the oldest free ones.  Arrays under ``min_bytes`` (256 KiB:
    malloc serves them from its heap, without mapping) are plain numpy arrays."""

    def __init__(self, cap_bytes: int, min_bytes: int = 1 << 18):
        self.cap = int(cap_bytes)
        self.min_bytes = int(min_bytes)
        self._free: list = []          # free uint8 buffers, oldest first
        self._free_bytes = 0
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0

    def _release(self, buf: np.ndarray) -> None:
        # (a finalizer can run inside empty()'s locked region on this thread: never block)
        if buf.nbytes > self.cap or not self._lock.acquire(blocking=False):
            return
        try:
            while self._free and self._free_bytes + buf.nbytes > self.cap:
                self._free_bytes -= self._free.pop(0).nbytes
            self._free.append(buf)
            self._free_bytes += buf.nbytes
        finally:
            self._lock.release()

    def empty(self, shape, dtype) -> np.ndarray:
        """An uninitialised C-contiguous array, from a recycled buffer when one fits."""
        dt = np.dtype(dtype)
        nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
        if nbytes < self.min_bytes or nbytes > self.cap:
            return np.empty(shape, dtype=dt)
        buf = None
        with self._lock:
            for i in range(len(self._free) - 1, -1, -1):     # the most recently returned first
                if self._free[i].nbytes == nbytes:
                    buf = self._free.pop(i)
                    self._free_bytes -= nbytes
                    break
        if buf is None:
            self.misses += 1
            buf = np.empty(nbytes, dtype=np.uint8)
        else:
            self.hits += 1
        owner = (C.c_char * nbytes).from_buffer(buf)
        weakref.finalize(owner, self._release, buf).atexit = False
        return np.frombuffer(owner, dtype=dt).reshape(shape)

    def free_bytes(self) -> int:
        return self._free_bytes

    def clear(self) -> None:
        with self._lock:
            self._free.clear()
            self._free_bytes = 0


HOST_POOL = HostPool(int(float(os.environ.get("RL_HOST_POOL_MB", "1024")) * (1 << 20)))


@dataclass
class Outputs:
    """Host-side SoA result buffers [B][N] for one mode."""

    x: np.ndarray
    y: np.ndarray
    heading: np.ndarray
    kappa: np.ndarray
    alpha_total: np.ndarray
    alpha_last: np.ndarray
    evals: np.ndarray
    accepts: np.ndarray
    v: Optional[np.ndarray] = None
    ax: Optional[np.ndarray] = None
    lap: Optional[np.ndarray] = None
    vpass_sweeps: Optional[np.ndarray] = None

    @classmethod
    def alloc(cls, B: int, N: int, max_outer: int, mintime: bool, zero: bool = True,
              pool: Optional[HostPool] = None) -> "Outputs":
        """Result arrays of one mode; zero=False leaves them uninitialised (np.empty, or
        recycled buffers of ``pool``), for a call that writes every element (rl_optimize:
        every column, counter and lap)."""
        if zero:
            mk = np.zeros
        elif pool is not None:
            mk = pool.empty
        else:
            mk = np.empty
        z = lambda: mk((B, N), dtype=np.float64)  # noqa: E731
        o = cls(x=z(), y=z(), heading=z(), kappa=z(), alpha_total=z(), alpha_last=z(),
                evals=mk((B, max_outer), dtype=np.int32),
                accepts=mk((B, max_outer), dtype=np.int32))
        if mintime:
            o.v = z()
            o.ax = z()
            o.lap = mk(B, dtype=np.float64)
            o.vpass_sweeps = mk((B, max_outer + 1), dtype=np.int32)
        return o

    def as_c(self) -> RlOut:
        o = RlOut()
        for n in ("x", "y", "heading", "kappa", "alpha_total", "alpha_last", "v", "ax", "lap"):
            setattr(o, n, dptr(getattr(self, n)))
        o.evals = iptr(self.evals)
        o.accepts = iptr(self.accepts)
        o.vpass_sweeps = iptr(self.vpass_sweeps)
        return o


class RlSpline(C.Structure):
    """centerline::Spline1D (ref:403-446)."""
    _fields_ = [("s", C.POINTER(C.c_double)), ("a", C.POINTER(C.c_double)), ("b", C.POINTER(C.c_double)),
                ("c", C.POINTER(C.c_double)), ("d", C.POINTER(C.c_double)), ("n", C.c_int32), ("_pad", C.c_int32)]


class RlGeomProblem(C.Structure):
    """Inputs of pipeline::compute_geom_and_save (ref:1288-1335)."""
    _fields_ = [("spx", RlSpline), ("spy", RlSpline), ("s0", C.c_double), ("L", C.c_double),
                ("Kmax", C.c_int32), ("denomN", C.c_int32), ("emit_closed_duplicate", C.c_int32),
                ("closed", C.c_int32), ("inner_seg", C.POINTER(C.c_double)), ("outer_seg", C.POINTER(C.c_double)),
                ("Ei", C.c_int32), ("Eo", C.c_int32)]


RL_GEOM_COLS = 9
GEOM_COLS = ("s", "x", "y", "heading_rad", "curvature", "dist_to_inner", "dist_to_outer", "width", "v_kappa_mps")


@dataclass
class GeomProblem:
    """Step 6 inputs: the x(s), y(s) splines as knots [10][n] (x: s,a,b,c,d then y:
    s,a,b,c,d), s0, L, Kmax, denomN (ref:1308-1309), ring segments [E,4]."""

    knots: np.ndarray
    s0: float
    L: float
    Kmax: int
    denomN: int
    inner_seg: np.ndarray
    outer_seg: np.ndarray
    closed: bool = True
    emit_closed_duplicate: bool = True

    def __post_init__(self):
        self.knots = np.ascontiguousarray(self.knots, dtype=np.float64).reshape(10, -1)
        self.inner_seg = np.ascontiguousarray(self.inner_seg, dtype=np.float64).reshape(-1, 4)
        self.outer_seg = np.ascontiguousarray(self.outer_seg, dtype=np.float64).reshape(-1, 4)

    @property
    def rows(self) -> int:
        return int(self.Kmax) + (1 if self.emit_closed_duplicate else 0)

    def as_c(self) -> RlGeomProblem:
        g = RlGeomProblem()
        n = self.knots.shape[1]
        for sp, off in ((g.spx, 0), (g.spy, 5)):
            sp.s, sp.a, sp.b, sp.c, sp.d = (dptr(self.knots[off + j]) for j in range(5))
            sp.n = n
        g.s0, g.L = float(self.s0), float(self.L)
        g.Kmax, g.denomN = int(self.Kmax), int(self.denomN)
        g.emit_closed_duplicate = 1 if self.emit_closed_duplicate else 0
        g.closed = 1 if self.closed else 0
        g.inner_seg, g.outer_seg = dptr(self.inner_seg), dptr(self.outer_seg)
        g.Ei, g.Eo = self.inner_seg.shape[0], self.outer_seg.shape[0]
        return g


def cfg_array(cfgs) -> tuple:
    """list of RlCfg (or one) -> (ctypes array, n)."""
    if isinstance(cfgs, RlCfg):
        cfgs = [cfgs]
    arr = (RlCfg * len(cfgs))(*cfgs)
    return arr, len(cfgs)


def seed_array(seeds) -> Optional[np.ndarray]:
    if seeds is None:
        return None
    return np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64))


def u64ptr(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def declare_optimize(fn) -> None:
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(RlProblem), C.POINTER(RlCfg), C.c_int32, C.POINTER(C.c_uint64),
                   C.c_int32, C.POINTER(RlOut), C.POINTER(RlOut)]


_LIB = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load librl.so (the HIP path).  Raises if it is missing: there is no fallback."""
    global _LIB
    if _LIB is not None and path == LIB_PATH:
        return _LIB
    if not os.path.exists(path):
        raise RuntimeError(f"librl.so not built at {path}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = C.CDLL(path)
    declare_optimize(lib.rl_optimize)
    lib.rl_cfg_default.argtypes = [C.POINTER(RlCfg)]
    lib.rl_cfg_default.restype = None
    lib.rl_cfg_set_mu.argtypes = [C.POINTER(RlCfg), C.c_double]
    lib.rl_cfg_set_mu.restype = None
    lib.rl_ring_segments.argtypes = [C.POINTER(C.c_double), C.c_int32, C.c_int32, C.POINTER(C.c_double)]
    lib.rl_ring_segments.restype = C.c_int
    lib.rl_seed_value.argtypes = [C.c_uint64, C.c_int32, C.c_double]
    lib.rl_seed_value.restype = C.c_double
    lib.rl_plan_create.argtypes = [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(RlProblem), C.POINTER(RlCfg),
                                   C.c_int32, C.POINTER(C.c_uint64), C.c_int32, C.c_int32]
    lib.rl_plan_create.restype = C.c_int
    lib.rl_plan_run.argtypes = [C.c_void_p, C.c_void_p]
    lib.rl_plan_run.restype = C.c_int
    if path == LIB_PATH or hasattr(lib, "rl_plan_run_group"):   # (A/B builds of older sources lack it)
        lib.rl_plan_run_group.argtypes = [C.POINTER(C.c_void_p), C.c_int32, C.c_void_p]
        lib.rl_plan_run_group.restype = C.c_int
    lib.rl_plan_fetch.argtypes = [C.c_void_p, C.POINTER(RlOut), C.POINTER(RlOut)]
    lib.rl_plan_fetch.restype = C.c_int
    lib.rl_plan_device_outputs.argtypes = [C.c_void_p, C.c_int32, C.POINTER(RlOut)]
    lib.rl_plan_device_outputs.restype = C.c_int
    lib.rl_plan_bind_device_outputs.argtypes = [C.c_void_p, C.c_int32, C.POINTER(RlOut)]
    lib.rl_plan_bind_device_outputs.restype = C.c_int
    lib.rl_plan_kernel_ms.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_float)]
    lib.rl_plan_kernel_ms.restype = C.c_int
    lib.rl_plan_destroy.argtypes = [C.c_void_p]
    lib.rl_plan_destroy.restype = C.c_int
    if hasattr(lib, "rl_plan_set_shape_batch"):   # absent only in older experiment builds (A/B bases)
        lib.rl_plan_set_shape_batch.argtypes = [C.c_void_p, C.c_int32]
        lib.rl_plan_set_shape_batch.restype = C.c_int
        lib.rl_plan_shape.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.rl_plan_shape.restype = C.c_int
    lib.rl_device_count.restype = C.c_int
    lib.rl_last_error.restype = C.c_char_p
    lib.rl_abi_version.restype = C.c_int
    lib.rl_kernel_variant.argtypes = [C.c_int32]
    lib.rl_kernel_variant.restype = C.c_int
    if hasattr(lib, "rl_kernel_shape"):     # absent only in older experiment builds (A/B bases)
        lib.rl_kernel_shape.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.rl_kernel_shape.restype = C.c_int
    lib.rl_geom.argtypes = [C.POINTER(RlGeomProblem), C.POINTER(RlCfg), C.c_int32, C.POINTER(C.c_double),
                            C.POINTER(C.c_float)]
    lib.rl_geom.restype = C.c_int
    if hasattr(lib, "rl_corridor"):      # absent only in older experiment builds (A/B bases)
        lib.rl_corridor.argtypes = [C.POINTER(RlProblem), C.POINTER(RlCfg), C.c_int32, C.POINTER(C.c_double),
                                    C.POINTER(C.c_double)]
        lib.rl_corridor.restype = C.c_int
    lib.rl_lap_eval.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int32, C.c_int32, C.c_int32,
                                C.POINTER(RlCfg), C.c_int32, C.c_int32, C.POINTER(RlOut), C.POINTER(C.c_float)]
    lib.rl_lap_eval.restype = C.c_int
    lib.rl_format_csv.argtypes = [C.POINTER(C.c_double), C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_int64,
                                  C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.rl_format_csv.restype = C.c_int
    if hasattr(lib, "rl_optimize_multi"):   # absent only in older experiment builds (A/B bases)
        lib.rl_optimize_multi.argtypes = [C.POINTER(RlProblem), C.POINTER(RlCfg), C.c_int32, C.POINTER(C.c_uint64),
                                          C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(RlOut),
                                          C.POINTER(RlOut)]
        lib.rl_optimize_multi.restype = C.c_int
    if hasattr(lib, "rl_last_call_ms"):     # absent only in older experiment builds (A/B bases)
        lib.rl_last_call_ms.argtypes = [C.POINTER(C.c_float), C.POINTER(C.c_float)]
        lib.rl_last_call_ms.restype = C.c_int
        lib.rl_release_plan_cache.argtypes = []
        lib.rl_release_plan_cache.restype = C.c_int
    if hasattr(lib, "rl_last_call_times"):  # absent only in older experiment builds (A/B bases)
        lib.rl_last_call_times.argtypes = [C.POINTER(C.c_float)] * 4
        lib.rl_last_call_times.restype = C.c_int
        lib.rl_plan_cache_info.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        lib.rl_plan_cache_info.restype = C.c_int
    if hasattr(lib, "rl_last_call_download"):   # absent only in older experiment builds (A/B bases)
        lib.rl_last_call_download.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.rl_last_call_download.restype = C.c_int
    if path == LIB_PATH:
        _LIB = lib
    return lib


def kernel_shape(N: int, B: int, mode: int) -> tuple:
    """(K samples per lane, T lanes per instance) librl.so launches for (N, B, mode)."""
    lib = load_library()
    k, t = C.c_int32(), C.c_int32()
    rc = lib.rl_kernel_shape(int(N), int(B), int(mode), C.byref(k), C.byref(t))
    if rc != RL_OK:
        raise RuntimeError(f"rl_kernel_shape({N}, {B}, {mode}) = {rc}")
    return k.value, t.value


def cfg_field_names() -> list:
    return [n for n, _ in RlCfg._fields_ if not n.startswith("_")]


__all__ = [n for n in dir() if not n.startswith("_") and n not in ("C", "os", "np", "fields", "dataclass", "Optional")]
