"""Build the native pieces in-tree (they travel to the GPU box with the snapshot).

  _lib/librl.so          HIP kernels for gfx950 + the C-ABI (include/rl_abi.h)
  _lib/fsd_raceline      single-file C++17 host CLI (host/raceline.cpp) over the C-ABI
  oracle/liboracle.so    CPU checker (test infrastructure, see oracle/)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_DIR = os.path.join(PKG, "_lib")
INCLUDE = os.path.join(REPO, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

KERNEL_SRCS = ["csrc/rl_kernels.hip", "csrc/rl_kernels_group.hip", "csrc/rl_kernels_lat.hip", "csrc/rl_kernels_mid.hip", "csrc/rl_stream.hip", "csrc/rl_geom.hip", "csrc/rl_format.hip", "csrc/rl_abi.cpp"]
KERNEL_DEPS = KERNEL_SRCS + ["csrc/rl_optimize_body.h", "csrc/rl_optimize_body.inc", "csrc/rl_kernels.h", "csrc/rl_device.h", "csrc/rl_math.h", "csrc/rl_corridor.h"]
# -ffp-contract=off: HIP defaults to fusing a*b+c into FMA, which would change
# the reference's roundings.
HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
             "-I" + INCLUDE, "-Wno-unused-command-line-argument"]
# per-source extra flags of the product build: the latency shapes run one wave per SIMD,
# where nothing hides a dependent instruction's latency but the wave's own independent
# instructions, so their translation units use LLVM's ILP-oriented schedulers (A/B,
# B=1 training_map min-curv 1.43 -> 1.31 ms, C3-shaped min-time 4.73 -> 4.31
# ms); the throughput kernels were slower under max-ilp and gain ~0.2-2 % from the
# iterative occupancy scheduler; the streaming kernel keeps the default
# RL_PRIO=3 (rl_kernels.h progress_prio): the throughput shapes, two or more instances per
# CU, raise the priority of the instance that is behind (C2 8.35 -> 8.03 -> 7.96 ms, C4's
# one-wave shape -8..-10 %, profiles/r06/ab_prio.log, ab_prio3.log); the latency shapes hold
# one instance per CU
TU_FLAGS = {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc", "-DRL_PRIO=3"],
            "csrc/rl_kernels_group.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc", "-DRL_PRIO=3"],
            "csrc/rl_kernels_lat.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp", "-DRL_BODY_CALL=0"],
            "csrc/rl_kernels_mid.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp", "-DRL_BODY_CALL=0"]}


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(os.path.join(PKG, d) if not os.path.isabs(d) else d) > t for d in deps)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd)}")
    return r.stdout


def build_lib(force: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    out = os.path.join(LIB_DIR, "librl.so")
    deps = KERNEL_DEPS + [os.path.join(INCLUDE, "rl_abi.h")]
    if force or _stale(out, deps):
        _compile_link(KERNEL_SRCS, [], out, os.path.join(LIB_DIR, "obj"))
    return out


def _compile_link(srcs, flags, out, objdir, tu_flags=None) -> None:
    """One hipcc process per translation unit (in parallel), then one link: the
    kernel file alone takes ~100 s, so the others compile beside it.  tu_flags:
    extra flags per source (TU_FLAGS by default)."""
    tu_flags = TU_FLAGS if tu_flags is None else tu_flags
    from concurrent.futures import ThreadPoolExecutor

    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    with ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        for f in [ex.submit(_run, [HIPCC, *HIP_FLAGS, *flags, *tu_flags.get(s, []), "-c", s, "-o", o], PKG)
                  for s, o in zip(srcs, objs)]:
            f.result()
    tmp = out + ".tmp"
    _run([HIPCC, *HIP_FLAGS, "-shared", *objs, "-o", tmp], cwd=PKG)
    os.replace(tmp, out)


def build_variant(name: str, defines: dict) -> str:
    """Experiment build: _lib/variants/librl_<name>.so with -D overrides (A/B timing only);
    a "_tu" entry maps sources to their extra flags (replacing those sources' TU_FLAGS)."""
    defines = dict(defines)
    tu = {**TU_FLAGS, **defines.pop("_tu", {})}
    vdir = os.path.join(LIB_DIR, "variants")
    os.makedirs(vdir, exist_ok=True)
    out = os.path.join(vdir, f"librl_{name}.so")
    flags = [f"-D{k}={v}" for k, v in defines.items()]
    _compile_link(KERNEL_SRCS, flags, out, os.path.join(vdir, "obj_" + name), tu)
    return out


def build_host(force: bool = False) -> str:
    """host/raceline.cpp -> _lib/fsd_raceline, linked against librl.so (rpath $ORIGIN)."""
    lib = build_lib(force)
    out = os.path.join(LIB_DIR, "fsd_raceline")
    src = os.path.join(PKG, "host", "raceline.cpp")
    if not os.path.exists(src):
        return ""
    if force or _stale(out, [src, lib, os.path.join(INCLUDE, "rl_abi.h")]):
        cxx = shutil.which("g++") or "c++"
        _run([cxx, "-std=c++17", "-O2", "-ffp-contract=off", "-I" + INCLUDE, src, "-o", out,
              "-L" + LIB_DIR, "-lrl", "-Wl,-rpath,$ORIGIN"], cwd=PKG)
    return out


def build_oracle() -> str:
    _run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle.so"])
    return os.path.join(REPO, "oracle", "liboracle.so")


def build_ref_oracle() -> str:
    """oracle/_ref: the reference compiled from /root/reference where it lies (build container only)."""
    if not os.path.exists("/root/reference/src/main.cpp"):
        return ""
    _run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    return os.path.join(REPO, "oracle", "_ref", "libref_harness.so")


def build_all(force: bool = False) -> None:
    build_lib(force)
    build_host(force)
    build_oracle()
    build_ref_oracle()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", os.listdir(LIB_DIR))
