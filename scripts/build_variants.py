"""Build A/B variant libraries into _lib/variants/ (experiments only)."""
import os, sys
from concurrent.futures import ThreadPoolExecutor
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from practice_path_planning_for_formula_student_driverless_amd import build as B
VARIANTS = {
    "base": {},
    "k4t512w2": {"RL_MID_K": 4, "RL_MID_T": 512, "RL_MID_W": 2},
    "k4t512w4": {"RL_MID_K": 4, "RL_MID_T": 512, "RL_MID_W": 4},
    "ck4": {"RL_CK": 4},
    "mt_k8t256": {"RL_MIDMT_K": 8, "RL_MIDMT_T": 256},
    "old_w": {"RL_SMALLMT_W": 4, "RL_SMALL_W": 4, "RL_S8MT_W": 2},   # before the per-mode occupancy A/B
    "smc_w4": {"RL_SMALL_W": 4},
    "smc_w3": {"RL_SMALL_W": 3},
    "smt_w3": {"RL_SMALLMT_W": 3},
    "s8mt_w2": {"RL_S8MT_W": 2},
    "bt1": {"RL_BT_BATCH": 1},
    "bt6": {"RL_BT_BATCH": 6},
    "bt8": {"RL_BT_BATCH": 8},
    "sck1": {"RL_SCK": 1},
    "sck4": {"RL_SCK": 4},
    "sts512": {"RL_STS": 512},
    "sts256": {"RL_STS": 256},
    "ck4tight": {"RL_CK": 4, "RL_MD_TIGHT": 1},
    "ck1": {"RL_CK": 1},
    "a12_0": {"RL_A12_REG": 0},
    "a12_1": {"RL_A12_REG": 1},
    "a12_2": {"RL_A12_REG": 2},
    "a12mt1": {"RL_A12_MT": 1},
    "a12mt2": {"RL_A12_MT": 2},
    "a12mt3": {"RL_A12_MT": 3},
    "blk8": {"RL_BLKSZ": 8},
    "blk32": {"RL_BLKSZ": 32},
    "nofuse": {"RL_SFUSE": 0},
    "svp0": {"RL_SVP_REG": 0},
    "lat_k2": {"RL_LAT1_K": 2, "RL_LAT2_K": 4, "RL_LAT3_K": 4},   # (2,128) / (4,128) / (4,256) latency shapes
    "lat1k2": {"RL_LAT1_K": 2},          # (2,128) for N <= 256 (ghost samples at K = 2)
    "lat2k1": {"RL_LAT2_K": 1},          # (1,512) for 256 < N <= 512 (8 waves, one sample per lane)
    "probe_nob1": {"RL_PROBE_NOB1": 1},
    "probe_nozb": {"RL_PROBE_NOZB": 1},
    "zbghost0": {"RL_ZB_GHOST": 0},      # the ghost samples' clamps always in the select forms  # timing probe: every projection clamp as maxNum/minNum (zero signs may differ)
    "ghost0": {"RL_GHOST": 0},
    "along": {"RL_ALONG": 1},            # along-ray corridor block culling (rl_corridor.h)
    "spec0": {"RL_SPEC_GRAD": 0},        # latency shapes without the speculative gradient
    "vfast0": {"RL_VSTEP_FAST": 0},      # v-pass steps with the select forms of max(0, .) / min
    "latfit0": {"RL_LAT_FIT": 0},
    "sts512": {"RL_STS": 512, "RL_STS_MINW": 4},   # streaming kernel: two 512-thread instances per CU
    "sts256": {"RL_STS": 256, "RL_STS_MINW": 4},   # four 256-thread instances per CU        # the (1, 256) / (1, 512) latency table instead of K = 1 on just enough waves
    # scheduler A/B (build.py TU_FLAGS holds the product's choice; "_tu" overrides per source)
    "lat_default": {"_tu": {"csrc/rl_kernels_lat.hip": []}},
    "mid_default": {"_tu": {"csrc/rl_kernels_mid.hip": []}},
    "mid_ilp": {"_tu": {"csrc/rl_kernels_mid.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}},
    "lat_iilp": {"_tu": {"csrc/rl_kernels_lat.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}},
    "thr_ilp": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}},
    "thr_minreg": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]}},
    "thr_memclause": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]}},
    "thr_default": {"_tu": {"csrc/rl_kernels.hip": []}},
    "thr_bias0": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc", "-mllvm", "-amdgpu-schedule-metric-bias=0"]}},
    "thr_trackers": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc", "-mllvm", "-amdgpu-use-amdgpu-trackers"]}},
    "thr_def_bias0": {"_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-schedule-metric-bias=0"]}},
    "stream_bias0": {"_tu": {"csrc/rl_stream.hip": ["-mllvm", "-amdgpu-schedule-metric-bias=0"]}},
    "stream_maxocc": {"_tu": {"csrc/rl_stream.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"]}},
    # (iterative-ilp on rl_kernels.hip crashes this LLVM's register allocator on <8,256,closed,mintime>)
    "stream_iilp": {"_tu": {"csrc/rl_stream.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]}},
    "btfmt": {"RL_BT_FIRST_MT": 1, "RL_BT_ADAPT": 0},
    "btfixed": {"RL_BT_ADAPT": 0},
    "prio": {"RL_PRIO": 1},              # wave priority falling with the outer iteration (tail balance)
    "prio2": {"RL_PRIO": 2},             # the same with two levels
    "prio3": {"RL_PRIO": 3, "_tu": {"csrc/rl_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"],
                                    "csrc/rl_kernels_group.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"]}},   # end-weighted levels
    "prio_s": {"RL_PRIO": 1, "RL_SPRIO": 1},   # and in the streaming kernel
    "stamps": {"RL_STAMPS": 1},          # diagnostic (scripts/stamps.py); not A/B-timed
    "stamps_eval": {"RL_STAMPS": 1, "RL_STAMPS_EVAL": 1},   # + the latency evaluation's phases (scripts/stamps_lat.py)
    "count": {"RL_COUNT": 1},            # diagnostic (scripts/counts_c5.py); not A/B-timed
}
if __name__ == "__main__":
    names = sys.argv[1:] or [n for n in VARIANTS if n not in ("stamps", "count")]
    import shutil; shutil.rmtree(os.path.join(B.LIB_DIR, "variants"), ignore_errors=True)
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(lambda n: B.build_variant(n, VARIANTS[n]), names):
            print("built", p)
