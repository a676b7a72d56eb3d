/*
 * rl_abi.h — C-ABI of the MI355X batched raceline optimizer (steps 7–8 of the
 * reference pipeline).
 *
 * This is the drop-in boundary.  Each entry point replaces one reference
 * function.  "ref" means /root/reference/src/main.cpp (snapshot 2025-10-17).
 *
 *   rl_optimize / rl_plan_*   replace
 *       raceline_min_curv::compute_min_curvature_raceline   (ref:683-764)
 *       raceline_min_time::compute_min_time_raceline         (ref:905-1052)
 *     as called from pipeline::compute_raceline_and_save     (ref:1347-1348)
 *     and pipeline::compute_mintime_and_save                  (ref:1397-1398).
 *   rl_cfg                    mirrors the hot-path subset of cfg::Config (ref:47-119).
 *   rl_cfg_default            mirrors the cfg::Config default initialisers (ref:77-113).
 *   rl_ring_segments          mirrors edges::ringEdges / edges::polylineEdges (ref:251-260).
 *
 * Conventions:
 *   - Plain C types only; the caller owns every buffer; no exception crosses the ABI.
 *   - Return value 0 on success, a negative RL_E* code on failure; rl_last_error()
 *     returns a human-readable message for the calling thread.
 *   - All arithmetic is IEEE fp64.  Points are interleaved [N][2] (x,y), like the
 *     reference's vector<Vec2>.  Segments are [E][4] (x0,y0,x1,y1), like the
 *     reference's vector<pair<Vec2,Vec2>>.
 *   - Results are structure-of-arrays [B][N] (instance-major).
 *   - The compute path is the HIP/gfx950 kernel.  There is no CPU fallback:
 *     with no usable GPU every compute entry point returns RL_ENODEV.
 */
#ifndef RL_ABI_H
#define RL_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 5

/* error codes */
#define RL_OK          0
#define RL_EINVAL     -1   /* bad argument (NULL pointer, N<0, B<1, n_cfg not 1 or B, ...) */
#define RL_ENODEV     -2   /* no HIP device / device not usable                           */
#define RL_EHIP       -3   /* a HIP runtime call failed                                   */
#define RL_ENOMEM     -4   /* device or host allocation failed                            */
#define RL_ETOOBIG    -5   /* N exceeds what the selected kernel supports                 */

/* optimisation modes (bitmask for rl_plan_create) */
#define RL_MODE_MINCURV 1  /* compute_min_curvature_raceline (ref:683) */
#define RL_MODE_MINTIME 2  /* compute_min_time_raceline      (ref:905) */

/*
 * Hot-path knobs of cfg::Config (ref:47-119).  Field names and meanings are the
 * reference's.  Note the static-initialisation quirk (ref:102): a_total_max is
 * NOT derived from mu at run time; rl_cfg_set_mu() recomputes it the way a
 * recompiled reference would (mu*9.81).
 */
typedef struct rl_cfg {
    double  veh_width_m;         /* ref:77  corridor updates use this (ref:753, 1037)   */
    double  safety_margin_m;     /* ref:78                                               */
    double  lambda_smooth;       /* ref:81                                               */
    int32_t max_outer_iters;     /* ref:82                                               */
    int32_t max_inner_iters;     /* ref:83                                               */
    double  step_init;           /* ref:84                                               */
    double  step_min;            /* ref:85                                               */
    double  armijo_c;            /* ref:86                                               */
    double  kappa_eps;           /* ref:89                                               */
    double  v_cap_mps;           /* ref:90                                               */
    double  mass_kg;             /* ref:93                                               */
    double  Cd;                  /* ref:94                                               */
    double  A_front_m2;          /* ref:95                                               */
    double  rho_air;             /* ref:96                                               */
    double  c_rr;                /* ref:97                                               */
    double  P_max_W;             /* ref:98                                               */
    double  mu;                  /* ref:101 (informational: the hot path reads a_total_max) */
    double  a_total_max;         /* ref:102                                              */
    double  a_lat_max;           /* ref:103                                              */
    double  a_long_acc_cap;      /* ref:104                                              */
    double  a_long_brake_cap;    /* ref:105                                              */
    double  w_time_gain;         /* ref:108                                              */
    double  time_gamma_power;    /* ref:109                                              */
    int32_t time_weight_use_inv_v; /* ref:110 (bool)                                     */
    int32_t max_vpass_iters;     /* ref:112                                              */
    double  inv_v_gain;          /* ref:111                                              */
    int32_t use_total_ge_lat;    /* ref:113 (bool)                                       */
    int32_t _pad0;
} rl_cfg;

/*
 * One track problem: the inputs of compute_*_raceline (ref:683-686, 905-909).
 *   center_xy  [N][2]   centerline samples (closing duplicate already popped, ref:1681-1683)
 *   L                   spline arc length (ref:464); h = L/N (ref:690, 913)
 *   inner_seg  [Ei][4]  inner ring segments (ringEdges / polylineEdges of inner_from_mids)
 *   outer_seg  [Eo][4]  outer ring segments
 *   veh_width           the function argument used for the INITIAL corridor only (ref:706, 930)
 *   closed              closed-loop (periodic) operators when nonzero
 */
typedef struct rl_problem {
    const double* center_xy;
    int32_t       N;
    int32_t       closed;
    double        L;
    const double* inner_seg;
    int32_t       Ei;
    int32_t       Eo;
    const double* outer_seg;
    double        veh_width;
} rl_problem;

/*
 * Caller-allocated results, structure-of-arrays, instance-major [B][N].
 * Any pointer may be NULL to skip that output.  v / ax / lap / vpass_sweeps are
 * written for RL_MODE_MINTIME only.
 *   evals        [B][max_outer_iters]   cost/grad evaluations per outer iteration
 *                                       (the E_k of SURVEY.md §3; 0 for skipped outers)
 *   accepts      [B][max_outer_iters]   accepted PGD steps per outer iteration
 *   vpass_sweeps [B][max_outer_iters+1] v-pass sweeps actually executed per call
 *                                       (early exit once a sweep changes nothing is exact)
 */
typedef struct rl_out {
    double*  x;
    double*  y;
    double*  heading;
    double*  kappa;
    double*  alpha_total;
    double*  alpha_last;
    double*  v;
    double*  ax;
    double*  lap;
    int32_t* evals;
    int32_t* accepts;
    int32_t* vpass_sweeps;
} rl_out;

/* ---------------------------------------------------------------- config */
void rl_cfg_default(rl_cfg* cfg);
/* mu sweep helper: sets mu and a_total_max = mu*9.81 (ref:101-102) */
void rl_cfg_set_mu(rl_cfg* cfg, double mu);

/* ------------------------------------------------------------- geometry
 * Ring → segments, like edges::ringEdges (closed, ref:251-255: n segments with wrap)
 * or edges::polylineEdges (open, ref:256-260: n-1 segments).  seg_out must hold
 * [n][4] doubles.  Returns the number of segments written (>=0) or RL_EINVAL.     */
int rl_ring_segments(const double* ring_xy, int32_t n, int32_t closed, double* seg_out);

/* α-seed of instance b at sample i (build-defined):
 *   seed 0            -> 0.0 (the reference starts from α≡0, ref:720)
 *   otherwise         -> sigma * xi, xi ~ U(-1,1) from splitmix64(seed, i),
 * clamped to the initial corridor [lo_i, hi_i] by the optimizer itself.          */
double rl_seed_value(uint64_t seed, int32_t i, double sigma);
#define RL_SEED_SIGMA 0.25

/* ------------------------------------------------------------ one-shot
 * Optimise B instances of one problem.  cfg has n_cfg entries (1 = broadcast,
 * or B = one per instance).  seeds has B entries or is NULL (all zero = exactly
 * the reference).  out_mincurv / out_mintime may be NULL to skip that mode.
 * Synchronous: host buffers in, host buffers out (PCIe included), on the calling
 * thread's current HIP device.  Device plans and pinned staging buffers are reused
 * across calls from a small process-wide cache keyed by (device, N, B, n_cfg,
 * max_outer_iters, closed, kernel variant) and the ring segments (bitwise): a repeat
 * call uploads only the centreline, cfg and seeds.  rl_lap_eval shares the cache.  */
int rl_optimize(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg,
                const uint64_t* seeds, int32_t B,
                rl_out* out_mincurv, rl_out* out_mintime);
/* Timing of this thread's last successful rl_optimize / rl_lap_eval: *kernel_ms = HIP-event
 * time from the first to the last kernel of the call, *call_ms = wall time of the whole
 * call (uploads, kernels, downloads into the caller's buffers).  Either may be NULL.    */
int rl_last_call_ms(float* kernel_ms, float* call_ms);
/* The same call's times split: *run_ms = the run bracket (as rl_last_call_ms' kernel_ms:
 * first kernel start to last kernel end), *mincurv_ms / *mintime_ms = each optimiser kernel
 * alone from its own start and end events (-1 when that mode did not run), *call_ms = wall
 * time of the whole call.  Any pointer may be NULL. */
int rl_last_call_times(float* run_ms, float* mincurv_ms, float* mintime_ms, float* call_ms);
/* How the same call downloaded its results.  Calls whose results exceed 8 MiB overlap the
 * download with the kernel: every instance signals its completion into pinned host memory,
 * and each group of completed instances (16 per optimiser) is copied out while later
 * instances still compute (RL_OVERLAP_DOWNLOAD=0 in the environment turns this off).
 * *groups = the groups of the call (0: one download after the kernel), *groups_signalled =
 * those queued on their instances' flags (the rest waited for the kernel's end).  Either
 * pointer may be NULL.  (Not in the reference: the drop-in's own transfer path.) */
int rl_last_call_download(int32_t* groups, int32_t* groups_signalled);
/* Free the idle plans and pinned buffers of the cache (device memory returns to HIP). */
int rl_release_plan_cache(void);
/* Idle plans in the cache and the device / pinned host bytes they hold.  The cache keeps
 * at most 8 idle plans and RL_PLAN_CACHE_MB (environment, default 2048) MiB of device plus
 * pinned memory, evicting the least recently used; a plan larger than that on its own is
 * released when its call returns.  Any pointer may be NULL. */
int rl_plan_cache_info(int32_t* entries, int64_t* device_bytes, int64_t* pinned_bytes);

/* ------------------------------------------------------------ multi-device
 * rl_optimize over n_dev devices (SURVEY.md §8b device list, §8e): the B instances are
 * split into contiguous blocks (block d = instances [B*d/n, B*(d+1)/n), n = min(n_dev, B)),
 * one plan and HIP stream per device, all devices enqueued before the first download;
 * each block's results are copied to its offset of the caller's host outputs (the final
 * gather).  devices: n_dev device indices (a device may repeat: two plans on one device),
 * or NULL for 0..n_dev-1.  Same cfg/seeds/out conventions as rl_optimize; every cfg is
 * checked before any device work.  Every block runs the kernel shape rl_optimize picks for
 * the whole batch B (rl_plan_set_shape_batch), so on devices with the same CU count the
 * results equal rl_optimize's bit for bit, counters included (the shapes sum J and the
 * lap in different tree orders).  The calling thread's current device is unchanged on
 * return. */
int rl_optimize_multi(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg,
                      const uint64_t* seeds, int32_t B, const int32_t* devices, int32_t n_dev,
                      rl_out* out_mincurv, rl_out* out_mintime);

/* ---------------------------------------------------- device-resident plan
 * For repeated runs with inputs already resident in HBM (bench, services).
 * create: allocates device buffers on `device` and uploads the inputs.
 * run:    enqueues the optimisation on `hip_stream` (a hipStream_t; NULL = the
 *         plan's own stream) and returns immediately.  With both modes and a batch
 *         that leaves the GPU partly idle (B x waves per instance <= 8 x CUs), the
 *         min-time kernel runs on a second plan-owned stream, concurrently with the
 *         min-curvature kernel; `hip_stream` waits for both.
 * fetch:  copies results to host (synchronises the stream used by run).
 * device_outputs: device pointers of the result arrays (for collectives).       */
typedef struct rl_plan rl_plan;

int rl_plan_create(rl_plan** plan, int32_t device, const rl_problem* prob,
                   const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds,
                   int32_t B, int32_t modes);
int rl_plan_run(rl_plan* plan, void* hip_stream);
/* rl_plan_run of n plans of one device in as few launches as their kernel shapes allow (a
 * sweep of many small plans: C4's 14 (track, mode) plans of 512 one-wave instances).  Every
 * (plan, mode) whose shape is a one-wave throughput shape ((4|5|8, 64): N <= 512 in a batch
 * that fills the GPU) joins one launch with the other plans of its mode, K and closed flag
 * (up to 8 plans per launch), the instances of all of them in one grid; other
 * plans run as rl_plan_run.  The launches run concurrently on plan-owned streams, after
 * everything queued on `hip_stream` (NULL: the first plan's stream), which waits for all of
 * them.  Results equal each plan's own rl_plan_run bit for bit.  A plan may appear once. */
int rl_plan_run_group(rl_plan* const* plans, int32_t n, void* hip_stream);
int rl_plan_fetch(rl_plan* plan, rl_out* out_mincurv, rl_out* out_mintime);
/* which: RL_MODE_MINCURV or RL_MODE_MINTIME; fills device pointers (same layout as
 * rl_out, NULL where the mode does not produce the field). */
int rl_plan_device_outputs(rl_plan* plan, int32_t which, rl_out* dev_out);
/* Bind caller-owned DEVICE buffers (same layout as rl_out: [B][N] arrays, lap [B],
 * evals/accepts [B][max_outer_iters], vpass_sweeps [B][max_outer_iters+1]) as the
 * result storage of mode `which`; NULL fields keep the plan's own buffers.  Lets a
 * framework (e.g. torch tensors for an RCCL gather) receive results without copies. */
int rl_plan_bind_device_outputs(rl_plan* plan, int32_t which, const rl_out* dev_out);
/* device time of the last run, in ms, measured with HIP events on the run stream:
 * idx 0 = the whole run, 1 = the min-curvature kernel, 2 = the min-time kernel. */
int rl_plan_kernel_ms(rl_plan* plan, int32_t idx, float* ms);
/* The batch size the plan's kernel shape is chosen for (rl_kernel_shape's B); 0 = the plan's
 * own B (the default).  Shapes differ in the tree order of the J / decrease / lap sums, so
 * the last bits of J and the lap (and on a near-tie an Armijo decision) can depend on the
 * shape: plans that must give identical results take the same shape batch.  Plans that run
 * concurrently on one device should pass the total instance count in flight, so that none
 * takes a latency shape meant to spread its instances over the whole GPU.  Takes effect
 * at the next rl_plan_run. */
int rl_plan_set_shape_batch(rl_plan* plan, int32_t shape_B);
/* The kernel shape rl_plan_run launches for `mode` (K = 0: the streaming kernel). */
int rl_plan_shape(rl_plan* plan, int32_t mode, int32_t* K, int32_t* T);
int rl_plan_destroy(rl_plan* plan);

/* B lap evaluations of given paths: heading/curvature
 * (heading_curv_from_points_generic, ref:595-620) and velocity_profile_forward_backward
 * (ref:782-862) with h = L[b]/N on path b — the min-time driver's final step
 * (ref:1045-1048) and the debug dump's centreline / min-curvature laps (ref:1466-1478),
 * i.e. compute_min_time_raceline with max_outer_iters = 0.  paths_xy [B][N][2], L [B];
 * `out` receives heading, kappa, v, ax, lap and vpass_sweeps [B][1] (x, y echo the path,
 * alphas are 0); evals/accepts may be NULL.  cfg[n_cfg] as in rl_optimize.
 * *kernel_ms (optional): HIP-event time of the kernel. */
int rl_lap_eval(const double* paths_xy, const double* L, int32_t N, int32_t B, int32_t closed,
                const rl_cfg* cfg, int32_t n_cfg, int32_t device, rl_out* out, float* kernel_ms);

/* ------------------------------------------------------- step 6: geometry
 * pipeline::compute_geom_and_save (ref:1295-1335), the rows of <base>_with_geom.csv:
 * the centreline spline evaluated at s_k = s0 + L*(k/denomN), heading, curvature,
 * ray distances to the rings along ±n (distancesToRings, ref:513-524), width and
 * v_kappa.  SURVEY §8f row 1. */

/* centerline::Spline1D (ref:403-446): knots s[n], coefficients a,b,c,d [n] */
typedef struct rl_spline {
    const double* s;
    const double* a;
    const double* b;
    const double* c;
    const double* d;
    int32_t n;
    int32_t _pad;
} rl_spline;

typedef struct rl_geom_problem {
    rl_spline spx, spy;          /* x(s), y(s) from splineUniformResample (ref:448-474)      */
    double s0, L;                /* resample origin and length (ref:465)                      */
    int32_t Kmax;                /* rows before the duplicate: closed ? samples : Ncenter (ref:1308) */
    int32_t denomN;              /* closed ? samples : max(1, samples) (ref:1309)             */
    int32_t emit_closed_duplicate; /* cfg emit_closed_duplicate: one more row (L, row 0) (ref:1331) */
    int32_t closed;              /* ring segments are ringEdges (1) / polylineEdges (0) inputs */
    const double* inner_seg;     /* [Ei][4] */
    const double* outer_seg;     /* [Eo][4] */
    int32_t Ei, Eo;
} rl_geom_problem;

#define RL_GEOM_COLS 9           /* s_rel,x,y,heading_rad,curvature,dist_to_inner,dist_to_outer,width,v_kappa_mps */

/* Rows (Kmax + emit_closed_duplicate) x RL_GEOM_COLS into host `rows` (row-major),
 * computed on `device`.  cfg supplies kappa_eps, a_lat_max, v_cap_mps.  *kernel_ms
 * (optional) receives the HIP-event time of the geometry kernel.  Returns the row
 * count or RL_E*. */
int rl_geom(const rl_geom_problem* gp, const rl_cfg* cfg, int32_t device, double* rows, float* kernel_ms);

/* ------------------------------------------------------ CSV number format
 * SURVEY §8f row 3.  The reference writes every CSV with std::fixed + precision(9)
 * (ref:1284, 1303, 1354, 1418, 1495), i.e. glibc "%.9f": exact value rounded to 9
 * fraction digits with ties to even, "-" whenever the sign bit is set, "nan"/"-nan",
 * "inf"/"-inf".  rl_format_csv formats a row-major table [rows][cols] on the GPU into
 * `out` as "v,v,...,v\n" rows (no header).  *out_len receives the byte count (also when
 * out_cap is too small: then RL_ETOOBIG); row_offsets [rows+1] (optional) the start of
 * every row.  Values with |x| >= 9.2e9 are rejected (RL_ETOOBIG). */
int rl_format_csv(const double* table, int64_t rows, int32_t cols, int32_t device, char* out, int64_t out_cap,
                  int64_t* out_len, int64_t* row_offsets);

/* ------------------------------------------------------------ corridor
 * The optimisers' first corridor (ref:692-711) for the path prob->center_xy:
 * normals_from_points_generic (ref:581-593), then per sample
 *   hi = max(0, dpos - guard), lo = -max(0, dneg - guard),
 *   guard = prob->veh_width*0.5 + cfg->safety_margin_m,
 * dpos / dneg the safe_ray distances (ref:694-699) along +n / -n to the nearer ring.
 * The same device code as the optimiser's corridor passes (rl_corridor.h), run in
 * the optimiser's scan mapping.  lo, hi: [N] host buffers.  Returns RL_OK or RL_E*. */
int rl_corridor(const rl_problem* prob, const rl_cfg* cfg, int32_t device, double* lo, double* hi);

/* ------------------------------------------------------------- runtime */
int         rl_device_count(void);
const char* rl_last_error(void);
int         rl_abi_version(void);
/* samples per lane of the THROUGHPUT shape for N (4: N <= 256, 5: N <= 320, 8: N <= 4096;
 * 1 = the streaming kernel), or RL_ETOOBIG.  Batches small enough for a latency shape launch fewer samples per lane:
 * rl_kernel_shape(N, B, mode) reports the shape a launch actually uses. */
int         rl_kernel_variant(int32_t N);
/* the kernel shape of a launch: *K samples per lane (0 = the streaming kernel) and *T lanes
 * per instance for N samples, a batch of B and mode RL_MODE_MINCURV or RL_MODE_MINTIME on
 * the calling thread's current device.  Batches that need at most one wave per SIMD in a
 * latency shape (one instance spread over a CU, 1-4 samples per lane) get it; larger ones
 * the throughput shapes (4-8 samples per lane).  RL_LAT_SHAPES=0 in the environment keeps
 * the throughput shapes for every batch.  Returns RL_OK or RL_E*. */
int         rl_kernel_shape(int32_t N, int32_t B, int32_t mode, int32_t* K, int32_t* T);

#ifdef __cplusplus
}
#endif
#endif /* RL_ABI_H */
