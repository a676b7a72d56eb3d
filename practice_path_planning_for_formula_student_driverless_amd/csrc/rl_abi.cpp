// rl_abi.cpp — C-ABI implementation (include/rl_abi.h): argument checks, device
// buffers, one HIP stream per plan, HIP-event timing.  The compute path is the
// gfx950 kernel in rl_kernels.hip; there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>
#include <unistd.h>

#include "rl_abi.h"
#include "rl_device.h"
#include "rl_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t _e = (expr);                                                       \
        if (_e != hipSuccess) return fail(RL_EHIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

// std::max (ref:506 uses std::max(1e-30, ...))
inline double smax_h(double a, double b) { return (a < b) ? b : a; }

// Segment record from (x0,y0,x1,y1); vx,vy,denom exactly as the reference computes
// them (ref:482, 505-506).  mx,my,hr for conservative culling.
rl::SegRec make_segrec(const double* q) {
    rl::SegRec r;
    r.x0 = q[0];
    r.y0 = q[1];
    r.vx = q[2] - q[0];
    r.vy = q[3] - q[1];
    r.denom = smax_h(1e-30, r.vx * r.vx + r.vy * r.vy);
    r.mx = 0.5 * (q[0] + q[2]);
    r.my = 0.5 * (q[1] + q[3]);
    r.hr = 0.5 * std::sqrt(r.vx * r.vx + r.vy * r.vy) * (1.0 + 1e-9) + 1e-12;
    return r;
}

// Host image of one ring in the entry-stream form of rl_corridor.h: the vertices of
// each chain of consecutive segments (a segment starts a new chain unless its start
// equals the previous segment's end bit for bit), entry v holding the record of the
// segment that ends at v; padded to blocks of 32 with NaN entries.
struct RingHost {
    std::vector<double> vtx;        // [M][2]
    std::vector<rl::SegRec> rec;    // [M]
    std::vector<uint32_t> flag;     // [M/32]
    std::vector<double> blk;        // [M/B][4] block circles (rl_corridor.h block culling)
    int M = 0, E = 0;
    double dl0 = 0, dl32 = 0;
};

RingHost make_ring(const double* s, int E) {
    RingHost R;
    R.E = E;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    rl::SegRec dummy;
    dummy.x0 = dummy.y0 = dummy.vx = dummy.vy = dummy.mx = dummy.my = dummy.hr = nan;
    dummy.denom = 1.0;
    std::vector<char> ends;
    auto push = [&](double x, double y, const rl::SegRec& r, bool end) {
        R.vtx.push_back(x);
        R.vtx.push_back(y);
        R.rec.push_back(r);
        ends.push_back(end);
    };
    double vmax = 0, rv = 0;
    bool nonfinite = false;        // std::max below drops a NaN second argument: tracked here
    for (int e = 0; e < E; ++e) {
        const double* q = s + 4 * e;
        for (int j = 0; j < 4; ++j) nonfinite |= !std::isfinite(q[j]);
        if (e == 0 || !(q[0] == s[4 * e - 2] && q[1] == s[4 * e - 1])) push(q[0], q[1], dummy, false);
        const rl::SegRec r = make_segrec(q);
        push(q[2], q[3], r, true);
        vmax = std::max(vmax, std::fabs(r.vx) + std::fabs(r.vy));
        rv = std::max(rv, std::max(std::fabs(q[0]) + std::fabs(q[1]), std::fabs(q[2]) + std::fabs(q[3])));
    }
    while (ends.size() % 32) push(nan, nan, dummy, false);
    R.M = (int)ends.size();
    R.flag.assign(R.M / 32, 0u);
    for (int v = 0; v < R.M; ++v)
        if (ends[v]) R.flag[v / 32] |= 0x80000000u >> (v % 32);
    // A NaN/inf coordinate anywhere makes dl0/dl32 NaN: every pair of the ring is then a
    // candidate (rl_corridor.h `bad`) and the exact expressions propagate the values like
    // the reference
    R.dl0 = 4e-12 * (1.0 + vmax) + 4e-15 * rv;
    R.dl32 = 1e-6 * rv;
    if (nonfinite || !(vmax == vmax) || !(rv == rv)) R.dl0 = R.dl32 = nan;
    if (!(rv <= 1e30)) R.dl32 = INFINITY;          // beyond fp32 range: the fp32 filter keeps every pair
    // Per block of RL_BLK entries: a circle holding both endpoints of every segment that
    // ends in the block (the start point of the segment ending at v is entry v-1's
    // vertex, bit for bit). R = -1: no segment ends there; R = +inf: a non-finite
    // coordinate, so the block is never skipped.
    const int nb = R.M / rl::RL_BLK;
    R.blk.assign((size_t)4 * nb, 0.0);
    for (int b = 0; b < nb; ++b) {
        double px[2 * rl::RL_BLK], py[2 * rl::RL_BLK];
        int n = 0;
        for (int v = b * rl::RL_BLK; v < (b + 1) * rl::RL_BLK; ++v) {
            if (!ends[v]) continue;
            px[n] = R.rec[v].x0; py[n++] = R.rec[v].y0;
            px[n] = R.vtx[2 * v]; py[n++] = R.vtx[2 * v + 1];
        }
        double* o = &R.blk[(size_t)4 * b];
        if (n == 0) { o[2] = -1.0; continue; }
        bool finite = true;
        double x0 = px[0], x1 = px[0], y0 = py[0], y1 = py[0];
        for (int j = 0; j < n; ++j) {
            finite = finite && std::isfinite(px[j]) && std::isfinite(py[j]);
            x0 = std::min(x0, px[j]); x1 = std::max(x1, px[j]);
            y0 = std::min(y0, py[j]); y1 = std::max(y1, py[j]);
        }
        const double cx = 0.5 * (x0 + x1), cy = 0.5 * (y0 + y1);
        double rad = 0.0;
        for (int j = 0; j < n; ++j) rad = std::max(rad, std::hypot(px[j] - cx, py[j] - cy));
        o[0] = cx;
        o[1] = cy;
        o[2] = finite ? rad * (1.0 + 1e-9) + 1e-12 * (1.0 + std::fabs(cx) + std::fabs(cy)) : INFINITY;
    }
    // fp32 copies for the side filter (rl_corridor.h ring_rays): vertices, then block
    // circles with the radius rounded up; packed after the fp64 circles
    std::vector<float> f32((size_t)2 * R.M + (size_t)4 * nb + (size_t)4 * R.M, 0.0f);
    for (int v = 0; v < 2 * R.M; ++v) f32[v] = (float)R.vtx[v];
    for (int b = 0; b < nb; ++b) {
        float* o = &f32[(size_t)2 * R.M + (size_t)4 * b];
        o[0] = (float)R.blk[(size_t)4 * b];
        o[1] = (float)R.blk[(size_t)4 * b + 1];
        const double rb = R.blk[(size_t)4 * b + 2];
        float rf = (float)rb;
        if ((double)rf < rb) rf = std::nextafter(rf, INFINITY);
        o[2] = rf;
    }
    for (int v = 0; v < R.M; ++v) {     // segment midpoints and half lengths (rounded up)
        float* o = &f32[(size_t)2 * R.M + (size_t)4 * nb + (size_t)4 * v];
        o[0] = (float)R.rec[v].mx;
        o[1] = (float)R.rec[v].my;
        const double hr = R.rec[v].hr;
        float hf = (float)hr;
        if ((double)hf < hr) hf = std::nextafter(hf, INFINITY);
        o[2] = hf;
    }
    const size_t n64 = R.blk.size();
    R.blk.resize(rl::ring_blk_doubles((size_t)R.M), 0.0);
    std::memcpy(&R.blk[n64], f32.data(), f32.size() * sizeof(float));
    return R;
}

struct ModeBufs {
    double *x = nullptr, *y = nullptr, *heading = nullptr, *kappa = nullptr, *alpha_total = nullptr,
           *alpha_last = nullptr, *v = nullptr, *ax = nullptr, *lap = nullptr, *nx = nullptr, *ny = nullptr;
    int32_t *evals = nullptr, *accepts = nullptr, *sweeps = nullptr;
    rl::StreamBufs sb{};      // large-N variant only
};

// variant: register-resident (N <= 4096) unless N is larger or RL_FORCE_STREAM=1 (testing)
bool use_stream(int N) {
    if (N > rl::RL_REG_MAX_N) return true;
    const char* f = std::getenv("RL_FORCE_STREAM");
    return f && f[0] == '1';
}

int device_cus(int dev) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return 256;
    return n;
}
// waves of one instance in the kernel launch_optimize / launch_stream picks for (N, B, mode)
int waves_per_instance(int N, int B, bool mintime, bool stream, int cus) {
    if (stream) return (rl::stream_threads() + 63) / 64;      // rl_stream.hip
    const rl::Shape s = rl::pick_shape(N, B, mintime, cus);
    if (s.K <= 0) return 16;
    return (s.T + 63) / 64;
}

}  // namespace

struct rl_plan {
    int device = 0;
    int N = 0, B = 0, modes = 0, ncfg = 0, max_outer = 0, closed = 1, Ei = 0, Eo = 0;
    // batch size the kernel shape is chosen for (rl_plan_set_shape_batch; 0 = B): the
    // shapes sum J and the lap in different orders, so plans whose results must equal
    // each other's bit for bit use the same one (rl_optimize_multi: the whole call's B)
    int shape_B = 0;
    bool stream = false;              // streaming kernel (use_stream at creation)
    double L = 0, veh_width = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t last_stream = nullptr;
    // both modes in one run: the min-time kernel runs on aux_stream, concurrently with the
    // min-curvature kernel (the optimisers are independent); the run stream waits for it
    hipStream_t aux_stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // run start, mode starts, run end
    hipEvent_t ev_end[2] = {nullptr, nullptr};                 // mode ends
    bool ran = false;
    double* d_center = nullptr;
    double* d_Ls = nullptr;           // per-instance L (lap evaluation) or nullptr
    int64_t center_stride = 0;        // doubles between instances' centres (0: shared)
    double* d_vtx = nullptr;
    rl::SegRec* d_rec = nullptr;
    uint32_t* d_flag = nullptr;
    double* d_blk = nullptr;
    int ring_M[2] = {0, 0};
    double ring_dl0[2] = {0, 0}, ring_dl32[2] = {0, 0};
    rl_cfg* d_cfg = nullptr;
    uint64_t* d_seeds = nullptr;
    ModeBufs mb[2];
    // per-mode instance completion flags of the next run (run_cached's overlapped
    // download; nullptr: none) and the value the kernel stores into them
    uint32_t* done[2] = {nullptr, nullptr};
    uint32_t epoch = 0;
    // outer iteration 0's corridor, cast once per run for the whole batch (KParams::lo0/hi0):
    // its bounds, the cfg margin all instances share (margin_uniform), and the event the
    // concurrent min-time stream waits for
    double *d_lo0 = nullptr, *d_hi0 = nullptr;
    double margin0 = 0;
    bool margin_uniform = false;
    hipEvent_t ev_c = nullptr;
    std::vector<void*> allocs;

    template <class T>
    int alloc(T** p, size_t n) {
        if (n == 0) n = 1;
        hipError_t e = hipMalloc((void**)p, n * sizeof(T));
        if (e != hipSuccess) return fail(RL_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        allocs.push_back((void*)*p);
        dev_bytes += n * sizeof(T);
        return RL_OK;
    }
    size_t dev_bytes = 0;             // device memory held (plan cache budget)
};

namespace {
int run_cached(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds, int32_t B,
               int32_t modes, const double* centers, const double* Ls, rl_out* out_mc, rl_out* out_mt, float* kms);
}  // namespace

extern "C" {

const char* rl_last_error(void) { return g_err.c_str(); }
int rl_abi_version(void) { return RL_ABI_VERSION; }

int rl_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// samples per lane of the register-resident kernel (4 or 8), 1 for the streaming
// kernel, RL_ETOOBIG beyond it
int rl_kernel_variant(int32_t N) {
    if (N > rl::RL_STREAM_MAX_N) return RL_ETOOBIG;
    if (use_stream(N)) return 1;
    int k = rl::pick_k(N);
    return k < 0 ? RL_ETOOBIG : k;
}

// cfg::Config defaults, ref:77-113
// (K, T) the library launches for N samples, a batch of B and `mode` (one of
// RL_MODE_MINCURV / RL_MODE_MINTIME) on the calling thread's current device
int rl_kernel_shape(int32_t N, int32_t B, int32_t mode, int32_t* K, int32_t* T) {
    if (!K || !T || B < 1 || (mode != RL_MODE_MINCURV && mode != RL_MODE_MINTIME))
        return fail(RL_EINVAL, "rl_kernel_shape: bad argument");
    if (N < 1 || N > rl::RL_STREAM_MAX_N) return fail(RL_ETOOBIG, "rl_kernel_shape: N out of range");
    if (use_stream(N)) { *K = 0; *T = rl::stream_threads(); return RL_OK; }   // streaming kernel (samples strided)
    int dev = 0;
    const int cus = (hipGetDevice(&dev) == hipSuccess) ? device_cus(dev) : 256;
    const rl::Shape s = rl::pick_shape(N, B, mode == RL_MODE_MINTIME, cus);
    *K = s.K;
    *T = s.T;
    return RL_OK;
}

void rl_cfg_default(rl_cfg* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->veh_width_m = 1.0;
    c->safety_margin_m = 0.05;
    c->lambda_smooth = 1.6e-3;
    c->max_outer_iters = 14;
    c->max_inner_iters = 120;
    c->step_init = 0.65;
    c->step_min = 1e-6;
    c->armijo_c = 1e-5;
    c->kappa_eps = 1e-6;
    c->v_cap_mps = 27.0;
    c->mass_kg = 255.0;
    c->Cd = 0.30;
    c->A_front_m2 = 1.00;
    c->rho_air = 1.225;
    c->c_rr = 0.015;
    c->P_max_W = 80000.0;
    c->mu = 1.17;
    c->a_total_max = c->mu * 9.81;   // ref:102 (evaluated once)
    c->a_lat_max = 11.0;
    c->a_long_acc_cap = 8.0;
    c->a_long_brake_cap = 11.0;
    c->w_time_gain = 1.0;
    c->time_gamma_power = 2.0;
    c->time_weight_use_inv_v = 0;
    c->inv_v_gain = 0.1;
    c->max_vpass_iters = 6;
    c->use_total_ge_lat = 1;
}

void rl_cfg_set_mu(rl_cfg* c, double mu) {
    if (!c) return;
    c->mu = mu;
    c->a_total_max = mu * 9.81;
}

// edges::ringEdges ref:251-255 / edges::polylineEdges ref:256-260
int rl_ring_segments(const double* ring_xy, int32_t n, int32_t closed, double* seg_out) {
    if (n < 0 || (n > 0 && (!ring_xy || !seg_out))) return fail(RL_EINVAL, "rl_ring_segments: bad argument");
    if (closed) {
        for (int i = 0; i < n; ++i) {
            int j = (i + 1) % n;
            seg_out[4 * i] = ring_xy[2 * i];
            seg_out[4 * i + 1] = ring_xy[2 * i + 1];
            seg_out[4 * i + 2] = ring_xy[2 * j];
            seg_out[4 * i + 3] = ring_xy[2 * j + 1];
        }
        return n;
    }
    if (n < 2) return 0;
    for (int i = 0; i + 1 < n; ++i) {
        seg_out[4 * i] = ring_xy[2 * i];
        seg_out[4 * i + 1] = ring_xy[2 * i + 1];
        seg_out[4 * i + 2] = ring_xy[2 * i + 2];
        seg_out[4 * i + 3] = ring_xy[2 * i + 3];
    }
    return n - 1;
}

double rl_seed_value(uint64_t seed, int32_t i, double sigma) { return rl::seed_value(seed, i, sigma); }

int rl_plan_set_shape_batch(rl_plan* plan, int32_t shape_B) {
    if (!plan || shape_B < 0) return fail(RL_EINVAL, "rl_plan_set_shape_batch: bad argument");
    plan->shape_B = shape_B;
    return RL_OK;
}

int rl_plan_shape(rl_plan* plan, int32_t mode, int32_t* K, int32_t* T) {
    if (!plan || !K || !T || (mode != RL_MODE_MINCURV && mode != RL_MODE_MINTIME))
        return fail(RL_EINVAL, "rl_plan_shape: bad argument");
    if (plan->stream) { *K = 0; *T = rl::stream_threads(); return RL_OK; }
    const rl::Shape s = rl::pick_shape(std::max(plan->N, 1), plan->shape_B > 0 ? plan->shape_B : plan->B,
                                       mode == RL_MODE_MINTIME, device_cus(plan->device));
    *K = s.K;
    *T = s.T;
    return RL_OK;
}

int rl_plan_destroy(rl_plan* plan) {
    if (!plan) return RL_OK;
    hipSetDevice(plan->device);
    // every stream that may still run a kernel of this plan drains before its buffers go:
    // a run that failed after queueing the min-time kernel on aux_stream, but before the
    // run stream waited for it, leaves that kernel reading and writing them
    if (plan->last_stream) hipStreamSynchronize(plan->last_stream);
    if (plan->aux_stream) hipStreamSynchronize(plan->aux_stream);
    if (plan->own_stream) hipStreamSynchronize(plan->own_stream);
    for (void* p : plan->allocs) hipFree(p);
    for (auto& e : plan->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : plan->ev_end)
        if (e) hipEventDestroy(e);
    if (plan->ev_c) hipEventDestroy(plan->ev_c);
    if (plan->own_stream) hipStreamDestroy(plan->own_stream);
    if (plan->aux_stream) hipStreamDestroy(plan->aux_stream);
    delete plan;
    return RL_OK;
}

// rl_plan_create with optional per-instance centres [B][N][2] and lengths [B]
// (centers/Ls non-NULL: prob->center_xy and prob->L are ignored)
static int plan_create_ex(rl_plan** out, int32_t device, const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg,
                          const uint64_t* seeds, int32_t B, int32_t modes, const double* centers, const double* Ls);

int rl_plan_create(rl_plan** out, int32_t device, const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg,
                   const uint64_t* seeds, int32_t B, int32_t modes) {
    return plan_create_ex(out, device, prob, cfg, n_cfg, seeds, B, modes, nullptr, nullptr);
}

static int alloc_mode(rl_plan* p, int m);

// the cfg margin of outer iteration 0's guard, if every instance has the same one (bitwise)
static void set_margin(rl_plan* p, const rl_cfg* cfg, int n_cfg) {
    p->margin0 = cfg[0].safety_margin_m;
    p->margin_uniform = true;
    for (int c = 1; c < n_cfg; ++c)
        if (std::memcmp(&cfg[c].safety_margin_m, &p->margin0, sizeof(double)) != 0) p->margin_uniform = false;
}

// argument checks shared by every entry point that builds or reuses a plan (no device call)
static int check_inputs(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg, int32_t B, int32_t modes,
                        const double* centers) {
    if (!prob || !cfg) return fail(RL_EINVAL, "problem/cfg is NULL");
    if (B < 1) return fail(RL_EINVAL, "B must be >= 1");
    if (n_cfg != 1 && n_cfg != B) return fail(RL_EINVAL, "n_cfg must be 1 or B");
    if (prob->N < 0) return fail(RL_EINVAL, "N < 0");
    if ((modes & (RL_MODE_MINCURV | RL_MODE_MINTIME)) == 0 || (modes & ~3)) return fail(RL_EINVAL, "bad modes");
    // any L is accepted like the reference (h = L/N, ref:690); only the pointer is checked
    if (prob->N > 0 && !prob->center_xy && !centers) return fail(RL_EINVAL, "center_xy is NULL");
    if (prob->Ei < 0 || prob->Eo < 0 || (prob->Ei > 0 && !prob->inner_seg) || (prob->Eo > 0 && !prob->outer_seg))
        return fail(RL_EINVAL, "bad segments");
    const int mo = cfg[0].max_outer_iters;
    for (int c = 0; c < n_cfg; ++c) {
        if (cfg[c].max_outer_iters != mo) return fail(RL_EINVAL, "max_outer_iters must be equal across cfgs");
        if (cfg[c].max_outer_iters < 0 || cfg[c].max_inner_iters < 0 || cfg[c].max_vpass_iters < 0)
            return fail(RL_EINVAL, "negative iteration count");
    }
    if (prob->N > rl::RL_STREAM_MAX_N) return fail(RL_ETOOBIG, "N exceeds the streaming kernel (N <= 1048576)");
    return RL_OK;
}

static int plan_create_ex(rl_plan** out, int32_t device, const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg,
                          const uint64_t* seeds, int32_t B, int32_t modes, const double* centers, const double* Ls) {
    if (!out) return fail(RL_EINVAL, "plan out pointer is NULL");
    *out = nullptr;
    if (int rc0 = check_inputs(prob, cfg, n_cfg, B, modes, centers)) return rc0;
    const int mo = cfg[0].max_outer_iters;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RL_ENODEV, "device index out of range");
    HIPCHK(hipSetDevice(device));

    rl_plan* p = new rl_plan();
    p->device = device;
    p->N = prob->N;
    p->B = B;
    p->modes = modes;
    p->ncfg = n_cfg;
    p->max_outer = mo;
    p->closed = prob->closed ? 1 : 0;
    p->L = prob->L;
    p->veh_width = prob->veh_width;
    p->Ei = prob->Ei;
    p->Eo = prob->Eo;
    p->stream = use_stream(p->N);
    int rc = RL_OK;
    auto cleanup = [&](int code) {
        rl_plan_destroy(p);
        return code;
    };
    if (hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&p->aux_stream, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(RL_EHIP, "hipStreamCreate failed"));
    for (auto& e : p->ev)
        if (hipEventCreate(&e) != hipSuccess) return cleanup(fail(RL_EHIP, "hipEventCreate failed"));
    for (auto& e : p->ev_end)
        if (hipEventCreate(&e) != hipSuccess) return cleanup(fail(RL_EHIP, "hipEventCreate failed"));
    if (hipEventCreateWithFlags(&p->ev_c, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(RL_EHIP, "hipEventCreate failed"));
    set_margin(p, cfg, n_cfg);

    const size_t N = (size_t)std::max(p->N, 1);
    RingHost rh[2] = {make_ring(prob->inner_seg, prob->Ei), make_ring(prob->outer_seg, prob->Eo)};
    const size_t Mt = (size_t)rh[0].M + rh[1].M;
    for (int r = 0; r < 2; ++r) { p->ring_M[r] = rh[r].M; p->ring_dl0[r] = rh[r].dl0; p->ring_dl32[r] = rh[r].dl32; }
    p->center_stride = centers ? (int64_t)2 * (int64_t)N : 0;
    if (Ls && (rc = p->alloc(&p->d_Ls, (size_t)B))) return cleanup(rc);
    if ((rc = p->alloc(&p->d_center, centers ? 2 * N * (size_t)B : 2 * N)) || (rc = p->alloc(&p->d_vtx, 2 * Mt)) ||
        (rc = p->alloc(&p->d_rec, Mt)) || (rc = p->alloc(&p->d_flag, Mt / 32)) ||
        (rc = p->alloc(&p->d_blk, rl::ring_blk_doubles(Mt))) || (rc = p->alloc(&p->d_cfg, (size_t)n_cfg)) || (rc = p->alloc(&p->d_seeds, (size_t)B)) ||
        (rc = p->alloc(&p->d_lo0, N)) || (rc = p->alloc(&p->d_hi0, N)))
        return cleanup(rc);
    hipStream_t st = p->own_stream;
    if (p->N > 0 && hipMemcpyAsync(p->d_center, centers ? centers : prob->center_xy,
                                   (centers ? (size_t)B : 1) * 2 * N * sizeof(double), hipMemcpyHostToDevice, st))
        return cleanup(fail(RL_EHIP, "upload center"));
    if (Ls && hipMemcpyAsync(p->d_Ls, Ls, (size_t)B * sizeof(double), hipMemcpyHostToDevice, st))
        return cleanup(fail(RL_EHIP, "upload L"));
    for (int r = 0, off = 0; r < 2; off += rh[r].M, ++r) {
        const RingHost& R = rh[r];
        if (R.M == 0) continue;
        if (hipMemcpyAsync(p->d_vtx + 2 * (size_t)off, R.vtx.data(), R.vtx.size() * sizeof(double), hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_rec + off, R.rec.data(), R.rec.size() * sizeof(rl::SegRec), hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_flag + off / 32, R.flag.data(), R.flag.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_blk + rl::ring_blk_doubles((size_t)off), R.blk.data(), R.blk.size() * sizeof(double),
                           hipMemcpyHostToDevice, st))
            return cleanup(fail(RL_EHIP, "upload rings"));
        // the copies read the host vectors: wait before they go out of scope
        if (hipStreamSynchronize(st) != hipSuccess) return cleanup(fail(RL_EHIP, "upload sync"));
    }
    if (hipMemcpyAsync(p->d_cfg, cfg, (size_t)n_cfg * sizeof(rl_cfg), hipMemcpyHostToDevice, st))
        return cleanup(fail(RL_EHIP, "upload cfg"));
    std::vector<uint64_t> sd((size_t)B, 0);
    if (seeds) std::memcpy(sd.data(), seeds, (size_t)B * sizeof(uint64_t));
    if (hipMemcpyAsync(p->d_seeds, sd.data(), (size_t)B * sizeof(uint64_t), hipMemcpyHostToDevice, st))
        return cleanup(fail(RL_EHIP, "upload seeds"));
    for (int m = 0; m < 2; ++m)
        if ((modes & (1 << m)) && (rc = alloc_mode(p, m))) return cleanup(rc);
    if (hipStreamSynchronize(st) != hipSuccess) return cleanup(fail(RL_EHIP, "upload sync"));
    *out = p;
    return RL_OK;
}

// result and scratch buffers of mode m (0: min-curv, 1: min-time); a no-op if present
static int alloc_mode(rl_plan* p, int m) {
    ModeBufs& mb = p->mb[m];
    if (mb.nx) return RL_OK;
    const size_t BN = (size_t)p->B * (size_t)std::max(p->N, 1);
    const int mo = p->max_outer, B = p->B;
    int rc;
    if ((rc = p->alloc(&mb.x, BN)) || (rc = p->alloc(&mb.y, BN)) || (rc = p->alloc(&mb.heading, BN)) ||
        (rc = p->alloc(&mb.kappa, BN)) || (rc = p->alloc(&mb.alpha_total, BN)) ||
        (rc = p->alloc(&mb.alpha_last, BN)) || (rc = p->alloc(&mb.nx, BN)) || (rc = p->alloc(&mb.ny, BN)) ||
        (rc = p->alloc(&mb.evals, (size_t)B * std::max(mo, 1))) ||
        (rc = p->alloc(&mb.accepts, (size_t)B * std::max(mo, 1))))
        return rc;
    if (m == 1) {
        if ((rc = p->alloc(&mb.v, BN)) || (rc = p->alloc(&mb.ax, BN)) || (rc = p->alloc(&mb.lap, (size_t)B)) ||
            (rc = p->alloc(&mb.sweeps, (size_t)B * (mo + 1))))
            return rc;
    }
    if (p->stream) {
        if ((rc = p->alloc(&mb.sb.base, BN * rl::RL_STREAM_ARRAYS))) return rc;   // [B][15][N]
    }
    return RL_OK;
}

// the launch parameters of mode m (0: min-curv, 1: min-time) of plan p
static void fill_kparams(const rl_plan* p, int m, int sB, bool pre0, rl::KParams& kp) {
    const ModeBufs& mb = p->mb[m];
    kp = rl::KParams{};
    kp.center = p->d_center;
    kp.center_stride = p->center_stride;
    kp.Ls = p->d_Ls;
    for (int r = 0, off = 0; r < 2; off += p->ring_M[r], ++r) {
        kp.ring[r].vtx = (const double2*)(p->d_vtx + 2 * (size_t)off);
        kp.ring[r].rec = p->d_rec + off;
        kp.ring[r].flag = p->d_flag + off / 32;
        kp.ring[r].blk = p->d_blk + rl::ring_blk_doubles((size_t)off);
        kp.ring[r].M = p->ring_M[r];
        kp.ring[r].E = r == 0 ? p->Ei : p->Eo;
        kp.ring[r].dl0 = p->ring_dl0[r];
        kp.ring[r].dl32 = p->ring_dl32[r];
    }
    kp.cfg = p->d_cfg;
    kp.seeds = p->d_seeds;
    kp.x = mb.x; kp.y = mb.y; kp.heading = mb.heading; kp.kappa = mb.kappa;
    kp.alpha_total = mb.alpha_total; kp.alpha_last = mb.alpha_last;
    kp.v = mb.v; kp.ax = mb.ax; kp.lap = mb.lap; kp.nx = mb.nx; kp.ny = mb.ny;
    kp.evals = mb.evals; kp.accepts = mb.accepts; kp.sweeps = mb.sweeps;
    kp.N = p->N; kp.Ei = p->Ei; kp.Eo = p->Eo; kp.ncfg = p->ncfg; kp.B = p->B; kp.closed = p->closed;
    kp.shape_B = sB;
    kp.L = p->L; kp.veh_width = p->veh_width;
    kp.done = p->done[m];
    kp.epoch = p->epoch;
    kp.lo0 = pre0 ? p->d_lo0 : nullptr;
    kp.hi0 = pre0 ? p->d_hi0 : nullptr;
}

int rl_plan_run(rl_plan* p, void* hip_stream) {
    if (!p) return fail(RL_EINVAL, "plan is NULL");
    HIPCHK(hipSetDevice(p->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : p->own_stream;
    p->last_stream = st;
    HIPCHK(hipEventRecord(p->ev[0], st));
    // Both modes: run the min-time kernel concurrently on the aux stream when one kernel
    // leaves the GPU partly idle (B x waves per instance below two waves per SIMD on every
    // CU: C4's 512 single-wave instances per track, the drop-in B=1).  Larger batches fill
    // the GPU with either kernel alone and run them one after the other (C3: concurrent
    // 74.2 ms vs 73.1 ms sequential).
    const int cus = device_cus(p->device);
    const int sB = p->shape_B > 0 ? p->shape_B : p->B;
    const bool both = (p->modes & (RL_MODE_MINCURV | RL_MODE_MINTIME)) == (RL_MODE_MINCURV | RL_MODE_MINTIME) &&
                      (int64_t)p->B * std::max(waves_per_instance(p->N, sB, false, p->stream, cus),
                                               waves_per_instance(p->N, sB, true, p->stream, cus)) <=
                          (int64_t)8 * cus;
    // Outer iteration 0's corridor is the same for every instance (P = the shared centre, the
    // problem's veh_width, one cfg margin): cast it once here, rl_corridor_kernel, and let the
    // instances load it.  Only for batches that fill the GPU in a throughput shape (or the
    // streaming kernel): a latency-shape batch would wait for the extra launch longer than its
    // instances save (~1/14 of their corridor time).  RL_CORRIDOR0=0 turns it off (A/B, tests).
    const int first_m = (p->modes & RL_MODE_MINCURV) ? 0 : 1;
    bool pre0 = p->N > 0 && p->max_outer > 0 && p->center_stride == 0 && p->margin_uniform && p->B >= 2;
    if (pre0 && !p->stream) {
        const rl::Shape s = rl::pick_shape(p->N, sB, first_m == 1, cus), lat = rl::lat_shape(p->N);
        pre0 = !(s.K == lat.K && s.T == lat.T);
    }
    if (pre0) {
        const char* e = std::getenv("RL_CORRIDOR0");
        pre0 = !(e && e[0] == '0');
    }
    if (pre0) {
        HIPCHK(hipEventRecord(p->ev[1 + first_m], st));        // (inside the first mode's time)
        rl::CorrParams c{};
        c.center = p->d_center;
        c.N = p->N;
        c.closed = p->closed;
        for (int r = 0, off = 0; r < 2; off += p->ring_M[r], ++r) {
            c.ring[r].vtx = (const double2*)(p->d_vtx + 2 * (size_t)off);
            c.ring[r].rec = p->d_rec + off;
            c.ring[r].flag = p->d_flag + off / 32;
            c.ring[r].blk = p->d_blk + rl::ring_blk_doubles((size_t)off);
            c.ring[r].M = p->ring_M[r];
            c.ring[r].E = r == 0 ? p->Ei : p->Eo;
            c.ring[r].dl0 = p->ring_dl0[r];
            c.ring[r].dl32 = p->ring_dl32[r];
        }
        c.guard = p->veh_width * 0.5 + p->margin0;              // ref:706, as the kernels form it
        c.lo = p->d_lo0;
        c.hi = p->d_hi0;
        const hipError_t e = rl::launch_corridor(c, st);
        if (e != hipSuccess) return fail(RL_EHIP, std::string("corridor launch: ") + hipGetErrorString(e));
        HIPCHK(hipEventRecord(p->ev_c, st));
    }
    if (both) HIPCHK(hipStreamWaitEvent(p->aux_stream, pre0 ? p->ev_c : p->ev[0], 0));   // everything queued before
    for (int m = 0; m < 2; ++m) {
        if (!(p->modes & (1 << m))) continue;
        hipStream_t st_run = st;
        st = (both && m == 1) ? p->aux_stream : st_run;
        ModeBufs& mb = p->mb[m];
        const size_t BN = (size_t)p->B * (size_t)std::max(p->N, 1);
        if (p->N == 0 || p->max_outer == 0) {
            // ref:689 / 912 — N==0 returns an empty Result; zero the counters
            HIPCHK(hipMemsetAsync(mb.evals, 0, sizeof(int32_t) * p->B * std::max(p->max_outer, 1), st));
            HIPCHK(hipMemsetAsync(mb.accepts, 0, sizeof(int32_t) * p->B * std::max(p->max_outer, 1), st));
            if (m == 1) {
                HIPCHK(hipMemsetAsync(mb.lap, 0, sizeof(double) * p->B, st));
                HIPCHK(hipMemsetAsync(mb.sweeps, 0, sizeof(int32_t) * p->B * (p->max_outer + 1), st));
            }
            if (p->N == 0) {
                // no kernel: record the mode's events anyway, so rl_plan_kernel_ms(1 + m)
                // reports the (empty) interval instead of failing on an unrecorded event
                HIPCHK(hipEventRecord(p->ev[1 + m], st));
                HIPCHK(hipEventRecord(p->ev_end[m], st));
                st = st_run;
                continue;
            }
        }
        (void)BN;
        rl::KParams kp;
        fill_kparams(p, m, sB, pre0, kp);
        if (!(pre0 && m == first_m)) HIPCHK(hipEventRecord(p->ev[1 + m], st));
        hipError_t e = p->stream ? rl::launch_stream(kp, mb.sb, m == 1, st) : rl::launch_optimize(kp, m == 1, st);
        if (e != hipSuccess) return fail(RL_EHIP, std::string("kernel launch: ") + hipGetErrorString(e));
        HIPCHK(hipEventRecord(p->ev_end[m], st));
        st = st_run;
    }
    if (both) HIPCHK(hipStreamWaitEvent(st, p->ev_end[1], 0));
    HIPCHK(hipEventRecord(p->ev[3], st));
    p->ran = true;
    return RL_OK;
}

// rl_plan_run of n plans (one device) as few launches as their shapes allow: every (plan,
// mode) whose kernel shape is a one-wave throughput shape (rl::group_shape) joins the group
// launch of its (mode, K, closed) class, up to RL_GROUP_MAX plans per launch; the
// other plans run as rl_plan_run on their own streams.  The launches run concurrently, each
// on a plan-owned stream after everything queued on `hip_stream`, which waits for all of
// them.  Results equal each plan's own rl_plan_run bit for bit (the same instance code, the
// plan's own shape); the batch-wide first corridor is left to the instances.  Every plan's
// rl_plan_kernel_ms(.., 0) is the whole group's run, its mode times its launch's.
int rl_plan_run_group(rl_plan* const* plans, int32_t n, void* hip_stream) {
    if (!plans || n < 1) return fail(RL_EINVAL, "rl_plan_run_group: no plans");
    for (int i = 0; i < n; ++i) {
        if (!plans[i]) return fail(RL_EINVAL, "rl_plan_run_group: a plan is NULL");
        if (plans[i]->device != plans[0]->device) return fail(RL_EINVAL, "rl_plan_run_group: plans on different devices");
        for (int j = 0; j < i; ++j)
            if (plans[j] == plans[i]) return fail(RL_EINVAL, "rl_plan_run_group: a plan is listed twice");
    }
    HIPCHK(hipSetDevice(plans[0]->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : plans[0]->own_stream;
    const int cus = device_cus(plans[0]->device);
    struct Item {
        rl_plan* p;
        int m;
    };
    // class key: mode, K, closed.  A launch whose plans include a ragged N (N % K != 0) runs
    // the ragged form for all of them (it covers every N, bit for bit): one launch per class
    // instead of two (C4: 4 launches, all concurrent at 4 HW queues; 13.25 against 13.52 ms
    // split by N % K, profiles/r06/c4_group.log)
    std::vector<std::pair<std::array<int, 3>, std::vector<Item>>> classes;
    std::vector<rl_plan*> solo;
    for (int i = 0; i < n; ++i) {
        rl_plan* p = plans[i];
        const int sB = p->shape_B > 0 ? p->shape_B : p->B;
        bool ok = !p->stream && p->N > 0 && p->max_outer > 0 && (p->modes & 3);
        std::array<int, 3> key[2];
        for (int m = 0; m < 2 && ok; ++m) {
            if (!(p->modes & (1 << m))) continue;
            const rl::Shape s = rl::pick_shape(p->N, sB, m == 1, cus);
            ok = rl::group_shape(s);
            key[m] = {m, s.K, p->closed ? 1 : 0};
        }
        if (!ok) {
            solo.push_back(p);
            continue;
        }
        for (int m = 0; m < 2; ++m) {
            if (!(p->modes & (1 << m))) continue;
            auto it = std::find_if(classes.begin(), classes.end(), [&](const auto& c) { return c.first == key[m]; });
            if (it == classes.end()) {
                classes.push_back({key[m], {}});
                it = classes.end() - 1;
            }
            it->second.push_back({p, m});
        }
    }
    // the plans of a class longest first (by N): the grid dispatches its workgroups in order,
    // so its last ones are the shorter instances (C4 13.39 -> 13.14 ms, profiles/r06/c4_group.log)
    for (auto& c : classes)
        std::stable_sort(c.second.begin(), c.second.end(), [](const Item& x, const Item& y) { return x.p->N > y.p->N; });
    // the launches: class chunks of up to RL_GROUP_MAX plans, then the solo plans
    struct Launch {
        int cls;
        size_t i0;
        int cnt;
        hipStream_t ls;
    };
    std::vector<Launch> launches;
    std::vector<hipStream_t> pool;                   // grouped plans' own and aux streams
    for (auto& c : classes)
        for (const Item& it : c.second)
            for (hipStream_t x : {it.p->own_stream, it.p->aux_stream})
                if (std::find(pool.begin(), pool.end(), x) == pool.end()) pool.push_back(x);
    for (size_t ci = 0; ci < classes.size(); ++ci)
        for (size_t i0 = 0; i0 < classes[ci].second.size(); i0 += rl::RL_GROUP_MAX)
            launches.push_back({(int)ci, i0, (int)std::min<size_t>(rl::RL_GROUP_MAX, classes[ci].second.size() - i0),
                                pool[launches.size() % pool.size()]});
    // fork: every launch stream waits for what `hip_stream` has queued, before any launch
    // (a solo plan's rl_plan_run re-records its own events)
    hipEvent_t start = plans[0]->ev_c;               // (a disable-timing event of the group)
    HIPCHK(hipEventRecord(start, st));
    for (const Launch& L : launches) HIPCHK(hipStreamWaitEvent(L.ls, start, 0));
    for (rl_plan* p : solo) HIPCHK(hipStreamWaitEvent(p->own_stream, start, 0));
    for (int i = 0; i < n; ++i) {
        HIPCHK(hipEventRecord(plans[i]->ev[0], st));
        plans[i]->last_stream = st;
    }
    std::vector<hipEvent_t> ends;
    for (const Launch& L : launches) {
        const int m = classes[L.cls].first[0];
        const rl::Shape s{classes[L.cls].first[1], 64};
        const std::vector<Item>& items = classes[L.cls].second;
        rl::KGroup g{};
        g.n = L.cnt;
        int blocks = 0;
        bool ragged = false;
        for (int j = 0; j < L.cnt; ++j) {
            rl_plan* p = items[L.i0 + j].p;
            fill_kparams(p, m, p->shape_B > 0 ? p->shape_B : p->B, false, g.p[j]);
            g.start[j] = blocks;
            blocks += p->B;
            ragged |= p->N % s.K != 0;
        }
        for (int j = 0; j < L.cnt; ++j) HIPCHK(hipEventRecord(items[L.i0 + j].p->ev[1 + m], L.ls));
        const hipError_t e = rl::launch_optimize_group(g, s, classes[L.cls].first[2] != 0, ragged, m == 1, L.ls);
        if (e != hipSuccess) return fail(RL_EHIP, std::string("group launch: ") + hipGetErrorString(e));
        for (int j = 0; j < L.cnt; ++j) HIPCHK(hipEventRecord(items[L.i0 + j].p->ev_end[m], L.ls));
        ends.push_back(items[L.i0 + L.cnt - 1].p->ev_end[m]);
    }
    for (rl_plan* p : solo) {
        const int rc = rl_plan_run(p, p->own_stream);
        if (rc != RL_OK) return rc;
        ends.push_back(p->ev[3]);
        p->last_stream = st;
    }
    for (hipEvent_t e : ends) HIPCHK(hipStreamWaitEvent(st, e, 0));
    for (int i = 0; i < n; ++i) {
        HIPCHK(hipEventRecord(plans[i]->ev[3], st));
        plans[i]->ran = true;
    }
    return RL_OK;
}

// B lap evaluations: heading_curv_from_points_generic + velocity_profile_forward_backward
// with h = L[b]/N on path b (ref:1045-1048, and the debug laps ref:1466-1478) = the
// min-time driver with max_outer_iters = 0 on per-instance centres.
int rl_lap_eval(const double* paths_xy, const double* L, int32_t N, int32_t B, int32_t closed, const rl_cfg* cfg,
                int32_t n_cfg, int32_t device, rl_out* out, float* kernel_ms) {
    if (!paths_xy || !L || !cfg || !out) return fail(RL_EINVAL, "rl_lap_eval: NULL argument");
    if (B < 1 || N < 0) return fail(RL_EINVAL, "rl_lap_eval: B < 1 or N < 0");
    if (n_cfg != 1 && n_cfg != B) return fail(RL_EINVAL, "n_cfg must be 1 or B");
    std::vector<rl_cfg> c(cfg, cfg + n_cfg);
    for (auto& x : c) x.max_outer_iters = 0;
    rl_problem pr{};
    pr.N = N;
    pr.closed = closed;
    pr.L = L[0];
    int ndev = 0, cur = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RL_ENODEV, "device index out of range");
    const bool restore = hipGetDevice(&cur) == hipSuccess;
    HIPCHK(hipSetDevice(device));
    float ms[3];
    const int rc = run_cached(&pr, c.data(), n_cfg, nullptr, B, RL_MODE_MINTIME, paths_xy, L, nullptr, out, ms);
    if (rc == RL_OK && kernel_ms) *kernel_ms = ms[2];
    if (restore) hipSetDevice(cur);
    return rc;
}

// pipeline::compute_geom_and_save rows (ref:1295-1335) on the device
int rl_corridor(const rl_problem* prob, const rl_cfg* cfg, int32_t device, double* lo, double* hi) {
    if (!prob || !cfg || !lo || !hi) return fail(RL_EINVAL, "rl_corridor: NULL argument");
    if (prob->N < 0 || (prob->N > 0 && !prob->center_xy)) return fail(RL_EINVAL, "rl_corridor: bad centre");
    if (prob->Ei < 0 || prob->Eo < 0 || (prob->Ei > 0 && !prob->inner_seg) || (prob->Eo > 0 && !prob->outer_seg))
        return fail(RL_EINVAL, "rl_corridor: bad segments");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RL_ENODEV, "device index out of range");
    HIPCHK(hipSetDevice(device));
    const int N = prob->N;
    if (N == 0) return RL_OK;
    RingHost rh[2] = {make_ring(prob->inner_seg, prob->Ei), make_ring(prob->outer_seg, prob->Eo)};
    const size_t Mt = (size_t)rh[0].M + rh[1].M;
    std::vector<void*> mem;
    auto dalloc = [&](size_t bytes) -> void* {
        void* q = nullptr;
        if (hipMalloc(&q, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
        mem.push_back(q);
        return q;
    };
    auto release = [&](int code) {
        for (void* q : mem) hipFree(q);
        return code;
    };
    double* d_c = (double*)dalloc(2 * (size_t)N * sizeof(double));
    double* d_out = (double*)dalloc(2 * (size_t)N * sizeof(double));
    double* d_vtx = (double*)dalloc(2 * Mt * sizeof(double));
    rl::SegRec* d_rec = (rl::SegRec*)dalloc(Mt * sizeof(rl::SegRec));
    uint32_t* d_flag = (uint32_t*)dalloc(Mt / 32 * sizeof(uint32_t));
    double* d_blk = (double*)dalloc(rl::ring_blk_doubles(Mt) * sizeof(double));
    if (!d_c || !d_out || !d_vtx || !d_rec || !d_flag || !d_blk) return release(fail(RL_ENOMEM, "rl_corridor: hipMalloc failed"));
    rl::CorrParams c{};
    c.center = d_c;
    c.N = N;
    c.closed = prob->closed ? 1 : 0;
    c.guard = prob->veh_width * 0.5 + cfg->safety_margin_m;     // ref:706
    c.lo = d_out;
    c.hi = d_out + N;
    bool ok = hipMemcpy(d_c, prob->center_xy, 2 * (size_t)N * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
    for (int r = 0, off = 0; r < 2; off += rh[r].M, ++r) {
        const RingHost& R = rh[r];
        if (R.M)
            ok = ok &&
                 hipMemcpy(d_vtx + 2 * (size_t)off, R.vtx.data(), R.vtx.size() * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
                 hipMemcpy(d_rec + off, R.rec.data(), R.rec.size() * sizeof(rl::SegRec), hipMemcpyHostToDevice) == hipSuccess &&
                 hipMemcpy(d_flag + off / 32, R.flag.data(), R.flag.size() * sizeof(uint32_t), hipMemcpyHostToDevice) == hipSuccess &&
                 hipMemcpy(d_blk + rl::ring_blk_doubles((size_t)off), R.blk.data(), R.blk.size() * sizeof(double),
                           hipMemcpyHostToDevice) == hipSuccess;
        c.ring[r].vtx = (const double2*)(d_vtx + 2 * (size_t)off);
        c.ring[r].rec = d_rec + off;
        c.ring[r].flag = d_flag + off / 32;
        c.ring[r].blk = d_blk + rl::ring_blk_doubles((size_t)off);
        c.ring[r].M = R.M;
        c.ring[r].E = R.E;
        c.ring[r].dl0 = R.dl0;
        c.ring[r].dl32 = R.dl32;
    }
    if (!ok) return release(fail(RL_EHIP, "rl_corridor: upload"));
    if (rl::launch_corridor(c, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return release(fail(RL_EHIP, "rl_corridor: kernel"));
    if (hipMemcpy(lo, d_out, (size_t)N * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hi, d_out + N, (size_t)N * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
        return release(fail(RL_EHIP, "rl_corridor: download"));
    return release(RL_OK);
}

int rl_geom(const rl_geom_problem* gp, const rl_cfg* cfg, int32_t device, double* rows, float* kernel_ms) {
    if (!gp || !cfg || !rows) return fail(RL_EINVAL, "rl_geom: NULL argument");
    if (gp->Kmax < 0 || gp->denomN == 0) return fail(RL_EINVAL, "rl_geom: Kmax < 0 or denomN == 0");
    if (gp->spx.n != gp->spy.n || gp->spx.n < 0) return fail(RL_EINVAL, "rl_geom: spline sizes differ");
    if (gp->Ei < 0 || gp->Eo < 0 || (gp->Ei > 0 && !gp->inner_seg) || (gp->Eo > 0 && !gp->outer_seg))
        return fail(RL_EINVAL, "rl_geom: bad segments");
    const int nk = gp->spx.n;
    const rl_spline* sp[2] = {&gp->spx, &gp->spy};
    for (int a = 0; a < 2; ++a)
        if (nk > 0 && (!sp[a]->s || !sp[a]->a || !sp[a]->b || !sp[a]->c || !sp[a]->d))
            return fail(RL_EINVAL, "rl_geom: NULL spline array");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RL_ENODEV, "device index out of range");
    HIPCHK(hipSetDevice(device));
    const int nrows = gp->Kmax + (gp->emit_closed_duplicate ? 1 : 0);
    if (gp->Kmax == 0) {                      // no rows computed: the duplicate is (L, 0, ..., 0)
        if (nrows) { std::memset(rows, 0, sizeof(double) * RL_GEOM_COLS); rows[0] = gp->L; }
        if (kernel_ms) *kernel_ms = 0.0f;
        return nrows;
    }
    RingHost rh[2] = {make_ring(gp->inner_seg, gp->Ei), make_ring(gp->outer_seg, gp->Eo)};
    std::vector<double> kn((size_t)10 * std::max(nk, 1), 0.0);
    for (int a = 0; a < 2; ++a) {
        const double* arr[5] = {sp[a]->s, sp[a]->a, sp[a]->b, sp[a]->c, sp[a]->d};
        for (int j = 0; j < 5; ++j)
            if (nk) std::memcpy(&kn[(size_t)(5 * a + j) * nk], arr[j], sizeof(double) * nk);
    }
    const size_t Mt = (size_t)rh[0].M + rh[1].M;
    std::vector<void*> mem;
    auto dalloc = [&](size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
        mem.push_back(p);
        return p;
    };
    auto release = [&](int code) {
        for (void* p : mem) hipFree(p);
        return code;
    };
    double* d_kn = (double*)dalloc(kn.size() * sizeof(double));
    double* d_vtx = (double*)dalloc(2 * Mt * sizeof(double));
    rl::SegRec* d_rec = (rl::SegRec*)dalloc(Mt * sizeof(rl::SegRec));
    uint32_t* d_flag = (uint32_t*)dalloc(Mt / 32 * sizeof(uint32_t));
    double* d_blk = (double*)dalloc(rl::ring_blk_doubles(Mt) * sizeof(double));
    double* d_rows = (double*)dalloc((size_t)nrows * RL_GEOM_COLS * sizeof(double));
    if (!d_kn || !d_vtx || !d_rec || !d_flag || !d_blk || !d_rows) return release(fail(RL_ENOMEM, "rl_geom: hipMalloc failed"));
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return release(fail(RL_EHIP, "rl_geom: stream"));
    auto finish = [&](int code) {
        if (e0) hipEventDestroy(e0);
        if (e1) hipEventDestroy(e1);
        hipStreamSynchronize(st);
        hipStreamDestroy(st);
        return release(code);
    };
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return finish(fail(RL_EHIP, "rl_geom: events"));
    if (hipMemcpyAsync(d_kn, kn.data(), kn.size() * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess)
        return finish(fail(RL_EHIP, "rl_geom: upload knots"));
    rl::GeomParams g{};
    for (int r = 0, off = 0; r < 2; off += rh[r].M, ++r) {
        const RingHost& R = rh[r];
        if (R.M) {
            if (hipMemcpyAsync(d_vtx + 2 * (size_t)off, R.vtx.data(), R.vtx.size() * sizeof(double), hipMemcpyHostToDevice, st) ||
                hipMemcpyAsync(d_rec + off, R.rec.data(), R.rec.size() * sizeof(rl::SegRec), hipMemcpyHostToDevice, st) ||
                hipMemcpyAsync(d_flag + off / 32, R.flag.data(), R.flag.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st) ||
                hipMemcpyAsync(d_blk + rl::ring_blk_doubles((size_t)off), R.blk.data(), R.blk.size() * sizeof(double),
                               hipMemcpyHostToDevice, st))
                return finish(fail(RL_EHIP, "rl_geom: upload rings"));
        }
        g.ring[r].vtx = (const double2*)(d_vtx + 2 * (size_t)off);
        g.ring[r].rec = d_rec + off;
        g.ring[r].flag = d_flag + off / 32;
        g.ring[r].blk = d_blk + rl::ring_blk_doubles((size_t)off);
        g.ring[r].M = R.M;
        g.ring[r].E = R.E;
        g.ring[r].dl0 = R.dl0;
        g.ring[r].dl32 = R.dl32;
    }
    g.kx = d_kn;
    g.ky = d_kn + 5 * (size_t)nk;
    g.nk = nk;
    g.Kmax = gp->Kmax;
    g.denomN = gp->denomN;
    g.emit_dup = gp->emit_closed_duplicate ? 1 : 0;
    g.s0 = gp->s0;
    g.L = gp->L;
    g.kappa_eps = cfg->kappa_eps;
    g.a_lat_max = cfg->a_lat_max;
    g.v_cap = cfg->v_cap_mps;
    g.rows = d_rows;
    if (hipEventRecord(e0, st) != hipSuccess) return finish(fail(RL_EHIP, "rl_geom: event"));
    if (rl::launch_geom(g, st) != hipSuccess) return finish(fail(RL_EHIP, "rl_geom: kernel launch"));
    if (hipEventRecord(e1, st) != hipSuccess) return finish(fail(RL_EHIP, "rl_geom: event"));
    if (hipMemcpyAsync(rows, d_rows, (size_t)nrows * RL_GEOM_COLS * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return finish(fail(RL_EHIP, "rl_geom: download"));
    if (kernel_ms) {
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        *kernel_ms = ms;
    }
    return finish(nrows);
}

// glibc "%.9f" CSV rows of a host table, formatted on the device (rl_format.hip)
int rl_format_csv(const double* table, int64_t rows, int32_t cols, int32_t device, char* out, int64_t out_cap,
                  int64_t* out_len, int64_t* row_offsets) {
    if (!out_len || rows < 0 || cols < 1 || (rows > 0 && !table) || (out_cap > 0 && !out))
        return fail(RL_EINVAL, "rl_format_csv: bad argument");
    *out_len = 0;
    if (rows == 0) {
        if (row_offsets) row_offsets[0] = 0;
        return RL_OK;
    }
    if (rows > (int64_t)1 << 31) return fail(RL_ETOOBIG, "rl_format_csv: more than 2^31 rows");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RL_ENODEV, "device index out of range");
    HIPCHK(hipSetDevice(device));
    const uint64_t cap = (uint64_t)rows * (uint64_t)cols * 22;
    double* d_tab = nullptr;
    char* d_out = nullptr;
    uint64_t* d_offs = nullptr;
    hipStream_t st = nullptr;
    auto done = [&](int code) {
        if (st) { hipStreamSynchronize(st); hipStreamDestroy(st); }
        if (d_tab) hipFree(d_tab);
        if (d_out) hipFree(d_out);
        if (d_offs) hipFree(d_offs);
        return code;
    };
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return done(fail(RL_EHIP, "stream"));
    if (hipMalloc((void**)&d_tab, (size_t)rows * cols * 8) != hipSuccess || hipMalloc((void**)&d_out, cap) != hipSuccess ||
        hipMalloc((void**)&d_offs, (size_t)(rows + 1) * 8) != hipSuccess)
        return done(fail(RL_ENOMEM, "rl_format_csv: hipMalloc failed"));
    if (hipMemcpyAsync(d_tab, table, (size_t)rows * cols * 8, hipMemcpyHostToDevice, st) != hipSuccess)
        return done(fail(RL_EHIP, "rl_format_csv: upload"));
    uint64_t total = 0;
    const int rc = rl::format_rows(d_tab, rows, cols, d_out, cap, d_offs, &total, st);
    if (rc == -1) return done(fail(RL_ETOOBIG, "rl_format_csv: a value with |x| >= 9.2e9"));
    if (rc != 0) return done(fail(RL_EHIP, "rl_format_csv: device formatting failed"));
    *out_len = (int64_t)total;
    if ((int64_t)total > out_cap) return done(fail(RL_ETOOBIG, "rl_format_csv: out_cap too small (see *out_len)"));
    if (hipMemcpyAsync(out, d_out, total, hipMemcpyDeviceToHost, st) != hipSuccess ||
        (row_offsets && hipMemcpyAsync(row_offsets, d_offs, (size_t)(rows + 1) * 8, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return done(fail(RL_EHIP, "rl_format_csv: download"));
    return done(RL_OK);
}

int rl_plan_kernel_ms(rl_plan* p, int32_t idx, float* ms) {
    if (!p || !ms || !p->ran) return fail(RL_EINVAL, "plan not run");
    HIPCHK(hipSetDevice(p->device));
    HIPCHK(hipEventSynchronize(p->ev[3]));
    // idx 0: whole run; 1: min-curv kernel; 2: min-time kernel
    hipEvent_t a, b;
    const bool mc = p->modes & RL_MODE_MINCURV, mt = p->modes & RL_MODE_MINTIME;
    if (idx == 0) { a = p->ev[0]; b = p->ev[3]; }
    else if (idx == 1 && mc) { a = p->ev[1]; b = p->ev_end[0]; }
    else if (idx == 2 && mt) { a = p->ev[2]; b = p->ev_end[1]; }
    else return fail(RL_EINVAL, "kernel index not in this plan");
    HIPCHK(hipEventElapsedTime(ms, a, b));
    return RL_OK;
}

// the (host destination, device source, bytes) copies that fill `o` from mode m's results
struct CopyJob {
    void* dst;
    const void* src;
    size_t bytes;
};
static void out_jobs(const rl_plan* p, int m, const rl_out* o, std::vector<CopyJob>& jobs) {
    if (!o) return;
    const ModeBufs& mb = p->mb[m];
    const size_t BN = (size_t)p->B * (size_t)p->N;
    auto add = [&](void* dst, const void* src, size_t bytes) {
        if (dst && src && bytes) jobs.push_back({dst, src, bytes});
    };
    add(o->x, mb.x, BN * 8);
    add(o->y, mb.y, BN * 8);
    add(o->heading, mb.heading, BN * 8);
    add(o->kappa, mb.kappa, BN * 8);
    add(o->alpha_total, mb.alpha_total, BN * 8);
    add(o->alpha_last, mb.alpha_last, BN * 8);
    add(o->evals, mb.evals, (size_t)p->B * p->max_outer * 4);
    add(o->accepts, mb.accepts, (size_t)p->B * p->max_outer * 4);
    if (m == 1) {
        add(o->v, mb.v, BN * 8);
        add(o->ax, mb.ax, BN * 8);
        add(o->lap, mb.lap, (size_t)p->B * 8);
        add(o->vpass_sweeps, mb.sweeps, (size_t)p->B * (p->max_outer + 1) * 4);
    }
}

static int fetch_mode(rl_plan* p, int m, rl_out* o, hipStream_t st) {
    std::vector<CopyJob> jobs;
    out_jobs(p, m, o, jobs);
    for (const CopyJob& j : jobs) {
        hipError_t e = hipMemcpyAsync(j.dst, j.src, j.bytes, hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) return fail(RL_EHIP, std::string("download: ") + hipGetErrorString(e));
    }
    return RL_OK;
}

int rl_plan_fetch(rl_plan* p, rl_out* out_mc, rl_out* out_mt) {
    if (!p) return fail(RL_EINVAL, "plan is NULL");
    if ((out_mc && !(p->modes & RL_MODE_MINCURV)) || (out_mt && !(p->modes & RL_MODE_MINTIME)))
        return fail(RL_EINVAL, "requested a mode the plan did not run");
    HIPCHK(hipSetDevice(p->device));
    hipStream_t st = p->last_stream ? p->last_stream : p->own_stream;
    int rc;
    if ((rc = fetch_mode(p, 0, out_mc, st)) || (rc = fetch_mode(p, 1, out_mt, st))) return rc;
    HIPCHK(hipStreamSynchronize(st));
    return RL_OK;
}

int rl_plan_bind_device_outputs(rl_plan* p, int32_t which, const rl_out* d) {
    if (!p || !d) return fail(RL_EINVAL, "NULL argument");
    int m = (which == RL_MODE_MINCURV) ? 0 : (which == RL_MODE_MINTIME ? 1 : -1);
    if (m < 0 || !(p->modes & which)) return fail(RL_EINVAL, "mode not in plan");
    ModeBufs& mb = p->mb[m];
    if (d->x) mb.x = d->x;
    if (d->y) mb.y = d->y;
    if (d->heading) mb.heading = d->heading;
    if (d->kappa) mb.kappa = d->kappa;
    if (d->alpha_total) mb.alpha_total = d->alpha_total;
    if (d->alpha_last) mb.alpha_last = d->alpha_last;
    if (m == 1) {
        if (d->v) mb.v = d->v;
        if (d->ax) mb.ax = d->ax;
        if (d->lap) mb.lap = d->lap;
        if (d->vpass_sweeps) mb.sweeps = d->vpass_sweeps;
    }
    if (d->evals) mb.evals = d->evals;
    if (d->accepts) mb.accepts = d->accepts;
    return RL_OK;
}

int rl_plan_device_outputs(rl_plan* p, int32_t which, rl_out* d) {
    if (!p || !d) return fail(RL_EINVAL, "NULL argument");
    int m = (which == RL_MODE_MINCURV) ? 0 : (which == RL_MODE_MINTIME ? 1 : -1);
    if (m < 0 || !(p->modes & which)) return fail(RL_EINVAL, "mode not in plan");
    ModeBufs& mb = p->mb[m];
    std::memset(d, 0, sizeof(*d));
    d->x = mb.x; d->y = mb.y; d->heading = mb.heading; d->kappa = mb.kappa;
    d->alpha_total = mb.alpha_total; d->alpha_last = mb.alpha_last;
    d->v = mb.v; d->ax = mb.ax; d->lap = mb.lap;
    d->evals = mb.evals; d->accepts = mb.accepts; d->vpass_sweeps = mb.sweeps;
    return RL_OK;
}

// ------------------------------------------------------------------ plan cache
// rl_optimize and rl_lap_eval are the reference's own use: one synchronous call per track
// and mode (ref:1347, 1397, 1466-1478), host buffers in and out.  Building a plan per call
// (a hipMalloc per array, a stream, events) and copying through pageable memory cost more
// than the kernel at small B, so these calls reuse plans from a small process-wide cache,
// keyed by the plan's shape and the ring segments (compared bit for bit): a hit uploads
// only the centreline, cfg and seeds.  Every copy is staged through pinned host memory
// owned by the entry; results are downloaded array by array, each with an event, and
// host threads copy an array out as soon as its event completes.  An entry in use is
// checked out, so concurrent callers never share one.  The cache object is never
// destroyed (no HIP call at process exit); rl_release_plan_cache() frees the idle plans.
}  // extern "C"

namespace {

constexpr int kCacheEntries = 8;                       // idle plans kept
// device + pinned host bytes kept idle (RL_PLAN_CACHE_MB overrides; 0 disables caching).
// An entry larger than the budget on its own is not kept either, so one oversized call
// leaves nothing allocated behind it.
constexpr size_t kCacheBytesDefault = (size_t)2 << 30;
size_t cache_budget() {
    const char* s = std::getenv("RL_PLAN_CACHE_MB");
    if (!s || !*s) return kCacheBytesDefault;
    char* end = nullptr;
    const unsigned long long mb = std::strtoull(s, &end, 10);
    if (end == s) return kCacheBytesDefault;
    return (size_t)mb << 20;
}
constexpr int kJobEvents = 512;   // download events of an entry (download_staged, download_overlapped)

struct CacheEntry {
    rl_plan* p = nullptr;
    int device = 0, N = 0, B = 0, ncfg = 0, mo = 0, closed = 0, Ei = 0, Eo = 0;
    bool stream = false, centers = false, Ls = false;
    std::vector<double> segs;                          // inner then outer segments
    unsigned char* pin = nullptr;                      // pinned staging
    size_t pin_bytes = 0;
    hipEvent_t ev[kJobEvents] = {};
    // overlapped download (download_overlapped): per-mode instance completion flags in
    // coherent pinned memory, the epoch of the last run, and the copy stream
    uint32_t* flags = nullptr;
    int flags_n = 0;
    uint32_t epoch = 0;
    hipStream_t dl = nullptr;
    uint64_t tick = 0;

    bool same(const CacheEntry& k) const {
        return device == k.device && N == k.N && B == k.B && ncfg == k.ncfg && mo == k.mo && closed == k.closed &&
               Ei == k.Ei && Eo == k.Eo && stream == k.stream && centers == k.centers && Ls == k.Ls &&
               segs.size() == k.segs.size() &&
               (segs.empty() || std::memcmp(segs.data(), k.segs.data(), segs.size() * sizeof(double)) == 0);
    }
    // device memory of the plan plus the pinned staging buffer (both stay allocated while idle)
    size_t bytes() const { return (p ? p->dev_bytes : 0) + pin_bytes + (size_t)flags_n * sizeof(uint32_t); }
};

void destroy_entry(CacheEntry* e) {
    if (!e) return;
    if (e->p) {
        hipSetDevice(e->p->device);
        rl_plan_destroy(e->p);
    }
    for (hipEvent_t& v : e->ev)
        if (v) hipEventDestroy(v);
    if (e->dl) {
        hipStreamSynchronize(e->dl);
        hipStreamDestroy(e->dl);
    }
    if (e->flags) hipHostFree(e->flags);
    if (e->pin) hipHostFree(e->pin);
    delete e;
}

struct PlanCache {
    std::mutex mu;
    std::vector<CacheEntry*> idle;
    uint64_t tick = 0;

    CacheEntry* take(const CacheEntry& key) {
        std::lock_guard<std::mutex> g(mu);
        for (size_t i = 0; i < idle.size(); ++i)
            if (idle[i]->same(key)) {
                CacheEntry* e = idle[i];
                idle.erase(idle.begin() + (long)i);
                return e;
            }
        return nullptr;
    }
    void give(CacheEntry* e) {
        std::vector<CacheEntry*> evict;
        const size_t budget = cache_budget();
        {
            std::lock_guard<std::mutex> g(mu);
            e->tick = ++tick;
            idle.push_back(e);
            auto total = [&]() {
                size_t t = 0;
                for (CacheEntry* q : idle) t += q->bytes();
                return t;
            };
            // least recently used first, down to the newest entry itself when it alone
            // exceeds the budget
            while (!idle.empty() && ((int)idle.size() > kCacheEntries || total() > budget)) {
                auto lru = std::min_element(idle.begin(), idle.end(),
                                            [](CacheEntry* x, CacheEntry* y) { return x->tick < y->tick; });
                evict.push_back(*lru);
                idle.erase(lru);
            }
        }
        for (CacheEntry* q : evict) destroy_entry(q);
    }
    void info(int32_t* entries, int64_t* dev_bytes, int64_t* pin_bytes) {
        std::lock_guard<std::mutex> g(mu);
        int64_t d = 0, h = 0;
        for (CacheEntry* q : idle) {
            d += q->p ? (int64_t)q->p->dev_bytes : 0;
            h += (int64_t)q->pin_bytes;
        }
        if (entries) *entries = (int32_t)idle.size();
        if (dev_bytes) *dev_bytes = d;
        if (pin_bytes) *pin_bytes = h;
    }
    void clear() {
        std::vector<CacheEntry*> all;
        {
            std::lock_guard<std::mutex> g(mu);
            all.swap(idle);
        }
        for (CacheEntry* q : all) destroy_entry(q);
    }
};
PlanCache& plan_cache() {
    static PlanCache* c = new PlanCache();
    return *c;
}

thread_local float g_last_kernel_ms = -1.0f, g_last_call_ms = -1.0f;
thread_local float g_last_mode_ms[2] = {-1.0f, -1.0f};    // min-curv / min-time kernel of the last call
thread_local int g_last_groups = 0, g_last_groups_signalled = 0;   // the last call's download groups

int ensure_pinned(CacheEntry* e, size_t bytes) {
    if (bytes <= e->pin_bytes) return RL_OK;
    if (e->pin) hipHostFree(e->pin);
    e->pin = nullptr;
    e->pin_bytes = 0;
    const size_t want = std::max(bytes, (size_t)1 << 16);
    if (hipHostMalloc((void**)&e->pin, want, hipHostMallocDefault) != hipSuccess) {
        e->pin = nullptr;
        return fail(RL_ENOMEM, "hipHostMalloc (pinned staging) failed");
    }
    e->pin_bytes = want;
    return RL_OK;
}

// Download `jobs` through the entry's pinned staging (from byte `base` on): one async copy
// per job on stream st with an event after each (the last event covers any jobs beyond
// the pool), then host threads copy each job out in 4 MiB pieces as soon as its event has
// completed, so the host copies overlap the transfers still in flight.
int download_staged(CacheEntry* e, hipStream_t st, const std::vector<CopyJob>& jobs, size_t base) {
    struct Piece {
        unsigned char* dst;
        const unsigned char* src;
        size_t bytes;
        int ev;
    };
    std::vector<Piece> pieces;
    size_t off = base, total = 0;
    const size_t kPiece = (size_t)4 << 20;
    for (size_t j = 0; j < jobs.size(); ++j) {
        if (hipMemcpyAsync(e->pin + off, jobs[j].src, jobs[j].bytes, hipMemcpyDeviceToHost, st) != hipSuccess)
            return fail(RL_EHIP, "download (staged) failed");
        const int evi = (int)std::min(j, (size_t)kJobEvents - 1);
        const bool last = j + 1 == jobs.size();
        if ((size_t)evi == j || last)
            if (hipEventRecord(e->ev[evi], st) != hipSuccess) return fail(RL_EHIP, "hipEventRecord failed");
        for (size_t q = 0; q < jobs[j].bytes; q += kPiece)
            pieces.push_back({(unsigned char*)jobs[j].dst + q, e->pin + off + q, std::min(kPiece, jobs[j].bytes - q), evi});
        off += (jobs[j].bytes + 255) & ~(size_t)255;
        total += jobs[j].bytes;
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    auto work = [&]() {
        for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
            if (hipEventSynchronize(e->ev[pieces[i].ev]) != hipSuccess) {
                bad = true;
                return;
            }
            std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].bytes);
        }
    };
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nthr = total < ((size_t)8 << 20) ? 1 : (int)std::min<size_t>({8, hw, pieces.size()});
    // helper threads are an optimisation: if one cannot be started (std::system_error,
    // std::bad_alloc), the calling thread does its share, and no exception leaves the C ABI
    std::vector<std::thread> th;
    try {
        th.reserve((size_t)std::max(0, nthr - 1));
        for (int t = 1; t < nthr; ++t) th.emplace_back(work);
    } catch (...) {
    }
    work();
    for (auto& t : th) t.join();
    if (bad) return fail(RL_EHIP, "download (staged): event wait failed");
    return RL_OK;
}

// bytes of the staging area a job list needs (256-B aligned pieces)
size_t staged_bytes(const std::vector<CopyJob>& jobs) {
    size_t t = 0;
    for (const CopyJob& j : jobs) t += (j.bytes + 255) & ~(size_t)255;
    return t;
}

// ---- overlapped download (large batches)
// The kernel of an rl_optimize call finishes its instances over its whole run (a batch of
// B instances takes B / (instances resident) rounds), but a download that waits for the
// kernel moves all of their results after it (C2: 98 MB, 40 % of the call).
// Here every instance signals its completion (KParams::done, signal_done in rl_kernels.h)
// into coherent pinned memory; the calling thread watches the flags and, as soon as every
// instance of a group has signalled, queues that group's result slices (instance-major
// arrays: one contiguous slice per array) on a copy stream, while the kernel still computes
// later instances.  Helper threads copy each group out of the pinned staging as its copies
// land.  The launch is the one rl_plan_run makes anyway, so the results are those of the
// plan path bit for bit.  A kernel that ends without signalling some instance (or any HIP
// failure) takes the stream-ordered path for the rest: the copy stream waits for the
// kernel's end event.  RL_OVERLAP_DOWNLOAD=0 turns the overlap off (A/B, tests).
constexpr size_t kOverlapMinBytes = (size_t)8 << 20;  // smaller downloads: one staged pass
constexpr int kGroupsPerMode = 16;                     // groups of a mode
static_assert(2 * kGroupsPerMode <= kJobEvents, "one download event per group");

bool overlap_enabled() {
    const char* s = std::getenv("RL_OVERLAP_DOWNLOAD");
    return !(s && s[0] == '0');
}

int ensure_flags(CacheEntry* e, int B) {
    if (!e->dl && hipStreamCreateWithFlags(&e->dl, hipStreamNonBlocking) != hipSuccess) {
        e->dl = nullptr;
        return fail(RL_EHIP, "hipStreamCreate (download stream) failed");
    }
    if (e->flags && e->flags_n >= 2 * B) return RL_OK;
    if (e->flags) hipHostFree(e->flags);
    e->flags = nullptr;
    e->flags_n = 0;
    if (hipHostMalloc((void**)&e->flags, (size_t)2 * B * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped) !=
        hipSuccess) {
        e->flags = nullptr;
        return fail(RL_ENOMEM, "hipHostMalloc (completion flags) failed");
    }
    std::memset(e->flags, 0, (size_t)2 * B * sizeof(uint32_t));
    e->flags_n = 2 * B;
    e->epoch = 0;
    return RL_OK;
}

// Ask the kernel for writable pages behind [p, p + n) now (MADV_POPULATE_WRITE, Linux 5.14;
// errors ignored): a page already present is left as it is, so this never changes the
// caller's data and may run while another thread copies into the same range.  Fresh output
// arrays (the reference's own use) would otherwise take their page faults inside the copies
// after the kernel.
void populate_write(void* p, size_t n) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
    static const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    if (!n) return;
    const uintptr_t a = (uintptr_t)p & ~(pg - 1), b = ((uintptr_t)p + n + pg - 1) & ~(pg - 1);
    (void)madvise((void*)a, b - a, MADV_POPULATE_WRITE);
}

#ifdef RL_OVL_TRACE
// diagnostic builds: times (ms since the call's entry) of one rl_optimize call, printed to
// stderr as one JSON line when the call returns
struct OvlTrace {
    std::chrono::steady_clock::time_point t0;
    double launched = -1, kend = -1, dma = -1, copied = -1;
    int nthr = 0;
    std::vector<double> pub;
};
thread_local OvlTrace g_tr;
double tr_ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_tr.t0).count(); }
#endif

// jm[m]: mode m's download jobs (out_jobs order, every array instance-major over the plan's B
// instances).  Called after rl_plan_run queued the kernels with p->done set.
int download_overlapped(CacheEntry* e, rl_plan* p, const std::vector<CopyJob> (&jm)[2], uint32_t epoch) {
    const int B = p->B;
    const int G = std::min(kGroupsPerMode, B);
    struct Group {
        int m, b0, b1;
        int s0, s1;                                    // its slices [s0, s1)
    };
    struct Piece {
        unsigned char* dst;
        const unsigned char* src;
        size_t bytes;
        int slice;
    };
    std::vector<Group> groups;
    for (int m = 0; m < 2; ++m)
        if (!jm[m].empty())
            for (int g = 0; g < G; ++g)
                groups.push_back({m, (int)((int64_t)B * g / G), (int)((int64_t)B * (g + 1) / G), 0, 0});
    // staging offsets: array-major, as download_staged lays them out
    std::vector<size_t> job_off[2];
    size_t off = 0;
    for (int m = 0; m < 2; ++m)
        for (const CopyJob& j : jm[m]) {
            job_off[m].push_back(off);
            off += (j.bytes + 255) & ~(size_t)255;
        }
    // slices in publication order (group-major): slice g.s0 + k is array k of group g;
    // slice_ev[s] is the event recorded after its copy (set when queued, before publication)
    std::vector<int> slice_ev;
    std::vector<Piece> pieces;
    const size_t kPiece = (size_t)1 << 20;
    for (Group& g : groups) {
        g.s0 = (int)slice_ev.size();
        for (size_t k = 0; k < jm[g.m].size(); ++k) {
            const CopyJob& j = jm[g.m][k];
            const size_t row = j.bytes / (size_t)B;    // bytes of one instance
            const size_t o = (size_t)g.b0 * row, n = (size_t)(g.b1 - g.b0) * row;
            const int si = (int)slice_ev.size();
            slice_ev.push_back(-1);
            for (size_t q = 0; q < n; q += kPiece)
                pieces.push_back({(unsigned char*)j.dst + o + q, e->pin + job_off[g.m][k] + o + q, std::min(kPiece, n - q), si});
        }
        g.s1 = (int)slice_ev.size();
    }
    std::atomic<size_t> next{0}, next_pop{0};
    std::atomic<int> published{0};                     // slices queued (publication order)
    std::atomic<bool> bad{false};
    auto work = [&](bool populate) {
        if (populate)                                  // while the first instances still compute
            for (size_t i; (i = next_pop.fetch_add(1)) < jm[0].size() + jm[1].size();) {
                const CopyJob& j = i < jm[0].size() ? jm[0][i] : jm[1][i - jm[0].size()];
                populate_write(j.dst, j.bytes);
            }
        for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
            const int si = pieces[i].slice;
            while (published.load(std::memory_order_acquire) <= si) {
                if (bad.load()) return;
                std::this_thread::sleep_for(std::chrono::microseconds(10));
            }
            if (hipEventSynchronize(e->ev[slice_ev[si]]) != hipSuccess) {
                bad = true;
                return;
            }
            std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].bytes);
        }
    };
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nthr = (int)std::min<size_t>({8, hw, pieces.size() + 1});
    std::vector<std::thread> th;
    try {
        th.reserve((size_t)std::max(0, nthr - 1));
        for (int t = 1; t < nthr; ++t) th.emplace_back(work, true);
    } catch (...) {
    }
    // the calling thread watches the flags and queues each finished group's copies
    const volatile uint32_t* fl = e->flags;
    bool joined[2] = {false, false};
    int signalled = 0;
#ifdef RL_OVL_TRACE     // diagnostic builds: when each group was queued, and the kernel's end
    g_tr.pub.assign(groups.size(), -1.0);
#endif
    auto group_done = [&](const Group& g) {
        for (int b = g.b0; b < g.b1; ++b)
            if (fl[(size_t)g.m * B + b] != epoch) return false;
        return true;
    };
    int next_ev = 0;
    for (size_t gi = 0; gi < groups.size() && !bad.load();) {
        const Group& g = groups[gi];
        for (int b = g.b0;;) {
            while (b < g.b1 && fl[(size_t)g.m * B + b] == epoch) ++b;
            if (b == g.b1) break;
            if (joined[g.m]) break;
            const hipError_t q = hipEventQuery(p->ev_end[g.m]);
            if (q == hipSuccess) {
                // the kernel has ended: every flag it stored is visible now, so a flag that
                // arrived between the read above and the query counts as signalled
                while (b < g.b1 && fl[(size_t)g.m * B + b] == epoch) ++b;
                if (b == g.b1) break;
                // ended without this flag: stream order from here on
                if (hipStreamWaitEvent(e->dl, p->ev_end[g.m], 0) != hipSuccess) bad = true;
                joined[g.m] = true;
                break;
            }
            if (q != hipErrorNotReady) {
                bad = true;
                break;
            }
            std::this_thread::yield();
        }
        if (bad.load()) break;
        // the batch: this group and every following group of the mode that is complete too
        // (after the kernel's end, all of them) -- one copy per array over the batch, so a
        // burst of finishing instances moves as few large copies (1 MB copies ran at ~21 GB/s,
        // against 56 GB/s for large ones: round-6 trace)
        size_t ge = gi + 1;
        while (ge < groups.size() && groups[ge].m == g.m && (joined[g.m] || group_done(groups[ge]))) ++ge;
        const Group& gl = groups[ge - 1];
        for (size_t k = 0; k < jm[g.m].size() && !bad.load(); ++k) {
            const CopyJob& j = jm[g.m][k];
            const size_t row = j.bytes / (size_t)B;
            const size_t o = (size_t)g.b0 * row, n = (size_t)(gl.b1 - g.b0) * row;
            const int ev = std::min(next_ev++, kJobEvents - 1);   // (a reused event only waits longer)
            if (hipMemcpyAsync(e->pin + job_off[g.m][k] + o, (const unsigned char*)j.src + o, n, hipMemcpyDeviceToHost,
                               e->dl) != hipSuccess ||
                hipEventRecord(e->ev[ev], e->dl) != hipSuccess)
                bad = true;
            for (size_t h = gi; h < ge; ++h) slice_ev[groups[h].s0 + k] = ev;
        }
        if (bad.load()) break;
        published.store(gl.s1, std::memory_order_release);
        for (size_t h = gi; h < ge; ++h) {
            if (!joined[g.m]) ++signalled;
#ifdef RL_OVL_TRACE
            g_tr.pub[h] = tr_ms();
#endif
        }
        gi = ge;
    }
#ifdef RL_OVL_TRACE
    if (hipEventSynchronize(p->ev_end[groups.back().m]) == hipSuccess) g_tr.kend = tr_ms();
    if (!slice_ev.empty() && slice_ev.back() >= 0 && hipEventSynchronize(e->ev[slice_ev.back()]) == hipSuccess)
        g_tr.dma = tr_ms();
    g_tr.nthr = nthr;
#endif
    work(false);
    for (auto& t : th) t.join();
#ifdef RL_OVL_TRACE
    g_tr.copied = tr_ms();
#endif
    const bool synced = hipStreamSynchronize(e->dl) == hipSuccess;
    if (bad.load() || !synced) return fail(RL_EHIP, "download (overlapped) failed");
    g_last_groups = (int)groups.size();
    g_last_groups_signalled = signalled;
    return RL_OK;
}

// rl_optimize / rl_lap_eval through the plan cache (see above).  kms[0..2]: HIP-event
// times of the whole run, the min-curvature and the min-time kernel (-1 if not run).
int run_cached(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds, int32_t B,
               int32_t modes, const double* centers, const double* Ls, rl_out* out_mc, rl_out* out_mt, float* kms) {
    const auto t0 = std::chrono::steady_clock::now();
#ifdef RL_OVL_TRACE
    g_tr = OvlTrace{};
    g_tr.t0 = t0;
#endif
    g_last_kernel_ms = g_last_call_ms = g_last_mode_ms[0] = g_last_mode_ms[1] = -1.0f;
    g_last_groups = g_last_groups_signalled = 0;
    if (int rc = check_inputs(prob, cfg, n_cfg, B, modes, centers)) return rc;
    int ndev = 0, dev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= ndev) dev = 0;
    CacheEntry key;
    key.device = dev;
    key.N = prob->N;
    key.B = B;
    key.ncfg = n_cfg;
    key.mo = cfg[0].max_outer_iters;
    key.closed = prob->closed ? 1 : 0;
    key.Ei = prob->Ei;
    key.Eo = prob->Eo;
    key.stream = use_stream(prob->N);
    key.centers = centers != nullptr;
    key.Ls = Ls != nullptr;
    key.segs.assign(prob->inner_seg, prob->inner_seg + 4 * (size_t)prob->Ei);
    key.segs.insert(key.segs.end(), prob->outer_seg, prob->outer_seg + 4 * (size_t)prob->Eo);
    PlanCache& pc = plan_cache();
    CacheEntry* e = pc.take(key);
    const size_t N2 = 2 * (size_t)std::max(prob->N, 1);
    const size_t up_ctr = prob->N > 0 ? (centers ? (size_t)B : 1) * N2 * sizeof(double) : 0;
    const size_t up_ls = Ls ? (size_t)B * sizeof(double) : 0;
    const size_t up_cfg = (size_t)n_cfg * sizeof(rl_cfg), up_seed = (size_t)B * sizeof(uint64_t);
    const size_t up_bytes = ((up_ctr + 255) & ~(size_t)255) + ((up_ls + 255) & ~(size_t)255) +
                            ((up_cfg + 255) & ~(size_t)255) + up_seed;
    int rc = RL_OK;
    auto drop = [&](int code) {
        const std::string msg = g_err;
        destroy_entry(e);
        g_err = msg;
        return code;
    };
    if (!e) {
        rl_plan* p = nullptr;
        if ((rc = plan_create_ex(&p, dev, prob, cfg, n_cfg, seeds, B, modes, centers, Ls))) return rc;
        e = new CacheEntry(std::move(key));
        e->p = p;
        for (hipEvent_t& v : e->ev)
            if (hipEventCreateWithFlags(&v, hipEventDisableTiming) != hipSuccess) return drop(fail(RL_EHIP, "hipEventCreate failed"));
    } else {
        rl_plan* p = e->p;
        if (hipSetDevice(p->device) != hipSuccess) return drop(fail(RL_EHIP, "hipSetDevice failed"));
        for (int m = 0; m < 2; ++m)
            if ((modes & (1 << m)) && (rc = alloc_mode(p, m))) return drop(rc);
        p->L = prob->L;
        p->veh_width = prob->veh_width;
        if ((rc = ensure_pinned(e, up_bytes))) return drop(rc);
        hipStream_t st = p->own_stream;
        size_t off = 0;
        auto up = [&](void* d, const void* h, size_t bytes) -> bool {
            if (!bytes) return true;
            std::memcpy(e->pin + off, h, bytes);
            const bool ok = hipMemcpyAsync(d, e->pin + off, bytes, hipMemcpyHostToDevice, st) == hipSuccess;
            off += (bytes + 255) & ~(size_t)255;
            return ok;
        };
        std::vector<uint64_t> sd;
        if (!seeds) sd.assign((size_t)B, 0);
        if (!up(p->d_center, centers ? centers : prob->center_xy, up_ctr) || !up(p->d_Ls, Ls, up_ls) ||
            !up(p->d_cfg, cfg, up_cfg) || !up(p->d_seeds, seeds ? seeds : sd.data(), up_seed))
            return drop(fail(RL_EHIP, "upload (staged) failed"));
        set_margin(p, cfg, n_cfg);
    }
    rl_plan* p = e->p;
    p->modes = modes;
    std::vector<CopyJob> jm[2], jobs;
    out_jobs(p, 0, (modes & RL_MODE_MINCURV) ? out_mc : nullptr, jm[0]);
    out_jobs(p, 1, (modes & RL_MODE_MINTIME) ? out_mt : nullptr, jm[1]);
    jobs = jm[0];
    jobs.insert(jobs.end(), jm[1].begin(), jm[1].end());
    // the staging area serves the uploads first, then (after the kernel has started, or
    // stream-ordered after it) the downloads; a reallocation waits for the uploads queued
    const size_t down_bytes = staged_bytes(jobs);
    if (down_bytes > e->pin_bytes) {
        if (hipStreamSynchronize(p->own_stream) != hipSuccess) return drop(fail(RL_EHIP, "upload sync"));
        if ((rc = ensure_pinned(e, down_bytes))) return drop(rc);
    }
    const bool overlap = overlap_enabled() && p->N > 0 && B >= 2 && down_bytes >= kOverlapMinBytes;
    uint32_t epoch = 0;
    if (overlap) {
        if ((rc = ensure_flags(e, B))) return drop(rc);
        uint32_t* dflags = nullptr;
        if (hipHostGetDevicePointer((void**)&dflags, e->flags, 0) != hipSuccess || !dflags)
            return drop(fail(RL_EHIP, "hipHostGetDevicePointer (completion flags) failed"));
        if (++e->epoch == 0) {                         // wrapped: no flag may hold the new epoch
            std::memset(e->flags, 0, (size_t)e->flags_n * sizeof(uint32_t));
            e->epoch = 1;
        }
        epoch = e->epoch;
        p->epoch = epoch;
        // (test hook RL_OVERLAP_TEST_NOSIGNAL=1: the kernels do not signal, so every group takes
        // the stream-ordered fallback after the kernel's end -- tests/test_gpu_parity.py)
        const char* ns = std::getenv("RL_OVERLAP_TEST_NOSIGNAL");
        const bool nosig = ns && ns[0] == '1';
        for (int m = 0; m < 2; ++m) p->done[m] = (jm[m].empty() || nosig) ? nullptr : dflags + (size_t)m * B;
    }
    rc = rl_plan_run(p, nullptr);
#ifdef RL_OVL_TRACE
    g_tr.launched = tr_ms();
#endif
    p->done[0] = p->done[1] = nullptr;                 // later runs of this plan signal nothing
    if (rc) return drop(rc);
    if (overlap) rc = download_overlapped(e, p, jm, epoch);
    else rc = download_staged(e, p->own_stream, jobs, 0);
    if (rc) return drop(rc);
    if (hipStreamSynchronize(p->own_stream) != hipSuccess) return drop(fail(RL_EHIP, "stream sync"));
    float ms[3] = {-1.0f, -1.0f, -1.0f};
    for (int i = 0; i < 3; ++i) {
        const bool has = i == 0 || (i == 1 && (modes & RL_MODE_MINCURV)) || (i == 2 && (modes & RL_MODE_MINTIME));
        if (has && (rc = rl_plan_kernel_ms(p, i, &ms[i]))) return drop(rc);
    }
    if (kms) std::memcpy(kms, ms, sizeof(ms));
    pc.give(e);
    g_last_kernel_ms = ms[0];
    g_last_mode_ms[0] = ms[1];
    g_last_mode_ms[1] = ms[2];
    g_last_call_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
#ifdef RL_OVL_TRACE
    std::fprintf(stderr, "{\"ovl_trace\": {\"launched_ms\": %.3f, \"kernel_ms\": %.3f, \"kernel_end_seen_ms\": %.3f, "
                 "\"dma_done_ms\": %.3f, \"copies_done_ms\": %.3f, \"return_ms\": %.3f, \"threads\": %d, \"published_ms\": [",
                 g_tr.launched, ms[1] > 0 ? ms[1] : ms[2], g_tr.kend, g_tr.dma, g_tr.copied, tr_ms(), g_tr.nthr);
    for (size_t i = 0; i < g_tr.pub.size(); ++i) std::fprintf(stderr, "%s%.3f", i ? ", " : "", g_tr.pub[i]);
    std::fprintf(stderr, "]}}\n");
#endif
    return RL_OK;
}

}  // namespace

extern "C" {

int rl_optimize(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds, int32_t B,
                rl_out* out_mincurv, rl_out* out_mintime) {
    int modes = (out_mincurv ? RL_MODE_MINCURV : 0) | (out_mintime ? RL_MODE_MINTIME : 0);
    if (!modes) return fail(RL_EINVAL, "no output requested");
    return run_cached(prob, cfg, n_cfg, seeds, B, modes, nullptr, nullptr, out_mincurv, out_mintime, nullptr);
}

int rl_last_call_ms(float* kernel_ms, float* call_ms) {
    if (g_last_call_ms < 0.0f) return fail(RL_EINVAL, "no successful rl_optimize / rl_lap_eval on this thread");
    if (kernel_ms) *kernel_ms = g_last_kernel_ms;
    if (call_ms) *call_ms = g_last_call_ms;
    return RL_OK;
}

int rl_last_call_times(float* run_ms, float* mincurv_ms, float* mintime_ms, float* call_ms) {
    if (g_last_call_ms < 0.0f) return fail(RL_EINVAL, "no successful rl_optimize / rl_lap_eval on this thread");
    if (run_ms) *run_ms = g_last_kernel_ms;
    if (mincurv_ms) *mincurv_ms = g_last_mode_ms[0];
    if (mintime_ms) *mintime_ms = g_last_mode_ms[1];
    if (call_ms) *call_ms = g_last_call_ms;
    return RL_OK;
}

int rl_last_call_download(int32_t* groups, int32_t* groups_signalled) {
    if (g_last_call_ms < 0.0f) return fail(RL_EINVAL, "no successful rl_optimize / rl_lap_eval on this thread");
    if (groups) *groups = g_last_groups;
    if (groups_signalled) *groups_signalled = g_last_groups_signalled;
    return RL_OK;
}

int rl_plan_cache_info(int32_t* entries, int64_t* device_bytes, int64_t* pinned_bytes) {
    plan_cache().info(entries, device_bytes, pinned_bytes);
    return RL_OK;
}

int rl_release_plan_cache(void) {
    int dev = 0;
    const bool have = hipGetDevice(&dev) == hipSuccess;
    plan_cache().clear();
    if (have) hipSetDevice(dev);
    return RL_OK;
}

// rl_optimize over several devices (SURVEY §8b device list, §8e): contiguous instance
// blocks, one plan and stream per device, every device enqueued before the first
// download, and each block's results copied to its offset of the caller's host outputs
// (the final gather).  Instances never span devices: block d holds [b0_d, b1_d).
int rl_optimize_multi(const rl_problem* prob, const rl_cfg* cfg, int32_t n_cfg, const uint64_t* seeds, int32_t B,
                      const int32_t* devices, int32_t n_dev, rl_out* out_mincurv, rl_out* out_mintime) {
    int modes = (out_mincurv ? RL_MODE_MINCURV : 0) | (out_mintime ? RL_MODE_MINTIME : 0);
    if (!modes) return fail(RL_EINVAL, "no output requested");
    if (n_dev < 1) return fail(RL_EINVAL, "n_dev must be >= 1");
    // every cfg (all blocks) is checked up front: the output offsets below use cfg[0]'s
    // max_outer_iters for every block
    if (int rc0 = check_inputs(prob, cfg, n_cfg, B, modes, nullptr)) return rc0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RL_ENODEV, "no HIP device");
    std::vector<int> devs((size_t)n_dev);
    for (int d = 0; d < n_dev; ++d) {
        devs[d] = devices ? devices[d] : d;
        if (devs[d] < 0 || devs[d] >= ndev) return fail(RL_ENODEV, "device index out of range");
    }
    int cur = 0;
    const bool restore = hipGetDevice(&cur) == hipSuccess;
    const int nb = std::min(n_dev, B);             // no empty blocks
    const int mo = cfg[0].max_outer_iters;
    const size_t N = (size_t)std::max(prob->N, 0);
    std::vector<rl_plan*> plans((size_t)nb, nullptr);
    auto release = [&](int code) {
        std::string e = g_err;
        for (rl_plan* q : plans) rl_plan_destroy(q);
        if (restore) hipSetDevice(cur);
        g_err = e;
        return code;
    };
    auto block = [&](int d, int& b0, int& b1) {
        b0 = (int)((int64_t)B * d / nb);
        b1 = (int)((int64_t)B * (d + 1) / nb);
    };
    int rc;
    for (int d = 0; d < nb; ++d) {
        int b0, b1;
        block(d, b0, b1);
        // every block takes the kernel shape rl_optimize would take for the whole batch, so
        // the results equal rl_optimize's bit for bit (the shapes' J / lap sum orders differ)
        if ((rc = rl_plan_create(&plans[d], devs[d], prob, n_cfg == 1 ? cfg : cfg + b0, n_cfg == 1 ? 1 : b1 - b0,
                                 seeds ? seeds + b0 : nullptr, b1 - b0, modes)) ||
            (rc = rl_plan_set_shape_batch(plans[d], B)) || (rc = rl_plan_run(plans[d], nullptr)))
            return release(rc);
    }
    auto shifted = [&](const rl_out* o, int b0, rl_out& s) -> rl_out* {
        if (!o) return nullptr;
        s = *o;
        const size_t bn = (size_t)b0 * N;
        double** f[] = {&s.x, &s.y, &s.heading, &s.kappa, &s.alpha_total, &s.alpha_last, &s.v, &s.ax};
        for (double** q : f)
            if (*q) *q += bn;
        if (s.lap) s.lap += b0;
        if (s.evals) s.evals += (size_t)b0 * mo;
        if (s.accepts) s.accepts += (size_t)b0 * mo;
        if (s.vpass_sweeps) s.vpass_sweeps += (size_t)b0 * (mo + 1);
        return &s;
    };
    for (int d = 0; d < nb; ++d) {
        int b0, b1;
        block(d, b0, b1);
        rl_out smc, smt;
        if ((rc = rl_plan_fetch(plans[d], shifted(out_mincurv, b0, smc), shifted(out_mintime, b0, smt))))
            return release(rc);
    }
    return release(RL_OK);
}

#ifdef RL_STAMPS
// diagnostic builds only: per-phase cycle totals of the last launch (see rl_kernels.hip)
int rl_debug_stamps(unsigned long long* host, int nblocks) { return rl::debug_stamps(host, nblocks); }
int rl_debug_stamps_stream(unsigned long long* host, int nblocks) { return rl::debug_stamps_stream(host, nblocks); }
int rl_debug_stamps_lat(unsigned long long* host, int nblocks) { return rl::debug_stamps_lat(host, nblocks); }
int rl_debug_stamps_mid(unsigned long long* host, int nblocks) { return rl::debug_stamps_mid(host, nblocks); }
#endif
#ifdef RL_COUNT
// diagnostic builds only: corridor work counters of the stream kernel's translation unit
int rl_debug_counts(unsigned long long* host, int reset) { return rl::debug_counts(host, reset); }
int rl_debug_counts_geom(unsigned long long* host, int reset) { return rl::debug_counts_geom(host, reset); }
int rl_debug_counts_reg(unsigned long long* host, int reset) { return rl::debug_counts_reg(host, reset); }
#endif

}  // extern "C"
