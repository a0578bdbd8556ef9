/*
 * rt_capi.cpp — implementation of include/rt_capi.h (host side, HIP runtime).
 *
 * Owns the device scene (one HBM allocation in the layout of rt_device.h), a stream,
 * timing events and a staging buffer for host-output renders.  No exception crosses
 * the boundary; every entry point returns an rt_status.
 */
#ifndef RT_CLUSTER_COS_DEFAULT  // build-time default of RT_OPT_CLUSTER_COS (x 1000)
#define RT_CLUSTER_COS_DEFAULT 400
#endif
#ifndef RT_CLU_SAH  // 1: sphere clusters from surface-area splits instead of median splits
#define RT_CLU_SAH 1  // (A/B round 4, bitwise equal: c5 PATH64 -0.9%, F64 -0.4%, F32 -1.1%; c3 +-1%)
#endif
#ifndef RT_WALL_ORDER_DEFAULT   // build-time default of RT_OPT_WALL_ORDER (A/B builds)
#define RT_WALL_ORDER_DEFAULT 0
#endif
#ifndef RT_PIXEL_PAIRS_DEFAULT  // build-time default of RT_OPT_PIXEL_PAIRS (A/B builds)
#define RT_PIXEL_PAIRS_DEFAULT 0
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/rt_capi.h"
#include "rt_device.h"
#include <chrono>

#ifndef RT_DRY_LAUNCH     // diagnostic build: 1 = no kernel launch in rt_render_device*,
#define RT_DRY_LAUNCH 0   // 2 = nor rt_multi's per-frame runtime calls (never in the product)
#endif
#ifndef RT_HOST_PROFILE   // diagnostic build: per-phase host time of rt_render_device, printed
#define RT_HOST_PROFILE 0 // to stderr by rt_ctx_destroy (never in the product)
#endif
#if RT_HOST_PROFILE
static double g_hp[5];
static long g_hn;
static inline double hp_now() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define HP(i) (g_hp[(i)] += (g_hn > 50 ? hp_now() - hp_t : 0.0), hp_t = hp_now())  // warm calls only
#else
#define HP(i) ((void)0)
#endif

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    void* d_scene = nullptr;
    size_t scene_bytes = 0;
    bool have_scene = false;
    struct SceneHost {
        int nS = 0, nW = 0, nP = 0;
        bool int_exp = true;
        size_t off_s64 = 0, off_w32 = 0, off_w64 = 0, off_sj = 0, off_wj = 0, off_mat = 0,
               off_mat32 = 0, off_wnn = 0, total = 0;
        struct CluSet {  // sphere clusters (rt_device.h) of one leaf size, nclu 0 = none
            size_t off_clu = 0, off_csph = 0, off_cord = 0;
            int nclu = 0, clu_axis = 0, ls = 0;
            float clu_oinf = 0.0f;
        } cset[2];  // [0]: the F32 kernels' (CLU_SIZE), [1]: the fp64 kernels' (CLU_SIZE_D)
        // the device image of the scene (rt_device.h layout), built in 256-byte aligned host
        // memory so its records (alignas 32-128) may be written through their own types
        struct alignas(256) Blk {
            char b[256];
        };
        std::vector<Blk> blocks;
        char* image() { return reinterpret_cast<char*>(blocks.data()); }
        std::vector<double> h_sph;  // nS x {cx, cy, cz, radius^2, radius}
        std::vector<double> h_wal;  // nW x {P, n, X, Y, length, width}
        std::vector<double> h_km;   // metallic of each material slot
    } sc;
    unsigned long long* d_stats = nullptr;
    int wave_cull_min = 24;  // spheres from which the wave cull pays (tools/sweep.py)
    bool eye_tables = true;  // RT_OPT_EYE_TABLES
    float clu_cos = RT_CLUSTER_COS_DEFAULT / 1000.0f;  // RT_OPT_CLUSTER_COS
    bool wall_order = RT_WALL_ORDER_DEFAULT;  // RT_OPT_WALL_ORDER
    bool tile_bins = true;   // RT_OPT_TILE_BINS
    bool row_order = true;   // RT_OPT_ROW_ORDER
    bool mirror_bins = true; // RT_OPT_MIRROR_BINS
    std::vector<int16_t> row_perm;  // rt_set_row_order: explicit tile-row dispatch order
    // Row feedback (RT_OPT_ROW_FEEDBACK): every render records each wave's cost
    // (KParams::tile_cost); every `feedback` frames a snapshot is copied to pinned host
    // memory behind the kernel and, once it has landed, the tile rows are ordered by their
    // most expensive tile (heaviest first) for the following renders of the same band.
    // Only the dispatch order changes: every tile is traced once per frame either way.
    int feedback = 32;             // refresh interval in frames, 0 = off
    bool pixel_pairs = RT_PIXEL_PAIRS_DEFAULT;  // RT_OPT_PIXEL_PAIRS
    uint16_t* d_cost = nullptr;    // device, d_cost_cap entries (one per wave)
    size_t d_cost_cap = 0;
    uint32_t* d_umax = nullptr;    // device, per dispatch unit: its most expensive wave
    uint32_t* h_umax = nullptr;    // pinned host snapshot of d_umax
    size_t umax_cap = 0;
    int cost_ul = 0;               // units per tile row (log2) of the pending snapshot
    hipEvent_t ev_cost = nullptr;  // snapshot landed
    bool cost_pending = false;
    // RT_OPT_ROW_FEEDBACK_ISOLATE (default 0): a sampled frame runs alone on the GPU — its
    // stream waits for the other streams' latest frames, and each other stream's next frame
    // waits for it — so its wave costs are not those of two frames sharing the CUs (frames
    // in flight overlap a frame's tail with the next one's start, which inflated or hid the
    // costs of the tiles dispatched first and could install a worse order for 32 frames)
    bool fb_isolate = false;
    hipEvent_t ev_iso = nullptr;         // recorded behind the sampled frame
    bool iso_pending = false;
    std::vector<hipStream_t> iso_seen;   // streams already ordered behind ev_iso
    struct Band {
        int32_t W = -1, row0 = -1, nrows = -1;
        unsigned long long scene_gen = 0;
        unsigned fb_epoch = 0;  // rt_set_option(RT_OPT_ROW_FEEDBACK) starts a new epoch
        int32_t tstride = 0, tphase = 0;  // interleaved parts (KParams::tstride)
        bool operator==(const Band& o) const {
            return W == o.W && row0 == o.row0 && nrows == o.nrows && scene_gen == o.scene_gen &&
                   fb_epoch == o.fb_epoch && tstride == o.tstride && tphase == o.tphase;
        }
    };
    unsigned fb_epoch = 0;  // a snapshot still in flight from an older epoch is not used
    Band cost_band;                // band of the pending snapshot
    Band fb_band;                  // band fb_perm was computed for
    std::vector<int16_t> fb_perm;  // over dispatch units: 2^fb_units_log2 per tile row
    int fb_units_log2 = 0;
    // RT_OPT_ROW_FEEDBACK_EMA: per-unit cost smoothed over the snapshots of one band
    // (acc = w*acc + (1-w)*new), so one noisy snapshot (tile costs measured while another
    // frame's waves shared the GPU) does not reorder the rows on its own; 0 = off
    int fb_ema = 0;                // w in percent
    std::vector<float> fb_acc;     // per dispatch unit, for fb_band

    int since_snapshot = 0;
    // RT_OPT_ROW_FEEDBACK_WARM: after a new band or scene, this many further snapshots are
    // taken back to back (each as soon as the previous one has landed) before the interval
    // applies, so the order settles within a few frames instead of a few intervals
    int fb_warm = 0;
    int warm_left = 0;
    // the per-frame boxes depend only on the scene, the camera, the row band and the
    // options: a render with the same inputs as the previous one reuses them (the host
    // part of a frame is ~60 us with mirror chains, more than the kernel at c2)
    struct BoxCache {
        bool valid = false;
        unsigned long long scene_gen = 0;
        rt_camera cam{};
        int32_t row0 = 0, nrows = 0, wave_cull = 0, opts = 0;
        int32_t nbox = 0, nwbox = 0, row_center = 0, mir_depth = 0;
        size_t nmbox = 0;
        rt::PrimBox box[rt::BIN_MAX_PRIMS];
        rt::PrimBox mbox[rt::MIR_MAX_BOXES];
    };
    mutable BoxCache box_cache;
    bool box_cache_on = true;  // RT_OPT_BOX_CACHE
    unsigned long long scene_gen = 0;  // bumped by every rt_set_scene
    void* d_out = nullptr;
    size_t d_out_cap = 0;
    unsigned long long* d_segs = nullptr;
    // Renders enqueued on caller streams (rt_render_device): per stream, an event recorded
    // behind its latest launch.  rt_set_scene and rt_ctx_destroy wait on every one of them
    // before they overwrite or free the device scene, so a frame still in flight on a
    // non-blocking stream never reads a half-replaced scene.
    struct Inflight {
        hipStream_t stream;
        hipEvent_t ev;
    };
    std::vector<Inflight> inflight;
    // RT_OPT_HOST_PIPELINE: rt_render_device_frames computes frame f+1's kernel arguments
    // (pixel boxes, mirror chains, eye tables: make_params) on a helper thread while this
    // thread launches frame f (see render_frames_pipelined)
    bool host_pipeline = true;
    struct Prep;
    Prep* prep = nullptr;
    // RT_OPT_FRAME_BATCH: the pipelined frame loop launches up to frame_batch consecutive
    // frames that share a stream as ONE grid (frame = blockIdx.z, rt::launch_trace_batch),
    // their kernel arguments in a device table copied from pinned memory in front of the
    // launch.  TAB_SLOTS groups may be in flight; a slot is reused once its launch (whose
    // stop event is tab_ev[slot]) has completed.
    int frame_batch = 1;
    static constexpr int TAB_SLOTS = 64;
    rt::KParams* h_tab = nullptr;  // pinned, TAB_SLOTS x RT_MULTI_BATCH_MAX
    rt::KParams* d_tab = nullptr;  // device, the same
    hipEvent_t tab_ev[TAB_SLOTS] = {};
    bool tab_busy[TAB_SLOTS] = {};
    int tab_next = 0;
    char last_err[256] = {0};
};

namespace {

int hip_fail(rt_ctx* ctx, hipError_t e, const char* what) {
    if (ctx)
        std::snprintf(ctx->last_err, sizeof ctx->last_err, "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_HIP;
}

#define RT_HIP(ctx, call)                                   \
    do {                                                    \
        hipError_t e_ = (call);                             \
        if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
    } while (0)

/* Makes the ctx's device current for the duration of an entry point and restores the
 * caller's current device on every return path (the boundary must not change it). */
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) err = hipSetDevice(device);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};

/* Before a launch on `st` (a caller stream): the stream's in-flight event, which the
 * launch signals on completion (rt::launch_trace's done_event); null for ctx->stream. */
#ifndef RT_TRACK_STREAMS
#define RT_TRACK_STREAMS 1
#endif
int launch_event(rt_ctx* ctx, hipStream_t st, hipEvent_t* ev) {
    *ev = nullptr;
    if (!RT_TRACK_STREAMS || st == ctx->stream) return RT_OK;  // rt_set_scene syncs ctx->stream
    for (auto& f : ctx->inflight)
        if (f.stream == st) {
            *ev = f.ev;
            return RT_OK;
        }
    constexpr size_t kMaxStreams = 16;
    if (ctx->inflight.size() >= kMaxStreams) {
        // many distinct streams: retire the oldest entry (wait for its frame) and reuse it
        rt_ctx::Inflight f = ctx->inflight.front();
        RT_HIP(ctx, hipEventSynchronize(f.ev));
        ctx->inflight.erase(ctx->inflight.begin());
        f.stream = st;
        ctx->inflight.push_back(f);
        *ev = f.ev;
        return RT_OK;
    }
    rt_ctx::Inflight f{st, nullptr};
    RT_HIP(ctx, hipEventCreate(&f.ev));
    ctx->inflight.push_back(f);
    *ev = f.ev;
    return RT_OK;
}

/* Every render this ctx has enqueued, on any stream, has finished. */
int wait_inflight(rt_ctx* ctx) {
    if (ctx->stream) RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (auto& f : ctx->inflight) RT_HIP(ctx, hipEventSynchronize(f.ev));
    for (int s = 0; s < rt_ctx::TAB_SLOTS; s++)  // batched launches (RT_OPT_FRAME_BATCH)
        if (ctx->tab_busy[s]) {
            RT_HIP(ctx, hipEventSynchronize(ctx->tab_ev[s]));
            ctx->tab_busy[s] = false;
        }
    return RT_OK;
}

/* vec.cpp restatements used to pack Wall invariants (same fp64 operations). */
struct hv3 {
    double x, y, z;
};
hv3 hcross(hv3 u, hv3 v) {  // vec.cpp:15
    return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
hv3 hnormalize(hv3 v) {  // vec.cpp:21 (v / length())
    double l = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    return {v.x / l, v.y / l, v.z / l};
}
bool hnan(hv3 v) { return std::isnan(v.x) || std::isnan(v.y) || std::isnan(v.z); }

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

int bytes_per_pixel(int32_t f) {
    switch (f) {
        case RT_OUT_RGB_F32: return 12;
        case RT_OUT_RGB_F64: return 24;
        case RT_OUT_RGBA8: return 4;
        case RT_OUT_RGBA8_WRAP: return 4;
        default: return 0;
    }
}

int check_render_args(const rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                      int32_t depth, int32_t precision, int32_t out_format) {
    if (!ctx || !cam) return RT_ERR_INVALID_ARG;
    if (!ctx->have_scene) return RT_ERR_NO_SCENE;
    if (cam->width < 0 || cam->height < 0 || nrows < 0) return RT_ERR_INVALID_ARG;
    if (row0 < 0 || row0 + nrows > cam->height) return RT_ERR_OUT_OF_RANGE;
    if (depth < 0) return RT_ERR_INVALID_ARG;
    if (depth > rt::max_depth()) return RT_ERR_UNSUPPORTED;
    if (precision < RT_PREC_F64 || precision > RT_PREC_PATH64) return RT_ERR_INVALID_ARG;
    if (bytes_per_pixel(out_format) == 0) return RT_ERR_INVALID_ARG;
    return RT_OK;
}

/* ---- primary-ray tile bins (rt_device.h PrimBox) -------------------------------------
 * A point X = o + u*d(x, i) of a primary ray has (u, u*x, u*i) = M^-1 (X - o) with
 * M = [o - TL, -dx, -dy] (columns), d(x, i) = o - (TL + dx*x + dy*i) (main.cpp:132-133).
 * The box of a convex hull is the box of its projected vertices (the map is projective,
 * convexity-preserving on u > 0), floor/ceil'd and widened by one pixel.  Conditions
 * that make the box a proof (DESIGN.md §3 "tile bins"):
 *   - a primitive is only boxed when the camera is clearly off it (sphere: |o - C| >
 *     r*sqrt(3) + delta; wall: |num| = |(P - o).n| > 1e-9 * scale, below which rounding of
 *     a near-grazing ray's t could be arbitrary), otherwise it keeps every tile;
 *   - hull entirely at u < 0: the line meets it behind the camera only (t < 0), never;
 *   - wall polygon clipped to u >= eps = |num| / (2 max|d|): hits at u < eps would lie
 *     closer to o than the wall's plane, impossible;
 *   - a sphere hull straddling u = 0 keeps every tile.
 * Outside the box by >= 1 pixel the exact ray misses the hull by an angle of ~1 pixel
 * while the reference's rounding moves a hit by ~1e-13 pixel (both scale alike with the
 * grazing angle), so the reference's test rejects the primitive as well. */
struct Proj {
    double r[3][3];  // rows of M^-1
    double o[3];
};
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline void cross3(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}
bool make_proj(const rt_camera* cam, Proj& P) {
    double e[3], c1[3], c2[3];
    for (int k = 0; k < 3; k++) {
        P.o[k] = cam->position[k];
        e[k] = cam->position[k] - cam->image_top_left[k];
        c1[k] = -cam->pixel_delta_x[k];
        c2[k] = -cam->pixel_delta_y[k];
    }
    double x12[3], x20[3], x01[3];
    cross3(c1, c2, x12);
    cross3(c2, e, x20);
    cross3(e, c1, x01);
    const double det = dot3(e, x12);
    if (!(std::fabs(det) > 0) || !std::isfinite(det)) return false;
    for (int k = 0; k < 3; k++) {
        P.r[0][k] = x12[k] / det;
        P.r[1][k] = x20[k] / det;
        P.r[2][k] = x01[k] / det;
    }
    return true;
}
inline double proj_u(const Proj& P, const double* X) {
    const double v[3] = {X[0] - P.o[0], X[1] - P.o[1], X[2] - P.o[2]};
    return dot3(P.r[0], v);
}
struct BoxAcc {
    double x0 = INFINITY, x1 = -INFINITY, i0 = INFINITY, i1 = -INFINITY;
    bool bad = false;
    void add(const Proj& P, const double* X) {
        const double v[3] = {X[0] - P.o[0], X[1] - P.o[1], X[2] - P.o[2]};
        const double u = dot3(P.r[0], v);
        const double x = dot3(P.r[1], v) / u, i = dot3(P.r[2], v) / u;
        if (!std::isfinite(x) || !std::isfinite(i) || !(u > 0)) bad = true;
        x0 = std::fmin(x0, x);
        x1 = std::fmax(x1, x);
        i0 = std::fmin(i0, i);
        i1 = std::fmax(i1, i);
    }
};

#ifndef RT_SPHERE_BOX_INTERVAL  // 1: sphere pixel boxes from the exact extent of the ball (two
#define RT_SPHERE_BOX_INTERVAL 1  // quadratics); 0: from the 8 corners of its bounding cube
#endif
/* Boxes of every primitive (material-slot order) for the camera P (origin P.o). */
void boxes_for(const rt_ctx* ctx, const Proj& P, double dmax, int32_t width, int32_t row0,
               int32_t nrows, rt::PrimBox* out, bool spheres = true) {
    const double W = width, R0 = row0, R1 = row0 + nrows - 1;
    const rt::PrimBox all{-1, (int16_t)width, (int16_t)(row0 - 1), (int16_t)(row0 + nrows)};
    const rt::PrimBox none{1, 0, 1, 0};
    auto to_box = [&](const BoxAcc& b) -> rt::PrimBox {
        if (b.bad) return all;
        const double x0 = std::floor(b.x0) - 1, x1 = std::ceil(b.x1) + 1;
        const double i0 = std::floor(b.i0) - 1, i1 = std::ceil(b.i1) + 1;
        if (x0 > W - 1 || x1 < 0 || i0 > R1 || i1 < R0) return none;
        return rt::PrimBox{(int16_t)std::fmax(x0, -1.0), (int16_t)std::fmin(x1, W),
                           (int16_t)std::fmax(i0, R0 - 1), (int16_t)std::fmin(i1, R1 + 1)};
    };
    const double* o = P.o;
    const double oabs = std::fabs(o[0]) + std::fabs(o[1]) + std::fabs(o[2]);
#if RT_SPHERE_BOX_INTERVAL
    // Exact x (and i) extent of the ball: the pixels with p/u = x form the plane
    // (b - x a).(X - o) = 0 through o (a, b, c = rows of M^-1), and it meets the ball
    // |X - C| <= r iff |(b - x a).(C - o)| <= r |b - x a|, i.e. x lies between the roots of
    // (uc^2 - r^2 |a|^2) x^2 - 2 (pc uc - r^2 a.b) x + (pc^2 - r^2 |b|^2) = 0 (the ball wholly
    // in front, u0 > 0, makes the leading coefficient positive).  Rounding is covered by the
    // one-pixel widening of to_box, as for the other hulls.
    const double aa = dot3(P.r[0], P.r[0]), ab = dot3(P.r[0], P.r[1]), ac = dot3(P.r[0], P.r[2]),
                 bb = dot3(P.r[1], P.r[1]), cc = dot3(P.r[2], P.r[2]);
    const double na = std::sqrt(aa);
#endif
    for (int s = 0; s < (spheres ? ctx->sc.nS : 0); s++) {
        const double* S = &ctx->sc.h_sph[5 * s];
        const double r = S[4];
        const double v[3] = {S[0] - o[0], S[1] - o[1], S[2] - o[2]};
        const double delta = 1e-6 * (1 + oabs + std::fabs(S[0]) + std::fabs(S[1]) + std::fabs(S[2]) + r);
        rt::PrimBox b = all;
        if (std::sqrt(dot3(v, v)) > r * 1.7320508075688772 + delta && r > 1e-9 * std::sqrt(dot3(v, v))) {
#if RT_SPHERE_BOX_INTERVAL
            const double uc = dot3(P.r[0], v), pc = dot3(P.r[1], v), qc = dot3(P.r[2], v);
            const double u0 = uc - r * na, u1 = uc + r * na;
            if (u1 < 0) {
                b = none;
            } else if (u0 > 0) {
                const double r2 = r * r;
                const double A = uc * uc - r2 * aa;
                const double Bx = pc * uc - r2 * ab, Cx = pc * pc - r2 * bb;
                const double By = qc * uc - r2 * ac, Cy = qc * qc - r2 * cc;
                const double sx = std::sqrt(std::fmax(0.0, Bx * Bx - A * Cx));
                const double sy = std::sqrt(std::fmax(0.0, By * By - A * Cy));
                BoxAcc acc;
                acc.x0 = (Bx - sx) / A;
                acc.x1 = (Bx + sx) / A;
                acc.i0 = (By - sy) / A;
                acc.i1 = (By + sy) / A;
                acc.bad = !(A > 0) || !std::isfinite(acc.x0) || !std::isfinite(acc.x1) ||
                          !std::isfinite(acc.i0) || !std::isfinite(acc.i1);
                b = to_box(acc);
            }
#else
            double umin = INFINITY, umax = -INFINITY;
            double X[8][3];
            for (int c = 0; c < 8; c++) {
                for (int k = 0; k < 3; k++) X[c][k] = S[k] + (((c >> k) & 1) ? r : -r);
                const double u = proj_u(P, X[c]);
                umin = std::fmin(umin, u);
                umax = std::fmax(umax, u);
            }
            if (umax < 0) {
                b = none;
            } else if (umin > 0) {
                BoxAcc acc;
                for (int c = 0; c < 8; c++) acc.add(P, X[c]);
                b = to_box(acc);
            }
#endif
        }
        out[s] = b;
    }
    for (int w = 0; w < ctx->sc.nW; w++) {
        const double* Wd = &ctx->sc.h_wal[14 * w];
        const double *Pw = Wd, *n = Wd + 3, *X = Wd + 6, *Y = Wd + 9;
        const double len = Wd[12], wid = Wd[13];
        const double pv[3] = {Pw[0] - o[0], Pw[1] - o[1], Pw[2] - o[2]};
        const double num = dot3(pv, n);
        const double scale = 1 + oabs + std::fabs(Pw[0]) + std::fabs(Pw[1]) + std::fabs(Pw[2]) + len + wid;
        rt::PrimBox b = all;
        if (std::fabs(num) > 1e-9 * scale && dmax > 0) {
            double V[4][3];  // P, P + len X, P + len X + wid Y, P + wid Y (cyclic)
            for (int k = 0; k < 3; k++) {
                V[0][k] = Pw[k];
                V[1][k] = Pw[k] + X[k] * len;
                V[2][k] = Pw[k] + X[k] * len + Y[k] * wid;
                V[3][k] = Pw[k] + Y[k] * wid;
            }
            double u[4], umax = -INFINITY;
            for (int c = 0; c < 4; c++) {
                u[c] = proj_u(P, V[c]);
                umax = std::fmax(umax, u[c]);
            }
            const double eps = 0.5 * std::fabs(num) / dmax;
            if (umax < eps) {
                b = none;  // every point behind the camera or closer than the wall's plane
            } else {
                BoxAcc acc;  // Sutherland-Hodgman against u >= eps
                for (int c = 0; c < 4; c++) {
                    const int c2 = (c + 1) & 3;
                    if (u[c] >= eps) acc.add(P, V[c]);
                    if ((u[c] >= eps) != (u[c2] >= eps)) {
                        const double t = (eps - u[c]) / (u[c2] - u[c]);
                        double Xc[3];
                        for (int k = 0; k < 3; k++) Xc[k] = V[c][k] + (V[c2][k] - V[c][k]) * t;
                        acc.add(P, Xc);
                    }
                }
                b = to_box(acc);
            }
        }
        out[ctx->sc.nS + w] = b;
    }
}

void frame_boxes(const rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                 rt::KParams& p) {
    p.nbox = 0;
    p.nwbox = 0;
    p.mir_depth = 0;
    const int np = ctx->sc.nS + ctx->sc.nW;
    const bool cull_walls = p.wave_cull && ctx->sc.nW > 0 && ctx->sc.nW < rt::BIN_MAX_PRIMS;
    if (!ctx->tile_bins || (p.wave_cull && !cull_walls) || np == 0 ||
        (!p.wave_cull && np > rt::BIN_MAX_PRIMS) || cam->width > 32000 || cam->height > 32000 ||
        nrows <= 0 || cam->width <= 0)
        return;
    Proj P;
    if (!make_proj(cam, P)) return;
    // largest |d| over the frame: d is affine in (x, i), so at a corner of the pixel grid
    double dmax = 0;
    for (int c = 0; c < 4; c++) {
        const double x = (c & 1) ? cam->width - 1 : 0, i = (c & 2) ? row0 + nrows - 1 : row0;
        double d[3];
        for (int k = 0; k < 3; k++)
            d[k] = cam->position[k] -
                   (cam->image_top_left[k] + cam->pixel_delta_x[k] * x + cam->pixel_delta_y[k] * i);
        dmax = std::fmax(dmax, std::sqrt(dot3(d, d)));
    }
    if (!(dmax > 0) || !std::isfinite(dmax)) return;
    if (p.wave_cull) {
        // scenes with the wave cull: the spheres keep the cone, the walls get boxes (box[w])
        std::vector<rt::PrimBox> all(np);
        boxes_for(ctx, P, dmax, cam->width, row0, nrows, all.data(), false);
        for (int w = 0; w < ctx->sc.nW; w++) p.box[w] = all[ctx->sc.nS + w];
        p.nwbox = ctx->sc.nW;
        return;
    }
    boxes_for(ctx, P, dmax, cam->width, row0, nrows, p.box);
    p.nbox = np;
    // dispatch order (rt_trace.hip tile_row): centre-out from the weighted median tile row
    // of the boxes' coverage, reflective primitives weighted up (their tiles bounce)
    if (ctx->row_order) {
        const int nty = (nrows + 7) / 8;
        std::vector<double> prof(nty, 0.0);
        for (int j = 0; j < np; j++) {
            const rt::PrimBox& b = p.box[j];
            const int x0 = std::max<int>(b.x0, 0), x1 = std::min<int>(b.x1, cam->width - 1);
            const int i0 = std::max<int>(b.i0, row0), i1 = std::min<int>(b.i1, row0 + nrows - 1);
            if (x0 > x1 || i0 > i1) continue;
            const double wgt = (1.0 + 3.0 * ctx->sc.h_km[j]) * (x1 - x0 + 1);
            for (int t = (i0 - row0) / 8; t <= (i1 - row0) / 8; t++) prof[t] += wgt;
        }
        double tot = 0;
        for (double v : prof) tot += v;
        double acc = 0;
        for (int t = 0; t < nty && tot > 0; t++) {
            acc += prof[t];
            if (acc >= 0.5 * tot) {
                p.row_center = t;
                break;
            }
        }
    }
    // mirror bins (rt_device.h): cameras mirrored along wall chains, each reflection
    // shifted by the reference's 1e-4 * normal origin offset (main.cpp:111); rows of
    // (R M)^-1 = R * rows of M^-1.  Reflected directions are unit vectors, not the d's,
    // but |R d| = |d| keeps dmax.  Only chains some tile can follow are computed (their
    // "reach" — the intersection of the boxes along the chain, widened by a tile — is
    // non-empty); every other sequence keeps all primitives.
    const int nW = ctx->sc.nW;
    int depth = 0;
    for (long tot = 0, lvl = 1; depth < rt::MIR_MAX_DEPTH && nW > 0; depth++) {
        lvl *= nW;
        tot += lvl * np;
        if (tot > rt::MIR_MAX_BOXES) break;
    }
    if (!ctx->mirror_bins || depth == 0) return;
    struct Node {
        Proj cam;
        rt::PrimBox reach;  // pixel region (incl. a tile of slack) where the chain can occur
    };
    const rt::PrimBox allb{-1, (int16_t)cam->width, (int16_t)(row0 - 1), (int16_t)(row0 + nrows)};
    auto meet = [](const rt::PrimBox& a, const rt::PrimBox& b) {
        rt::PrimBox r{std::max(a.x0, b.x0), std::min(a.x1, b.x1), std::max(a.i0, b.i0),
                      std::min(a.i1, b.i1)};
        return r;
    };
    auto empty = [](const rt::PrimBox& b) { return b.x0 > b.x1 || b.i0 > b.i1; };
    auto widen = [](rt::PrimBox b) {
        if (b.x0 > b.x1 || b.i0 > b.i1) return b;
        b.x0 = (int16_t)(b.x0 - 8);
        b.x1 = (int16_t)(b.x1 + 8);
        b.i0 = (int16_t)(b.i0 - 8);
        b.i1 = (int16_t)(b.i1 + 8);
        return b;
    };
    std::vector<Node> prev(1), cur;  // level 0: the camera itself, reach = the frame
    prev[0].cam = P;
    prev[0].reach = allb;
    std::vector<const rt::PrimBox*> prev_boxes(1, p.box);
    int off = 0;
    for (int L = 1; L <= depth; L++) {
        cur.assign(prev.size() * nW, Node{});
        std::vector<const rt::PrimBox*> cur_boxes(cur.size(), nullptr);
        for (size_t q0 = 0; q0 < prev.size(); q0++) {
            for (int w = 0; w < nW; w++) {
                const size_t q = q0 * nW + w;
                rt::PrimBox* out = p.mbox + (size_t)(off + q) * np;
                Node& nd = cur[q];
                nd.reach = empty(prev[q0].reach) ? prev[q0].reach
                                                 : meet(prev[q0].reach, widen(prev_boxes[q0][ctx->sc.nS + w]));
                if (empty(nd.reach)) {
                    for (int j = 0; j < np; j++) out[j] = allb;  // never followed: keep all
                    continue;
                }
                const double* Wd = &ctx->sc.h_wal[14 * w];
                const double *Pw = Wd, *n = Wd + 3;
                const Proj& pc = prev[q0].cam;
                const double op[3] = {pc.o[0] - Pw[0], pc.o[1] - Pw[1], pc.o[2] - Pw[2]};
                const double h = dot3(op, n);
                for (int k = 0; k < 3; k++) nd.cam.o[k] = (pc.o[k] - 2 * h * n[k]) + 1e-4 * n[k];
                for (int j = 0; j < 3; j++) {
                    const double rn = dot3(pc.r[j], n);
                    for (int k = 0; k < 3; k++) nd.cam.r[j][k] = pc.r[j][k] - 2 * rn * n[k];
                }
                boxes_for(ctx, nd.cam, dmax, cam->width, row0, nrows, out);
                cur_boxes[q] = out;
            }
        }
        off += (int)cur.size();
        prev.swap(cur);
        prev_boxes.swap(cur_boxes);
    }
    p.mir_depth = depth;
}

rt::KParams make_params(const rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                        int32_t depth, uint32_t flags, int32_t out_format, void* d_out,
                        unsigned long long* d_segs, int32_t precision) {
    rt::KParams p{};
    const char* base = static_cast<const char*>(ctx->d_scene);
    // section `off` of the device scene (null without one: rt_frame_boxes' host-only use)
    auto at = [base](size_t off) -> const char* { return base ? base + off : nullptr; };
    p.s32 = reinterpret_cast<const rt::SphG32*>(base);
    p.s64 = reinterpret_cast<const rt::SphG64*>(at(ctx->sc.off_s64));
    p.w32 = reinterpret_cast<const rt::Wall32*>(at(ctx->sc.off_w32));
    p.w64 = reinterpret_cast<const rt::Wall64*>(at(ctx->sc.off_w64));
    p.sph_j = reinterpret_cast<const int32_t*>(at(ctx->sc.off_sj));
    p.wall_j = reinterpret_cast<const int32_t*>(at(ctx->sc.off_wj));
    p.mat = reinterpret_cast<const rt::DevMat*>(at(ctx->sc.off_mat));
    p.mat32 = reinterpret_cast<const rt::DevMat32*>(at(ctx->sc.off_mat32));
    p.wnn = reinterpret_cast<const double(*)[4]>(at(ctx->sc.off_wnn));
    const auto& cs = ctx->sc.cset[precision == RT_PREC_F32 ? 0 : 1];
    p.clu = reinterpret_cast<const rt::Clu32*>(at(cs.off_clu));
    p.csph = reinterpret_cast<const rt::CluSph*>(at(cs.off_csph));
    p.cord = reinterpret_cast<const uint8_t*>(at(cs.off_cord));
    p.nclu = cs.nclu;
    p.clu_ls = cs.ls;
    p.clu_axis = cs.clu_axis;
    p.clu_cos = ctx->clu_cos;
    p.clu_oinf = cs.clu_oinf;
    p.nS = ctx->sc.nS;
    p.nW = ctx->sc.nW;
    p.int_exp = ctx->sc.int_exp ? 1 : 0;
    p.wave_cull = ctx->sc.nS >= ctx->wave_cull_min ? 1 : 0;
    p.W = cam->width;
    p.row0 = row0;
    p.nrows = nrows;
    p.depth = depth;
    p.flags = flags;
    p.outf = out_format;
    for (int k = 0; k < 3; k++) {
        p.pos[k] = cam->position[k];
        p.tl[k] = cam->image_top_left[k];
        p.dx[k] = cam->pixel_delta_x[k];
        p.dy[k] = cam->pixel_delta_y[k];
    }
    p.out = d_out;
    p.segs = d_segs;
    p.pairs = ctx->pixel_pairs ? 1 : 0;
    p.stats = ctx->d_stats;
    // eye tables (rt_device.h) for the linear-scan kernels: the same fp64 operations, in
    // the same order, as sphere_exact / wall_exact on a ray starting at cam->position
    p.eye = (ctx->eye_tables && !p.wave_cull && ctx->sc.nS <= rt::EYE_MAX_S && ctx->sc.nW <= rt::EYE_MAX_W) ? 1 : 0;
    if (p.eye) {
        const double* o = cam->position;
        for (int s = 0; s < ctx->sc.nS; s++) {
            const double* S = &ctx->sc.h_sph[5 * s];
            const double ox = o[0] - S[0], oy = o[1] - S[1], oz = o[2] - S[2];  // scene.cpp:45
            const double c = (ox * ox + oy * oy + oz * oz) - S[3];              // scene.cpp:51
            const double e[4] = {ox, oy, oz, c};
            for (int k = 0; k < 4; k++) p.eye_s[s][k] = e[k];
        }
        for (int w = 0; w < ctx->sc.nW; w++) {
            const double* P = &ctx->sc.h_wal[14 * w];
            const double* n = P + 3;
            p.eye_w[w] = (P[0] - o[0]) * n[0] + (P[1] - o[1]) * n[1] + (P[2] - o[2]) * n[2];  // scene.cpp:10
        }
    }
    // primary scan's wall order: nearest rectangle to the camera first, so the wall t-skip
    // (t > best) drops the bounds test of the walls it occludes.  Any order gives the
    // reference's winner (wall ties compare scene indices, rt_trace.hip wall_exact).
    p.wall_order_n = 0;
    p.wall_order = 0;
    if (ctx->wall_order && ctx->sc.nW > 1 && ctx->sc.nW <= 16) {
        const double* o = cam->position;
        double key[16];
        int ord[16];
        for (int w = 0; w < ctx->sc.nW; w++) {
            const double* Wd = &ctx->sc.h_wal[14 * w];
            const double *Pw = Wd, *X = Wd + 6, *Y = Wd + 9;
            const double v[3] = {o[0] - Pw[0], o[1] - Pw[1], o[2] - Pw[2]};
            // closest point of the rectangle P + a X + b Y (a in [0, len], b in [0, wid])
            const double a = std::min(std::max(v[0] * X[0] + v[1] * X[1] + v[2] * X[2], 0.0), Wd[12]);
            const double b = std::min(std::max(v[0] * Y[0] + v[1] * Y[1] + v[2] * Y[2], 0.0), Wd[13]);
            double d2 = 0.0;
            for (int k = 0; k < 3; k++) {
                const double e = v[k] - a * X[k] - b * Y[k];
                d2 += e * e;
            }
            key[w] = std::isnan(d2) ? 1e300 : d2;
            ord[w] = w;
        }
        std::stable_sort(ord, ord + ctx->sc.nW, [&](int x, int y) { return key[x] < key[y]; });
        for (int k = 0; k < ctx->sc.nW; k++) p.wall_order |= (uint64_t)ord[k] << (4 * k);
        p.wall_order_n = ctx->sc.nW;
    }
    // per-frame boxes, or the previous render's when its inputs were the same
    rt_ctx::BoxCache& bc = ctx->box_cache;
    const int32_t opts = (ctx->tile_bins ? 1 : 0) | (ctx->row_order ? 2 : 0) | (ctx->mirror_bins ? 4 : 0);
    if (ctx->box_cache_on && bc.valid && bc.scene_gen == ctx->scene_gen && bc.row0 == row0 && bc.nrows == nrows &&
        bc.wave_cull == p.wave_cull && bc.opts == opts &&
        std::memcmp(&bc.cam, cam, sizeof(rt_camera)) == 0) {
        p.nbox = bc.nbox;
        p.nwbox = bc.nwbox;
        p.row_center = bc.row_center;
        p.mir_depth = bc.mir_depth;
        std::memcpy(p.box, bc.box, sizeof p.box);
        std::memcpy(p.mbox, bc.mbox, bc.nmbox * sizeof(rt::PrimBox));
        return p;
    }
    frame_boxes(ctx, cam, row0, nrows, p);
    long nm = 0;
    for (long L = 1, lvl = 1; L <= p.mir_depth; L++) {
        lvl *= ctx->sc.nW;
        nm += lvl * p.nbox;
    }
    bc.valid = true;
    bc.scene_gen = ctx->scene_gen;
    bc.cam = *cam;
    bc.row0 = row0;
    bc.nrows = nrows;
    bc.wave_cull = p.wave_cull;
    bc.opts = opts;
    bc.nbox = p.nbox;
    bc.nwbox = p.nwbox;
    bc.row_center = p.row_center;
    bc.mir_depth = p.mir_depth;
    bc.nmbox = (size_t)nm;
    std::memcpy(bc.box, p.box, sizeof p.box);
    std::memcpy(bc.mbox, p.mbox, bc.nmbox * sizeof(rt::PrimBox));
    return p;
}

/* rt_set_scene's host half: the device image of the scene (rt_device.h layout) and the
 * host copies the per-frame boxes and eye tables use.  No device call. */
int pack_scene(const rt_prim* prims, int32_t n, rt_ctx::SceneHost& sc) {
    if (n < 0 || (n > 0 && !prims)) return RT_ERR_INVALID_ARG;
    struct Sph {
        double c[3], r;
        int32_t j;
    };
    struct Wal {
        double P[3], n[3], X[3], Y[3], len, wid;
        int32_t j;
    };
    std::vector<Sph> sph;
    std::vector<Wal> wal;
    for (int32_t j = 0; j < n; j++) {
        const rt_prim& q = prims[j];
        if (q.reserved != 0) return RT_ERR_INVALID_ARG;
        if (q.kind == RT_PRIM_SPHERE) {
            sph.push_back(Sph{{q.position[0], q.position[1], q.position[2]}, q.radius, j});
        } else if (q.kind == RT_PRIM_WALL) {
            const hv3 nrm{q.normal[0], q.normal[1], q.normal[2]};
            const hv3 X = hnormalize(hcross(nrm, hv3{0, 0, 1}));  // scene.cpp:18
            const hv3 Y = hnormalize(hcross(X, nrm));             // scene.cpp:19
            // A NaN basis (normal parallel to z) or NaN normal makes every projection NaN:
            // the reference can never report a hit for this wall, so it is not uploaded.
            if (hnan(X) || hnan(Y) || hnan(nrm)) continue;
            wal.push_back(Wal{{q.position[0], q.position[1], q.position[2]},
                              {nrm.x, nrm.y, nrm.z}, {X.x, X.y, X.z}, {Y.x, Y.y, Y.z},
                              q.length, q.width, j});
        } else {
            return RT_ERR_INVALID_ARG;
        }
    }
    const size_t nS = sph.size(), nW = wal.size(), ng = (nS + 3) / 4;
    const size_t off_s64 = align_up(ng * sizeof(rt::SphG32), 256);
    const size_t off_w32 = align_up(off_s64 + ng * sizeof(rt::SphG64), 256);
    const size_t off_w64 = align_up(off_w32 + nW * sizeof(rt::Wall32), 256);
    const size_t off_sj = align_up(off_w64 + nW * sizeof(rt::Wall64), 256);
    const size_t off_wj = align_up(off_sj + nS * sizeof(int32_t), 256);
    const size_t off_mat = align_up(off_wj + nW * sizeof(int32_t), 256);
    const size_t off_mat32 = align_up(off_mat + (nS + nW) * sizeof(rt::DevMat), 256);
    const size_t off_wnn = align_up(off_mat32 + (nS + nW) * sizeof(rt::DevMat32), 256);
    auto make_leaves = [&](int ls, std::vector<std::vector<int>>& leaves, int& clu_axis) {
        // sphere clusters (rt_device.h): leaves of <= ls spheres from binary splits (the
        // surface-area cut at a multiple of ls, RT_CLU_SAH; else the median of the widest axis)
        if (nS >= 2 * (size_t)ls && nS <= (size_t)ls * rt::CLU_MAX) {
            std::vector<int> all(nS);
            for (size_t s = 0; s < nS; s++) all[s] = (int)s;
            bool finite = true;
            for (const Sph& a : sph)
                finite = finite && std::isfinite(a.c[0]) && std::isfinite(a.c[1]) &&
                         std::isfinite(a.c[2]) && std::isfinite(a.r);
            // median split on the widest axis of the centres until <= ls per leaf
            std::function<void(std::vector<int>&, bool)> split = [&](std::vector<int>& ids, bool top) {
                if (ids.size() <= (size_t)ls) {
                    leaves.push_back(ids);
                    return;
                }
                double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
                for (int i : ids)
                    for (int q = 0; q < 3; q++) {
                        lo[q] = std::min(lo[q], sph[i].c[q]);
                        hi[q] = std::max(hi[q], sph[i].c[q]);
                    }
                int ax = 0;
                for (int q = 1; q < 3; q++)
                    if (hi[q] - lo[q] > hi[ax] - lo[ax]) ax = q;
                size_t mid = ids.size() / 2;
                if (RT_CLU_SAH) {
                    // surface-area split: over the three axes and the cut positions that keep the
                    // leaf count at its minimum (multiples of CLU_SIZE), the one minimising
                    // area(left box) * |left| + area(right box) * |right| (boxes of the balls)
                    const size_t n = ids.size();
                    double best = HUGE_VAL;
                    for (int q = 0; q < 3; q++) {
                        std::vector<int> v(ids);
                        std::sort(v.begin(), v.end(), [&](int a, int b) {
                            return sph[a].c[q] < sph[b].c[q] || (sph[a].c[q] == sph[b].c[q] && a < b);
                        });
                        auto area = [&](size_t b0, size_t b1) {
                            double l[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, h[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
                            for (size_t k = b0; k < b1; k++)
                                for (int z = 0; z < 3; z++) {
                                    const double rr = std::fabs(sph[v[k]].r);
                                    l[z] = std::min(l[z], sph[v[k]].c[z] - rr);
                                    h[z] = std::max(h[z], sph[v[k]].c[z] + rr);
                                }
                            const double e0 = h[0] - l[0], e1 = h[1] - l[1], e2 = h[2] - l[2];
                            return 2 * (e0 * e1 + e1 * e2 + e2 * e0);
                        };
                        for (size_t k = (size_t)ls; k < n; k += (size_t)ls) {
                            const double c = area(0, k) * (double)k + area(k, n) * (double)(n - k);
                            if (c < best) {
                                best = c;
                                ax = q;
                                mid = k;
                            }
                        }
                    }
                }
                if (top) clu_axis = ax;
                std::nth_element(ids.begin(), ids.begin() + mid, ids.end(), [&](int a, int b) {
                    return sph[a].c[ax] < sph[b].c[ax] || (sph[a].c[ax] == sph[b].c[ax] && a < b);
                });
                std::vector<int> l(ids.begin(), ids.begin() + mid), r(ids.begin() + mid, ids.end());
                split(l, false);
                split(r, false);
            };
            if (finite) split(all, true);
            if (leaves.size() > (size_t)rt::CLU_MAX) leaves.clear();
        }
    };
    // set 0: the F32 kernels' leaves (CLU_SIZE); set 1: the fp64 kernels' (CLU_SIZE_D, or
    // CLU_SIZE when that needs more than CLU_MAX leaves)
    std::vector<std::vector<int>> leaves[2];
    int clu_axis[2] = {0, 0}, lsz[2] = {rt::CLU_SIZE, rt::CLU_SIZE_D};
    make_leaves(lsz[0], leaves[0], clu_axis[0]);
    make_leaves(lsz[1], leaves[1], clu_axis[1]);
    if (leaves[1].empty() && lsz[1] != lsz[0]) {
        leaves[1] = leaves[0];
        clu_axis[1] = clu_axis[0];
        lsz[1] = lsz[0];
    }
    size_t off = align_up(off_wnn + nW * 4 * sizeof(double), 256);
    for (int q = 0; q < 2; q++) {
        auto& cs = sc.cset[q];
        const size_t nclu = leaves[q].size();
        cs.nclu = (int)nclu;
        cs.clu_axis = clu_axis[q];
        cs.ls = lsz[q];
        cs.off_clu = off;
        // room for a multiple of four cluster records (the kernels read the boxes in batches)
        cs.off_csph = align_up(cs.off_clu + ((nclu + 3) & ~(size_t)3) * sizeof(rt::Clu32), 256);
        cs.off_cord = align_up(cs.off_csph + nclu * lsz[q] * sizeof(rt::CluSph), 256);
        off = align_up(cs.off_cord + 8 * rt::CLU_MAX, 256);
    }
    const size_t total = off + 256;
    sc.blocks.assign((total + 255) / 256, {});
    sc.total = total;
    struct {
        char* p;
        char* data() { return p; }
    } host{sc.image()};
    auto* s32 = reinterpret_cast<rt::SphG32*>(host.data());
    auto* s64 = reinterpret_cast<rt::SphG64*>(host.data() + off_s64);
    auto* w32 = reinterpret_cast<rt::Wall32*>(host.data() + off_w32);
    auto* w64 = reinterpret_cast<rt::Wall64*>(host.data() + off_w64);
    auto* sj = reinterpret_cast<int32_t*>(host.data() + off_sj);
    auto* wj = reinterpret_cast<int32_t*>(host.data() + off_wj);
    auto* mat = reinterpret_cast<rt::DevMat*>(host.data() + off_mat);
    auto* mat32 = reinterpret_cast<rt::DevMat32*>(host.data() + off_mat32);
    auto* wnn = reinterpret_cast<double(*)[4]>(host.data() + off_wnn);
    auto put_mat = [&](size_t slot, const rt_material& m) {
        rt::DevMat& d = mat[slot];
        for (int k = 0; k < 3; k++) d.color[k] = m.color[k];
        d.ka = m.ambient;
        d.km = m.metallic;
        d.kd = m.diffuse;
        d.ks = m.specular;
        d.ex = m.specular_exponent;
        rt::DevMat32& f = mat32[slot];
        for (int k = 0; k < 3; k++) f.color[k] = (float)m.color[k];
        f.ka = (float)m.ambient;
        f.km = (float)m.metallic;
        f.kd = (float)m.diffuse;
        f.ks = (float)m.specular;
        f.ex = (float)m.specular_exponent;
    };
    for (size_t s = 0; s < nS; s++) {
        rt::SphG32& g = s32[s / 4];
        double* d = s64[s / 4].v[s % 4];
        for (int k = 0; k < 3; k++) {
            g.c[k][s % 4] = (float)sph[s].c[k];
            d[k] = sph[s].c[k];
        }
        g.c[3][s % 4] = (float)sph[s].r;
        d[3] = sph[s].r * sph[s].r;  // scene.cpp:51
        sj[s] = sph[s].j;
        put_mat(s, prims[sph[s].j].mat);
    }
    for (int set = 0; set < 2; set++) {
        auto& cset = sc.cset[set];
        const size_t nclu = (size_t)cset.nclu, ls = (size_t)cset.ls;
        const std::vector<std::vector<int>>& lv = leaves[set];
        auto* clu = reinterpret_cast<rt::Clu32*>(host.data() + cset.off_clu);
        auto* csph = reinterpret_cast<rt::CluSph*>(host.data() + cset.off_csph);
        double clu_scale = 1.0;
        std::vector<std::array<double, 3>> cen(nclu);
        for (size_t c = 0; c < nclu; c++) {
            double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            double scale = 1.0;
            for (size_t k = 0; k < ls; k++) {
                rt::CluSph& cs = csph[c * ls + k];
                cs.slot = -1;
                if (k >= lv[c].size()) continue;
                const int si = lv[c][k];
                for (int q = 0; q < 4; q++) cs.c[q] = s64[si / 4].v[si % 4][q];
                for (int q = 0; q < 4; q++) cs.f[q] = s32[si / 4].c[q][si % 4];
                cs.slot = si;
                for (int q = 0; q < 3; q++) {
                    const double rr = std::fabs(sph[si].r);
                    lo[q] = std::min(lo[q], sph[si].c[q] - rr);
                    hi[q] = std::max(hi[q], sph[si].c[q] + rr);
                    scale = std::max(scale, std::fabs(sph[si].c[q]) + rr);
                }
            }
            // margin: far above the fp32 rounding of the box, the ray and the slab arithmetic
            // (~1e-6 relative), so a ray the exact test finds hitting a ball enters the box
            const double m = 1e-3 * scale;
            clu_scale = std::max(clu_scale, scale);
            for (int q = 0; q < 3; q++) cen[c][q] = 0.5 * (lo[q] + hi[q]);
            for (int q = 0; q < 3; q++) {
                clu[c].lo[q] = (float)(lo[q] - m);
                clu[c].hi[q] = (float)(hi[q] + m);
            }
        }
        // near-to-far cluster order per direction octant: by the box centre along the octant's
        // diagonal (any order is exact; this one lets the lanes' pruning start from near hits)
        auto* cord = reinterpret_cast<uint8_t*>(host.data() + cset.off_cord);
        for (int o = 0; o < 8 && nclu > 0; o++) {
            const double sx = (o & 1) ? -1.0 : 1.0, sy = (o & 2) ? -1.0 : 1.0, sz = (o & 4) ? -1.0 : 1.0;
            std::vector<int> ord(nclu);
            for (size_t c = 0; c < nclu; c++) ord[c] = (int)c;
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
                return sx * cen[a][0] + sy * cen[a][1] + sz * cen[a][2] <
                       sx * cen[b][0] + sy * cen[b][1] + sz * cen[b][2];
            });
            for (size_t k = 0; k < nclu; k++) {
                cord[o * rt::CLU_MAX + k] = (uint8_t)ord[k];
                clu[ord[k]].rank[o] = (uint8_t)k;
            }
        }
        // origins up to 100x the scene's extent: fp32 errors of the slab test ~1e-5 x scale,
        // 100x below the box margin
        cset.clu_oinf = (float)(100.0 * clu_scale);
    }
    for (size_t w = 0; w < nW; w++) {
        const Wal& a = wal[w];
        for (int k = 0; k < 3; k++) {
            w64[w].P[k] = a.P[k];
            w64[w].n[k] = a.n[k];
            w64[w].X[k] = a.X[k];
            w64[w].Y[k] = a.Y[k];
            w32[w].P[k] = (float)a.P[k];
            w32[w].n[k] = (float)a.n[k];
            w32[w].X[k] = (float)a.X[k];
            w32[w].Y[k] = (float)a.Y[k];
        }
        w64[w].len = a.len;
        w64[w].wid = a.wid;
        w32[w].len = (float)a.len;
        w32[w].wid = (float)a.wid;
        wj[w] = a.j;
        put_mat(nS + w, prims[a.j].mat);
        const hv3 nn = hnormalize(hv3{a.n[0], a.n[1], a.n[2]});  // N.normalize(), vec.cpp:21
        wnn[w][0] = nn.x;
        wnn[w][1] = nn.y;
        wnn[w][2] = nn.z;
    }

    sc.nS = (int)nS;
    sc.nW = (int)nW;
    sc.nP = n;
    sc.int_exp = true;
    for (size_t k = 0; k < nS + nW; k++) {
        const double e = mat[k].ex;
        if (!(e >= 0.0 && e <= 1024.0 && e == std::floor(e))) sc.int_exp = false;
    }
    sc.h_km.assign(nS + nW, 0.0);
    for (size_t k = 0; k < nS + nW; k++) sc.h_km[k] = mat[k].km;
    sc.h_sph.assign(5 * nS, 0.0);
    for (size_t s = 0; s < nS; s++) {
        for (int k = 0; k < 4; k++) sc.h_sph[5 * s + k] = s64[s / 4].v[s % 4][k];
        sc.h_sph[5 * s + 4] = sph[s].r;
    }
    sc.h_wal.assign(14 * nW, 0.0);
    for (size_t w = 0; w < nW; w++) {
        for (int k = 0; k < 3; k++) {
            sc.h_wal[14 * w + k] = w64[w].P[k];
            sc.h_wal[14 * w + 3 + k] = w64[w].n[k];
            sc.h_wal[14 * w + 6 + k] = w64[w].X[k];
            sc.h_wal[14 * w + 9 + k] = w64[w].Y[k];
        }
        sc.h_wal[14 * w + 12] = w64[w].len;
        sc.h_wal[14 * w + 13] = w64[w].wid;
    }
    sc.off_s64 = off_s64;
    sc.off_w32 = off_w32;
    sc.off_w64 = off_w64;
    sc.off_sj = off_sj;
    sc.off_wj = off_wj;
    sc.off_mat = off_mat;
    sc.off_mat32 = off_mat32;
    sc.off_wnn = off_wnn;
    return RT_OK;
}


}  // namespace

extern "C" {

int rt_capi_version(void) { return RT_CAPI_VERSION; }

const char* rt_strerror(int status) {
    switch (status) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID_ARG: return "invalid argument";
        case RT_ERR_NO_DEVICE: return "no HIP device";
        case RT_ERR_HIP: return "HIP runtime error";
        case RT_ERR_OUT_OF_MEMORY: return "out of device memory";
        case RT_ERR_NO_SCENE: return "no scene uploaded";
        case RT_ERR_UNSUPPORTED: return "unsupported depth/flags";
        case RT_ERR_OUT_OF_RANGE: return "row band out of range";
        case RT_ERR_COMM: return "RCCL communication error";
        default: return "unknown status";
    }
}

const char* rt_last_hip_error(const rt_ctx* ctx) { return ctx ? ctx->last_err : ""; }

int32_t rt_out_bytes_per_pixel(int32_t out_format) { return bytes_per_pixel(out_format); }

int32_t rt_max_depth(void) { return rt::max_depth(); }

int32_t rt_tile_rows(void) { return rt::TILE_H; }

int rt_band_rows(int32_t height, int32_t nranks, int32_t rank, int32_t* row0, int32_t* nrows) {
    if (!row0 || !nrows || height < 0 || nranks <= 0 || rank < 0 || rank >= nranks)
        return RT_ERR_INVALID_ARG;
    // contiguous blocks, the first (height % nranks) ranks take one extra row
    const int32_t base = height / nranks, extra = height % nranks;
    *row0 = rank * base + (rank < extra ? rank : extra);
    *nrows = base + (rank < extra ? 1 : 0);
    return RT_OK;
}

int rt_camera_init(const double position[3], const double lookat[3], const double vup[3],
                   double vfov, double aspect_ratio, double image_width, rt_camera* cam) {
    /* Camera::init, scene.cpp:80-106, op for op (3.14 for pi kept). */
    if (!position || !lookat || !vup || !cam) return RT_ERR_INVALID_ARG;
    const hv3 pos{position[0], position[1], position[2]};
    const hv3 look{lookat[0], lookat[1], lookat[2]};
    const hv3 up{vup[0], vup[1], vup[2]};
    const double image_height = static_cast<int>(image_width / aspect_ratio);
    const hv3 pl{pos.x - look.x, pos.y - look.y, pos.z - look.z};
    const double focal_length = std::sqrt(pl.x * pl.x + pl.y * pl.y + pl.z * pl.z);
    const double theta = vfov * 3.14 / 180.0;
    const double h = std::tan(theta / 2);
    const double fov_height = 2 * h * focal_length;
    const double fov_width = fov_height * (static_cast<double>(image_width) / image_height);
    const hv3 w = hnormalize(pl);
    const hv3 u = hnormalize(hcross(up, w));
    const hv3 v = hcross(w, u);
    const hv3 fx{u.x * fov_width, u.y * fov_width, u.z * fov_width};
    const double nfh = -fov_height;
    const hv3 fy{v.x * nfh, v.y * nfh, v.z * nfh};
    const hv3 pdx{fx.x / image_width, fx.y / image_width, fx.z / image_width};
    const hv3 pdy{fy.x / image_height, fy.y / image_height, fy.z / image_height};
    const hv3 wf{w.x * focal_length, w.y * focal_length, w.z * focal_length};
    const hv3 ftl{((pos.x - wf.x) - fx.x / 2) - fy.x / 2, ((pos.y - wf.y) - fx.y / 2) - fy.y / 2,
                  ((pos.z - wf.z) - fx.z / 2) - fy.z / 2};
    const hv3 s{pdx.x + pdy.x, pdx.y + pdy.y, pdx.z + pdy.z};
    const hv3 itl{ftl.x + s.x * 0.5, ftl.y + s.y * 0.5, ftl.z + s.z * 0.5};
    const double p3[4][3] = {{pos.x, pos.y, pos.z}, {itl.x, itl.y, itl.z},
                             {pdx.x, pdx.y, pdx.z}, {pdy.x, pdy.y, pdy.z}};
    std::memcpy(cam->position, p3[0], sizeof p3[0]);
    std::memcpy(cam->image_top_left, p3[1], sizeof p3[1]);
    std::memcpy(cam->pixel_delta_x, p3[2], sizeof p3[2]);
    std::memcpy(cam->pixel_delta_y, p3[3], sizeof p3[3]);
    cam->width = static_cast<int32_t>(image_width);
    cam->height = static_cast<int32_t>(image_height);
    return RT_OK;
}

int rt_ctx_create(int device, rt_ctx** out) {
    if (!out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return RT_ERR_NO_DEVICE;
    rt_ctx* ctx = new (std::nothrow) rt_ctx();
    if (!ctx) return RT_ERR_OUT_OF_MEMORY;
    ctx->device = device;
    int st = RT_OK;
    DeviceGuard dg(device);
    do {
        hipError_t e;
        if ((e = dg.err) != hipSuccess) { st = hip_fail(ctx, e, "hipSetDevice"); break; }
        if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) {
            st = hip_fail(ctx, e, "hipStreamCreate"); break;
        }
        if ((e = hipEventCreate(&ctx->ev0)) != hipSuccess) { st = hip_fail(ctx, e, "hipEventCreate"); break; }
        if ((e = hipEventCreate(&ctx->ev1)) != hipSuccess) { st = hip_fail(ctx, e, "hipEventCreate"); break; }
        if ((e = hipEventCreateWithFlags(&ctx->ev_cost, hipEventDisableTiming)) != hipSuccess) {
            st = hip_fail(ctx, e, "hipEventCreate"); break;
        }
        if ((e = hipEventCreateWithFlags(&ctx->ev_iso, hipEventDisableTiming)) != hipSuccess) {
            st = hip_fail(ctx, e, "hipEventCreate"); break;
        }
        if ((e = hipMalloc(&ctx->d_segs, sizeof(unsigned long long))) != hipSuccess) {
            st = hip_fail(ctx, e, "hipMalloc(segs)"); break;
        }
    } while (0);
    if (st != RT_OK) {
        rt_ctx_destroy(ctx);
        return st;
    }
    *out = ctx;
    return RT_OK;
}

namespace {
void prep_shutdown(rt_ctx* ctx);  // RT_OPT_HOST_PIPELINE's helper thread (below)
}

int rt_ctx_destroy(rt_ctx* ctx) {
    if (!ctx) return RT_ERR_INVALID_ARG;
#if RT_HOST_PROFILE
    if (g_hn > 50) {
        const double m = (double)(g_hn - 50);
        std::fprintf(stderr, "host profile over %ld warm renders (us): args %.2f params %.2f rows+event %.2f launch %.2f snapshot %.2f\n",
                     g_hn - 50, g_hp[0] / m, g_hp[1] / m, g_hp[2] / m, g_hp[3] / m, g_hp[4] / m);
    }
#endif
    prep_shutdown(ctx);
    DeviceGuard dg(ctx->device);
    (void)wait_inflight(ctx);  // frames in flight on caller streams still read the scene
    for (auto& f : ctx->inflight) (void)hipEventDestroy(f.ev);
    ctx->inflight.clear();
    for (auto& e : ctx->tab_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->d_tab) (void)hipFree(ctx->d_tab);
    if (ctx->h_tab) (void)hipHostFree(ctx->h_tab);
    if (ctx->d_scene) (void)hipFree(ctx->d_scene);
    if (ctx->d_out) (void)hipFree(ctx->d_out);
    if (ctx->d_segs) (void)hipFree(ctx->d_segs);
    if (ctx->ev_cost) (void)hipEventSynchronize(ctx->ev_cost);
    if (ctx->d_cost) (void)hipFree(ctx->d_cost);
    if (ctx->d_umax) (void)hipFree(ctx->d_umax);
    if (ctx->h_umax) (void)hipHostFree(ctx->h_umax);
    if (ctx->ev_cost) (void)hipEventDestroy(ctx->ev_cost);
    if (ctx->ev_iso) (void)hipEventDestroy(ctx->ev_iso);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return RT_OK;
}

int rt_set_scene(rt_ctx* ctx, const rt_prim* prims, int32_t n) {
    if (!ctx || n < 0 || (n > 0 && !prims)) return RT_ERR_INVALID_ARG;
    rt_ctx::SceneHost sc;
    const int st = pack_scene(prims, n, sc);
    if (st != RT_OK) return st;
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    // no render of the old scene may still be running, on the ctx's stream or a caller's
    const int ws = wait_inflight(ctx);
    if (ws != RT_OK) return ws;
    if (sc.total > ctx->scene_bytes) {
        if (ctx->d_scene) RT_HIP(ctx, hipFree(ctx->d_scene));
        ctx->d_scene = nullptr;
        ctx->scene_bytes = 0;
        RT_HIP(ctx, hipMalloc(&ctx->d_scene, sc.total));
        ctx->scene_bytes = sc.total;
    }
    RT_HIP(ctx, hipMemcpy(ctx->d_scene, sc.image(), sc.total, hipMemcpyHostToDevice));
    ctx->sc = std::move(sc);
    ctx->have_scene = true;
    ctx->scene_gen++;
    return RT_OK;
}

int rt_frame_boxes(const rt_prim* prims, int32_t n, const rt_camera* cam, int32_t row0,
                   int32_t nrows, int16_t* out, int32_t cap, int32_t* nbox, int32_t* mir_depth) {
    if (!cam || !nbox || !mir_depth || cap < 0 || (cap > 0 && !out)) return RT_ERR_INVALID_ARG;
    if (row0 < 0 || nrows < 0 || row0 + nrows > cam->height) return RT_ERR_OUT_OF_RANGE;
    std::unique_ptr<rt_ctx> ctx(new (std::nothrow) rt_ctx());  // host-only: no device resources
    if (!ctx) return RT_ERR_OUT_OF_MEMORY;
    const int st = pack_scene(prims, n, ctx->sc);
    if (st != RT_OK) return st;
    ctx->wave_cull_min = 0x7fffffff;  // as the linear-scan kernels see the scene
    std::unique_ptr<rt::KParams> p(new (std::nothrow) rt::KParams);
    if (!p) return RT_ERR_OUT_OF_MEMORY;
    *p = make_params(ctx.get(), cam, row0, nrows, 0, 0, RT_OUT_RGB_F32, nullptr, nullptr,
                     RT_PREC_F64);
    long total = p->nbox;
    for (long L = 1, lvl = 1; L <= p->mir_depth; L++) {
        lvl *= ctx->sc.nW;
        total += lvl * p->nbox;
    }
    *nbox = p->nbox;
    *mir_depth = p->mir_depth;
    if (total > cap) return RT_ERR_INVALID_ARG;
    for (int j = 0; j < p->nbox; j++) std::memcpy(out + 4 * j, &p->box[j], sizeof(rt::PrimBox));
    for (long j = p->nbox; j < total; j++)
        std::memcpy(out + 4 * j, &p->mbox[j - p->nbox], sizeof(rt::PrimBox));
    return RT_OK;
}

int rt_set_option(rt_ctx* ctx, int32_t option, int64_t value) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    switch (option) {
        case RT_OPT_WAVE_CULL_MIN_SPHERES:
            if (value < 0) return RT_ERR_INVALID_ARG;
            ctx->wave_cull_min = value > 0x7fffffff ? 0x7fffffff : (int)value;
            return RT_OK;
        case RT_OPT_STATS_DEVICE_PTR:
            ctx->d_stats = reinterpret_cast<unsigned long long*>(static_cast<intptr_t>(value));
            return RT_OK;
        case RT_OPT_CLUSTER_COS:
            if (value < -2000 || value > 2000) return RT_ERR_INVALID_ARG;
            ctx->clu_cos = (float)value / 1000.0f;
            return RT_OK;
        case RT_OPT_WALL_ORDER:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->wall_order = value == 1;
            return RT_OK;
        case RT_OPT_EYE_TABLES:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->eye_tables = value == 1;
            return RT_OK;
        case RT_OPT_TILE_BINS:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->tile_bins = value == 1;
            return RT_OK;
        case RT_OPT_BOX_CACHE:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->box_cache_on = value == 1;
            return RT_OK;
        case RT_OPT_MIRROR_BINS:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->mirror_bins = value == 1;
            return RT_OK;
        case RT_OPT_ROW_ORDER:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->row_order = value == 1;
            return RT_OK;
        case RT_OPT_PIXEL_PAIRS:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->pixel_pairs = value == 1;
            return RT_OK;
        case RT_OPT_ROW_FEEDBACK_EMA:
            if (value < 0 || value > 95) return RT_ERR_INVALID_ARG;
            ctx->fb_ema = (int)value;
            return RT_OK;
        case RT_OPT_HOST_PIPELINE:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->host_pipeline = value == 1;
            return RT_OK;
        case RT_OPT_FRAME_BATCH:
            if (value < 1 || value > RT_MULTI_BATCH_MAX) return RT_ERR_INVALID_ARG;
            ctx->frame_batch = (int)value;
            return RT_OK;
        case RT_OPT_ROW_FEEDBACK_ISOLATE:
            if (value != 0 && value != 1) return RT_ERR_INVALID_ARG;
            ctx->fb_isolate = value == 1;
            return RT_OK;
        case RT_OPT_ROW_FEEDBACK_WARM:
            if (value < 0 || value > 1000) return RT_ERR_INVALID_ARG;
            ctx->fb_warm = (int)value;
            return RT_OK;
        case RT_OPT_ROW_FEEDBACK:
            if (value < 0 || value > 1000000) return RT_ERR_INVALID_ARG;
            ctx->feedback = (int)value;
            ctx->fb_epoch++;  // orders and snapshots taken so far belong to the old setting
            if (value == 0) {
                ctx->fb_perm.clear();
                ctx->fb_band = rt_ctx::Band{};
            }
            return RT_OK;
        default:
            return RT_ERR_INVALID_ARG;
    }
}

int rt_selftest(rt_ctx* ctx, int32_t test, uint64_t n, uint64_t seed, uint64_t* mismatches) {
    if (!ctx || !mismatches || test < 0 || test > 2) return RT_ERR_INVALID_ARG;
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    RT_HIP(ctx, hipMemsetAsync(ctx->d_segs, 0, sizeof(unsigned long long), ctx->stream));
    const int e = rt::launch_selftest(test, n, seed, ctx->d_segs, ctx->stream);
    if (e != (int)hipSuccess) return hip_fail(ctx, (hipError_t)e, "launch k_selftest");
    unsigned long long h = 0;
    RT_HIP(ctx, hipMemcpyAsync(&h, ctx->d_segs, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *mismatches = h;
    return RT_OK;
}

/* Explicit tile-row dispatch order (a permutation of 0 .. n-1), used by renders whose grid
 * has exactly n tile rows; n == 0 clears it. */
int rt_set_row_order(rt_ctx* ctx, const int16_t* perm, int32_t n) {
    if (!ctx || n < 0 || n > rt::ROW_PERM_MAX || (n > 0 && !perm)) return RT_ERR_INVALID_ARG;
    std::vector<char> seen(n, 0);
    for (int j = 0; j < n; j++) {
        if (perm[j] < 0 || perm[j] >= n || seen[perm[j]]) return RT_ERR_INVALID_ARG;
        seen[perm[j]] = 1;
    }
    ctx->row_perm.assign(perm, perm + n);
    return RT_OK;
}

#ifndef RT_ROW_UNITS_MAX_LOG2
#define RT_ROW_UNITS_MAX_LOG2 3
#endif
/* Dispatch units per tile row for the measured order (log2): rows split in up to 8 parts
 * while the units fit row_perm and keep >= 8 tiles each — the ordering gets finer where a
 * row holds both heavy and light tiles (replay of c2's measured wave times: whole rows
 * -15%, quarter rows -19% vs centre-out). */
static int units_log2(int gy, int gx) {
    if (rt::BLOCK != 64) return 0;
    for (int k = RT_ROW_UNITS_MAX_LOG2; k > 0; k--)
        if ((gy << k) <= rt::ROW_PERM_MAX && ((gx + (1 << k) - 1) >> k) >= 8) return k;
    return 0;
}

/* Dispatch units ordered by their most expensive wave (heaviest first; ties keep the lower
 * unit), from the per-unit maxima of a cost snapshot (k_unit_max).  Host work is O(nu):
 * the keys are 16-bit (wave costs saturate at 65535), sorted by a stable two-pass radix
 * sort — the comparison sort it replaces took ~100 us on the thread that enqueues frames,
 * long enough to starve the GPU once per snapshot. */
static void order_units(const uint32_t* umax, int nu, std::vector<int16_t>& perm,
                        std::vector<float>& acc, bool acc_valid, int ema) {
    // smoothed over the band's snapshots (RT_OPT_ROW_FEEDBACK_EMA), else this snapshot's
    const float w = ema / 100.0f;
    const bool smooth = acc_valid && (int)acc.size() == nu && ema > 0;
    if (!smooth) acc.assign(nu, 0.0f);
    std::vector<uint16_t> key(nu);
    for (int u = 0; u < nu; u++) {
        const float m = (float)std::min<uint32_t>(umax[u], 65535u);
        const float a = smooth ? w * acc[u] + (1.0f - w) * m : m;
        acc[u] = a;
        key[u] = (uint16_t)(65535u - (uint32_t)std::min(a + 0.5f, 65535.0f));  // descending
    }
    std::vector<int16_t> tmp(nu);
    perm.resize(nu);
    for (int u = 0; u < nu; u++) perm[u] = (int16_t)u;
    for (int sh = 0; sh < 16; sh += 8) {
        unsigned cnt[257] = {0};
        for (int k = 0; k < nu; k++) cnt[((key[perm[k]] >> sh) & 255) + 1]++;
        for (int b = 0; b < 256; b++) cnt[b + 1] += cnt[b];
        for (int k = 0; k < nu; k++) tmp[cnt[(key[perm[k]] >> sh) & 255]++] = perm[k];
        perm.swap(tmp);
    }
}

/* Before a launch: the row order (explicit, else the feedback's for this band) and the
 * cost buffer.  Returns an rt_status. */
static int prepare_rows(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                        hipStream_t st, rt::KParams& p) {
    const int gy = (nrows + rt::TILE_H - 1) / rt::TILE_H;
    const int per_row = ((cam->width + rt::TILE_W - 1) / rt::TILE_W) * (rt::BLOCK / 64);
    const rt_ctx::Band band{cam->width, row0, nrows, ctx->scene_gen, ctx->fb_epoch, p.tstride, p.tphase};
    if (ctx->cost_pending && hipEventQuery(ctx->ev_cost) == hipSuccess) {
        ctx->cost_pending = false;
        ctx->iso_pending = false;  // the sampled frame has finished: nothing left to order
        const rt_ctx::Band& b = ctx->cost_band;
        const int bgy = (b.nrows + rt::TILE_H - 1) / rt::TILE_H;
        const int ul = ctx->cost_ul;
        const bool same = ctx->fb_band == b && ctx->fb_units_log2 == ul;  // keep smoothing
        ctx->fb_units_log2 = ul;
        order_units(ctx->h_umax, bgy << ul, ctx->fb_perm, ctx->fb_acc, same, ctx->fb_ema);
        ctx->fb_band = b;
    }
    p.row_units_log2 = 0;
    if (!ctx->row_perm.empty()) {
        if ((int)ctx->row_perm.size() == gy && gy <= rt::ROW_PERM_MAX) {
            p.row_perm_n = gy;
            std::memcpy(p.row_perm, ctx->row_perm.data(), gy * sizeof(int16_t));
        }
    } else if (ctx->feedback > 0 && ctx->fb_band == band && !ctx->fb_perm.empty()) {
        const int nu = gy << ctx->fb_units_log2;
        if ((int)ctx->fb_perm.size() == nu && nu <= rt::ROW_PERM_MAX) {
            p.row_units_log2 = ctx->fb_units_log2;
            p.row_perm_n = nu;
            std::memcpy(p.row_perm, ctx->fb_perm.data(), nu * sizeof(int16_t));
        }
    }
    // sample this frame's costs when a snapshot is due (snapshot_costs copies them)
    p.tile_cost = nullptr;
    if (ctx->feedback <= 0 || !ctx->row_perm.empty() || gy > rt::ROW_PERM_MAX || ctx->cost_pending)
        return RT_OK;
    if (!(ctx->fb_band == band)) {
        ctx->warm_left = ctx->fb_warm;  // a new band or scene: the first snapshot, then the warm ones
    } else if (ctx->warm_left > 0) {
        ctx->warm_left--;
    } else if (++ctx->since_snapshot < ctx->feedback) {
        return RT_OK;
    }
    const size_t need = (size_t)gy * per_row;
    const size_t nu = (size_t)gy << units_log2(gy, per_row);
    if (need > ctx->d_cost_cap || nu > ctx->umax_cap) {
        // grow (rare): nothing in flight may still use the old buffers
        RT_HIP(ctx, hipStreamSynchronize(st));
        const int ws = wait_inflight(ctx);
        if (ws != RT_OK) return ws;
        if (ctx->cost_pending) RT_HIP(ctx, hipEventSynchronize(ctx->ev_cost));
        ctx->cost_pending = false;
        const size_t cap = std::max(need, ctx->d_cost_cap), ucap = std::max<size_t>({nu, ctx->umax_cap, 64});
        if (ctx->d_cost) RT_HIP(ctx, hipFree(ctx->d_cost));
        if (ctx->d_umax) RT_HIP(ctx, hipFree(ctx->d_umax));
        if (ctx->h_umax) RT_HIP(ctx, hipHostFree(ctx->h_umax));
        ctx->d_cost = nullptr;
        ctx->d_umax = nullptr;
        ctx->h_umax = nullptr;
        ctx->d_cost_cap = 0;
        ctx->umax_cap = 0;
        RT_HIP(ctx, hipMalloc(&ctx->d_cost, cap * sizeof(uint16_t)));
        RT_HIP(ctx, hipMalloc(&ctx->d_umax, ucap * sizeof(uint32_t)));
        RT_HIP(ctx, hipHostMalloc(&ctx->h_umax, ucap * sizeof(uint32_t), hipHostMallocDefault));
        ctx->d_cost_cap = cap;
        ctx->umax_cap = ucap;
    }
    p.tile_cost = ctx->d_cost;
    return RT_OK;
}

/* After a launch that sampled its costs (every `feedback` frames, or at once for a band the
 * order does not cover yet): copy them back behind the kernel. */
static int snapshot_costs(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                          hipStream_t st, const rt::KParams& p) {
    if (!p.tile_cost) return RT_OK;
    const rt_ctx::Band band{cam->width, row0, nrows, ctx->scene_gen, ctx->fb_epoch, p.tstride, p.tphase};
    const int gy = (nrows + rt::TILE_H - 1) / rt::TILE_H;
    const int gx = ((cam->width + rt::TILE_W - 1) / rt::TILE_W) * (rt::BLOCK / 64);
    const int ul = units_log2(gy, gx);
    // per-unit maxima on the device, then nu words back (not every wave's cost)
    const int e = rt::launch_unit_max(ctx->d_cost, gy, gx, ul, ctx->d_umax, st);
    if (e != (int)hipSuccess) return hip_fail(ctx, (hipError_t)e, "launch k_unit_max");
    RT_HIP(ctx, hipMemcpyAsync(ctx->h_umax, ctx->d_umax, ((size_t)gy << ul) * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, st));
    RT_HIP(ctx, hipEventRecord(ctx->ev_cost, st));
    ctx->cost_pending = true;
    ctx->cost_band = band;
    ctx->cost_ul = ul;
    ctx->since_snapshot = 0;
    return RT_OK;
}

/* RT_OPT_ROW_FEEDBACK_ISOLATE: before a launch on `st` — a sampled frame first waits for
 * this ctx's latest frame on every other stream; any other frame whose stream has not yet
 * been ordered behind the pending sampled frame waits for it once.  Device-side waits only
 * (the host never blocks); streams are the ones launch_event tracks. */
static int isolate_before(rt_ctx* ctx, hipStream_t st, bool sampled) {
    if (!ctx->fb_isolate) return RT_OK;
    if (sampled) {
        // (ctx->stream is not tracked: rt_render synchronises it before returning)
        for (const auto& f : ctx->inflight)
            if (f.stream != st) RT_HIP(ctx, hipStreamWaitEvent(st, f.ev, 0));
        return RT_OK;
    }
    if (!ctx->iso_pending) return RT_OK;
    for (hipStream_t s : ctx->iso_seen)
        if (s == st) return RT_OK;
    RT_HIP(ctx, hipStreamWaitEvent(st, ctx->ev_iso, 0));
    ctx->iso_seen.push_back(st);
    return RT_OK;
}
static int isolate_after(rt_ctx* ctx, hipStream_t st, bool sampled) {
    if (!ctx->fb_isolate || !sampled) return RT_OK;
    RT_HIP(ctx, hipEventRecord(ctx->ev_iso, st));
    ctx->iso_pending = true;
    ctx->iso_seen.assign(1, st);
    return RT_OK;
}

/* RT_OPT_HOST_PIPELINE's helper thread.  A batch (rt_render_device_frames) posts its frames;
 * the helper computes each frame's make_params into a ring of RING slots, at most RING frames
 * ahead of the launching thread, which takes a slot, finishes the frame (row order, launch,
 * cost snapshot) and releases it.  make_params only reads the ctx (scene, options) and its
 * own box cache, which no other code touches while a batch runs; everything that changes
 * ctx state (the row feedback) stays on the launching thread. */
struct rt_ctx::Prep {
    static constexpr int RING = 3;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool quit = false;
    // the posted batch (valid while gen is odd... see worker): read by the helper only
    const rt_camera* cams = nullptr;
    int32_t ncams = 0, row0 = 0, nrows = 0, depth = 0, precision = 0, out_format = 0, nframes = 0;
    uint32_t flags = 0;
    void* const* d_outs = nullptr;
    int32_t nouts = 0;
    std::atomic<uint64_t> posted{0}, done{0};  // batches posted / finished by the helper
    std::atomic<int> produced{0}, consumed{0};
    std::atomic<bool> stop{false};             // the launching thread gave up on the batch
    rt::KParams slot[RING];
};

namespace {
void prep_main(rt_ctx* ctx) {
    rt_ctx::Prep& q = *ctx->prep;
    uint64_t seen = 0;
    for (;;) {
        uint64_t g = q.posted.load(std::memory_order_acquire);
        for (int it = 0; g == seen && it < 2048; it++) {
            std::this_thread::yield();
            g = q.posted.load(std::memory_order_acquire);
        }
        if (g == seen) {
            std::unique_lock<std::mutex> lk(q.mu);
            q.cv.wait(lk, [&] { return q.quit || q.posted.load(std::memory_order_acquire) != seen; });
            if (q.quit) return;
            g = q.posted.load(std::memory_order_acquire);
        }
        seen = g;
        for (int f = 0; f < q.nframes; f++) {
            while (f - q.consumed.load(std::memory_order_acquire) >= rt_ctx::Prep::RING &&
                   !q.stop.load(std::memory_order_acquire))
                std::this_thread::yield();
            if (q.stop.load(std::memory_order_acquire)) break;
            q.slot[f % rt_ctx::Prep::RING] =
                make_params(ctx, &q.cams[f % q.ncams], q.row0, q.nrows, q.depth, q.flags, q.out_format,
                            q.d_outs[f % q.nouts], nullptr, q.precision);
            q.produced.store(f + 1, std::memory_order_release);
        }
        q.done.store(seen, std::memory_order_release);
    }
}
void prep_shutdown(rt_ctx* ctx) {
    if (!ctx->prep) return;
    {
        std::lock_guard<std::mutex> lk(ctx->prep->mu);
        ctx->prep->quit = true;
    }
    ctx->prep->cv.notify_one();
    if (ctx->prep->th.joinable()) ctx->prep->th.join();
    delete ctx->prep;
    ctx->prep = nullptr;
}
}  // namespace

/* Pixel rows of interleaved part `part` of `nparts` (tile rows part, part + nparts, ...). */
static int32_t interleaved_rows(int32_t height, int32_t nparts, int32_t part) {
    const int32_t T = (height + rt::TILE_H - 1) / rt::TILE_H;
    int32_t n = 0;
    for (int32_t t = part; t < T; t += nparts) n += std::min(rt::TILE_H, height - t * rt::TILE_H);
    return n;
}

/* One frame whose arguments are complete (prepare_rows done): the stream's in-flight event,
 * the isolation waits, the launch, the cost snapshot of a sampled frame. */
static int launch_prepared(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                           const rt::KParams& p, int32_t precision, hipStream_t hs,
                           double* hp = nullptr) {
#if RT_HOST_PROFILE
    double hp_local = hp ? *hp : hp_now();
    double& hp_t = hp ? *hp : hp_local;
#else
    (void)hp;
#endif
    hipEvent_t done = nullptr;
    int st = launch_event(ctx, hs, &done);
    if (st != RT_OK) return st;
    const bool sampled = p.tile_cost != nullptr;
    st = isolate_before(ctx, hs, sampled);
    if (st != RT_OK) return st;
    HP(2);
    // RT_DRY_LAUNCH (diagnostic builds, tools/multi_host_cost.py): every host step of the
    // frame but the kernel launch, to separate the host's own work from the runtime's
    const int e = RT_DRY_LAUNCH ? (int)hipSuccess : rt::launch_trace(p, precision, hs, done);
    if (e != (int)hipSuccess) return hip_fail(ctx, (hipError_t)e, "launch k_trace");
    if (RT_DRY_LAUNCH) return RT_OK;
    st = isolate_after(ctx, hs, sampled);
    if (st != RT_OK) return st;
    HP(3);
    st = snapshot_costs(ctx, cam, row0, nrows, hs, p);
    HP(4);
    return st;
}

/* rt_render_device and rt_render_device_interleaved: a contiguous band [row0, row0 + nrows)
 * (nparts == 0) or interleaved part `part` of `nparts` (nrows = its pixel rows). */
static int render_device_impl(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                              int32_t nparts, int32_t part, int32_t out_frame, int32_t depth,
                              int32_t precision, uint32_t flags, int32_t out_format, void* d_out,
                              uint64_t* d_segments, void* stream, const rt::KParams* pre = nullptr) {
#if RT_HOST_PROFILE
    double hp_t = hp_now();
    g_hn++;
#endif
    int st = check_render_args(ctx, cam, row0, nrows, depth, precision, out_format);
    if (st != RT_OK) return st;
    if (!d_out && nrows > 0 && cam->width > 0) return RT_ERR_INVALID_ARG;
    // the ctx's buffers (row feedback) and the launch belong to ctx->device, whatever
    // device the caller has current
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    HP(0);
    // an interleaved part's tile rows span the frame: its pixel boxes are the whole frame's
    // (pre: computed by the host pipeline's helper thread, contiguous bands only)
    rt::KParams p = pre ? *pre
                        : make_params(ctx, cam, nparts > 1 ? 0 : row0, nparts > 1 ? cam->height : nrows,
                                      depth, flags, out_format, d_out,
                                      reinterpret_cast<unsigned long long*>(d_segments), precision);
    if (nparts > 1) {
        p.row0 = 0;
        p.nrows = nrows;
        p.tstride = nparts;
        p.tphase = part;
        p.frame_h = cam->height;
        p.out_frame = out_frame ? 1 : 0;
        p.pairs = 0;  // the two-pixel kernel is contiguous-only
        // centre-out dispatch from the part's tile row nearest the frame's heavy row
        const int nt = (nrows + rt::TILE_H - 1) / rt::TILE_H;
        p.row_center = std::max(0, std::min(nt - 1, (p.row_center - part) / nparts));
    }
    HP(1);
    void* s = stream ? stream : static_cast<void*>(ctx->stream);
    hipStream_t hs = static_cast<hipStream_t>(s);
    st = prepare_rows(ctx, cam, row0, nrows, hs, p);
    if (st != RT_OK) return st;
#if RT_HOST_PROFILE
    return launch_prepared(ctx, cam, row0, nrows, p, precision, hs, &hp_t);
#else
    return launch_prepared(ctx, cam, row0, nrows, p, precision, hs);
#endif
}

int rt_render_device(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows,
                     int32_t depth, int32_t precision, uint32_t flags, int32_t out_format,
                     void* d_out, uint64_t* d_segments, void* stream) {
    return render_device_impl(ctx, cam, row0, nrows, 0, 0, 0, depth, precision, flags, out_format,
                              d_out, d_segments, stream);
}

int rt_interleaved_rows(int32_t height, int32_t nparts, int32_t part, int32_t* nrows) {
    if (!nrows || height < 0 || nparts <= 0 || part < 0 || part >= nparts) return RT_ERR_INVALID_ARG;
    *nrows = interleaved_rows(height, nparts, part);
    return RT_OK;
}

int rt_render_device_interleaved(rt_ctx* ctx, const rt_camera* cam, int32_t nparts, int32_t part,
                                 int32_t depth, int32_t precision, uint32_t flags,
                                 int32_t out_format, void* d_out, int32_t out_frame_rows,
                                 uint64_t* d_segments, void* stream) {
    if (!ctx || !cam || nparts <= 0 || part < 0 || part >= nparts || cam->height < 0)
        return RT_ERR_INVALID_ARG;
    if (nparts == 1)  // the whole frame: a contiguous band, stored at its frame rows anyway
        return render_device_impl(ctx, cam, 0, cam->height, 0, 0, 0, depth, precision, flags,
                                  out_format, d_out, d_segments, stream);
    if (rt::TILE_H != 8) return RT_ERR_UNSUPPORTED;  // parts are dealt in 8-row tile rows
    return render_device_impl(ctx, cam, 0, interleaved_rows(cam->height, nparts, part), nparts,
                              part, out_frame_rows, depth, precision, flags, out_format, d_out,
                              d_segments, stream);
}

/* RT_OPT_FRAME_BATCH: a group of n >= 2 prepared frames of one stream (their arguments in
 * the pinned table slot s) as one launch — the slot copied into the device table behind the
 * stream's earlier work, then one grid of n frames whose stop event marks the slot free
 * again; n == 1 is an ordinary launch. */
static int launch_group(rt_ctx* ctx, int s, int n, const rt_camera* cam, int32_t row0, int32_t nrows,
                        int32_t precision, hipStream_t hs) {
    if (n <= 0) return RT_OK;
    rt::KParams* grp = ctx->h_tab + (size_t)s * RT_MULTI_BATCH_MAX;
    if (n == 1) return launch_prepared(ctx, cam, row0, nrows, grp[0], precision, hs);
    int st = isolate_before(ctx, hs, false);
    if (st != RT_OK) return st;
    rt::KParams* dst = ctx->d_tab + (size_t)s * RT_MULTI_BATCH_MAX;
    RT_HIP(ctx, hipMemcpyAsync(dst, grp, (size_t)n * sizeof(rt::KParams), hipMemcpyHostToDevice, hs));
    const int e = RT_DRY_LAUNCH ? (int)hipSuccess
                                : rt::launch_trace_batch(dst, grp[0], n, precision, hs, ctx->tab_ev[s]);
    if (e != (int)hipSuccess) return hip_fail(ctx, (hipError_t)e, "launch k_trace_tab");
    ctx->tab_busy[s] = !RT_DRY_LAUNCH;
    ctx->tab_next = (s + 1) % rt_ctx::TAB_SLOTS;
    return RT_OK;
}

/* The pipelined frame loop with RT_OPT_FRAME_BATCH: consecutive frames are grouped while they
 * share a stream (frames on one stream run in order anyway), write distinct buffers, have
 * the same grid (a row order change between them starts a new group) and are not sampled by
 * the row feedback (a sampled frame runs alone, through the stamped kernels, then its cost
 * snapshot); each group is one launch.  Every frame's arguments, row order and feedback
 * bookkeeping are the per-frame loop's, so the output is identical. */
static int launch_frame_groups(rt_ctx* ctx, const rt_camera* cams, int32_t ncams, int32_t row0,
                               int32_t nrows, int32_t precision, void* const* d_outs, int32_t nouts,
                               void* const* streams, int32_t nstreams, int32_t nframes) {
    rt_ctx::Prep& q = *ctx->prep;
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    if (!ctx->d_tab) {
        const size_t n = (size_t)rt_ctx::TAB_SLOTS * RT_MULTI_BATCH_MAX;
        for (auto& e : ctx->tab_ev)
            if (!e) RT_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (!ctx->h_tab) RT_HIP(ctx, hipHostMalloc(&ctx->h_tab, n * sizeof(rt::KParams), hipHostMallocDefault));
        RT_HIP(ctx, hipMalloc(&ctx->d_tab, n * sizeof(rt::KParams)));
    }
    int st = RT_OK;
    int32_t f = 0;
    while (f < nframes && st == RT_OK) {
        void* const stf = nstreams > 0 ? streams[f % nstreams] : nullptr;
        hipStream_t hs = static_cast<hipStream_t>(stf ? stf : static_cast<void*>(ctx->stream));
        const int s = ctx->tab_next;  // this group's table slot: free once its last launch ended
        if (ctx->tab_busy[s]) {
            RT_HIP(ctx, hipEventSynchronize(ctx->tab_ev[s]));
            ctx->tab_busy[s] = false;
        }
        rt::KParams* grp = ctx->h_tab + (size_t)s * RT_MULTI_BATCH_MAX;
        const void* outs[RT_MULTI_BATCH_MAX];
        int n = 0;
        const rt_camera* cam0 = &cams[f % ncams];
        while (f < nframes && n < ctx->frame_batch) {
            void* const st2 = nstreams > 0 ? streams[f % nstreams] : nullptr;
            void* const out = d_outs[f % nouts];
            if (n > 0 && (st2 != stf || std::find(outs, outs + n, out) != outs + n)) break;
            while (q.produced.load(std::memory_order_acquire) <= f) std::this_thread::yield();
            rt::KParams& p = grp[n];
            p = q.slot[f % rt_ctx::Prep::RING];
            q.consumed.store(f + 1, std::memory_order_release);
            const rt_camera* cam = &cams[f % ncams];
            st = prepare_rows(ctx, cam, row0, nrows, hs, p);
            if (st != RT_OK) break;
            const bool other_grid = n > 0 && (p.W != grp[0].W || p.nrows != grp[0].nrows ||
                                              p.row_units_log2 != grp[0].row_units_log2);
            if (p.tile_cost || other_grid) {
                // this frame alone (after the frames grouped so far), through the per-frame path
                const rt::KParams one = p;
                st = launch_group(ctx, s, n, cam0, row0, nrows, precision, hs);
                if (st == RT_OK) st = launch_prepared(ctx, cam, row0, nrows, one, precision, hs);
                n = 0;
                f++;
                break;
            }
            outs[n++] = out;
            f++;
        }
        if (st == RT_OK) st = launch_group(ctx, s, n, cam0, row0, nrows, precision, hs);
    }
    // the helper thread must not wait for a consumer that stopped early
    q.consumed.store(nframes, std::memory_order_release);
    return st;
}

/* rt_render_device_frames with the host pipeline (RT_OPT_HOST_PIPELINE): the helper thread
 * computes make_params of the next frames while this thread launches the current one, so a
 * frame costs the host max(arguments, launch) instead of their sum.  Same launches, same
 * order, same arguments as the sequential loop. */
static int render_frames_pipelined(rt_ctx* ctx, const rt_camera* cams, int32_t ncams, int32_t row0,
                                   int32_t nrows, int32_t depth, int32_t precision, uint32_t flags,
                                   int32_t out_format, void* const* d_outs, int32_t nouts,
                                   void* const* streams, int32_t nstreams, int32_t nframes) {
    if (!ctx->prep) {
        ctx->prep = new (std::nothrow) rt_ctx::Prep();
        if (!ctx->prep) return RT_ERR_OUT_OF_MEMORY;
        try {
            ctx->prep->th = std::thread(prep_main, ctx);
        } catch (...) {
            delete ctx->prep;
            ctx->prep = nullptr;
            return RT_ERR_OUT_OF_MEMORY;
        }
    }
    rt_ctx::Prep& q = *ctx->prep;
    q.cams = cams;
    q.ncams = ncams;
    q.row0 = row0;
    q.nrows = nrows;
    q.depth = depth;
    q.precision = precision;
    q.flags = flags;
    q.out_format = out_format;
    q.d_outs = d_outs;
    q.nouts = nouts;
    q.nframes = nframes;
    q.produced.store(0, std::memory_order_relaxed);
    q.consumed.store(0, std::memory_order_relaxed);
    q.stop.store(false, std::memory_order_relaxed);
    uint64_t g;
    {
        std::lock_guard<std::mutex> lk(q.mu);
        g = q.posted.load(std::memory_order_relaxed) + 1;
        q.posted.store(g, std::memory_order_release);
    }
    q.cv.notify_one();
    int st = RT_OK;
    if (ctx->frame_batch > 1) {
        st = launch_frame_groups(ctx, cams, ncams, row0, nrows, precision, d_outs, nouts, streams,
                                 nstreams, nframes);
    } else {
        for (int32_t f = 0; f < nframes; f++) {
            while (q.produced.load(std::memory_order_acquire) <= f) std::this_thread::yield();
            void* stf = nstreams > 0 ? streams[f % nstreams] : nullptr;
            st = render_device_impl(ctx, &cams[f % ncams], row0, nrows, 0, 0, 0, depth, precision, flags,
                                    out_format, d_outs[f % nouts], nullptr, stf,
                                    &q.slot[f % rt_ctx::Prep::RING]);
            q.consumed.store(f + 1, std::memory_order_release);
            if (st != RT_OK) break;
        }
    }
    // the helper is done with this batch before its arguments (cams, d_outs) go out of scope
    q.stop.store(true, std::memory_order_release);
    while (q.done.load(std::memory_order_acquire) != g) std::this_thread::yield();
    return st;
}

int rt_render_device_frames(rt_ctx* ctx, const rt_camera* cams, int32_t ncams, int32_t row0,
                            int32_t nrows, int32_t depth, int32_t precision, uint32_t flags,
                            int32_t out_format, void* const* d_outs, int32_t nouts,
                            void* const* streams, int32_t nstreams, int32_t nframes) {
    if (!ctx || !cams || ncams <= 0 || !d_outs || nouts <= 0 || nframes < 0 ||
        (nstreams > 0 && !streams) || nstreams < 0)
        return RT_ERR_INVALID_ARG;
    if (ctx->host_pipeline && nframes >= 2 && !RT_DRY_LAUNCH) {
        // every frame's arguments checked up front (the pipeline's helper computes them
        // unchecked); a batch with an invalid frame takes the sequential loop, which stops
        // at that frame with its status
        bool ok = true;
        for (int32_t c = 0; c < ncams && c < nframes && ok; c++)
            ok = check_render_args(ctx, &cams[c], row0, nrows, depth, precision, out_format) == RT_OK;
        for (int32_t f = 0; f < nframes && f < nouts && ok; f++)
            ok = d_outs[f] != nullptr || nrows == 0 || cams[f % ncams].width == 0;
        if (ok)
            return render_frames_pipelined(ctx, cams, ncams, row0, nrows, depth, precision, flags,
                                           out_format, d_outs, nouts, streams, nstreams, nframes);
    }
    for (int32_t f = 0; f < nframes; f++) {
        void* st = nstreams > 0 ? streams[f % nstreams] : nullptr;
        const int e = rt_render_device(ctx, &cams[f % ncams], row0, nrows, depth, precision,
                                       flags, out_format, d_outs[f % nouts], nullptr, st);
        if (e != RT_OK) return e;
    }
    return RT_OK;
}

int rt_render(rt_ctx* ctx, const rt_camera* cam, int32_t row0, int32_t nrows, int32_t depth,
              int32_t precision, uint32_t flags, int32_t out_format, void* out,
              int32_t count_segments, rt_stats* stats) {
    int st = check_render_args(ctx, cam, row0, nrows, depth, precision, out_format);
    if (st != RT_OK) return st;
    const size_t bytes = (size_t)nrows * (size_t)cam->width * (size_t)bytes_per_pixel(out_format);
    if (!out && bytes > 0) return RT_ERR_INVALID_ARG;
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    if (bytes > ctx->d_out_cap) {
        RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->d_out) RT_HIP(ctx, hipFree(ctx->d_out));
        ctx->d_out = nullptr;
        ctx->d_out_cap = 0;
        RT_HIP(ctx, hipMalloc(&ctx->d_out, bytes));
        ctx->d_out_cap = bytes;
    }
    unsigned long long* segs = count_segments ? ctx->d_segs : nullptr;
    if (segs) RT_HIP(ctx, hipMemsetAsync(segs, 0, sizeof *segs, ctx->stream));
    rt::KParams p = make_params(ctx, cam, row0, nrows, depth, flags, out_format,
                                ctx->d_out, segs, precision);
    st = prepare_rows(ctx, cam, row0, nrows, ctx->stream, p);
    if (st != RT_OK) return st;
    RT_HIP(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    const int e = rt::launch_trace(p, precision, ctx->stream);
    if (e != (int)hipSuccess) return hip_fail(ctx, (hipError_t)e, "launch k_trace");
    RT_HIP(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    st = snapshot_costs(ctx, cam, row0, nrows, ctx->stream, p);
    if (st != RT_OK) return st;
    if (bytes > 0)
        RT_HIP(ctx, hipMemcpyAsync(out, ctx->d_out, bytes, hipMemcpyDeviceToHost, ctx->stream));
    unsigned long long hsegs = 0;
    if (segs)
        RT_HIP(ctx, hipMemcpyAsync(&hsegs, segs, sizeof hsegs, hipMemcpyDeviceToHost, ctx->stream));
    RT_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (stats) {
        float ms = 0.f;
        RT_HIP(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        stats->ms = ms;
        stats->segments = hsegs;
    }
    return RT_OK;
}

}  // extern "C"

int rt_tile_row_costs(rt_ctx* ctx, const rt_camera* cam, int32_t depth, int32_t precision,
                      uint32_t flags, float* costs, int32_t n) {
    const int32_t H = cam ? cam->height : 0;
    int st = check_render_args(ctx, cam, 0, H, depth, precision, RT_OUT_RGB_F32);
    if (st != RT_OK) return st;
    const int gy = (H + rt::TILE_H - 1) / rt::TILE_H;
    if (!costs || n != gy) return RT_ERR_INVALID_ARG;
    if (gy == 0 || cam->width == 0) {
        for (int t = 0; t < n; t++) costs[t] = 0.0f;
        return RT_OK;
    }
    DeviceGuard dg(ctx->device);
    RT_HIP(ctx, dg.err);
    const int per_row = ((cam->width + rt::TILE_W - 1) / rt::TILE_W) * (rt::BLOCK / 64);
    const size_t nw = (size_t)gy * per_row;
    const size_t out_bytes = (size_t)H * cam->width * 12;
    // scratch for this call only (the frame's pixels and every wave's cost)
    void* d_img = nullptr;
    uint16_t* d_c = nullptr;
    std::vector<uint16_t> h_c(nw);
    auto release = [&] {
        if (d_img) (void)hipFree(d_img);
        if (d_c) (void)hipFree(d_c);
    };
    hipError_t e = hipMalloc(&d_img, out_bytes);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_c), nw * sizeof(uint16_t));
    if (e == hipSuccess) e = hipMemsetAsync(d_c, 0, nw * sizeof(uint16_t), ctx->stream);
    if (e != hipSuccess) {
        release();
        return hip_fail(ctx, e, "rt_tile_row_costs buffers");
    }
    rt::KParams p = make_params(ctx, cam, 0, H, depth, flags, RT_OUT_RGB_F32, d_img, nullptr, precision);
    p.pairs = 0;        // one tile per wave: costs[t] sums tile row t's waves
    p.tile_cost = d_c;  // the stamped kernels
    const int le = rt::launch_trace(p, precision, ctx->stream);
    if (le == (int)hipSuccess) e = hipMemcpyAsync(h_c.data(), d_c, nw * sizeof(uint16_t), hipMemcpyDeviceToHost, ctx->stream);
    if (le == (int)hipSuccess && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    release();
    if (le != (int)hipSuccess) return hip_fail(ctx, (hipError_t)le, "launch k_trace (stamped)");
    if (e != hipSuccess) return hip_fail(ctx, e, "rt_tile_row_costs copy");
    for (int t = 0; t < gy; t++) {
        double s = 0.0;
        for (int k = 0; k < per_row; k++) s += h_c[(size_t)t * per_row + k];
        costs[t] = (float)s;
    }
    return RT_OK;
}

#if RT_HOST_BENCH
/* Diagnostic build only (-DRT_HOST_BENCH=1, tools/host_bench.py): the per-frame host work of
 * a render, timed on the CPU with no device — out_us[0] = make_params (everything the host
 * computes per frame), [1] = frame_boxes alone, [2] = the KParams value-init + copy. */
extern "C" int rt_host_bench(const rt_prim* prims, int32_t n, const rt_camera* cam, int32_t row0,
                             int32_t nrows, int32_t iters, double* out_us) {
    std::unique_ptr<rt_ctx> ctx(new rt_ctx());
    const int st = pack_scene(prims, n, ctx->sc);
    if (st != RT_OK) return st;
    ctx->have_scene = true;
    ctx->wave_cull_min = 0x7fffffff;
    std::unique_ptr<rt::KParams> p(new rt::KParams);
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
    };
    volatile int sink = 0;
    auto t0 = clk::now();
    for (int k = 0; k < iters; k++) {
        *p = make_params(ctx.get(), cam, row0, nrows, 4, 0, RT_OUT_RGB_F32, nullptr, nullptr, RT_PREC_PATH64);
        sink += p->nbox;
    }
    auto t1 = clk::now();
    for (int k = 0; k < iters; k++) {
        frame_boxes(ctx.get(), cam, row0, nrows, *p);
        sink += p->nbox;
    }
    auto t2 = clk::now();
    for (int k = 0; k < iters; k++) {
        rt::KParams q{};
        q.nbox = k;
        *p = q;
        sink += p->nbox;
    }
    auto t3 = clk::now();
    out_us[0] = us(t0, t1) / iters;
    out_us[1] = us(t1, t2) / iters;
    out_us[2] = us(t2, t3) / iters;
    (void)sink;
    return RT_OK;
}
#endif
