/*
 * rt_trace.hip — the per-pixel trace/shade hot path for gfx950 (CDNA4), one thread
 * per pixel.  Replaces the reference's rt_scene loop (main.cpp:124-139) and
 * everything under it: primary ray generation (main.cpp:132-134),
 * recursive_ray_tracing (main.cpp:89-119), find_closest_hit (main.cpp:67-84),
 * Sphere::intersect (scene.cpp:40-78), Wall::intersect (scene.cpp:4-35), the shading
 * helpers out_color / diffuse_shading / specular (main.cpp:28-62) and vec3
 * (vec.cpp:3-57).
 *
 * Precisions (template PREC):
 *   PREC_F64   the reference's fp64 arithmetic.  This TU is built with
 *              -ffp-contract=off, so nothing is fused that the reference (x86-64, no
 *              FMA) does not fuse; where operations are restructured for speed the
 *              result is provably bit-identical (see "exact rewrites" below).  The only
 *              non-bit-exact operations are pow (x^e by squaring for integer e, sky
 *              z^0.25 as sqrt(sqrt(z))): <= a few ulp, vs glibc's correctly rounded pow.
 *   PREC_F32   fp32 with fused multiply-adds and hardware rcp/rsq/sqrt/exp/log: the
 *              throughput path; flips at geometric discontinuities.
 *   PREC_MIXED fp32 conservative cull in the primitive scan, PREC_F64's exact test on
 *              every primitive the cull cannot reject, fp64 shading: output == F64.
 *   PREC_PATH64 PREC_F64's exact ray path (hits, positions, normals, reflections) with
 *              the colour arithmetic (shading, sky, lerp) in fp32: every pixel follows the
 *              reference's path, colours within ~1e-6 (no discontinuity flips).
 *
 * Exact rewrites (each identity holds in IEEE binary64 barring overflow/underflow):
 *   - b = 2*dot(d,oc) is exact, so b*b - (4a)*c == 4*(dot*dot - a*c) and
 *     (-b - sqrt(det)) / (2a) == (-dot - sqrt(det/4)) / a (power-of-two scalings
 *     commute with rounding; sqrt(4x) == 2*sqrt(x)).
 *   - x / y for several x and one y: LLVM's fp64 division is rcp + two Newton steps +
 *     one fma correction wrapped in div_scale/div_fixup, which are identities for
 *     normal-range operands; sharing the refined reciprocal across numerators gives
 *     the same bits (checked on device by rt_selftest, tests/test_gpu_parity.py).
 *   - normalize(-d) == -normalize(d) (negation commutes with rounding).
 *
 * Recursion -> iteration with identical rounding: the reference returns
 * lerp(local, traced, metallic) from the innermost bounce outward (vec.cpp:45-49).
 * Each bounce pushes (shading scalar s, sun scalar, material slot) onto a per-thread
 * register stack indexed by the wave-uniform bounce counter; the stack is unwound in
 * reverse with the same operations, so local = color*s is recomputed bit-identically.
 */
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include <algorithm>
#include <type_traits>

#include "rt_device.h"

#ifndef RT_WALLS_FIRST
#define RT_WALLS_FIRST 1
#endif
#ifndef RT_WALL_NOSIGN     // 1: the wall test forms t = num/den for every lane and keeps t > 0 and
#define RT_WALL_NOSIGN 1   // t <= best in ONE branch, instead of a sign pre-test branch, then a
#endif                     // t > 0 branch, then the t-skip branch (fewer exec-mask instructions)
#ifndef RT_F32_WALL_FLAT   // F32 wall test without the sign pre-test branch: one branch per wall
#define RT_F32_WALL_FLAT 1
#endif
#ifndef RT_WALL_BOUNDS_FLAT  // A/B knob: the wall's four bounds in one predicate (measured
#define RT_WALL_BOUNDS_FLAT 0    // neutral at c1-c5: off)
#endif
#ifndef RT_SPHERE_ONEBRANCH  // 1: Sphere::intersect's two early rejections (b > 0, det < 0)
#define RT_SPHERE_ONEBRANCH 1  // share one branch (det/4 formed for every lane: 2 VALU)
#endif
#ifndef RT_WALL_TSKIP      // 1: a wall whose t exceeds the current best skips its bounds
#define RT_WALL_TSKIP 1    // test (exact: the reference's strict < rejects it anyway);
#endif                     // fp64 paths only (the branch costs the fp32 path ~1% at c5)
#ifndef RT_TERMINAL_F32    // PATH64: the last segment of a path (sky, or the hit at max
#define RT_TERMINAL_F32 1  // depth) feeds colour only, so its normalisations run in fp32
#endif
#ifndef RT_LAZY_TERMS      // PATH64: |d|^2, 1/|d|^2, |d| only when a sphere test or a
#define RT_LAZY_TERMS 0    // reflection needs them (wave-uniform; A/B: +2% at c2, off)
#endif
#ifndef RT_PEEL            // 1: the primary segment peeled off the bounce loop (straight-line);
#define RT_PEEL 2          // 2: the first bounce too (c2 PATH64 -3%, F64 -4% over 1)
#endif
#ifndef RT_SKY_FAST        // PATH64/F32 linear scan: a tile whose keep mask is empty (no primitive's
#define RT_SKY_FAST 1      // pixel box meets it: every primary ray misses) shades its sky/ground
#endif                     // at once, without |d|^2, 1/|d|^2, |d| or the bounce loop
#ifndef RT_BOX_SCHED_BARRIER
#define RT_BOX_SCHED_BARRIER 1
#endif
#ifndef RT_CLUSTERS        // 1: cull kernels' wide-cone waves scan per-lane sphere clusters
#define RT_CLUSTERS 1
#endif
#ifndef RT_CLU_OCT         // 1: lanes walk their clusters in a per-octant near-to-far order
#define RT_CLU_OCT 1
#endif
#ifndef RT_CLU_OCT_F32     // the same for the F32 kernels (A/B: c5 F32 +4.5%, PATH64 -2..2.5%)
#define RT_CLU_OCT_F32 0
#endif
#ifndef RT_CLUSTERS_F64    // 1: the same for the fp64-colour (F64, MIXED) cull kernels (A/B:
                           // c5 F64 -44%, MIXED -36%, c3 F64 -14.5%, MIXED -9%)
#define RT_CLUSTERS_F64 1
#endif
#ifndef RT_CLUSTERS_F32    // 1: the same for the F32 cull kernels
#define RT_CLUSTERS_F32 1
#endif
#ifndef RT_WALL_ORDER      // 1: the primary scan visits walls in the host's per-frame order
#define RT_WALL_ORDER 1    // (nearest to the camera first) when KParams::wall_order is set
#endif
#ifndef RT_WALL_PAIRS      // exact wall tests two at a time in one basic block (ILP)
#define RT_WALL_PAIRS 0    // A/B: +10% at c2 (lost t-skip, +16 VGPRs), off
#endif
#ifndef RT_UNWIND_KEND
#define RT_UNWIND_KEND 1
#endif
#ifndef RT_WAVE_TIMES      // diagnostic build: per-wave start/end stamps into KParams::stats
#define RT_WAVE_TIMES 0    // (tools/wave_times.py); never on in the product
#endif
#ifndef RT_STAGE_TIMES     // diagnostic build: shader-clock stamps at stage boundaries of every
#define RT_STAGE_TIMES 0   // wave into KParams::stats (tools/stage_times.py); never in the product
#endif
#if RT_STAGE_TIMES
#define STAGE(i) (g_stage[(i)] = __builtin_amdgcn_s_memtime())
#else
#define STAGE(i) \
    do {         \
    } while (0)
#endif
#ifndef RT_DIAG            // diagnostic build: count wave/lane entries of branch bodies
#define RT_DIAG 0          // into g_diag (rt_diag_read); never on in the product
#endif
#ifndef RT_STAMP
#define RT_STAMP 0  // 1 in rt_trace_stamp.hip: the same kernels, recording each wave's cost
#endif
#if RT_DIAG && RT_STAMP
#undef RT_DIAG
#define RT_DIAG 0
#endif
#if RT_DIAG
__device__ unsigned long long g_diag[16];
#define DIAG(i)                                                                     \
    do {                                                                            \
        const uint64_t b_ = __ballot(1);                                            \
        if ((uint64_t)__lane_id() == (uint64_t)__builtin_ctzll(b_)) {                \
            atomicAdd(&g_diag[(i)], 1ull);                                          \
            atomicAdd(&g_diag[(i) + 1], (unsigned long long)__popcll(b_));          \
        }                                                                           \
    } while (0)
#else
#define DIAG(i) \
    do {        \
    } while (0)
#endif
#ifndef RT_WPE_PATH64           // occupancy targets (waves_per_eu below), A/B knobs
#define RT_WPE_PATH64 5
#endif
#ifndef RT_WPE_PATH64_CULL_BONUS  // PATH64 cull kernels, depth <= 8, no sun: 6 waves/SIMD (79
#define RT_WPE_PATH64_CULL_BONUS 1   // VGPRs, no scratch; A/B c5 -4.1%, c3 -6.1% vs 5, round 4)
#endif
#ifndef RT_WPE_PATH64_LIN_BONUS
#define RT_WPE_PATH64_LIN_BONUS 0
#endif
#ifndef RT_WPE_MIXED_CULL_DROP  // MIXED cull kernels at depth > 4: one wave less
#define RT_WPE_MIXED_CULL_DROP 1
#endif
#ifndef RT_WPE_F32_BONUS
#define RT_WPE_F32_BONUS 0
#endif
#ifndef RT_WPE_CULL64_BONUS  // F64/MIXED cull kernels: one wave/SIMD more since the recursion
#define RT_WPE_CULL64_BONUS 1    // stack moved to LDS (A/B: c5 F64 -3.5%, c3 F64 -5.6% vs 4 waves)
#endif
#ifndef RT_WPE_F64_LIN_BONUS
#define RT_WPE_F64_LIN_BONUS 0
#endif
#ifndef RT_STACK_LDS      // 1: the cull kernels keep the recursion stack in LDS (trace_pixel_d)
#define RT_STACK_LDS 1
#endif
/* RT_AB_SLIM (A/B builds only, tools/build_variant.sh): instantiate the PATH64 no-sun
 * kernels of depth <= 8 alone (c1-c5's bench kernels), so an experiment compiles in a
 * fraction of the full family's time; any other launch fails with hipErrorInvalidValue. */
#ifndef RT_AB_SLIM
#define RT_AB_SLIM 0
#endif
#ifndef RT_F32_READLANE   // F32 survivor records: 1 = v_readlane from the culling lane,
#define RT_F32_READLANE 0 // 0 = scalar loads (A/B: c5 -13%); fp64 paths keep v_readlane
#endif

namespace rt {
// The kernels are built twice, as rt::kno (this file) and rt::kst (rt_trace_stamp.hip, for
// the frames whose costs the host samples for the dispatch order, rt_capi.cpp): a wave-start
// s_memtime costs ~15% at c2 wherever it sits (tools/ab.py), so the plain kernels have none.
#if RT_STAMP
namespace kst {
#else
namespace kno {
#endif

/* ------------------------------------------------------------------------ */
/* fp64 vector math, vec.cpp:3-57 (this TU: -ffp-contract=off)               */
/* ------------------------------------------------------------------------ */
struct d3 {
    double x, y, z;
};
__device__ __forceinline__ d3 D3(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return D3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return D3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ d3 operator-(d3 a) { return D3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ d3 operator*(d3 a, d3 b) { return D3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ d3 operator*(d3 a, double s) { return D3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double lensq(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ d3 lerp(d3 a, d3 b, double t) {
    return D3(a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z));
}
__device__ __forceinline__ d3 ld3(const double* p) { return D3(p[0], p[1], p[2]); }

/* Reciprocal refined exactly as LLVM's fp64 division refines it (rcp + 2 Newton). */
__device__ __forceinline__ double rcp_refined(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(r, e, r);
}
/* a / b correctly rounded, given r = rcp_refined(b) (a == 0 keeps IEEE's signed zero). */
__device__ __forceinline__ double div_r(double a, double b, double r) {
    const double q = a * r;
    const double e = __builtin_fma(-b, q, a);
    const double q1 = __builtin_fma(e, r, q);
    return a == 0.0 ? q : q1;
}
/* a / b for a != 0 (or where the sign of a zero quotient cannot matter): div_r without
 * its a == 0 select. */
__device__ __forceinline__ double div_r_nz(double a, double b, double r) {
    const double q = a * r;
    const double e = __builtin_fma(-b, q, a);
    return __builtin_fma(e, r, q);
}
/* sqrt(x) correctly rounded: LLVM's fp64 sqrt sequence (rsq + Goldschmidt/Newton
 * refinement) without its range scaling, which is the identity for x >= 2^-767; smaller
 * (and zero/negative) arguments take the library path. */
#ifndef RT_SQRT_UNIFORM   // 1: the rare-argument fallback behind a wave-uniform test (one
#define RT_SQRT_UNIFORM 0 // ballot) instead of a divergent branch (exec-mask save/restore)
#endif
__device__ __forceinline__ double sqrt_fast(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
#ifndef RT_SQRT_FLAT      // A/B knob (off: +2..4% VALU-bound): 1 = sqrt_e without a branch: LLVM's own range scaling (x < 2^-767 is
#define RT_SQRT_FLAT 0    // scaled by 2^256, the root by 2^-128) and its +-0/+inf passthrough as
#endif                    // selects — the same instructions the library path runs, so the same bits
__device__ __forceinline__ double sqrt_e(double x) {
    if (RT_SQRT_FLAT) {
        const bool sm = x < 0x1p-767;
        const double xs = __builtin_amdgcn_ldexp(x, sm ? 256 : 0);
        const double y = __builtin_amdgcn_rsq(xs);
        double g = xs * y;
        double h = y * 0.5;
        const double r = __builtin_fma(-h, g, 0.5);
        g = __builtin_fma(g, r, g);
        double d = __builtin_fma(-g, g, xs);
        h = __builtin_fma(h, r, h);
        g = __builtin_fma(d, h, g);
        d = __builtin_fma(-g, g, xs);
        g = __builtin_fma(d, h, g);
        g = __builtin_amdgcn_ldexp(g, sm ? -128 : 0);
        // +-0 and +inf are their own roots (LLVM: v_cmp_class mask 0x260)
        return __builtin_amdgcn_class(xs, 0x260) ? xs : g;
    }
    if (RT_SQRT_UNIFORM) {
        const bool ok = x >= 0x1p-767 && x <= DBL_MAX;
        if (__builtin_expect(__ballot(!ok) != 0, 0)) return ok ? sqrt_fast(x) : sqrt(x);
        return sqrt_fast(x);
    }
    // tiny, zero, negative, NaN and +inf take the library path (+inf: rsq(inf) = 0 would
    // give inf * 0 = NaN below; the library passes inf through)
    if (!(x >= 0x1p-767 && x <= DBL_MAX)) return sqrt(x);
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
/* v / len(v) component-wise (vec.cpp:21), one shared reciprocal. */
__device__ __forceinline__ d3 normalize_e(d3 v) {
    const double l = sqrt_e(lensq(v));
    const double r = rcp_refined(l);
    return D3(div_r(v.x, l, r), div_r(v.y, l, r), div_r(v.z, l, r));
}
__device__ __forceinline__ d3 div3(d3 v, double l, double r) {
    return D3(div_r(v.x, l, r), div_r(v.y, l, r), div_r(v.z, l, r));
}
/* x^n for x >= 0 and integer n >= 0 by binary powering. */
__device__ __forceinline__ double pow_int(double x, int n) {
    double acc = 1.0, b = x;
    while (n) {
        if (n & 1) acc *= b;
        n >>= 1;
        if (n) b *= b;
    }
    return acc;
}
/* x^e for x >= 0.  INT_EXP (host-checked at rt_set_scene: every specular exponent is an
 * integer in [0, 1024], as in the reference scene and all configs: 30, 50) compiles only
 * the binary powering; otherwise the general pow() is kept — it is large, and its
 * register footprint counts for the whole kernel even where it never runs. */
template <bool INT_EXP>
__device__ __forceinline__ double pow_e(double x, double e) {
    if (INT_EXP) return pow_int(x, (int)e);
    if (e >= 0.0 && e <= 1024.0 && e == __builtin_rint(e)) return pow_int(x, (int)e);
    return pow(x, e);
}

typedef float f2 __attribute__((ext_vector_type(2)));

/* fp32 vector math (throughput path; FMAs explicit) */
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 F3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator-(f3 a) { return F3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float fdot(f3 a, f3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ f3 fnormalize(f3 a) { return a * frsq(fdot(a, a)); }
__device__ __forceinline__ f3 fmad3(f3 a, float s, f3 b) {  // a*s + b
    return F3(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z));
}
__device__ __forceinline__ float fmax3abs(float a, float b, float c) {
    return fmaxf(fmaxf(fabsf(a), fabsf(b)), fabsf(c));
}
/* x^e for x >= 0 via v_log_f32 / v_exp_f32 (pow(0,e>0) = 0, pow(x,0) = 1). */
__device__ __forceinline__ float fpow(float x, float e) {
    if (e == 0.0f) return 1.0f;
    return __builtin_amdgcn_exp2f(e * __builtin_amdgcn_logf(x));
}

/* main.cpp:14-19 */
__device__ __forceinline__ d3 ground_color() { return D3(0.025, 0.05, 0.075); }
__device__ __forceinline__ d3 sky_low() { return D3(0.36, 0.45, 0.57); }
__device__ __forceinline__ d3 sky_high() { return D3(0.14, 0.21, 0.49); }
__device__ __forceinline__ d3 sun_color() { return D3(1.64, 1.27, 0.99); }
__device__ __forceinline__ d3 sun_direction() { return D3(.7, .4, .7); }

/* Largest bounce count compiled: the register stack is sized per instantiation. */
constexpr int MAXD_SMALL = 4;
constexpr int MAXD_MID = 8;
constexpr int MAXD_REF = 10;  // rt_scene's default recursion depth (main.cpp:89)
constexpr int MAXD_LARGE = 16;

/* Waves deep into their paths are the kernel's critical path (its tail): from the
 * RT_PRIO_FROM-th bounce on, a wave asks the sequencer for a higher issue priority. */
#ifndef RT_PRIO_FROM
#define RT_PRIO_FROM 0   // 0 = off
#endif
__device__ __forceinline__ void bounce_priority(int k) {
    if (RT_PRIO_FROM > 0) {
        if (k == RT_PRIO_FROM) __builtin_amdgcn_s_setprio(1);
        if (k == RT_PRIO_FROM + 1) __builtin_amdgcn_s_setprio(2);
        if (k == RT_PRIO_FROM + 2) __builtin_amdgcn_s_setprio(3);
    }
}

/* ------------------------------------------------------------------------ */
/* closest hit (find_closest_hit, main.cpp:67-84)                            */
/* ------------------------------------------------------------------------ */
/* Winner of the scan.  The reference's strict `0 < d < best` scan in scene order returns
 * the lowest scene index among the minimum distance; spheres are visited in scene order
 * (ties among them keep the earlier one) and a wall that ties the best compares scene
 * indices, so the winner is the same. */
struct HitD {
    double dist;  // the value find_closest_hit compares (sphere: world, wall: parametric)
    double pt;    // sphere: parameter of the intersection point used for the normal
    int slot;     // material slot: sphere s -> s, wall w -> nS + w; -1 = miss
};

struct RayD {
    d3 o, d;
    double a;     // |d|^2
    double ra;    // rcp_refined(a)
    double dlen;  // sqrt(a) == d.length()
};

/* Sphere::intersect (scene.cpp:40-78), exact, in the scaled form (file header).  Only
 * branches that can produce an accepted distance are evaluated; every skip is exact:
 *   dot > 0 (b > 0)    -> proj = (-b - sqrt(det)) / 2a < 0, rejected by d > 0
 *   x < 0 (det < 0)    -> miss (scene.cpp:57)
 *   -dot - sqrt(x) <= 0 -> proj <= 0, rejected
 * and p1 is never the minimum: (-b+sq)/2a >= (-b-sq)/2a by monotonic rounding. */
__device__ __forceinline__ int scene_index(const KParams& p, int slot) {
    return slot < p.nS ? p.sph_j[slot] : p.wall_j[slot - p.nS];
}

/* IN_ORDER: spheres visited in increasing index before any wall, so a tie keeps the
 * earlier hit (strict <, main.cpp:77); otherwise a tie compares scene indices. */
/* oc = origin - center and c = |oc|^2 - r^2 given (eye tables) or computed here. */
template <bool IN_ORDER = true>
__device__ __forceinline__ void sphere_exact_oc(const d3 oc, const double c, int s,
                                                const RayD& r, HitD& h,
                                                const KParams* p = nullptr) {
    const double dt = dot(r.d, oc);  // b / 2
    const double x = dt * dt - r.a * c;  // det / 4
    if (RT_SPHERE_ONEBRANCH) {
        if (dt > 0 || !(x >= 0)) return;  // one branch for both rejections
    } else {
        if (dt > 0) return;
        if (!(x >= 0)) return;
    }
    DIAG(2);
    double proj, pt;
    if (x == 0) {
        pt = div_r(-dt, r.a, r.ra);  // -b / (2a)
        proj = 2.0 * pt;             // (-b - sqrt(0)) / a: scene.cpp:65's /a kept
    } else {
        const double num = -dt - sqrt_e(x);
        if (!(num > 0)) return;
        proj = div_r(num, r.a, r.ra);
        pt = proj;
    }
    const double dist = proj * r.dlen;  // world distance, scene.cpp:77
    bool take = dist > 0 && dist < h.dist;
    if (!IN_ORDER && !take && dist > 0 && dist == h.dist && h.slot >= 0)
        take = scene_index(*p, s) < scene_index(*p, h.slot);
    if (take) {
        h.dist = dist;
        h.pt = pt;
        h.slot = s;
    }
}
template <bool IN_ORDER = true>
__device__ __forceinline__ void sphere_exact(const double* S, int s, const RayD& r, HitD& h,
                                             const KParams* p = nullptr) {
    const d3 oc = r.o - D3(S[0], S[1], S[2]);
    sphere_exact_oc<IN_ORDER>(oc, lensq(oc) - S[3], s, r, h, p);
}

/* Wall::intersect (scene.cpp:4-35), exact.  t = num/denom is formed only when the signs
 * make t > 0 possible (denom == 0 or NaN can never pass the bounds check). */
template <bool EYE = false>
__device__ __forceinline__ void wall_exact(const Wall64& Wl, int w, const KParams& p,
                                           const RayD& r, HitD& h) {
    const d3 n = ld3(Wl.n);
    const d3 P = ld3(Wl.P);
    const double den = dot(n, r.d);
    const double num = EYE ? p.eye_w[w] : dot(P - r.o, n);
    double t;
    if (RT_WALL_NOSIGN) {
        // t <= 0 (opposite signs or num == 0), NaN (0/0) and +-inf (den == 0: rcp_refined
        // gives NaN) all fail t > 0, as in the reference (scene.cpp:12); the zero-quotient
        // sign does not matter since 0 fails t > 0 either way
        t = div_r_nz(num, den, rcp_refined(den));
        if (!(t > 0) || (RT_WALL_TSKIP && t > h.dist)) return;  // t > best loses anyway
    } else {
        if (!((num > 0 && den > 0) || (num < 0 && den < 0))) return;
        DIAG(4);
        t = div_r(num, den, rcp_refined(den));
        if (!(t > 0)) return;
        if (RT_WALL_TSKIP && t > h.dist) return;  // loses to the current best either way
    }
    DIAG(6);
    const d3 q = (r.o + r.d * t) - P;  // ray::at (scene.h:16) minus the corner
    const double px = dot(q, ld3(Wl.X));
    const double py = dot(q, ld3(Wl.Y));
    // RT_WALL_BOUNDS_FLAT: all four bounds in one predicate (no branch between px and py)
    const bool inb = RT_WALL_BOUNDS_FLAT
                         ? ((px >= 0) & (px <= Wl.len) & (py >= 0) & (py <= Wl.wid))
                         : (px >= 0 && px <= Wl.len && py >= 0 && py <= Wl.wid);
    if (inb) {
        bool take = t < h.dist;
        if (!take && t == h.dist && h.slot >= 0)  // tie: the lower scene index wins (rare)
            take = p.wall_j[w] < scene_index(p, h.slot);
        if (take) {
            h.dist = t;
            h.slot = p.nS + w;
        }
    }
}

/* The same test as wall_exact without its early exits, for two walls evaluated in one
 * basic block (independent dependency chains the scheduler can interleave: a wave's
 * scan is latency-bound on its critical path).  For lanes that pass the sign test t is
 * bit-identical to wall_exact's; ok = the reference reports a hit at parametric t. */
template <bool EYE>
__device__ __forceinline__ void wall_eval(const Wall64& Wl, int w, const KParams& p,
                                          const RayD& r, double& t, bool& ok) {
    const d3 n = ld3(Wl.n);
    const d3 P = ld3(Wl.P);
    const double den = dot(n, r.d);
    const double num = EYE ? p.eye_w[w] : dot(P - r.o, n);
    const bool sgn = (num > 0 && den > 0) || (num < 0 && den < 0);
    const double dd = sgn ? den : 1.0;  // masked lanes: any finite divisor
    t = div_r(num, dd, rcp_refined(dd));
    const d3 q = (r.o + r.d * t) - P;
    const double px = dot(q, ld3(Wl.X));
    const double py = dot(q, ld3(Wl.Y));
    ok = sgn && t > 0 && px >= 0 && px <= Wl.len && py >= 0 && py <= Wl.wid;
}
__device__ __forceinline__ void wall_take(const KParams& p, int w, double t, bool ok, HitD& h) {
    if (!ok) return;
    bool take = t < h.dist;
    if (!take && t == h.dist && h.slot >= 0)  // tie: the lower scene index wins (rare)
        take = p.wall_j[w] < scene_index(p, h.slot);
    if (take) {
        h.dist = t;
        h.slot = p.nS + w;
    }
}
template <bool EYE>
__device__ __forceinline__ void wall_pair(const KParams& p, int w0, int w1, const RayD& r,
                                          HitD& h) {
    double t0, t1;
    bool ok0, ok1;
    wall_eval<EYE>(p.w64[w0], w0, p, r, t0, ok0);
    wall_eval<EYE>(p.w64[w1], w1, p, r, t1, ok1);
    wall_take(p, w0, t0, ok0, h);  // scene order
    wall_take(p, w1, t1, ok1, h);
}

/* MIXED: fp32 conservative cull in front of the exact sphere test.  A sphere is skipped
 * only when the fp32 evaluation proves, with a margin covering its rounding error, that
 * the exact test rejects it (det < 0, or b > 0).  Margins:
 *   |b/2 error| <= 18u*dinf*B,  |det/4 error| <= 133u*a*B^2 + ...,  B = |o|inf+|C|inf+r,
 * bounded here by K*dinf*B and 8K*a*B^2 with K = 512u. */
struct RayF {
    f3 o, d;
    float a;
    float kb;     // K * dinf
    float kdet;   // 8K * a
    float oinf;
};
constexpr float CULL_U = 1.0f / 16777216.0f;  // 2^-24
constexpr float CULL_K = 512.0f * CULL_U;

__device__ __forceinline__ bool sphere_cull(const float* S, const RayF& r) {
    const f3 oc = r.o - F3(S[0], S[1], S[2]);
    const float bh = fdot(r.d, oc);
    const float c = fmaf(-S[3], S[3], fdot(oc, oc));
    const float det = fmaf(bh, bh, -r.a * c);
    const float B = r.oinf + fmax3abs(S[0], S[1], S[2]) + S[3];
    return (bh > r.kb * B) || (det < -r.kdet * (B * B));
}

__device__ __forceinline__ bool wall_cull(const Wall32& Wl, const RayF& r) {
    const f3 n = F3(Wl.n[0], Wl.n[1], Wl.n[2]), P = F3(Wl.P[0], Wl.P[1], Wl.P[2]);
    const float den = fdot(n, r.d);
    const float num = fdot(P - r.o, n);
    const float B = r.oinf + fmax3abs(P.x, P.y, P.z);
    const float mnum = CULL_K * B;
    const float mden = r.kb;
    if ((num < -mnum && den > mden) || (num > mnum && den < -mden)) return true;  // t < 0
    if (fabsf(num) <= 64.0f * mnum || fabsf(den) <= 64.0f * mden) return false;   // ill-conditioned
    // t's relative error <= mnum/|num| + mden/|den| (<= 1/32 here); bound the point error.
    const float t = num * frcp(den);
    const float rel = mnum / fabsf(num) + mden / fabsf(den) + 4.0f * CULL_U;
    const f3 q = fmad3(r.d, t, r.o) - P;
    const float len_dt = fsqrt(r.a) * fabsf(t);
    const float err = 2.0f * len_dt * rel + CULL_K * (B + len_dt + Wl.len + Wl.wid);
    const float px = fdot(q, F3(Wl.X[0], Wl.X[1], Wl.X[2]));
    const float py = fdot(q, F3(Wl.Y[0], Wl.Y[1], Wl.Y[2]));
    return px < -err || px > Wl.len + err || py < -err || py > Wl.wid + err;
}

/* ------------------------------------------------------------------------ */
/* wave-cooperative sphere cull                                              */
/* ------------------------------------------------------------------------ */
/* Every lane of a wave scans the same primitive list, so the wave can cull the list
 * once for all its live rays: bound them by a cone (apex = centre of the origins' box,
 * widened by its half-diagonal rho; axis = mean direction; half-angle = the widest
 * direction), test 64 spheres at a time against it — lane l tests sphere c0 + l — and
 * ballot the survivors.  A ray o_i + t d_i (t >= 0) that meets ball(C, r) puts
 * o_c + t d_i inside ball(C, r + rho), so a sphere whose inflated ball misses the cone
 * is missed by every live ray: the exact per-lane test would reject it (det < 0 or no
 * positive root).  Margins (1e-4 relative + absolute) dwarf the fp32 error of the bound.
 * Cost per bounce: ten wave reductions + ceil(nS/64) cull passes; enabled by the host
 * when the scene is large enough to pay for it (KParams::wave_cull). */
/* Wave64 reductions returning a wave-uniform (scalar) value: a butterfly inside each
 * 16-lane row with DPP (xor 1, xor 2, half-mirror, mirror — each step leaves groups
 * uniform, so a mirror acts as the next xor), then the four row results read out with
 * v_readlane.  Every lane must be active (the bounce loops are converged). */
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wsum(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
#ifndef RT_DPP_ASM
#define RT_DPP_ASM 1
#endif
#if RT_DPP_ASM
/* In IEEE mode fminf/fmaxf of a value the compiler cannot prove canonical (a DPP move,
 * a readlane) gets a v_max x,x,x canonicalise first, which also blocks folding the DPP
 * move into the min: five VALU per step.  The operands here are never NaN (origins,
 * cosines), so the steps are written as fused v_min/v_max_f32_dpp, one VALU each; the
 * four row results meet through row_bcast:15 / row_bcast:31 in lane 63.  s_nop 1 before
 * each DPP read covers the VALU-write -> DPP-read hazard the compiler cannot see. */
#define RT_WRED(OP)                                                                        \
    "s_nop 1\n\t" OP " %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"          \
    "s_nop 1\n\t" OP " %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"               \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"             \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"             \
    "s_nop 1"
__device__ __forceinline__ float wmin(float v) {
    asm volatile(RT_WRED("v_min_f32_dpp") : "+v"(v));
    return lane_f(v, 63);
}
__device__ __forceinline__ float wmax(float v) {
    asm volatile(RT_WRED("v_max_f32_dpp") : "+v"(v));
    return lane_f(v, 63);
}
#undef RT_WRED
#else
__device__ __forceinline__ float wmin(float v) {
    v = fminf(v, dpp<0xB1>(v));
    v = fminf(v, dpp<0x4E>(v));
    v = fminf(v, dpp<0x141>(v));
    v = fminf(v, dpp<0x140>(v));
    return fminf(fminf(lane_f(v, 0), lane_f(v, 16)), fminf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ float wmax(float v) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    v = fmaxf(v, dpp<0x141>(v));
    v = fmaxf(v, dpp<0x140>(v));
    return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
#endif
__device__ __forceinline__ float uni(float v) { return v; }  // reductions are already scalar
__device__ __forceinline__ double lane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

struct Cone {
    f3 apex;
    f3 u;
    float rho, cos_t, sin_t, scale;
    bool on;
};

__device__ __forceinline__ Cone wave_cone(f3 o, f3 d, bool alive) {
    Cone c;
    const float inf = __builtin_inff();
    const f3 lo = F3(uni(wmin(alive ? o.x : inf)), uni(wmin(alive ? o.y : inf)),
                     uni(wmin(alive ? o.z : inf)));
    const f3 hi = F3(uni(wmax(alive ? o.x : -inf)), uni(wmax(alive ? o.y : -inf)),
                     uni(wmax(alive ? o.z : -inf)));
    c.apex = (lo + hi) * 0.5f;
    const f3 ext = (hi - lo) * 0.5f;
    c.rho = fsqrt(fdot(ext, ext)) * 1.0001f;
    c.scale = fmax3abs(c.apex.x, c.apex.y, c.apex.z) + c.rho;
    const f3 dn = alive ? fnormalize(d) : F3(0.f, 0.f, 0.f);
    const f3 su = F3(uni(wsum(dn.x)), uni(wsum(dn.y)), uni(wsum(dn.z)));
    c.u = fnormalize(su);
    c.cos_t = uni(wmin(alive ? fdot(c.u, dn) : 1.0f)) - 1e-4f;
    c.sin_t = fsqrt(fmaxf(0.0f, 1.0f - c.cos_t * c.cos_t));
    c.on = c.cos_t > 0.05f;  // a near-hemispherical fan culls nothing: skip the pass
    return c;
}

/* The primary segment's cone (RT_EYE_CONE): every primary ray starts at the camera, so the
 * apex is that shared origin (rho 0 — what wave_cone's box reductions return for equal
 * origins, without them), the axis the sum of the first and last live lanes' directions
 * (any axis is valid: the half-angle is measured against it), and one reduction remains:
 * the widest live direction. */
#ifndef RT_EYE_CONE
#define RT_EYE_CONE 1
#endif
__device__ __forceinline__ Cone wave_cone_eye(f3 o, f3 d, bool alive) {
    Cone c;
    const uint64_t am = __ballot(alive);
    const int l0 = am ? __builtin_ctzll(am) : 0;
    const int l1 = am ? 63 - __builtin_clzll(am) : 0;
    c.apex = F3(lane_f(o.x, l0), lane_f(o.y, l0), lane_f(o.z, l0));
    c.rho = 0.0f;
    c.scale = fmax3abs(c.apex.x, c.apex.y, c.apex.z);
    const f3 dn = alive ? fnormalize(d) : F3(0.f, 0.f, 0.f);
    c.u = fnormalize(F3(lane_f(dn.x, l0) + lane_f(dn.x, l1), lane_f(dn.y, l0) + lane_f(dn.y, l1),
                        lane_f(dn.z, l0) + lane_f(dn.z, l1)));
    c.cos_t = uni(wmin(alive ? fdot(c.u, dn) : 1.0f)) - 1e-4f;
    c.sin_t = fsqrt(fmaxf(0.0f, 1.0f - c.cos_t * c.cos_t));
    c.on = c.cos_t > 0.05f;
    return c;
}

/* Cull pass over spheres [c0, c0+64): lane l tests sphere c0 + l.  Returns the ballot of
 * survivors; *lb receives (in lane l) a lower bound on sphere c0+l's hit distance for any
 * live ray of the wave: |hit - o_i| >= |C - o_i| - r >= |C - apex| - rho - r. */
struct SphRec {
    float f[4];   // fp32 {cx, cy, cz, r} of sphere c0 + lane
    double d[4];  // fp64 {cx, cy, cz, r^2} (WANT64 && !RT_CULL_REC64_SCALAR only)
};
/* RT_CULL_REC64_SCALAR: the cull pass loads only the fp32 records (16 B per lane instead of
 * 48: ~1.5% of the spheres survive the cone), and each survivor's fp64 record comes in
 * afterwards by one wave-uniform scalar load (the index is a ballot bit) instead of eight
 * v_readlane from the testing lane's registers. */
#ifndef RT_CULL_REC64_SCALAR
#define RT_CULL_REC64_SCALAR 1
#endif
template <bool WANT64>
__device__ __forceinline__ uint64_t cull_chunk(const KParams& p, const Cone& cn, int c0,
                                               float* lb, SphRec& rec) {
    const int s = c0 + (int)(threadIdx.x & 63);
    bool keep = false;
    float bound = 0.0f;
    if (s < p.nS) {
        keep = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) rec.f[k] = p.s32[s >> 2].c[k][s & 3];
        const float* S = rec.f;
        if (WANT64 && !RT_CULL_REC64_SCALAR) {
#pragma unroll
            for (int k = 0; k < 4; ++k) rec.d[k] = p.s64[s >> 2].v[s & 3][k];
        }
        const f3 v = F3(S[0], S[1], S[2]) - cn.apex;
        const float L2 = fdot(v, v);
        const float R = S[3] + cn.rho +
                        1e-4f * (1.0f + cn.scale + fmax3abs(S[0], S[1], S[2]) + S[3]);
        if (L2 > R * R) {  // apex outside the inflated ball
            const float il = frsq(L2);
            bound = fmaxf(0.0f, (L2 * il - R) * 0.9999f);
            if (cn.on) {
                const float sa = fminf(R * il, 1.0f);
                const float ca = fsqrt(fmaxf(0.0f, 1.0f - sa * sa));
                const float cphi = fdot(cn.u, v) * il;
                keep = cphi >= cn.cos_t * ca - cn.sin_t * sa - 1e-4f;
            }
        }
    }
    *lb = bound;
    const uint64_t m = __ballot(keep);
    // diagnostics (KParams::stats: [0] cull passes, [1] spheres kept, [2] spheres considered)
    if (p.stats != nullptr && (threadIdx.x & 63) == 0) {
        const int nin = p.nS - c0 < 64 ? p.nS - c0 : 64;
        atomicAdd(p.stats + 0, 1ull);
        atomicAdd(p.stats + 1, (unsigned long long)__popcll(m));
        atomicAdd(p.stats + 2, (unsigned long long)nin);
    }
    return m;
}

__device__ __forceinline__ RayF make_rayf(const RayD& r) {
    RayF rf;
    rf.o = F3((float)r.o.x, (float)r.o.y, (float)r.o.z);
    rf.d = F3((float)r.d.x, (float)r.d.y, (float)r.d.z);
    rf.a = fdot(rf.d, rf.d);
    rf.kb = CULL_K * fmax3abs(rf.d.x, rf.d.y, rf.d.z);
    rf.kdet = 8.0f * CULL_K * rf.a;
    rf.oinf = fmax3abs(rf.o.x, rf.o.y, rf.o.z);
    return rf;
}
/* DBL_MAX as an opaque scalar (SGPR pair): as a literal the register allocator of the deep
 * cull kernels kept it in a VGPR pair and spilled that to scratch, reloading it inside the
 * sphere loop; from SGPRs each use is a plain copy.  (The linear-scan kernels, which did not
 * spill, keep the literal: A/B c1 +2..12% otherwise.) */
#ifndef RT_DMAX_SGPR
#define RT_DMAX_SGPR 1
#endif
__device__ __forceinline__ double dbl_max_s() {
    if (!RT_DMAX_SGPR) return DBL_MAX;
    uint32_t lo, hi;
    asm("s_mov_b32 %0, -1" : "=s"(lo));
    asm("s_mov_b32 %0, 0x7fefffff" : "=s"(hi));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ HitD no_hit() {
    HitD h;
    h.dist = DBL_MAX;
    h.pt = 0;
    h.slot = -1;
    return h;
}
/* sphere s (wave-uniform index), exact, behind the MIXED per-lane fp32 cull */
template <bool MIXED>
__device__ __forceinline__ void sphere_by_index(const KParams& p, int s, const RayD& r,
                                                const RayF& rf, HitD& h) {
    const float Sf[4] = {p.s32[s >> 2].c[0][s & 3], p.s32[s >> 2].c[1][s & 3],
                         p.s32[s >> 2].c[2][s & 3], p.s32[s >> 2].c[3][s & 3]};
    if (MIXED && sphere_cull(Sf, rf)) return;
    sphere_exact(p.s64[s >> 2].v[s & 3], s, r, h);
}
#ifndef RT_WALL_SLOAD  // 1: the cull kernels' wall records through scalar loads (asm)
#define RT_WALL_SLOAD 1
#endif
/* Wall w's fp64 record as two s_load_dwordx16 (the cull kernels: see clusters_mask's box
 * loads for why the compiler's own loads there go through the vector memory path). */
__device__ __forceinline__ Wall64 wall64_sload(const Wall64* q) {
    typedef int v16i __attribute__((ext_vector_type(16)));
    struct Two {
        v16i a, b;
    } t;
    asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=s"(t.a), "=s"(t.b)
                 : "s"(q)
                 : "memory");
    return __builtin_bit_cast(Wall64, t);
}
/* RT_WALL_PRE32 (A/B): the exact-path scans' walls decided in fp32 first.
 * Each wall's t and bounds are evaluated in fp32 with wall_cull's error model (relative
 * error of t <= rel, of the hit point <= err): a wall the exact test must reject (t <= 0 by
 * the signs, or a point outside the rectangle by more than err) is dropped; a wall it must
 * accept (signs and bounds clear of the margins) bounds the final best from above by
 * t (1 + 2 rel); and only the walls whose lower bound t (1 - 2 rel) does not exceed that
 * bound (or the spheres' best) run the exact fp64 test, in scene order.  Every wall that can
 * win or tie the final best is among them, so the winner — and h — are bitwise the full
 * scan's.  fp64 FMAs issue at the fp32 rate on gfx950 (§3), so this pays only if the exact
 * bodies it skips outweigh the fp32 pass over every wall. */
#ifndef RT_WALL_PRE32
#define RT_WALL_PRE32 0
#endif
constexpr int PRE32_MAXW = 6;
template <bool EYE>
__device__ __forceinline__ void walls_pre32(const KParams& p, const RayD& r, HitD& h) {
    const RayF rf = make_rayf(r);
    const float dl = fsqrt(rf.a);
    float tlo[PRE32_MAXW];
    double U = h.dist;
#pragma unroll
    for (int w = 0; w < PRE32_MAXW; ++w) {
        tlo[w] = __builtin_nanf("");  // never tested
        if (w >= p.nW) continue;      // wave-uniform
        const Wall32& Wl = p.w32[w];
        const f3 n = F3(Wl.n[0], Wl.n[1], Wl.n[2]), P = F3(Wl.P[0], Wl.P[1], Wl.P[2]);
        const float den = fdot(n, rf.d);
        const float num = fdot(P - rf.o, n);
        const float B = rf.oinf + fmax3abs(P.x, P.y, P.z);
        const float mnum = CULL_K * B, mden = rf.kb;
        const bool behind = (num < -mnum && den > mden) || (num > mnum && den < -mden);
        const bool illc = fabsf(num) <= 64.0f * mnum || fabsf(den) <= 64.0f * mden;
        const float t = num * frcp(den);
        // wall_cull's relative error of t, the quotients through reciprocals (+1% for their
        // own rounding)
        const float rel = 1.01f * (mnum * frcp(fabsf(num)) + mden * frcp(fabsf(den))) + 4.0f * CULL_U;
        const f3 q = fmad3(rf.d, t, rf.o) - P;
        const float len_dt = dl * fabsf(t);
        const float err = 2.0f * len_dt * rel + CULL_K * (B + len_dt + Wl.len + Wl.wid);
        const float px = fdot(q, F3(Wl.X[0], Wl.X[1], Wl.X[2]));
        const float py = fdot(q, F3(Wl.Y[0], Wl.Y[1], Wl.Y[2]));
        const bool outb = px < -err || px > Wl.len + err || py < -err || py > Wl.wid + err;
        const bool inb = px >= err && px <= Wl.len - err && py >= err && py <= Wl.wid - err;
        const float m2 = 2.0f * rel * fabsf(t);
        const bool never = behind || (!illc && outb);
        // well conditioned and not behind: fp32 num and den carry the exact signs, so t > 0
        // here is the exact t > 0
        const bool sure = !illc && !behind && inb && t > 0.0f;
        tlo[w] = never ? __builtin_nanf("") : (illc ? -__builtin_inff() : t - m2);
        if (sure) U = fmin(U, (double)(t + m2));
    }
#pragma unroll
    for (int w = 0; w < PRE32_MAXW; ++w) {
        if (w >= p.nW) break;
        if ((double)tlo[w] <= U) wall_exact<EYE>(p.w64[w], w, p, r, h);
    }
}

template <bool MIXED, bool EYE = false, bool SL = false>
__device__ __forceinline__ void walls_d(const KParams& p, const RayD& r, const RayF& rf, HitD& h) {
    if constexpr (RT_WALL_PRE32 && !MIXED && !SL) {
        if (p.nW <= PRE32_MAXW) {  // wave-uniform
            walls_pre32<EYE>(p, r, h);
            return;
        }
    }
    for (int w = 0; w < p.nW; ++w) {
        if (!MIXED && !SL && RT_WALL_PAIRS && w + 1 < p.nW) {
            wall_pair<EYE>(p, w, w + 1, r, h);
            ++w;
            continue;
        }
        if (MIXED && wall_cull(p.w32[w], rf)) continue;
        if (SL)
            wall_exact<EYE>(wall64_sload(p.w64 + w), w, p, r, h);
        else
            wall_exact<EYE>(p.w64[w], w, p, r, h);
    }
}

/* Walls against the wave's cone (RT_CULL_WALL_CONE): lane w tests wall w's circumscribed
 * ball (centre P + X len/2 + Y wid/2, radius half the diagonal: every point the exact test
 * can accept — the rectangle, its bounds checked in fp64 to ~1e-15 — lies in it) exactly as
 * cull_chunk tests a sphere, with the same margins; a wall whose inflated ball misses the
 * cone is missed by every live ray.  nW <= 64, all lanes active. */
/* May a ray of the cone meet ball(C, rad)?  cull_chunk's test and margins. */
__device__ __forceinline__ bool cone_ball(const Cone& cn, const f3 C, float rad) {
    const f3 v = C - cn.apex;
    const float L2 = fdot(v, v);
    const float R = rad + cn.rho + 1e-4f * (1.0f + cn.scale + fmax3abs(C.x, C.y, C.z) + rad);
    if (!(L2 > R * R)) return true;  // apex inside the inflated ball (or NaN): keep
    const float il = frsq(L2);
    const float sa = fminf(R * il, 1.0f);
    const float ca = fsqrt(fmaxf(0.0f, 1.0f - sa * sa));
    const float cphi = fdot(cn.u, v) * il;
    return cphi >= cn.cos_t * ca - cn.sin_t * sa - 1e-4f;
}
/* Wall w's circumscribed ball (fp32): the rectangle's centre and half its diagonal. */
__device__ __forceinline__ bool cone_wall(const Cone& cn, const Wall32& Wl) {
    const float hl = 0.5f * Wl.len, hw = 0.5f * Wl.wid;
    const f3 C = F3(fmaf(Wl.Y[0], hw, fmaf(Wl.X[0], hl, Wl.P[0])),
                    fmaf(Wl.Y[1], hw, fmaf(Wl.X[1], hl, Wl.P[1])),
                    fmaf(Wl.Y[2], hw, fmaf(Wl.X[2], hl, Wl.P[2])));
    return cone_ball(cn, C, fsqrt(fmaf(hl, hl, hw * hw)) * 1.0001f);
}
__device__ __forceinline__ uint64_t ballot_u(bool b) {
    const uint64_t m = __ballot(b);
    return ((uint64_t)__builtin_amdgcn_readfirstlane((unsigned)(m >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((unsigned)m);
}
__device__ __forceinline__ uint64_t wall_cone_mask(const KParams& p, const Cone& cn) {
    const int w = (int)(threadIdx.x & 63);
    return ballot_u(w < p.nW && cone_wall(cn, p.w32[w]));
}

/* The cull kernels' primary walls behind the wall pixel boxes (RT_CULL_WALL_BINS): only
 * the walls whose box meets the wave's tile (wave-uniform mask, bit w = wall w), in index
 * order as walls_d. */
template <bool MIXED>
__device__ __forceinline__ void walls_d_kept(const KParams& p, const RayD& r, const RayF& rf,
                                             HitD& h, uint64_t wm) {
    while (wm) {
        const int w = __builtin_ctzll(wm);
        wm &= wm - 1;
        if (MIXED && wall_cull(p.w32[w], rf)) continue;
        if (RT_WALL_SLOAD)
            wall_exact<false>(wall64_sload(p.w64 + w), w, p, r, h);
        else
            wall_exact<false>(p.w64[w], w, p, r, h);
    }
}

/* RT_SPH_PRECULL: the linear scans' unbinned segments (a bounce whose lanes follow no
 * common wall chain: every sphere is tested) run MIXED's conservative fp32 cull
 * (sphere_cull, the same predicate bit for bit) two spheres per packed instruction first,
 * and the exact test only where a lane's cull cannot prove the miss — at c2 ~9 of 10
 * exact sphere tests of such a scan reject every lane. */
#ifndef RT_SPH_PRECULL
#define RT_SPH_PRECULL 1
#endif
/* sphere_cull for spheres k0, k0 + 1 of group G in packed fp32 (v_pk_fma / v_pk_mul: each
 * element rounds as the scalar fmaf / * does, so the predicate is sphere_cull's). */
__device__ __forceinline__ void sphere_cull_pair(const SphG32& G, int k0, const RayF& r, bool& cull0,
                                                 bool& cull1) {
    const f2 cx = {G.c[0][k0], G.c[0][k0 + 1]}, cy = {G.c[1][k0], G.c[1][k0 + 1]};
    const f2 cz = {G.c[2][k0], G.c[2][k0 + 1]}, rr = {G.c[3][k0], G.c[3][k0 + 1]};
    const f2 ocx = f2(r.o.x) - cx, ocy = f2(r.o.y) - cy, ocz = f2(r.o.z) - cz;
    const f2 bh = __builtin_elementwise_fma(
        f2(r.d.x), ocx, __builtin_elementwise_fma(f2(r.d.y), ocy, f2(r.d.z) * ocz));
    const f2 cq = __builtin_elementwise_fma(
        -rr, rr, __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz)));
    const f2 det = __builtin_elementwise_fma(bh, bh, -f2(r.a) * cq);
    const float B0 = r.oinf + fmax3abs(cx.x, cy.x, cz.x) + rr.x;
    const float B1 = r.oinf + fmax3abs(cx.y, cy.y, cz.y) + rr.y;
    cull0 = (bh.x > r.kb * B0) || (det.x < -r.kdet * (B0 * B0));
    cull1 = (bh.y > r.kb * B1) || (det.y < -r.kdet * (B1 * B1));
}

/* Linear scan (no wave cull): groups of 4 spheres per scalar load.  EYE: the primary
 * segment, origin terms from the eye tables (rt_device.h). */
template <bool MIXED, bool EYE>
__device__ __forceinline__ HitD closest_hit_d(const KParams& p, const RayD& r) {
    DIAG(0);
    HitD h = no_hit();
    RayF rf;
    constexpr bool PRE_K = RT_SPH_PRECULL && !MIXED && !EYE;
    // (wave-uniform: scenes of a few spheres — c1's one — do not pay for the ray's fp32 copy,
    // A/B c1 +7%)
    const bool PRE = PRE_K && p.nS >= 4;
    if (MIXED || PRE) rf = make_rayf(r);
    const int ng = (p.nS + 3) >> 2;
    for (int g = 0; g < ng; ++g) {
        if (PRE) {
            const SphG32 G = p.s32[g];  // one s_load_dwordx16
            bool cu[4];
            sphere_cull_pair(G, 0, rf, cu[0], cu[1]);
            sphere_cull_pair(G, 2, rf, cu[2], cu[3]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * g + k;
                if (s < p.nS && !cu[k]) sphere_exact(p.s64[g].v[k], s, r, h);
            }
        } else if (MIXED) {
            const SphG32 G = p.s32[g];  // one s_load_dwordx16
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * g + k;
                const float Sf[4] = {G.c[0][k], G.c[1][k], G.c[2][k], G.c[3][k]};
                if (s < p.nS && !sphere_cull(Sf, rf)) {
                    if (EYE) {
                        const double* E = p.eye_s[s];
                        sphere_exact_oc(D3(E[0], E[1], E[2]), E[3], s, r, h);
                    } else {
                        sphere_exact(p.s64[g].v[k], s, r, h);
                    }
                }
            }
        } else if (EYE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * g + k;
                const double* E = p.eye_s[s];
                if (s < p.nS) sphere_exact_oc(D3(E[0], E[1], E[2]), E[3], s, r, h);
            }
        } else {
            const SphG64 G = p.s64[g];  // two s_load_dwordx16
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = 4 * g + k;
                if (s < p.nS) sphere_exact(G.v[k], s, r, h);
            }
        }
    }
    walls_d<MIXED, EYE>(p, r, rf, h);
    return h;
}

/* Primary segment behind the tile bins (rt_device.h PrimBox): only the primitives whose
 * pixel box meets the wave's tile are tested, spheres in increasing index (the strict-<
 * tie rule holds: a skipped sphere cannot hit), then walls.  keep is wave-uniform. */
template <bool MIXED, bool EYE>
__device__ __forceinline__ HitD closest_hit_bin(const KParams& p, const RayD& r, uint64_t keep) {
    DIAG(0);
    HitD h = no_hit();
    RayF rf;
    if (MIXED) rf = make_rayf(r);
    uint64_t sm = p.nS >= 64 ? keep : keep & ((1ull << p.nS) - 1);
    while (sm) {
        const int s = __builtin_ctzll(sm);
        sm &= sm - 1;
        if (EYE) {
            const double* E = p.eye_s[s];
            sphere_exact_oc(D3(E[0], E[1], E[2]), E[3], s, r, h);
        } else {
            sphere_by_index<MIXED>(p, s, r, rf, h);
        }
    }
    uint64_t wm = p.nS >= 64 ? 0 : keep >> p.nS;
    if (EYE && RT_WALL_ORDER && p.wall_order_n == p.nW) {
        // primary rays: the walls nearest to the camera first (host order, KParams::
        // wall_order), so a wall behind the best hit skips its bounds test (t-skip); any
        // order finds the reference's winner (wall ties compare scene indices)
        uint64_t ord = p.wall_order;
        for (int k = 0; k < p.nW && wm; ++k, ord >>= 4) {
            const int w = (int)(ord & 15);
            if (!((wm >> w) & 1)) continue;
            wm &= ~(1ull << w);
            wall_exact<EYE>(p.w64[w], w, p, r, h);
        }
        return h;
    }
    while (wm) {
        const int w = __builtin_ctzll(wm);
        wm &= wm - 1;
        if (!MIXED && RT_WALL_PAIRS && wm) {
            const int w1 = __builtin_ctzll(wm);
            wm &= wm - 1;
            wall_pair<EYE>(p, w, w1, r, h);
            continue;
        }
        if (MIXED && wall_cull(p.w32[w], rf)) continue;
        wall_exact<EYE>(p.w64[w], w, p, r, h);
    }
    return h;
}

/* out_color, main.cpp:28-37: only normalize(v).z is used; z^0.25 as sqrt(sqrt(z)). */
__device__ __forceinline__ d3 sky_d(const RayD& r, double nvz) {
    if (r.d.z < 0.0) return ground_color();
    return lerp(sky_low(), sky_high(), sqrt_e(sqrt_e(nvz)));
}

/* Shading of one hit (main.cpp:99-104 + diffuse_shading + specular), returning
 * s = diffuse*kd + spec*ks + ka (local = color * s) and the (optional) sun scalar.
 * Shared normalisations are computed once: the same operations on the same operands
 * as the reference's repeated calls. */
struct ShadeD {
    double s;
    double ksun;
};
template <bool INT_EXP>
__device__ __forceinline__ ShadeD shade_d(const DevMat& m, const d3 pos, const d3 nn,
                                          const d3 view, bool sun) {
    const d3 ldir = normalize_e(D3(0.0 - pos.x, 0.0 - pos.y, 0.0 - pos.z));  // LIGHT_POS - pos
    const double lamb = dot(ldir, nn);
    const double diffuse = lamb > 0 ? lamb : 0;
    double res = dot(normalize_e(view + ldir), nn);
    res = res > 0 ? res : 0;
    const double spec = pow_e<INT_EXP>(res, m.ex);
    ShadeD sh;
    sh.s = diffuse * m.kd + spec * m.ks + m.ka;
    sh.ksun = 0;
    if (sun) {  // build-defined (rt_oracle.c sun_term)
        const d3 sd = normalize_e(sun_direction());
        double a = dot(sd, nn);
        a = a > 0 ? a : 0;
        double hs = dot(normalize_e(view + sd), nn);
        hs = hs > 0 ? hs : 0;
        sh.ksun = a * m.kd + pow_e<INT_EXP>(hs, m.ex) * m.ks;
    }
    return sh;
}

/* local = color * s (+ (SUN_COLOR * color) * ksun): identical operations at push and at
 * unwind. */
__device__ __forceinline__ d3 local_color_d(const DevMat& m, double s, double ksun, bool sun) {
    const d3 col = ld3(m.color);
    d3 L = col * s;
    if (sun) L = L + (sun_color() * col) * ksun;
    return L;
}

__device__ __forceinline__ RayD make_ray(d3 o, d3 d) {
    RayD r;
    r.o = o;
    r.d = d;
    r.a = lensq(d);
    r.ra = rcp_refined(r.a);
    r.dlen = sqrt_e(r.a);
    return r;
}
/* Origin and direction only: |d|^2, its reciprocal and |d| are formed by ray_terms when a
 * sphere test or a reflection needs them (wave-uniform decisions; walls and fp32 terminal
 * shading use none of them). */
__device__ __forceinline__ RayD make_ray_lazy(d3 o, d3 d) {
    RayD r;
    r.o = o;
    r.d = d;
    r.a = r.ra = r.dlen = 0.0;
    return r;
}
__device__ __forceinline__ void ray_terms(RayD& r) {
    r.a = lensq(r.d);
    r.ra = rcp_refined(r.a);
    r.dlen = sqrt_e(r.a);
}

/* fp32 shading of one hit for PATH64: the same formulas as shade_d on the exact fp64
 * geometry rounded to fp32 (colour only — nothing here feeds the next ray). */
__device__ __forceinline__ float2 shade_f(const DevMat32& m, const f3 pos, const f3 nn,
                                          const f3 nv, bool sun) {
    const float kd = m.kd, ks = m.ks, ka = m.ka, ex = m.ex;
    const f3 ldir = fnormalize(-pos);
    const float lamb = fmaxf(fdot(ldir, nn), 0.0f);
    const float res = fmaxf(fdot(fnormalize(ldir - nv), nn), 0.0f);
    float2 r;
    r.x = fmaf(lamb, kd, fmaf(fpow(res, ex), ks, ka));
    r.y = 0.0f;
    if (sun) {
        const f3 sd = fnormalize(F3(.7f, .4f, .7f));
        const float sa = fmaxf(fdot(sd, nn), 0.0f);
        const float hs = fmaxf(fdot(fnormalize(sd - nv), nn), 0.0f);
        r.y = fmaf(sa, kd, fpow(hs, ex) * ks);
    }
    return r;
}
__device__ __forceinline__ f3 local_color_f(const DevMat32& m, float s, float ksun, bool sun) {
    const f3 col = F3(m.color[0], m.color[1], m.color[2]);
    f3 L = col * s;
    if (sun) L = fmad3(F3(1.64f * col.x, 1.27f * col.y, 0.99f * col.z), ksun, L);
    return L;
}
__device__ __forceinline__ f3 tof(d3 v) { return F3((float)v.x, (float)v.y, (float)v.z); }

/* PATH64's terminal miss (out_color, main.cpp:28-37) in fp32: ground below the horizon by
 * the exact direction's sign, else the sky lerp at normalize(d).z^0.25. */
__device__ __forceinline__ f3 sky32(const d3& d) {
    const f3 nv32 = fnormalize(tof(d));
    if (d.z < 0.0) return F3(0.025f, 0.05f, 0.075f);
    const float tz = fsqrt(fsqrt(nv32.z));
    return F3(fmaf(tz, 0.14f - 0.36f, 0.36f), fmaf(tz, 0.21f - 0.45f, 0.45f),
              fmaf(tz, 0.49f - 0.57f, 0.57f));
}

/* Dispatch order of tile rows (workgroup row blockIdx.y -> tile row).  Per-tile cost is
 * very uneven (sky/ground tiles end after one segment, tiles over reflective walls bounce
 * to full depth), and a heavy wave dispatched late ends the kernel long after the last
 * light one: the dispatcher goes row by row, so rows are visited centre-out from the
 * host's estimate of the heaviest row (KParams::row_center, rt_capi.cpp) — heavy work
 * first, the cheap rows fill in around it.  Identity when row_center < 0. */
// Wave-start loads.  1: no early return before the trace (a workgroup past the end of a
// row part runs with every lane invalid) and the primary box load is unconditional, so it
// no longer waits on nbox (A/B: c2 PATH64 -0.1..1.3%, F32 -1.3..2.6%, c1 -1..4.5%, c3
// +-0.6%).  2: also every wave-start kernel-argument value in ONE batch with one wait,
// pinned by an empty asm (A/B: c2 PATH64 +15%, F64 +7% — slower, off).
#ifndef RT_EARLY_LOADS
#define RT_EARLY_LOADS 1
#endif
#ifndef RT_TILE_PAIRS      // 1: each wave traces two tiles one after the other — dispatch
#define RT_TILE_PAIRS 0    // unit j and unit n-1-j of the row order (heavy with light), so
#endif                     // the per-wave start cost is paid once per 128 pixels (A/B knob)
#ifndef RT_PERM_FIRST      // A/B knob: 1 = take the explicit order when it covers the grid
#define RT_PERM_FIRST 0    // (wave-uniform branch) and skip the centre-out arithmetic
#endif
__device__ __forceinline__ uint32_t row_perm_word(const KParams& p, int j) {
    return reinterpret_cast<const uint32_t*>(p.row_perm)[min(j >> 1, ROW_PERM_MAX / 2 - 1)];
}
/* c = row_center, rpn = row_perm_n, w = row_perm_word(j): the loaded values */
__device__ __forceinline__ int tile_row_of(int c, int rpn, uint32_t w, int j, int n) {
    const int L = min(c, n - 1 - c);  // rows c-L .. c+L alternate
    const int d = (j + 1) >> 1;
    const int alt = (j & 1) ? c + d : c - d;
    const int e = j - 2 * L;  // one side is exhausted: continue on the other
    const int rest = (c - L == 0) ? c + L + e : c - L - e;
    int t = j <= 2 * L ? alt : rest;
    t = (c < 0 || c >= n) ? j : t;
    const int pj = (int16_t)((j & 1) ? (w >> 16) : (w & 0xffff));
    return rpn == n ? pj : t;
}
__device__ __forceinline__ int tile_row(const KParams& p, int j, int n) {
    if (RT_PERM_FIRST && p.row_perm_n == n) {
        const uint32_t w = row_perm_word(p, j);
        return (int16_t)((j & 1) ? (w >> 16) : (w & 0xffff));
    }
    // branch-free (scalar selects), so that its kernel-argument loads — including the dword
    // holding entry j of an explicit order (a 16-bit load would be a vector load) — issue in
    // the wave's first batch instead of one dependent round trip after another
    return tile_row_of(p.row_center, p.row_perm_n, row_perm_word(p, j), j, n);
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
/* The primitives whose pixel box meets this wave's 8x8 tile (rt_device.h PrimBox): lane l
 * tests box l, one ballot.  box_load issues the load (early, so its latency hides behind
 * ray generation), box_keep does the branch-free compare and the ballot.  All lanes
 * active. */
__device__ __forceinline__ uint64_t box_load(const KParams& p, const PrimBox* boxes) {
    const int l = threadIdx.x & 63;
    const uint64_t v = *reinterpret_cast<const uint64_t*>(boxes + (l < p.nbox ? l : 0));
    return l < p.nbox ? v : 0x80007fff80007fffull;  // x0 = i0 = 32767 > x1 = i1: never meets
}
/* Pixel origin of the wave's 8x8 tile from a lane's own pixel (every wave covers an 8x8
 * square, lane = 8 * row + column): wave-uniform, independent of how tiles map to
 * workgroups. */
struct TileO {
    int x0, y0;
};
__device__ __forceinline__ TileO tile_origin(int x, int i) {
    const int lane = threadIdx.x & 63;
    return {__builtin_amdgcn_readfirstlane(x - (lane & 7)),
            __builtin_amdgcn_readfirstlane(i - (lane >> 3))};
}
/* The primary boxes: p.box always holds BIN_MAX_PRIMS (= 64) entries, so lane l's load is
 * in bounds whatever nbox is; the select after it needs nbox, the load does not. */
__device__ __forceinline__ uint64_t box_load_primary(const KParams& p) {
    static_assert(BIN_MAX_PRIMS == 64, "one box per lane");
    const int l = threadIdx.x & 63;
    const uint64_t v = *reinterpret_cast<const uint64_t*>(p.box + l);
    return l < p.nbox ? v : 0x80007fff80007fffull;
}
/* The cull kernels' wall boxes (RT_CULL_WALL_BINS): p.box[0 .. nwbox-1] = walls 0.. */
__device__ __forceinline__ uint64_t box_load_walls(const KParams& p) {
    const int l = threadIdx.x & 63;
    const uint64_t v = *reinterpret_cast<const uint64_t*>(p.box + l);
    return l < p.nwbox ? v : 0x80007fff80007fffull;
}
__device__ __forceinline__ uint64_t box_keep(uint64_t raw, TileO t) {
    const int x0 = (int16_t)(raw & 0xffff), x1 = (int16_t)((raw >> 16) & 0xffff);
    const int i0 = (int16_t)((raw >> 32) & 0xffff), i1 = (int16_t)(raw >> 48);
    const bool hit = (x0 <= t.x0 + 7) & (x1 >= t.x0) & (i0 <= t.y0 + 7) & (i1 >= t.y0);
    return uniform64(__ballot(hit));
}
__device__ __forceinline__ uint64_t tile_keep(const KParams& p, const PrimBox* boxes, TileO t) {
    return box_keep(box_load(p, boxes), t);
}

/* Bounce k <= mir_depth after chains of wall hits (rt_device.h "mirror bins"): a lane whose
 * previous k segments hit walls w1..wk has a ray of the camera mirrored along that chain,
 * so it can only hit primitives whose box for that chain meets the tile.  The wave's keep
 * mask is the union over the distinct chains its live lanes followed (at most
 * RT_MIR_CHAINS of them; more, or a sphere anywhere in a chain, returns ~0 = scan all).
 * st_m: the lane's material-slot stack (valid where alive).  All lanes active; k
 * wave-uniform. */
#ifndef RT_MIR_CHAINS
#define RT_MIR_CHAINS 1  // A/B: 4 chains = the same speed at c2, more SALU
#endif
template <int MAXD>
__device__ __forceinline__ uint64_t mirror_keep(const KParams& p, bool alive, const int* st_m,
                                                int k, TileO t) {
    uint64_t todo = uniform64(__ballot(alive));
    if (todo == 0 || k > p.mir_depth) return ~0ull;
    uint64_t keep = 0;
    for (int c = 0; c < RT_MIR_CHAINS; ++c) {
        const int l0 = __builtin_ctzll(todo);
        bool same = alive;
        int q = 0, off = 0, lvl = 1;
#pragma unroll
        for (int j = 0; j < MIR_MAX_DEPTH && j < MAXD; ++j) {
            if (j < k) {
                const int sj = __builtin_amdgcn_readlane(st_m[j], l0);
                if (sj < p.nS) return ~0ull;  // a sphere bounce: no linear mirror
                same = same && st_m[j] == sj;
                q = q * p.nW + (sj - p.nS);
                if (j > 0) off += lvl;
                lvl *= p.nW;
            }
        }
        keep |= tile_keep(p, p.mbox + (off + q) * p.nbox, t);
        todo &= ~uniform64(__ballot(same));
        if (todo == 0) return keep;
    }
    return ~0ull;
}

/* find_closest_hit for one segment of every live lane: the wave-culled scan (CULL) or the
 * linear scan.  Converged: every lane of the wave calls it (alive masks the tests). */
/* Sphere clusters (rt_device.h Clu32/CluSph): a wide-cone wave's lanes each test their own
 * ray against the cluster boxes, then walk their own clusters — against the first split's
 * axis along the ray, so roughly near to far — skipping a cluster whose box entry already
 * lies beyond the lane's best hit, and run the exact test (order-independent tie rule) on
 * its spheres.  Conservative: the boxes are the balls' bounds widened by 1e-3 x the scene
 * extent, against fp32 slab errors ~1e-5 x extent for origins within 100 x the extent
 * (others test every cluster, unpruned); a skipped cluster's spheres lie at a world
 * distance >= t_entry |d| > best, so they lose even a tie.  slab_t: entry parameter of the
 * ray into the box (0 inside), +inf on a miss; NaN slab terms (origin on a box plane with
 * d = 0 there: the ray misses the ball by the margin) reject. */
/* RT_CLU_OCT: the lane walks its clusters near to far in the host's order for its
 * direction octant (Clu32::rank, KParams::cord); otherwise in index order, reversed when
 * the ray runs against the first split's axis. */
__device__ __forceinline__ int clu_octant(const f3 d) {
    return (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0);
}
template <bool OCT>
__device__ __forceinline__ int clu_bit(const Clu32& B, int oct, int c) {
    if (!OCT) return c;
    const uint32_t lo = *reinterpret_cast<const uint32_t*>(B.rank);
    const uint32_t hi = *reinterpret_cast<const uint32_t*>(B.rank + 4);
    return (int)(((oct < 4 ? lo : hi) >> (8 * (oct & 3))) & 0xff);
}
#ifndef RT_CLU_FAST  // 1: the cluster box pass RT_CLU_UNROLL boxes per iteration (scalar loads in one
#define RT_CLU_FAST 1  // batch), slab planes as one fma each, the octant rank by one v_perm_b32,
#endif                 // a 32-bit candidate mask while nclu <= 32
#ifndef RT_CLU_UNROLL
#define RT_CLU_UNROLL 2
#endif
#ifndef RT_CLU_SCHED
#define RT_CLU_SCHED 1
#endif
#ifndef RT_CLU_SLOAD  // 1: the box pass's boxes through scalar loads (asm), see clusters_mask
#define RT_CLU_SLOAD 1
#endif
#ifndef RT_CULL_WALL_CONE  // 1: the cull kernels' bounce segments test only the walls whose
#define RT_CULL_WALL_CONE 1 // circumscribed ball meets the wave's cone (wall_cone_mask)
#endif
#ifndef RT_CULL_WALL_BINS  // 1: the cull kernels' primary segment tests only the walls whose
#define RT_CULL_WALL_BINS 1 // pixel box meets the tile (KParams::nwbox; spheres keep the cone)
#endif
/* Slab planes: RT_CLU_FAST forms (lo - o) / d as fma(lo, 1/d, -o/d) with o/d rounded once
 * per ray.  Its error along the ray, 2^-24 |o| |d| / |d_axis| per plane, scales with the
 * same 1 / |d_axis| as the box margin's slack (margin |d| / |d_axis|), so for origins within
 * clu_oinf (100 x the extent, margin 1e-3 x the extent) the widened box still contains the
 * balls' slabs.  d_axis = 0: NaN plane terms drop out of the min / max (no constraint),
 * which is conservative. */
struct SlabRay {
    f3 o, inv, oi;  // origin, 1/d, o/d (fma form)
};
__device__ __forceinline__ SlabRay slab_ray(const f3 o, const f3 d) {
    SlabRay r;
    r.o = o;
    r.inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    r.oi = F3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    return r;
}
__device__ __forceinline__ void slab_tt(const Clu32& B, const SlabRay& s, float& tn, float& tf) {
    float x1, x2, y1, y2, z1, z2;
    if (RT_CLU_FAST) {
        x1 = fmaf(B.lo[0], s.inv.x, -s.oi.x), x2 = fmaf(B.hi[0], s.inv.x, -s.oi.x);
        y1 = fmaf(B.lo[1], s.inv.y, -s.oi.y), y2 = fmaf(B.hi[1], s.inv.y, -s.oi.y);
        z1 = fmaf(B.lo[2], s.inv.z, -s.oi.z), z2 = fmaf(B.hi[2], s.inv.z, -s.oi.z);
    } else {
        x1 = (B.lo[0] - s.o.x) * s.inv.x, x2 = (B.hi[0] - s.o.x) * s.inv.x;
        y1 = (B.lo[1] - s.o.y) * s.inv.y, y2 = (B.hi[1] - s.o.y) * s.inv.y;
        z1 = (B.lo[2] - s.o.z) * s.inv.z, z2 = (B.hi[2] - s.o.z) * s.inv.z;
    }
    tn = fmaxf(fmaxf(fminf(x1, x2), fminf(y1, y2)), fmaxf(fminf(z1, z2), 0.0f));
    tf = fminf(fminf(fmaxf(x1, x2), fmaxf(y1, y2)), fmaxf(z1, z2));
}
__device__ __forceinline__ float slab_t(const Clu32& B, const SlabRay& s) {
    float tn, tf;
    slab_tt(B, s, tn, tf);
    return tn <= tf ? tn : __builtin_inff();
}
/* The lane's candidate clusters as a bit mask: bit k = the cluster at rank k of the lane's
 * octant order (OCT) or cluster k, for the clusters whose box the lane's ray meets (every
 * cluster when !near).  RT_CLU_FAST: RT_CLU_UNROLL boxes per iteration (the clusters array holds
 * room for a multiple of four records; the rest are masked off by c < nclu). */
template <bool OCT, bool WIDE>
__device__ __forceinline__ uint64_t clusters_mask(const KParams& p, const SlabRay& s, bool alive,
                                                  bool near, int oct) {
    // rank of cluster c in the lane's octant order: byte `oct` of Clu32::rank
    const uint32_t sel = (uint32_t)oct | 0x0c0c0c00u;  // v_perm_b32: byte 0 <- byte oct, rest 0
    using M = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    M cm = 0;
    const int n4 = (p.nclu + 3) & ~3;
    for (int c0 = 0; c0 < n4; c0 += RT_CLU_UNROLL) {
        Clu32 Bs[RT_CLU_UNROLL];  // wave-uniform: one batch of scalar loads
#if RT_CLU_SLOAD
        // the compiler cannot prove that nothing in the cull kernels writes the boxes (the
        // DPP asm, the LDS stack), so it loads them through the vector memory path, one VMEM
        // round trip per iteration; read here as two s_load_dwordx8 instead (reads through
        // the scalar cache; the scene is constant while a kernel runs)
        static_assert(RT_CLU_UNROLL == 2 && sizeof(Clu32) == 32, "two 32-byte boxes per batch");
        {
            typedef int v8i __attribute__((ext_vector_type(8)));
            v8i r0, r1;
            const Clu32* q = p.clu + c0;
            asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx8 %1, %2, 0x20\n\t"
                         "s_waitcnt lgkmcnt(0)"
                         : "=s"(r0), "=s"(r1)
                         : "s"(q)
                         : "memory");
            Bs[0] = __builtin_bit_cast(Clu32, r0);
            Bs[1] = __builtin_bit_cast(Clu32, r1);
        }
#else
#pragma unroll
        for (int u = 0; u < RT_CLU_UNROLL; ++u) Bs[u] = p.clu[c0 + u];
#endif
#pragma unroll
        for (int u = 0; u < RT_CLU_UNROLL; ++u) {
            // one box at a time (a handful of VGPRs), not four interleaved
            if (RT_CLU_SCHED) __builtin_amdgcn_sched_barrier(0);
            const int c = c0 + u;
            const Clu32& B = Bs[u];
            float tn, tf;
            slab_tt(B, s, tn, tf);
            const bool in = alive && c < p.nclu && (!near || tn <= tf);
            uint32_t bit = (uint32_t)c;
            if (OCT) {
                const uint32_t lo = *reinterpret_cast<const uint32_t*>(B.rank);
                const uint32_t hi = *reinterpret_cast<const uint32_t*>(B.rank + 4);
                bit = __builtin_amdgcn_perm(hi, lo, sel);
            }
            cm |= (M)in << bit;
        }
    }
    return (uint64_t)cm;
}
__device__ __forceinline__ void clusters_scan(const KParams& p, const RayD& r, bool alive, HitD& h) {
    const f3 o = F3((float)r.o.x, (float)r.o.y, (float)r.o.z);
    const f3 d = F3((float)r.d.x, (float)r.d.y, (float)r.d.z);
    const SlabRay sr = slab_ray(o, d);
    const bool near = fmax3abs(o.x, o.y, o.z) <= p.clu_oinf;
    const int oct = clu_octant(d);
    uint64_t cm = 0;  // bit k: the cluster at rank k of this lane's octant order
    if (RT_CLU_FAST) {
        cm = p.nclu <= 32 ? clusters_mask<RT_CLU_OCT, false>(p, sr, alive, near, oct)
                          : clusters_mask<RT_CLU_OCT, true>(p, sr, alive, near, oct);
    } else {
        for (int c = 0; c < p.nclu; ++c) {  // wave-uniform: scalar loads of the box
            const bool in = !near || slab_t(p.clu[c], sr) < __builtin_inff();
            cm |= (uint64_t)(alive && in) << clu_bit<RT_CLU_OCT>(p.clu[c], oct, c);
        }
    }
    const float dax = p.clu_axis == 0 ? d.x : (p.clu_axis == 1 ? d.y : d.z);
    const bool rev = !RT_CLU_OCT && dax < 0.0f;
    while (__any(cm != 0)) {
        if (cm != 0) {
            DIAG(6);  // (diagnostic build) one walk step: lanes with a cluster left
            const int k = rev ? 63 - __builtin_clzll(cm) : __builtin_ctzll(cm);
            cm &= ~(1ull << k);
            const int c = RT_CLU_OCT ? (int)p.cord[oct * CLU_MAX + k] : k;
            const float t = near ? slab_t(p.clu[c], sr) : 0.0f;
            if ((double)t * r.dlen * (1.0 - 1e-3) <= h.dist) {
                DIAG(14);  // (diagnostic build) lanes whose cluster is not pruned
                // leaves of CLU_SIZE_D, or CLU_SIZE for the scenes that need more than
                // CLU_MAX of those (unrolled as one CLU_SIZE loop: a runtime trip count made
                // the PATH64 cull kernel spill, A/B +10..17%)
                const CluSph* cs = p.csph + c * p.clu_ls;
#pragma unroll
                for (int k = 0; k < CLU_SIZE; ++k) {
                    if (k == CLU_SIZE_D && p.clu_ls == CLU_SIZE_D) break;
                    const int s = cs[k].slot;
                    if (s >= 0) sphere_exact<false>(cs[k].c, s, r, h, &p);
                }
            }
        }
    }
}

template <bool MIXED, bool CULL, bool CLU>
__device__ __forceinline__ HitD scan_d(const KParams& p, const RayD& r, bool alive,
                                       bool primary, bool binned, uint64_t keep) {
    HitD h = no_hit();
    if (CULL) h.dist = dbl_max_s();  // the deep kernels (see dbl_max_s)
    if (CULL) {
        // walls first: their distances then bound the sphere tests
        RayF rf;
        if (MIXED) rf = make_rayf(r);
        const f3 co = F3((float)r.o.x, (float)r.o.y, (float)r.o.z);
        const f3 cd = F3((float)r.d.x, (float)r.d.y, (float)r.d.z);
        const Cone cn = (RT_EYE_CONE && primary) ? wave_cone_eye(co, cd, alive)
                                                 : wave_cone(co, cd, alive);
        if (RT_WALLS_FIRST) {
            uint64_t wm = ~0ull;  // walls to test (bit w = wall w; walls past 63: all)
            if (RT_CULL_WALL_BINS && primary && binned)
                wm = keep;  // the primary segment: the walls' pixel boxes
            else if (RT_CULL_WALL_CONE && cn.on && p.nW > 0 && p.nW <= 64)
                wm = wall_cone_mask(p, cn);  // the bounces: the wave's cone
            if (alive) {
                if (wm != ~0ull)
                    walls_d_kept<MIXED>(p, r, rf, h, wm);
                else
                    walls_d<MIXED, false, RT_WALL_SLOAD>(p, r, rf, h);
            }
        }
        // a wide cone (live rays pointing everywhere) culls little: each lane its own clusters
        // (every precision since round 3: with the recursion stack in LDS the fp64-colour
        // kernels have the registers for it — A/B c5 F64 -44%, MIXED -36%, c3 -9..15%; in
        // round 2 it cost c3 F64 +40%)
        const bool clusters = RT_CLUSTERS && CLU && p.nclu > 0 && cn.cos_t < p.clu_cos;
#if RT_DIAG
        if (alive) DIAG(0);  // wave-level segments of the cull kernels (tools/diag_run.py --cull)
        if (clusters && alive) DIAG(4);
#endif
        if (clusters) clusters_scan(p, r, alive, h);
        for (int c0 = 0; !clusters && c0 < p.nS; c0 += 64) {
            float lb;
            SphRec rec;
            uint64_t m = cull_chunk<true>(p, cn, c0, &lb, rec);
            // survivors in index order; each record comes out of the testing lane's
            // registers (v_readlane), no memory round trip
            while (m) {
                const int l = __builtin_ctzll(m);
                m &= m - 1;
                const double bound = (double)lane_f(lb, l);
                // exact skip: the sphere's distance is >= bound > this lane's best
                if (alive && bound <= h.dist) {
                    DIAG(12);  // (diagnostic build) one cone survivor tested
                    const int sidx = c0 + l;
                    const float Sf[4] = {lane_f(rec.f[0], l), lane_f(rec.f[1], l),
                                         lane_f(rec.f[2], l), lane_f(rec.f[3], l)};
                    if (!(MIXED && sphere_cull(Sf, rf))) {
                        if (RT_CULL_REC64_SCALAR) {
                            sphere_exact<false>(p.s64[sidx >> 2].v[sidx & 3], sidx, r, h, &p);
                        } else {
                            const double Sd[4] = {lane_d(rec.d[0], l), lane_d(rec.d[1], l),
                                                  lane_d(rec.d[2], l), lane_d(rec.d[3], l)};
                            sphere_exact<false>(Sd, sidx, r, h, &p);
                        }
                    }
                }
            }
        }
        if (!RT_WALLS_FIRST && alive) walls_d<MIXED>(p, r, rf, h);
    } else if (alive) {
        // primary, p.eye and p.bins are wave-uniform: one scan or another per wave (MIXED
        // keeps its fp32 cull in front of every test: no eye tables, A/B +1.5%)
        if (binned) {
            h = (!MIXED && primary && p.eye) ? closest_hit_bin<MIXED, true>(p, r, keep)
                                             : closest_hit_bin<MIXED, false>(p, r, keep);
        } else {
            h = (!MIXED && primary && p.eye) ? closest_hit_d<MIXED, true>(p, r)
                                             : closest_hit_d<MIXED, false>(p, r);
        }
    }
    return h;
}

/* One pixel on the exact fp64 ray path.  COLOR64: colour arithmetic in fp64 too (F64 /
 * MIXED, the parity modes); otherwise in fp32 (PATH64). */
template <bool MIXED, bool COLOR64, bool SUN, bool INT_EXP, bool CULL, int MAXD>
__device__ __forceinline__ d3 trace_pixel_d(const KParams& p, int x, int i, bool alive,
                                            int& segs, uint64_t& t_start, uint64_t braw_in,
                                            uint64_t* g_stage = nullptr) {
    using CT = typename std::conditional<COLOR64, double, float>::type;
    const d3 cpos = ld3(p.pos);
    const d3 pc = (ld3(p.tl) + ld3(p.dx) * (double)x) + ld3(p.dy) * (double)i;  // main.cpp:132
    uint64_t braw = 0;
    if (!CULL)
        braw = RT_EARLY_LOADS >= 2 ? braw_in : RT_EARLY_LOADS ? box_load_primary(p) : box_load(p, p.box);
    else if (RT_CULL_WALL_BINS && p.nwbox > 0)  // (wave-uniform: scenes with walls only)
        braw = box_load_walls(p);
    // main.cpp:133-134 (direction not normalised); the sphere terms only where needed
    // (PATH64: the fp32 terminal segment needs none of them)
    constexpr bool LAZY = RT_LAZY_TERMS && !COLOR64 && !CULL && RT_TERMINAL_F32;
    constexpr bool SKYF = RT_SKY_FAST && !COLOR64 && !CULL && RT_TERMINAL_F32;
    RayD r = (LAZY || SKYF) ? make_ray_lazy(cpos, cpos - pc) : make_ray(cpos, cpos - pc);
    bool terms = !LAZY;
    STAGE(1);
    constexpr bool sun = SUN;
    // the wave's start stamp for the dispatch-order feedback (stamped build only): here,
    // between ray generation and the box compare's wait on its load
    t_start = RT_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    if (RT_BOX_SCHED_BARRIER) __builtin_amdgcn_sched_barrier(0);  // compare after ray gen
    const TileO tile = tile_origin(x, i);
    uint64_t keep = ~0ull;
    if (!CULL) {
        keep = box_keep(braw, tile);  // all lanes active
        if (p.nbox == 0) keep = ~0ull;
    } else if (RT_CULL_WALL_BINS && p.nwbox > 0) {  // (wave-uniform)
        keep = box_keep(braw, tile);  // the walls' boxes (bit w = wall w)
    }
    STAGE(6);
    if (SKYF) {
        if (keep == 0) {  // wave-uniform: every primary ray of the tile misses (tile bins)
            f3 c = F3(0.f, 0.f, 0.f);
            if (alive) {
                ++segs;
                c = sky32(r.d);
            }
            STAGE(2);
            STAGE(3);
            STAGE(4);
            return D3(c.x, c.y, c.z);
        }
        if (!LAZY) ray_terms(r);
    }
    const uint64_t smask = p.nS >= 64 ? ~0ull : (1ull << p.nS) - 1;

    // The register stack of the recursion (per level: shading scalar, sun scalar, material
    // slot).  In the cull kernels (deep configs) it lives in LDS instead (RT_STACK_LDS): a
    // VGPR array indexed by the runtime bounce counter costs a select per element on every
    // push and holds 2-3 VGPRs per level for the whole bounce loop, which is what the deep
    // fp64 kernels spilled to scratch.  LDS: one ds_write per value per bounce, one read
    // per level in the unwind, [level][lane] so a wave's accesses are conflict-free.
    constexpr bool LSTK = RT_STACK_LDS >= 2 || (RT_STACK_LDS && CULL);  // 2: every kernel
    __shared__ CT lds_s[LSTK ? MAXD * BLOCK : 1];
    __shared__ CT lds_k[(LSTK && SUN) ? MAXD * BLOCK : 1];
    __shared__ int lds_m[LSTK ? MAXD * BLOCK : 1];
    CT st_s[LSTK ? 1 : MAXD];
    CT st_k[LSTK ? 1 : MAXD];
    int st_m[LSTK ? 1 : MAXD];
    const int tid = (int)threadIdx.x;
    auto push = [&](int k, CT sv, CT kv, int mv) __attribute__((always_inline)) {
        if constexpr (LSTK) {
            lds_s[k * BLOCK + tid] = sv;
            if (SUN) lds_k[k * BLOCK + tid] = kv;
            lds_m[k * BLOCK + tid] = mv;
        } else {
            st_s[k] = sv;
            st_k[k] = kv;
            st_m[k] = mv;
        }
    };
    auto ld_s = [&](int q) __attribute__((always_inline)) -> CT {
        if constexpr (LSTK) return lds_s[q * BLOCK + tid]; else return st_s[q];
    };
    auto ld_k = [&](int q) __attribute__((always_inline)) -> CT {
        if constexpr (LSTK) return SUN ? lds_k[q * BLOCK + tid] : (CT)0; else return st_k[q];
    };
    auto ld_m = [&](int q) __attribute__((always_inline)) -> int {
        if constexpr (LSTK) return lds_m[q * BLOCK + tid]; else return st_m[q];
    };
    int n = 0;
    d3 c64 = D3(0, 0, 0);
    f3 c32 = F3(0.f, 0.f, 0.f);
    // One segment (one closest-hit query per live lane) at bounce k.  Converged: lanes
    // whose path ended stay (alive == false) so the wave can reduce over its live rays; k
    // is wave-uniform.
    auto segment = [&](const int k) __attribute__((always_inline)) {
        bounce_priority(k);
        // tile bins: the primary segment, and the first bounce when the whole wave
        // reflected off one wall (both wave-uniform)
        uint64_t km = ~0ull;
        if (!CULL && k == 0 && p.nbox > 0) km = keep;
        if (!CULL && k >= 1 && k <= p.mir_depth) km = mirror_keep<MAXD>(p, alive, st_m, k, tile);
        if (CULL && RT_CULL_WALL_BINS && k == 0) km = keep;  // ~0 when the walls have no boxes
        if (LAZY && !terms && (km & smask) != 0) {  // a sphere may be tested
            ray_terms(r);
            terms = true;
        }
#if RT_DIAG
        if (k >= 1 && __any(alive)) {
            if (km != ~0ull) DIAG(12);
            else DIAG(14);
        }
#endif
        const HitD h = scan_d<MIXED, CULL, !COLOR64 || RT_CLUSTERS_F64>(p, r, alive, k == 0, km != ~0ull, km);
        if (k == 0) STAGE(2);
        const bool last = k >= p.depth || k >= MAXD;  // remaining_iterations <= 0 (main.cpp:105)
        if (LAZY && !terms && __any(alive && !last && h.slot >= 0)) {  // a reflection follows
            ray_terms(r);
            terms = true;
        }
        if (!alive) return;
        ++segs;
        if (!COLOR64 && RT_TERMINAL_F32 && (last || h.slot < 0)) {
            // PATH64, last segment of the path: nothing here feeds another ray
            DIAG(10);
            if (h.slot < 0) {
                c32 = sky32(r.d);
            } else {
                const f3 nv32 = fnormalize(tof(r.d));
                const d3 pos = r.o + r.d * h.dist;
                f3 N32;
                if (h.slot < p.nS) {
                    const double* S = p.s64[h.slot >> 2].v[h.slot & 3];
                    N32 = tof((r.o + r.d * h.pt) - D3(S[0], S[1], S[2]));
                } else {
                    N32 = tof(ld3(p.w64[h.slot - p.nS].n));
                }
                const DevMat32& m32 = p.mat32[h.slot];
                const float2 sh = shade_f(m32, tof(pos), fnormalize(N32), nv32, sun);
                c32 = local_color_f(m32, sh.x, sh.y, sun);
            }
            alive = false;
            return;
        }
        DIAG(8);
        const double rdl = rcp_refined(r.dlen);
        const d3 nv = div3(r.d, r.dlen, rdl);  // normalize(d); normalize(-d) == -nv
        if (h.slot < 0) {
            if (COLOR64) {
                c64 = sky_d(r, nv.z);
            } else if (r.d.z < 0.0) {
                c32 = F3(0.025f, 0.05f, 0.075f);
            } else {
                const float tz = fsqrt(fsqrt((float)nv.z));
                c32 = F3(fmaf(tz, 0.14f - 0.36f, 0.36f), fmaf(tz, 0.21f - 0.45f, 0.45f),
                         fmaf(tz, 0.49f - 0.57f, 0.57f));
            }
            alive = false;
            return;
        }
        const d3 pos = r.o + r.d * h.dist;  // main.cpp:99 (sphere world distance used as t)
        d3 N;
        if (h.slot < p.nS) {
            const double* S = p.s64[h.slot >> 2].v[h.slot & 3];
            N = (r.o + r.d * h.pt) - D3(S[0], S[1], S[2]);  // un-normalised, length r
        } else {
            N = ld3(p.w64[h.slot - p.nS].n);
        }
        const DevMat& m = p.mat[h.slot];
        // normalize(N): a wall's is a scene constant (host, same IEEE operations); the MIXED
        // cull kernels keep recomputing it (the select costs them 4 VGPRs and a wave/SIMD)
        const d3 nn = (h.slot < p.nS || (MIXED && CULL)) ? normalize_e(N)
                                                           : ld3(p.wnn[h.slot - p.nS]);
        CT s, ks;
        if (COLOR64) {
            const ShadeD sh = shade_d<INT_EXP>(m, pos, nn, -nv, sun);
            s = sh.s;
            ks = sh.ksun;
        } else {
            const float2 sh = shade_f(p.mat32[h.slot], tof(pos), tof(nn), tof(nv), sun);
            s = sh.x;
            ks = sh.y;
        }
        if (last) {
            if (COLOR64)
                c64 = local_color_d(m, s, ks, sun);
            else
                c32 = local_color_f(p.mat32[h.slot], s, ks, sun);
            alive = false;
            return;
        }
        push(k, s, ks, h.slot);
        n = k + 1;
        // start + reflect(d, N) (main.cpp:111-113, vec.cpp:51-57)
        const double cc = 2 * dot(nv, nn);
        if (LAZY) {
            r = make_ray_lazy(pos + N * .0001, nv - nn * cc);
            terms = false;
        } else {
            r = make_ray(pos + N * .0001, nv - nn * cc);
        }
        };
    // The primary segment is peeled off the bounce loop (RT_PEEL): it runs as straight-line
    // code with k == 0 folded, so the loop's phi copies and control are only paid by waves
    // that bounce.
    int kend = 0;  // wave-uniform: bounce iterations run (every lane's n <= kend)
    if (RT_PEEL >= 2) {
        if (__any(alive)) {
            segment(0);
            if (!__any(alive)) {
                kend = 1;
            } else {
                segment(1);
                for (int k = 2;; ++k) {
                    if (!__any(alive)) {
                        kend = k;
                        break;
                    }
                    segment(k);
                }
            }
        }
    } else if (RT_PEEL) {
        if (__any(alive)) {
            segment(0);
            for (int k = 1;; ++k) {
                if (!__any(alive)) {
                    kend = k;
                    break;
                }
                segment(k);
            }
        }
    } else {
        for (int k = 0;; ++k) {
            if (!__any(alive)) {
                kend = k;
                break;
            }
            segment(k);
        }
    }
    STAGE(3);
    for (int q = MAXD - 1; q >= 0; --q) {
        if ((!RT_UNWIND_KEND || q < kend) && q < n) {  // uniform test: levels no lane reached
            const int mq = ld_m(q);
            const DevMat& m = p.mat[mq];
            if (COLOR64) {
                const d3 L = local_color_d(m, ld_s(q), ld_k(q), sun);
                c64 = lerp(L, c64, m.km);  // vec.cpp:45-49 via main.cpp:117
            } else {
                const DevMat32& m32 = p.mat32[mq];
                const f3 L = local_color_f(m32, ld_s(q), ld_k(q), sun);
                const float km = m32.km;
                c32 = F3(fmaf(km, c32.x - L.x, L.x), fmaf(km, c32.y - L.y, L.y),
                         fmaf(km, c32.z - L.z, L.z));
            }
        }
    }
    STAGE(4);
    if (COLOR64) return c64;
    return D3(c32.x, c32.y, c32.z);
}

/* ------------------------------------------------------------------------ */
/* PATH64, two pixels per lane (RT_OPT_PIXEL_PAIRS)                          */
/* ------------------------------------------------------------------------ */
/* A wave traces a 16x8 tile: lane l holds pixel (x0 + l%8, i0 + l/8) and the pixel 8
 * columns to its right.  At c2 the primary pass issues about as many SALU, branch and
 * scalar-load instructions as VALU and a SIMD issues ~one instruction per
 * quad-cycle there; those are per-wave costs (the primitive's record, the loop, the
 * exec-mask bookkeeping of each test's branch), so two pixels per lane pay them once for
 * 128 pixels, and each test's two independent dependency chains share one branch.
 * Every test is trace_pixel_d's (PATH64: exact fp64 paths, fp32 colour) evaluated for
 * both pixels of the lane under ONE branch taken when either pixel needs its body; the
 * results are kept by predicated selects, so each pixel's hit, path and colour are
 * bitwise those of the one-pixel kernel (tested: test_pixel_pairs_bitwise). */
template <int MAXD>
struct PxS {  // one pixel's path state (its register stack lives in separate arrays: the
    RayD r;   // promotion of a dynamically indexed array to registers needs an array alloca)
    int n;
    f3 c;
    bool alive;
};


/* sphere_exact_oc's accept path for one pixel, branch-free given g (the early rejections
 * passed).  The x == 0 case of scene.cpp:64-66 folds in: sqrt(0) = 0 gives num == -dt
 * exactly, so q = div_r(num, a) is its pt and its proj is 2q (the reference's /a); for
 * x > 0 num <= 0 gives q <= 0, rejected by dist > 0 as sphere_exact_oc's num test does. */
__device__ __forceinline__ void sphere_accept(double dt, double x, bool g, int s, const RayD& r,
                                              HitD& h) {
    const bool x0 = x == 0;
    const double sq = sqrt_e(g && !x0 ? x : 1.0);
    const double num = -dt - (x0 ? 0.0 : sq);
    const double q = div_r(num, r.a, r.ra);
    const double dist = (x0 ? 2.0 * q : q) * r.dlen;  // world distance, scene.cpp:77
    const bool take = g && num > 0 && dist > 0 && dist < h.dist;
    h.dist = take ? dist : h.dist;
    h.pt = take ? q : h.pt;
    h.slot = take ? s : h.slot;
}
/* Sphere s for both pixels (spheres in index order: strict < keeps the earlier). */
template <int MAXD>
__device__ __forceinline__ void sphere_pair(const d3 oc0, double c0, const d3 oc1, double c1,
                                            int s, const PxS<MAXD>& a, const PxS<MAXD>& b,
                                            HitD& ha, HitD& hb) {
    const double dta = dot(a.r.d, oc0), dtb = dot(b.r.d, oc1);
    const double xa = dta * dta - a.r.a * c0, xb = dtb * dtb - b.r.a * c1;
    const bool ga = a.alive && !(dta > 0 || !(xa >= 0));
    const bool gb = b.alive && !(dtb > 0 || !(xb >= 0));
    if (ga || gb) {
        DIAG(2);
        sphere_accept(dta, xa, ga, s, a.r, ha);
        sphere_accept(dtb, xb, gb, s, b.r, hb);
    }
}
/* wall_exact's bounds test and take for one pixel, branch-free given g (t > 0, t <= best). */
__device__ __forceinline__ void wall_accept(const Wall64& Wl, int w, const KParams& p, double t,
                                            bool g, const RayD& r, const d3 P, HitD& h) {
    const d3 q = (r.o + r.d * t) - P;  // ray::at (scene.h:16) minus the corner
    const double px = dot(q, ld3(Wl.X));
    const double py = dot(q, ld3(Wl.Y));
    const bool inb = g && px >= 0 && px <= Wl.len && py >= 0 && py <= Wl.wid;
    bool take = inb && t < h.dist;
    if (inb && !take && t == h.dist && h.slot >= 0)  // tie: the lower scene index wins (rare)
        take = p.wall_j[w] < scene_index(p, h.slot);
    h.dist = take ? t : h.dist;
    h.slot = take ? p.nS + w : h.slot;
}
template <bool EYE, int MAXD>
__device__ __forceinline__ void wall_pair_px(const Wall64& Wl, int w, const KParams& p,
                                             const PxS<MAXD>& a, const PxS<MAXD>& b, HitD& ha,
                                             HitD& hb) {
    const d3 n = ld3(Wl.n);
    const d3 P = ld3(Wl.P);
    const double dena = dot(n, a.r.d), denb = dot(n, b.r.d);
    const double numa = EYE ? p.eye_w[w] : dot(P - a.r.o, n);
    const double numb = EYE ? p.eye_w[w] : dot(P - b.r.o, n);
    // as wall_exact (RT_WALL_NOSIGN, RT_WALL_TSKIP): t <= 0, NaN, +-inf and t > best fail
    const double ta = div_r_nz(numa, dena, rcp_refined(dena));
    const double tb = div_r_nz(numb, denb, rcp_refined(denb));
    const bool ga = a.alive && ta > 0 && !(ta > ha.dist);
    const bool gb = b.alive && tb > 0 && !(tb > hb.dist);
    if (ga || gb) {
        DIAG(6);
        wall_accept(Wl, w, p, ta, ga, a.r, P, ha);
        wall_accept(Wl, w, p, tb, gb, b.r, P, hb);
    }
}
template <bool EYE, int MAXD>
__device__ __forceinline__ void sphere_pair_idx(const KParams& p, int s, const PxS<MAXD>& a,
                                                const PxS<MAXD>& b, HitD& ha, HitD& hb) {
    if (EYE) {
        const double* E = p.eye_s[s];
        const d3 oc = D3(E[0], E[1], E[2]);
        sphere_pair(oc, E[3], oc, E[3], s, a, b, ha, hb);
    } else {
        const double* S = p.s64[s >> 2].v[s & 3];
        const d3 C = D3(S[0], S[1], S[2]);
        const d3 oca = a.r.o - C, ocb = b.r.o - C;
        sphere_pair(oca, lensq(oca) - S[3], ocb, lensq(ocb) - S[3], s, a, b, ha, hb);
    }
}
/* closest_hit_bin / closest_hit_d for both pixels of every lane (keep wave-uniform). */
template <bool EYE, int MAXD>
__device__ __forceinline__ void scan_pair_bin(const KParams& p, const PxS<MAXD>& a,
                                              const PxS<MAXD>& b, uint64_t keep, HitD& ha,
                                              HitD& hb) {
    uint64_t sm = p.nS >= 64 ? keep : keep & ((1ull << p.nS) - 1);
    while (sm) {
        const int s = __builtin_ctzll(sm);
        sm &= sm - 1;
        sphere_pair_idx<EYE>(p, s, a, b, ha, hb);
    }
    uint64_t wm = p.nS >= 64 ? 0 : keep >> p.nS;
    while (wm) {
        const int w = __builtin_ctzll(wm);
        wm &= wm - 1;
        wall_pair_px<EYE>(p.w64[w], w, p, a, b, ha, hb);
    }
}
template <bool EYE, int MAXD>
__device__ __forceinline__ void scan_pair_all(const KParams& p, const PxS<MAXD>& a,
                                              const PxS<MAXD>& b, HitD& ha, HitD& hb) {
    for (int s = 0; s < p.nS; ++s) sphere_pair_idx<EYE>(p, s, a, b, ha, hb);
    for (int w = 0; w < p.nW; ++w) wall_pair_px<EYE>(p.w64[w], w, p, a, b, ha, hb);
}

/* Tile bins for a 16-pixel-wide tile (box_keep's compare, one ballot). */
__device__ __forceinline__ uint64_t box_keep16(uint64_t raw, TileO t) {
    const int x0 = (int16_t)(raw & 0xffff), x1 = (int16_t)((raw >> 16) & 0xffff);
    const int i0 = (int16_t)((raw >> 32) & 0xffff), i1 = (int16_t)(raw >> 48);
    const bool hit = (x0 <= t.x0 + 15) & (x1 >= t.x0) & (i0 <= t.y0 + 7) & (i1 >= t.y0);
    return uniform64(__ballot(hit));
}
/* mirror_keep (RT_MIR_CHAINS = 1) over both pixels of every lane: the keep mask of the wall
 * chain that every live pixel of the wave followed, or ~0. */
template <int MAXD>
__device__ __forceinline__ uint64_t mirror_keep_pair(const KParams& p, const PxS<MAXD>& a,
                                                     const PxS<MAXD>& b, const int* ma,
                                                     const int* mb, int k, TileO t) {
    const uint64_t todo = uniform64(__ballot(a.alive || b.alive));
    if (todo == 0 || k > p.mir_depth) return ~0ull;
    const int l0 = __builtin_ctzll(todo);
    const bool lead_a = __builtin_amdgcn_readlane((int)a.alive, l0) != 0;
    bool same_a = true, same_b = true;
    int q = 0, off = 0, lvl = 1;
#pragma unroll
    for (int j = 0; j < MIR_MAX_DEPTH && j < MAXD; ++j) {
        if (j < k) {
            const int sj = __builtin_amdgcn_readlane(lead_a ? ma[j] : mb[j], l0);
            if (sj < p.nS) return ~0ull;  // a sphere bounce: no linear mirror
            same_a = same_a && ma[j] == sj;
            same_b = same_b && mb[j] == sj;
            q = q * p.nW + (sj - p.nS);
            if (j > 0) off += lvl;
            lvl *= p.nW;
        }
    }
    if (uniform64(__ballot((a.alive && !same_a) || (b.alive && !same_b))) != 0) return ~0ull;
    const int l = threadIdx.x & 63;
    const PrimBox* boxes = p.mbox + (off + q) * p.nbox;
    const uint64_t raw = *reinterpret_cast<const uint64_t*>(boxes + (l < p.nbox ? l : 0));
    return box_keep16(l < p.nbox ? raw : 0x80007fff80007fffull, t);
}

/* trace_pixel_d<PATH64>'s per-pixel work after the scan of segment k (the lambda's body). */
template <bool SUN, int MAXD>
__device__ __forceinline__ void pair_after_scan(const KParams& p, PxS<MAXD>& s, float* st_s,
                                                float* st_k, int* st_m, const HitD& h, int k,
                                                int& segs) {
    if (!s.alive) return;
    ++segs;
    const bool last = k >= p.depth || k >= MAXD;  // remaining_iterations <= 0 (main.cpp:105)
    if (last || h.slot < 0) {  // the path's last segment: colour only, in fp32
        if (h.slot < 0) {
            s.c = sky32(s.r.d);
        } else {
            const f3 nv32 = fnormalize(tof(s.r.d));
            const d3 pos = s.r.o + s.r.d * h.dist;
            f3 N32;
            if (h.slot < p.nS) {
                const double* S = p.s64[h.slot >> 2].v[h.slot & 3];
                N32 = tof((s.r.o + s.r.d * h.pt) - D3(S[0], S[1], S[2]));
            } else {
                N32 = tof(ld3(p.w64[h.slot - p.nS].n));
            }
            const DevMat32& m32 = p.mat32[h.slot];
            const float2 sh = shade_f(m32, tof(pos), fnormalize(N32), nv32, SUN);
            s.c = local_color_f(m32, sh.x, sh.y, SUN);
        }
        s.alive = false;
        return;
    }
    const double rdl = rcp_refined(s.r.dlen);
    const d3 nv = div3(s.r.d, s.r.dlen, rdl);  // normalize(d)
    const d3 pos = s.r.o + s.r.d * h.dist;     // main.cpp:99
    d3 N;
    if (h.slot < p.nS) {
        const double* S = p.s64[h.slot >> 2].v[h.slot & 3];
        N = (s.r.o + s.r.d * h.pt) - D3(S[0], S[1], S[2]);  // un-normalised, length r
    } else {
        N = ld3(p.w64[h.slot - p.nS].n);
    }
    const d3 nn = h.slot < p.nS ? normalize_e(N) : ld3(p.wnn[h.slot - p.nS]);
    const float2 sh = shade_f(p.mat32[h.slot], tof(pos), tof(nn), tof(nv), SUN);
    st_s[k] = sh.x;
    st_k[k] = sh.y;
    st_m[k] = h.slot;
    s.n = k + 1;
    const double cc = 2 * dot(nv, nn);
    s.r = make_ray(pos + N * .0001, nv - nn * cc);  // main.cpp:111-113
}

template <bool SUN, int MAXD>
__device__ __forceinline__ void trace_pair_p64(const KParams& p, int x, int i, bool va, bool vb,
                                               int& segs, uint64_t& t_start, f3& ca, f3& cb) {
    const d3 cpos = ld3(p.pos);
    const d3 pca = (ld3(p.tl) + ld3(p.dx) * (double)x) + ld3(p.dy) * (double)i;  // main.cpp:132
    const d3 pcb = (ld3(p.tl) + ld3(p.dx) * (double)(x + 8)) + ld3(p.dy) * (double)i;
    const uint64_t braw = box_load_primary(p);
    PxS<MAXD> a, b;
    float as_[MAXD], ak_[MAXD], bs_[MAXD], bk_[MAXD];
    int am_[MAXD], bm_[MAXD];
    a.r = make_ray_lazy(cpos, cpos - pca);  // main.cpp:133-134
    b.r = make_ray_lazy(cpos, cpos - pcb);
    a.alive = va;
    b.alive = vb;
    a.n = b.n = 0;
    a.c = b.c = F3(0.f, 0.f, 0.f);
    t_start = RT_STAMP ? __builtin_amdgcn_s_memtime() : 0;
    if (RT_BOX_SCHED_BARRIER) __builtin_amdgcn_sched_barrier(0);
    const TileO tile = tile_origin(x, i);
    uint64_t keep = box_keep16(braw, tile);
    if (p.nbox == 0) keep = ~0ull;
    if (keep == 0) {  // every primary ray of the 16x8 tile misses (sky fast path)
        if (va) {
            ++segs;
            a.c = sky32(a.r.d);
        }
        if (vb) {
            ++segs;
            b.c = sky32(b.r.d);
        }
        ca = a.c;
        cb = b.c;
        return;
    }
    ray_terms(a.r);
    ray_terms(b.r);
    auto segment = [&](const int k) __attribute__((always_inline)) {
        uint64_t km = ~0ull;
        if (k == 0 && p.nbox > 0) km = keep;
        if (k >= 1 && k <= p.mir_depth) km = mirror_keep_pair<MAXD>(p, a, b, am_, bm_, k, tile);
        HitD ha = no_hit(), hb = no_hit();
        const bool eye = k == 0 && p.eye;
        if (km != ~0ull) {
            if (eye)
                scan_pair_bin<true>(p, a, b, km, ha, hb);
            else
                scan_pair_bin<false>(p, a, b, km, ha, hb);
        } else {
            if (eye)
                scan_pair_all<true>(p, a, b, ha, hb);
            else
                scan_pair_all<false>(p, a, b, ha, hb);
        }
        pair_after_scan<SUN, MAXD>(p, a, as_, ak_, am_, ha, k, segs);
        pair_after_scan<SUN, MAXD>(p, b, bs_, bk_, bm_, hb, k, segs);
    };
    int kend = 0;  // wave-uniform: bounce iterations run
    if (__any(a.alive || b.alive)) {
        segment(0);
        if (!__any(a.alive || b.alive)) {
            kend = 1;
        } else {
            segment(1);
            for (int k = 2;; ++k) {
                if (!__any(a.alive || b.alive)) {
                    kend = k;
                    break;
                }
                segment(k);
            }
        }
    }
    // unwind (main.cpp:117 via vec.cpp:45-49), innermost bounce first
    for (int q = MAXD - 1; q >= 0; --q) {
        if (q < kend) {
            if (q < a.n) {
                const DevMat32& m = p.mat32[am_[q]];
                const f3 L = local_color_f(m, as_[q], ak_[q], SUN);
                a.c = F3(fmaf(m.km, a.c.x - L.x, L.x), fmaf(m.km, a.c.y - L.y, L.y),
                         fmaf(m.km, a.c.z - L.z, L.z));
            }
            if (q < b.n) {
                const DevMat32& m = p.mat32[bm_[q]];
                const f3 L = local_color_f(m, bs_[q], bk_[q], SUN);
                b.c = F3(fmaf(m.km, b.c.x - L.x, L.x), fmaf(m.km, b.c.y - L.y, L.y),
                         fmaf(m.km, b.c.z - L.z, L.z));
            }
        }
    }
    ca = a.c;
    cb = b.c;
}

/* ------------------------------------------------------------------------ */
/* fp32 throughput path                                                      */
/* ------------------------------------------------------------------------ */
/* fp32 sphere test (scaled form; det == 0 keeps scene.cpp:65's 2x distance).
 * IN_ORDER as for sphere_exact. */
template <bool IN_ORDER = true>
__device__ __forceinline__ void sphere_f(const float* S, int s, f3 o, f3 d, float a, float ra,
                                         float rl, float& best, float& bpt, int& slot,
                                         const KParams* p = nullptr) {
    const f3 oc = o - F3(S[0], S[1], S[2]);
    const float bh = fdot(d, oc);
    const float cq = fmaf(-S[3], S[3], fdot(oc, oc));
    const float det = fmaf(bh, bh, -a * cq);
    if (bh <= 0.0f && det >= 0.0f) {
        const float num = -bh - fsqrt(det);
        const float proj = (det == 0.0f) ? -2.0f * bh * ra : num * ra;
        const float dist = proj * a * rl;  // proj * |d|
        const bool ok = (det == 0.0f || num > 0.0f) && dist > 0.0f;
        bool take = ok && dist < best;
        if (!IN_ORDER && ok && !take && dist == best && slot >= 0)
            take = scene_index(*p, s) < scene_index(*p, slot);
        if (take) {
            best = dist;
            bpt = (det == 0.0f) ? -bh * ra : proj;
            slot = s;
        }
    }
}

/* clusters_scan for the F32 kernels: the same walk over the lane's own clusters with the
 * fp32 sphere test (sphere_f, scene-index tie rule); a pruned cluster's spheres lie at a
 * distance >= t_entry |d| > best (box margin 1e-3 x the scene extent). */
__device__ __forceinline__ void clusters_scan_f(const KParams& p, f3 o, f3 d, float a, float ra,
                                                float rl, bool alive, float& best, float& bpt,
                                                int& slot) {
    const SlabRay sr = slab_ray(o, d);
    const bool near = fmax3abs(o.x, o.y, o.z) <= p.clu_oinf;
    const int oct = clu_octant(d);
    uint64_t cm = 0;
    if (RT_CLU_FAST) {
        cm = p.nclu <= 32 ? clusters_mask<RT_CLU_OCT_F32, false>(p, sr, alive, near, oct)
                          : clusters_mask<RT_CLU_OCT_F32, true>(p, sr, alive, near, oct);
    } else {
        for (int c = 0; c < p.nclu; ++c) {
            const bool in = !near || slab_t(p.clu[c], sr) < __builtin_inff();
            cm |= (uint64_t)(alive && in) << clu_bit<RT_CLU_OCT_F32>(p.clu[c], oct, c);
        }
    }
    const float dax = p.clu_axis == 0 ? d.x : (p.clu_axis == 1 ? d.y : d.z);
    const bool rev = !RT_CLU_OCT_F32 && dax < 0.0f;
    const float dl = a * rl;  // |d|
    while (__any(cm != 0)) {
        if (cm != 0) {
            const int k = rev ? 63 - __builtin_clzll(cm) : __builtin_ctzll(cm);
            cm &= ~(1ull << k);
            const int c = RT_CLU_OCT_F32 ? (int)p.cord[oct * CLU_MAX + k] : k;
            const float t = near ? slab_t(p.clu[c], sr) : 0.0f;
            if (t * dl * (1.0f - 1e-3f) <= best) {
                const CluSph* cs = p.csph + c * CLU_SIZE;
#pragma unroll
                for (int k = 0; k < CLU_SIZE; ++k) {
                    const int s = cs[k].slot;
                    if (s >= 0) sphere_f<false>(cs[k].f, s, o, d, a, ra, rl, best, bpt, slot, &p);
                }
            }
        }
    }
}

/* Two spheres (k0, k0+1 of group G) per packed fp32 instruction: the cheap prefix
 * (oc, b/2, c, det) runs as v_pk_* on {sphere k0, sphere k0+1}; the rare hit path
 * (sqrt, divide, compare) per sphere.  Same arithmetic as sphere_f, lane for lane. */
__device__ __forceinline__ void sphere_pair_f(const SphG32& G, int k0, int s0, int nS, f3 o,
                                              f3 d, float a, float ra, float rl, float& best,
                                              float& bpt, int& slot) {
    const f2 cx = {G.c[0][k0], G.c[0][k0 + 1]}, cy = {G.c[1][k0], G.c[1][k0 + 1]};
    const f2 cz = {G.c[2][k0], G.c[2][k0 + 1]}, rr = {G.c[3][k0], G.c[3][k0 + 1]};
    const f2 ocx = f2(o.x) - cx, ocy = f2(o.y) - cy, ocz = f2(o.z) - cz;
    const f2 bh = __builtin_elementwise_fma(
        f2(d.x), ocx, __builtin_elementwise_fma(f2(d.y), ocy, f2(d.z) * ocz));
    const f2 cq = __builtin_elementwise_fma(
        -rr, rr, __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz)));
    const f2 det = __builtin_elementwise_fma(bh, bh, -f2(a) * cq);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (s0 + k >= nS) break;
        const float b1 = bh[k], d1 = det[k];
        if (b1 <= 0.0f && d1 >= 0.0f) {
            const float num = -b1 - fsqrt(d1);
            const float proj = (d1 == 0.0f) ? -2.0f * b1 * ra : num * ra;
            const float dist = proj * a * rl;
            if ((d1 == 0.0f || num > 0.0f) && dist > 0.0f && dist < best) {
                best = dist;
                bpt = (d1 == 0.0f) ? -b1 * ra : proj;
                slot = s0 + k;
            }
        }
    }
}

/* A 64-byte record (Wall32, SphG32) as one s_load_dwordx16: the F32 cull kernels' walls and
 * cone survivors (see clusters_mask's box loads). */
template <class T>
__device__ __forceinline__ T rec64_sload(const T* q) {
    static_assert(sizeof(T) == 64, "one s_load_dwordx16");
    typedef int v16i __attribute__((ext_vector_type(16)));
    v16i a;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(a)
                 : "s"(q)
                 : "memory");
    return __builtin_bit_cast(T, a);
}
template <bool SL = false>
__device__ __forceinline__ void walls_f(const KParams& p, f3 o, f3 d, float& best, int& slot,
                                        uint64_t wmask = ~0ull) {
    for (int w = 0; w < p.nW; ++w) {
        if (w < 64 && !((wmask >> w) & 1)) continue;  // wave-uniform (tile bins)
        const Wall32 Wl = SL ? rec64_sload(p.w32 + w) : p.w32[w];
        const f3 nw = F3(Wl.n[0], Wl.n[1], Wl.n[2]), P = F3(Wl.P[0], Wl.P[1], Wl.P[2]);
        const float den = fdot(nw, d);
        const float num = fdot(P - o, nw);
        // RT_F32_WALL_FLAT: no sign pre-test branch; t <= 0, NaN and inf fail below
        if (!RT_F32_WALL_FLAT && !((num > 0 && den > 0) || (num < 0 && den < 0))) continue;
        const float t = num * frcp(den);
        const f3 q = fmad3(d, t, o) - P;
        const float px = fdot(q, F3(Wl.X[0], Wl.X[1], Wl.X[2]));
        const float py = fdot(q, F3(Wl.Y[0], Wl.Y[1], Wl.Y[2]));
        const bool sgn = RT_F32_WALL_FLAT || ((num > 0 && den > 0) || (num < 0 && den < 0));
        if (sgn && t > 0 && px >= 0 && px <= Wl.len && py >= 0 && py <= Wl.wid) {
            bool take = t < best;
            if (!take && t == best && slot >= 0) take = p.wall_j[w] < scene_index(p, slot);
            if (take) {
                best = t;
                slot = p.nS + w;
            }
        }
    }
}

template <bool SUN, bool CULL, int MAXD>
__device__ __forceinline__ f3 trace_pixel_f(const KParams& p, int x, int i, bool alive,
                                            int& segs, uint64_t& t_start, uint64_t braw_in) {
    const d3 pcd = (ld3(p.tl) + ld3(p.dx) * (double)x) + ld3(p.dy) * (double)i;
    const d3 dd = ld3(p.pos) - pcd;
    f3 o = F3((float)p.pos[0], (float)p.pos[1], (float)p.pos[2]);
    f3 d = F3((float)dd.x, (float)dd.y, (float)dd.z);
    constexpr bool sun = SUN;

    float st_s[MAXD];
    float st_k[MAXD];
    int st_m[MAXD];
    int n = 0;
    f3 c = F3(0.f, 0.f, 0.f);
    t_start = RT_STAMP ? __builtin_amdgcn_s_memtime() : 0;  // see trace_pixel_d
    const TileO tile = tile_origin(x, i);
#if RT_EARLY_LOADS >= 2
    // unconditional compare (all lanes active), so the wave-start box load is not sunk
    uint64_t keep = CULL ? ~0ull : box_keep(braw_in, tile);
    if (p.nbox <= 0) keep = ~0ull;
#else
    const uint64_t keep = (!CULL && p.nbox > 0) ? tile_keep(p, p.box, tile) : ~0ull;
#endif
    // the cull kernels' primary walls behind their pixel boxes (RT_CULL_WALL_BINS)
    uint64_t wkeep = ~0ull;
    if (CULL && RT_CULL_WALL_BINS && p.nwbox > 0) wkeep = box_keep(box_load_walls(p), tile);
    if (!CULL && RT_SKY_FAST && keep == 0) {
        // wave-uniform: every primary ray misses (tile bins): the loop's miss shading below,
        // operation for operation, without the loop
        if (alive) {
            ++segs;
            const f3 nv = d * frsq(fdot(d, d));
            if (d.z < 0.0f) {
                c = F3(0.025f, 0.05f, 0.075f);
            } else {
                const float tz = fsqrt(fsqrt(nv.z));
                c = F3(fmaf(tz, 0.14f - 0.36f, 0.36f), fmaf(tz, 0.21f - 0.45f, 0.45f),
                       fmaf(tz, 0.49f - 0.57f, 0.57f));
            }
        }
        return c;
    }
    auto segment = [&](const int k) __attribute__((always_inline)) {
        bounce_priority(k);
        const float a = fdot(d, d);
        const float ra = frcp(a);
        const float rl = frsq(a);
        float best = FLT_MAX, bpt = 0.0f;
        int slot = -1;
        // tile bins: the primary segment, and the first bounce when the whole wave
        // reflected off one wall (both wave-uniform)
        uint64_t km = ~0ull;
        if (!CULL && k == 0 && p.nbox > 0) km = keep;
        if (!CULL && k >= 1 && k <= p.mir_depth) km = mirror_keep<MAXD>(p, alive, st_m, k, tile);
        const bool binned = km != ~0ull;
        if (!CULL && binned) {
            // kept spheres in index order, kept walls
            if (alive) {
                uint64_t sm = p.nS >= 64 ? km : km & ((1ull << p.nS) - 1);
                while (sm) {
                    const int s = __builtin_ctzll(sm);
                    sm &= sm - 1;
                    const SphG32& G = p.s32[s >> 2];
                    const float Sf[4] = {G.c[0][s & 3], G.c[1][s & 3], G.c[2][s & 3], G.c[3][s & 3]};
                    sphere_f(Sf, s, o, d, a, ra, rl, best, bpt, slot);
                }
                walls_f(p, o, d, best, slot, p.nS >= 64 ? 0 : km >> p.nS);
            }
        } else if (CULL) {
            const Cone cn = (RT_EYE_CONE && k == 0) ? wave_cone_eye(o, d, alive)
                                                    : wave_cone(o, d, alive);
            if (RT_WALLS_FIRST) {
                uint64_t wm = k == 0 ? wkeep : ~0ull;
                if (RT_CULL_WALL_CONE && k > 0 && cn.on && p.nW > 0 && p.nW <= 64)
                    wm = wall_cone_mask(p, cn);
                if (alive) walls_f<RT_WALL_SLOAD>(p, o, d, best, slot, wm);
            }
            // wide cone: each lane its own sphere clusters (clusters_scan)
            const bool clusters = RT_CLUSTERS_F32 && p.nclu > 0 && cn.cos_t < p.clu_cos;
            if (clusters) clusters_scan_f(p, o, d, a, ra, rl, alive, best, bpt, slot);
            for (int c0 = 0; !clusters && c0 < p.nS; c0 += 64) {
                float lb;
                SphRec rec;
                uint64_t m = cull_chunk<false>(p, cn, c0, &lb, rec);
                // (a distance skip costs more than it saves at fp32 test prices: A/B)
                if (alive) {
                    while (m) {
                        const int l = __builtin_ctzll(m);
                        m &= m - 1;
                        const int sidx = c0 + l;
                        float Sf[4];
                        if (RT_F32_READLANE) {
                            Sf[0] = lane_f(rec.f[0], l);
                            Sf[1] = lane_f(rec.f[1], l);
                            Sf[2] = lane_f(rec.f[2], l);
                            Sf[3] = lane_f(rec.f[3], l);
                        } else {
                            // (not through rec64_sload: a wait per survivor, c5 +31%)
                            const SphG32& G = p.s32[sidx >> 2];
                            Sf[0] = G.c[0][sidx & 3];
                            Sf[1] = G.c[1][sidx & 3];
                            Sf[2] = G.c[2][sidx & 3];
                            Sf[3] = G.c[3][sidx & 3];
                        }
                        sphere_f<false>(Sf, sidx, o, d, a, ra, rl, best, bpt, slot, &p);
                    }
                }
            }
            if (!RT_WALLS_FIRST && alive) walls_f(p, o, d, best, slot);
        } else if (alive) {
            const int ng = (p.nS + 3) >> 2;
            for (int g = 0; g < ng; ++g) {
                const SphG32 G = p.s32[g];  // one s_load_dwordx16
#pragma unroll
                for (int h2 = 0; h2 < 2; ++h2) {
                    const int s0 = 4 * g + 2 * h2;
                    if (s0 >= p.nS) break;
                    sphere_pair_f(G, 2 * h2, s0, p.nS, o, d, a, ra, rl, best, bpt, slot);
                }
            }
        }
        if (!alive) return;
        ++segs;
        if (!CULL && !binned) walls_f(p, o, d, best, slot);
        const f3 nv = d * rl;
        if (slot < 0) {
            if (d.z < 0.0f) {
                c = F3(0.025f, 0.05f, 0.075f);
            } else {
                const float tz = fsqrt(fsqrt(nv.z));
                c = F3(fmaf(tz, 0.14f - 0.36f, 0.36f), fmaf(tz, 0.21f - 0.45f, 0.45f),
                       fmaf(tz, 0.49f - 0.57f, 0.57f));
            }
            alive = false;
            return;
        }
        const f3 pos = fmad3(d, best, o);
        f3 N;
        if (slot < p.nS) {
            const SphG32& G = p.s32[slot >> 2];
            N = fmad3(d, bpt, o) - F3(G.c[0][slot & 3], G.c[1][slot & 3], G.c[2][slot & 3]);
        } else {
            const Wall32& Wl = p.w32[slot - p.nS];
            N = F3(Wl.n[0], Wl.n[1], Wl.n[2]);
        }
        const DevMat32& m = p.mat32[slot];
        const f3 nn = fnormalize(N);
        const float2 sh = shade_f(m, pos, nn, nv, sun);
        if (k >= p.depth || k >= MAXD) {
            c = local_color_f(m, sh.x, sh.y, sun);
            alive = false;
            return;
        }
        st_s[k] = sh.x;
        st_k[k] = sh.y;
        st_m[k] = slot;
        n = k + 1;
        const float cc = 2.0f * fdot(nv, nn);
        o = fmad3(N, 1e-4f, pos);
        d = fmad3(nn, -cc, nv);
        };
    int kend = 0;  // wave-uniform: bounce iterations run (every lane's n <= kend)
    // the primary segment and the first bounce peeled (see trace_pixel_d); the F32 cull
    // kernels peel the primary only (the second copy: c3 +6%, c5 +9%)
    if (RT_PEEL >= 2 && !CULL) {
        if (__any(alive)) {
            segment(0);
            if (!__any(alive)) {
                kend = 1;
            } else {
                segment(1);
                for (int k = 2;; ++k) {
                    if (!__any(alive)) {
                        kend = k;
                        break;
                    }
                    segment(k);
                }
            }
        }
    } else if (RT_PEEL) {
        if (__any(alive)) {
            segment(0);
            for (int k = 1;; ++k) {
                if (!__any(alive)) {
                    kend = k;
                    break;
                }
                segment(k);
            }
        }
    } else {
        for (int k = 0;; ++k) {
            if (!__any(alive)) {
                kend = k;
                break;
            }
            segment(k);
        }
    }
    for (int q = MAXD - 1; q >= 0; --q) {
        if ((!RT_UNWIND_KEND || q < kend) && q < n) {  // uniform test: levels no lane reached
            const DevMat32& m = p.mat32[st_m[q]];
            const f3 L = local_color_f(m, st_s[q], st_k[q], sun);
            const float km = m.km;
            c = F3(fmaf(km, c.x - L.x, L.x), fmaf(km, c.y - L.y, L.y), fmaf(km, c.z - L.z, L.z));
        }
    }
    return c;
}

/* ------------------------------------------------------------------------ */
/* epilogue + kernel                                                         */
/* ------------------------------------------------------------------------ */
/* RGBA8: clamp to [0,1] then truncate v*255, the in-range behaviour of
 * SDL_MapRGB(val*255) with its implicit double->Uint8 conversion (main.cpp:345). */
__device__ __forceinline__ unsigned q8(double v) {
    v = v > 0.0 ? v : 0.0;  // NaN -> 0
    v = v < 1.0 ? v : 1.0;
    return (unsigned)(v * 255.0);
}
/* RGBA8_WRAP: the reference's x86-64 bytes for every value — cvttsd2si of v*255 (int32,
 * toward zero; NaN and |v*255| >= 2^31 give 0x80000000), then the low byte. */
__device__ __forceinline__ unsigned q8_wrap(double v) {
    const double t = v * 255.0;
    const int i = (t > -2147483649.0 && t < 2147483648.0) ? (int)t : (int)0x80000000u;
    return (unsigned)i & 0xffu;
}

__device__ __forceinline__ void store_px(const KParams& p, size_t px, double cr, double cg,
                                         double cb) {
    if (p.outf == OUT_RGB_F32) {
        float* o = static_cast<float*>(p.out) + px * 3;
        o[0] = (float)cr;
        o[1] = (float)cg;
        o[2] = (float)cb;
    } else if (p.outf == OUT_RGB_F64) {
        double* o = static_cast<double*>(p.out) + px * 3;
        o[0] = cr;
        o[1] = cg;
        o[2] = cb;
    } else if (p.outf == OUT_RGBA8) {
        const unsigned v = q8(cr) | (q8(cg) << 8) | (q8(cb) << 16) | (255u << 24);
        static_cast<unsigned*>(p.out)[px] = v;
    } else {
        const unsigned v = q8_wrap(cr) | (q8_wrap(cg) << 8) | (q8_wrap(cb) << 16) | (255u << 24);
        static_cast<unsigned*>(p.out)[px] = v;
    }
}
__device__ __forceinline__ void store_pixel(const KParams& p, int r, int x, double cr, double cg,
                                            double cb) {
    store_px(p, (size_t)r * (size_t)p.W + (size_t)x, cr, cg, cb);
}

__device__ __forceinline__ void count_segments(const KParams& p, int segs) {
    if (p.segs == nullptr) return;
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off, 64);  // wave64 sum
    if ((threadIdx.x & 63) == 0) atomicAdd(p.segs, (unsigned long long)segs);
}

/* Occupancy target per instantiation (waves per SIMD; MI355X_MICROARCH.md: <= 128 VGPRs
 * for 4, <= 96 for 5).  The fp64-colour paths carry the most state. */
template <int PREC, bool SUN, bool INT_EXP, bool CULL, int MAXD>
constexpr int waves_per_eu() {
    // The register stack costs 2-5 VGPRs per level and the cull's per-lane records ~12, so
    // the target steps down with depth tier and cull.  Checked with `make asm`
    // (ScratchSize 0 for every no-sun integer-exponent variant; the rare sun +
    // non-integer-exponent deep fp64 variants run at 2 waves and may spill a little).
    const int tier = MAXD >= 16 ? 2 : (MAXD >= 10 ? 1 : 0);
    int w = 0;
    if (PREC == PREC_F64 && !CULL && !SUN && tier == 0) return 4 + RT_WPE_F64_LIN_BONUS;
    if (PREC == PREC_F32)
        // (cull kernels one wave more since the sphere clusters: A/B c5 -4%, c3 -1% vs 5)
        w = 5 + RT_WPE_F32_BONUS - (tier > 0 ? 1 : 0) - ((SUN && tier == 2) ? 1 : 0) +
            ((CULL && !SUN && tier == 0) ? 1 : 0);
    else if (PREC == PREC_PATH64)
        // (5 waves: A/B c5 -7%, c3 -5% with 20 B of spills in the cull kernels; the sun
        // variants, whose spills would be 56-96 B, keep 4)
        w = RT_WPE_PATH64 - (tier == 2 ? 1 : 0) - (SUN ? 1 : 0) +
            ((!CULL && !SUN && tier == 0) ? RT_WPE_PATH64_LIN_BONUS : 0) +
            ((CULL && !SUN && tier == 0) ? RT_WPE_PATH64_CULL_BONUS : 0);
    else
        w = (INT_EXP ? (SUN ? 3 : 4) : (SUN ? 2 : 3)) - (tier > 0 ? 1 : 0) -
            ((PREC == PREC_MIXED && CULL && MAXD >= 8) ? RT_WPE_MIXED_CULL_DROP : 0) +
            (CULL ? RT_WPE_CULL64_BONUS : 0);
    return w < 2 ? 2 : w;
}

/* The store's pixel coordinates are formed again after the trace from the wave-uniform
 * tile (SGPRs) and the lane id read with v_mbcnt (not threadIdx.x, so the compiler cannot
 * merge it with the first computation): otherwise x, r and the valid flag stay live across
 * the whole bounce loop, and in the deep cull kernels (c5) they were what the register
 * allocator spilled to scratch — one store and one reload per lane, 12 B each. */
#ifndef RT_STORE_RECOMPUTE
#define RT_STORE_RECOMPUTE 1
#endif
__device__ __forceinline__ int lane_mbcnt() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

/* Rows of a band's tile row trow, sub-row sr (0..TILE_H-1): the frame row i it traces and
 * whether it exists, and the output row it is stored at.  A contiguous band (tstride <= 1)
 * is rows [row0, row0 + nrows), stored band-relative.  An interleaved part (KParams::tstride
 * = nparts > 1, rt_render_device_interleaved) owns the frame's tile rows tphase, tphase +
 * tstride, ...; it stores them back to back (band-relative) or, with out_frame, at their
 * frame rows. */
struct BandRow {
    int i, out;
    bool ok;
};
__device__ __forceinline__ BandRow band_row(const KParams& p, int trow, int sr) {
    const int rloc = trow * TILE_H + sr;
    BandRow b;
    if (p.tstride > 1) {
        b.i = (p.tphase + trow * p.tstride) * TILE_H + sr;
        b.ok = b.i < p.frame_h;
        b.out = p.out_frame ? b.i : rloc;
    } else {
        b.i = p.row0 + rloc;
        b.ok = rloc < p.nrows;
        b.out = rloc;
    }
    return b;
}

/* One tile per wave: tile column bx, tile row trow (after the row order), gx tile columns. */
template <int PREC, bool SUN, bool INT_EXP, bool CULL, int MAXD>
__device__ __forceinline__ void trace_tile(const KParams& p, int bx, int trow, int gx,
                                           uint64_t braw) {
#if RT_WAVE_TIMES
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = bx * TILE_W + (TILE_W > 8 ? (wave & 1) * 8 : 0) + (lane & 7);
    const BandRow br = band_row(p, trow, (TILE_H > 8 ? (wave >> 1) * 8 : 0) + (lane >> 3));
    const bool valid = x < p.W && br.ok;
    uint64_t t_tile = 0;  // the wave's start stamp (taken inside trace_pixel_*)
    const int i = br.i;
    int segs = 0;
    // every lane runs the (converged) bounce loop; only valid lanes trace and store
    // the store's coordinates (see RT_STORE_RECOMPUTE)
    auto store = [&](double cr, double cg, double cb) __attribute__((always_inline)) {
        if (RT_STORE_RECOMPUTE && CULL && BLOCK == 64) {  // (linear kernels: no spill, A/B +1..12%)
            const int l2 = lane_mbcnt();
            const int xs = bx * TILE_W + (l2 & 7);
            const BandRow bs = band_row(p, trow, l2 >> 3);
            if (xs < p.W && bs.ok) store_pixel(p, bs.out, xs, cr, cg, cb);
        } else if (valid) {
            store_pixel(p, br.out, x, cr, cg, cb);
        }
    };
    if (PREC == PREC_F32) {
        const f3 c = trace_pixel_f<SUN, CULL, MAXD>(p, x, i, valid, segs, t_tile, braw);
        store(c.x, c.y, c.z);
    } else {
#if RT_STAGE_TIMES
        uint64_t g_stage[8];
        STAGE(0);
        const d3 c =
            trace_pixel_d<PREC == PREC_MIXED, PREC != PREC_PATH64, SUN, INT_EXP, CULL, MAXD>(
                p, x, i, valid, segs, t_tile, braw, g_stage);
#else
        const d3 c =
            trace_pixel_d<PREC == PREC_MIXED, PREC != PREC_PATH64, SUN, INT_EXP, CULL, MAXD>(
                p, x, i, valid, segs, t_tile, braw);
#endif
        store(c.x, c.y, c.z);
#if RT_STAGE_TIMES
        STAGE(5);
        {
            int sg = segs;
            for (int off = 32; off > 0; off >>= 1) sg += __shfl_xor(sg, off, 64);
            if (p.stats != nullptr && lane == 0 && bx < gx) {
                const size_t wid = ((size_t)trow * gx + bx) * (BLOCK / 64) + wave;
                for (int q = 0; q < 6; ++q) p.stats[8 * wid + q] = g_stage[q];
                p.stats[8 * wid + 6] = (unsigned long long)sg;
                p.stats[8 * wid + 7] = g_stage[6];
            }
        }
#endif
    }
    count_segments(p, segs);
    if (RT_STAMP && lane == 0 && bx < gx) {
        // this tile's cost for the host's next tile-row order (rt_capi.cpp row feedback)
        const uint64_t c = (__builtin_amdgcn_s_memtime() - t_tile) >> 5;
        p.tile_cost[((size_t)trow * gx + bx) * (BLOCK / 64) + wave] = (uint16_t)(c < 65535 ? c : 65535);
    }
#if RT_WAVE_TIMES
    // diagnostic build: per wave {start, end, segments << 32 | CU id} (100 MHz clock)
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off, 64);
    if (p.stats != nullptr && lane == 0 && bx < gx) {
        const size_t wid = ((size_t)trow * gx + bx) * (BLOCK / 64) + wave;
        p.stats[3 * wid] = t_start;
        p.stats[3 * wid + 1] = __builtin_amdgcn_s_memrealtime();
        p.stats[3 * wid + 2] = ((unsigned long long)segs << 32) | (unsigned)__smid();
    }
#endif
}


/* One workgroup of a frame's grid (x: tile column or part of one, y: dispatch unit). */
template <int PREC, bool SUN, bool INT_EXP, bool CULL, int MAXD>
__device__ __forceinline__ void trace_grid(const KParams& p) {
    // workgroup row -> dispatch unit (a tile row, or a part of one: KParams::row_units_log2)
    // the primary pixel boxes (one per lane; wave-start load, used after ray generation)
    const uint64_t braw = (RT_EARLY_LOADS >= 2 && !CULL) ? box_load_primary(p) : 0;
    // dispatch units of the row order (tile rows or parts of them); with tile pairs the grid
    // has half as many rows
    const int n_units = RT_TILE_PAIRS
                            ? (((p.nrows + TILE_H - 1) / TILE_H) << p.row_units_log2)
                            : (int)gridDim.y;
#if RT_EARLY_LOADS >= 2
    // every kernel-argument value the wave start needs — the dispatch order's entry and ray
    // generation's scalars (main.cpp:132) — loaded in one batch with one wait
    const int j = blockIdx.y;
    const uint32_t pw = row_perm_word(p, j);
    const int rc = p.row_center, rpn = p.row_perm_n;
    {
        const double a0 = p.pos[0], a1 = p.pos[1], a2 = p.pos[2], b0 = p.tl[0], b1 = p.tl[1],
                     b2 = p.tl[2], c0 = p.dx[0], c1 = p.dx[1], c2 = p.dx[2], e0 = p.dy[0],
                     e1 = p.dy[1], e2 = p.dy[2];
        asm volatile("" ::"s"(a0), "s"(a1), "s"(a2), "s"(b0), "s"(b1), "s"(b2), "s"(c0),
                     "s"(c1), "s"(c2), "s"(e0), "s"(e1), "s"(e2), "s"(p.W), "s"(p.row0),
                     "s"(p.nbox), "s"(pw), "s"(rc), "s"(rpn), "s"(p.row_units_log2),
                     "s"(gridDim.x), "s"(gridDim.y));
    }
    const int u = tile_row_of(rc, rpn, pw, j, n_units);
#else
    const int u = tile_row(p, blockIdx.y, n_units);
#endif
    const int ul = p.row_units_log2;
    const int gx = (p.W + TILE_W - 1) / TILE_W;
#if RT_TILE_PAIRS
    // grid.y = ceil(units / 2): unit j, then unit n-1-j (none when they coincide)
    const int j1 = n_units - 1 - (int)blockIdx.y;
    const int u1 = tile_row(p, j1, n_units);
    const int bx0 = ((u & ((1 << ul) - 1)) * (int)gridDim.x) + (int)blockIdx.x;
    const int bx1 = ((u1 & ((1 << ul) - 1)) * (int)gridDim.x) + (int)blockIdx.x;
    trace_tile<PREC, SUN, INT_EXP, CULL, MAXD>(p, bx0, u >> ul, gx, braw);
    if (j1 > (int)blockIdx.y)
        trace_tile<PREC, SUN, INT_EXP, CULL, MAXD>(p, bx1, u1 >> ul, gx,
                                                   (RT_EARLY_LOADS >= 2 && !CULL) ? box_load_primary(p) : 0);
#else
    const int bx = ((u & ((1 << ul) - 1)) * (int)gridDim.x) + (int)blockIdx.x;
    // the last part of a row may be short (wave-uniform): such a wave's lanes are all
    // invalid (x >= W), so it can also run through with nothing to trace or store
    if (!RT_EARLY_LOADS && bx >= gx) return;
    trace_tile<PREC, SUN, INT_EXP, CULL, MAXD>(p, bx, u >> ul, gx, braw);
#endif
}

template <int PREC, bool SUN, bool INT_EXP, bool CULL, int MAXD>
__global__ void __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(waves_per_eu<PREC, SUN, INT_EXP, CULL, MAXD>(), 8)))
k_trace(KParams p) {
    trace_grid<PREC, SUN, INT_EXP, CULL, MAXD>(p);
}

#if !RT_STAMP
/* A batch of frames of one band in ONE launch (rt_render_device_frames with
 * RT_OPT_FRAME_BATCH): frame blockIdx.z's kernel arguments come from a device table the host
 * filled (one KParams per frame, copied in behind the previous work on the stream), the
 * same code as k_trace otherwise.  The table is addressed in the constant address space
 * (it is read-only while the kernel runs), like the kernel-argument segment: its fields
 * load through the scalar path and the pointers in it are known global — through a plain
 * pointer the compiler could not prove the table unclobbered by the kernel's own stores and
 * turned every access into a per-lane flat load.  The linear-scan kernels only (the cull
 * kernels' frames take one launch each). */
typedef __attribute__((address_space(4))) const KParams ConstKParams;
template <int PREC, bool SUN, bool INT_EXP, int MAXD>
__global__ void __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(waves_per_eu<PREC, SUN, INT_EXP, false, MAXD>(), 8)))
k_trace_tab(uint64_t tab_addr) {
    ConstKParams* tab = (ConstKParams*)tab_addr;
    trace_grid<PREC, SUN, INT_EXP, false, MAXD>(*(const KParams*)&tab[blockIdx.z]);
}
#endif

/* PATH64 linear scan, two pixels per lane (trace_pair_p64): tile pair bp of dispatch unit
 * u covers tile columns 2bp and 2bp + 1 of its tile row. */
#ifndef RT_WPE_PAIR
#define RT_WPE_PAIR 3
#endif
#if RT_WAVES_PER_BLOCK == 1 && !RT_TILE_PAIRS && !RT_AB_SLIM  // one-wave 8x8 tiles only (see launch_trace_ns)
template <bool SUN, int MAXD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RT_WPE_PAIR, 8)))
k_trace_pair(KParams p) {
    static_assert(BLOCK == 64 && TILE_W == 8 && TILE_H == 8, "one 8x8 tile pair per wave");
    const int u = tile_row(p, blockIdx.y, (int)gridDim.y);
    const int ul = p.row_units_log2;
    const int gx = (p.W + TILE_W - 1) / TILE_W;
    const int bx = 2 * (((u & ((1 << ul) - 1)) * (int)gridDim.x) + (int)blockIdx.x);
    const int trow = u >> ul;
    const int lane = threadIdx.x & 63;
    const int x = bx * TILE_W + (lane & 7);
    const int r = trow * TILE_H + (lane >> 3);
    const bool va = x < p.W && r < p.nrows, vb = x + 8 < p.W && r < p.nrows;
    const int i = p.row0 + r;
    int segs = 0;
    uint64_t t_tile = 0;
    f3 ca, cb;
    trace_pair_p64<SUN, MAXD>(p, x, i, va, vb, segs, t_tile, ca, cb);
    if (va) store_pixel(p, r, x, ca.x, ca.y, ca.z);
    if (vb) store_pixel(p, r, x + 8, cb.x, cb.y, cb.z);
    count_segments(p, segs);
    if (RT_STAMP && lane == 0) {
        // both tiles get the pair's cost (the host's row order reads per-tile costs)
        const uint64_t c = (__builtin_amdgcn_s_memtime() - t_tile) >> 5;
        const uint16_t c16 = (uint16_t)(c < 65535 ? c : 65535);
        if (bx < gx) p.tile_cost[(size_t)trow * gx + bx] = c16;
        if (bx + 1 < gx) p.tile_cost[(size_t)trow * gx + bx + 1] = c16;
    }
}
template <bool SUN>
static hipError_t launch_pair(const KParams& p, dim3 grid, hipStream_t st, hipEvent_t done) {
    auto go = [&](auto kern) {
        if (done)
            hipExtLaunchKernelGGL(kern, grid, dim3(64), 0, st, nullptr, done, 0, p);
        else
            hipLaunchKernelGGL(kern, grid, dim3(64), 0, st, p);
    };
    if (p.depth <= MAXD_SMALL)
        go(k_trace_pair<SUN, MAXD_SMALL>);
    else if (p.depth <= MAXD_MID)
        go(k_trace_pair<SUN, MAXD_MID>);
    else if (p.depth <= MAXD_REF)
        go(k_trace_pair<SUN, MAXD_REF>);
    else
        go(k_trace_pair<SUN, MAXD_LARGE>);
    return hipGetLastError();
}
#endif  // RT_WAVES_PER_BLOCK == 1 && !RT_TILE_PAIRS

template <int PREC, bool SUN, bool INT_EXP, bool CULL, int MAXD>
static void launch_one(const KParams& p, dim3 grid, hipStream_t st, hipEvent_t done,
                       const KParams* tab) {
#if !RT_STAMP
    if constexpr (!CULL) {
        if (tab) {  // grid.z frames, their arguments in the device table
            hipExtLaunchKernelGGL((k_trace_tab<PREC, SUN, INT_EXP, MAXD>), grid, dim3(BLOCK), 0, st,
                                  nullptr, done, 0, (uint64_t)(uintptr_t)tab);
            return;
        }
    }
#endif
    if (done)
        hipExtLaunchKernelGGL((k_trace<PREC, SUN, INT_EXP, CULL, MAXD>), grid, dim3(BLOCK), 0, st,
                              nullptr, done, 0, p);
    else
        hipLaunchKernelGGL((k_trace<PREC, SUN, INT_EXP, CULL, MAXD>), grid, dim3(BLOCK), 0, st, p);
}
template <int PREC, bool SUN, bool INT_EXP, bool CULL>
static hipError_t launch_depth(const KParams& p, dim3 grid, hipStream_t st, hipEvent_t done,
                               const KParams* tab) {
    if constexpr (RT_AB_SLIM && (PREC != PREC_PATH64 || SUN)) {
        return hipErrorInvalidValue;
    } else if constexpr (RT_AB_SLIM) {
        if (p.depth <= MAXD_SMALL)
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_SMALL>(p, grid, st, done, tab);
        else if (p.depth <= MAXD_MID)
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_MID>(p, grid, st, done, tab);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    } else {
        if (p.depth <= MAXD_SMALL)
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_SMALL>(p, grid, st, done, tab);
        else if (p.depth <= MAXD_MID)
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_MID>(p, grid, st, done, tab);
        else if (p.depth <= MAXD_REF)
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_REF>(p, grid, st, done, tab);
        else
            launch_one<PREC, SUN, INT_EXP, CULL, MAXD_LARGE>(p, grid, st, done, tab);
        return hipGetLastError();
    }
}
template <int PREC, bool SUN, bool INT_EXP>
static hipError_t launch_cull(const KParams& p, dim3 grid, hipStream_t st, hipEvent_t done,
                              const KParams* tab) {
    if (tab && p.wave_cull) return hipErrorNotSupported;  // no table kernels for the cull path
    return p.wave_cull ? launch_depth<PREC, SUN, INT_EXP, true>(p, grid, st, done, tab)
                       : launch_depth<PREC, SUN, INT_EXP, false>(p, grid, st, done, tab);
}
template <int PREC>
static hipError_t launch_prec(const KParams& p, dim3 grid, hipStream_t st, hipEvent_t done,
                              const KParams* tab = nullptr) {
    if constexpr (PREC == PREC_F64 || PREC == PREC_MIXED) {
        if (p.flags & FLAG_SUN)
            return p.int_exp ? launch_cull<PREC, true, true>(p, grid, st, done, tab)
                             : launch_cull<PREC, true, false>(p, grid, st, done, tab);
        return p.int_exp ? launch_cull<PREC, false, true>(p, grid, st, done, tab)
                         : launch_cull<PREC, false, false>(p, grid, st, done, tab);
    } else {
        return (p.flags & FLAG_SUN) ? launch_cull<PREC, true, true>(p, grid, st, done, tab)
                                    : launch_cull<PREC, false, true>(p, grid, st, done, tab);
    }
}

int max_depth_ns() { return MAXD_LARGE; }

#if RT_DIAG && !RT_STAMP
extern "C" int rt_diag_read(unsigned long long* out16) {
    const int e = (int)hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_diag), sizeof g_diag);
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof z);
    return e;
}
#endif

int launch_trace_ns(const KParams& p, int prec, void* stream, void* done_event,
                    const KParams* d_tab = nullptr, int nframes = 1) {
    if (p.W <= 0 || p.nrows <= 0) return (int)hipSuccess;
    const int ul = p.row_units_log2;
    const int units = ((p.nrows + TILE_H - 1) / TILE_H) << ul;
    const dim3 grid((((p.W + TILE_W - 1) / TILE_W) + (1 << ul) - 1) >> ul,
                    RT_TILE_PAIRS ? (units + 1) / 2 : units, d_tab ? nframes : 1);
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipEvent_t done = static_cast<hipEvent_t>(done_event);
    if (d_tab) {  // a batch of frames: the table kernels (linear scan, one pixel per lane)
        if (RT_TILE_PAIRS || p.wave_cull || p.pairs) return (int)hipErrorNotSupported;
        switch (prec) {
            case PREC_F64: return (int)launch_prec<PREC_F64>(p, grid, st, done, d_tab);
            case PREC_F32: return (int)launch_prec<PREC_F32>(p, grid, st, done, d_tab);
            case PREC_MIXED: return (int)launch_prec<PREC_MIXED>(p, grid, st, done, d_tab);
            case PREC_PATH64: return (int)launch_prec<PREC_PATH64>(p, grid, st, done, d_tab);
            default: return (int)hipErrorInvalidValue;
        }
    }
    // two pixels per lane exist only in one-wave (8x8 tile) builds: the pair kernel is not
    // instantiated for RT_WAVES_PER_BLOCK > 1 or RT_TILE_PAIRS (RT_OPT_PIXEL_PAIRS ignored)
#if RT_WAVES_PER_BLOCK == 1 && !RT_TILE_PAIRS && !RT_AB_SLIM
    if (p.pairs && prec == PREC_PATH64 && !p.wave_cull) {
        // 16x8 pixels per wave: half the tile columns per dispatch unit
        const int gxp = (((p.W + TILE_W - 1) / TILE_W) + 1) >> 1;
        const dim3 gp((gxp + (1 << ul) - 1) >> ul, units);
        return (int)((p.flags & FLAG_SUN) ? launch_pair<true>(p, gp, st, done)
                                          : launch_pair<false>(p, gp, st, done));
    }
#endif
    switch (prec) {
        case PREC_F64: return (int)launch_prec<PREC_F64>(p, grid, st, done);
        case PREC_F32: return (int)launch_prec<PREC_F32>(p, grid, st, done);
        case PREC_MIXED: return (int)launch_prec<PREC_MIXED>(p, grid, st, done);
        case PREC_PATH64: return (int)launch_prec<PREC_PATH64>(p, grid, st, done);
        default: return (int)hipErrorInvalidValue;
    }
}

#if !RT_STAMP
/* ------------------------------------------------------------------------ */
/* self-test of the exact helpers (rt_selftest)                              */
/* ------------------------------------------------------------------------ */
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
/* random doubles spanning the magnitudes the kernel divides: 2^-40 .. 2^40, both signs */
__device__ __forceinline__ double rnd_double(uint64_t bits) {
    const uint64_t mant = bits & 0xFFFFFFFFFFFFFull;
    const uint64_t ex = 1023 - 40 + ((bits >> 52) % 81);
    const uint64_t sign = (bits >> 63) << 63;
    return __longlong_as_double((long long)(sign | (ex << 52) | mant));
}

__global__ void k_selftest(int which, uint64_t n, uint64_t seed, unsigned long long* bad) {
    unsigned long long nbad = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t z0 = mix64(seed + 3 * i), z1 = mix64(seed + 3 * i + 1);
        if (which == 0) {
            const double a = rnd_double(z0), b = rnd_double(z1);
            const double q = div_r(a, b, rcp_refined(b));
            if (__double_as_longlong(q) != __double_as_longlong(a / b)) ++nbad;
            // the normalisation pattern: component / sqrt(sum of squares)
            const double c = rnd_double(mix64(seed + 3 * i + 2));
            const double l = sqrt(a * a + b * b + c * c);
            const double q2 = div_r(c, l, rcp_refined(l));
            if (__double_as_longlong(q2) != __double_as_longlong(c / l)) ++nbad;
        } else if (which == 2) {
            const double a = fabs(rnd_double(z0));
            if (__double_as_longlong(sqrt_e(a)) != __double_as_longlong(sqrt(a))) ++nbad;
            const double b = (double)(z1 >> 11) * (1.0 / 9007199254740992.0);  // [0,1)
            if (__double_as_longlong(sqrt_e(b)) != __double_as_longlong(sqrt(b))) ++nbad;
            // the scaled range: subnormals and tiny normals up to 2^-700, and 0 / inf
            const uint64_t z2 = mix64(seed + 3 * i + 2);
            const uint64_t ex = z2 % 324;  // biased exponent 0 (subnormal) .. 323
            const double c = __longlong_as_double((long long)((ex << 52) | (z1 & 0xFFFFFFFFFFFFFull)));
            if (__double_as_longlong(sqrt_e(c)) != __double_as_longlong(sqrt(c))) ++nbad;
            if (i == 0) {
                const double sp[3] = {0.0, -0.0, __builtin_inf()};
                for (int k = 0; k < 3; ++k)
                    if (__double_as_longlong(sqrt_e(sp[k])) != __double_as_longlong(sqrt(sp[k]))) ++nbad;
            }
        } else {
            const double x = (double)(z0 >> 11) * (1.0 / 9007199254740992.0);  // [0,1)
            const double e = (double)(1 + (z1 % 64));
            const double ref = pow(x, e), got = pow_int(x, (int)e);
            // squaring compounds rounding: x^64 carries up to ~63u
            const double tol = 128.0 * 2.220446049250313e-16 * fabs(ref) + 1e-300;
            if (fabs(got - ref) > tol) ++nbad;
        }
    }
    for (int off = 32; off > 0; off >>= 1) nbad += __shfl_xor(nbad, off, 64);
    if ((threadIdx.x & 63) == 0 && nbad) atomicAdd(bad, nbad);
}

int launch_selftest_ns(int which, uint64_t n, uint64_t seed, unsigned long long* d_bad,
                       void* stream) {
    hipLaunchKernelGGL(k_selftest, dim3(1024), dim3(256), 0, static_cast<hipStream_t>(stream),
                       which, n, seed, d_bad);
    return (int)hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* row feedback: per dispatch unit, the most expensive wave of a sampled frame */
/* ------------------------------------------------------------------------ */
/* One wave per tile row: unit (r << ul) + q covers waves [q*U, min(gx, q*U + U)) of row r
 * (gx waves per row, U = ceil(gx / 2^ul)), the same split as the kernel's dispatch units.
 * The host then reads nu words instead of every wave's cost (rt_capi.cpp order_units). */
__global__ void __launch_bounds__(64) k_unit_max(const uint16_t* __restrict__ cost, int gy, int gx,
                                                 int ul, uint32_t* __restrict__ umax) {
    const int r = blockIdx.x;
    if (r >= gy) return;
    const int upr = 1 << ul, U = (gx + upr - 1) >> ul;
    for (int q = 0; q < upr; q++) {
        const int x0 = q * U, x1 = min(gx, x0 + U);
        uint32_t m = 0;
        for (int x = x0 + (int)threadIdx.x; x < x1; x += 64) m = max(m, (uint32_t)cost[(size_t)r * gx + x]);
        for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        if (threadIdx.x == 0) umax[(r << ul) + q] = m;
    }
}

int launch_unit_max_ns(const uint16_t* cost, int gy, int gx, int ul, uint32_t* umax, void* stream) {
    if (gy <= 0 || gx <= 0) return (int)hipSuccess;
    hipLaunchKernelGGL(k_unit_max, dim3(gy), dim3(64), 0, static_cast<hipStream_t>(stream), cost, gy,
                       gx, ul, umax);
    return (int)hipGetLastError();
}
#endif  // !RT_STAMP

}  // namespace kno / kst

#if RT_STAMP
int launch_trace_stamped(const KParams& p, int prec, void* stream, void* done_event) {
    return kst::launch_trace_ns(p, prec, stream, done_event);
}
#else
int launch_trace_stamped(const KParams& p, int prec, void* stream, void* done_event);  // rt_trace_stamp.hip
int launch_trace(const KParams& p, int prec, void* stream, void* done_event) {
    return p.tile_cost != nullptr ? launch_trace_stamped(p, prec, stream, done_event)
                                  : kno::launch_trace_ns(p, prec, stream, done_event);
}
int max_depth() { return kno::max_depth_ns(); }
int launch_trace_batch(const KParams* d_tab, const KParams& p0, int nframes, int prec, void* stream,
                       void* done_event) {
    if (nframes <= 0) return (int)hipSuccess;
    return kno::launch_trace_ns(p0, prec, stream, done_event, d_tab, nframes);
}
int launch_selftest(int which, uint64_t n, uint64_t seed, unsigned long long* d_bad,
                    void* stream) {
    return kno::launch_selftest_ns(which, n, seed, d_bad, stream);
}
int launch_unit_max(const uint16_t* cost, int gy, int gx, int ul, uint32_t* umax, void* stream) {
    return kno::launch_unit_max_ns(cost, gy, gx, ul, umax, stream);
}
#endif

}  // namespace rt
