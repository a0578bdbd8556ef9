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
 *   PREC_F64   every operation in fp64, in the reference's order; this TU is built with
 *              -ffp-contract=off so nothing is fused (x86-64 reference codegen has no FMA).
 *              The output matches the reference's fp64 frame up to libm's last-bit
 *              differences in pow (OCML vs glibc).
 *   PREC_F32   fp32 with fused multiply-adds and hardware rcp/rsq/exp/log: the
 *              throughput path; flips at geometric discontinuities.
 *   PREC_MIXED fp32 conservative cull in the primitive scan, fp64 exact on every
 *              primitive the cull cannot reject, fp64 shading: output identical to F64.
 *
 * Recursion -> iteration with identical rounding: the reference returns
 * lerp(local, traced, metallic) from the innermost bounce outward (vec.cpp:45-49).
 * Each bounce pushes (shading scalar s, sun scalar, scene index) onto a per-thread
 * register stack indexed by the wave-uniform bounce counter, and the stack is unwound
 * in reverse with the same operations, so local = color*s is recomputed bit-identically.
 *
 * Launch: 256-thread workgroups, 16x16 pixel tiles, each wave an 8x8 square (ray
 * coherence: all 64 lanes test one primitive per iteration, its record read with
 * scalar loads; a primitive no lane can hit costs the wave a skipped branch).
 */
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include "rt_device.h"

namespace rt {

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
__device__ __forceinline__ d3 operator/(d3 a, double s) { return D3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double lensq(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ d3 normalize(d3 a) { return a / sqrt(lensq(a)); }
__device__ __forceinline__ d3 lerp(d3 a, d3 b, double t) {
    return D3(a.x + t * (b.x - a.x), a.y + t * (b.y - a.y), a.z + t * (b.z - a.z));
}
__device__ __forceinline__ d3 ld3(const double* p) { return D3(p[0], p[1], p[2]); }

/* fp32 vector math (throughput path) */
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
__device__ __forceinline__ f3 fnormalize(f3 a) { return a * frsq(fdot(a, a)); }
__device__ __forceinline__ f3 fmad3(f3 a, float s, f3 b) {  // a*s + b
    return F3(fmaf(a.x, s, b.x), fmaf(a.y, s, b.y), fmaf(a.z, s, b.z));
}
__device__ __forceinline__ f3 ld3f(const float* p) { return F3(p[0], p[1], p[2]); }
/* x^e for x >= 0 via v_log_f32 / v_exp_f32 (pow(0,e>0) = 0, pow(x,0) = 1). */
__device__ __forceinline__ float fpow(float x, float e) {
    if (e == 0.0f) return 1.0f;
    return __builtin_amdgcn_exp2f(e * __builtin_amdgcn_logf(x));
}

/* main.cpp:14-19 */
#define LIGHT_X 0.0
#define LIGHT_Y 0.0
#define LIGHT_Z 0.0
__device__ __forceinline__ d3 ground_color() { return D3(0.025, 0.05, 0.075); }
__device__ __forceinline__ d3 sky_low() { return D3(0.36, 0.45, 0.57); }
__device__ __forceinline__ d3 sky_high() { return D3(0.14, 0.21, 0.49); }
__device__ __forceinline__ d3 sun_color() { return D3(1.64, 1.27, 0.99); }
__device__ __forceinline__ d3 sun_direction() { return D3(.7, .4, .7); }

/* Largest bounce count compiled: the stack is sized per instantiation. */
constexpr int MAXD_SMALL = 4;
constexpr int MAXD_MID = 8;
constexpr int MAXD_LARGE = 16;

/* ------------------------------------------------------------------------ */
/* fp64 closest hit (find_closest_hit, main.cpp:67-84)                       */
/* ------------------------------------------------------------------------ */
struct HitD {
    double dist;  // the value find_closest_hit compares (sphere: world, wall: parametric)
    double pt;    // sphere: the parameter of the intersection point used for the normal
    int j;        // scene index, -1 = miss
    int slot;     // index into the sphere or wall array
    bool sphere;
};

/* Accept rule of main.cpp:77 in an order-independent form: the reference's strict
 * `0 < d < best` scan in scene order returns the lowest j among the minimum d, so any
 * visiting order gives the same winner with ties broken on j. */
__device__ __forceinline__ bool better(double dist, int j, const HitD& h) {
    return dist > 0 && (dist < h.dist || (dist == h.dist && j < h.j));
}

/* Sphere::intersect (scene.cpp:40-78), exact.  Only the branches that can produce an
 * accepted distance are evaluated; every skip is exact:
 *   det < 0                 -> miss (scene.cpp:57)
 *   b > 0                   -> proj = (-b - sqrt(det)) / (2a) < 0, rejected by d > 0
 *   -b - sqrt(det) <= 0     -> proj <= 0 (or NaN), rejected
 * and p1 is never the minimum: (-b+sq)/(2a) >= (-b-sq)/(2a) by monotonic rounding. */
__device__ __forceinline__ void sphere_test_d(const DevSphere& S, const d3 o, const d3 d,
                                              const double a, const double two_a,
                                              const double four_a, const double dlen, int s,
                                              HitD& h) {
    const d3 oc = o - D3(S.c[0], S.c[1], S.c[2]);
    const double b = 2 * dot(d, oc);
    if (b > 0) return;
    const double c = lensq(oc) - S.r2;
    const double det = b * b - four_a * c;
    if (!(det >= 0)) return;
    double proj, pt;
    if (det == 0) {
        pt = -b / two_a;
        proj = (-b - sqrt(det)) / a;  // scene.cpp:65 (/a, not /2a) kept
    } else {
        const double num = -b - sqrt(det);
        if (!(num > 0)) return;
        proj = num / two_a;
        pt = proj;
    }
    const double dist = proj * dlen;  // world distance, scene.cpp:77
    if (better(dist, S.j, h)) {
        h.dist = dist;
        h.pt = pt;
        h.j = S.j;
        h.slot = s;
        h.sphere = true;
    }
}

/* Wall::intersect (scene.cpp:4-35), exact.  t = num/denom is formed only when the
 * signs make t > 0 possible (denom == 0 or NaN can never pass the bounds check). */
__device__ __forceinline__ void wall_test_d(const DevWall& Wl, const d3 o, const d3 d, int w,
                                            HitD& h) {
    const d3 n = D3(Wl.n[0], Wl.n[1], Wl.n[2]);
    const d3 P = D3(Wl.P[0], Wl.P[1], Wl.P[2]);
    const double denom = dot(n, d);
    const double num = dot(P - o, n);
    if (!((num > 0 && denom > 0) || (num < 0 && denom < 0))) return;
    const double t = num / denom;
    if (!(t > 0)) return;
    const d3 ip = o + d * t;  // ray::at, scene.h:16
    const d3 q = ip - P;
    const double px = dot(q, D3(Wl.X[0], Wl.X[1], Wl.X[2]));
    const double py = dot(q, D3(Wl.Y[0], Wl.Y[1], Wl.Y[2]));
    if (px >= 0 && px <= Wl.len && py >= 0 && py <= Wl.wid) {
        if (better(t, Wl.j, h)) {  // parametric t compared as-is (main.cpp:77)
            h.dist = t;
            h.j = Wl.j;
            h.slot = w;
            h.sphere = false;
        }
    }
}

/* MIXED: fp32 conservative cull in front of the exact sphere test.  A sphere is skipped
 * only when the fp32 evaluation proves, with a margin covering its rounding error, that
 * the exact test would reject it (det < 0, or b > 0).  See DESIGN.md §mixed. */
struct RayF {
    f3 o, d;
    float a;      // |d|^2
    float dinf;   // max |d_i|
    float oinf;   // max |o_i|
};
constexpr float CULL_U = 1.0f / 16777216.0f;  // 2^-24
constexpr float CULL_K = 512.0f * CULL_U;     // generous multiple of the unit roundoff

__device__ __forceinline__ bool sphere_cull_f(const DevSphere& S, const RayF& r) {
    const f3 oc = r.o - F3(S.cf[0], S.cf[1], S.cf[2]);
    const float bh = fdot(r.d, oc);                // b/2
    const float c = fmaf(-S.rf, S.rf, fdot(oc, oc));
    const float det = fmaf(bh, bh, -r.a * c);       // det/4
    const float B = r.oinf + fmaxf(fmaxf(fabsf(S.cf[0]), fabsf(S.cf[1])), fabsf(S.cf[2])) + S.rf;
    const float mb = CULL_K * r.dinf * B;
    const float mdet = CULL_K * (r.a * B * B + bh * bh + r.a * fabsf(c));
    return (bh > mb) || (det < -mdet);
}

__device__ __forceinline__ bool wall_cull_f(const DevWall& Wl, const RayF& r) {
    const f3 n = ld3f(Wl.nf), P = ld3f(Wl.Pf);
    const f3 po = P - r.o;
    const float den = fdot(n, r.d);
    const float num = fdot(po, n);
    const float B = r.oinf + fmaxf(fmaxf(fabsf(P.x), fabsf(P.y)), fabsf(P.z));
    const float mnum = CULL_K * B;
    const float mden = CULL_K * r.dinf;
    if ((num < -mnum && den > mden) || (num > mnum && den < -mden)) return true;  // t < 0
    if (fabsf(num) <= 64.0f * mnum || fabsf(den) <= 64.0f * mden) return false;   // ill-conditioned
    // t's relative error <= mnum/|num| + mden/|den| (<= 1/32 here); bound the point error.
    const float t = num * frcp(den);
    const float rel = mnum / fabsf(num) + mden / fabsf(den) + 4.0f * CULL_U;
    const f3 q = fmad3(r.d, t, r.o) - P;
    const float len_dt = sqrtf(r.a) * fabsf(t);
    const float err = 2.0f * len_dt * rel + CULL_K * (B + len_dt + Wl.lenf + Wl.widf);
    const float px = fdot(q, ld3f(Wl.Xf));
    const float py = fdot(q, ld3f(Wl.Yf));
    return px < -err || px > Wl.lenf + err || py < -err || py > Wl.widf + err;
}

template <bool MIXED>
__device__ __forceinline__ HitD closest_hit_d(const KParams& p, const d3 o, const d3 d,
                                              const double a, const double dlen) {
    HitD h;
    h.dist = DBL_MAX;
    h.pt = 0;
    h.j = -1;
    h.slot = 0;
    h.sphere = false;
    const double two_a = 2 * a, four_a = 4 * a;
    RayF rf;
    if (MIXED) {
        rf.o = F3((float)o.x, (float)o.y, (float)o.z);
        rf.d = F3((float)d.x, (float)d.y, (float)d.z);
        rf.a = fdot(rf.d, rf.d);
        rf.dinf = fmaxf(fmaxf(fabsf(rf.d.x), fabsf(rf.d.y)), fabsf(rf.d.z));
        rf.oinf = fmaxf(fmaxf(fabsf(rf.o.x), fabsf(rf.o.y)), fabsf(rf.o.z));
    }
    for (int s = 0; s < p.nS; ++s) {
        const DevSphere& S = p.sph[s];
        if (MIXED && sphere_cull_f(S, rf)) continue;
        sphere_test_d(S, o, d, a, two_a, four_a, dlen, s, h);
    }
    for (int w = 0; w < p.nW; ++w) {
        const DevWall& Wl = p.wal[w];
        if (MIXED && wall_cull_f(Wl, rf)) continue;
        wall_test_d(Wl, o, d, w, h);
    }
    return h;
}

/* out_color, main.cpp:28-37 (float skyGradient 0.25f promoted to double). */
__device__ __forceinline__ d3 out_color_d(d3 v) {
    if (v.z < 0.0) return ground_color();
    v = normalize(v);
    return lerp(sky_low(), sky_high(), pow(v.z, (double)0.25f));
}

/* Shading of one hit (main.cpp:99-104 + diffuse_shading + specular), returning
 * s = diffuse*kd + spec*ks + ka (local = color * s), the unit normal and the
 * (optional) sun scalar.  Shared normalisations are computed once: they are the same
 * operations on the same operands as the reference's repeated calls. */
struct ShadeD {
    double s;
    double ksun;
};
__device__ __forceinline__ ShadeD shade_d(const DevMat& m, const d3 pos, const d3 N, const d3 view,
                                          bool sun) {
    const d3 lv = D3(LIGHT_X - pos.x, LIGHT_Y - pos.y, LIGHT_Z - pos.z);
    const d3 ldir = normalize(lv);
    const d3 nn = normalize(N);
    const double lamb = dot(ldir, nn);
    const double diffuse = lamb > 0 ? lamb : 0;
    const d3 halfway = normalize(view + ldir);
    double res = dot(halfway, nn);
    res = res > 0 ? res : 0;
    const double spec = pow(res, m.ex);
    ShadeD r;
    r.s = diffuse * m.kd + spec * m.ks + m.ka;
    r.ksun = 0;
    if (sun) {  // build-defined (rt_oracle.c sun_term)
        const d3 sd = normalize(sun_direction());
        double a = dot(sd, nn);
        a = a > 0 ? a : 0;
        double hs = dot(normalize(view + sd), nn);
        hs = hs > 0 ? hs : 0;
        r.ksun = a * m.kd + pow(hs, m.ex) * m.ks;
    }
    return r;
}

/* local = color * s (+ (SUN_COLOR * color) * ksun) — identical operations at push
 * and at unwind. */
__device__ __forceinline__ d3 local_color_d(const DevMat& m, double s, double ksun, bool sun) {
    const d3 col = ld3(m.color);
    d3 L = col * s;
    if (sun) L = L + (sun_color() * col) * ksun;
    return L;
}

template <bool MIXED, int MAXD>
__device__ __forceinline__ d3 trace_pixel_d(const KParams& p, int x, int i, int& segs) {
    const d3 cpos = ld3(p.pos);
    const d3 pc = (ld3(p.tl) + ld3(p.dx) * (double)x) + ld3(p.dy) * (double)i;  // main.cpp:132
    d3 o = cpos;
    d3 d = cpos - pc;  // main.cpp:133 (not normalised)
    const bool sun = (p.flags & FLAG_SUN) != 0;

    double st_s[MAXD];
    double st_k[MAXD];
    int st_j[MAXD];
    int n = 0;
    d3 c;
    for (int k = 0;; ++k) {
        ++segs;
        const double a = lensq(d);
        const double dlen = sqrt(a);
        const HitD h = closest_hit_d<MIXED>(p, o, d, a, dlen);
        if (h.j < 0) {
            c = out_color_d(d);
            break;
        }
        const d3 pos = o + d * h.dist;  // main.cpp:99 (sphere world distance used as t)
        d3 N;
        if (h.sphere) {
            const DevSphere& S = p.sph[h.slot];
            N = (o + d * h.pt) - D3(S.c[0], S.c[1], S.c[2]);  // un-normalised, length r
        } else {
            const DevWall& Wl = p.wal[h.slot];
            N = D3(Wl.n[0], Wl.n[1], Wl.n[2]);
        }
        const DevMat& m = p.mat[h.j];
        const d3 nv = d / dlen;  // normalize(d) == -normalize(-d) bit for bit
        const ShadeD sh = shade_d(m, pos, N, -nv, sun);
        if (k >= p.depth || k >= MAXD) {  // remaining_iterations <= 0 (main.cpp:105)
            c = local_color_d(m, sh.s, sh.ksun, sun);
            break;
        }
        st_s[k] = sh.s;
        st_k[k] = sh.ksun;
        st_j[k] = h.j;
        n = k + 1;
        // reflect(d, N) (vec.cpp:51-57) and the offset start (main.cpp:111-113)
        const d3 nn = normalize(N);
        const double cc = 2 * dot(nv, nn);
        o = pos + N * .0001;
        d = nv - nn * cc;
    }
    for (int q = MAXD - 1; q >= 0; --q) {
        if (q < n) {
            const DevMat& m = p.mat[st_j[q]];
            const d3 L = local_color_d(m, st_s[q], st_k[q], sun);
            c = lerp(L, c, m.km);  // vec.cpp:45-49 via main.cpp:117
        }
    }
    return c;
}

/* ------------------------------------------------------------------------ */
/* fp32 throughput path                                                      */
/* ------------------------------------------------------------------------ */
struct HitF {
    float dist, pt;
    int j, slot;
    bool sphere;
};

template <int MAXD>
__device__ __forceinline__ f3 trace_pixel_f(const KParams& p, int x, int i, int& segs) {
    const f3 cpos = F3((float)p.pos[0], (float)p.pos[1], (float)p.pos[2]);
    // ray generation in fp64 (cheap, once per pixel) then rounded
    const d3 pcd = (ld3(p.tl) + ld3(p.dx) * (double)x) + ld3(p.dy) * (double)i;
    const d3 dd = ld3(p.pos) - pcd;
    f3 o = cpos;
    f3 d = F3((float)dd.x, (float)dd.y, (float)dd.z);
    const bool sun = (p.flags & FLAG_SUN) != 0;

    float st_s[MAXD];
    float st_k[MAXD];
    int st_j[MAXD];
    int n = 0;
    f3 c;
    for (int k = 0;; ++k) {
        ++segs;
        const float a = fdot(d, d);
        const float inv_a = frcp(a);
        const float dlen = sqrtf(a);
        HitF h;
        h.dist = FLT_MAX;
        h.pt = 0;
        h.j = -1;
        h.slot = 0;
        h.sphere = false;
        for (int s = 0; s < p.nS; ++s) {
            const DevSphere& S = p.sph[s];
            const f3 oc = o - ld3f(S.cf);
            const float bh = fdot(d, oc);
            if (bh > 0) continue;
            const float cq = fdot(oc, oc) - S.r2f;
            const float det = fmaf(bh, bh, -a * cq);
            if (!(det >= 0)) continue;
            float proj, pt;
            if (det == 0) {
                pt = -bh * inv_a;
                proj = 2.0f * pt;  // scene.cpp:65 quirk: -b/a = 2 * (-b/2a)
            } else {
                const float num = -bh - sqrtf(det);
                if (!(num > 0)) continue;
                proj = num * inv_a;
                pt = proj;
            }
            const float dist = proj * dlen;
            if (dist > 0 && (dist < h.dist || (dist == h.dist && S.j < h.j))) {
                h.dist = dist; h.pt = pt; h.j = S.j; h.slot = s; h.sphere = true;
            }
        }
        for (int w = 0; w < p.nW; ++w) {
            const DevWall& Wl = p.wal[w];
            const f3 nw = ld3f(Wl.nf), P = ld3f(Wl.Pf);
            const float den = fdot(nw, d);
            const float num = fdot(P - o, nw);
            if (!((num > 0 && den > 0) || (num < 0 && den < 0))) continue;
            const float t = num / den;
            if (!(t > 0)) continue;
            const f3 q = fmad3(d, t, o) - P;
            const float px = fdot(q, ld3f(Wl.Xf));
            const float py = fdot(q, ld3f(Wl.Yf));
            if (px >= 0 && px <= Wl.lenf && py >= 0 && py <= Wl.widf &&
                (t < h.dist || (t == h.dist && Wl.j < h.j))) {
                h.dist = t; h.j = Wl.j; h.slot = w; h.sphere = false;
            }
        }
        if (h.j < 0) {
            if (d.z < 0.0f) {
                c = F3(0.025f, 0.05f, 0.075f);
            } else {
                const float z = d.z * frsq(a);
                const float tz = sqrtf(sqrtf(z));
                c = F3(fmaf(tz, 0.14f - 0.36f, 0.36f), fmaf(tz, 0.21f - 0.45f, 0.45f),
                       fmaf(tz, 0.49f - 0.57f, 0.57f));
            }
            break;
        }
        const f3 pos = fmad3(d, h.dist, o);
        f3 N;
        if (h.sphere) {
            N = fmad3(d, h.pt, o) - ld3f(p.sph[h.slot].cf);
        } else {
            N = ld3f(p.wal[h.slot].nf);
        }
        const DevMat& m = p.mat[h.j];
        const float kd = (float)m.kd, ks = (float)m.ks, ka = (float)m.ka, ex = (float)m.ex;
        const f3 nv = d * frsq(a);
        const f3 nn = fnormalize(N);
        const f3 ldir = fnormalize(-pos);
        const float lamb = fmaxf(fdot(ldir, nn), 0.0f);
        const float res = fmaxf(fdot(fnormalize(ldir - nv), nn), 0.0f);
        float s = fmaf(lamb, kd, fmaf(fpow(res, ex), ks, ka));
        float ksun = 0.0f;
        if (sun) {
            const f3 sd = fnormalize(F3(.7f, .4f, .7f));
            const float sa = fmaxf(fdot(sd, nn), 0.0f);
            const float hs = fmaxf(fdot(fnormalize(sd - nv), nn), 0.0f);
            ksun = fmaf(sa, kd, fpow(hs, ex) * ks);
        }
        if (k >= p.depth || k >= MAXD) {
            const f3 col = F3((float)m.color[0], (float)m.color[1], (float)m.color[2]);
            c = col * s;
            if (sun) c = fmad3(F3(1.64f * col.x, 1.27f * col.y, 0.99f * col.z), ksun, c);
            break;
        }
        st_s[k] = s;
        st_k[k] = ksun;
        st_j[k] = h.j;
        n = k + 1;
        const float cc = 2.0f * fdot(nv, nn);
        o = fmad3(N, 1e-4f, pos);
        d = fmad3(nn, -cc, nv);
    }
    for (int q = MAXD - 1; q >= 0; --q) {
        if (q < n) {
            const DevMat& m = p.mat[st_j[q]];
            const f3 col = F3((float)m.color[0], (float)m.color[1], (float)m.color[2]);
            f3 L = col * st_s[q];
            if (sun) L = fmad3(F3(1.64f * col.x, 1.27f * col.y, 0.99f * col.z), st_k[q], L);
            const float km = (float)m.km;
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

__device__ __forceinline__ void store_pixel(const KParams& p, int r, int x, double cr, double cg,
                                            double cb) {
    const size_t px = (size_t)r * (size_t)p.W + (size_t)x;
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
    } else {
        const unsigned v = q8(cr) | (q8(cg) << 8) | (q8(cb) << 16) | (255u << 24);
        static_cast<unsigned*>(p.out)[px] = v;
    }
}

__device__ __forceinline__ void count_segments(const KParams& p, int segs) {
    if (p.segs == nullptr) return;
    // wave reduction (64 lanes), one atomic per wave
    for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(p.segs, (unsigned long long)segs);
}

template <int PREC, int MAXD>
__global__ void __launch_bounds__(BLOCK) k_trace(KParams p) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * TILE_W + (wave & 1) * 8 + (lane & 7);
    const int r = blockIdx.y * TILE_H + (wave >> 1) * 8 + (lane >> 3);
    const bool valid = x < p.W && r < p.nrows;
    int segs = 0;
    if (valid) {
        const int i = p.row0 + r;
        if (PREC == PREC_F32) {
            const f3 c = trace_pixel_f<MAXD>(p, x, i, segs);
            store_pixel(p, r, x, c.x, c.y, c.z);
        } else {
            const d3 c = trace_pixel_d<PREC == PREC_MIXED, MAXD>(p, x, i, segs);
            store_pixel(p, r, x, c.x, c.y, c.z);
        }
    }
    count_segments(p, segs);
}

template <int PREC>
static hipError_t launch_prec(const KParams& p, dim3 grid, hipStream_t st) {
    if (p.depth <= MAXD_SMALL)
        hipLaunchKernelGGL((k_trace<PREC, MAXD_SMALL>), grid, dim3(BLOCK), 0, st, p);
    else if (p.depth <= MAXD_MID)
        hipLaunchKernelGGL((k_trace<PREC, MAXD_MID>), grid, dim3(BLOCK), 0, st, p);
    else
        hipLaunchKernelGGL((k_trace<PREC, MAXD_LARGE>), grid, dim3(BLOCK), 0, st, p);
    return hipGetLastError();
}

int max_depth() { return MAXD_LARGE; }

int launch_trace(const KParams& p, int prec, void* stream) {
    if (p.W <= 0 || p.nrows <= 0) return (int)hipSuccess;
    const dim3 grid((p.W + TILE_W - 1) / TILE_W, (p.nrows + TILE_H - 1) / TILE_H);
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (prec) {
        case PREC_F64: return (int)launch_prec<PREC_F64>(p, grid, st);
        case PREC_F32: return (int)launch_prec<PREC_F32>(p, grid, st);
        case PREC_MIXED: return (int)launch_prec<PREC_MIXED>(p, grid, st);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace rt
