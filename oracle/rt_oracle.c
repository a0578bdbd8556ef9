/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 * fp64 restatement of the reference hot path, written to reproduce the reference's
 * rounding op-for-op: same operation order, no FMA contraction (built with
 * -ffp-contract=off), same libm calls.  Every quirk is kept on purpose; each function
 * cites the reference line it restates.  The sun term (RT_FLAG_SUN) is a
 * build-defined extension with no reference implementation (parity unpinned).
 */
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { double x, y, z; } v3;

/* vec.cpp:3-57 — every operator evaluated in the reference's order. */
static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 ld(const double* p) { return mk(p[0], p[1], p[2]); }
static inline void st(double* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline double lensq(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }  /* vec.cpp:7 */
static inline double len(v3 v) { return sqrt(lensq(v)); }                        /* vec.cpp:3 */
static inline double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* vec.cpp:11 */
static inline v3 cross(v3 u, v3 v) {                                              /* vec.cpp:15 */
    return mk(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, double d) { return mk(a.x * d, a.y * d, a.z * d); }
static inline v3 divs(v3 a, double t) { return mk(a.x / t, a.y / t, a.z / t); }
static inline v3 normalize(v3 v) { return divs(v, len(v)); }                      /* vec.cpp:21 */
static inline v3 lerp(v3 a, v3 b, double d) {                                     /* vec.cpp:45 */
    return mk(a.x + d * (b.x - a.x), a.y + d * (b.y - a.y), a.z + d * (b.z - a.z));
}
static inline v3 reflect(v3 v, v3 n) {                                            /* vec.cpp:51 */
    v3 nn = normalize(n);
    v3 nv = normalize(v);
    double c = 2 * dot(nv, nn);
    return sub(nv, muls(nn, c));
}

/* main.cpp:14-19 */
static const v3 LIGHT_POS = {0, 0, 0};
static const v3 GROUND_COLOR = {0.025, 0.05, 0.075};
static const v3 SKY_LOW = {0.36, 0.45, 0.57};
static const v3 SKY_HIGH = {0.14, 0.21, 0.49};
static const v3 SUN_COLOR = {1.64, 1.27, 0.99};
static const v3 SUN_DIRECTION = {.7, .4, .7};

typedef struct { double distance; v3 normal; int hit; } coll;

/* Wall::intersect — scene.cpp:4-35.  Returns PARAMETRIC t; the basis (scene.cpp:18-19)
 * is NaN for normals parallel to z, so such walls never report a hit. */
static coll wall_intersect(const rt_prim* w, v3 o, v3 d) {
    v3 P = ld(w->position), n = ld(w->normal);
    double denominator = dot(n, d);
    double t = dot(sub(P, o), n) / denominator;
    if (t > 0) {
        v3 ip = add(o, muls(d, t));                       /* ray::at, scene.h:16 */
        v3 wall_right = normalize(cross(n, mk(0, 0, 1)));
        v3 wall_up = normalize(cross(wall_right, n));
        v3 q = sub(ip, P);
        double px = dot(q, wall_right);
        double py = dot(q, wall_up);
        if (px >= 0 && px <= w->length && py >= 0 && py <= w->width) {
            coll c = {t, n, 1};
            return c;
        }
    }
    coll c = {-1, {0, 0, 0}, 0};
    return c;
}

/* Sphere::intersect — scene.cpp:40-78.  Returns WORLD distance proj*|d| and the
 * un-normalised normal P-C; det==0 uses -b/a for proj (scene.cpp:65 bug kept). */
static coll sphere_intersect(const rt_prim* s, v3 o, v3 d) {
    v3 C = ld(s->position);
    double r = s->radius;
    v3 oc = sub(o, C);
    double a = lensq(d);
    double b = 2 * dot(d, oc);
    double c = lensq(oc) - r * r;
    double det = b * b - 4 * a * c;
    double proj;
    if (det < 0) {
        coll m = {-1, {0, 0, 0}, 0};
        return m;
    }
    v3 ip;
    if (det == 0) {
        ip = add(o, muls(d, (-b / (2 * a))));
        proj = (-b - sqrt(det)) / a;
    } else {
        double p1 = (-b + sqrt(det)) / (2 * a);
        double p2 = (-b - sqrt(det)) / (2 * a);
        proj = p1 < p2 ? p1 : p2;
        ip = add(o, muls(d, proj));
    }
    coll h = {proj * len(d), sub(ip, C), 1};
    return h;
}

static coll prim_intersect(const rt_prim* p, v3 o, v3 d) {
    return p->kind == RT_PRIM_SPHERE ? sphere_intersect(p, o, d) : wall_intersect(p, o, d);
}

/* find_closest_hit — main.cpp:67-84: strict 0 < d < best, scene order. */
static int closest_hit(const rt_prim* prims, int n, v3 o, v3 d, coll* out) {
    coll best = {DBL_MAX, {0, 0, 0}, 0};
    int idx = -1;
    for (int j = 0; j < n; j++) {
        coll c = prim_intersect(&prims[j], o, d);
        if (c.distance > 0 && c.distance < best.distance) {
            best = c;
            idx = j;
        }
    }
    *out = best;
    return idx;
}

/* out_color — main.cpp:28-37. skyGradient is the float 0.25 promoted to double. */
static v3 out_color(v3 v) {
    if (v.z < 0.0) return GROUND_COLOR;
    v = normalize(v);
    const float sky_gradient = 1. / 4.;
    return lerp(SKY_LOW, SKY_HIGH, pow(v.z, (double)sky_gradient));
}

/* diffuse_shading — main.cpp:42-48 */
static double diffuse_shading(v3 pos, v3 normal, v3 light_pos) {
    v3 light_dir = normalize(sub(light_pos, pos));
    double lambertian = dot(light_dir, normalize(normal));
    return lambertian > 0 ? lambertian : 0;
}

/* specular (Blinn-Phong half-vector term, before pow) — main.cpp:53-62 */
static double specular(v3 pos, v3 normal, v3 light_pos, v3 view_dir) {
    view_dir = normalize(view_dir);
    normal = normalize(normal);
    v3 light_dir = normalize(sub(light_pos, pos));
    v3 halfway = normalize(add(view_dir, light_dir));
    double result = dot(halfway, normal);
    return result > 0 ? result : 0;
}

/* Build-defined sun term (no reference implementation; parity unpinned).
 * Directional Lambert + Blinn-Phong toward s = normalize(SUN_DIRECTION), no shadows:
 *   add = SUN_COLOR * color * (max(0, s.N)*kd + pow(max(0, normalize(V+s).N), exp)*ks) */
static v3 sun_term(v3 normal, v3 view_dir, const rt_material* m) {
    v3 s = normalize(SUN_DIRECTION);
    v3 nn = normalize(normal);
    v3 vv = normalize(view_dir);
    double sd = dot(s, nn);
    sd = sd > 0 ? sd : 0;
    double sh = dot(normalize(add(vv, s)), nn);
    sh = sh > 0 ? sh : 0;
    double k = sd * m->diffuse + pow(sh, m->specular_exponent) * m->specular;
    v3 col = ld(m->color);
    return muls(mulv(SUN_COLOR, col), k);
}

/* recursive_ray_tracing — main.cpp:89-119 (recursion kept: identical rounding order). */
static v3 trace(const rt_prim* prims, int n, v3 o, v3 d, int remaining, uint32_t flags,
                uint64_t* segs, uint64_t* sig) {
    coll col;
    (*segs)++;
    int idx = closest_hit(prims, n, o, d, &col);
    *sig = *sig * 1000003ull + (uint64_t)(idx + 1);  /* path signature (tests only) */
    if (idx < 0) return out_color(d);
    v3 pos = add(o, muls(d, col.distance));
    const rt_material* mat = &prims[idx].mat;
    double diffuse_intensity = diffuse_shading(add(o, muls(d, col.distance)), col.normal, LIGHT_POS);
    double specular_intensity =
        pow(specular(pos, col.normal, LIGHT_POS, neg(d)), mat->specular_exponent);
    v3 local = muls(ld(mat->color),
                    diffuse_intensity * mat->diffuse + specular_intensity * mat->specular +
                        mat->ambient);
    if (flags & RT_FLAG_SUN) local = add(local, sun_term(col.normal, neg(d), mat));
    if (remaining <= 0) return local;
    v3 start = add(pos, muls(col.normal, .0001));
    v3 refl = reflect(d, col.normal);
    v3 rt = trace(prims, n, start, refl, remaining - 1, flags, segs, sig);
    return lerp(local, rt, mat->metallic);
}

/* ---- exported per-function restatements -------------------------------- */
void orc_sphere_intersect(const rt_prim* s, const double o[3], const double d[3], double* dist,
                          double normal[3], int* hit) {
    coll c = sphere_intersect(s, ld(o), ld(d));
    *dist = c.distance; st(normal, c.normal); *hit = c.hit;
}
void orc_wall_intersect(const rt_prim* w, const double o[3], const double d[3], double* dist,
                        double normal[3], int* hit) {
    coll c = wall_intersect(w, ld(o), ld(d));
    *dist = c.distance; st(normal, c.normal); *hit = c.hit;
}
void orc_out_color(const double v[3], double rgb[3]) { st(rgb, out_color(ld(v))); }
double orc_diffuse_shading(const double pos[3], const double normal[3], const double light[3]) {
    return diffuse_shading(ld(pos), ld(normal), ld(light));
}
double orc_specular(const double pos[3], const double normal[3], const double light[3],
                    const double view[3]) {
    return specular(ld(pos), ld(normal), ld(light), ld(view));
}
void orc_reflect(const double v[3], const double n[3], double out[3]) {
    st(out, reflect(ld(v), ld(n)));
}
int orc_find_closest_hit(const rt_prim* prims, int n, const double o[3], const double d[3],
                         double* dist, double normal[3]) {
    coll c;
    int idx = closest_hit(prims, n, ld(o), ld(d), &c);
    *dist = c.distance; st(normal, c.normal);
    return idx;
}
void orc_trace(const rt_prim* prims, int n, const double o[3], const double d[3], int depth,
               uint32_t flags, double rgb[3], uint64_t* segments) {
    uint64_t s = 0, sig = 0;
    st(rgb, trace(prims, n, ld(o), ld(d), depth, flags, &s, &sig));
    if (segments) *segments = s;
}

/* Camera::init — scene.cpp:80-106 (3.14 for pi kept; returns {dx, dy}). */
int orc_camera_init(const double position[3], const double lookat[3], const double vup[3],
                    double vfov, double aspect_ratio, double image_width, rt_camera* cam) {
    v3 pos = ld(position), look = ld(lookat), up = ld(vup);
    double image_height = (int)(image_width / aspect_ratio);
    double focal_length = len(sub(pos, look));
    double theta = vfov * 3.14 / 180.0;
    double h = tan(theta / 2);
    double fov_height = 2 * h * focal_length;
    double fov_width = fov_height * ((double)image_width / image_height);
    v3 w = normalize(sub(pos, look));
    v3 u = normalize(cross(up, w));
    v3 v = cross(w, u);
    v3 fov_x = muls(u, fov_width);
    v3 fov_y = muls(v, -fov_height);
    v3 pdx = divs(fov_x, image_width);
    v3 pdy = divs(fov_y, image_height);
    v3 fov_top_left = sub(sub(sub(pos, muls(w, focal_length)), divs(fov_x, 2)), divs(fov_y, 2));
    v3 itl = add(fov_top_left, muls(add(pdx, pdy), 0.5));
    st(cam->position, pos);
    st(cam->image_top_left, itl);
    st(cam->pixel_delta_x, pdx);
    st(cam->pixel_delta_y, pdy);
    cam->width = (int32_t)image_width;
    cam->height = (int32_t)image_height;
    return (int)image_height;
}

/* rt_scene — main.cpp:124-139, rows in parallel (the OpenMP path README.md:13 claims;
 * per-pixel arithmetic is unchanged so the frame is identical at any thread count). */
uint64_t orc_render(const rt_prim* prims, int n, const rt_camera* cam, int row0, int nrows,
                    int depth, uint32_t flags, double* out64, float* out32, uint64_t* path_sig,
                    int nthreads) {
    const int W = cam->width;
    const v3 TL = ld(cam->image_top_left), dx = ld(cam->pixel_delta_x),
             dy = ld(cam->pixel_delta_y), pos = ld(cam->position);
    uint64_t total = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : total)
#endif
    for (int r = 0; r < nrows; r++) {
        const int i = row0 + r;
        uint64_t segs = 0;
        for (int j = 0; j < W; j++) {
            v3 pixel_center = add(add(TL, muls(dx, j)), muls(dy, i));
            v3 cam_pixel = sub(pos, pixel_center);
            uint64_t sig = 0;
            v3 c = trace(prims, n, pos, cam_pixel, depth, flags, &segs, &sig);
            size_t k = ((size_t)r * W + j) * 3;
            if (path_sig) path_sig[(size_t)r * W + j] = sig;
            if (out64) { out64[k] = c.x; out64[k + 1] = c.y; out64[k + 2] = c.z; }
            if (out32) { out32[k] = (float)c.x; out32[k + 1] = (float)c.y; out32[k + 2] = (float)c.z; }
        }
        total += segs;
    }
    (void)nthreads;
    return total;
}

/* ---- scenes -------------------------------------------------------------- */
static void set_mat(rt_material* m, double r, double g, double b, double metallic) {
    /* Material(color, metallic=.5, ambient=.1, diffuse=.9, specular=.4, exp=50), scene.h:48 */
    m->color[0] = r; m->color[1] = g; m->color[2] = b;
    m->metallic = metallic; m->ambient = .1; m->diffuse = .9; m->specular = .4;
    m->specular_exponent = 50;
}

static void set_wall(rt_prim* p, v3 P, v3 raw_n, double length, double width, double* raw_out) {
    p->kind = RT_PRIM_WALL; p->reserved = 0;
    st(p->position, P);
    st(p->normal, normalize(raw_n));   /* Wall ctor normalises, scene.h:73 */
    p->radius = 0; p->length = length; p->width = width;
    if (raw_out) st(raw_out, raw_n);
}

static void set_sphere(rt_prim* p, v3 C, double r) {
    p->kind = RT_PRIM_SPHERE; p->reserved = 0;
    st(p->position, C);
    p->normal[0] = p->normal[1] = p->normal[2] = 0;
    p->radius = r; p->length = 0; p->width = 0;
}

int orc_default_scene(rt_prim* out, double* raw_normals) {
    memset(out, 0, 3 * sizeof(rt_prim));
    /* main.cpp:160 Sphere(Material(RGB(0,1,0), 0.5), (1.5,0,0), .5) */
    set_mat(&out[0].mat, 0, 1, 0, 0.5);
    set_sphere(&out[0], mk(1.5, 0, 0), .5);
    /* main.cpp:162 Wall(Material(RGB(0,0,1)), (3,2,0), (0,-1,0), 1, 1) */
    set_mat(&out[1].mat, 0, 0, 1, .5);
    set_wall(&out[1], mk(3.0, 2, 0), mk(0, -1, 0), 1, 1, raw_normals ? raw_normals : 0);
    /* main.cpp:163 Wall(Material(RGB(0,1,0)), (3,-3,0), (0,1,0), 2, 2) */
    set_mat(&out[2].mat, 0, 1, 0, .5);
    set_wall(&out[2], mk(3.0, -3, 0), mk(0, 1, 0), 2, 2, raw_normals ? raw_normals + 3 : 0);
    return 3;
}

/* SplitMix64 + U() = (next() >> 40) * 2^-24. */
static uint64_t sm_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double sm_u(uint64_t* s) { return (double)(sm_next(s) >> 40) * (1.0 / 16777216.0); }

int orc_synthetic_scene(int n_spheres, int n_walls, uint64_t seed, rt_prim* out,
                        double* raw_normals) {
    static const double WN[6][3] = {{0, -1, 0}, {0, 1, 0}, {-1, 0, 0},
                                    {-.70710678, -.70710678, 0}, {-.70710678, .70710678, 0},
                                    {1, 0, 0}};
    static const double WP[6][3] = {{3, 4, -1}, {3, -4, -1}, {10, -4, -1},
                                    {8, 3, -1}, {8, -6, -1}, {-10, -4, -1}};
    if (n_walls > 6 || n_walls < 0 || n_spheres < 0) return -1;
    uint64_t s = seed;
    int k = 0;
    memset(out, 0, (size_t)(n_spheres + n_walls) * sizeof(rt_prim));
    for (int i = 0; i < n_spheres; i++, k++) {
        double x = 2 + 6 * sm_u(&s);
        double y = -3 + 6 * sm_u(&s);
        double z = -1 + 3 * sm_u(&s);
        double r = .3 + .5 * sm_u(&s);
        double cr = sm_u(&s);
        double cg = sm_u(&s);
        double cb = sm_u(&s);
        double metallic = sm_u(&s);
        set_mat(&out[k].mat, cr, cg, cb, metallic);
        set_sphere(&out[k], mk(x, y, z), r);
    }
    for (int w = 0; w < n_walls; w++, k++) {
        double g = .2 + .6 * sm_u(&s);
        set_mat(&out[k].mat, g, g, g, .5);
        set_wall(&out[k], ld(WP[w]), ld(WN[w]), 8, 4, raw_normals ? raw_normals + 3 * w : 0);
    }
    return k;
}

/* main.cpp:345: SDL_MapRGB(surface->format, val.x * 255, val.y * 255, val.z * 255) with
 * Uint8 parameters.  The reference's x86-64 build converts with cvttsd2si (truncation to
 * int32; NaN and values outside the int32 range give INT32_MIN) and keeps the low byte:
 * in-range pixels truncate, highlights above 1.0 wrap modulo 256. */
static uint8_t surface_byte(double v) {
    const double t = v * 255;
    const int32_t i = (t > -2147483649.0 && t < 2147483648.0) ? (int32_t)t : INT32_MIN;
    return (uint8_t)((uint32_t)i & 0xffu);
}
void orc_surface_u8(const double* rgb, size_t npx, uint8_t* out) {
    for (size_t k = 0; k < 3 * npx; k++) out[k] = surface_byte(rgb[k]);
}
