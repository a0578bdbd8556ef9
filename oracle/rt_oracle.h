/*
 * rt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (fp64, plain C, OpenMP over rows) of the reference's per-pixel
 * trace/shade path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / the timed CPU baseline — never as the
 * product path (the product is ray-tracer-from-scratch_amd/, which fails loudly
 * without its HIP library).
 *
 * Parity pin: tests/test_oracle_golden.py checks this restatement bit-for-bit against
 * frames and known-answer values produced by the reference's own vec.cpp / scene.cpp /
 * main.cpp hot-path functions, compiled from /root/reference by oracle/Makefile into
 * oracle/_ref (fixtures committed under tests/golden/ by tests/golden/make_golden.py).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_capi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per-function restatements (known-answer tests). */
void orc_sphere_intersect(const rt_prim* s, const double o[3], const double d[3],
                          double* dist, double normal[3], int* hit);
void orc_wall_intersect(const rt_prim* w, const double o[3], const double d[3],
                        double* dist, double normal[3], int* hit);
void orc_out_color(const double v[3], double rgb[3]);
double orc_diffuse_shading(const double pos[3], const double normal[3], const double light[3]);
double orc_specular(const double pos[3], const double normal[3], const double light[3],
                    const double view[3]);
void orc_reflect(const double v[3], const double n[3], double out[3]);
int orc_find_closest_hit(const rt_prim* prims, int n, const double o[3], const double d[3],
                         double* dist, double normal[3]);
void orc_trace(const rt_prim* prims, int n, const double o[3], const double d[3], int depth,
               uint32_t flags, double rgb[3], uint64_t* segments);

/* Camera::init restatement (scene.cpp:80-106). Returns image height. */
int orc_camera_init(const double position[3], const double lookat[3], const double vup[3],
                    double vfov, double aspect_ratio, double image_width, rt_camera* cam);

/* rt_scene restatement (main.cpp:124-139) over rows [row0,row0+nrows).
 * out64 (H*W*3 doubles), out32 (floats) and path_sig (one uint64 per pixel: a hash of the
 * sequence of hit indices, used by tests to locate geometric discontinuities) may be
 * NULL.  nthreads <= 0: OpenMP default.  Returns the number of closest-hit queries. */
uint64_t orc_render(const rt_prim* prims, int n, const rt_camera* cam, int row0, int nrows,
                    int depth, uint32_t flags, double* out64, float* out32, uint64_t* path_sig,
                    int nthreads);

/* Synthetic scene of SURVEY §8d (SplitMix64, seed): n_spheres then n_walls (<= 6).
 * raw_normals (n_walls*3, may be NULL) receives the un-normalised wall normals as
 * passed to the Wall constructor.  Returns the primitive count. */
int orc_synthetic_scene(int n_spheres, int n_walls, uint64_t seed, rt_prim* out,
                        double* raw_normals);

/* The reference scene of main.cpp:160-163 (1 sphere + 2 walls). Returns 3. */
int orc_default_scene(rt_prim* out, double* raw_normals);

/* main.cpp:345's surface bytes: SDL_MapRGB(fmt, val.x*255, ...) converts each double to
 * its Uint8 parameter implicitly; on the reference's x86-64 build that is cvttsd2si
 * (int32 toward zero; NaN / out of range -> INT32_MIN) then the low byte.  npx pixels of
 * 3 doubles -> 3 bytes each. */
void orc_surface_u8(const double* rgb, size_t npx, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
