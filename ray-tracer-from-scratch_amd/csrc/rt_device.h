/*
 * rt_device.h — device-side scene records and launch arguments (internal; not ABI).
 *
 * HBM layout of one uploaded scene (one allocation, built by rt_set_scene):
 *
 *   [DevSphere x nS][DevWall x nW][DevMat x nP]
 *
 * Spheres and walls are split by kind so the per-ray scan (find_closest_hit,
 * main.cpp:67-84) runs two branch-free loops instead of a virtual call per primitive;
 * each record keeps its scene index j so ties still resolve to the lowest index as the
 * reference's strict `<` scan does.  Records are wave-uniform (every lane of a wave
 * tests the same primitive), so the kernels read them with scalar loads (one
 * s_load_dwordx16 per sphere) — or broadcast them out of LDS — never per lane.
 * Ray-invariant wall work the reference redoes per test (the basis, scene.cpp:18-19)
 * and r*r (scene.cpp:51) are computed once on the host with the same fp64 operations,
 * so every value is bit-identical to the reference's.
 */
#ifndef RT_DEVICE_H
#define RT_DEVICE_H

#include <stdint.h>

namespace rt {

struct alignas(16) DevSphere {  // 64 B
    double c[3];   // Sphere::center
    double r2;     // radius * radius (scene.cpp:51, same fp64 product)
    float cf[3];   // fp32 copies for the F32 path / MIXED cull
    float r2f;
    float rf;      // radius (fp32), cull scale
    int32_t j;     // scene index
    int32_t pad[2];
};
static_assert(sizeof(DevSphere) == 64, "DevSphere layout");

struct alignas(16) DevWall {  // 176 B
    double P[3];   // Wall::position (corner)
    double n[3];   // Wall::normal (unit, as the ctor stores it)
    double X[3];   // normalize(cross(n, (0,0,1)))      scene.cpp:18
    double Y[3];   // normalize(cross(X, n))             scene.cpp:19
    double len, wid;
    float Pf[3], nf[3], Xf[3], Yf[3];
    float lenf, widf;
    int32_t j;
    int32_t pad;
};
static_assert(sizeof(DevWall) == 176, "DevWall layout");

struct alignas(16) DevMat {  // 64 B, indexed by scene index
    double color[3];
    double ka, km, kd, ks, ex;
};
static_assert(sizeof(DevMat) == 64, "DevMat layout");

enum { PREC_F64 = 0, PREC_F32 = 1, PREC_MIXED = 2 };
enum { OUT_RGB_F32 = 0, OUT_RGB_F64 = 1, OUT_RGBA8 = 2 };
enum { FLAG_SUN = 1 };

// Pixel tile of one 256-thread workgroup: 4 waves, each an 8x8 pixel square.
constexpr int TILE_W = 16;
constexpr int TILE_H = 16;
constexpr int BLOCK = 256;

struct KParams {
    const DevSphere* sph;
    const DevWall* wal;
    const DevMat* mat;
    int32_t nS, nW, nP;
    int32_t W, row0, nrows, depth;
    uint32_t flags;
    int32_t outf;
    double pos[3], tl[3], dx[3], dy[3];
    void* out;
    unsigned long long* segs;  // may be null
};

// Host-side launcher (rt_trace.hip).  Returns a hipError_t as int.
int launch_trace(const KParams& p, int prec, void* stream);
int max_depth();

}  // namespace rt

#endif
