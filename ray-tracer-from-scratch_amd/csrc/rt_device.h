/*
 * rt_device.h — device-side scene layout and launch arguments (internal; not ABI).
 *
 * HBM layout of one uploaded scene (one allocation, built by rt_set_scene; every
 * section 256-B aligned, sphere sections padded to a multiple of 4 records):
 *
 *   SphG32 [ceil(nS/4)]   4 spheres per 64 B  : cx[4] cy[4] cz[4] r[4]  fp32 (SoA)
 *   SphG64 [ceil(nS/4)]   4 spheres per 128 B : {cx, cy, cz, radius^2} fp64
 *   Wall32 [nW]           64 B  : P, n, X, Y, length, width            fp32
 *   Wall64 [nW]           128 B : P, n, X, Y, length, width            fp64
 *   int32  sph_j[nS]      scene index of each sphere (tie-break only)
 *   int32  wall_j[nW]     scene index of each wall (tie-break only)
 *   DevMat [nS + nW]      64 B, spheres first then walls, indexed by "material slot"
 *   DevMat32 [nS + nW]    32 B, fp32 copy for the fp32 colour paths
 *   double wnn[nW][4]     normalize(n) of each wall (32 B)
 *
 * The per-ray scan (find_closest_hit, main.cpp:67-84) runs one loop over sphere groups
 * and one over walls instead of a virtual call per primitive.  Every lane of a wave tests
 * the same primitive, so records are wave-uniform: a whole group of 4 spheres arrives
 * with one s_load_dwordx16 into scalar registers and feeds the VALU as scalar operands
 * (no LDS traffic, no VGPRs, one scalar-load latency per 4 spheres).  Spheres keep scene
 * order, so ties between spheres resolve by position in the array; a wall that ties the
 * current best compares scene indices (strict `<` in scene order == lowest index wins).
 * Ray-invariant work the reference redoes per test — the wall basis (scene.cpp:18-19)
 * and radius*radius (scene.cpp:51) — is computed once on the host with the same fp64
 * operations, so every value is bit-identical to the reference's.
 */
#ifndef RT_DEVICE_H
#define RT_DEVICE_H

#include <stdint.h>

namespace rt {

struct alignas(64) SphG32 {
    float c[4][4];   // [component cx, cy, cz, radius][sphere]: SoA so that two spheres'
                     // same component form an SGPR pair for packed fp32 (v_pk_*) math
};
struct alignas(128) SphG64 {
    double v[4][4];  // [sphere][cx, cy, cz, radius*radius]
};
struct alignas(64) Wall32 {
    float P[3], n[3], X[3], Y[3], len, wid, pad[2];
};
struct alignas(128) Wall64 {
    double P[3], n[3], X[3], Y[3], len, wid, pad[2];
};
struct alignas(64) DevMat {
    double color[3];
    double ka, km, kd, ks, ex;
};
static_assert(sizeof(SphG32) == 64 && sizeof(SphG64) == 128, "sphere group layout");
static_assert(sizeof(Wall32) == 64 && sizeof(Wall64) == 128, "wall layout");
struct alignas(32) DevMat32 {
    float color[3];
    float ka, km, kd, ks, ex;
};
static_assert(sizeof(DevMat) == 64, "material layout");
static_assert(sizeof(DevMat32) == 32, "material layout");

enum { PREC_F64 = 0, PREC_F32 = 1, PREC_MIXED = 2, PREC_PATH64 = 3 };
enum { OUT_RGB_F32 = 0, OUT_RGB_F64 = 1, OUT_RGBA8 = 2, OUT_RGBA8_WRAP = 3 };
enum { FLAG_SUN = 1 };

// Pixel tile of one workgroup: RT_WAVES_PER_BLOCK waves (1, 2 or 4), each an 8x8 square.
// One wave per workgroup measured fastest (tools/ab.py: c5 -15..21%, c3 -7..12%, c2 -2%
// vs four): finer dispatch granularity at 3-5 waves/SIMD.
#ifndef RT_WAVES_PER_BLOCK
#define RT_WAVES_PER_BLOCK 1
#endif
constexpr int BLOCK = 64 * RT_WAVES_PER_BLOCK;
constexpr int TILE_W = RT_WAVES_PER_BLOCK >= 2 ? 16 : 8;
constexpr int TILE_H = RT_WAVES_PER_BLOCK >= 4 ? 16 : 8;

// Camera-origin ("eye") tables of the primary segment.  Every primary ray starts at the
// camera position, so the origin-only terms of both tests — Sphere::intersect's
// ray_sphere_vec and c (scene.cpp:45, 51) and Wall::intersect's numerator
// dot(position - origin, normal) (scene.cpp:10) — are the same for every pixel of a
// frame.  The host evaluates them once per render with the reference's fp64 operations
// (bit-identical values) and passes them in the kernel arguments, which the kernel reads
// with scalar loads: the primary test then costs the direction-dependent half only.
// Used by the F64/PATH64 linear-scan kernels when the scene fits (eye != 0); A/B at
// c2: -2..3%.  (The fp32 path measured slower with them.)
constexpr int EYE_MAX_S = 32;
constexpr int EYE_MAX_W = 16;

// Primary-ray tile bins.  Every primary ray starts at the camera o with direction
// d(x, i) = o - (TL + dx*x + dy*i) (main.cpp:132-133), so a point X = o + u*d(x, i) has
// pixel coordinates (x, i) = (p/u, q/u) where (u, p, q) = M^-1 (X - o), M = [o - TL, -dx,
// -dy]: a projective map.  Per frame the host projects each primitive's convex hull (a
// sphere's bounding cube, a wall's rectangle clipped to u >= eps) to a pixel bounding box
// widened by one pixel (rt_capi.cpp frame_boxes); the kernel ANDs its 8x8 tile against
// the boxes (one lane per primitive, one ballot) and the primary scan tests only the
// primitives whose box meets the tile.  A primitive outside the box by >= 1 pixel is
// missed by the exact ray by an angle ~1e12 times the reference's rounding, so the
// reference's own test rejects it too.  Scenes of <= 64 primitives.
constexpr int BIN_MAX_PRIMS = 64;
// Mirror bins.  A reflection off a plane is linear: the first-bounce ray of pixel (x, i)
// off wall w (origin pos + 1e-4 n, direction reflect(d, n), main.cpp:111-113) lies on the
// line from the camera mirrored in w's plane (shifted by 1e-4 n) with direction R d(x, i),
// R = I - 2 n n^T, again affine in (x, i); a chain of wall bounces composes the
// reflections.  So a wave whose live rays all followed the same wall sequence can cull
// the next segment with the pixel boxes of that virtual camera, computed per frame like
// the primary boxes for every sequence of up to MIR_MAX_DEPTH walls that some tile can
// follow.  Sequence (w1..wL) of level L: boxes at mbox[(off_L + q) * nbox ..], q the
// base-nW number w1..wL, off_L = nW + nW^2 + .. + nW^(L-1).
constexpr int MIR_MAX_DEPTH = 3;
#ifndef RT_MIR_MAX_BOXES
#define RT_MIR_MAX_BOXES 256
#endif
constexpr int MIR_MAX_BOXES = RT_MIR_MAX_BOXES;
struct PrimBox {
    int16_t x0, x1, i0, i1;  // inclusive pixel box (frame rows); x0 > x1 = never hit
};

// Sphere clusters for the cull kernels' wide-cone waves (rt_trace.hip clusters_scan).  The
// host splits the spheres at the median of the centres' widest axis until each leaf holds
// <= CLU_SIZE of them (rt_capi.cpp build_clusters); each leaf gets an fp32 box around its
// balls widened by a margin far above fp32 rounding, and a copy of its spheres' exact fp64
// records in leaf order.  A lane tests its own ray against the leaf boxes, then runs the
// exact test on the spheres of its own leaves only: a wave's iteration count is its worst
// lane's, not the union of its lanes' candidates (which is what the wave cone pays when the
// live rays point everywhere).
// Two leaf sizes, one cluster set each: the F32 kernels' walk (cheap sphere tests, so the
// box pass dominates) wants few leaves, the fp64 kernels' walk (exact fp64 tests) small ones
// (A/B round 4: leaves of 4 vs 8, c3 PATH64 -6%, c5 -0.5..0.9%, but F32 c5 +7.6%).  The fp64
// set falls back to CLU_SIZE leaves when its own would exceed CLU_MAX.
#ifndef RT_CLU_SIZE
#define RT_CLU_SIZE 8
#endif
#ifndef RT_CLU_SIZE_D
#define RT_CLU_SIZE_D 4
#endif
constexpr int CLU_SIZE = RT_CLU_SIZE;      // F32 kernels
constexpr int CLU_SIZE_D = RT_CLU_SIZE_D;  // fp64-path kernels (F64, MIXED, PATH64)
constexpr int CLU_MAX = 64;
static_assert(CLU_SIZE_D <= CLU_SIZE, "the fp64 walk's loop covers CLU_SIZE_D or CLU_SIZE");
struct alignas(32) Clu32 {
    float lo[3], hi[3];
    uint8_t rank[8];  // position of this cluster in the near-to-far order of each direction
                      // octant (bit 0/1/2 = d.x/d.y/d.z < 0): the host sorts the clusters by
                      // their centroid along the octant's diagonal
};
struct alignas(64) CluSph {
    double c[4];     // cx, cy, cz, radius^2 (the SphG64 record)
    float f[4];      // cx, cy, cz, radius (the SphG32 record, F32 kernels)
    int32_t slot;    // material slot = sphere index, -1 = padding
    int32_t pad[3];
};
static_assert(sizeof(Clu32) == 32 && sizeof(CluSph) == 64, "cluster layout");

// Dispatch order given explicitly: up to ROW_PERM_MAX units (tile rows of 8 pixel rows, or
// parts of them), int16 each, in the kernel arguments.
#ifndef RT_ROW_PERM_MAX
#define RT_ROW_PERM_MAX 2048
#endif
constexpr int ROW_PERM_MAX = RT_ROW_PERM_MAX;

struct KParams {
    const SphG32* s32;
    const SphG64* s64;
    const Wall32* w32;
    const Wall64* w64;
    const int32_t* sph_j;
    const int32_t* wall_j;
    const DevMat* mat;     // [nS + nW]
    const DevMat32* mat32; // [nS + nW]
    const double (*wnn)[4];  // [nW] normalize(wall normal) (vec.cpp:21, host), the normal
                             // every reflection / shading step normalises again
    int32_t nS, nW;
    int32_t int_exp;       // every specular exponent is an integer in [0, 1024]
    int32_t wave_cull;     // cull spheres per wave (rt_trace.hip) before the per-lane tests
    int32_t W, row0, nrows, depth;
    uint32_t flags;
    int32_t outf;
    double pos[3], tl[3], dx[3], dy[3];
    void* out;
    unsigned long long* segs;   // may be null
    unsigned long long* stats;  // diagnostic counters, may be null (rt_set_option)
    int32_t nbox;               // primitives with a PrimBox (nS + nW), 0 = tile bins off
    int32_t row_center;         // tile row dispatched first (rt_trace.hip tile_row), -1 = off
    uint16_t* tile_cost;        // per wave (workgroup row-major over the frame's tiles, then
                                // wave): shader cycles / 32, saturated; null = not recorded
    int32_t row_units_log2;     // each tile row split into 2^k dispatch units (k > 0 only
                                // with a row_perm over units: unit u = row (u >> k), part
                                // (u & (2^k - 1)) of ceil(tiles / 2^k) tiles)
    int32_t row_perm_n;         // dispatch units in row_perm (== the grid's rows), 0 = unused
    int16_t row_perm[ROW_PERM_MAX];  // dispatch order of tile rows (rt_trace.hip tile_row)
    PrimBox box[BIN_MAX_PRIMS]; // material-slot order: spheres, then walls (scenes with the
                                // wave cull: the walls' boxes only, box[w] = wall w)
    int32_t nwbox;              // wave-cull scenes: walls with a PrimBox in box[] (0 = off)
    int32_t mir_depth;          // wall-sequence levels with mirror boxes (0 = off)
    int32_t pairs;              // RT_OPT_PIXEL_PAIRS: PATH64 linear-scan frames trace two
                                // pixels per lane (16x8 pixels per wave)
    PrimBox mbox[MIR_MAX_BOXES];  // [sequence][slot j]: primitive j through the camera
                                  // mirrored along the sequence (see above)
    int32_t eye;                        // eye tables below valid
    int32_t wall_order_n;               // walls in wall_order (== nW), 0 = index order
    uint64_t wall_order;                // primary scan's wall visiting order, 4 bits per
                                        // wall slot, nearest to the camera first (host)
    double eye_s[EYE_MAX_S][4];         // sphere s: {oc.x, oc.y, oc.z, |oc|^2 - r^2}
    double eye_w[EYE_MAX_W];            // wall w: dot(P - pos, n)
    const Clu32* clu;      // [nclu] sphere-cluster boxes (cull kernels), see above
    const CluSph* csph;    // [nclu * clu_ls] their spheres in cluster order
    const uint8_t* cord;   // [8][CLU_MAX] cluster at each rank of each octant's order
    int32_t nclu;          // 0 = no clusters
    int32_t clu_ls;        // spheres per leaf record: CLU_SIZE_D or CLU_SIZE (F32: CLU_SIZE)
    int32_t clu_axis;      // axis of the first split (0..2): lanes walk clusters against it
    float clu_cos;         // wide-cone waves (cone cos(half-angle) < clu_cos) use clusters
    float clu_oinf;        // rays whose |origin|inf exceeds it test every cluster (the box
                           // margin covers fp32 rounding only for origins near the scene)
    // interleaved parts (rt_render_device_interleaved): tstride > 1 = the band is the
    // frame's tile rows tphase, tphase + tstride, ... (nrows = their pixel rows, row0 = 0);
    // frame_h = frame height; out_frame = store at frame rows instead of back to back
    int32_t tstride, tphase, frame_h, out_frame;
};
// by-value kernel arguments of up to 16 KB arrive intact (tools/ubench/kernarg_size.hip,
// kernarg_stale.hip: consistent across back-to-back launches)
static_assert(sizeof(KParams) <= 16384, "kernel arguments over 16 KB");

// Host-side launchers (rt_trace.hip).  Return a hipError_t as int.  done_event (a
// hipEvent_t, may be null) is signalled by the kernel's own completion (hipExtLaunchKernel
// stop event: no separate marker packet, unlike a hipEventRecord behind the launch).
int launch_trace(const KParams& p, int prec, void* stream, void* done_event = nullptr);
// nframes frames of one band in ONE launch (grid.z = frame): d_tab = their KParams in device
// memory, p0 = a host copy of the first (grid, kernel choice: every frame must share its W,
// nrows, row_units_log2, depth, flags, precision and scene).  The linear-scan kernels only:
// hipErrorNotSupported for a wave-cull scene or RT_OPT_PIXEL_PAIRS.
int launch_trace_batch(const KParams* d_tab, const KParams& p0, int nframes, int prec, void* stream,
                       void* done_event);
int max_depth();
// Device self-test of the exact fp64 helpers against IEEE operations:
// which 0 = division (shared reciprocal), 1 = integer-exponent pow vs pow(),
// 2 = sqrt_e vs sqrt(); adds the number of mismatches (division, sqrt: bitwise;
// pow: > 128 ulp) to *d_bad.
int launch_selftest(int which, uint64_t n, uint64_t seed, unsigned long long* d_bad,
                    void* stream);
// Row feedback: umax[(r << ul) + q] = the largest of cost[r * gx + q * U ..] over dispatch
// unit q of row r (U = ceil(gx / 2^ul)), for gy rows of gx wave costs.
int launch_unit_max(const uint16_t* cost, int gy, int gx, int ul, uint32_t* umax, void* stream);

}  // namespace rt

#endif
