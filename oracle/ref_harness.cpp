/*
 * ref_harness.cpp — TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile into
 * oracle/_ref/libref.so, only where /root/reference exists (this container); never
 * shipped, never on the product path.
 *
 * It drives the REFERENCE's own code — vec.cpp and scene.cpp compiled unmodified from
 * /root/reference, and the hot-path functions of /root/reference/main.cpp (lines 1-139:
 * out_color, diffuse_shading, specular, find_closest_hit, recursive_ray_tracing,
 * rt_scene) compiled from that file with only its `#include <SDL.h>` line and its SDL
 * main() (lines 140-397) left out (SDL2 is not installed; nothing is stubbed) — and
 * exposes them through a C API so tests/golden/make_golden.py can record known-answer
 * values and frames as fixtures.  No reference source is copied into the repository.
 */
#include <memory>
#include <stdexcept>
#include <vector>

#include "scene.h"  /* /root/reference/scene.h via -I */
#include "../include/rt_capi.h"

/* Symbols defined by /root/reference/main.cpp:28-139. */
RGB out_color(vec3 v);
double diffuse_shading(vec3 pos, vec3 normal, vec3 light_pos);
double specular(vec3 pos, vec3 normal, vec3 light_pos, vec3 view_dir);
Collision find_closest_hit(const std::vector<std::unique_ptr<SceneGeometry>>& scene, ray r);
RGB recursive_ray_tracing(const std::vector<std::unique_ptr<SceneGeometry>>& scene, ray r,
                          int remaining_iterations);
void rt_scene(std::vector<vec3> u, const std::vector<std::unique_ptr<SceneGeometry>>& scene,
              const Camera& cam, std::vector<std::vector<RGB>>& frame_buffer);

namespace {

vec3 V(const double* p) { return vec3(p[0], p[1], p[2]); }
void S(double* p, const vec3& v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

Material M(const rt_material& m) {
    /* positional order (color, metallic, ambient, diffuse, specular, exp), scene.h:48 */
    return Material(V(m.color), m.metallic, m.ambient, m.diffuse, m.specular,
                    m.specular_exponent);
}

/* raw_normals: the un-normalised normal handed to each Wall constructor (3 per prim). */
std::vector<std::unique_ptr<SceneGeometry>> build(const rt_prim* p, const double* raw, int n) {
    std::vector<std::unique_ptr<SceneGeometry>> scene;
    for (int j = 0; j < n; j++) {
        if (p[j].kind == RT_PRIM_SPHERE)
            scene.push_back(std::make_unique<Sphere>(M(p[j].mat), V(p[j].position), p[j].radius));
        else
            scene.push_back(std::make_unique<Wall>(M(p[j].mat), V(p[j].position), V(raw + 3 * j),
                                                   p[j].length, p[j].width));
    }
    return scene;
}

Camera make_cam(const double* pos, const double* lookat, const double* vup, double vfov,
                double aspect, double width) {
    Camera cam;
    cam.aspect_ratio = aspect;
    cam.image_width = width;
    cam.movement_speed = 0.1;
    cam.vfov = vfov;
    cam.position = V(pos);
    cam.lookat = V(lookat);
    cam.vup = V(vup);
    return cam;
}

}  // namespace

extern "C" {

int ref_camera_init(const double* pos, const double* lookat, const double* vup, double vfov,
                    double aspect, double width, double out12[12]) {
    Camera cam = make_cam(pos, lookat, vup, vfov, aspect, width);
    std::vector<vec3> u = cam.init();
    S(out12 + 0, cam.position);
    S(out12 + 3, cam.image_top_left);
    S(out12 + 6, u[0]);
    S(out12 + 9, u[1]);
    return (int)cam.image_height;
}

/* Renders the frame exactly as rt_scene does (main.cpp:127-138) but with an explicit
 * depth; depth == 10 calls the reference's rt_scene itself.  out = H*W*3 doubles,
 * framebuffer allocated [H][W] (main.cpp:243's [W][H] throws for non-square frames). */
int ref_render(const rt_prim* prims, const double* raw_normals, int n, const double* pos,
               const double* lookat, const double* vup, double vfov, double aspect,
               double width, int depth, double* out) {
    try {
        Camera cam = make_cam(pos, lookat, vup, vfov, aspect, width);
        std::vector<vec3> u = cam.init();
        auto scene = build(prims, raw_normals, n);
        const int H = (int)cam.image_height, W = (int)cam.image_width;
        std::vector<std::vector<RGB>> fb(H, std::vector<RGB>(W, RGB(0, 0, 0)));
        if (depth == 10) {
            rt_scene(u, scene, cam, fb);
        } else {
            for (int i = 0; i < cam.image_height; i++)
                for (int j = 0; j < cam.image_width; j++) {
                    auto pixel_center = cam.image_top_left + u[0] * j + u[1] * i;
                    auto cam_pixel = cam.position - pixel_center;
                    ray cam_pixel_ray(cam_pixel, cam.position);
                    fb.at(i).at(j) = recursive_ray_tracing(scene, cam_pixel_ray, depth);
                }
        }
        for (int i = 0; i < H; i++)
            for (int j = 0; j < W; j++) S(out + ((size_t)i * W + j) * 3, fb[i][j]);
        return H;
    } catch (const std::exception&) {
        return -1;
    }
}

/* Reference rt_scene with the framebuffer allocated as main.cpp:243 does ([W][H]):
 * returns 0 on success, 1 if it threw std::out_of_range (non-square frames). */
int ref_rt_scene_wh_alloc(const rt_prim* prims, const double* raw_normals, int n,
                          const double* pos, const double* lookat, const double* vup,
                          double vfov, double aspect, double width) {
    Camera cam = make_cam(pos, lookat, vup, vfov, aspect, width);
    std::vector<vec3> u = cam.init();
    auto scene = build(prims, raw_normals, n);
    std::vector<std::vector<RGB>> fb((size_t)cam.image_width,
                                     std::vector<RGB>((size_t)cam.image_height, RGB(0, 0, 0)));
    try {
        rt_scene(u, scene, cam, fb);
    } catch (const std::out_of_range&) {
        return 1;
    }
    return 0;
}

int ref_trace(const rt_prim* prims, const double* raw_normals, int n, const double* o,
              const double* d, int depth, double rgb[3]) {
    auto scene = build(prims, raw_normals, n);
    S(rgb, recursive_ray_tracing(scene, ray(V(d), V(o)), depth));
    return 0;
}

int ref_find_closest_hit(const rt_prim* prims, const double* raw_normals, int n, const double* o,
                         const double* d, double* dist, double normal[3]) {
    auto scene = build(prims, raw_normals, n);
    Collision c = find_closest_hit(scene, ray(V(d), V(o)));
    *dist = c.distance;
    S(normal, c.normal);
    return c.hit_object_index;
}

void ref_sphere_intersect(const double* center, double radius, const double* o, const double* d,
                          double* dist, double normal[3], int* hit) {
    Sphere s(Material(RGB(1, 1, 1)), V(center), radius);
    Collision c = s.intersect(ray(V(d), V(o)));
    *dist = c.distance; S(normal, c.normal); *hit = c.hit;
}

void ref_wall_intersect(const double* position, const double* raw_normal, double length,
                        double width, const double* o, const double* d, double* dist,
                        double normal[3], int* hit) {
    Wall w(Material(RGB(1, 1, 1)), V(position), V(raw_normal), length, width);
    Collision c = w.intersect(ray(V(d), V(o)));
    *dist = c.distance; S(normal, c.normal); *hit = c.hit;
}

/* main.cpp:345's surface packing: SDL_MapRGB(format, val.x * 255, val.y * 255, val.z * 255)
 * takes Uint8 parameters, so each double converts implicitly at the call — undefined above
 * 255 in C++; what this g++ -O3 x86-64 build does (the reference's CMake flags) is recorded
 * as fixtures.  pack_rgb has SDL_MapRGB's parameter types; the call has main.cpp's form. */
typedef uint8_t Uint8;
static __attribute__((noinline)) void pack_rgb(Uint8* out, Uint8 r, Uint8 g, Uint8 b) {
    out[0] = r;
    out[1] = g;
    out[2] = b;
}
void ref_surface_u8(const double* rgb, size_t npx, uint8_t* out) {
    for (size_t k = 0; k < npx; k++) {
        const RGB val(rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]);
        pack_rgb(out + 3 * k, val.x * 255, val.y * 255, val.z * 255);
    }
}

void ref_out_color(const double* v, double rgb[3]) { S(rgb, out_color(V(v))); }
double ref_diffuse_shading(const double* pos, const double* normal, const double* light) {
    return diffuse_shading(V(pos), V(normal), V(light));
}
double ref_specular(const double* pos, const double* normal, const double* light,
                    const double* view) {
    return specular(V(pos), V(normal), V(light), V(view));
}
void ref_reflect(const double* v, const double* n, double out[3]) {
    S(out, vec3::reflect(V(v), V(n)));
}
void ref_normalize(const double* v, double out[3]) { S(out, V(v).normalize()); }

}  // extern "C"
