/*
 * rt/scene.h — the reference's scene API (/root/reference/scene.h:1-112) plus the frame
 * operator rt_scene (main.cpp:124-139), kept name-for-name so the reference's main.cpp
 * links against this library instead of its own renderer:
 *
 *   ray, Collision, Material (constructor order (color, metallic, ambient, diffuse,
 *   specular, exp) with defaults .5/.1/.9/.4/50 — scene.h:48), the SceneGeometry
 *   plugin interface (virtual intersect, get_material), Wall, Sphere, Camera
 *   (init() returns {pixel_delta_x, pixel_delta_y}), and
 *   void rt_scene(std::vector<vec3> u, scene, cam, frame_buffer).
 *
 * What changes is underneath: rt_scene flattens the scene through SceneGeometry::pack()
 * into rt_prim records and renders the frame on the MI355X through the C-ABI
 * (include/rt_capi.h).  SceneGeometry::intersect stays available on the host with the
 * reference's semantics (world distance for spheres, parametric t for walls).
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <memory>
#include <vector>

#include "../rt_capi.h"
#include "vec.h"

#define DEFAULT_MAT Material(RGB(1, 1, 1), .9, .9, .3, 30)

class ray {
    vec3 direction;
    point3 origin;

public:
    ray() {}
    ray(const vec3 direction, const point3 origin) : direction{direction}, origin{origin} {}
    point3 at(double t) const { return origin + direction * t; }
    vec3 get_direction() const { return direction; }
    vec3 get_origin() const { return origin; }
};

struct Collision {
    double distance;
    vec3 normal;
    bool hit;
    int hit_object_index;
    Collision(double distance, vec3 normal, bool hit, int hit_object_index)
        : distance{distance}, normal{normal}, hit{hit}, hit_object_index{hit_object_index} {}
};

struct Material {
    RGB color;
    double ambient;
    double metallic;
    double diffuse;
    double specular;
    double specular_exponent;
    Material(RGB color, double metallic = .5, double ambient = .1, double diffuse = .9,
             double specular = .4, double specular_exponent = 50)
        : color{color}, ambient{ambient}, metallic{metallic}, diffuse{diffuse},
          specular{specular}, specular_exponent{specular_exponent} {}
};

/* The primitive plugin interface (scene.h:51-60).  pack() is the hook the GPU path
 * needs: it writes the object's state into a flat rt_prim record.  It is not pure, so a
 * subclass written against the reference's interface (intersect only) still compiles; the
 * default throws std::invalid_argument ("unsupported primitive"), which rt_scene lets
 * through before any device work — the kernels know spheres and walls only. */
class SceneGeometry {
    Material mat;

public:
    explicit SceneGeometry(Material mat) : mat(mat) {}
    virtual ~SceneGeometry() {}
    virtual Collision intersect(ray r) const = 0;
    virtual void pack(rt_prim* out) const;
    Material get_material() const { return mat; }

protected:
    void pack_material(rt_prim* out) const;
};

class Wall : public SceneGeometry {
    point3 position;  // corner
    vec3 normal;      // normalised by the constructor (scene.h:73)
    double length;
    double width;

public:
    Wall(Material mat = DEFAULT_MAT, point3 position = point3(0, 0, 0),
         vec3 normal = vec3(0, 0, 0), double length = 1.0, double width = 1.0)
        : SceneGeometry{mat}, position{position}, normal{normal.normalize()}, length{length},
          width{width} {}
    Collision intersect(ray r) const override;
    void pack(rt_prim* out) const override;
};

class Sphere : public SceneGeometry {
    point3 center;
    double radius;

public:
    Sphere(Material mat = DEFAULT_MAT, point3 center = point3(0, 0, 0), double radius = 1.0)
        : SceneGeometry{mat}, center{center}, radius{radius} {}
    Collision intersect(ray r) const override;
    void pack(rt_prim* out) const override;
};

class Camera {
    vec3 forward_vec();
    vec3 right_vec();
    vec3 up_vec();

public:
    vec3 direction, fov_top_left, image_top_left, pixel_delta_x, pixel_delta_y;
    double movement_speed, aspect_ratio, image_width, image_height, focal_length, vfov;

    point3 position = point3(0, 0, -1);
    point3 lookat = point3(0, 0, 0);
    vec3 vup = vec3(0, 1, 0);

    Camera() {}
    std::vector<vec3> init();

    void forward();
    void backward();
    void left();
    void right();
    void rotate_left_right(double angle);
    void rotate_up_down(double angle);
};

/* The frame operator of main.cpp:124-139, rendered on the GPU: fills
 * frame_buffer.at(row).at(col) for every pixel (throws std::out_of_range exactly where
 * the reference's .at() would, e.g. a [W][H]-allocated buffer for a non-square frame).
 * Depth is recursive_ray_tracing's default 10 (main.cpp:89). */
void rt_scene(std::vector<vec3> u, const std::vector<std::unique_ptr<SceneGeometry>>& scene,
              const Camera& cam, std::vector<std::vector<RGB>>& frame_buffer);

/* Options of the GPU frame operator (not in the reference): device, precision
 * (RT_PREC_*; default RT_PREC_MIXED whose output equals the fp64 path), recursion
 * depth (default 10) and flags (RT_FLAG_SUN).  `devices` with more than one entry renders
 * every frame row-tiled across those GPUs and gathers it into devices[0] (rt_multi_*,
 * BASELINE config 4; `transport` RT_TRANSPORT_RCCL, or RT_TRANSPORT_COPY, which also takes
 * one GPU listed several times); one entry with RT_TRANSPORT_RCCL_LOOPBACK goes through
 * the same operator with a one-rank communicator.  The frame is bitwise the one-GPU frame. */
struct RtSceneOptions {
    int device = 0;
    int precision = RT_PREC_MIXED;
    int depth = 10;
    unsigned flags = 0;
    std::vector<int> devices;
    int transport = RT_TRANSPORT_RCCL;
};
void rt_scene_set_options(const RtSceneOptions& opts);
RtSceneOptions rt_scene_get_options();
/* Releases rt_scene's process-wide renderer (device memory, worker threads, the RCCL
 * communicator of a row-tiled renderer); the next rt_scene call makes a new one.  It also
 * runs from an atexit handler registered when the renderer is made — i.e. after the HIP
 * and RCCL runtimes have initialised, so before their own teardown — never from a static
 * destructor. */
void rt_scene_shutdown();

#endif
