// Drop-in check of the C++ API mirror (include/rt/scene.h): host code written the way
// the reference's main.cpp uses its API (main.cpp:146-163, 243, 329) links against
// librt_host.so + librt_amd.so instead of the reference's renderer.
//   dropin_main kat                 host-side SceneGeometry::intersect / Camera::init values
//   dropin_main render W H [depth]  rt_scene on the GPU; writes H*W*3 doubles to stdout
//   dropin_main throws W H          [W][H]-allocated framebuffer (main.cpp:243): prints 1 if
//                                   rt_scene throws std::out_of_range
//   dropin_main plugin              a SceneGeometry subclass written against the reference's
//                                   interface (intersect only) compiles; rt_scene prints 1 if
//                                   it throws std::invalid_argument (no device needed)
//   dropin_main render_multi W H N [transport]  rt_scene row-tiled over N ranks on device 0
//                                   (RtSceneOptions::devices = {0 x N}); same output as render
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#include "rt/scene.h"

static std::vector<std::unique_ptr<SceneGeometry>> default_scene() {
    std::vector<std::unique_ptr<SceneGeometry>> scene = {};
    scene.push_back(std::make_unique<Sphere>(Material(RGB(0, 1, 0), 0.5), point3(1.5, 0, 0), .5));
    scene.push_back(std::make_unique<Wall>(Material(RGB(0, 0, 1)), point3(3.0, 2, 0), vec3(0, -1, 0), 1, 1));
    scene.push_back(std::make_unique<Wall>(Material(RGB(0, 1, 0)), point3(3.0, -3, 0), vec3(0, 1, 0), 2, 2));
    return scene;
}

// a primitive plugin as a reference user would write it (scene.h:51-60: intersect only)
class Disc : public SceneGeometry {
public:
    Disc() : SceneGeometry(Material(RGB(1, 0, 0))) {}
    Collision intersect(ray) const override { return Collision(-1, vec3(0, 0, 0), false, -1); }
};

static Camera make_camera(int w, int h) {
    Camera cam;
    cam.aspect_ratio = (double)w / h;
    cam.image_width = w;
    cam.movement_speed = 0.1;
    cam.vfov = 90;
    cam.position = point3(0, 0, 0);
    cam.lookat = point3(-1, 0, 0);
    cam.vup = vec3(0, 0, -1);
    return cam;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    if (mode == "kat") {
        Sphere s(Material(RGB(1, 1, 1)), point3(3, 0, 0), 1.0);
        const double dirs[][3] = {{1, 0, 0}, {2, 0, 0}, {-1, 0, 0}};
        for (auto& d : dirs) {
            Collision c = s.intersect(ray(vec3(d[0], d[1], d[2]), point3(0, 0, 0)));
            std::printf("sphere %.17g %.17g %.17g %.17g %d\n", c.distance, c.normal.x, c.normal.y,
                        c.normal.z, (int)c.hit);
        }
        Collision t = s.intersect(ray(vec3(1, 0, 0), point3(0, 1, 0)));  // tangent: /a quirk
        std::printf("tangent %.17g\n", t.distance);
        Wall w(Material(RGB(1, 1, 1)), point3(3, -1, -1), vec3(-1, 0, 0), 2, 2);
        Collision c = w.intersect(ray(vec3(2, 0, 0), point3(0, 0, 0)));
        std::printf("wall %.17g %d\n", c.distance, (int)c.hit);
        Wall zw(Material(RGB(1, 1, 1)), point3(-1, -1, 3), vec3(0, 0, 1), 2, 2);
        std::printf("zwall %d\n", (int)zw.intersect(ray(vec3(0, 0, 1), point3(0, 0, 0))).hit);
        Camera cam = make_camera(640, 480);
        std::vector<vec3> u = cam.init();
        std::printf("camera %.17g %.17g %.17g %.17g %.17g\n", cam.image_height, cam.image_top_left.y,
                    cam.image_top_left.z, u[0].y, u[1].z);
        vec3 r = vec3::reflect(vec3(1, -1, 0), vec3(0, 2, 0));
        std::printf("reflect %.17g %.17g %.17g\n", r.x, r.y, r.z);
        return 0;
    }
    if (mode == "render" && argc >= 4) {
        const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
        RtSceneOptions o = rt_scene_get_options();
        if (argc >= 5) o.depth = std::atoi(argv[4]);
        rt_scene_set_options(o);
        auto scene = default_scene();
        Camera cam = make_camera(W, H);
        auto u = cam.init();
        std::vector<std::vector<RGB>> frame_buffer(H, std::vector<RGB>(W, RGB(0, 0, 0)));
        rt_scene(u, scene, cam, frame_buffer);
        for (int i = 0; i < H; i++)
            for (int j = 0; j < W; j++) {
                const double v[3] = {frame_buffer[i][j].x, frame_buffer[i][j].y, frame_buffer[i][j].z};
                std::fwrite(v, sizeof v, 1, stdout);
            }
        return 0;
    }
    if (mode == "plugin") {
        auto scene = default_scene();
        scene.push_back(std::make_unique<Disc>());
        Camera cam = make_camera(32, 32);
        auto u = cam.init();
        std::vector<std::vector<RGB>> frame_buffer(32, std::vector<RGB>(32, RGB(0, 0, 0)));
        try {
            rt_scene(u, scene, cam, frame_buffer);
        } catch (const std::invalid_argument& e) {
            std::printf("1 %s\n", e.what());
            return 0;
        }
        std::printf("0\n");
        return 0;
    }
    if (mode == "render_multi" && argc >= 5) {
        const int W = std::atoi(argv[2]), H = std::atoi(argv[3]), N = std::atoi(argv[4]);
        RtSceneOptions o = rt_scene_get_options();
        o.devices.assign(N, 0);
        o.transport = argc >= 6 ? std::atoi(argv[5]) : RT_TRANSPORT_COPY;
        rt_scene_set_options(o);
        auto scene = default_scene();
        Camera cam = make_camera(W, H);
        auto u = cam.init();
        std::vector<std::vector<RGB>> frame_buffer(H, std::vector<RGB>(W, RGB(0, 0, 0)));
        for (int rep = 0; rep < 2; rep++) rt_scene(u, scene, cam, frame_buffer);
        for (int i = 0; i < H; i++)
            for (int j = 0; j < W; j++) {
                const double v[3] = {frame_buffer[i][j].x, frame_buffer[i][j].y, frame_buffer[i][j].z};
                std::fwrite(v, sizeof v, 1, stdout);
            }
        return 0;
    }
    if (mode == "throws" && argc >= 4) {
        const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
        auto scene = default_scene();
        Camera cam = make_camera(W, H);
        auto u = cam.init();
        std::vector<std::vector<RGB>> frame_buffer(W, std::vector<RGB>(H, RGB(0, 0, 0)));
        try {
            rt_scene(u, scene, cam, frame_buffer);
        } catch (const std::out_of_range&) {
            std::printf("1\n");
            return 0;
        }
        std::printf("0\n");
        return 0;
    }
    return 2;
}
