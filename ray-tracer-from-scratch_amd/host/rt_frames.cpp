/*
 * host/rt_frames.cpp — headless version of the reference's interactive frame loop
 * (main.cpp:144-392) on the MI355X path, with its performance log.
 *
 * Same camera and scene as main.cpp:146-163 (SCREEN_WIDTH 640, ASPECT_RATIO 4/3 evaluated
 * as the integer 1 -> a 640x640 frame, vfov 90, the sphere + two walls), the frame buffer
 * allocated [SCREEN_WIDTH][image_height] as main.cpp:243 does, and per frame the same
 * stages timed the same way: rt_scene (the drop-in frame operator, include/rt/scene.h),
 * the two vestigial stamps (outpainting, shading), the surface update (the
 * SDL_MapRGB(val*255) packing loop of main.cpp:337-348 into a 32-bit RGBA8888 surface
 * with the masks of main.cpp:193) and the presentation step (no window here: timed, empty).
 * Keys come from a script instead of SDL events (one per frame, cycled): w/s/a/d move the
 * camera as main.cpp:262-292 does (init() is not called again, main.cpp:154).  At exit the
 * averages are printed in main.cpp:386-391's format (integer averages, as std::accumulate
 * over int64 divided by size() gives).
 *
 *   rt_frames [--frames N] [--keys wwaassdd] [--width W] [--depth D] [--precision f64|mixed|
 *             path64|f32] [--scene default|synthetic:S,W[,seed]] [--ppm file] [--gpu-surface]
 *
 * --gpu-surface replaces rt_scene + the host packing loop by one rt_render with the
 * kernel's RT_OUT_RGBA8_WRAP epilogue: the same bytes main.cpp:345 produces, highlights
 * above 1.0 wrapping modulo 256 as the reference's x86-64 build does.
 */
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/rt/scene.h"

namespace {

using clk = std::chrono::high_resolution_clock;

struct Args {
    int frames = 100;
    std::string keys = "";
    int width = 640;  // SCREEN_WIDTH, main.cpp:22
    int depth = 10;   // recursive_ray_tracing's default, main.cpp:89
    int precision = RT_PREC_PATH64;
    std::string scene = "default";
    std::string ppm;
    bool gpu_surface = false;
};

int parse_precision(const std::string& s) {
    if (s == "f64") return RT_PREC_F64;
    if (s == "mixed") return RT_PREC_MIXED;
    if (s == "path64") return RT_PREC_PATH64;
    if (s == "f32") return RT_PREC_F32;
    std::fprintf(stderr, "unknown precision %s\n", s.c_str());
    std::exit(2);
}

Args parse(int argc, char** argv) {
    Args a;
    for (int k = 1; k < argc; k++) {
        const std::string o = argv[k];
        auto val = [&]() -> std::string {
            if (k + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", o.c_str());
                std::exit(2);
            }
            return argv[++k];
        };
        if (o == "--frames") a.frames = std::atoi(val().c_str());
        else if (o == "--keys") a.keys = val();
        else if (o == "--width") a.width = std::atoi(val().c_str());
        else if (o == "--depth") a.depth = std::atoi(val().c_str());
        else if (o == "--precision") a.precision = parse_precision(val());
        else if (o == "--scene") a.scene = val();
        else if (o == "--ppm") a.ppm = val();
        else if (o == "--gpu-surface") a.gpu_surface = true;
        else {
            std::fprintf(stderr, "unknown option %s\n", o.c_str());
            std::exit(2);
        }
    }
    return a;
}

/* SplitMix64 synthetic scene of SURVEY §8d (same draws as rtamd/scenes.py). */
struct SplitMix64 {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double U() { return (double)(next() >> 40) * (1.0 / 16777216.0); }
};

void build_scene(const std::string& spec, std::vector<std::unique_ptr<SceneGeometry>>& scene) {
    if (spec == "default") {  // main.cpp:160-163
        scene.push_back(std::make_unique<Sphere>(Material(RGB(0, 1, 0), 0.5), point3(1.5, 0, 0), .5));
        scene.push_back(std::make_unique<Wall>(Material(RGB(0, 0, 1)), point3(3.0, 2, 0), vec3(0, -1, 0), 1, 1));
        scene.push_back(std::make_unique<Wall>(Material(RGB(0, 1, 0)), point3(3.0, -3, 0), vec3(0, 1, 0), 2, 2));
        return;
    }
    int ns = 0, nw = 0;
    unsigned long long seed = 1234;
    if (std::sscanf(spec.c_str(), "synthetic:%d,%d,%llu", &ns, &nw, &seed) < 2 || nw < 0 || nw > 6) {
        std::fprintf(stderr, "bad --scene %s\n", spec.c_str());
        std::exit(2);
    }
    SplitMix64 g{seed};
    for (int k = 0; k < ns; k++) {
        const double x = 2 + 6 * g.U(), y = -3 + 6 * g.U(), z = -1 + 3 * g.U(), r = .3 + .5 * g.U();
        const double cr = g.U(), cg = g.U(), cb = g.U(), m = g.U();
        scene.push_back(std::make_unique<Sphere>(Material(RGB(cr, cg, cb), m), point3(x, y, z), r));
    }
    const double nrm[6][3] = {{0, -1, 0}, {0, 1, 0}, {-1, 0, 0}, {-.70710678, -.70710678, 0},
                              {-.70710678, .70710678, 0}, {1, 0, 0}};
    const double pos[6][3] = {{3, 4, -1}, {3, -4, -1}, {10, -4, -1}, {8, 3, -1}, {8, -6, -1}, {-10, -4, -1}};
    for (int w = 0; w < nw; w++) {
        const double c = .2 + .6 * g.U();
        scene.push_back(std::make_unique<Wall>(Material(RGB(c, c, c)), point3(pos[w][0], pos[w][1], pos[w][2]),
                                               vec3(nrm[w][0], nrm[w][1], nrm[w][2]), 8, 4));
    }
}

/* SDL_MapRGB's Uint8 argument from val*255 (main.cpp:345): the double converts implicitly,
 * which the reference's x86-64 build does with cvttsd2si (truncate to int32; NaN and values
 * outside the int32 range give INT32_MIN) and the low byte — in-range values truncate,
 * highlights above 1.0 wrap modulo 256 (1.084 displays as 20).  Written without the
 * undefined conversion so any compiler gives those bytes. */
inline uint8_t to_u8(double v) {
    const double t = v * 255;
    const int32_t i = (t > -2147483649.0 && t < 2147483648.0) ? (int32_t)t : INT32_MIN;
    return (uint8_t)((uint32_t)i & 0xffu);
}

}  // namespace

int main(int argc, char** argv) {
    const Args a = parse(argc, argv);
    Camera cam;  // main.cpp:146-153
    constexpr float ASPECT_RATIO = 4 / 3;  // main.cpp:25: integer division, 1
    cam.aspect_ratio = ASPECT_RATIO;
    cam.image_width = a.width;
    cam.movement_speed = 0.1;
    cam.vfov = 90;
    cam.position = point3(0, 0, 0);
    cam.lookat = point3(-1, 0, 0);
    cam.vup = vec3(0, 0, -1);
    auto u = cam.init();
    std::vector<std::unique_ptr<SceneGeometry>> scene;
    build_scene(a.scene, scene);

    RtSceneOptions opts = rt_scene_get_options();
    opts.depth = a.depth;
    opts.precision = a.precision;
    rt_scene_set_options(opts);

    const int W = a.width, H = (int)cam.image_height;
    std::vector<std::vector<RGB>> frame_buffer(W, std::vector<RGB>(H, RGB(0, 0, 0)));  // main.cpp:243
    std::vector<uint32_t> surface((size_t)W * H);  // 32 bpp, pitch W*4 (main.cpp:193)

    // --gpu-surface: the C-ABI directly, RGBA8 epilogue in the kernel
    rt_ctx* ctx = nullptr;
    if (a.gpu_surface) {
        if (rt_ctx_create(opts.device, &ctx) != RT_OK) {
            std::fprintf(stderr, "rt_ctx_create failed\n");
            return 1;
        }
        std::vector<rt_prim> prims(scene.size());
        for (size_t j = 0; j < scene.size(); j++) scene[j]->pack(&prims[j]);
        if (rt_set_scene(ctx, prims.data(), (int32_t)prims.size()) != RT_OK) return 1;
    }

    std::vector<int64_t> total_times, rt_times, outpainting_times, shading_times,
        surface_update_times, sdl_rendering_times;
    int frame_number = 0;
    for (int f = 0; f < a.frames; f++) {
        if (!a.keys.empty()) {  // main.cpp:259-294
            switch (a.keys[f % a.keys.size()]) {
                case 'w': cam.forward(); break;
                case 's': cam.backward(); break;
                case 'a': cam.left(); break;
                case 'd': cam.right(); break;
                default: break;
            }
        }
        const auto rt_start_time = clk::now();
        if (a.gpu_surface) {
            rt_camera c{};
            const vec3* v[4] = {&cam.position, &cam.image_top_left, &u.at(0), &u.at(1)};
            double* dst[4] = {c.position, c.image_top_left, c.pixel_delta_x, c.pixel_delta_y};
            for (int k = 0; k < 4; k++) {
                dst[k][0] = v[k]->x;
                dst[k][1] = v[k]->y;
                dst[k][2] = v[k]->z;
            }
            c.width = W;
            c.height = H;
            if (rt_render(ctx, &c, 0, H, a.depth, a.precision, 0, RT_OUT_RGBA8_WRAP, surface.data(), 0,
                          nullptr) != RT_OK) {
                std::fprintf(stderr, "rt_render failed: %s\n", rt_last_hip_error(ctx));
                return 1;
            }
        } else {
            rt_scene(u, scene, cam, frame_buffer);
        }
        const auto rt_end_time = clk::now();
        const auto outpainting_end_time = clk::now();
        const auto shading_end_time = clk::now();
        if (!a.gpu_surface) {  // main.cpp:337-348
            for (int i = 0; i < H; i++)
                for (int j = 0; j < W; j++) {
                    const RGB val = frame_buffer.at(i).at(j);
                    surface[(size_t)i * W + j] = ((uint32_t)to_u8(val.x) << 24) |
                                                 ((uint32_t)to_u8(val.y) << 16) |
                                                 ((uint32_t)to_u8(val.z) << 8) | 0xFFu;
                }
        }
        const auto surface_end_time = clk::now();
        const auto render_end_time = clk::now();  // no window to present to

        using us = std::chrono::microseconds;
        using ms = std::chrono::milliseconds;
        rt_times.push_back(std::chrono::duration_cast<us>(rt_end_time - rt_start_time).count());
        outpainting_times.push_back(std::chrono::duration_cast<us>(outpainting_end_time - rt_end_time).count());
        shading_times.push_back(std::chrono::duration_cast<us>(shading_end_time - outpainting_end_time).count());
        surface_update_times.push_back(std::chrono::duration_cast<ms>(surface_end_time - shading_end_time).count());
        sdl_rendering_times.push_back(std::chrono::duration_cast<ms>(render_end_time - surface_end_time).count());
        total_times.push_back(std::chrono::duration_cast<ms>(render_end_time - rt_start_time).count());
        frame_number++;
    }
    if (ctx) rt_ctx_destroy(ctx);

    if (!a.ppm.empty() && frame_number > 0) {  // the last frame's surface
        FILE* fp = std::fopen(a.ppm.c_str(), "wb");
        if (!fp) return 1;
        std::fprintf(fp, "P6\n%d %d\n255\n", W, H);
        for (size_t k = 0; k < surface.size(); k++) {
            const uint32_t px = surface[k];
            uint8_t rgb[3];
            if (a.gpu_surface) {  // kernel RGBA8: R in the low byte
                rgb[0] = px & 0xFF, rgb[1] = (px >> 8) & 0xFF, rgb[2] = (px >> 16) & 0xFF;
            } else {               // RGBA8888 masks of main.cpp:193
                rgb[0] = px >> 24, rgb[1] = (px >> 16) & 0xFF, rgb[2] = (px >> 8) & 0xFF;
            }
            std::fwrite(rgb, 1, 3, fp);
        }
        std::fclose(fp);
    }

    if (frame_number == 0) return 0;
    // main.cpp:386-391
    auto avg = [](const std::vector<int64_t>& v) { return std::accumulate(v.begin(), v.end(), 0) / v.size(); };
    std::cout << "Number of frames: " << frame_number << " : " << avg(total_times) << " ms average frame time\n";
    std::cout << "   " << avg(rt_times) << " microseconds for average raytracing\n";
    std::cout << "   " << avg(outpainting_times) << " microseconds for average outpainting\n";
    std::cout << "   " << avg(shading_times) << " microseconds for average shading\n";
    std::cout << "   " << avg(surface_update_times) << " milliseconds for surface average update\n";
    std::cout << "   " << avg(sdl_rendering_times) << " milliseconds for average SDL rendering\n";
    return 0;
}
