/*
 * host/rt_scene.cpp — the drop-in frame operator (main.cpp:124-139) on the GPU path.
 *
 * Same signature and observable behaviour as the reference: fills
 * frame_buffer.at(i).at(j) for every row i < image_height and column j < image_width,
 * with RGB values of recursive_ray_tracing at depth 10.  Underneath, the scene is
 * flattened through SceneGeometry::pack() and rendered by the HIP kernel through the
 * C-ABI with fp64 output (RT_OUT_RGB_F64), so the values are the fp64 path's.
 *
 * The reference has no context argument, so a process-wide renderer is created on first
 * use (device/precision from rt_scene_set_options; with several devices a row-tiled
 * rt_multi whose bands are gathered into the first); like the reference, rt_scene is
 * meant to be called from one thread.  A primitive without a GPU record (a SceneGeometry
 * subclass that does not override pack()) throws std::invalid_argument before any device
 * work.
 */
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt/scene.h"

namespace {

struct Global {
    std::mutex mu;
    RtSceneOptions opts;
    rt_ctx* ctx = nullptr;
    int ctx_device = -1;
    rt_multi* multi = nullptr;       // opts.devices.size() > 1: row-tiled across GPUs
    std::vector<int> multi_devices;
    int multi_transport = -1;
    std::vector<double> staging;
    std::vector<rt_prim> uploaded;  // the scene on the device (re-uploaded only on change)
    bool uploaded_tiled = false;    // ... of the tiled (rt_multi) or the one-GPU renderer
    bool atexit_set = false;
    // no destructor: a function-static's destructor runs in an order unspecified relative
    // to the HIP and RCCL runtimes' own teardown; rt_scene_shutdown (atexit) releases
    void release() {
        if (ctx) rt_ctx_destroy(ctx);
        if (multi) rt_multi_destroy(multi);
        ctx = nullptr;
        multi = nullptr;
        ctx_device = -1;
        multi_devices.clear();
        multi_transport = -1;
        uploaded.clear();
    }
};

Global& global() {
    static Global* g = new Global();  // never destroyed (see Global::release)
    return *g;
}

/* After the first renderer exists (the HIP runtime — and RCCL for a tiled renderer — is
 * initialised by then), so the handler runs before their exit-time teardown. */
void register_shutdown(Global& g) {
    if (g.atexit_set) return;
    g.atexit_set = true;
    std::atexit([] { rt_scene_shutdown(); });
}

void check(int st, rt_ctx* ctx, const char* what) {
    if (st != RT_OK)
        throw std::runtime_error(std::string(what) + ": " + rt_strerror(st) + " " +
                                 rt_last_hip_error(ctx));
}

void check_multi(int st, rt_multi* m, const char* what) {
    if (st != RT_OK)
        throw std::runtime_error(std::string(what) + ": " + rt_strerror(st) + " " +
                                 rt_multi_last_error(m));
}

}  // namespace

void rt_scene_shutdown() {
    Global& g = global();
    std::lock_guard<std::mutex> lk(g.mu);
    g.release();
}

void rt_scene_set_options(const RtSceneOptions& opts) {
    Global& g = global();
    std::lock_guard<std::mutex> lk(g.mu);
    g.opts = opts;
}

RtSceneOptions rt_scene_get_options() {
    Global& g = global();
    std::lock_guard<std::mutex> lk(g.mu);
    return g.opts;
}

void rt_scene(std::vector<vec3> u, const std::vector<std::unique_ptr<SceneGeometry>>& scene,
              const Camera& cam, std::vector<std::vector<RGB>>& frame_buffer) {
    Global& g = global();
    std::lock_guard<std::mutex> lk(g.mu);
    // flatten first: a primitive the GPU path does not know throws before any device work
    std::vector<rt_prim> prims(scene.size());
    for (size_t j = 0; j < scene.size(); j++) scene[j]->pack(&prims[j]);
    // several devices, or one with the loopback transport (the gather's RCCL calls on one GPU)
    const bool tiled = g.opts.devices.size() > 1 ||
                       (g.opts.devices.size() == 1 && g.opts.transport == RT_TRANSPORT_RCCL_LOOPBACK);
    if (tiled && (!g.multi || g.multi_devices != g.opts.devices ||
                  g.multi_transport != g.opts.transport)) {
        if (g.multi) rt_multi_destroy(g.multi);
        g.multi = nullptr;
        const int n = (int)g.opts.devices.size();
        const int st = rt_multi_create(g.opts.devices.data(), n, n, 0, nullptr, g.opts.transport,
                                       &g.multi);
        if (st != RT_OK) throw std::runtime_error(std::string("rt_multi_create: ") + rt_strerror(st));
        g.multi_devices = g.opts.devices;
        g.multi_transport = g.opts.transport;
        g.uploaded.clear();
    } else if (!tiled && (!g.ctx || g.ctx_device != g.opts.device)) {
        if (g.ctx) rt_ctx_destroy(g.ctx);
        g.ctx = nullptr;
        check(rt_ctx_create(g.opts.device, &g.ctx), nullptr, "rt_ctx_create");
        g.ctx_device = g.opts.device;
        g.uploaded.clear();
    }
    register_shutdown(g);
    if (tiled != g.uploaded_tiled) g.uploaded.clear();
    g.uploaded_tiled = tiled;
    // the interactive loop renders the same scene frame after frame (main.cpp:329): keep it
    // resident on the device and upload only when the packed records change
    if (g.uploaded.empty() || prims.size() != g.uploaded.size() ||
        std::memcmp(prims.data(), g.uploaded.data(), prims.size() * sizeof(rt_prim)) != 0) {
        g.uploaded.clear();
        if (tiled)
            check_multi(rt_multi_set_scene(g.multi, prims.data(), (int32_t)prims.size()), g.multi,
                        "rt_multi_set_scene");
        else
            check(rt_set_scene(g.ctx, prims.data(), (int32_t)prims.size()), g.ctx, "rt_set_scene");
        g.uploaded = prims;
    }

    rt_camera c{};
    const vec3* v[4] = {&cam.position, &cam.image_top_left, &u.at(0), &u.at(1)};
    double* dst[4] = {c.position, c.image_top_left, c.pixel_delta_x, c.pixel_delta_y};
    for (int k = 0; k < 4; k++) {
        dst[k][0] = v[k]->x;
        dst[k][1] = v[k]->y;
        dst[k][2] = v[k]->z;
    }
    const int W = (int)cam.image_width, H = (int)cam.image_height;
    c.width = W;
    c.height = H;
    g.staging.resize((size_t)W * H * 3);
    if (tiled)
        check_multi(rt_multi_render(g.multi, &c, g.opts.depth, g.opts.precision, g.opts.flags,
                                    RT_OUT_RGB_F64, g.staging.data(), nullptr),
                    g.multi, "rt_multi_render");
    else
        check(rt_render(g.ctx, &c, 0, H, g.opts.depth, g.opts.precision, g.opts.flags,
                        RT_OUT_RGB_F64, g.staging.data(), 0, nullptr),
              g.ctx, "rt_render");
    for (int i = 0; i < H; i++)
        for (int j = 0; j < W; j++) {
            const double* p = &g.staging[((size_t)i * W + j) * 3];
            frame_buffer.at(i).at(j) = RGB(p[0], p[1], p[2]);  // main.cpp:136 indexing
        }
}
