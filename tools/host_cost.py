#!/usr/bin/env python3
"""Host cost of one rt_render_device call vs the GPU time of its frame, per library build
(is the frame loop host-bound?).   python tools/host_cost.py lib/librt_amd.so [more.so ...]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402
import ctypes as C  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    cfg = scenes.CONFIGS[os.environ.get("CFG", "c2")]
    prims = scenes.to_prims(cfg.scene())
    arr = (capi.rt_prim * len(prims))(*prims)
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = torch.empty((cam.height, cam.width, 3), device=dev)
    libs = [capi.load(os.path.abspath(p)) for p in sys.argv[1:]]
    ctxs = []
    for lib in libs:
        h = C.c_void_p()
        capi.check(lib.rt_ctx_create(0, C.byref(h)))
        capi.check(lib.rt_set_scene(h, arr, len(prims)))
        for opt, v in ((capi.RT_OPT_BOX_CACHE, int(os.environ.get("BOXCACHE", "0"))),):
            lib.rt_set_option(h, opt, v)
        ctxs.append(h)
    n = 200
    for rnd in range(3):
        for path, lib, h in zip(sys.argv[1:], libs, ctxs):
            for _ in range(20):
                lib.rt_render_device(h, C.byref(cam), 0, cam.height, cfg.depth, capi.RT_PREC_PATH64,
                                     0, 0, C.c_void_p(out.data_ptr()), None, C.c_void_p(st.cuda_stream))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            for _ in range(n):
                lib.rt_render_device(h, C.byref(cam), 0, cam.height, cfg.depth, capi.RT_PREC_PATH64,
                                     0, 0, C.c_void_p(out.data_ptr()), None, C.c_void_p(st.cuda_stream))
            t1 = time.perf_counter()
            e1.record(st)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"lib": os.path.basename(path), "round": rnd,
                              "host_us_per_call": round((t1 - t0) / n * 1e6, 2),
                              "gpu_us_per_frame": round(e0.elapsed_time(e1) / n * 1e3, 2),
                              "wall_us_per_frame": round((t2 - t0) / n * 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
