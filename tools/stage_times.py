#!/usr/bin/env python3
"""Where a wave's life goes, stage by stage, from a diagnostic build (-DRT_STAGE_TIMES=1):
s_memtime (shader clock) at kernel entry (0), after primary ray generation (1), after the
tile-bin keep mask (stats slot 7), after the primary scan (2), after the bounce loop (3), after the unwind (4), after the store (5).
Exact paths, linear-scan kernels only (the cull kernels use KParams::stats for counters).

    tools/build_variant.sh st -DRT_STAGE_TIMES=1
    python tools/stage_times.py --lib ray-tracer-from-scratch_amd/lib/ab/st.so --setups c2:4:path64,c2:0:path64
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402

NAMES = ["raygen", "scan0", "bounces", "unwind", "store"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--setups", default="c2:4:path64")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    lib = capi.load(args.lib)
    h = C.c_void_p()
    capi.check(lib.rt_ctx_create(0, C.byref(h)))
    stream = torch.cuda.Stream(dev)
    for su in args.setups.split(","):
        name, depth, prec = su.split(":")
        cfg = scenes.CONFIGS[name]
        prims = scenes.to_prims(cfg.scene())
        arr = (capi.rt_prim * len(prims))(*prims)
        capi.check(lib.rt_set_scene(h, arr, len(prims)))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        W, H = cam.width, cam.height
        nw = ((W + 7) // 8) * ((H + 7) // 8)
        buf = torch.zeros(8 * nw, dtype=torch.int64, device=dev)
        out = torch.empty((H, W, 3), dtype=torch.float32, device=dev)
        pc = capi.PRECISIONS[prec]

        def launch():
            capi.check(lib.rt_render_device(h, C.byref(cam), 0, H, int(depth), pc, 0, 0,
                                            C.c_void_p(out.data_ptr()), None,
                                            C.c_void_p(stream.cuda_stream)))
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, 0))
        for _ in range(40):
            launch()
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, buf.data_ptr()))
        launch()
        torch.cuda.synchronize()
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, 0))
        a = buf.view(nw, 8).cpu().numpy().astype(np.float64)
        t = a[:, :6]
        segs = a[:, 6]
        d = np.diff(t, axis=1)
        life = t[:, 5] - t[:, 0]
        r = dict(setup=su, waves=int(nw), life_cyc_mean=round(life.mean(), 1),
                 life_cyc_p50=round(float(np.median(life)), 1),
                 keep_after_raygen_mean=round(float((a[:, 7] - t[:, 1]).mean()), 1),
                 scan_after_keep_mean=round(float((t[:, 2] - a[:, 7]).mean()), 1))
        for k, nm in enumerate(NAMES):
            r[nm + "_mean"] = round(float(d[:, k].mean()), 1)
            r[nm + "_p50"] = round(float(np.median(d[:, k])), 1)
        # waves by segment count: light (one segment per lane) vs heavy
        light = segs <= 64
        r["light_frac"] = round(float(light.mean()), 3)
        if light.any():
            r["light_life_mean"] = round(float(life[light].mean()), 1)
            r["light_stage_means"] = [round(float(d[light, k].mean()), 1) for k in range(5)]
        if (~light).any():
            r["heavy_life_mean"] = round(float(life[~light].mean()), 1)
            r["heavy_stage_means"] = [round(float(d[~light, k].mean()), 1) for k in range(5)]
        span = (t[:, 5].max() - t[:, 0].min())
        r["span_cyc"] = round(float(span), 1)
        print(json.dumps(r), flush=True)
    lib.rt_ctx_destroy(h)


if __name__ == "__main__":
    main()
