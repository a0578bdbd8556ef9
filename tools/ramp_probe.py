#!/usr/bin/env python3
"""Per-frame GPU time over the first frames of a fresh renderer (one stream, an event pair
per frame): separates start-up effects (clock ramp from idle, the row order's first
snapshot) from the steady state the long bench runs reach.

    python tools/ramp_probe.py [--frames 400] [--config c2] [--precision path64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))

from rtamd import capi, scenes  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precision", default="path64")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--feedback", type=int, nargs="+", default=[32, 0])
    ap.add_argument("--warm", type=int, nargs="+", default=[0],
                    help="RT_OPT_ROW_FEEDBACK_WARM values (each run per feedback value)")
    ap.add_argument("--idle-ms", type=float, default=300.0, help="host sleep before each run")
    ap.add_argument("--chunk", type=int, default=1,
                    help="frames per event pair (>1: chunk averages, low event overhead)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS[args.config]
    prims = scenes.to_prims(cfg.scene())
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    prec = capi.PRECISIONS[args.precision]
    for fb, warm in [(f, w) for f in args.feedback for w in args.warm]:
        rend = capi.Renderer(0)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK_WARM, warm)
        rend.set_option(capi.RT_OPT_BOX_CACHE, 0)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, fb)
        rend.set_scene(prims)
        torch.cuda.synchronize()
        time.sleep(args.idle_ms * 1e-3)
        nch = args.frames // args.chunk
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(nch + 1)]
        ev[0].record(st)
        t0 = time.perf_counter()
        for c in range(nch):
            for _ in range(args.chunk):
                rend.render_device(cam, cfg.depth, out.data_ptr(), prec, 0, capi.RT_OUT_RGB_F32,
                                   stream=st.cuda_stream)
            ev[c + 1].record(st)
        enq = (time.perf_counter() - t0) / (nch * args.chunk) * 1e6
        torch.cuda.synchronize()
        us = [ev[c].elapsed_time(ev[c + 1]) * 1e3 / args.chunk for c in range(nch)]
        if args.chunk > 1:
            print(json.dumps({"feedback": fb, "warm": warm, "chunk": args.chunk, "host_enqueue_us": round(enq, 2),
                              "us_per_frame_by_chunk": [round(u, 2) for u in us]}), flush=True)
            rend.close()
            continue
        buckets = [1, 2, 4, 8, 16, 32, 64, 128, 256, args.frames]
        res = {}
        lo = 0
        for b in buckets:
            if b > args.frames or b <= lo:
                continue
            seg = us[lo:b]
            res[f"{lo}-{b - 1}"] = round(sum(seg) / len(seg), 2)
            lo = b
        print(json.dumps({"config": args.config, "precision": args.precision, "feedback": fb, "warm": warm,
                          "us_per_frame_by_frame_range": res}), flush=True)
        rend.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
