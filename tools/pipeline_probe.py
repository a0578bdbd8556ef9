#!/usr/bin/env python3
"""Frames in flight: c2 frame throughput with the frames of a loop spread over S streams
(S output buffers, frame f on stream f mod S), so one frame's tail (its last heavy waves)
overlaps the next frame's start.  Prints one JSON line per (config, precision, S).

    python tools/pipeline_probe.py [--config c2] [--frames 400] [--streams 1 2 3 4]
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
    ap.add_argument("--config", nargs="+", default=["c2"])
    ap.add_argument("--precision", nargs="+", default=["path64"])
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3, 4])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--box-cache", type=int, nargs="+", default=[0],
                    help="RT_OPT_BOX_CACHE values to run (1: the host reuses the boxes of an "
                         "unchanged camera, i.e. the launch without the per-frame box work)")
    args = ap.parse_args()

    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for cname in args.config:
        cfg = scenes.CONFIGS[cname]
        prims = scenes.to_prims(cfg.scene())
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        W, H = cam.width, cam.height
        rend = capi.Renderer(0)
        rend.set_scene(prims)
        smax = max(args.streams)
        streams = [torch.cuda.Stream(dev) for _ in range(smax)]
        outs = [torch.empty((H, W, 3), dtype=torch.float32, device=dev) for _ in range(smax)]
        segs = torch.zeros(1, dtype=torch.int64, device=dev)
        for pname in args.precision:
            prec = capi.PRECISIONS[pname]
            rend.render_device(cam, cfg.depth, outs[0].data_ptr(), prec, 0, capi.RT_OUT_RGB_F32,
                               d_segments=segs.data_ptr(), stream=streams[0].cuda_stream)
            torch.cuda.synchronize()
            nseg = int(segs.item())
            segs.zero_()
            for S, bc in [(S, bc) for bc in args.box_cache for S in args.streams]:
                rend.set_option(capi.RT_OPT_BOX_CACHE, bc)
                best = None
                enq = None
                for _ in range(args.reps):
                    # warm-up (row feedback settles), then the timed loop
                    for f in range(64):
                        rend.render_device(cam, cfg.depth, outs[f % S].data_ptr(), prec, 0,
                                           capi.RT_OUT_RGB_F32, stream=streams[f % S].cuda_stream)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for f in range(args.frames):
                        rend.render_device(cam, cfg.depth, outs[f % S].data_ptr(), prec, 0,
                                           capi.RT_OUT_RGB_F32, stream=streams[f % S].cuda_stream)
                    te = time.perf_counter() - t0
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    best = dt if best is None else min(best, dt)
                    enq = te if enq is None else min(enq, te)
                ms = best / args.frames * 1e3
                print(json.dumps({"config": cname, "precision": pname, "streams": S,
                                  "box_cache": bc, "ms_per_frame": round(ms, 5),
                                  "host_enqueue_ms_per_frame": round(enq / args.frames * 1e3, 5),
                                  "grays": round(nseg / (ms * 1e-3) / 1e9, 2)}), flush=True)
        rend.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
