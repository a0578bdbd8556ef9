#!/usr/bin/env python3
"""Variance of a short timed region (the driver's 20-step bench) across row-order samples:
in one process, R times — drop the row order (RT_OPT_ROW_FEEDBACK reset), W warmup frames,
sync, K timed frames (frames in flight on F streams, one rt_render_device_frames call each),
sync — and print the region's us/frame per trial, plus the one-stream kernel time after it.

    python tools/region_probe.py [--trials 12] [--steps 20] [--warmup 5] [--fif 2]
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
    ap.add_argument("--trials", type=int, default=12)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fif", type=int, default=2)
    ap.add_argument("--opt", action="append", default=[], help="rt_set_option NAME=VALUE")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS[args.config]
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    rend = capi.Renderer(0)
    rend.set_option(capi.RT_OPT_BOX_CACHE, 0)
    for o in args.opt:
        k, v = o.split("=")
        rend.set_option(getattr(capi, "RT_OPT_" + k), int(v))
    rend.set_scene(scenes.to_prims(cfg.scene()))
    prec = capi.PRECISIONS[args.precision]
    sts = [torch.cuda.Stream(dev) for _ in range(args.fif)]
    outs = [torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
            for _ in range(args.fif)]
    optr = [o.data_ptr() for o in outs]
    sptr = [s.cuda_stream for s in sts]
    # warm the clock
    rend.render_device_frames([cam], cfg.depth, optr, prec, streams=sptr, nframes=2000)
    torch.cuda.synchronize()
    res = []
    for _ in range(args.trials):
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 32)
        rend.render_device_frames([cam], cfg.depth, optr, prec, streams=sptr, nframes=args.warmup)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rend.render_device_frames([cam], cfg.depth, optr, prec, streams=sptr, nframes=args.steps)
        torch.cuda.synchronize()
        region = (time.perf_counter() - t0) / args.steps * 1e6
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sts[0])
        rend.render_device_frames([cam], cfg.depth, optr[:1], prec, streams=sptr[:1], nframes=20)
        e1.record(sts[0])
        torch.cuda.synchronize()
        res.append((round(region, 2), round(e0.elapsed_time(e1) / 20 * 1e3, 2)))
    regs = sorted(r[0] for r in res)
    print(json.dumps({"fif": args.fif, "opts": args.opt, "trials_us_region_kernel": res,
                      "region_median": regs[len(regs) // 2], "region_max": regs[-1]}), flush=True)
    rend.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
