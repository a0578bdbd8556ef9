#!/usr/bin/env python3
"""In-process A/B of the two frame-loop paths at N = 1 (bench.py's tiled vs frames modes):
rt_multi_render_device_frames (one-rank MultiRenderer) and rt_render_device_frames (plain
Renderer), 200-frame loops of c2 on two streams, interleaved rounds."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [torch.empty((cam.height, cam.width, 3), device=dev) for _ in range(2)]
    op = [o.data_ptr() for o in outs]
    sp = [s.cuda_stream for s in sts]
    fb = int(os.environ.get("FB", "32"))
    r = capi.Renderer(0)
    r.set_option(capi.RT_OPT_BOX_CACHE, 0)
    r.set_option(capi.RT_OPT_ROW_FEEDBACK, fb)
    r.set_scene(prims)
    ema = os.environ.get("EMA")
    if ema is not None:   # A/B of the row-feedback smoothing: "multi" = a second plain ctx
        r.set_option(capi.RT_OPT_ROW_FEEDBACK_EMA, 0)
        m = capi.Renderer(0)
        m.set_option(capi.RT_OPT_ROW_FEEDBACK_EMA, int(ema))
    else:
        m = capi.MultiRenderer([0])
    m.set_option(capi.RT_OPT_BOX_CACHE, 0)
    m.set_option(capi.RT_OPT_ROW_FEEDBACK, fb)
    m.set_scene(prims)
    n = int(os.environ.get("N", "200"))

    def run(which):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sts[0])
        sts[1].wait_stream(sts[0])
        if which == "multi" and ema is not None:
            m.render_device_frames([cam], cfg.depth, op, capi.RT_PREC_PATH64, streams=sp, nframes=n)
        elif which == "multi":
            m.render_device_frames([cam], cfg.depth, op, capi.RT_PREC_PATH64, streams=sp, nframes=n)
        else:
            r.render_device_frames([cam], cfg.depth, op, capi.RT_PREC_PATH64, streams=sp, nframes=n)
        sts[0].wait_stream(sts[1])
        e1.record(sts[0])
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    for w in ("multi", "plain"):
        run(w)
    res = {"multi": [], "plain": []}
    for _ in range(int(os.environ.get("ROUNDS", "6"))):
        for w in ("multi", "plain"):
            res[w].append(round(run(w), 2))
    print(json.dumps({"row_feedback": fb, "ema_b": ema, "us_per_frame": res, "median": {k: sorted(v)[len(v) // 2] for k, v in res.items()}}))


if __name__ == "__main__":
    main()
