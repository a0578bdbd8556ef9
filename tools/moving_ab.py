#!/usr/bin/env python3
"""Fly-through A/B of RT_OPT_ROW_FEEDBACK intervals: 200 frames, the camera moving `step`
scene units per frame along +x; per-frame stream time (min of 2 passes)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precision", default="path64")
    ap.add_argument("--values", default="0,4,8,16,32")
    ap.add_argument("--steps", default="0.0,0.002,0.01,0.03")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    rend = capi.Renderer(0)
    rend.set_option(capi.RT_OPT_BOX_CACHE, 0)
    cfg = scenes.CONFIGS[args.config]
    rend.set_scene(scenes.to_prims(cfg.scene()))
    ca = scenes.camera_args(cfg.width, cfg.height)
    out = torch.empty((cfg.height, cfg.width, 3), dtype=torch.float32, device=dev)
    pc = capi.PRECISIONS[args.precision]
    for step in [float(x) for x in args.steps.split(",")]:
        cams = []
        for f in range(200):
            a = dict(ca)
            a["position"] = (ca["position"][0] + step * f, ca["position"][1], ca["position"][2])
            a["lookat"] = (ca["lookat"][0] + step * f, ca["lookat"][1], ca["lookat"][2])
            cams.append(capi.camera_init(**a))
        r = {"config": args.config, "step": step}
        for v in [int(x) for x in args.values.split(",")]:
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK, v)
            best = None
            for _ in range(2):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for c in cams:
                    rend.render_device(c, cfg.depth, out.data_ptr(), pc, 0, 0,
                                       stream=stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / len(cams)
                best = ms if best is None else min(best, ms)
            r[f"us[{v}]"] = round(best * 1000, 2)
        print(json.dumps(r), flush=True)
    rend.close()


if __name__ == "__main__":
    main()
