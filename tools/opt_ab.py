#!/usr/bin/env python3
"""Interleaved in-process A/B of an rt_set_option value (same device, same clock state):

    python tools/opt_ab.py --option TILE_BINS --values 0,1 --configs c1,c2 --precisions path64,f64

Times back-to-back rt_render_device launches (HIP events on one stream), min over rounds."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--option", default="TILE_BINS")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--configs", default="c1,c2")
    ap.add_argument("--precisions", default="path64,f64,mixed")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sun", action="store_true")
    ap.add_argument("--depth", type=int, default=-1, help="-1 = the config's depth")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    rend = capi.Renderer(0)
    opt = getattr(capi, "RT_OPT_" + args.option)
    vals = [int(v) for v in args.values.split(",")]
    flags = capi.RT_FLAG_SUN if args.sun else 0
    for cname in args.configs.split(","):
        cfg = scenes.CONFIGS[cname]
        rend.set_scene(scenes.to_prims(cfg.scene()))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        out = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
        for pname in args.precisions.split(","):
            pc = capi.PRECISIONS[pname]
            t = {v: [] for v in vals}
            for _ in range(args.rounds):
                for v in vals:
                    rend.set_option(opt, v)
                    for _ in range(2):
                        rend.render_device(cam, (cfg.depth if args.depth < 0 else args.depth), out.data_ptr(), pc, flags, 0,
                                           stream=stream.cuda_stream)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        rend.render_device(cam, (cfg.depth if args.depth < 0 else args.depth), out.data_ptr(), pc, flags, 0,
                                           stream=stream.cuda_stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    t[v].append(e0.elapsed_time(e1) / args.reps)
            r = {"config": cname, "precision": pname, "option": args.option}
            for v in vals:
                r[f"ms[{v}]"] = round(min(t[v]), 4)
            for v in vals[1:]:
                r[f"ratio[{v}/{vals[0]}]"] = round(min(t[v]) / min(t[vals[0]]), 3)
            print(json.dumps(r), flush=True)
    rend.close()


if __name__ == "__main__":
    main()
