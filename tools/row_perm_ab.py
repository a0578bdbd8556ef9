#!/usr/bin/env python3
"""A/B of explicit tile-row dispatch orders (rt_set_row_order) on one config: the default
centre-out order vs permutations from a JSON {name: [rows...]}; checks identical pixels."""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--perms", required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precisions", default="path64,f32,f64")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    import torch
    perms = json.load(open(args.perms))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    lib = capi.load()
    h = C.c_void_p()
    capi.check(lib.rt_ctx_create(0, C.byref(h)))
    cfg = scenes.CONFIGS[args.config]
    prims = scenes.to_prims(cfg.scene())
    arr = (capi.rt_prim * len(prims))(*prims)
    capi.check(lib.rt_set_scene(h, arr, len(prims)))
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    H = cam.height

    def setp(name):
        if name == "default":
            capi.check(lib.rt_set_row_order(h, None, 0))
        else:
            v = perms[name]
            a = (C.c_int16 * len(v))(*v)
            capi.check(lib.rt_set_row_order(h, a, len(v)))

    for pname in args.precisions.split(","):
        pc = capi.PRECISIONS[pname]
        names = ["default"] + list(perms)
        outs = {n: torch.empty((H, cam.width, 3), dtype=torch.float32, device=dev) for n in names}

        def launch(n):
            capi.check(lib.rt_render_device(h, C.byref(cam), 0, H, cfg.depth, pc, 0, 0,
                                            C.c_void_p(outs[n].data_ptr()), None,
                                            C.c_void_p(stream.cuda_stream)))
        t = {n: [] for n in names}
        for _ in range(args.rounds):
            for n in names:
                setp(n)
                launch(n)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.reps):
                    launch(n)
                e1.record(stream)
                torch.cuda.synchronize()
                t[n].append(e0.elapsed_time(e1) / args.reps)
        r = {"config": args.config, "precision": pname}
        for n in names:
            r[n + "_us"] = round(1000 * min(t[n]), 2)
            if n != "default":
                r[n + "_same"] = bool(torch.equal(outs[n], outs["default"]))
        print(json.dumps(r), flush=True)
    capi.check(lib.rt_set_row_order(h, None, 0))
    lib.rt_ctx_destroy(h)


if __name__ == "__main__":
    main()
