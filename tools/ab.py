#!/usr/bin/env python3
"""Interleaved A/B of two builds of librt_amd.so in ONE process (same device, same clock
state — cdna_hip_programming.md §5.4 rule 24).

    python tools/ab.py --a lib/librt_amd.so --b /path/to/other.so --configs c2,c5 --precisions f32
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402
import ctypes as C  # noqa: E402


class Lib:
    def __init__(self, path):
        self.lib = capi.load(path)
        h = C.c_void_p()
        capi.check(self.lib.rt_ctx_create(0, C.byref(h)))
        self.ctx = h

    def set_scene(self, prims):
        arr = (capi.rt_prim * len(prims))(*prims)
        self._arr = arr
        capi.check(self.lib.rt_set_scene(self.ctx, arr, len(prims)))

    def launch(self, cam, depth, d_out, prec, stream):
        capi.check(self.lib.rt_render_device(self.ctx, C.byref(cam), 0, cam.height, depth, prec, 0,
                                             0, C.c_void_p(d_out), None, C.c_void_p(stream)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--more", default="", help="comma-separated extra builds c,d,...")
    ap.add_argument("--configs", default="c2,c5")
    ap.add_argument("--precisions", default="f64,path64,f32")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=VALUE: rt_set_option(RT_OPT_NAME) on every build that knows it")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    libs = {"a": Lib(args.a), "b": Lib(args.b)}
    for k, path in zip("cdefgh", [x for x in args.more.split(",") if x]):
        libs[k] = Lib(path)
    for o in args.opt:
        name, val = o.split("=")
        for L in libs.values():
            # an older build rejects an option it does not know: leave it at its default
            L.lib.rt_set_option(L.ctx, getattr(capi, "RT_OPT_" + name), int(val))
    for cname in args.configs.split(","):
        cfg = scenes.CONFIGS[cname]
        prims = scenes.to_prims(cfg.scene())
        for L in libs.values():
            L.set_scene(prims)
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        out = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
        for pname in args.precisions.split(","):
            prec = capi.PRECISIONS[pname]
            t = {k: [] for k in libs}
            for _ in range(args.rounds):
                for k, L in libs.items():
                    L.launch(cam, cfg.depth, out.data_ptr(), prec, stream.cuda_stream)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        L.launch(cam, cfg.depth, out.data_ptr(), prec, stream.cuda_stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    t[k].append(e0.elapsed_time(e1) / args.reps)
            r = {"config": cname, "precision": pname}
            # same pixels from every build (max |delta| against build a)
            imgs = {}
            for k, L in libs.items():
                o = torch.full_like(out, -1.0)
                torch.cuda.synchronize()  # the fill is on torch's stream, the launch on `stream`
                L.launch(cam, cfg.depth, o.data_ptr(), prec, stream.cuda_stream)
                torch.cuda.synchronize()
                imgs[k] = o
            for k in libs:
                if k != "a":
                    r[k + "_maxdiff"] = float((imgs[k] - imgs["a"]).abs().max())
            for k in libs:
                r[k + "_ms"] = round(min(t[k]), 4)
            for k in libs:
                if k != "a":
                    r[k + "_over_a"] = round(min(t[k]) / min(t["a"]), 3)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
