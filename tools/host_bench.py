#!/usr/bin/env python3
"""Per-frame host work of a render on the CPU (no device): a diagnostic build of the C-ABI
(-DRT_HOST_BENCH=1) times make_params (pixel boxes, mirror chains, eye tables, arguments),
frame_boxes alone and the KParams copy, for a config's full frame and its 1/8 bands.

    tools/build_variant.sh hb -DRT_AB_SLIM=1 -DRT_HOST_BENCH=1
    python tools/host_bench.py --lib ray-tracer-from-scratch_amd/lib/ab/hb.so --config c2"""
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
    ap.add_argument("--lib", required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--iters", type=int, default=3000)
    args = ap.parse_args()
    lib = capi.load(os.path.abspath(args.lib))
    lib.rt_host_bench.restype = C.c_int
    cfg = scenes.CONFIGS[args.config]
    prims = scenes.to_prims(cfg.scene())
    arr = (capi.rt_prim * len(prims))(*prims)
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = (C.c_double * 4)()
    bands = [(0, cam.height)] + [capi.band_rows(cam.height, 8, r) for r in range(8)]
    for r0, nr in bands:
        capi.check(lib.rt_host_bench(arr, len(prims), C.byref(cam), r0, nr, args.iters, out))
        print(json.dumps({"config": args.config, "row0": r0, "nrows": nr,
                          "make_params_us": round(out[0], 3), "frame_boxes_us": round(out[1], 3),
                          "kparams_copy_us": round(out[2], 3)}), flush=True)


if __name__ == "__main__":
    main()
