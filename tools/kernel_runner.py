#!/usr/bin/env python3
"""Launch the trace kernel K times on one config/precision (for rocprofv3 runs).

    python tools/kernel_runner.py --config c2 --precision f64 --launches 10
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precision", default="mixed")
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--sun", action="store_true")
    ap.add_argument("--depth", type=int, default=-1, help="-1 = the config's depth")
    ap.add_argument("--lib", default="", help="another build of librt_amd.so (A/B)")
    ap.add_argument("--opt", action="append", default=[],
                    help="rt_set_option NAME=VALUE (e.g. PIXEL_PAIRS=1), repeatable")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    cfg = scenes.CONFIGS[args.config]
    if args.lib:
        capi._lib = capi.load(os.path.abspath(args.lib))
    rend = capi.Renderer(0)
    for o in args.opt:
        name, val = o.split("=")
        rend.set_option(getattr(capi, "RT_OPT_" + name), int(val))
    rend.set_scene(scenes.to_prims(cfg.scene()))
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
    for _ in range(args.launches):
        rend.render_device(cam, cfg.depth if args.depth < 0 else args.depth, out.data_ptr(), capi.PRECISIONS[args.precision],
                           capi.RT_FLAG_SUN if args.sun else 0, capi.RT_OUT_RGB_F32,
                           stream=stream.cuda_stream)
    torch.cuda.synchronize()
    rend.close()


if __name__ == "__main__":
    main()
