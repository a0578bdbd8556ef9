#!/usr/bin/env python3
"""Launch a sequence of (scene, depth, precision) setups, `--launches` each, in one process,
for a rocprofv3 --pmc pass: per-dispatch counters then attribute instruction counts to
the parts of the path (primary scan vs bounces, spheres vs walls, shading floor).

    python tools/pmc_breakdown.py --setups c2:4:path64,c2:0:path64,s8w0:0:path64 > order.json
A setup is CONFIG:DEPTH:PRECISION where CONFIG is a config name (c1..c5) at its size or
sNwM = synthetic_scene(N, M) at 1920x1080.
"""
import argparse
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--setups", required=True)
    ap.add_argument("--launches", type=int, default=3)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    rend = capi.Renderer(0)
    segs_t = torch.zeros(1, dtype=torch.int64, device=dev)
    order = []
    for su in args.setups.split(","):
        name, depth, prec = su.split(":")
        m = re.fullmatch(r"s(\d+)w(\d+)", name)
        if m:
            sc, w, h = scenes.synthetic_scene(int(m.group(1)), int(m.group(2))), 1920, 1080
        else:
            cfg = scenes.CONFIGS[name]
            sc, w, h = cfg.scene(), cfg.width, cfg.height
        rend.set_scene(scenes.to_prims(sc))
        cam = capi.camera_init(**scenes.camera_args(w, h))
        out = torch.empty((h, w, 3), dtype=torch.float32, device=dev)
        segs_t.zero_()
        for k in range(args.launches):
            rend.render_device(cam, int(depth), out.data_ptr(), capi.PRECISIONS[prec], 0,
                               capi.RT_OUT_RGB_F32, d_segments=segs_t.data_ptr() if k == 0 else 0,
                               stream=stream.cuda_stream)
        torch.cuda.synchronize()
        order.append(dict(setup=su, launches=args.launches, segments=int(segs_t.item()),
                          pixels=w * h))
    rend.close()
    print(json.dumps(order))


if __name__ == "__main__":
    main()
