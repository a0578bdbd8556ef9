#!/usr/bin/env python3
"""Kernel-time sweep over configs x precisions on one GPU (HIP events on a dedicated
stream, interleaved rounds in one process — cdna_hip_programming.md §5.4 rule 24).

    python tools/sweep.py [--configs c1,c2,c3,c5] [--precisions f64,mixed,f32] [--reps 20]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3,c5")
    ap.add_argument("--precisions", default="f64,mixed,path64,f32")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sun", action="store_true")
    ap.add_argument("--cull", default="default", help="wave-cull min spheres: default|always|never|N")
    ap.add_argument("--depths", default="", help="comma-separated depths overriding the config's")
    ap.add_argument("--eye", type=int, default=1, help="RT_OPT_EYE_TABLES (0/1)")
    ap.add_argument("--bins", type=int, default=1, help="RT_OPT_TILE_BINS (0/1)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    rend = capi.Renderer(0)
    cull = {"default": None, "always": 0, "never": 2**31 - 1}.get(args.cull, None)
    if cull is None and args.cull != "default":
        cull = int(args.cull)
    if cull is not None:
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, cull)
    rend.set_option(capi.RT_OPT_EYE_TABLES, args.eye)
    rend.set_option(capi.RT_OPT_TILE_BINS, args.bins)
    flags = capi.RT_FLAG_SUN if args.sun else 0
    rows = []
    jobs = []
    for cname in args.configs.split(","):
        cfg = scenes.CONFIGS[cname]
        for dep in ([int(x) for x in args.depths.split(",")] if args.depths else [cfg.depth]):
            jobs.append((cname, cfg, dep))
    for cname, cfg, depth in jobs:
        sc = cfg.scene()
        rend.set_scene(scenes.to_prims(sc))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        out = torch.empty((cam.height, cam.width, 3), dtype=torch.float32, device=dev)
        segs_t = torch.zeros(1, dtype=torch.int64, device=dev)
        precs = args.precisions.split(",")
        times = {p: [] for p in precs}
        segs = None
        for rnd in range(args.rounds):
            for p in precs:
                pc = capi.PRECISIONS[p]
                if segs is None:
                    rend.render_device(cam, depth, out.data_ptr(), pc, flags, 0,
                                       d_segments=segs_t.data_ptr(), stream=stream.cuda_stream)
                    torch.cuda.synchronize()
                    segs = int(segs_t.item())
                for _ in range(2):
                    rend.render_device(cam, depth, out.data_ptr(), pc, flags, 0,
                                       stream=stream.cuda_stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.reps):
                    rend.render_device(cam, depth, out.data_ptr(), pc, flags, 0,
                                       stream=stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / args.reps)
        # diagnostic: cull selectivity (one extra launch with counters on)
        st = torch.zeros(3, dtype=torch.int64, device=dev)
        rend.set_option(capi.RT_OPT_STATS_DEVICE_PTR, st.data_ptr())
        rend.render_device(cam, depth, out.data_ptr(), capi.PRECISIONS[precs[0]], flags, 0,
                           stream=stream.cuda_stream)
        torch.cuda.synchronize()
        rend.set_option(capi.RT_OPT_STATS_DEVICE_PTR, 0)
        culls, kept, considered = (int(v) for v in st.tolist())
        for p in precs:
            ms = min(times[p])
            r = dict(config=cname, depth=depth, precision=p, cull=args.cull, eye=args.eye, ms_min=round(ms, 4),
                     ms_med=round(sorted(times[p])[len(times[p]) // 2], 4), segments=segs,
                     grays=round(segs / (ms * 1e-3) / 1e9, 3), culls=culls,
                     kept_frac=round(kept / considered, 4) if considered else None)
            rows.append(r)
            print(json.dumps(r), flush=True)
    rend.close()


if __name__ == "__main__":
    main()
