#!/usr/bin/env python3
"""Distribution of the driver's timed window: W windows of K consecutive frames (bench.py's
timed loop: frames in flight on F streams, one C-ABI call per window), each bracketed by a
device synchronize, after a 200-frame warm loop — per window the wall-clock and stream-event
ms/frame.  Several option sets run one after another in one process, each on a fresh
renderer (--variants 'name:OPT=V,OPT=V;name2:...', option names without RT_OPT_).

    python tools/window_probe.py --windows 30 --steps 20 --variants 'base:;iso0:ROW_FEEDBACK_ISOLATE=0'
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precision", default="path64")
    ap.add_argument("--windows", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--fif", type=int, default=2, help="streams (frames round-robin over them)")
    ap.add_argument("--bufs", type=int, default=0, help="frame buffers (default: one per stream)")
    ap.add_argument("--lib", default="", help="another build of librt_amd.so")
    ap.add_argument("--warm", type=int, default=200)
    ap.add_argument("--variants", default="base:")
    ap.add_argument("--clock", action="store_true",
                    help="bracket every window with a shader-clock probe (tools/ubench/"
                         "libclock_probe.so, ~2 us each): MHz before and after the window")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="host sleep between windows (idle GPU), to see clocks drop")
    ap.add_argument("--clock-during", type=int, default=0,
                    help="also run the clock probe on a side stream DURING the window, spinning "
                         "this many 10-ns ticks (the shader clock under the window's load)")
    ap.add_argument("--gap-spin", action="store_true",
                    help="fill the gap with a GPU spin kernel instead of idling")
    ap.add_argument("--lead", type=int, default=0,
                    help="frames run (untimed, then one sync) right before each timed window, "
                         "after the gap: bench.py's steady-state loop + warmup in front of its "
                         "timed region")
    args = ap.parse_args()
    import ctypes as C
    import torch
    dev = torch.device("cuda", 0)
    if args.lib:
        capi._lib = capi.load(os.path.abspath(args.lib))
    cfg = scenes.CONFIGS[args.config]
    prims = scenes.to_prims(cfg.scene())
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    prec = capi.PRECISIONS[args.precision]
    streams = [torch.cuda.Stream(dev) for _ in range(args.fif)]
    clk = None
    if args.clock:   # (after torch's HIP runtime is up: the probe library links the same one)
        capi.load()
        clk = C.CDLL(os.path.join(REPO, "tools", "ubench", "libclock_probe.so"))
        clk.clock_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_ulonglong]
    sp = [s.cuda_stream for s in streams]
    outs = [torch.empty((cam.height, cam.width, 3), device=dev) for _ in range(args.bufs or args.fif)]
    ptrs = [o.data_ptr() for o in outs]
    segs = torch.zeros(1, dtype=torch.int64, device=dev)
    vars_ = []
    for spec in args.variants.split(";"):   # every renderer first, warmed
        name, _, opts = spec.partition(":")
        r = capi.Renderer(0)
        r.set_option(capi.RT_OPT_BOX_CACHE, 0)
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=")
            r.set_option(getattr(capi, "RT_OPT_" + k), int(v))
        r.set_scene(prims)
        segs.zero_()
        r.render_device(cam, cfg.depth, ptrs[0], prec, d_segments=segs.data_ptr(), stream=sp[0])
        torch.cuda.synchronize()
        nseg = int(segs.item())
        r.render_device_frames([cam], cfg.depth, ptrs, prec, streams=sp, nframes=args.warm)
        torch.cuda.synchronize()
        vars_.append({"name": name, "opts": opts, "r": r, "nseg": nseg, "wall": [], "gpu": []})
    cbuf = torch.zeros((max(1, args.windows * len(vars_)), 3, 2), dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    T0 = time.perf_counter()
    wi = 0
    # windows interleaved across the variants (drift of clocks/box cancels out)
    for _ in range(args.windows):
        for v in vars_:
            torch.cuda.synchronize()
            if args.gap_ms > 0:
                if args.gap_spin:
                    with torch.cuda.stream(streams[0]):
                        torch.cuda._sleep(int(args.gap_ms * 2.4e6))
                    torch.cuda.synchronize()
                else:
                    time.sleep(args.gap_ms * 1e-3)
            if args.lead > 0:
                v["r"].render_device_frames([cam], cfg.depth, ptrs, prec, streams=sp, nframes=args.lead)
                torch.cuda.synchronize()
            if clk is not None:
                clk.clock_probe(C.c_void_p(sp[0]), C.c_void_p(cbuf[wi, 0].data_ptr()), 200)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            v.setdefault("t", []).append(round((t0 - T0) * 1e3, 2))
            e0.record(streams[0])
            for s in streams[1:]:
                s.wait_stream(streams[0])
            tc = time.perf_counter()
            if clk is not None and args.clock_during > 0:
                side.wait_stream(streams[0])
                clk.clock_probe(C.c_void_p(side.cuda_stream), C.c_void_p(cbuf[wi, 2].data_ptr()),
                                args.clock_during)
            v["r"].render_device_frames([cam], cfg.depth, ptrs, prec, streams=sp, nframes=args.steps)
            v.setdefault("host", []).append((time.perf_counter() - tc) / args.steps * 1e3)
            for s in streams[1:]:
                streams[0].wait_stream(s)
            e1.record(streams[0])
            if clk is not None:
                clk.clock_probe(C.c_void_p(sp[0]), C.c_void_p(cbuf[wi, 1].data_ptr()), 200)
            torch.cuda.synchronize()
            v["wall"].append((time.perf_counter() - t0) / args.steps * 1e3)
            v["gpu"].append(e0.elapsed_time(e1) / args.steps)
            v.setdefault("wi", []).append(wi)
            wi += 1
    for v in vars_:
        v["r"].close()
        wall, gpu = v["wall"], v["gpu"]
        q = sorted(wall)
        res = {"variant": v["name"], "options": v["opts"], "config": cfg.name, "precision": args.precision,
               "steps": args.steps, "fif": args.fif, "windows": args.windows,
               "wall_ms_median": round(statistics.median(wall), 4), "wall_ms_min": round(q[0], 4),
               "wall_ms_p90": round(q[int(0.9 * (len(q) - 1))], 4), "wall_ms_max": round(q[-1], 4),
               "gpu_ms_median": round(statistics.median(gpu), 4),
               "grays_median": round(v["nseg"] / (statistics.median(wall) * 1e-3) / 1e9, 1),
               "wall_ms": [round(x, 4) for x in wall],
               "gpu_ms": [round(x, 4) for x in gpu],
               "host_call_ms_per_frame": [round(x, 4) for x in v["host"]],
               "t_ms": v["t"]}
        if clk is not None:
            cb = cbuf.cpu().numpy()
            mhz = lambda a: round(100.0 * float(a[0]) / max(1.0, float(a[1])), 1)
            res["mhz_before"] = [mhz(cb[w, 0]) for w in v["wi"]]
            res["mhz_after"] = [mhz(cb[w, 1]) for w in v["wi"]]
            if args.clock_during > 0:
                res["mhz_during"] = [mhz(cb[w, 2]) for w in v["wi"]]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
