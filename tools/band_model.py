#!/usr/bin/env python3
"""Inputs of the row-tiled scaling model, measured on ONE MI355X: for each
split N in {1, 2, 4, 8} of a config's frame into rt_band_rows bands, every band's
one-stream kernel time (its own ctx, measured row order warm, HIP events around
back-to-back launches), its host time per frame (rt_render_device with the GPU held busy),
and the bytes it sends to the root.  The gather term needs the xGMI link rate, which one
GPU cannot measure: the model takes it as a parameter.
With --layout interleaved the parts are rt_interleaved_rows parts (tile rows dealt
round-robin, rt_render_device_interleaved), launched one at a time behind a GPU spin.
With --frame-batch B (contiguous / weighted bands) each band is also measured the way a rank
runs it under RT_OPT_FRAME_BATCH: its frames on ONE stream into B distinct buffers, B frames
per launch — GPU time per frame (kernel_us_fbB) and host time per frame behind a GPU spin
(host_us_fbB).
    python tools/band_model.py [--config c2] [--precision path64] [--layout contiguous]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def pipelined_us(torch, st, st2, launch_on, n, extra=(), frames=None):
    """Per-frame GPU time of n frames round-robin over 2 + len(extra) streams (frames in
    flight: one frame's tail overlaps the next ones' start, as in bench.py's frame loop).
    A first untimed pass warms every stream (its first launch carries one-time costs).
    frames(streams, m): enqueue m frames by one C-ABI call (rt_render_device_frames, as a
    rank's frame loop does: no Python between frames); else launch_on(stream, buf) per frame."""
    sts = [st, st2] + list(extra)
    for timed in (False, True):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for s_ in sts[1:]:
            s_.wait_stream(st)
        m = n if timed else len(sts)
        if frames is not None:
            frames(sts, m)
        for k in range(m if frames is None else 0):
            launch_on(sts[k % len(sts)], k % 2)
        for s_ in sts[1:]:
            st.wait_stream(s_)
        e1.record(st)
        torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n * 1e3, 2)


def interleaved_part(capi, torch, st, cam, depth, prec, prims, out, segs, N, r, n, st2=None, out2=None,
                     extra=()):
    """One interleaved part's kernel / host time per frame and the bytes it sends."""
    W = cam.width
    nr = capi.interleaved_rows(cam.height, N, r)
    rend = capi.Renderer(0)
    rend.set_scene(prims)

    def launch(d_seg=0):
        rend.render_device_interleaved(cam, depth, N, r, out.data_ptr(), prec,
                                       d_segments=d_seg, stream=st.cuda_stream)

    def launch_on(s, b):
        rend.render_device_interleaved(cam, depth, N, r, (out, out2)[b].data_ptr(), prec,
                                       stream=s.cuda_stream)
    for _ in range(40):
        launch()
    segs.zero_()
    launch(segs.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):   # the launches queue behind the spin: e0..e1 is GPU time only
        torch.cuda._sleep(int(2e8))
    e0.record(st)
    t0 = time.perf_counter()
    for _ in range(n):
        launch()
    host_us = (time.perf_counter() - t0) / n * 1e6
    e1.record(st)
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / n
    fif2 = pipelined_us(torch, st, st2, launch_on, n)
    fif4 = pipelined_us(torch, st, st2, launch_on, n, extra)
    rend.close()
    return {"rank": r, "nrows": nr, "kernel_us": round(kms * 1e3, 2), "kernel_us_fif2": fif2,
            "kernel_us_fif4": fif4,
            "host_us": round(host_us, 2), "segments": int(segs.item()),
            "send_bytes_f32": 0 if r == 0 else nr * W * 12,
            "send_bytes_rgba8": 0 if r == 0 else nr * W * 4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--precision", default="path64")
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--frame-batch", type=int, default=0,
                    help="also time B frames per launch (RT_OPT_FRAME_BATCH)")
    ap.add_argument("--frame-streams", type=int, default=1,
                    help="with --frame-batch: consecutive blocks of B frames go to S streams in "
                         "turn (S launches of B frames in flight)")
    ap.add_argument("--layout", choices=("contiguous", "interleaved", "weighted"), default="contiguous",
                    help="weighted: contiguous bands cut by rt_weighted_band_rows over the "
                         "measured tile-row costs of one full-frame render (rt_tile_row_costs)")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    cfg = scenes.CONFIGS[args.config]
    prims = scenes.to_prims(cfg.scene())
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    H, W = cam.height, cam.width
    prec = capi.PRECISIONS[args.precision]
    out = torch.empty((H, W, 3), device=dev)
    out2 = torch.empty((H, W, 3), device=dev)
    st2 = torch.cuda.Stream(dev)
    extra = [torch.cuda.Stream(dev) for _ in range(2)]   # 4 frames in flight
    segs = torch.zeros(1, dtype=torch.int64, device=dev)
    n = args.launches
    res = {"config": args.config, "precision": args.precision, "width": W, "height": H,
           "layout": args.layout, "frame_batch": args.frame_batch, "frame_streams": args.frame_streams,
           "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "splits": {}}
    inter = args.layout == "interleaved"
    weights = None
    if args.layout == "weighted":
        wr = capi.Renderer(0)
        wr.set_scene(prims)
        weights = wr.tile_row_costs(cam, cfg.depth, prec)
        wr.close()
        res["weights"] = [round(float(x), 1) for x in weights]
    for N in [int(x) for x in args.splits.split(",")]:
        bands = []
        for r in range(N):
            if inter:
                bands.append(interleaved_part(capi, torch, st, cam, cfg.depth, prec, prims, out,
                                              segs, N, r, n, st2, out2, extra))
                continue
            r0, nr = (capi.weighted_band_rows(H, N, r, weights) if weights is not None
                      else capi.band_rows(H, N, r))
            rend = capi.Renderer(0)
            rend.set_scene(prims)
            for _ in range(40):   # warm: the measured row order for this band settles
                rend.render_device(cam, cfg.depth, out.data_ptr(), prec, row0=r0, nrows=nr,
                                   stream=st.cuda_stream)
            segs.zero_()
            rend.render_device(cam, cfg.depth, out.data_ptr(), prec, row0=r0, nrows=nr,
                               d_segments=segs.data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            rend.render_device_frames([cam], cfg.depth, [out.data_ptr()], prec, row0=r0, nrows=nr,
                                      streams=[st.cuda_stream], nframes=n)
            e1.record(st)
            torch.cuda.synchronize()
            kms = e0.elapsed_time(e1) / n
            # host time per frame: launches queued behind a GPU spin, so the host never waits
            with torch.cuda.stream(st):
                torch.cuda._sleep(int(2e8))
            t0 = time.perf_counter()
            rend.render_device_frames([cam], cfg.depth, [out.data_ptr()], prec, row0=r0, nrows=nr,
                                      streams=[st.cuda_stream], nframes=n)
            host_us = (time.perf_counter() - t0) / n * 1e6
            torch.cuda.synchronize()
            lo = lambda s_, b: rend.render_device(cam, cfg.depth, (out, out2)[b].data_ptr(), prec,
                                                  row0=r0, nrows=nr, stream=s_.cuda_stream)
            fr = lambda sts_, m: rend.render_device_frames(
                [cam], cfg.depth, [out.data_ptr(), out2.data_ptr()], prec, row0=r0, nrows=nr,
                streams=[x.cuda_stream for x in sts_], nframes=m)
            fif2 = pipelined_us(torch, st, st2, lo, n, frames=fr)
            fif4 = pipelined_us(torch, st, st2, lo, n, extra, frames=fr)
            fbk = {}
            if args.frame_batch > 1:
                B = args.frame_batch
                S = max(1, min(4, args.frame_streams))
                rend.set_option(capi.RT_OPT_FRAME_BATCH, B)
                bufs = [out, out2] + [torch.empty((nr, W, 3), device=dev) for _ in range(B * S - 2)]
                ptrs = [b_.data_ptr() for b_ in bufs[:B * S]]
                fst = ([st, st2] + list(extra))[:S]
                sps = [s_.cuda_stream for s_ in fst for _ in range(B)]  # blocks of B frames per stream
                for timed in (False, True):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                    for s_ in fst[1:]:
                        s_.wait_stream(st)
                    rend.render_device_frames([cam], cfg.depth, ptrs, prec, row0=r0, nrows=nr,
                                              streams=sps, nframes=n if timed else 2 * B * S)
                    for s_ in fst[1:]:
                        st.wait_stream(s_)
                    e1.record(st)
                    torch.cuda.synchronize()
                fbk[f"kernel_us_fb{B}"] = round(e0.elapsed_time(e1) / n * 1e3, 2)
                for s_ in fst:
                    with torch.cuda.stream(s_):
                        torch.cuda._sleep(int(2e8))
                t0 = time.perf_counter()
                rend.render_device_frames([cam], cfg.depth, ptrs, prec, row0=r0, nrows=nr,
                                          streams=sps, nframes=n)
                fbk[f"host_us_fb{B}"] = round((time.perf_counter() - t0) / n * 1e6, 2)
                torch.cuda.synchronize()
                rend.set_option(capi.RT_OPT_FRAME_BATCH, 1)
                del bufs
            rend.close()
            bands.append({"rank": r, "row0": r0, "nrows": nr, "kernel_us": round(kms * 1e3, 2),
                          "kernel_us_fif2": fif2, "kernel_us_fif4": fif4, **fbk,
                          "host_us": round(host_us, 2), "segments": int(segs.item()),
                          "send_bytes_f32": 0 if r == 0 else nr * W * 12,
                          "send_bytes_rgba8": 0 if r == 0 else nr * W * 4})
        res["splits"][N] = {
            "bands": bands,
            "max_kernel_us": max(b["kernel_us"] for b in bands),
            "max_kernel_us_fif2": max(b["kernel_us_fif2"] for b in bands),
            "max_kernel_us_fif4": max(b["kernel_us_fif4"] for b in bands),
            "max_host_us": max(b["host_us"] for b in bands),
            **({f"max_kernel_us_fb{args.frame_batch}": max(b[f"kernel_us_fb{args.frame_batch}"] for b in bands),
                f"max_host_us_fb{args.frame_batch}": max(b[f"host_us_fb{args.frame_batch}"] for b in bands)}
               if args.frame_batch > 1 and not inter else {}),
            "root_in_bytes_f32": sum(b["send_bytes_f32"] for b in bands),
            "root_in_bytes_rgba8": sum(b["send_bytes_rgba8"] for b in bands),
            "max_link_bytes_f32": max(b["send_bytes_f32"] for b in bands),
        }
        print(json.dumps({"N": N, **{k: v for k, v in res["splits"][N].items() if k != "bands"}}),
              file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
