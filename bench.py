#!/usr/bin/env python3
"""bench.py — Mrays/s + ms/frame of the MI355X trace/shade path (BASELINE.json metric).

A "step" is one pass of the hot path over one batch of synthetic input: every rank
renders one full frame of the configured scene (default c2: 1920x1080, 8 spheres +
4 walls, reflection depth 4) into HBM through the C-ABI (rt_render_device), the scene
already resident on the device.  With N ranks the batch is N frames of a camera
fly-through (rank r renders frame r: the camera moved r steps forward the way
Camera::forward moves it, scene.cpp:121) — frames are independent units, sharded with
no data-path collective, so `scaling` is "weak".  Consecutive frames of a rank go to
`--frames-in-flight` output buffers on as many streams (default 2, a double-buffered frame
loop): every frame is rendered in full, and one frame's last (heaviest) waves overlap the
next frame's first instead of leaving the GPU draining between launches; `kernel_ms` is
the one-frame-at-a-time kernel duration.  `--mode tiled` instead splits ONE
frame into row bands across ranks and gathers them to rank 0 (RCCL), the strong-scaling
layout of BASELINE config 4.

Rays = segments = closest-hit queries (primary + reflection), counted exactly by the
kernel in an untimed census launch.

Order of a run: census; the side measurements (per-precision sweep, sun extension, moving
camera — before the timed region, so it starts on a GPU at its running clock rather than
on the ramp out of idle); W warmup steps; K timed steps; the one-stream kernel time.  The
warmup and timed steps of frames mode are enqueued by one rt_render_device_frames call
each (every frame's own host work and launch, as a C++ frame loop over rt_render_device
would do them, without Python's per-call overhead).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--precision mixed]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))

from rtamd import capi, scenes  # noqa: E402

METRIC = "Mrays/sec + ms/frame at 1920×1080 depth=4; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
VALU_PEAK_TFLOPS = {"f32": 157.3, "mixed": 157.3, "path64": 157.3, "f64": 78.6}  # spec
DTYPE = {"f64": "f64", "mixed": "f64", "path64": "f64+f32", "f32": "f32"}
PARITY = {  # what each precision guarantees vs the reference (tests/test_gpu_parity.py)
    "f64": "per-pixel |delta| <= 1e-12 vs the reference's fp64 frames",
    "mixed": "bit-identical to f64",
    "path64": "exact fp64 ray paths (hits, normals, reflections); fp32 colour: every pixel "
              "within 2e-5 of the reference, no discontinuity flips",
    "f32": "|delta| <= 1e-4 on >= 99.5% of pixels at depth <= 4 (flips at discontinuities)",
}


def flop_per_segment(n_sph: int, n_wall: int) -> int:
    """SURVEY §8d convention: F_seg = 30*N_sphere + 38*N_wall + 60 (FMA = 2)."""
    return 30 * n_sph + 38 * n_wall + 60


def scene_bytes(n_sph: int, n_wall: int, n_prim: int) -> int:
    return 64 * n_sph + 176 * n_wall + 64 * n_prim   # DevSphere / DevWall / DevMat records


def cpu_baseline(cfg, prims, cam, depth, flags, budget_s: float):
    """The oracle's OpenMP restatement (the 'OpenMP CPU path') on this host's cores, on a
    bounded sample of the same frame: a centred band of rows sized to ~budget_s."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc_mod   # test infrastructure: the timed CPU baseline leg only
    orc = orc_mod.Oracle()
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    H = cam.height
    probe = min(H, 16)
    r0 = max(0, H // 2 - probe // 2)
    t = time.perf_counter()
    orc.render(prims, cam, depth, flags, row0=r0, nrows=probe, nthreads=cores, want64=False)
    per_row = max(1e-6, (time.perf_counter() - t) / probe)
    rows = int(min(H, max(probe, budget_s / per_row)))
    r0 = max(0, H // 2 - rows // 2)
    # repeat the band until the budget is spent (small frames finish in milliseconds)
    segs, dt, reps = 0, 0.0, 0
    while reps == 0 or (dt < budget_s and reps < 10000):
        t = time.perf_counter()
        _, _, s = orc.render(prims, cam, depth, flags, row0=r0, nrows=rows, nthreads=cores,
                             want64=False)
        dt += time.perf_counter() - t
        segs += s
        reps += 1
    return {"value": round(segs / dt / 1e6, 3), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "sample": f"{reps} x rows {r0}..{r0 + rows - 1} of the same {cam.width}x{H} frame "
                      f"({rows * cam.width} px, {segs} segments in {dt:.2f} s), fp64 oracle "
                      f"restatement (-O2, no FMA), OpenMP schedule(dynamic,1) over rows",
            "ms_per_frame": round(dt / reps / rows * H * 1e3, 2)}


def load_traffic(path: str, workload: str, precision: str):
    """Per-launch HBM bytes measured by rocprofv3 --pmc (profiles/)."""
    try:
        with open(path) as fh:
            d = json.load(fh)
        e = d.get(workload, {}).get(precision)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(scenes.CONFIGS))
    ap.add_argument("--precision", default="path64", choices=sorted(capi.PRECISIONS))
    ap.add_argument("--mode", default="frames", choices=["frames", "tiled"])
    ap.add_argument("--out", default="rgb_f32", choices=["rgb_f32", "rgba8"],
                    help="timed output format: linear fp32 RGB (12 B/px, parity buffer) or the "
                         "clamp+truncate RGBA8 epilogue (4 B/px; cuts the tiled gather 3x)")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="frames mode: consecutive frames go to F output buffers on F streams "
                         "(a triple-buffered frame loop), so one frame's last waves overlap the "
                         "next frame's first; 1 = one stream, frames back to back")
    ap.add_argument("--sun", action="store_true", help="build-defined sun term (off = parity)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true", help="skip the per-precision kernel sweep")
    ap.add_argument("--row-feedback", type=int, default=32,
                    help="RT_OPT_ROW_FEEDBACK: refresh interval (frames) of the measured "
                         "tile-row dispatch order, 0 = off (scheduling only)")
    ap.add_argument("--box-cache", type=int, default=0, choices=[0, 1],
                    help="RT_OPT_BOX_CACHE: reuse the host's per-frame pixel boxes when the "
                         "camera is unchanged (0 = recompute every frame)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # RT_BENCH_BACKEND=gloo: rehearsal of the N-rank code path on fewer GPUs than ranks
    # (ranks share devices round-robin; RCCL refuses two ranks on one GPU).  Not a
    # measurement: the driver's multi-GPU runs use the default, RCCL ("nccl").
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            dist.barrier()

    cfg = scenes.CONFIGS[args.config]
    sc = cfg.scene()
    prims = scenes.to_prims(sc)
    n_sph = sum(1 for o in sc if o.kind == capi.RT_PRIM_SPHERE)
    n_wall = len(sc) - n_sph
    prec = capi.PRECISIONS[args.precision]
    flags = capi.RT_FLAG_SUN if args.sun else 0
    depth = cfg.depth

    rend = capi.Renderer(local)
    rend.set_option(capi.RT_OPT_BOX_CACHE, args.box_cache)
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)
    rend.set_scene(prims)
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    W, H = cam.width, cam.height
    if args.mode == "frames":
        # frame `rank` of a fly-through: Camera::forward moves position by
        # forward_vec()*movement_speed = (1,0,0)*0.1 and never re-calls init().
        cam.position[0] += 0.1 * rank
        row0, nrows = 0, H
    else:
        row0, nrows = capi.band_rows(H, world, rank)
    band_max = -(-H // world) if args.mode == "tiled" else H

    # dedicated streams: the C-ABI maps a NULL stream to its own, so torch's legacy
    # default stream (handle 0) would put the launches and the timing events apart
    fif = max(1, args.frames_in_flight) if args.mode == "frames" else 1
    streams = [torch.cuda.Stream(dev) for _ in range(fif)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    # sized for fp32 RGB: the per-precision sweep below always writes 12 B/px into them;
    # frames in flight: one output buffer per stream (every frame is rendered in full)
    outs = [torch.empty((band_max, W, 3), dtype=torch.float32, device=dev) for _ in range(fif)]
    out = outs[0]
    out_fmt = capi.RT_OUT_RGBA8 if args.out == "rgba8" else capi.RT_OUT_RGB_F32
    segs_t = torch.zeros(1, dtype=torch.int64, device=dev)

    def launch(d_segs: int = 0, dst=None, slot: int = 0):
        rend.render_device(cam, depth, (dst if dst is not None else outs[slot]).data_ptr(), prec,
                           flags, out_fmt, row0=row0, nrows=nrows, d_segments=d_segs,
                           stream=streams[slot].cuda_stream)

    tiled = None
    if args.mode == "tiled" and world > 1:
        from rtamd import tiling
        # double-buffered: the gather of frame k (RCCL stream) overlaps the render of k+1
        tiled = tiling.TiledFrames(lambda r0, n, buf: launch(dst=buf), H, W,
                                   4 if args.out == "rgba8" else 3,
                                   torch.uint8 if args.out == "rgba8" else torch.float32,
                                   dev, depth=2)

    nstep = [0]

    def step():
        if tiled is not None:
            tiled.submit()
        else:
            launch(slot=nstep[0] % fif)
            nstep[0] += 1

    out_ptrs = [o.data_ptr() for o in outs]
    st_ptrs = [s_.cuda_stream for s_ in streams]

    def run_steps(n: int):
        """n consecutive steps: frames mode enqueues them with ONE C-ABI call
        (rt_render_device_frames: each frame's own host work and launch, minus the Python
        per-call overhead, so the host stays ahead of the GPU as a C++ frame loop would)."""
        if tiled is not None:
            for _ in range(n):
                step()
            return
        k = nstep[0] % fif
        rend.render_device_frames([cam], depth, out_ptrs[k:] + out_ptrs[:k], prec, flags,
                                  out_fmt, row0=row0, nrows=nrows,
                                  streams=st_ptrs[k:] + st_ptrs[:k], nframes=n)
        nstep[0] += n

    def join_streams():
        # stream 0 waits for every other stream's work (the end-of-region event is then
        # behind every frame of the region)
        for s_ in streams[1:]:
            stream.wait_stream(s_)

    # census: exact segment count of this rank's share (untimed)
    launch(segs_t.data_ptr())
    torch.cuda.synchronize(dev)
    my_segs = int(segs_t.item())
    tot = torch.tensor([my_segs], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    total_segs = int(tot.item())

    # Side measurements (per-precision kernel sweep, sun extension, moving camera) run
    # BEFORE the warmup and the timed region, on every rank (rank 0 reports them).  They
    # are measurements of their own; running them first also means the timed region
    # starts on a GPU at its sustained clock, as inside a running frame loop, rather than
    # on the ramp out of idle (tools/ramp_probe.py: frames 4-255 after idle run ~7%
    # slower than later ones, so a 20-step region would measure the ramp).
    nsw = 200
    sweep = {}
    sun_ext = None
    if not args.no_sweep:
        for pname, pc in capi.PRECISIONS.items():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            rend.render_device(cam, depth, out.data_ptr(), pc, flags, capi.RT_OUT_RGB_F32,
                               row0=row0, nrows=nrows, stream=stream.cuda_stream)
            e0.record(stream)
            for _ in range(nsw):
                rend.render_device(cam, depth, out.data_ptr(), pc, flags, capi.RT_OUT_RGB_F32,
                                   row0=row0, nrows=nrows, stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            kms = e0.elapsed_time(e1) / nsw
            sweep[pname] = {"kernel_ms": round(kms, 4),
                            "mrays_per_s": round(my_segs / (kms * 1e-3) / 1e6, 1),
                            "dtype": DTYPE[pname], "parity": PARITY[pname]}
        if not args.sun:
            # config 2's "sun" is reported as a separate extension run (same ray
            # paths and segment count; the sun only adds shading terms)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            rend.render_device(cam, depth, out.data_ptr(), prec, capi.RT_FLAG_SUN,
                               capi.RT_OUT_RGB_F32, row0=row0, nrows=nrows, stream=stream.cuda_stream)
            e0.record(stream)
            for _ in range(nsw):
                rend.render_device(cam, depth, out.data_ptr(), prec, capi.RT_FLAG_SUN,
                                   capi.RT_OUT_RGB_F32, row0=row0, nrows=nrows,
                                   stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            kms = e0.elapsed_time(e1) / nsw
            sun_ext = {"precision": args.precision, "kernel_ms": round(kms, 4),
                       "mrays_per_s": round(my_segs / (kms * 1e-3) / 1e6, 1),
                       "parity": "sun term is build-defined (constants main.cpp:18-19, unused "
                                 "by the reference): pinned to the oracle, not the reference"}

    moving = None
    if not args.no_sweep and args.mode == "frames":
        # the measured tile-row order on a camera that moves every frame (a fly-through of
        # 200 frames, 0.01 scene units per frame toward the scene — rays travel toward +x,
        # main.cpp:133): the order is refreshed every RT_OPT_ROW_FEEDBACK frames, so it
        # lags the view; per-frame ms with the feedback on and off (kernel stream time)
        ca = scenes.camera_args(W, H)
        cams = []
        for f in range(200):
            dx = 0.01 * f
            a = dict(ca)
            a["position"] = (ca["position"][0] + dx, ca["position"][1], ca["position"][2])
            a["lookat"] = (ca["lookat"][0] + dx, ca["lookat"][1], ca["lookat"][2])
            cams.append(capi.camera_init(**a))
        moving = {"frames": len(cams), "step": "0.01 units/frame along +x"}
        for fb in (0, args.row_feedback):
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK, fb)
            best = None
            for _ in range(2):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for c in cams:
                    rend.render_device(c, depth, out.data_ptr(), prec, flags, capi.RT_OUT_RGB_F32,
                                       row0=row0, nrows=nrows, stream=stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                ms = e0.elapsed_time(e1) / len(cams)
                best = ms if best is None else min(best, ms)
            moving[f"ms_per_frame_row_feedback_{fb}"] = round(best, 4)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)

    # the moving camera left the row feedback holding another view's order: drop it (with
    # any snapshot still in flight), so the first warmup frame samples this camera afresh,
    # with frames in flight as the timed steps run them.  (Measured with 20-step regions,
    # interleaved on one box: an order sampled from isolated launches — synchronous census
    # frames, or the sweep's back-to-back frames — runs the frames-in-flight loop 4-8%
    # slower on average and erratically (78-120 Grays/s); one sampled among frames in
    # flight gives 116-121; more back-to-back samples inside a 20-step region cost more than
    # they gain.)
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)

    run_steps(args.warmup)
    if tiled is not None:
        tiled.drain()
    barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    run_steps(args.steps)
    if tiled is not None:
        tiled.drain()
    join_streams()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed_s = float(elapsed.item())
    stream_ms = ev0.elapsed_time(ev1) / args.steps

    # per-launch kernel time: one stream, launches back to back (HIP events on that stream)
    ek0 = torch.cuda.Event(enable_timing=True)
    ek1 = torch.cuda.Event(enable_timing=True)
    nk = max(10, args.steps)
    ek0.record(stream)
    rend.render_device_frames([cam], depth, [out.data_ptr()], prec, flags, out_fmt, row0=row0,
                              nrows=nrows, streams=[stream.cuda_stream], nframes=nk)
    ek1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = ek0.elapsed_time(ek1) / nk

    result = None
    if rank == 0:
        ms_step = elapsed_s / args.steps * 1e3
        value = total_segs * args.steps / elapsed_s / 1e6
        frames_per_step = world if args.mode == "frames" else 1
        px_step = W * H * frames_per_step
        kernel_s = kernel_ms * 1e-3
        out_bytes = nrows * W * (4 if args.out == "rgba8" else 12)
        alg_bytes = out_bytes + scene_bytes(n_sph, n_wall, len(sc))
        workload = f"{cfg.name}:{W}x{H}:d{depth}:s{n_sph}w{n_wall}"
        # PMC traffic was collected on the fp32 RGB output only
        traffic = (load_traffic(args.traffic_json, workload, args.precision)
                   if args.out == "rgb_f32" else None)
        flops = my_segs * flop_per_segment(n_sph, n_wall)
        valu_peak = VALU_PEAK_TFLOPS[args.precision]
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "frames" else "strong",
            "vs_baseline": None,
            "dtype": DTYPE[args.precision],
            "data": "synthetic",
            "config": {
                "workload": workload,
                "scene": cfg.description + (" + sun" if args.sun else ""),
                "width": W, "height": H, "depth": depth,
                "spheres": n_sph, "walls": n_wall,
                "precision": args.precision,
                "output": args.out,
                "parity": PARITY[args.precision],
                "frames_per_step": frames_per_step,
                "segments_per_step": total_segs,
                "segments_per_pixel": round(total_segs / px_step, 4),
                "parallelism": (f"frame-sharded x{world}" if args.mode == "frames"
                                else f"row-tiled x{world} + gather"),
                "host_box_cache": bool(args.box_cache),
                "row_feedback": args.row_feedback,
                "frames_in_flight": fif,
                "backend": backend if world > 1 else None,
            },
            "ms_per_frame": round(ms_step / frames_per_step if args.mode == "frames" else ms_step, 4),
            "mpx_per_s": round(px_step * args.steps / elapsed_s / 1e6, 2),
            # one frame at a time on one stream (HIP events around back-to-back launches):
            # the per-frame latency, and the kernel duration the rooflines are priced on
            "kernel_ms": round(kernel_ms, 4),
            "stream_ms_per_step": round(stream_ms, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(alg_bytes / kernel_s / 1e9, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(alg_bytes / kernel_s / 1e9 / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": alg_bytes,
                "note": "north_star-mandated HBM view; the kernel is FP VALU-bound, see roofline_valu",
            },
            "roofline_valu": {
                "bound": "valu",
                "achieved": round(flops / kernel_s / 1e12, 3),
                "peak": valu_peak,
                "unit": "TFLOP/s",
                "frac": round(flops / kernel_s / 1e12 / valu_peak, 4),
                "flop_per_launch": flops,
                "convention": "SURVEY 8d: F_seg = 30*N_sphere + 38*N_wall + 60, FMA = 2",
            },
            "cpu_baseline": None,
            "precision_sweep": sweep or None,
            "sun_extension": sun_ext,
            "moving_camera": moving,
        }
        if world == 1 and not args.no_cpu_baseline and args.cpu_seconds > 0:
            result["cpu_baseline"] = cpu_baseline(cfg, prims, cam, depth, flags, args.cpu_seconds)
        print(json.dumps(result), flush=True)
    rend.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
