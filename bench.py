#!/usr/bin/env python3
"""bench.py — Mrays/s + ms/frame of the MI355X trace/shade path (BASELINE.json metric).

A "step" is one frame of the hot path over synthetic input: the configured scene (default
c2: 1920x1080, 8 spheres + 4 walls, reflection depth 4) rendered in full into HBM through
the C-ABI, the scene already resident on the device.

Default mode `tiled` (BASELINE configs 2 and 4): ONE frame per step split into contiguous
row bands across the N ranks (one process per GPU), each band rendered by its rank, and the
bands gathered into rank 0's frame buffer with RCCL send/recv inside the C-ABI's multi-GPU
frame operator (rt_multi_*, csrc/rt_multi.cpp) — `scaling` "strong" (total work fixed).  At
N = 1 the one band is the whole frame, rendered in place (no gather).  Consecutive frames go
to `--frames-in-flight` frame buffers on as many streams (default 2): every frame is
rendered and gathered in full, and frame k+1's render overlaps frame k's tail and gather.
With N > 1 the bench also reports, as a side field (`frame_sharded`), the weak layout: N
independent frames of a camera fly-through per step, no collective.  `--mode frames` makes
that the headline instead.

Rays = segments = closest-hit queries (primary + reflection), counted exactly by the
kernel in an untimed census launch.

Order of a run: census; side measurements (per-precision kernel sweep, sun-on frame loop,
moving-camera frame loop, and `steady_state`: the timed loop itself over 200 frames —
before the timed region, so it starts on a GPU at its running clock with the measured
tile-row order settled, as inside a running frame loop); W warmup + K timed steps, each
enqueued by one C-ABI call per region
(rt_multi_render_device_frames / rt_render_device_frames: every frame's own host work and
launch, as a C++ frame loop does them, without Python's per-call overhead); the one-stream
kernel time; the frame-sharded side run (N > 1); the CPU baseline (rank 0, N = 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--precision mixed]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Process model: one process per GPU.  Under a launcher (torch.distributed.run: RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_* in the environment) every process is one rank.  Without
one, `--gpus N` > 1 makes this process a supervisor: it starts N child processes of this
script (one per rank, RANK = LOCAL_RANK = r, MASTER_ADDR 127.0.0.1, a free port) before
anything touches the GPU, forwards rank 0's JSON line, and if
any child exits non-zero or the --deadline passes it stops the others and exits non-zero
naming the rank.  Every rank also has its own deadline watchdog.  `--transport ipc` runs
the row-tiled operator's process-per-GPU code across processes on ONE GPU
(RT_TRANSPORT_IPC, a rehearsal: torch.distributed over gloo, the gather through HIP IPC).
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
              "within 2e-5 of the reference, no discontinuity flips (full c2 / c3 frames vs the "
              "oracle: max |delta| 1.6e-6 / 2.0e-6, equal segment counts)",
    "f32": "|delta| <= 1e-4 on >= 99.5% of pixels at depth <= 4 (flips at discontinuities)",
}


def flop_per_segment(n_sph: int, n_wall: int) -> int:
    """SURVEY §8d convention: F_seg = 30*N_sphere + 38*N_wall + 60 (FMA = 2)."""
    return 30 * n_sph + 38 * n_wall + 60


def scene_bytes(n_sph: int, n_wall: int, n_prim: int) -> int:
    return 64 * n_sph + 176 * n_wall + 64 * n_prim   # DevSphere / DevWall / DevMat records


def cpu_threads() -> dict:
    """The host's threads as the CPU baseline sees them (OMP_NUM_THREADS =
    nproc).  On a shared GPU box OMP_NUM_THREADS is this job's CPU share, and the machine's
    full core count (nproc) is not ours to use, so OMP_NUM_THREADS wins when it is set."""
    affinity = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = int(omp) if omp and omp.isdigit() and int(omp) > 0 else affinity
    return {"threads": threads, "nproc": os.cpu_count(), "affinity": affinity,
            "OMP_NUM_THREADS": omp}


def cpu_baseline(cfg, prims, cam, depth, flags, budget_s: float):
    """The oracle's OpenMP restatement (the 'OpenMP CPU path') on this host's cores, on a
    bounded sample of the same frame: a centred band of rows sized to ~budget_s / 3, timed
    three times, best of 3."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc_mod   # test infrastructure: the timed CPU baseline leg only
    orc = orc_mod.Oracle()
    th = cpu_threads()
    cores = th["threads"]
    H = cam.height
    probe = min(H, 16)
    r0 = max(0, H // 2 - probe // 2)
    t = time.perf_counter()
    orc.render(prims, cam, depth, flags, row0=r0, nrows=probe, nthreads=cores, want64=False)
    per_row = max(1e-6, (time.perf_counter() - t) / probe)
    rows = int(min(H, max(probe, budget_s / 3 / per_row)))
    r0 = max(0, H // 2 - rows // 2)
    runs = []
    for _ in range(3):
        # repeat the band until a third of the budget is spent (small frames take ms)
        segs, dt, reps = 0, 0.0, 0
        while reps == 0 or (dt < budget_s / 3 and reps < 10000):
            t = time.perf_counter()
            _, _, s = orc.render(prims, cam, depth, flags, row0=r0, nrows=rows, nthreads=cores,
                                 want64=False)
            dt += time.perf_counter() - t
            segs += s
            reps += 1
        runs.append((segs / dt, dt / reps, reps, segs, dt))
    best = max(runs)
    return {"value": round(best[0] / 1e6, 3), "unit": "Mrays/s", "cores": cores, "kind": "port",
            "threads": th,
            "sample": f"best of 3 runs, each {best[2]} x rows {r0}..{r0 + rows - 1} of the same "
                      f"{cam.width}x{H} frame ({rows * cam.width} px; best run {best[3]} "
                      f"segments in {best[4]:.2f} s), fp64 oracle restatement (-O3, no FMA), "
                      f"OpenMP schedule(dynamic,1) over rows on {cores} threads",
            "runs_mrays_per_s": [round(r[0] / 1e6, 3) for r in runs],
            "ms_per_frame": round(best[1] / rows * H * 1e3, 2)}


def load_profile(path: str, workload: str, precision: str):
    """Per-launch numbers measured by rocprofv3 --pmc (profiles/)."""
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(workload, {}).get(precision)
    except (OSError, ValueError, KeyError, TypeError, AttributeError):
        return None


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def supervise(args, argv) -> int:
    """`--gpus N` > 1 without a launcher: N child processes of this script, one per rank,
    started before anything here touches the GPU (no torch.cuda, no librt_amd.so in this
    process).  Rank 0's stdout (its one JSON line) is forwarded; the other ranks' stdout goes
    to stderr.  A child exiting non-zero or the deadline passing stops every other child
    (SIGTERM, then SIGKILL) and exits non-zero with the rank named."""
    import signal
    import subprocess
    import threading
    n = args.gpus
    port = free_port()
    script = os.path.abspath(__file__)
    procs, lines = [], []

    def die_with_parent():
        # a child gets SIGTERM if the supervisor dies (e.g. killed by an outer time limit)
        import ctypes
        try:
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG
        except (OSError, AttributeError):
            pass

    def on_term(signum, frame):
        for p_ in procs:
            if p_.poll() is None:
                p_.send_signal(signal.SIGTERM)
        print(f"bench supervisor: signal {signum}: ranks stopped", file=sys.stderr, flush=True)
        os._exit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      preexec_fn=die_with_parent))

    def pump():
        for ln in procs[0].stdout:
            lines.append(ln.decode(errors="replace"))

    th = threading.Thread(target=pump, daemon=True)
    th.start()
    t0 = time.monotonic()
    beat = t0
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = f"rank {bad[0][0]} exited with status {bad[0][1]}"
            break
        if all(c == 0 for c in codes):
            break
        now = time.monotonic()
        if now - t0 > args.deadline:
            late = [r for r, c in enumerate(codes) if c is None]
            failed = f"deadline {args.deadline:.0f} s passed with rank(s) {late} still running"
            break
        if now - beat > 60:
            beat = now
            print(f"bench supervisor: {n} ranks running for {now - t0:.0f} s", file=sys.stderr,
                  flush=True)
        time.sleep(0.05)
    if failed:
        print(f"bench supervisor: {failed}; stopping the other ranks", file=sys.stderr, flush=True)
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t1 = time.monotonic()
        while any(p.poll() is None for p in procs) and time.monotonic() - t1 < 10:
            time.sleep(0.05)
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()
        th.join(5)
        return 3
    th.join(10)
    for ln in lines:
        sys.stdout.write(ln)
    sys.stdout.flush()
    return 0


PHASE = ["start"]


def start_watchdog(seconds: float, rank: int) -> None:
    """Ends this rank's process (status 124) if it is still running after `seconds`: a peer
    rank that failed leaves this one blocked in a collective or a stream wait that never
    completes, which must become an exit naming the rank, not a silent hang."""
    import threading

    def fire():
        print(f"bench rank {rank}: deadline {seconds:.0f} s passed in phase '{PHASE[0]}'",
              file=sys.stderr, flush=True)
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(scenes.CONFIGS))
    ap.add_argument("--precision", default="path64", choices=sorted(capi.PRECISIONS))
    ap.add_argument("--mode", default="tiled", choices=["tiled", "frames"],
                    help="tiled: one frame per step, row bands across ranks + gather (strong); "
                         "frames: one frame per rank per step, no collective (weak)")
    ap.add_argument("--out", default="rgb_f32", choices=["rgb_f32", "rgba8"],
                    help="timed output format: linear fp32 RGB (12 B/px, parity buffer) or the "
                         "clamp+truncate RGBA8 epilogue (4 B/px; cuts the tiled gather 3x)")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="consecutive frames go to F frame buffers on F streams (double-buffered "
                         "by default), so one frame's last waves and gather overlap the next "
                         "frame's render; 1 = one stream, frames back to back")
    ap.add_argument("--tiler", default="native", choices=["native", "torch"],
                    help="tiled mode: the C-ABI's rt_multi (RCCL send/recv in C++), or "
                         "rtamd.tiling over torch.distributed")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "copy", "ipc"],
                    help="rt_multi transport: rccl (the product), copy (one process only, "
                         "--local-ranks), ipc (one process per rank on any number of GPUs, "
                         "HIP IPC + a shared-memory mailbox: the rehearsal of the "
                         "process-per-GPU path on one GPU; torch.distributed over gloo)")
    ap.add_argument("--band-layout", default="weighted", choices=["equal", "weighted"],
                    help="tiled mode, N > 1: rank r's rows of the frame — equal contiguous bands "
                         "(rt_band_rows), or contiguous bands cut so each carries 1/N of the "
                         "tile-row costs rank 0 measures once on its GPU and broadcasts "
                         "(rt_weighted_band_rows, RT_OPT_MULTI_LAYOUT 2)")
    ap.add_argument("--rank-frames", type=int, default=4,
                    help="N > 1: band frames in flight per rank (RT_OPT_MULTI_FRAMES)")
    ap.add_argument("--rank-batch", type=int, default=8,
                    help="N > 1: frames per gather (RT_OPT_MULTI_BATCH): each rank sends its bands "
                         "of that many frames in one ncclSend, the root scatters them with one "
                         "kernel (the per-frame exchange's host calls cost more than a 1/8 band)")
    ap.add_argument("--frame-batch", type=int, default=0,
                    help="RT_OPT_FRAME_BATCH: frames per launch — at N > 1 a rank's band frames of "
                         "one gather go to the GPU in blocks of this many per stream (0 = auto: 2, "
                         "so a gather of 8 is 4 launches on 4 streams; tools/band_model.py, "
                         "DESIGN §5); at N = 1 an explicit B > 1 launches B consecutive frames of "
                         "a stream as one grid (measured slower than 2 streams: off)")
    ap.add_argument("--local-ranks", type=int, default=1,
                    help="rehearsal only (one process): split the frame over this many ranks "
                         "on this one GPU with the peer-copy transport; not a measurement")
    ap.add_argument("--sun", action="store_true", help="build-defined sun term (off = parity)")
    ap.add_argument("--steady-frames", type=int, default=200,
                    help="frames of the steady-state loop run right before the warmup and timed "
                         "region (a side measurement; it also leaves the row order settled)")
    ap.add_argument("--windows", type=int, default=40,
                    help="windows of --steps frames run right before the warmup, each like the "
                         "timed region (their ms/frame distribution is reported)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the config-5 side run (row-tiled 7680x4320 frames)")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the side measurements (precision sweep, sun and moving-camera "
                         "loops, frame-sharded side run)")
    ap.add_argument("--row-feedback", type=int, default=32,
                    help="RT_OPT_ROW_FEEDBACK: refresh interval (frames) of the measured "
                         "tile-row dispatch order, 0 = off (scheduling only)")
    ap.add_argument("--box-cache", type=int, default=0, choices=[0, 1],
                    help="RT_OPT_BOX_CACHE: reuse the host's per-frame pixel boxes when the "
                         "camera is unchanged (0 = recompute every frame)")
    ap.add_argument("--hw-queues", type=int, default=16, choices=range(0, 33), metavar="Q",
                    help="N > 1 with a GPU per rank: GPU_MAX_HW_QUEUES for each rank (0 = leave "
                         "the environment's).  A rank keeps RT_OPT_MULTI_FRAMES band frames in "
                         "flight on their own streams, which need their own hardware queues: "
                         "HIP's default (and the GPU boxes' environment) is 4 per process, shared "
                         "round-robin by every stream it makes (tools/band_model.py, DESIGN §5).  "
                         "Set before HIP initialises, so it overrides the environment's value.  "
                         "Ranks that share a GPU (rehearsals) keep the environment's: several "
                         "processes with 16 queues each on one GPU run far slower "
                         "(tools/ab_hw_queues.sh, profiles/r06/probes/ab_hw_queues.jsonl)")
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="seconds: the supervisor (and each rank's watchdog) ends the run "
                         "non-zero if it is still going")
    ap.add_argument("--fault-rank", type=int, default=-1,
                    help="test hook: this rank's frame right after the gather check fails "
                         "(RT_OPT_MULTI_FAULT) — every rank must then exit non-zero")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--valu-json", default=os.path.join(REPO, "profiles", "pmc_valu.json"))
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return supervise(args, sys.argv[1:] if argv is None else list(argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world} (launch N ranks with --gpus N)",
              file=sys.stderr)
        return 2
    start_watchdog(args.deadline, rank)
    if os.environ.get("RT_BENCH_TEST_HANG"):   # test hook: a rank stuck before any GPU work
        PHASE[0] = "test hang"
        while True:
            time.sleep(1)

    # stdout carries the ONE JSON line: anything the libraries print there (RCCL's version
    # banner when a communicator is made) goes to stderr, the JSON to a private copy of fd 1
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    # read by the HIP runtime at its initialisation (below: torch.cuda.set_device); counting
    # devices does not initialise it on this image
    if world > 1 and args.hw_queues > 0 and world <= torch.cuda.device_count():
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

    # RT_BENCH_BACKEND=gloo (or --transport ipc): rehearsal of the N-rank code path on fewer
    # GPUs than ranks (ranks share devices round-robin; RCCL refuses two ranks on one GPU, so
    # the tiled mode then uses the torch tiler over gloo, or with --transport ipc the native
    # operator over HIP IPC).  Not a measurement: the driver's multi-GPU runs use the
    # default, RCCL ("nccl").
    backend = os.environ.get("RT_BENCH_BACKEND", "gloo" if args.transport == "ipc" else "nccl")
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
    tiled_mode = args.mode == "tiled"
    tiler = args.tiler if not (tiled_mode and world > 1 and backend == "gloo"
                               and args.transport != "ipc") else "torch"
    PHASE[0] = "setup"

    rend = capi.Renderer(local)   # census, side measurements, frames mode, kernel time
    if world == 1 and args.frame_batch > 1:
        rend.set_option(capi.RT_OPT_FRAME_BATCH, min(capi.RT_MULTI_BATCH_MAX, args.frame_batch))
    rend.set_option(capi.RT_OPT_BOX_CACHE, args.box_cache)
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)
    rend.set_scene(prims)
    cam0 = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    W, H = cam0.width, cam0.height
    out_fmt = capi.RT_OUT_RGBA8 if args.out == "rgba8" else capi.RT_OUT_RGB_F32
    ch, tdt = (4, torch.uint8) if args.out == "rgba8" else (3, torch.float32)

    # frames mode: frame `rank` of a fly-through (Camera::forward moves position by
    # forward_vec()*movement_speed = (1,0,0)*0.1 and never re-calls init(), scene.cpp:121)
    cam_fly = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    cam_fly.position[0] += 0.1 * rank
    cam = cam0 if tiled_mode else cam_fly
    # this rank's rows: its band of the one frame (tiled), or the whole frame (frames).
    # Weighted bands: rank 0 measures every tile row's cost on one full render of the frame
    # (untimed, rt_tile_row_costs) and broadcasts it, so every rank cuts the same bands.
    layout = {"equal": 0, "weighted": 2}[args.band_layout] \
        if (world > 1 or args.local_ranks > 1) else 0
    weights = None
    if tiled_mode and layout == 2:
        w_ = [rend.tile_row_costs(cam0, depth, prec, flags).tolist() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(w_, src=0)
        weights = w_[0]
    if tiled_mode and layout == 2:
        row0, nrows = capi.weighted_band_rows(H, world, rank, weights)
    elif tiled_mode:
        row0, nrows = capi.band_rows(H, world, rank)
    else:
        row0, nrows = 0, H

    fif = max(1, args.frames_in_flight)
    streams = [torch.cuda.Stream(dev) for _ in range(fif)]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    st_ptrs = [s_.cuda_stream for s_ in streams]
    rank_batch = max(1, min(capi.RT_MULTI_BATCH_MAX, args.rank_batch))
    frame_batch = max(1, min(capi.RT_MULTI_BATCH_MAX, args.frame_batch if args.frame_batch > 0 else 2))
    # frame buffers: the whole frame on rank 0 (tiled: the bands are gathered into it) or on
    # every rank (frames mode); fp32-RGB sized, which the sweep below also writes.  The
    # batched exchange (N > 1) needs a distinct buffer per frame of a batch (rt_capi.h
    # RT_OPT_MULTI_BATCH): 2 x B of them, so consecutive batches never share one and every
    # frame is whole in its buffer
    full = (not tiled_mode) or rank == 0
    nbuf = fif
    if tiled_mode and tiler == "native" and (world > 1 or args.local_ranks > 1) and full:
        nbuf = max(fif, 2 * rank_batch)
    fb1 = world == 1 and args.local_ranks <= 1 and args.frame_batch > 1   # N = 1 frame batching
    if fb1:
        nbuf = max(nbuf, args.frame_batch)
    outs = [torch.empty((H if full else max(1, nrows), W, 3), dtype=torch.float32, device=dev)
            for _ in range(nbuf)]
    out = outs[0]
    out_ptrs = [o.data_ptr() for o in outs]
    segs_t = torch.zeros(1, dtype=torch.int64, device=dev)

    # ---- census: exact segment count of this rank's rows (untimed) ----
    PHASE[0] = "census"
    rend.render_device(cam, depth, out.data_ptr(), prec, flags, capi.RT_OUT_RGB_F32, row0=row0,
                       nrows=nrows, d_segments=segs_t.data_ptr(), stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    my_segs = int(segs_t.item())
    tot = torch.tensor([my_segs], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    total_segs = int(tot.item())
    frame_segs = total_segs if tiled_mode else my_segs   # one frame

    # ---- the tiled frame operator ----
    PHASE[0] = "operator setup"
    multi = None
    torch_tiled = None
    if tiled_mode and tiler == "native":
        if world > 1 and args.transport == "ipc":
            # any shared bytes name the IPC mailbox: rank 0's random id, broadcast
            uid = [os.urandom(capi.RT_MULTI_ID_BYTES) if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            multi = capi.MultiRenderer([local], nranks=world, first_rank=rank, unique_id=uid[0],
                                       transport=capi.RT_TRANSPORT_IPC)
        elif world > 1:
            uid = [capi.multi_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            multi = capi.MultiRenderer([local], nranks=world, first_rank=rank, unique_id=uid[0])
        elif args.local_ranks > 1 or args.transport == "copy":
            multi = capi.MultiRenderer([local] * args.local_ranks,
                                       transport=capi.RT_TRANSPORT_COPY)
        else:
            multi = capi.MultiRenderer([local])
        multi.set_option(capi.RT_OPT_BOX_CACHE, args.box_cache)
        multi.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)
        multi.set_option(capi.RT_OPT_MULTI_TIMEOUT_MS, int(args.deadline * 1000))
        if fb1:   # N = 1: the one band is the frame, rendered by the operator's own ctx
            multi.set_option(capi.RT_OPT_FRAME_BATCH, min(capi.RT_MULTI_BATCH_MAX, args.frame_batch))
        multi.set_scene(prims)
        if layout == 2:
            multi.set_row_weights(weights)
        multi.set_option(capi.RT_OPT_MULTI_LAYOUT, layout)
        if multi.nranks > 1:
            multi.set_option(capi.RT_OPT_MULTI_FRAMES, max(1, min(capi.RT_MULTI_SLOTS, args.rank_frames)))
            multi.set_option(capi.RT_OPT_MULTI_BATCH, rank_batch)
            multi.set_option(capi.RT_OPT_FRAME_BATCH, frame_batch)
    elif tiled_mode:
        from rtamd import tiling
        # double-buffered: the gather of frame k (collective stream) overlaps the render of k+1
        torch_tiled = tiling.TiledFrames(
            lambda r0, n, buf: rend.render_device(cam, depth, buf.data_ptr(), prec, flags, out_fmt,
                                                  row0=r0, nrows=n, stream=stream.cuda_stream),
            H, W, ch, tdt, dev, depth=2)
    n_ranks = multi.nranks if multi is not None else world

    # ---- the gathered frames against rank 0's own one-GPU render of the same frame, bitwise
    # (untimed): the row-tiled operator must only move bytes (pixels are independent).  Both
    # exchanges the operator has: the batched one (3 batches of B frames over 2 B buffers,
    # so the third batch renders into the first one's buffers) and the per-frame one (3
    # frames over 2 buffers); EVERY buffer is compared ----
    PHASE[0] = "gather check"
    gather_check = None
    if tiled_mode:
        ref = None
        nbytes = H * W * (4 if args.out == "rgba8" else 12)
        if rank == 0:
            ref = torch.empty((H, W, ch), dtype=tdt, device=dev)
            rend.render_device(cam, depth, ref.data_ptr(), prec, flags, out_fmt,
                               stream=stream.cuda_stream)
        chk = multi
        op_name = None
        if multi is not None and world == 1 and multi.nranks == 1:
            # one GPU: the timed operator renders the frame in place (no communicator); check
            # the gather's RCCL calls here instead, untimed, through a one-rank loopback
            # communicator (the root's band sent to itself: ncclCommInitRank, the group,
            # ncclSend/ncclRecv, ncclCommGetAsyncError all run), batched as N > 1 runs are
            chk = capi.MultiRenderer([local], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK)
            chk.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)
            chk.set_scene(prims)
            op_name = ("rt_multi, RT_TRANSPORT_RCCL_LOOPBACK: RCCL send/recv of the one band "
                       "through a one-rank communicator (the timed N = 1 loop renders in place)")
        elif multi is not None:
            op_name = (f"rt_multi, {multi.nranks} ranks, "
                       + {"rccl": "RCCL send/recv", "ipc": "HIP IPC copies between processes "
                          "(rehearsal)", "copy": "peer copies (rehearsal)"}[
                           args.transport if world > 1 else "copy"]
                       + f", {args.band_layout} bands")
        checks = {}
        if chk is not None:
            nb = 2 * rank_batch
            cbufs = ([torch.empty((H, W, ch), dtype=tdt, device=dev) for _ in range(nb)]
                     if rank == 0 else [])
            cptrs = [b_.data_ptr() for b_ in cbufs]
            cases = [("batched", rank_batch, nb, 3 * rank_batch), ("per_frame", 1, 2, 3)]
            for name, bsz, nbs, nfr in cases:
                if name == "batched" and bsz == 1:
                    continue
                chk.set_option(capi.RT_OPT_MULTI_BATCH, bsz)
                for b_ in cbufs:
                    b_.fill_(255 if tdt == torch.uint8 else -1.0)
                torch.cuda.synchronize(dev)
                chk.render_device_frames([cam], depth, cptrs[:nbs] if chk.has_root else [], prec,
                                         flags, out_fmt,
                                         streams=st_ptrs[:2] if chk.has_root else st_ptrs[:1],
                                         nframes=nfr)
                torch.cuda.synchronize(dev)
                chk.sync()
                barrier()
                if rank == 0:
                    rb = ref.view(torch.uint8).flatten()[:nbytes]
                    eqs = [bool(torch.equal(b_.view(torch.uint8).flatten()[:nbytes], rb))
                           for b_ in cbufs[:nbs]]
                    checks[name] = {"frames": nfr, "buffers": nbs, "frames_per_gather": bsz,
                                    "every_buffer_bitwise_equal": all(eqs)}
            if multi is not None and multi.nranks > 1:
                chk.set_option(capi.RT_OPT_MULTI_BATCH, rank_batch)
            if chk is not multi:
                chk.close()
            del cbufs
        elif torch_tiled is not None:
            h_ = torch_tiled.submit()
            torch_tiled.wait(h_)
            torch_tiled.drain()
            torch.cuda.synchronize(dev)
            if rank == 0:
                got = torch_tiled.frame(h_[0]).view(torch.uint8).flatten()[:nbytes]
                checks["per_frame"] = {"frames": 1, "every_buffer_bitwise_equal":
                                       bool(torch.equal(got, ref.view(torch.uint8).flatten()[:nbytes]))}
                del got
        barrier()
        if rank == 0:
            eq = bool(checks) and all(c["every_buffer_bitwise_equal"] for c in checks.values())
            gather_check = {"bitwise_equal_to_one_gpu_frame": eq, "ranks": n_ranks,
                            "output": args.out, **checks,
                            "operator": op_name if multi is not None
                            else "rtamd.tiling (torch.distributed gather)"}
            if not eq:
                print(f"bench: a gathered {n_ranks}-rank frame differs from the one-GPU frame",
                      file=sys.stderr)
            del ref

    if args.fault_rank == rank:
        if multi is not None:
            # test hook: this rank's next frame fails once its part of the exchange is queued
            multi.set_option(capi.RT_OPT_MULTI_FAULT, 1)
            print(f"bench rank {rank}: injecting a fault into the next frame", file=sys.stderr)
        else:   # the torch tiler: the rank fails outright (its peers wait in a collective)
            raise RuntimeError(f"bench rank {rank}: injected failure (--fault-rank)")

    def run_steps(n: int):
        """n consecutive frames, enqueued by ONE C-ABI call (or the torch tiler's loop)."""
        if multi is not None:
            if multi.has_root:
                multi.render_device_frames([cam], depth, out_ptrs, prec, flags, out_fmt,
                                           streams=st_ptrs, nframes=n)
            else:   # non-root ranks: the band renders and sends; stream 0 waits for the sends
                multi.render_device_frames([cam], depth, [], prec, flags, out_fmt,
                                           streams=st_ptrs[:1], nframes=n)
        elif torch_tiled is not None:
            for _ in range(n):
                torch_tiled.submit()
            torch_tiled.drain()
        else:
            rend.render_device_frames([cam], depth, out_ptrs, prec, flags, out_fmt, row0=row0,
                                      nrows=nrows, streams=st_ptrs, nframes=n)

    def join_streams():
        for s_ in streams[1:]:
            stream.wait_stream(s_)

    sync_evs = [torch.cuda.Event() for _ in range(len(streams) + 1)]

    def hot_sync():
        """torch.cuda.synchronize, reached by polling events on this rank's streams first: a
        host core that sleeps in a blocking wait clocks down, and the frames enqueued right
        after took 19-24 us of host time each instead of 9-10 (measured) —
        slower than the GPU renders them, so the GPU starved in the next timed window."""
        for e_, s_ in zip(sync_evs, streams + [torch.cuda.current_stream(dev)]):
            e_.record(s_)
        for e_ in sync_evs:
            while not e_.query():
                pass
        torch.cuda.synchronize(dev)

    def timed_frames(cams, nframes, fl, nrep=2):
        """Best ms/frame of nframes frames of `cams` (cycled) through the frames-in-flight
        loop on this rank's rows (HIP events on stream 0, every stream joined)."""
        best = None
        for _ in range(nrep):
            torch.cuda.synchronize(dev)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for s_ in streams[1:]:
                s_.wait_stream(stream)
            rend.render_device_frames(cams, depth, out_ptrs, prec, fl, capi.RT_OUT_RGB_F32,
                                      row0=row0, nrows=nrows, streams=st_ptrs, nframes=nframes)
            join_streams()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / nframes
            best = ms if best is None else min(best, ms)
        return best

    # ---- side measurements (before the timed region; rank 0 reports) ----
    nsw = 200
    sweep, sun_ext, moving = {}, None, None
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
        if not args.sun and rank == 0 and world == 1:
            # config 2's literal "+ sun": the same frame loop as the headline (frames in
            # flight, fp32 RGB) with the build-defined sun term on — same ray paths and
            # segment count (the sun only adds shading terms)
            ms = timed_frames([cam], nsw, capi.RT_FLAG_SUN)
            sun_ext = {"precision": args.precision, "ms_per_frame": round(ms, 4),
                       "mrays_per_s": round(my_segs / (ms * 1e-3) / 1e6, 1),
                       "frames_in_flight": fif, "frames": nsw,
                       "parity": "sun term is build-defined (constants main.cpp:18-19, unused "
                                 "by the reference): pinned to the oracle, not the reference"}
        if rank == 0 and world == 1:
            # a camera moving every frame (a fly-through of 200 frames, 0.01 scene units per
            # frame along +x: rays travel toward +x, main.cpp:133) through the same
            # frames-in-flight loop, with the measured row order refreshed every
            # RT_OPT_ROW_FEEDBACK frames (so it lags the view) and off
            ca = scenes.camera_args(W, H)
            cams = []
            for f in range(200):
                a = dict(ca)
                a["position"] = (ca["position"][0] + 0.01 * f, ca["position"][1], ca["position"][2])
                a["lookat"] = (ca["lookat"][0] + 0.01 * f, ca["lookat"][1], ca["lookat"][2])
                cams.append(capi.camera_init(**a))
            segs_t.zero_()
            for c in cams:   # census of the 200 frames (untimed)
                rend.render_device(c, depth, out.data_ptr(), prec, flags, capi.RT_OUT_RGB_F32,
                                   row0=row0, nrows=nrows, d_segments=segs_t.data_ptr(),
                                   stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            mv_segs = int(segs_t.item())
            moving = {"frames": len(cams), "step": "0.01 units/frame along +x",
                      "frames_in_flight": fif, "segments": mv_segs}
            for fb in (0, args.row_feedback):
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, fb)
                ms = timed_frames(cams, len(cams), flags)
                moving[f"ms_per_frame_row_feedback_{fb}"] = round(ms, 4)
                moving[f"mrays_per_s_row_feedback_{fb}"] = round(
                    mv_segs / len(cams) / (ms * 1e-3) / 1e6, 1)
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)

    # the side loops left `rend`'s row feedback holding another view's order: drop it (with
    # any snapshot still in flight), so its next frame samples this camera afresh
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, args.row_feedback)

    # ---- steady state: the timed loop itself over 200 frames (a side measurement, before
    # the warmup).  It also leaves the product path's measured tile-row order settled for
    # this camera, as in a running frame loop; without it a short timed region (the driver
    # runs 20 steps) spends its first frames on the order's ramp-up (measured: 20-step
    # regions 33-40 us/frame vs 29 over 200 frames) ----
    steady = None
    PHASE[0] = "steady state"
    if not args.no_sweep:
        nst = max(1, args.steady_frames)
        torch.cuda.synchronize(dev)
        if multi is not None:
            multi.sync()
        barrier()
        es0 = torch.cuda.Event(enable_timing=True)
        es1 = torch.cuda.Event(enable_timing=True)
        ts0 = time.perf_counter()
        es0.record(stream)
        for s_ in streams[1:]:
            s_.wait_stream(stream)
        run_steps(nst)
        join_streams()
        es1.record(stream)
        hot_sync()
        if multi is not None:
            multi.sync()
        barrier()
        tst = torch.tensor([time.perf_counter() - ts0], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tst, op=dist.ReduceOp.MAX)
        steady = {"frames": nst, "ms_per_step": round(float(tst.item()) / nst * 1e3, 4),
                  "mrays_per_s": round(total_segs * nst / float(tst.item()) / 1e6, 1),
                  "stream_ms_per_step": round(es0.elapsed_time(es1) / nst, 4)}

    # ---- window rhythm: R windows exactly like the timed region (K frames by one call,
    # bracketed by the same syncs and barrier), back to back.  Their ms/frame is the
    # distribution the timed window is one sample of (reported), and the timed window then
    # runs as the next window of the same rhythm: the GPU's clock governor ramps its shader
    # clock over ~20 ms of sustained load (2.2 -> 2.4 GHz measured inside the frames) and a
    # host core that slept clocks down ----
    windows = None
    if not args.no_sweep and args.windows > 0:
        wms = []
        for _ in range(args.windows):
            hot_sync()
            barrier()
            tw0 = time.perf_counter()
            run_steps(args.steps)
            torch.cuda.synchronize(dev)   # as the timed region ends (see there)
            barrier()
            wms.append((time.perf_counter() - tw0) / args.steps * 1e3)
        if multi is not None:
            multi.sync()
        tw = torch.tensor(wms, dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tw, op=dist.ReduceOp.MAX)
        q = sorted(tw.tolist())
        windows = {"windows": len(q), "frames_per_window": args.steps,
                   "ms_per_step_median": round(q[len(q) // 2], 4),
                   "ms_per_step_p10": round(q[int(0.1 * (len(q) - 1))], 4),
                   "ms_per_step_p90": round(q[int(0.9 * (len(q) - 1))], 4),
                   "mrays_per_s_median": round(total_segs / (q[len(q) // 2] * 1e-3) / 1e6, 1)}

    # ---- warmup + timed region ----
    PHASE[0] = "timed region"
    run_steps(args.warmup)
    hot_sync()
    if multi is not None:
        multi.sync()
    barrier()
    hot_sync()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1s = [torch.cuda.Event(enable_timing=True) for _ in streams]
    t0 = time.perf_counter()
    ev0.record(stream)
    for s_ in streams[1:]:
        s_.wait_stream(stream)
    run_steps(args.steps)
    t_enq = time.perf_counter() - t0   # host time to enqueue the K frames (diagnostic)
    for e_, s_ in zip(ev1s, streams):  # (while the GPU still renders: off the critical path)
        e_.record(s_)
    # every stream of the device, the gathered frames included (N > 1: the caller streams
    # wait on the gather).  Called while the GPU still renders: the HIP runtime retires the
    # finished launches during the wait — polling until the GPU is done and only then
    # synchronizing left ~25 us of that bookkeeping after the last frame (measured)
    torch.cuda.synchronize(dev)
    t_synced = time.perf_counter() - t0
    barrier()
    t1 = time.perf_counter()
    if multi is not None:
        multi.sync()   # RCCL's asynchronous errors (after the timed region)
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed_s = float(elapsed.item())
    stream_ms = max(ev0.elapsed_time(e_) for e_ in ev1s) / args.steps

    # ---- per-launch kernel time: this rank's rows, one stream, launches back to back ----
    # (after 64 untimed frames of `rend`, whose measured row order the side loops reset)
    rend.render_device_frames([cam], depth, [out.data_ptr()], prec, flags, out_fmt, row0=row0,
                              nrows=nrows, streams=[stream.cuda_stream], nframes=64)
    ek0 = torch.cuda.Event(enable_timing=True)
    ek1 = torch.cuda.Event(enable_timing=True)
    nk = max(50, args.steps)
    ek0.record(stream)
    rend.render_device_frames([cam], depth, [out.data_ptr()], prec, flags, out_fmt, row0=row0,
                              nrows=nrows, streams=[stream.cuda_stream], nframes=nk)
    ek1.record(stream)
    torch.cuda.synchronize(dev)
    kernel_ms = ek0.elapsed_time(ek1) / nk

    # ---- N > 1 side run: the weak (frame-sharded) layout, same frame loop, no collective --
    sharded = None
    PHASE[0] = "side runs"
    if tiled_mode and world > 1 and not args.no_sweep:
        # whole frames on every rank: full-size buffers (a non-root rank's `outs` hold a band)
        if full:
            fl_outs = out_ptrs
        else:
            fl_bufs = [torch.empty((H, W, 3), dtype=torch.float32, device=dev) for _ in range(fif)]
            fl_outs = [b.data_ptr() for b in fl_bufs]
        segs_t.zero_()
        rend.render_device(cam_fly, depth, fl_outs[0], prec, flags, capi.RT_OUT_RGB_F32,
                           d_segments=segs_t.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t_segs = segs_t.clone()
        dist.all_reduce(t_segs, op=dist.ReduceOp.SUM)
        nfs = max(20, args.steps // 2)
        rend.render_device_frames([cam_fly], depth, fl_outs, prec, flags, out_fmt,
                                  streams=st_ptrs, nframes=args.warmup)
        torch.cuda.synchronize(dev)
        barrier()
        ts0 = time.perf_counter()
        rend.render_device_frames([cam_fly], depth, fl_outs, prec, flags, out_fmt,
                                  streams=st_ptrs, nframes=nfs)
        torch.cuda.synchronize(dev)
        barrier()
        ts = torch.tensor([time.perf_counter() - ts0], dtype=torch.float64, device=dev)
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        sharded = {"value": round(int(t_segs.item()) * nfs / float(ts.item()) / 1e6, 2),
                   "unit": "Mrays/s", "scaling": "weak", "frames_per_step": world,
                   "ms_per_step": round(float(ts.item()) / nfs * 1e3, 4),
                   "parallelism": f"frame-sharded x{world} (fly-through, no collective)"}

    # ---- N > 1 side run: the same row-tiled frames with the RGBA8 epilogue as transport
    # (4 B/px instead of 12: the root's inbound bytes, which bound config 4, shrink 3x) ----
    tiled8 = None
    if multi is not None and world > 1 and args.out == "rgb_f32" and not args.no_sweep:
        n8 = max(50, args.steps)
        multi.render_device_frames([cam], depth, out_ptrs if multi.has_root else [], prec, flags,
                                   capi.RT_OUT_RGBA8, streams=st_ptrs if multi.has_root else st_ptrs[:1],
                                   nframes=args.warmup)
        torch.cuda.synchronize(dev)
        multi.sync()
        barrier()
        t80 = time.perf_counter()
        multi.render_device_frames([cam], depth, out_ptrs if multi.has_root else [], prec, flags,
                                   capi.RT_OUT_RGBA8, streams=st_ptrs if multi.has_root else st_ptrs[:1],
                                   nframes=n8)
        torch.cuda.synchronize(dev)
        multi.sync()
        barrier()
        t8 = torch.tensor([time.perf_counter() - t80], dtype=torch.float64, device=dev)
        dist.all_reduce(t8, op=dist.ReduceOp.MAX)
        tiled8 = {"frames": n8, "output": "rgba8 (4 B/px gathered)",
                  "ms_per_step": round(float(t8.item()) / n8 * 1e3, 4),
                  "value": round(total_segs * n8 / float(t8.item()) / 1e6, 2), "unit": "Mrays/s"}

    # ---- side run: BASELINE config 5 (7680x4320, 256 spheres, depth 8; the north_star's
    # 8-GPU roofline run) through the same frame operator, row-tiled over the N ranks with
    # the interleaved layout (tile rows dealt round-robin: the sphere cloud's heavy rows are
    # shared; contiguous bands leave one rank 2.7x the average, tools/band_model.py) ----
    c5 = None
    if multi is not None and not args.no_sweep and args.config != "c5" and not args.no_c5:
        c5cfg = scenes.CONFIGS["c5"]
        c5sc = c5cfg.scene()
        c5prims = scenes.to_prims(c5sc)
        c5cam = capi.camera_init(**scenes.camera_args(c5cfg.width, c5cfg.height))
        c5n = 8
        multi.set_scene(c5prims)
        rend.set_scene(c5prims)
        layouts = (1, 0) if multi.nranks > 1 else (0,)
        # per-frame exchange for these 400-MB frames (the batched one would need 2 B frame
        # buffers; a c5 part's exchange calls are negligible next to its 0.3 ms render)
        if multi.nranks > 1:
            multi.set_option(capi.RT_OPT_MULTI_BATCH, 1)
        c5 = {"workload": f"c5:{c5cfg.width}x{c5cfg.height}:d{c5cfg.depth}:s256w0",
              "precision": args.precision, "frames": c5n}
        # census of this rank's rows (interleaved parts: same total as any layout)
        nr5 = capi.interleaved_rows(c5cfg.height, world, rank)
        cbuf = torch.empty((max(1, nr5), c5cfg.width, 3), dtype=torch.float32, device=dev)
        segs_t.zero_()
        rend.render_device_interleaved(c5cam, c5cfg.depth, world, rank, cbuf.data_ptr(), prec,
                                       d_segments=segs_t.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        s5 = segs_t.clone()
        if world > 1:
            dist.all_reduce(s5, op=dist.ReduceOp.SUM)
        c5segs = int(s5.item())
        del cbuf
        f5 = ([torch.empty((c5cfg.height, c5cfg.width, 3), dtype=torch.float32, device=dev)
               for _ in range(2)] if multi.has_root else [])
        p5 = [b.data_ptr() for b in f5]
        sp5 = st_ptrs[:2] if multi.has_root else st_ptrs[:1]
        for lay in layouts:
            multi.set_option(capi.RT_OPT_MULTI_LAYOUT, lay)
            multi.render_device_frames([c5cam], c5cfg.depth, p5, prec, flags, capi.RT_OUT_RGB_F32,
                                       streams=sp5, nframes=2)
            torch.cuda.synchronize(dev)
            multi.sync()
            barrier()
            t50 = time.perf_counter()
            multi.render_device_frames([c5cam], c5cfg.depth, p5, prec, flags, capi.RT_OUT_RGB_F32,
                                       streams=sp5, nframes=c5n)
            torch.cuda.synchronize(dev)
            multi.sync()
            barrier()
            t5 = torch.tensor([time.perf_counter() - t50], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(t5, op=dist.ReduceOp.MAX)
            name = "interleaved" if lay == 1 else ("contiguous" if multi.nranks > 1 else "one GPU")
            c5[name] = {"ms_per_frame": round(float(t5.item()) / c5n * 1e3, 3),
                        "mrays_per_s": round(c5segs * c5n / float(t5.item()) / 1e6, 1)}
        c5["segments_per_frame"] = c5segs
        multi.set_option(capi.RT_OPT_MULTI_LAYOUT, 0)
        if multi.nranks > 1:
            multi.set_option(capi.RT_OPT_MULTI_BATCH, rank_batch)
        del f5

    # distinct GPUs under the ranks (a rehearsal runs several ranks on one GPU)
    dv = torch.zeros(max(64, local + 1), dtype=torch.int64, device=dev)
    dv[local] = 1
    if world > 1:
        dist.all_reduce(dv, op=dist.ReduceOp.MAX)
    devices_used = int((dv > 0).sum().item())
    PHASE[0] = "report"
    result = None
    if rank == 0:
        ms_step = elapsed_s / args.steps * 1e3
        value = total_segs * args.steps / elapsed_s / 1e6
        frames_per_step = 1 if tiled_mode else world
        px_step = W * H * frames_per_step
        kernel_s = kernel_ms * 1e-3
        out_bytes = nrows * W * (4 if args.out == "rgba8" else 12)
        alg_bytes = out_bytes + scene_bytes(n_sph, n_wall, len(sc))
        tag = cfg.name if not (tiled_mode and world > 1) else "c4"
        workload = f"{tag}:{W}x{H}:d{depth}:s{n_sph}w{n_wall}"
        kern_workload = f"{cfg.name}:{W}x{H}:d{depth}:s{n_sph}w{n_wall}"
        # PMC was collected on the one-GPU kernel (the whole frame, fp32 RGB output); a
        # 1/N band's kernel is not the profiled one
        traffic = None
        if args.out == "rgb_f32" and nrows == H:
            e = load_profile(args.traffic_json, kern_workload, args.precision)
            traffic = None if e is None else float(e["hbm_bytes_per_launch"])
        valu_hw = load_profile(args.valu_json, kern_workload, args.precision) if nrows == H else None
        flops = my_segs * flop_per_segment(n_sph, n_wall)
        valu_peak = VALU_PEAK_TFLOPS[args.precision]
        if tiled_mode:
            gname = ({"rccl": "RCCL send/recv, rt_multi", "ipc": "HIP IPC copies, rt_multi (rehearsal)",
                      "copy": "peer copies, rt_multi"}[args.transport] if multi is not None
                     else "torch.distributed " + backend)
            par = (f"row-tiled x{world} + gather ({gname})"
                   if world > 1 else "one GPU (the one band is the whole frame)")
            if args.local_ranks > 1:
                par = f"REHEARSAL: {args.local_ranks} ranks on one GPU, peer copies"
        else:
            par = f"frame-sharded x{world}"
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if tiled_mode else "weak",
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
                "parallelism": par,
                "band_rows_rank0": nrows,
                "band_layout": args.band_layout if (tiled_mode and (world > 1 or args.local_ranks > 1)) else None,
                "rank_frames_in_flight": args.rank_frames if (tiled_mode and (world > 1 or args.local_ranks > 1)) else None,
                "frames_per_gather": args.rank_batch if (tiled_mode and world > 1) else None,
                "frames_per_launch": (frame_batch if (multi is not None and multi.nranks > 1)
                                      else (args.frame_batch if fb1 else 1)),
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                "host_box_cache": bool(args.box_cache),
                "row_feedback": args.row_feedback,
                "frames_in_flight": fif,
                "backend": backend if world > 1 else None,
                "transport": args.transport if world > 1 else None,
                "devices": devices_used,
                "rehearsal": devices_used < n_ranks,
                "frame_buffers": nbuf,
            },
            "ms_per_frame": round(ms_step / frames_per_step, 4),
            "mpx_per_s": round(px_step * args.steps / elapsed_s / 1e6, 2),
            # one frame (this rank's rows) at a time on one stream (HIP events around
            # back-to-back launches): the per-frame latency the rooflines are priced on
            "kernel_ms": round(kernel_ms, 4),
            "stream_ms_per_step": round(stream_ms, 4),
            "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "timed_edges_us": {"synchronized": round(t_synced * 1e6, 1),
                               "end": round((t1 - t0) * 1e6, 1)},
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
                "convention": "SURVEY 8d: F_seg = 30*N_sphere + 38*N_wall + 60, FMA = 2 — "
                              "algorithmic-equivalent: it prices a full linear scan, while "
                              "the kernels cull (tile bins, cone, clusters), so it credits "
                              "work never executed (c5 gives 1.26x peak); `hw` is measured",
                "hw": valu_hw,
            },
            "cpu_baseline": None,
            "precision_sweep": sweep or None,
            "sun_extension": sun_ext,
            "moving_camera": moving,
            "steady_state": steady,
            "window_rhythm": windows,
            "frame_sharded": sharded,
            "tiled_rgba8": tiled8,
            "c5_tiled": c5,
            "gather_check": gather_check,
        }
        if world == 1 and not args.no_cpu_baseline and args.cpu_seconds > 0:
            result["cpu_baseline"] = cpu_baseline(cfg, prims, cam0, depth, flags, args.cpu_seconds)
        print(json.dumps(result), file=json_out, flush=True)
    if multi is not None:
        multi.close()
    rend.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
