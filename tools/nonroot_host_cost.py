#!/usr/bin/env python3
"""Host µs per frame of what a NON-ROOT rank of the process-per-GPU gather enqueues
(rt_multi.cpp enqueue_rank, RCCL transport), emulated call for call in one thread on one
GPU with the GPU held busy behind a spin kernel (so no call waits for it):

    hipStreamWaitEvent(render[s], ev_sent[s])       band slot s free (its last send done)
    rt_render_device(band rows -> band[s], render[s])
    hipEventRecord(ev_rendered[s], render[s])
    hipStreamWaitEvent(comm, ev_rendered[s])
    <send>                                           ncclSend; here a same-device copy of the
                                                     band, or an RCCL self send/recv pair
    hipEventRecord(ev_sent[s], comm)
    hipStreamWaitEvent(caller, ev_sent[s])           only when the caller passes a stream

Also each piece alone, the render through the pipelined frame loop (per-frame launches, and
RT_OPT_FRAME_BATCH = 4 / 8: a rank's band frames on one stream as one launch per group), and
the RCCL one-rank loopback operator's frame (its root enqueues a self ncclSend/ncclRecv group
per frame, or per batch of 4 or 10 frames with RT_OPT_MULTI_BATCH, with and without
RT_OPT_FRAME_BATCH; 2 B frame buffers, as a batch needs a distinct buffer per frame).
One GPU, one process: the runtime serialises nothing here that a rank process would not.

    python tools/nonroot_host_cost.py > nonroot.json   (CFG=c2, NB=8 by default)
"""
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS[os.environ.get("CFG", "c2")]
    nb = int(os.environ.get("NB", "8"))
    n = int(os.environ.get("N", "20"))
    slots = 4
    prims = scenes.to_prims(cfg.scene())
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    H, W = cam.height, cam.width
    r0, nr = capi.band_rows(H, nb, nb // 2)  # a middle band (the c2 heavy rows)
    fmt = capi.RT_OUT_RGBA8
    nbytes = nr * W * 4
    rs = [torch.cuda.Stream(dev) for _ in range(slots)]
    comm = torch.cuda.Stream(dev)
    caller = torch.cuda.Stream(dev)
    band = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(16)]
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    hip = C.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_uint]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipStreamWaitEvent.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]

    def ev():
        e = C.c_void_p()
        assert hip.hipEventCreateWithFlags(C.byref(e), 2) == 0  # hipEventDisableTiming
        return e
    ev_rendered = [ev() for _ in range(slots)]
    ev_sent = [ev() for _ in range(slots)]
    for s in range(slots):
        hip.hipEventRecord(ev_sent[s], C.c_void_p(comm.cuda_stream))
    r = capi.Renderer(0)
    r.set_scene(prims)
    torch.cuda.synchronize()

    def spin():
        for s_ in rs + [comm, caller]:
            with torch.cuda.stream(s_):
                torch.cuda._sleep(int(4e8))

    def timed(fn, nrep=4):
        best = 1e9
        for _ in range(nrep):
            torch.cuda.synchronize()
            spin()
            t0 = time.perf_counter()
            fn()
            best = min(best, (time.perf_counter() - t0) / n * 1e6)
            torch.cuda.synchronize()
        return round(best, 2)

    def render(s):
        r.render_device(cam, cfg.depth, band[s].data_ptr(), capi.RT_PREC_PATH64, 0, fmt, row0=r0,
                        nrows=nr, stream=rs[s].cuda_stream)

    def frame(f, send, caller_wait):
        s = f % slots
        hip.hipStreamWaitEvent(C.c_void_p(rs[s].cuda_stream), ev_sent[s], 0)
        render(s)
        hip.hipEventRecord(ev_rendered[s], C.c_void_p(rs[s].cuda_stream))
        hip.hipStreamWaitEvent(C.c_void_p(comm.cuda_stream), ev_rendered[s], 0)
        if send:
            hip.hipMemcpyAsync(C.c_void_p(dst.data_ptr()), C.c_void_p(band[s].data_ptr()), nbytes, 3,
                               C.c_void_p(comm.cuda_stream))
        hip.hipEventRecord(ev_sent[s], C.c_void_p(comm.cuda_stream))
        if caller_wait:
            hip.hipStreamWaitEvent(C.c_void_p(caller.cuda_stream), ev_sent[s], 0)

    res = {"cfg": cfg.name, "band": f"rows {r0}..{r0 + nr - 1} of {H} (1/{nb})", "output": "rgba8",
           "frames_per_call": n}
    res["render_only"] = timed(lambda: [render(f % slots) for f in range(n)])
    res["render_frames_pipelined"] = timed(lambda: r.render_device_frames(
        [cam], cfg.depth, [b.data_ptr() for b in band[:slots]], capi.RT_PREC_PATH64, 0, fmt, row0=r0,
        nrows=nr, streams=[s_.cuda_stream for s_ in rs], nframes=n))
    # a batch's band frames on ONE stream (what rt_multi's batch_send does with
    # RT_OPT_FRAME_BATCH): per-frame launches vs one launch per group of B
    for fb in (1, 4, 8):
        r.set_option(capi.RT_OPT_FRAME_BATCH, fb)
        res[f"render_frames_one_stream_frame_batch{fb}"] = timed(lambda: r.render_device_frames(
            [cam], cfg.depth, [b.data_ptr() for b in band[:max(fb, 4)]], capi.RT_PREC_PATH64, 0, fmt,
            row0=r0, nrows=nr, streams=[rs[0].cuda_stream], nframes=n))
    r.set_option(capi.RT_OPT_FRAME_BATCH, 1)
    res["hipEventRecord"] = timed(lambda: [hip.hipEventRecord(ev_rendered[f % slots], C.c_void_p(
        rs[f % slots].cuda_stream)) for f in range(n)])
    res["hipStreamWaitEvent"] = timed(lambda: [hip.hipStreamWaitEvent(C.c_void_p(comm.cuda_stream),
                                                                      ev_sent[f % slots], 0) for f in range(n)])
    res["hipMemcpyAsync_band"] = timed(lambda: [hip.hipMemcpyAsync(
        C.c_void_p(dst.data_ptr()), C.c_void_p(band[f % slots].data_ptr()), nbytes, 3,
        C.c_void_p(comm.cuda_stream)) for f in range(n)])
    res["nonroot_frame_no_send"] = timed(lambda: [frame(f, False, False) for f in range(n)])
    res["nonroot_frame_copy_send"] = timed(lambda: [frame(f, True, False) for f in range(n)])
    res["nonroot_frame_copy_send_caller_wait"] = timed(lambda: [frame(f, True, True) for f in range(n)])
    r.close()
    # the one-rank operators: COPY (no exchange) and RCCL loopback (a self send/recv group)
    for name, tr, b, fb in (("multi_1_copy", capi.RT_TRANSPORT_COPY, 1, 1),
                            ("multi_1_loopback", capi.RT_TRANSPORT_RCCL_LOOPBACK, 1, 1),
                            ("multi_1_loopback_batch4", capi.RT_TRANSPORT_RCCL_LOOPBACK, 4, 1),
                            ("multi_1_loopback_batch4_frame_batch", capi.RT_TRANSPORT_RCCL_LOOPBACK, 4, 4),
                            ("multi_1_loopback_batch8_frame_batch", capi.RT_TRANSPORT_RCCL_LOOPBACK, 8, 8),
                            ("multi_1_loopback_batch10", capi.RT_TRANSPORT_RCCL_LOOPBACK, 10, 1)):
        frames = [torch.empty(H * W * 4, dtype=torch.uint8, device=dev) for _ in range(max(2, 2 * b))]
        with capi.MultiRenderer([0], transport=tr) as m:
            m.set_scene(prims)
            m.set_option(capi.RT_OPT_MULTI_BATCH, b)
            m.set_option(capi.RT_OPT_FRAME_BATCH, fb)
            sp = [rs[0].cuda_stream, rs[1].cuda_stream]
            m.render_device_frames([cam], cfg.depth, [f_.data_ptr() for f_ in frames], capi.RT_PREC_PATH64,
                                   0, fmt, streams=sp, nframes=4)
            torch.cuda.synchronize()
            res[name] = timed(lambda: m.render_device_frames(
                [cam], cfg.depth, [f_.data_ptr() for f_ in frames], capi.RT_PREC_PATH64, 0, fmt,
                streams=sp, nframes=n))
            torch.cuda.synchronize()
            m.sync()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
