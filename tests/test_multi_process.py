"""The multi-GPU frame operator's process-per-GPU path in REAL separate processes on one
MI355X: RT_TRANSPORT_IPC (include/rt_capi.h) — one process per rank, each an rt_multi handle
(nlocal = 1, first_rank = its rank), the exchange through a shared-memory mailbox, the
root's staging buffers shared by HIP IPC, the stream order across processes kept by
shared-memory counters set and awaited on the streams (host functions).  Everything
around the copies is the RCCL path's code (band slots, the batched exchange, the root's
staging and scatter, the non-root caller-stream waits, failure handling).

What it checks: the gathered frames of a moving camera are bitwise the one-GPU frames, in
every root buffer, per-frame and batched, contiguous / interleaved / cost-weighted bands
(config 4's full frame included); a rank that fails mid-exchange ends it for every process
(each returns an error, none hangs).  The reference renders each frame on one thread
(main.cpp:124-139, called once per frame at main.cpp:329); pixels are independent, so the
row-tiled frame must be bitwise the one-GPU frame.
"""
import os

import numpy as np
import pytest

from conftest import PKG, has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def _cam(w, h, dx=0.0):
    from rtamd import capi, scenes
    cam = capi.camera_init(**scenes.camera_args(w, h))
    cam.position[0] += dx   # Camera::forward without init() (main.cpp:265, scene.cpp:121)
    return cam


def _worker(rank, n, uid, case, q):
    import sys
    sys.path.insert(0, PKG)
    import torch
    from rtamd import capi, scenes
    res = {"rank": rank, "status": None, "error": ""}
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        w, h, nf, layout, batch, slots, weights, fault = (case[k] for k in (
            "w", "h", "nf", "layout", "batch", "slots", "weights", "fault"))
        fbatch = case.get("frame_batch", 1)
        fmt = case.get("fmt", capi.RT_OUT_RGB_F32)
        prec = case.get("prec", capi.RT_PREC_PATH64)
        prims = scenes.to_prims(scenes.CONFIGS["c2"].scene())
        cams = [_cam(w, h, 0.02 * k) for k in range(5)]
        m = capi.MultiRenderer([0], nranks=n, first_rank=rank, unique_id=uid,
                               transport=capi.RT_TRANSPORT_IPC)
        try:
            m.set_scene(prims)
            m.set_option(capi.RT_OPT_MULTI_LAYOUT, layout)
            m.set_option(capi.RT_OPT_MULTI_FRAMES, slots)
            m.set_option(capi.RT_OPT_MULTI_BATCH, batch)
            m.set_option(capi.RT_OPT_FRAME_BATCH, fbatch)
            m.set_option(capi.RT_OPT_MULTI_TIMEOUT_MS, 60000)
            if weights is not None:
                m.set_row_weights(weights)
            nb = case["nb"]
            sts = [torch.cuda.Stream(dev) for _ in range(2)]
            nbytes = h * w * capi.load().rt_out_bytes_per_pixel(fmt)
            bufs = ([torch.full((nbytes,), 255, dtype=torch.uint8, device=dev) for _ in range(nb)]
                    if rank == 0 else [])
            torch.cuda.synchronize()
            if fault and rank == fault:
                m.set_option(capi.RT_OPT_MULTI_FAULT, 1)
            m.render_device_frames(cams, 4, [b.data_ptr() for b in bufs], prec, 0, fmt,
                                   streams=[s.cuda_stream for s in (sts if rank == 0 else sts[:1])],
                                   nframes=nf)
            torch.cuda.synchronize()
            m.sync()
            if rank == 0:
                res["bufs"] = [b.cpu().numpy() for b in bufs]
            res["status"] = 0
        finally:
            m.close()
    except capi.RTError as e:
        res["status"] = e.status
        res["error"] = str(e)
    except Exception as e:   # noqa: BLE001 - reported to the parent
        res["status"] = -1
        res["error"] = repr(e)
    q.put(res)


def _run(n, case, timeout=150):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = os.urandom(128)
    procs = [ctx.Process(target=_worker, args=(r, n, uid, case, q)) for r in range(n)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=timeout) for _ in range(n)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return sorted(out, key=lambda r: r["rank"])


@pytest.fixture(scope="module")
def rend():
    from rtamd import capi
    r = capi.Renderer(0)
    yield r
    r.close()


F32, RGBA8, F64 = 0, 2, 1   # rt_out_format: RT_OUT_RGB_F32, RT_OUT_RGBA8, RT_OUT_RGB_F64


@pytest.mark.parametrize("n,w,h,layout,batch,slots,fbatch,fmt", [
    (2, 1920, 1080, 0, 1, 2, 1, F32),    # config 4's frame, per-frame exchange, contiguous bands
    (2, 1920, 1080, 2, 4, 4, 4, F32),    # config 4's frame, batched, one launch per batch
    (4, 1920, 1080, 2, 8, 4, 2, RGBA8),  # config 4, the bench's N > 1 settings, RGBA8 transport
    (3, 480, 270, 1, 1, 2, 1, F32),      # interleaved parts (staging + strided scatter)
    (3, 480, 270, 1, 1, 2, 1, F64),      # the same, fp64 frames (F64 precision)
    (4, 640, 360, 2, 3, 3, 1, F32),      # cost-weighted bands, batched (a third batch revisits buffers)
    (4, 640, 360, 0, 3, 3, 3, F32),      # the same with one launch per batch (RT_OPT_FRAME_BATCH)
    (4, 203, 117, 0, 2, 2, 1, RGBA8),    # ragged bands, RGBA8 rows of 812 B (4-byte scatter)
])
def test_ipc_processes_gather_bitwise(rend, n, w, h, layout, batch, slots, fbatch, fmt):
    from rtamd import capi, scenes
    prec = capi.RT_PREC_F64 if fmt == F64 else capi.RT_PREC_PATH64
    prims = scenes.to_prims(scenes.CONFIGS["c2"].scene())
    rend.set_scene(prims)
    cams = [_cam(w, h, 0.02 * k) for k in range(5)]
    refs = [rend.render(c, 4, prec, 0, fmt)[0] for c in cams]
    weights = rend.tile_row_costs(cams[0], 4, capi.RT_PREC_PATH64).tolist() if layout == 2 else None
    nf = 7
    nb = 2 if batch == 1 else min(nf, 2 * batch)
    case = dict(w=w, h=h, nf=nf, layout=layout, batch=batch, slots=slots, weights=weights,
                fault=0, nb=nb, frame_batch=fbatch, fmt=fmt, prec=prec)
    res = _run(n, case)
    assert all(r["status"] == 0 for r in res), [(r["rank"], r["status"], r["error"]) for r in res]
    bufs = res[0]["bufs"]
    for b in range(nb):
        lf = max(f for f in range(nf) if f % nb == b)
        assert np.array_equal(bufs[b], refs[lf % len(cams)].view(np.uint8).reshape(-1)), (n, layout, fmt, b)


@pytest.mark.parametrize("batch", [1, 4])
def test_ipc_a_failed_rank_ends_the_exchange_in_every_process(batch):
    """RT_OPT_MULTI_FAULT on rank 1 of 3 processes: rank 1's frame fails once its part was
    queued (RT_ERR_HIP), and the other processes' waits give up with RT_ERR_COMM — no
    process hangs (each reports within the test's timeout)."""
    from rtamd import capi
    case = dict(w=320, h=180, nf=9, layout=0, batch=batch, slots=2, weights=None, fault=1,
                nb=2 if batch == 1 else 8)
    res = _run(3, case, timeout=120)
    st = {r["rank"]: r["status"] for r in res}
    assert st[1] == capi.RT_ERR_HIP, res[1]["error"]
    assert st[0] == capi.RT_ERR_COMM and st[2] == capi.RT_ERR_COMM, [(r["rank"], r["error"]) for r in res]
