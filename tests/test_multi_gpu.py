"""The multi-GPU frame operator of the C-ABI (rt_multi_*, include/rt_capi.h) on an MI355X:
ONE frame split into row bands across ranks, each band rendered by its rank's own rt_ctx,
gathered into rank 0's frame buffer.  Every gathered frame must be bitwise the one-GPU
frame (pixels are independent; the reference renders the whole frame on one thread,
main.cpp:124-139).

One GPU box has one device and RCCL takes one rank per GPU, so:
  - RCCL runs at one rank through RT_TRANSPORT_RCCL_LOOPBACK: a communicator of one rank
    and the root's band sent to itself (ncclCommInitRank, ncclGroupStart/End, ncclSend,
    ncclRecv, ncclCommGetAsyncError all execute), bitwise against the one-GPU frame; the
    plain RT_TRANSPORT_RCCL at one rank makes no communicator (nothing is exchanged);
  - the N-rank orchestration — band offsets, ragged and empty bands, double-buffered band
    slots, worker threads doing each rank's host work, caller-stream ordering — runs with
    N ranks on the same GPU through RT_TRANSPORT_COPY (peer copies instead of RCCL
    send/recv), at BASELINE config 4's full size (1920x1080, 8 spheres + 4 walls, depth 4)
    for N = 2, 3, 4, 8, fp32 RGB and RGBA8.
"""
import numpy as np
import pytest

from conftest import has_gpu
from rtamd import capi, scenes

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def rend():
    r = capi.Renderer(0)
    yield r
    r.close()


def _cam(w, h, dx=0.0):
    cam = capi.camera_init(**scenes.camera_args(w, h))
    cam.position[0] += dx   # Camera::forward without init() (main.cpp:265, scene.cpp:121)
    return cam


@pytest.mark.parametrize("transport", [capi.RT_TRANSPORT_RCCL, capi.RT_TRANSPORT_RCCL_LOOPBACK])
def test_single_rank_rccl_equals_render(rend, transport):
    """One rank: the frame operator is rt_render of the whole frame — with the plain RCCL
    transport (no communicator) and with the loopback transport, whose root renders into
    its band slot and sends it to itself through a one-rank RCCL communicator."""
    sc = scenes.synthetic_scene(8, 4)
    prims = scenes.to_prims(sc)
    rend.set_scene(prims)
    with capi.MultiRenderer([0], transport=transport) as m:
        m.set_scene(prims)
        for (w, h) in ((160, 90), (1920, 1080)):
            cam = _cam(w, h)
            for prec, fmt in ((capi.RT_PREC_PATH64, capi.RT_OUT_RGB_F32),
                              (capi.RT_PREC_F64, capi.RT_OUT_RGB_F64),
                              (capi.RT_PREC_PATH64, capi.RT_OUT_RGBA8)):
                got, st = m.render(cam, 4, prec, 0, fmt)
                ref, _ = rend.render(cam, 4, prec, 0, fmt)
                assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (w, prec, fmt)
                assert st.ms > 0


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_copy_transport_c4_bands_bitwise(rend, n):
    """BASELINE config 4 at full size split across n ranks: bitwise the one-GPU frame, in
    the bench precision and F64, fp32 RGB and the RGBA8 transport."""
    cfg = scenes.CONFIGS["c2"]   # config 4 = config 2's frame on several GPUs
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    cam = _cam(cfg.width, cfg.height)
    with capi.MultiRenderer([0] * n, transport=capi.RT_TRANSPORT_COPY) as m:
        m.set_scene(prims)
        for prec, fmt in ((capi.RT_PREC_PATH64, capi.RT_OUT_RGB_F32),
                          (capi.RT_PREC_PATH64, capi.RT_OUT_RGBA8),
                          (capi.RT_PREC_F64, capi.RT_OUT_RGB_F32)):
            got, _ = m.render(cam, cfg.depth, prec, 0, fmt)
            ref, _ = rend.render(cam, cfg.depth, prec, 0, fmt)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (n, prec, fmt)


@pytest.mark.parametrize("n,w,h", [(8, 203, 117), (8, 37, 5), (3, 1, 1), (5, 64, 36)])
def test_ragged_and_empty_bands(rend, n, w, h):
    """Heights not divisible by the rank count (bands differ by one row) and heights below
    it (empty bands: nothing rendered or sent)."""
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4, seed=5))
    rend.set_scene(prims)
    cam = _cam(w, h)
    with capi.MultiRenderer([0] * n, transport=capi.RT_TRANSPORT_COPY) as m:
        m.set_scene(prims)
        got, _ = m.render(cam, 5, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F64)
        ref, _ = rend.render(cam, 5, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F64)
        assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


@pytest.mark.parametrize("transport,n,frames", [(capi.RT_TRANSPORT_COPY, 4, 2), (capi.RT_TRANSPORT_COPY, 4, 4),
                                                (capi.RT_TRANSPORT_RCCL, 1, 2),
                                                (capi.RT_TRANSPORT_RCCL_LOOPBACK, 1, 2),
                                                (capi.RT_TRANSPORT_RCCL_LOOPBACK, 1, 3)])
def test_frames_in_flight_on_caller_streams(rend, transport, n, frames):
    """The bench's frame loop: many frames of a moving camera enqueued back to back by one
    rt_multi_render_device_frames call into two device frame buffers on two caller streams
    (band slots reused every RT_MULTI_SLOTS frames while earlier sends may be in flight).
    Each buffer ends as the frame of the last camera written to it, bitwise; a frame read
    on its stream right after its call is complete (caller-stream ordering)."""
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    W, H = 480, 270
    cams = [_cam(W, H, 0.05 * k) for k in range(5)]
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)[0] for c in cams]
    bufs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device=dev) for _ in range(2)]
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    torch.cuda.synchronize()
    with capi.MultiRenderer([0] * n, transport=transport) as m:
        m.set_scene(prims)
        m.set_option(capi.RT_OPT_MULTI_FRAMES, frames)
        nf = 13
        m.render_device_frames(cams, 4, [b.data_ptr() for b in bufs], capi.RT_PREC_PATH64,
                               streams=[s.cuda_stream for s in sts], nframes=nf)
        torch.cuda.synchronize()
        m.sync()
        for b in range(2):
            last = max(f for f in range(nf) if f % 2 == b)
            got = bufs[b].cpu().numpy()
            assert np.array_equal(got.view(np.uint32), refs[last % len(cams)].view(np.uint32)), b
        # per-frame calls: a copy enqueued on the caller's stream right after the call sees
        # the whole frame (no host synchronisation in between)
        snaps = []
        for k in range(6):
            s = sts[k % 2]
            m.render_device(cams[k % len(cams)], 4, bufs[k % 2].data_ptr(), capi.RT_PREC_PATH64,
                            stream=s.cuda_stream)
            with torch.cuda.stream(s):
                snaps.append(bufs[k % 2].clone())
        torch.cuda.synchronize()
        m.sync()
        for k, snap in enumerate(snaps):
            assert np.array_equal(snap.cpu().numpy().view(np.uint32),
                                  refs[k % len(cams)].view(np.uint32)), k


def test_options_and_scene_reach_every_rank(rend):
    """rt_multi_set_option / rt_multi_set_scene apply to every rank's ctx: a scene swap and
    options that change only scheduling/culling (output-invariant) keep the frame bitwise
    the one-GPU frame of the new scene."""
    sa = scenes.to_prims(scenes.synthetic_scene(8, 4))
    sb = scenes.to_prims(scenes.synthetic_scene(64, 6))
    cam = _cam(320, 180)
    with capi.MultiRenderer([0] * 3, transport=capi.RT_TRANSPORT_COPY) as m:
        m.set_scene(sa)
        a, _ = m.render(cam, 4, capi.RT_PREC_PATH64)
        m.set_scene(sb)
        m.set_option(capi.RT_OPT_TILE_BINS, 0)
        m.set_option(capi.RT_OPT_ROW_FEEDBACK, 1)
        b1, _ = m.render(cam, 6, capi.RT_PREC_PATH64)
        b2, _ = m.render(cam, 6, capi.RT_PREC_PATH64)
        with pytest.raises(capi.RTError):
            m.set_option(999, 1)
    rend.set_scene(sa)
    ra, _ = rend.render(cam, 4, capi.RT_PREC_PATH64)
    rend.set_scene(sb)
    rb, _ = rend.render(cam, 6, capi.RT_PREC_PATH64)
    assert np.array_equal(a.view(np.uint32), ra.view(np.uint32))
    assert np.array_equal(b1.view(np.uint32), rb.view(np.uint32))
    assert np.array_equal(b2.view(np.uint32), rb.view(np.uint32))


def test_create_errors():
    """RCCL takes one rank per GPU; a device out of range, bad rank layouts and the COPY
    transport across processes are rejected with the documented status codes."""
    import ctypes as C
    lib = capi.load()
    h = C.c_void_p()

    def create(devs, nranks, first, uid=None, tr=capi.RT_TRANSPORT_RCCL):
        arr = (C.c_int32 * len(devs))(*devs)
        st = lib.rt_multi_create(arr, len(devs), nranks, first, uid, tr, C.byref(h))
        if st == capi.RT_OK:
            lib.rt_multi_destroy(h)
        return st

    assert create([0, 0], 2, 0) == capi.RT_ERR_UNSUPPORTED
    assert create([999], 1, 0) == capi.RT_ERR_NO_DEVICE
    assert create([0], 2, 1, None) == capi.RT_ERR_INVALID_ARG          # needs the shared id
    uid = (C.c_uint8 * capi.RT_MULTI_ID_BYTES)()
    assert create([0], 2, 1, uid, capi.RT_TRANSPORT_COPY) == capi.RT_ERR_UNSUPPORTED
    assert create([0], 1, 1) == capi.RT_ERR_INVALID_ARG                # rank past nranks
    assert create([0], 1, 0, uid, capi.RT_TRANSPORT_IPC) == capi.RT_ERR_INVALID_ARG  # IPC: >= 2 ranks
    assert create([0], 2, 1, None, capi.RT_TRANSPORT_IPC) == capi.RT_ERR_INVALID_ARG  # IPC: the id
    assert create([0], 65, 1, uid, capi.RT_TRANSPORT_IPC) == capi.RT_ERR_INVALID_ARG  # <= 64 ranks
    assert len(capi.multi_unique_id()) == capi.RT_MULTI_ID_BYTES


@pytest.mark.parametrize("scene,w,h,depth", [("c2", 1920, 1080, 4), ("s64w6", 480, 270, 6),
                                             ("s256w0", 203, 117, 8)])
def test_interleaved_parts_bitwise(rend, scene, w, h, depth):
    """rt_render_device_interleaved: every part of N in {2, 3, 8}, stored back to back and at
    its frame rows, reassembles the one-GPU frame bitwise — linear-scan kernels (c2 scene)
    and the cull kernels (64 and 256 spheres: wave cone, sphere clusters), ragged heights."""
    import torch
    dev = torch.device("cuda", 0)
    sc = scenes.CONFIGS["c2"].scene() if scene == "c2" else \
        scenes.synthetic_scene(int(scene[1:].split("w")[0]), int(scene.split("w")[1]))
    prims = scenes.to_prims(sc)
    rend.set_scene(prims)
    cam = _cam(w, h)
    ref, _ = rend.render(cam, depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
    st = torch.cuda.Stream(dev)
    for n in (2, 3, 8):
        frame = torch.full((h, w, 3), -1.0, device=dev)
        asm = np.full((h, w, 3), -1.0, np.float32)
        for p in range(n):
            rows = capi.interleaved_row_index(h, n, p)
            band = torch.full((max(1, len(rows)), w, 3), -1.0, device=dev)
            torch.cuda.synchronize()
            rend.render_device_interleaved(cam, depth, n, p, band.data_ptr(), capi.RT_PREC_PATH64,
                                           stream=st.cuda_stream)
            rend.render_device_interleaved(cam, depth, n, p, frame.data_ptr(), capi.RT_PREC_PATH64,
                                           out_frame_rows=True, stream=st.cuda_stream)
            torch.cuda.synchronize()
            if rows:
                asm[rows] = band.cpu().numpy()[:len(rows)]
        assert np.array_equal(asm.view(np.uint32), ref.view(np.uint32)), (scene, n)
        assert np.array_equal(frame.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (scene, n)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_multi_interleaved_layout_bitwise(rend, n):
    """RT_OPT_MULTI_LAYOUT = 1 (interleaved tile rows): config 4's frame and a 256-sphere
    cull scene gathered from n ranks (peer copies, strided into the frame rows) are bitwise
    the one-GPU frames, in one call and as frames in flight, fp32 RGB and the RGBA8
    transport; switching layouts between frames keeps them exact."""
    import torch
    dev = torch.device("cuda", 0)
    cases = [(scenes.CONFIGS["c2"].scene(), 1920, 1080, 4),
             (scenes.synthetic_scene(256, 0), 640, 360, 8)]
    with capi.MultiRenderer([0] * n, transport=capi.RT_TRANSPORT_COPY) as m:
        for sc, w, h, depth in cases:
            prims = scenes.to_prims(sc)
            rend.set_scene(prims)
            m.set_scene(prims)
            cam = _cam(w, h)
            ref, _ = rend.render(cam, depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
            for layout in (1, 0, 1):
                m.set_option(capi.RT_OPT_MULTI_LAYOUT, layout)
                got, _ = m.render(cam, depth, capi.RT_PREC_PATH64)
                assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (n, w, layout)
            # the RGBA8 transport (4 B/px parts, strided into the frame rows)
            ref8, _ = rend.render(cam, depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGBA8)
            got8, _ = m.render(cam, depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGBA8)
            assert np.array_equal(got8, ref8), (n, w, "rgba8")
            bufs = [torch.full((h, w, 3), -1.0, device=dev) for _ in range(2)]
            sts = [torch.cuda.Stream(dev) for _ in range(2)]
            torch.cuda.synchronize()
            m.render_device_frames([cam], depth, [b.data_ptr() for b in bufs], capi.RT_PREC_PATH64,
                                   streams=[s.cuda_stream for s in sts], nframes=5)
            torch.cuda.synchronize()
            m.sync()
            for b in bufs:
                assert np.array_equal(b.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (n, w)
        with pytest.raises(capi.RTError):
            m.set_option(capi.RT_OPT_MULTI_LAYOUT, 3)
        for bad in (0, capi.RT_MULTI_SLOTS + 1):
            with pytest.raises(capi.RTError):
                m.set_option(capi.RT_OPT_MULTI_FRAMES, bad)


def test_loopback_rccl_c4_full_size_frames_in_flight(rend):
    """RT_TRANSPORT_RCCL_LOOPBACK at config 4's full size: PATH64 fp32 RGB, RGBA8 and F64
    frames through RCCL send/recv (root to itself) bitwise the one-GPU frame, then 9 frames
    in flight alternating over two caller streams (the root's band slots reused while its
    self-sends are pending), every frame complete on its stream; rt_multi_sync checks RCCL's
    async error."""
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    cam = _cam(cfg.width, cfg.height)
    with capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK) as m:
        m.set_scene(prims)
        for prec, fmt in ((capi.RT_PREC_PATH64, capi.RT_OUT_RGB_F32),
                          (capi.RT_PREC_PATH64, capi.RT_OUT_RGBA8),
                          (capi.RT_PREC_F64, capi.RT_OUT_RGB_F32)):
            got, _ = m.render(cam, cfg.depth, prec, 0, fmt)
            ref, _ = rend.render(cam, cfg.depth, prec, 0, fmt)
            assert np.array_equal(got.view(np.uint8), ref.view(np.uint8)), (prec, fmt)
        ref, _ = rend.render(cam, cfg.depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
        bufs = [torch.full((cfg.height, cfg.width, 3), -1.0, device=dev) for _ in range(2)]
        sts = [torch.cuda.Stream(dev) for _ in range(2)]
        torch.cuda.synchronize()
        m.render_device_frames([cam], cfg.depth, [b.data_ptr() for b in bufs], capi.RT_PREC_PATH64,
                               streams=[s.cuda_stream for s in sts], nframes=9)
        torch.cuda.synchronize()
        m.sync()
        for b in bufs:
            assert np.array_equal(b.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("fmt", [capi.RT_OUT_RGB_F32, capi.RT_OUT_RGBA8])
def test_loopback_rccl_batched_gather(rend, fmt):
    """RT_OPT_MULTI_BATCH through a real (one-rank) RCCL communicator: the root renders its
    band of B frames back to back, sends them to itself in ONE ncclSend/ncclRecv pair into
    its staging buffer and scatters them into the frames with the scatter kernel.  A moving
    camera, 3 B + 1 frames over 2 B buffers on 2 caller streams (B = 3, 4; and B = 16 with 7
    frames over 7 buffers: one batch): EVERY buffer is bitwise the one-GPU frame of the last
    camera written to it — the third batch renders into the first one's buffers only after
    that batch's scatter.  Too few buffers for a batch (B = 3 over 2) is refused
    (RT_ERR_UNSUPPORTED) before anything is enqueued and the one-rank handle stays usable;
    B = 1 (the per-frame exchange) on the same handle."""
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    W, H = cfg.width, cfg.height
    cams = [_cam(W, H, 0.02 * k) for k in range(5)]
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, fmt)[0] for c in cams]
    ch = 3 if fmt == capi.RT_OUT_RGB_F32 else 1
    dt = torch.float32 if fmt == capi.RT_OUT_RGB_F32 else torch.int32
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    with capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK) as m:
        m.set_scene(prims)
        for b, nb, nf in ((3, 6, 10), (4, 8, 13), (16, 7, 7), (1, 2, 9)):
            m.set_option(capi.RT_OPT_MULTI_BATCH, b)
            bufs = [torch.full((H, W, ch), -1, dtype=dt, device=dev) for _ in range(nb)]
            torch.cuda.synchronize()
            m.render_device_frames(cams, 4, [x.data_ptr() for x in bufs], capi.RT_PREC_PATH64, 0, fmt,
                                   streams=[s.cuda_stream for s in sts], nframes=nf)
            torch.cuda.synchronize()
            m.sync()
            for i in range(nb):
                lf = max(f for f in range(nf) if f % nb == i)
                assert np.array_equal(bufs[i].cpu().numpy().view(np.uint32),
                                      refs[lf % len(cams)].view(np.uint32)), (b, i)
            del bufs
        m.set_option(capi.RT_OPT_MULTI_BATCH, 3)
        two = [torch.full((H, W, ch), -1, dtype=dt, device=dev) for _ in range(2)]
        with pytest.raises(capi.RTError) as e:
            m.render_device_frames(cams, 4, [x.data_ptr() for x in two], capi.RT_PREC_PATH64, 0, fmt,
                                   streams=[s.cuda_stream for s in sts], nframes=7)
        assert e.value.status == capi.RT_ERR_UNSUPPORTED
        # usable after the refusal: two frames (one batch of 2) into the two buffers
        m.render_device_frames(cams[:2], 4, [x.data_ptr() for x in two], capi.RT_PREC_PATH64, 0, fmt,
                               streams=[s.cuda_stream for s in sts], nframes=2)
        torch.cuda.synchronize()
        m.sync()
        for i in range(2):
            assert np.array_equal(two[i].cpu().numpy().view(np.uint32), refs[i].view(np.uint32)), i
        for bad in (0, capi.RT_MULTI_BATCH_MAX + 1):
            with pytest.raises(capi.RTError):
                m.set_option(capi.RT_OPT_MULTI_BATCH, bad)


@pytest.mark.parametrize("W,fmt", [(96, capi.RT_OUT_RGBA8), (97, capi.RT_OUT_RGB_F64)])
def test_batched_gather_ragged_empty_bands_and_root_limits(rend, W, fmt):
    """RT_OPT_MULTI_BATCH with ranks that have no rows (a 5-row frame over 8 THREADS handles:
    three empty bands, which post and send nothing), batches 3 + 2 over three root buffers
    (the second batch renders into two of the first one's buffers), in RGBA8 (16-byte
    scatter) and, 97 pixels wide, fp64 RGB (rows not a multiple of 16 bytes: the 4-byte
    scatter): every buffer bitwise its last frame.  And the root-only limit: a batching
    call with more than RT_MULTI_SLOTS distinct caller streams is refused
    (RT_ERR_UNSUPPORTED) before anything is enqueued, and a one-rank handle stays usable."""
    import os
    import torch
    dev = torch.device("cuda", 0)
    H, n = 5, 8
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
    rend.set_scene(prims)
    cams = [_cam(W, H, 0.03 * k) for k in range(5)]
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, fmt)[0] for c in cams]
    shape = (H, W, 1) if fmt == capi.RT_OUT_RGBA8 else (H, W, 6)
    uid = os.urandom(capi.RT_MULTI_ID_BYTES)
    hs = [capi.MultiRenderer([0], nranks=n, first_rank=r, unique_id=uid,
                             transport=capi.RT_TRANSPORT_THREADS) for r in range(n)]
    bufs = [torch.full(shape, -1, dtype=torch.int32, device=dev) for _ in range(3)]
    sts = [torch.cuda.Stream(dev) for _ in range(n)]
    try:
        for h in hs:
            h.set_scene(prims)
            h.set_option(capi.RT_OPT_MULTI_BATCH, 3)
        torch.cuda.synchronize()

        def drive(r, h):
            h.render_device_frames(cams, 4, [b.data_ptr() for b in bufs] if r == 0 else [],
                                   capi.RT_PREC_PATH64, 0, fmt, streams=[sts[r].cuda_stream], nframes=5)
        errs = _run_threads(hs, drive)
        assert errs == [None] * n, errs
        torch.cuda.synchronize()
        for h in hs:
            h.sync()
        for i, f in enumerate((3, 4, 2)):
            assert np.array_equal(bufs[i].cpu().numpy().view(np.uint32), refs[f].view(np.uint32)), i
    finally:
        for h in hs:
            h.close()
    with capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK) as m:
        m.set_scene(prims)
        m.set_option(capi.RT_OPT_MULTI_BATCH, 2)
        many = [torch.cuda.Stream(dev) for _ in range(capi.RT_MULTI_SLOTS + 1)]
        bufs = [torch.full(shape, -1, dtype=torch.int32, device=dev) for _ in range(len(many))]
        with pytest.raises(capi.RTError):
            m.render_device_frames([cams[0]], 4, [b.data_ptr() for b in bufs], capi.RT_PREC_PATH64, 0, fmt,
                                   streams=[s.cuda_stream for s in many], nframes=len(many))
        m.render_device_frames([cams[0]], 4, [b.data_ptr() for b in bufs[:2]], capi.RT_PREC_PATH64, 0, fmt,
                               streams=[s.cuda_stream for s in many[:2]], nframes=4)
        torch.cuda.synchronize()
        m.sync()
        for b in bufs[:2]:
            assert np.array_equal(b.cpu().numpy().view(np.uint32), refs[0].view(np.uint32))


@pytest.mark.parametrize("transport,frame_batch", [("threads", 1), ("loopback", 1), ("threads", 4),
                                                   ("loopback", 4), ("threads", 2), ("loopback", 2)])
def test_batched_frames_each_whole_in_its_own_buffer(rend, transport, frame_batch):
    """B = 4 frames of a moving camera into 4 distinct buffers — every buffer
    bitwise against ITS OWN one-GPU frame (not only the last frame written) — then 4 more
    frames into the same 4 buffers (a batch revisiting an earlier batch's buffers), again
    every buffer.  Over 3 THREADS handles (the process-per-GPU shape) and the one-rank
    loopback RCCL communicator.  Then the refusal: 4 frames over 2 buffers is RT_ERR_UNSUPPORTED
    on the root before anything is enqueued; the one-rank handle stays usable, and with
    peers (THREADS) the exchange ends for every handle (RT_ERR_COMM, no hang).
    frame_batch 4 (RT_OPT_FRAME_BATCH): every rank's band frames of a batch, and the root's
    rows of them over its two caller streams, go to the GPU as one launch; frame_batch 2:
    two launches of two frames on two streams per batch (the root's rows of a frame rendered
    on the other caller stream's launch, ordered around it)."""
    import os
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    W, H = 640, 360
    cams = [_cam(W, H, 0.02 * k) for k in range(8)]
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)[0] for c in cams]
    n = 3 if transport == "threads" else 1
    if transport == "threads":
        uid = os.urandom(capi.RT_MULTI_ID_BYTES)
        hs = [capi.MultiRenderer([0], nranks=n, first_rank=r, unique_id=uid,
                                 transport=capi.RT_TRANSPORT_THREADS) for r in range(n)]
    else:
        hs = [capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK)]
    bufs = [torch.full((H, W, 3), -1.0, device=dev) for _ in range(4)]
    root_sts = [torch.cuda.Stream(dev) for _ in range(2)]
    rank_sts = [torch.cuda.Stream(dev) for _ in range(n)]
    try:
        for h in hs:
            h.set_scene(prims)
            h.set_option(capi.RT_OPT_MULTI_BATCH, 4)
            h.set_option(capi.RT_OPT_FRAME_BATCH, frame_batch)
        torch.cuda.synchronize()

        def call(cs, ptrs):
            def drive(r, h):
                h.render_device_frames(cs, 4, ptrs if r == 0 else [], capi.RT_PREC_PATH64,
                                       streams=[s.cuda_stream for s in root_sts] if r == 0
                                       else [rank_sts[r].cuda_stream], nframes=len(cs))
            return _run_threads(hs, drive)

        for half in (cams[:4], cams[4:]):
            errs = call(half, [b.data_ptr() for b in bufs])
            assert errs == [None] * n, errs
            torch.cuda.synchronize()
            for h in hs:
                h.sync()
            for i in range(4):
                want = refs[cams.index(half[i])]
                assert np.array_equal(bufs[i].cpu().numpy().view(np.uint32), want.view(np.uint32)), i
        errs = call(cams[:4], [b.data_ptr() for b in bufs[:2]])
        assert isinstance(errs[0], capi.RTError) and errs[0].status == capi.RT_ERR_UNSUPPORTED, errs
        if n > 1:
            assert all(isinstance(e, capi.RTError) and e.status == capi.RT_ERR_COMM for e in errs[1:]), errs
            for h in hs:
                with pytest.raises(capi.RTError) as e:
                    h.sync()
                assert e.value.status == capi.RT_ERR_COMM
        else:
            errs = call(cams[:4], [b.data_ptr() for b in bufs])
            assert errs == [None], errs
            torch.cuda.synchronize()
            hs[0].sync()
            for i in range(4):
                assert np.array_equal(bufs[i].cpu().numpy().view(np.uint32), refs[i].view(np.uint32)), i
    finally:
        for h in hs:
            h.close()


def test_failure_before_the_gather_is_queued_keeps_the_communicator(rend):
    """A frame that fails before any rank queued its part of the gather (here: no scene
    yet, rejected before the root's loopback send/recv) returns its own status and leaves
    the RCCL communicator usable: the next frame, once the scene is set, is bitwise the
    one-GPU frame (a caller probing options must not brick the object)."""
    import torch
    dev = torch.device("cuda", 0)
    cam = _cam(64, 36)
    buf = torch.zeros((36, 64, 3), device=dev)
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
    m = capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK)
    try:
        with pytest.raises(capi.RTError) as e1:
            m.render_device(cam, 2, buf.data_ptr(), capi.RT_PREC_PATH64)
        assert e1.value.status == capi.RT_ERR_NO_SCENE
        m.set_scene(prims)
        m.render_device(cam, 2, buf.data_ptr(), capi.RT_PREC_PATH64)
        torch.cuda.synchronize()
        m.sync()
        rend.set_scene(prims)
        ref, _ = rend.render(cam, 2, capi.RT_PREC_PATH64)
        assert np.array_equal(buf.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    finally:
        m.close()


def test_failure_after_the_gather_is_queued_breaks_the_communicator(rend):
    """A frame that fails after the root's RCCL receives were queued (RT_OPT_MULTI_FAULT
    injects exactly that on the loopback communicator) leaves the exchange out of step: the
    rt_multi reports RT_ERR_COMM on every later frame and on rt_multi_sync (which aborts the
    communicator, ncclCommAbort, instead of waiting), and destroying it returns."""
    import torch
    dev = torch.device("cuda", 0)
    cam = _cam(64, 36)
    buf = torch.zeros((36, 64, 3), device=dev)
    m = capi.MultiRenderer([0], transport=capi.RT_TRANSPORT_RCCL_LOOPBACK)
    try:
        m.set_scene(scenes.to_prims(scenes.synthetic_scene(8, 4)))
        m.render_device(cam, 2, buf.data_ptr(), capi.RT_PREC_PATH64)   # a healthy frame first
        m.set_option(capi.RT_OPT_MULTI_FAULT, 1)
        with pytest.raises(capi.RTError) as e1:
            m.render_device(cam, 2, buf.data_ptr(), capi.RT_PREC_PATH64)
        assert e1.value.status == capi.RT_ERR_HIP
        with pytest.raises(capi.RTError) as e2:
            m.render_device(cam, 2, buf.data_ptr(), capi.RT_PREC_PATH64)
        assert e2.value.status == capi.RT_ERR_COMM
        with pytest.raises(capi.RTError) as e3:
            m.sync()
        assert e3.value.status == capi.RT_ERR_COMM
    finally:
        m.close()


def _run_threads(handles, fn):
    """Drive every THREADS handle from its own thread (as one process per GPU would) and
    return the per-rank exceptions (None = ok)."""
    import threading
    errs = [None] * len(handles)

    def body(r):
        try:
            fn(r, handles[r])
        except BaseException as e:   # noqa: BLE001 - reported by the caller
            errs[r] = e

    ths = [threading.Thread(target=body, args=(r,)) for r in range(len(handles))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
        assert not t.is_alive(), "a THREADS rank hung"
    return errs


@pytest.mark.parametrize("n,layout,frames,batch", [(2, 0, 2, 1), (3, 1, 2, 1), (8, 1, 4, 1), (4, 2, 3, 1),
                                                  (8, 2, 4, 1), (2, 0, 2, 3), (4, 2, 3, 4), (8, 0, 4, 2),
                                                  (8, 2, 4, 16), (3, 1, 2, 4)])
def test_threads_transport_runs_the_process_per_gpu_branches(rend, n, layout, frames, batch):
    """RT_TRANSPORT_THREADS: n rt_multi handles in this process, one per rank (nlocal = 1,
    first_rank = r, one shared id), each driven from its own thread exactly as the
    process-per-GPU bench drives its rank — so the branches the first multi-GPU run takes
    execute here on one GPU: the non-root ranks without a frame buffer (nbufs = 0) rendering
    into their band slots and "sending" (a peer copy matched through the mailbox instead of
    ncclSend), their caller streams waiting on the send (ev_sent), and the root receiving
    every part — contiguous bands straight into the frame rows (layout 0), interleaved parts
    into its staging buffers then scattered by strided copies (layout 1: the staging
    allocation, slot reuse and scatter of the RCCL path), cost-weighted bands (layout 2).
    Config 4's full frame (1920x1080, c2 scene, depth 4), 7 frames of a moving camera in
    flight over two root buffers, 2-4 band slots per rank (RT_OPT_MULTI_FRAMES): every buffer
    is bitwise the one-GPU frame of the last camera written to it, and a rank's band is
    already in the root's frame when its caller stream has passed the frame (checked on the
    last frame).  batch > 1 (RT_OPT_MULTI_BATCH): the batched exchange — each rank's bands of
    `batch` frames in one send, the root's one receive per rank into staging and one scatter
    kernel — over min(7, 2 x batch) root buffers (a batch needs a distinct buffer per frame;
    a third batch revisits the first one's buffers after its scatter);
    the interleaved layout keeps the per-frame exchange.  A batched rank's caller stream
    follows its send (the part is in the root's staging; the frame rows come with the
    root's scatter), so the per-rank snapshot applies to batch 1 only."""
    import os
    import torch
    dev = torch.device("cuda", 0)
    cfg = scenes.CONFIGS["c2"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    W, H = cfg.width, cfg.height
    cams = [_cam(W, H, 0.02 * k) for k in range(5)]
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)[0] for c in cams]
    weights = rend.tile_row_costs(cams[0], 4, capi.RT_PREC_PATH64) if layout == 2 else None
    uid = os.urandom(capi.RT_MULTI_ID_BYTES)
    hs = [capi.MultiRenderer([0], nranks=n, first_rank=r, unique_id=uid,
                             transport=capi.RT_TRANSPORT_THREADS) for r in range(n)]
    nf = 7
    nb = 2 if batch == 1 or layout == 1 else min(nf, 2 * batch)
    bufs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device=dev) for _ in range(nb)]
    root_sts = [torch.cuda.Stream(dev) for _ in range(2)]
    rank_sts = [torch.cuda.Stream(dev) for _ in range(n)]
    last = nf - 1
    snaps = [None] * n
    try:
        for h in hs:
            h.set_scene(prims)
            h.set_option(capi.RT_OPT_MULTI_LAYOUT, layout)
            h.set_option(capi.RT_OPT_MULTI_FRAMES, frames)
            h.set_option(capi.RT_OPT_MULTI_BATCH, batch)
            if weights is not None:
                h.set_row_weights(weights)
        torch.cuda.synchronize()

        def drive(r, h):
            if r == 0:
                h.render_device_frames(cams, 4, [b.data_ptr() for b in bufs],
                                       streams=[s.cuda_stream for s in root_sts], nframes=nf)
                return
            h.render_device_frames(cams, 4, [], streams=[rank_sts[r].cuda_stream], nframes=nf)
            # past this point on the caller's stream, the rank's last band has landed in the
            # root's frame (rt_multi_render_device: "a non-NULL stream ... waits for the rank's
            # band to have been sent")
            ev = torch.cuda.Event()
            ev.record(rank_sts[r])
            ev.synchronize()
            snaps[r] = bufs[last % nb].cpu().numpy()

        errs = _run_threads(hs, drive)
        assert errs == [None] * n, errs
        torch.cuda.synchronize()
        for h in hs:
            h.sync()
        for b in range(nb):
            lf = max(f for f in range(nf) if f % nb == b)
            got = bufs[b].cpu().numpy()
            assert np.array_equal(got.view(np.uint32), refs[lf % len(cams)].view(np.uint32)), (n, layout, b)
        ref_last = refs[last % len(cams)]
        for r in range(1, n if batch == 1 or layout == 1 else 1):
            if layout == 1:
                rows = capi.interleaved_row_index(H, n, r)
            elif layout == 2:
                r0, nr = capi.weighted_band_rows(H, n, r, weights)
                rows = list(range(r0, r0 + nr))
            else:
                r0, nr = capi.band_rows(H, n, r)
                rows = list(range(r0, r0 + nr))
            assert np.array_equal(snaps[r][rows].view(np.uint32), ref_last[rows].view(np.uint32)), (n, layout, r)
    finally:
        for h in hs:
            h.close()


@pytest.mark.parametrize("failing", [1, 0])
def test_threads_transport_a_failed_rank_ends_the_exchange(rend, failing):
    """A rank whose frame fails (no scene on that rank only) ends the exchange for every
    handle: a sender's failure (failing = 1) while the root waits for its part, and a failure
    on the root only (failing = 0, ADVICE r05: the root fails on its own rows before posting
    its receives, while the sender is already waiting for them).  The other handle returns
    RT_ERR_COMM instead of hanging; both are broken (later frames and rt_multi_sync:
    RT_ERR_COMM) and close cleanly."""
    import os
    import torch
    dev = torch.device("cuda", 0)
    cam = _cam(160, 90)
    uid = os.urandom(capi.RT_MULTI_ID_BYTES)
    hs = [capi.MultiRenderer([0], nranks=2, first_rank=r, unique_id=uid,
                             transport=capi.RT_TRANSPORT_THREADS) for r in range(2)]
    buf = torch.zeros((90, 160, 3), device=dev)
    st = torch.cuda.Stream(dev)
    try:
        hs[1 - failing].set_scene(scenes.to_prims(scenes.synthetic_scene(8, 4)))

        def drive(r, h):
            h.render_device(cam, 2, buf.data_ptr() if r == 0 else 0, capi.RT_PREC_PATH64,
                            stream=st.cuda_stream if r else 0)

        errs = _run_threads(hs, drive)
        other = 1 - failing
        assert isinstance(errs[other], capi.RTError) and errs[other].status == capi.RT_ERR_COMM, errs
        assert isinstance(errs[failing], capi.RTError) and errs[failing].status == capi.RT_ERR_NO_SCENE, errs
        for h in hs:
            with pytest.raises(capi.RTError) as e:
                h.sync()
            assert e.value.status == capi.RT_ERR_COMM
    finally:
        for h in hs:
            h.close()


def test_sync_deadline_breaks_the_exchange_instead_of_blocking(rend):
    """RT_OPT_MULTI_TIMEOUT_MS: rt_multi_sync polls the streams with a deadline instead of
    blocking.  Two THREADS handles; the root's caller stream (and so its comm stream, which
    waits on it) is held by a long queue of GPU work: with a 50 ms deadline the root's
    rt_multi_sync returns RT_ERR_COMM naming the deadline (the exchange is broken), and once
    the GPU drains both handles close cleanly.  (No communicator here: aborting one while its
    kernels are still queued is the RCCL path's business, not this test's.)"""
    import os
    import torch
    dev = torch.device("cuda", 0)
    cam = _cam(64, 36)
    buf = torch.zeros((36, 64, 3), device=dev)
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
    s, s1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    uid = os.urandom(capi.RT_MULTI_ID_BYTES)
    hs = [capi.MultiRenderer([0], nranks=2, first_rank=r, unique_id=uid,
                             transport=capi.RT_TRANSPORT_THREADS) for r in range(2)]
    try:
        for h in hs:
            h.set_scene(prims)

        def drive(r, h):
            h.render_device(cam, 2, buf.data_ptr() if r == 0 else 0, capi.RT_PREC_PATH64,
                            stream=(s if r == 0 else s1).cuda_stream)

        # one frame first: its lazy allocations (band buffers, per-stream state) may wait on
        # the device, which must happen before the hold below
        assert _run_threads(hs, drive) == [None, None]
        for h in hs:
            h.sync()
        hs[0].set_option(capi.RT_OPT_MULTI_TIMEOUT_MS, 50)
        # ~0.3 s of GPU work on the root's caller stream, enqueued in microseconds
        a = torch.randn((8192, 8192), device=dev)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            for _ in range(40):
                a = torch.tanh(a @ a)
        assert _run_threads(hs, drive) == [None, None]
        with pytest.raises(capi.RTError) as e:
            hs[0].sync()
        assert e.value.status == capi.RT_ERR_COMM
        assert "deadline" in str(e.value)
        torch.cuda.synchronize()
    finally:
        for h in hs:
            h.close()
