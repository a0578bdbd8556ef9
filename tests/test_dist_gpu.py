"""Multi-process row tiling with the HIP band renderer (world sizes 2 and 3, uneven bands):
every rank renders its band of a c2-scene frame through the C-ABI (rt_render_device on
cuda:0), rtamd.tiling gathers the bands to rank 0 — one frame (gather_frame) and frames back
to back with double buffering (TiledFrames, the bench's tiled mode) — and the assembled
frames must be bitwise the one-process frames.

One GPU box has one device, and RCCL refuses two ranks on one GPU, so the ranks share
cuda:0 and the collective is gloo (its CUDA-tensor gather); what this covers is the
product path of every rank — band offsets, ragged last band, padding, in-place slices on the
destination, buffer reuse — with the real kernels.  The RCCL transport itself is covered by
test_render_tiled_rccl_single_rank and by the driver's multi-GPU runs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, has_gpu

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame_args(k, w, h):
    from rtamd import scenes
    a = dict(scenes.camera_args(w, h))
    a["position"] = (a["position"][0] + 0.1 * k, a["position"][1], a["position"][2])
    return a


def _worker(rank, world, port, w, h, depth, fmt, q):
    import sys
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from rtamd import capi, scenes, tiling
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        rend = capi.Renderer(0)
        rend.set_scene(scenes.to_prims(scenes.synthetic_scene(8, 4)))
        ch, dt = (4, torch.uint8) if fmt == capi.RT_OUT_RGBA8 else (3, torch.float32)
        # a non-default render stream: the band waits for the buffer's producer
        # on the current stream, and the gather (on the current stream) for the band
        st = torch.cuda.Stream(dev)
        cams = [capi.camera_init(**_frame_args(k, w, h)) for k in range(3)]
        cur = {"k": 0}

        def band(row0, nrows, out):
            cs = torch.cuda.current_stream(dev)
            st.wait_stream(cs)
            rend.render_device(cams[cur["k"]], depth, out.data_ptr(), capi.RT_PREC_PATH64, 0,
                               fmt, row0=row0, nrows=nrows, stream=st.cuda_stream)
            cs.wait_stream(st)

        frame = tiling.gather_frame(band, h, w, ch, dt, dev)
        if rank == 0:
            q.put(("one", 0, frame.cpu().numpy()))
        tf = tiling.TiledFrames(band, h, w, ch, dt, dev, depth=2)
        for k in range(3):
            cur["k"] = k
            hd = tf.submit()
            if k >= 1:
                prev = (hd[0] + 1) % 2
                if tf.pending[prev] is not None:
                    tf.wait(tf.pending[prev])
                if rank == 0:
                    q.put(("seq", k - 1, tf.frame(prev).cpu().numpy()))
        tf.drain()
        if rank == 0:
            q.put(("seq", 2, tf.frame(0).cpu().numpy()))
        torch.cuda.synchronize(dev)
        rend.close()
    finally:
        dist.destroy_process_group()


# ragged heights, plus BASELINE config 4's full frame (1920x1080, 8 spheres + 4 walls,
# depth 4) in both transports: fp32 RGB and the RGBA8 epilogue
@pytest.mark.parametrize("world,w,h,fmt", [(2, 200, 113, 0), (3, 192, 101, 0), (3, 160, 90, 2),
                                           (2, 1920, 1080, 0), (3, 1920, 1080, 2)])
def test_row_tiled_hip_bands_equal_one_frame(world, w, h, fmt):
    from rtamd import capi, scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, 4, fmt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=150) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rend = capi.Renderer(0)
    try:
        rend.set_scene(scenes.to_prims(scenes.synthetic_scene(8, 4)))
        for tag, k, img in got:
            cam = capi.camera_init(**_frame_args(k, w, h))
            ref, _ = rend.render(cam, 4, capi.RT_PREC_PATH64, 0, fmt)
            assert img.shape == ref.shape, (tag, k)
            assert np.array_equal(img.view(np.uint8), ref.view(np.uint8)), (tag, k)
    finally:
        rend.close()
