"""Multi-process row tiling on CPU (gloo, world sizes 2 and 3): every rank renders its
band — here with the oracle, the CPU stand-in for the HIP band renderer — and
rtamd.tiling.gather_frame assembles the frame on rank 0, which must be bitwise the
single-process frame.  The GPU path runs the same gather_frame over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, depth, q):
    import sys
    for p in (PKG, os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as orc_mod
        from rtamd import scenes, tiling
        orc = orc_mod.Oracle()
        prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
        cam = orc.camera_init(**scenes.camera_args(w, h))

        def band(row0, nrows, out):
            o64, _, _ = orc.render(prims, cam, depth, row0=row0, nrows=nrows, nthreads=1)
            out[:nrows] = torch.from_numpy(o64)

        frame = tiling.gather_frame(band, h, w, 3, torch.float64, torch.device("cpu"))
        if rank == 0:
            q.put(frame.numpy().copy())
        # frames back to back with double buffering: frame k = camera moved k steps
        shift = {"k": 0}

        def band_k(row0, nrows, out):
            c2 = orc.camera_init(**scenes.camera_args(w, h))
            c2.position[0] += 0.1 * shift["k"]
            o64, _, _ = orc.render(prims, c2, depth, row0=row0, nrows=nrows, nthreads=1)
            out[:nrows] = torch.from_numpy(o64)

        tf = tiling.TiledFrames(band_k, h, w, 3, torch.float64, torch.device("cpu"), depth=2)
        for k in range(3):
            shift["k"] = k
            hd = tf.submit()
            if k >= 1:       # frame k-1 completes while frame k was submitted
                prev = (hd[0] + 1) % 2
                tf.wait(tf.pending[prev]) if tf.pending[prev] is not None else None
                if rank == 0:
                    q.put(("seq", k - 1, tf.frame(prev).numpy().copy()))
        tf.drain()
        if rank == 0:
            q.put(("seq", 2, tf.frame(2 % 2).numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, 48, 27), (3, 40, 37), (2, 32, 20)])
def test_row_tiled_gather_equals_single_frame(world, w, h, oracle):
    from rtamd import scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, 4, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=120)
    seq = [q.get(timeout=120) for _ in range(3)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
    cam = oracle.camera_init(**scenes.camera_args(w, h))
    ref, _, _ = oracle.render(prims, cam, 4)
    assert np.array_equal(frame.view(np.uint64), ref.view(np.uint64))
    for tag, k, img in seq:
        c2 = oracle.camera_init(**scenes.camera_args(w, h))
        c2.position[0] += 0.1 * k
        r2, _, _ = oracle.render(prims, c2, 4)
        assert np.array_equal(img.view(np.uint64), r2.view(np.uint64)), k


def test_band_partition_matches_c_abi():
    from rtamd import tiling, capi
    for h in (1, 27, 1080, 4320):
        for world in (1, 2, 4, 8):
            bands = [tiling.band_of(h, world, r) for r in range(world)]
            assert sum(n for _, n in bands) == h
            assert max(n for _, n in bands) - min(n for _, n in bands) <= 1
            assert bands == [capi.band_rows(h, world, r) for r in range(world)]


def _rgba8(o64):
    """The RGBA8 epilogue's rule (main.cpp:345 truncation, clamped; alpha 255)."""
    rgb = np.floor(np.clip(o64, 0.0, 1.0) * 255.0).astype(np.uint8)
    return np.concatenate([rgb, np.full(rgb.shape[:-1] + (1,), 255, np.uint8)], axis=-1)


def _worker_rgba8(rank, world, port, w, h, depth, q):
    import sys
    for p in (PKG, os.path.join(REPO, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as orc_mod
        from rtamd import scenes, tiling
        orc = orc_mod.Oracle()
        prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
        cam = orc.camera_init(**scenes.camera_args(w, h))

        def band(row0, nrows, out):
            o64, _, _ = orc.render(prims, cam, depth, row0=row0, nrows=nrows, nthreads=1)
            out[:nrows] = torch.from_numpy(_rgba8(o64))

        # the bench's tiled RGBA8 transport: 4 B/px uint8 bands, double-buffered
        tf = tiling.TiledFrames(band, h, w, 4, torch.uint8, torch.device("cpu"), depth=2)
        for _ in range(3):
            tf.submit()
        tf.drain()
        if rank == 0:
            q.put([tf.frame(s).numpy().copy() for s in range(2)])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, 40, 22), (3, 36, 29)])
def test_row_tiled_rgba8_gather(world, w, h, oracle):
    from rtamd import scenes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_rgba8, args=(r, world, port, w, h, 4, q))
             for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    prims = scenes.to_prims(scenes.synthetic_scene(8, 4))
    cam = oracle.camera_init(**scenes.camera_args(w, h))
    ref, _, _ = oracle.render(prims, cam, 4)
    for f in frames:
        assert f.dtype == np.uint8 and f.shape == (h, w, 4)
        assert np.array_equal(f, _rgba8(ref))
