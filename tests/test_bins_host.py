"""CPU check of the tile bins' host half (rt_frame_boxes, rt_capi.cpp frame_boxes): every
pixel whose path, in the oracle's fp64 restatement of the reference, hits primitive j on
its primary segment lies inside j's primary pixel box; every pixel whose primary ray hit
wall w (and whose first bounce off it hit j) lies inside j's box for the camera mirrored
in w; likewise for two-wall chains.  The kernel skips a primitive for an 8x8 tile only
when its box misses the whole tile, so this is the property the GPU path's exactness
rests on (the GPU test test_tile_bins_are_output_invariant checks the frames themselves).
No device is used."""
import math

import numpy as np
import pytest

from rtamd import capi, scenes

B = 1000003  # rt_oracle.c path signature: sig = sig * B + (scene index + 1) per segment


def _slots(sc):
    """scene index -> material slot (spheres in order, then walls that can ever be hit)."""
    sph = [j for j, o in enumerate(sc) if o.kind == capi.RT_PRIM_SPHERE]
    wal = []
    for j, o in enumerate(sc):
        if o.kind != capi.RT_PRIM_WALL:
            continue
        n = scenes.normalize3(o.normal)
        cz = (n[1], -n[0], 0.0)  # cross(n, z)
        if math.isnan(n[0]) or (cz[0] == 0.0 and cz[1] == 0.0):
            continue  # NaN basis: never hit, not uploaded
        wal.append(j)
    m = {j: s for s, j in enumerate(sph)}
    m.update({j: len(sph) + w for w, j in enumerate(wal)})
    return m, len(sph), len(wal)


def _decode(sig):
    """path signature -> list of scene indices (-1 = miss) per segment (<= 3 segments)."""
    sig = int(sig)
    digits = []
    while True:
        digits.append(sig % B)
        sig //= B
        if sig == 0:
            break
    return [d - 1 for d in reversed(digits)]


def _inside(box, x, i):
    return box[0] <= x <= box[1] and box[2] <= i <= box[3]


def _check(oracle, sc, cam, row0=0, nrows=None):
    prims = scenes.to_prims(sc)
    if nrows is None:
        nrows = cam.height - row0
    prim_boxes, mir, depth = capi.frame_boxes(prims, cam, row0, nrows)
    slot, nS, nW = _slots(sc)
    np_ = nS + nW
    assert len(prim_boxes) == np_
    _, _, _, sig = oracle.render(prims, cam, 2, row0=row0, nrows=nrows, want64=False,
                                 want_sig=True)
    lvl1 = mir[:nW * np_].reshape(nW, np_, 4) if depth >= 1 else None
    lvl2 = mir[nW * np_:nW * np_ + nW * nW * np_].reshape(nW, nW, np_, 4) if depth >= 2 else None
    checked = [0, 0, 0]
    for r in range(nrows):
        i = row0 + r
        for x in range(cam.width):
            path = _decode(sig[r, x])
            if path[0] < 0:
                continue
            s0 = slot[path[0]]
            assert _inside(prim_boxes[s0], x, i), ("primary", x, i, s0, prim_boxes[s0])
            checked[0] += 1
            if len(path) < 2 or path[1] < 0 or s0 < nS or lvl1 is None:
                continue
            w1, s1 = s0 - nS, slot[path[1]]
            assert _inside(lvl1[w1, s1], x, i), ("bounce 1", x, i, w1, s1, lvl1[w1, s1])
            checked[1] += 1
            if len(path) < 3 or path[2] < 0 or s1 < nS or lvl2 is None:
                continue
            w2, s2 = s1 - nS, slot[path[2]]
            assert _inside(lvl2[w1, w2, s2], x, i), ("bounce 2", x, i, w1, w2, s2)
            checked[2] += 1
    return prim_boxes, checked


def test_boxes_cover_every_primary_and_mirror_hit_config_scenes(oracle):
    for name in ("c1", "c2"):
        cfg = scenes.CONFIGS[name]
        # the config's scene and camera at a small size of the same aspect
        w, h = (160, 120) if name == "c1" else (192, 108)
        cam = capi.camera_init(**scenes.camera_args(w, h))
        boxes, checked = _check(oracle, cfg.scene(), cam)
        assert checked[0] > 0 and (name == "c1" or checked[1] > 0), (name, checked)
        # and the bins cull: a box covers on average well under the frame
        area = [max(0, min(b[1], w - 1) - max(b[0], 0) + 1) *
                max(0, min(b[3], h - 1) - max(b[2], 0) + 1) for b in boxes]
        assert np.mean(area) < 0.5 * w * h, (name, area)


def test_boxes_cover_hits_random_views(oracle):
    """Random scenes, cameras inside the room and close to walls, wide/narrow fields of
    view, row bands: the boxes stay conservative."""
    rng = np.random.default_rng(7)
    for trial in range(10):
        sc = scenes.synthetic_scene(int(rng.integers(0, 10)), int(rng.integers(1, 7)),
                                    seed=int(rng.integers(1 << 30)))
        for _ in range(int(rng.integers(0, 3))):
            nrm = rng.normal(size=3)
            sc.append(scenes.Wall(scenes.Material(tuple(rng.uniform(0, 1, 3)), .7),
                                  tuple(rng.uniform(-5, 8, 3)), tuple(nrm / np.linalg.norm(nrm)),
                                  float(rng.uniform(1, 6)), float(rng.uniform(1, 6))))
        pos = rng.uniform([-1, -3, -1], [6, 3, 2])
        look = pos + rng.normal(size=3)
        cam = capi.camera_init(pos, look, (0, 0, -1), float(rng.choice([30.0, 90.0, 140.0])),
                               4 / 3, 64.0)
        r0 = int(rng.integers(0, cam.height // 2))
        _check(oracle, sc, cam, row0=r0, nrows=cam.height - r0)


def test_frame_boxes_errors():
    cam = capi.camera_init(**scenes.camera_args(64, 36))
    prims = scenes.to_prims(scenes.synthetic_scene(2, 2))
    with pytest.raises(capi.RTError):
        capi.frame_boxes(prims, cam, 30, 10)  # band past the frame
    # too many primitives for the linear-scan bins: no boxes
    b, m, d = capi.frame_boxes(scenes.to_prims(scenes.synthetic_scene(70, 0)), cam)
    assert len(b) == 0 and d == 0


def test_frame_boxes_fuzz_bounds_and_capacity():
    """Host-code fuzz of the per-frame box assembly (rt_capi.cpp pack_scene, frame_boxes,
    boxes_for, the mirror-chain levels) — the hand-indexed host code `tools/asan_check.sh`
    runs under AddressSanitizer/UBSan: random scene sizes up to past the 64-primitive bin
    limit and 20 walls (mirror levels shrink with nW), degenerate primitives (zero and
    negative radii, z-normal and NaN-normal walls, far coordinates), cameras inside
    primitives and with extreme fields of view, random row bands, and capacities exactly
    at and one below the box count.  Every returned box lies in the frame/band widened by
    one pixel (or is the empty marker)."""
    rng = np.random.default_rng(2024)
    for trial in range(120):
        ns, nw = int(rng.integers(0, 70)), int(rng.integers(0, 21))
        sc = scenes.synthetic_scene(min(ns, 60), min(nw, 6), seed=int(rng.integers(1 << 30)))
        for _ in range(max(0, nw - 6)):
            nrm = rng.normal(size=3)
            if rng.random() < 0.15:
                nrm = np.array([0.0, 0.0, 1.0])           # never hit (NaN basis)
            sc.append(scenes.Wall(scenes.Material((.5, .5, .5), .5),
                                  tuple(rng.uniform(-30, 30, 3)), tuple(nrm / np.linalg.norm(nrm)),
                                  float(rng.uniform(0, 9)), float(rng.uniform(0, 9))))
        for _ in range(max(0, ns - 60)):
            sc.append(scenes.Sphere(scenes.Material((.3, .3, .3), .2),
                                    tuple(rng.uniform(-1e3, 1e3, 3)), float(rng.uniform(-1, 3))))
        if sc and rng.random() < 0.2:
            sc[0] = scenes.Sphere(scenes.Material((1, 1, 1), .5), (0.0, 0.0, 0.0), 0.0)
        prims = scenes.to_prims(sc)
        pos = rng.uniform([-2, -4, -2], [9, 4, 2])
        look = pos + rng.normal(size=3)
        vfov = float(rng.choice([0.5, 30.0, 90.0, 170.0, 179.9]))
        w = int(rng.choice([1, 8, 63, 200]))
        cam = capi.camera_init(pos, look, (0, 0, -1), vfov, float(rng.choice([1.0, 16 / 9, 0.3])), float(w))
        if cam.height <= 0:
            continue
        r0 = int(rng.integers(0, cam.height))
        nr = int(rng.integers(0, cam.height - r0 + 1))
        lib = capi.load()
        arr = (capi.rt_prim * max(1, len(prims)))(*prims)
        nb, md = capi.C.c_int32(), capi.C.c_int32()
        st = lib.rt_frame_boxes(arr, len(prims), capi.C.byref(cam), r0, nr, None, 0,
                                capi.C.byref(nb), capi.C.byref(md))
        # walls that can be hit (z-normal ones are not uploaded): nbox = spheres + those
        n_w = nb.value - sum(1 for o in sc if o.kind == capi.RT_PRIM_SPHERE) if nb.value else 0
        total = nb.value * sum(n_w ** L for L in range(md.value + 1))
        assert st == (capi.RT_OK if total == 0 else capi.RT_ERR_INVALID_ARG), trial
        if total == 0:
            continue
        out = np.full((total + 1, 4), 12345, np.int16)
        ptr = out.ctypes.data_as(capi.C.POINTER(capi.C.c_int16))
        if total > 1:   # one box short of the count: rejected, nothing written past cap
            assert lib.rt_frame_boxes(arr, len(prims), capi.C.byref(cam), r0, nr, ptr, total - 1,
                                      capi.C.byref(nb), capi.C.byref(md)) == capi.RT_ERR_INVALID_ARG
        assert lib.rt_frame_boxes(arr, len(prims), capi.C.byref(cam), r0, nr, ptr, total,
                                  capi.C.byref(nb), capi.C.byref(md)) == capi.RT_OK
        assert (out[total] == 12345).all()
        b = out[:total]
        empty = (b[:, 0] > b[:, 1]) | (b[:, 2] > b[:, 3])
        ok = empty | ((b[:, 0] >= -1) & (b[:, 1] <= cam.width) & (b[:, 2] >= r0 - 1) &
                      (b[:, 3] <= r0 + nr))
        assert ok.all(), trial
