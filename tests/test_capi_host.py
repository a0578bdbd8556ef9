"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/*.h
declares, and its host-only helpers (Camera::init restatement, band partition, format
sizes, status strings) behave — no device compute is issued here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO, has_gpu
from rtamd import capi, scenes


def _declared(header: str):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = capi.load()
    declared = _declared("rt_capi.h")
    assert len(declared) >= 12
    for name in declared:
        assert hasattr(lib, name), name
    bound = {n for n, _, _ in capi.SIGNATURES}
    assert set(declared) == bound, set(declared) ^ bound


def test_nm_dynamic_exports():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (rt_[a-z0-9_]+)$", out, flags=re.M))
    assert set(_declared("rt_capi.h")) <= exported


def test_struct_layout_matches_header():
    assert C.sizeof(capi.rt_material) == 8 * 8
    assert C.sizeof(capi.rt_prim) == 8 + 64 + 24 + 24 + 24
    assert C.sizeof(capi.rt_camera) == 12 * 8 + 8
    assert C.sizeof(capi.rt_stats) == 16


def test_camera_init_matches_reference_kat(kat):
    for c in kat["camera_init"]:
        a = c["args"]
        cam = capi.camera_init(a["position"], a["lookat"], a["vup"], a["vfov"], a["aspect_ratio"],
                               a["image_width"])
        assert cam.height == c["height"]
        for field in ("position", "image_top_left", "pixel_delta_x", "pixel_delta_y"):
            got = np.array(list(getattr(cam, field)))
            assert np.array_equal(got, np.array(c[field])), (c["name"], field)


def test_band_rows_partition():
    for h in (0, 1, 7, 36, 1080, 4321):
        for n in (1, 2, 3, 4, 8):
            rows = []
            for r in range(n):
                r0, nr = capi.band_rows(h, n, r)
                rows.extend(range(r0, r0 + nr))
            assert rows == list(range(h))
    with pytest.raises(capi.RTError):
        capi.band_rows(10, 2, 2)


def test_formats_and_status_strings():
    lib = capi.load()
    assert lib.rt_out_bytes_per_pixel(capi.RT_OUT_RGB_F32) == 12
    assert lib.rt_out_bytes_per_pixel(capi.RT_OUT_RGB_F64) == 24
    assert lib.rt_out_bytes_per_pixel(capi.RT_OUT_RGBA8) == 4
    assert lib.rt_out_bytes_per_pixel(99) == 0
    assert lib.rt_strerror(capi.RT_OK) == b"ok"
    assert lib.rt_strerror(capi.RT_ERR_OUT_OF_RANGE) == b"row band out of range"
    assert lib.rt_capi_version() == 2
    assert lib.rt_strerror(capi.RT_ERR_COMM) == b"RCCL communication error"
    assert lib.rt_max_depth() >= 10   # rt_scene's default depth (main.cpp:89)


def test_null_args_rejected_without_device():
    lib = capi.load()
    assert lib.rt_ctx_create(0, None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_ctx_destroy(None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_set_scene(None, None, 0) == capi.RT_ERR_INVALID_ARG
    cam = capi.rt_camera()
    assert lib.rt_render(None, C.byref(cam), 0, 0, 0, 0, 0, 0, None, 0, None) == \
        capi.RT_ERR_INVALID_ARG
    assert lib.rt_camera_init(None, None, None, 90.0, 1.0, 64.0, None) == capi.RT_ERR_INVALID_ARG


def test_python_and_c_synthetic_scenes_agree(oracle):
    for ns, nw in ((8, 4), (64, 6), (256, 0), (0, 6)):
        c_prims, _ = oracle.synthetic_scene(ns, nw)
        py_prims = scenes.to_prims(scenes.synthetic_scene(ns, nw))
        assert len(c_prims) == len(py_prims)
        for a, b in zip(c_prims, py_prims):
            assert bytes(a) == bytes(b)


def test_default_scene_matches_main_cpp(oracle):
    arr = (capi.rt_prim * 3)()
    oracle.lib.orc_default_scene(arr, None)
    py = scenes.to_prims(scenes.default_scene())
    for a, b in zip(arr, py):
        assert bytes(a) == bytes(b)


def test_config_cameras():
    for name, cfg in scenes.CONFIGS.items():
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        assert (cam.width, cam.height) == (cfg.width, cfg.height), name


def test_multi_args_rejected_without_device():
    """rt_multi_* argument checks happen before any device call."""
    lib = capi.load()
    h = C.c_void_p()
    devs = (C.c_int32 * 2)(0, 1)
    assert lib.rt_multi_create(devs, 2, 2, 0, None, 0, None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(None, 1, 1, 0, None, 0, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 0, 1, 0, None, 0, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 2, 1, 0, None, 0, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 1, 2, 0, None, 7, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    # one process per GPU needs the shared communicator id; COPY is one process only
    assert lib.rt_multi_create(devs, 1, 2, 1, None, 0, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    uid = (C.c_uint8 * capi.RT_MULTI_ID_BYTES)()
    assert lib.rt_multi_create(devs, 1, 2, 1, uid, 1, C.byref(h)) == capi.RT_ERR_UNSUPPORTED
    # the loopback transport is an RCCL transport: one rank per GPU, the shared id across
    # processes; an unknown transport is rejected
    assert lib.rt_multi_create(devs, 1, 2, 1, None, capi.RT_TRANSPORT_RCCL_LOOPBACK,
                               C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 1, 2, 0, None, 9, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    # THREADS (the in-process rehearsal of one process per GPU): one rank per handle, at least
    # two ranks, the shared id that keys its mailbox
    th = capi.RT_TRANSPORT_THREADS
    assert lib.rt_multi_create(devs, 1, 2, 0, None, th, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 2, 2, 0, uid, th, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_create(devs, 1, 1, 0, uid, th, C.byref(h)) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_set_row_weights(None, None, 0) == capi.RT_ERR_INVALID_ARG
    if not has_gpu():
        assert lib.rt_multi_create(devs, 1, 1, 0, None, 0, C.byref(h)) == capi.RT_ERR_NO_DEVICE
    assert lib.rt_multi_destroy(None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_set_scene(None, None, 0) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_set_option(None, 1, 1) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_sync(None) == capi.RT_ERR_INVALID_ARG
    cam = capi.rt_camera()
    assert lib.rt_multi_render(None, C.byref(cam), 0, 0, 0, 0, None, None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_render_device(None, C.byref(cam), 0, 0, 0, 0, None, None) == \
        capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_unique_id(None) == capi.RT_ERR_INVALID_ARG
    assert lib.rt_multi_last_error(None) == b""


def test_tile_rows_is_the_interleaving_unit():
    """rt_tile_rows(): the pixel rows per tile row of the kernels — the unit rt_multi's
    interleaved layout deals and scatters (one constant for both)."""
    assert capi.load().rt_tile_rows() == 8
    assert capi.interleaved_row_index(17, 2, 1) == list(range(8, 16))


def test_interleaved_rows_partition():
    """rt_interleaved_rows: the parts' tile rows (8 pixel rows, the frame's last one short)
    cover every frame row exactly once; parts differ by at most one tile row."""
    for h in (0, 1, 7, 8, 9, 36, 1080, 4321):
        for n in (1, 2, 3, 4, 8):
            rows = []
            sizes = []
            for p in range(n):
                idx = capi.interleaved_row_index(h, n, p)
                assert capi.interleaved_rows(h, n, p) == len(idx)
                rows.extend(idx)
                sizes.append(len(idx))
            assert sorted(rows) == list(range(h))
            assert max(sizes) - min(sizes) <= 8
    with pytest.raises(capi.RTError):
        capi.interleaved_rows(10, 2, 2)


def test_weighted_band_rows_partition_and_balance():
    """rt_weighted_band_rows (RT_OPT_MULTI_LAYOUT = 2): contiguous bands whose boundaries fall
    on tile rows, covering every frame row once, each boundary the tile row whose weight prefix
    is nearest r/N of the total — so the heaviest band carries at most 1/N of the weight plus
    one tile row's; equal weights give equal tile rows; no weight at all gives equal tile rows
    too; every rank computes the same boundaries from the same weights."""
    rng = np.random.default_rng(7)
    for h in (1, 7, 8, 9, 36, 1080, 4320):
        T = capi.tile_rows_of(h)
        for n in (1, 2, 3, 4, 8):
            for kind in ("rand", "peak", "equal", "zero"):
                if kind == "rand":
                    w = rng.random(T).astype(np.float32)
                elif kind == "peak":
                    w = np.exp(-((np.arange(T) - 0.6 * T) / max(1.0, 0.05 * T)) ** 2).astype(np.float32)
                elif kind == "equal":
                    w = np.ones(T, np.float32)
                else:
                    w = np.zeros(T, np.float32)
                rows, bands = [], []
                for r in range(n):
                    r0, nr = capi.weighted_band_rows(h, n, r, w)
                    assert nr >= 0
                    assert r0 % 8 == 0 or nr == 0 or r0 == h
                    rows.extend(range(r0, r0 + nr))
                    bands.append((r0, nr))
                assert rows == list(range(h)), (h, n, kind)
                tot = float(np.sum(w, dtype=np.float64))
                if kind in ("rand", "peak") and tot > 0:
                    for r0, nr in bands:
                        t0, t1 = r0 // 8, (r0 + nr + 7) // 8
                        assert float(np.sum(w[t0:t1], dtype=np.float64)) <= tot / n + 2 * float(w.max()) + 1e-6
                if kind in ("equal", "zero") and T >= n:
                    tiles = [(r0 + nr + 7) // 8 - r0 // 8 for r0, nr in bands]
                    assert max(tiles) - min(tiles) <= 1, (h, n, kind, tiles)
    with pytest.raises(capi.RTError):
        capi.weighted_band_rows(1080, 2, 0, [1.0] * 10)          # not one weight per tile row
    with pytest.raises(capi.RTError):
        capi.weighted_band_rows(16, 2, 0, [1.0, float("nan")])   # weights must be >= 0
    with pytest.raises(capi.RTError):
        capi.weighted_band_rows(16, 2, 2, [1.0, 1.0])            # rank past nranks
