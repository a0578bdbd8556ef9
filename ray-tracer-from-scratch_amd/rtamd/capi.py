"""ctypes binding of include/rt_capi.h (the C-ABI drop-in boundary).

This is the binding a Python host would add; bench.py and the GPU parity tests drive the
HIP path through it.  The library is loaded from the in-tree build
(ray-tracer-from-scratch_amd/lib/librt_amd.so); a missing library raises — there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_DIR, "lib")
# RT_AMD_LIB: another build of the same C-ABI (the host sanitizer build of `make asan`)
LIB_PATH = os.environ.get("RT_AMD_LIB") or os.path.join(LIB_DIR, "librt_amd.so")
HOST_LIB_PATH = os.path.join(LIB_DIR, "librt_host.so")

# ---- enums (rt_capi.h) ----------------------------------------------------
RT_OK = 0
RT_ERR_INVALID_ARG = 1
RT_ERR_NO_DEVICE = 2
RT_ERR_HIP = 3
RT_ERR_OUT_OF_MEMORY = 4
RT_ERR_NO_SCENE = 5
RT_ERR_UNSUPPORTED = 6
RT_ERR_OUT_OF_RANGE = 7
RT_ERR_COMM = 8

RT_TRANSPORT_RCCL = 0
RT_TRANSPORT_COPY = 1
RT_TRANSPORT_RCCL_LOOPBACK = 2
RT_TRANSPORT_THREADS = 3   # rehearsal: one handle per rank in one process (include/rt_capi.h)
RT_TRANSPORT_IPC = 4       # rehearsal: one process per rank, shared-memory mailbox + HIP IPC
RT_MULTI_ID_BYTES = 128
RT_MULTI_SLOTS = 4
RT_MULTI_BATCH_MAX = 16

RT_PRIM_SPHERE = 0
RT_PRIM_WALL = 1

RT_PREC_F64 = 0
RT_PREC_F32 = 1
RT_PREC_MIXED = 2
RT_PREC_PATH64 = 3
PRECISIONS = {"f64": RT_PREC_F64, "f32": RT_PREC_F32, "mixed": RT_PREC_MIXED,
              "path64": RT_PREC_PATH64}

RT_OUT_RGB_F32 = 0
RT_OUT_RGB_F64 = 1
RT_OUT_RGBA8 = 2
RT_OUT_RGBA8_WRAP = 3

RT_FLAG_SUN = 1

RT_OPT_WAVE_CULL_MIN_SPHERES = 1
RT_OPT_STATS_DEVICE_PTR = 2
RT_OPT_EYE_TABLES = 3
RT_OPT_TILE_BINS = 4
RT_OPT_ROW_ORDER = 5
RT_OPT_MIRROR_BINS = 6
RT_OPT_BOX_CACHE = 7
RT_OPT_ROW_FEEDBACK = 8
RT_OPT_PIXEL_PAIRS = 9
RT_OPT_ROW_FEEDBACK_WARM = 10
RT_OPT_WALL_ORDER = 11
RT_OPT_CLUSTER_COS = 12
RT_OPT_MULTI_LAYOUT = 13
RT_OPT_HOST_PIPELINE = 16
RT_OPT_MULTI_FRAMES = 17
RT_OPT_MULTI_FAULT = 18
RT_OPT_MULTI_BATCH = 19
RT_OPT_MULTI_TIMEOUT_MS = 20
RT_OPT_FRAME_BATCH = 21
RT_OPT_ROW_FEEDBACK_EMA = 14
RT_OPT_ROW_FEEDBACK_ISOLATE = 15


class rt_material(C.Structure):
    _fields_ = [
        ("color", C.c_double * 3),
        ("ambient", C.c_double),
        ("metallic", C.c_double),
        ("diffuse", C.c_double),
        ("specular", C.c_double),
        ("specular_exponent", C.c_double),
    ]


class rt_prim(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("reserved", C.c_int32),
        ("mat", rt_material),
        ("position", C.c_double * 3),
        ("normal", C.c_double * 3),
        ("radius", C.c_double),
        ("length", C.c_double),
        ("width", C.c_double),
    ]


class rt_camera(C.Structure):
    _fields_ = [
        ("position", C.c_double * 3),
        ("image_top_left", C.c_double * 3),
        ("pixel_delta_x", C.c_double * 3),
        ("pixel_delta_y", C.c_double * 3),
        ("width", C.c_int32),
        ("height", C.c_int32),
    ]


class rt_stats(C.Structure):
    _fields_ = [("ms", C.c_double), ("segments", C.c_uint64)]


# Every entry point include/rt_capi.h declares: (name, restype, argtypes).
_dbl3 = C.POINTER(C.c_double)
SIGNATURES = [
    ("rt_ctx_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_ctx_destroy", C.c_int, [C.c_void_p]),
    ("rt_strerror", C.c_char_p, [C.c_int]),
    ("rt_last_hip_error", C.c_char_p, [C.c_void_p]),
    ("rt_capi_version", C.c_int, []),
    ("rt_set_scene", C.c_int, [C.c_void_p, C.POINTER(rt_prim), C.c_int32]),
    ("rt_set_option", C.c_int, [C.c_void_p, C.c_int32, C.c_int64]),
    ("rt_render", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32,
      C.c_uint32, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(rt_stats)]),
    ("rt_render_device", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32,
      C.c_uint32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rt_render_device_frames", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
      C.c_uint32, C.c_int32, C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p),
      C.c_int32, C.c_int32]),
    ("rt_camera_init", C.c_int,
     [_dbl3, _dbl3, _dbl3, C.c_double, C.c_double, C.c_double, C.POINTER(rt_camera)]),
    ("rt_out_bytes_per_pixel", C.c_int32, [C.c_int32]),
    ("rt_band_rows", C.c_int,
     [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("rt_max_depth", C.c_int32, []),
    ("rt_tile_rows", C.c_int32, []),
    ("rt_frame_boxes", C.c_int,
     [C.POINTER(rt_prim), C.c_int32, C.POINTER(rt_camera), C.c_int32, C.c_int32,
      C.POINTER(C.c_int16), C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("rt_selftest", C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.c_uint64,
                              C.POINTER(C.c_uint64)]),
    ("rt_set_row_order", C.c_int, [C.c_void_p, C.POINTER(C.c_int16), C.c_int32]),
    ("rt_interleaved_rows", C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]),
    ("rt_render_device_interleaved", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_uint32,
      C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    # multi-GPU frame operator
    ("rt_multi_unique_id", C.c_int, [C.POINTER(C.c_uint8)]),
    ("rt_multi_create", C.c_int,
     [C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.c_int32,
      C.POINTER(C.c_void_p)]),
    ("rt_multi_destroy", C.c_int, [C.c_void_p]),
    ("rt_multi_last_error", C.c_char_p, [C.c_void_p]),
    ("rt_multi_set_scene", C.c_int, [C.c_void_p, C.POINTER(rt_prim), C.c_int32]),
    ("rt_multi_set_option", C.c_int, [C.c_void_p, C.c_int32, C.c_int64]),
    ("rt_multi_render_device", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_uint32, C.c_int32, C.c_void_p,
      C.c_void_p]),
    ("rt_multi_render_device_frames", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_int32, C.c_uint32, C.c_int32,
      C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p), C.c_int32, C.c_int32]),
    ("rt_multi_render", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_uint32, C.c_int32, C.c_void_p,
      C.POINTER(rt_stats)]),
    ("rt_multi_sync", C.c_int, [C.c_void_p]),
    ("rt_multi_set_row_weights", C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int32]),
    ("rt_weighted_band_rows", C.c_int,
     [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_int32),
      C.POINTER(C.c_int32)]),
    ("rt_tile_row_costs", C.c_int,
     [C.c_void_p, C.POINTER(rt_camera), C.c_int32, C.c_int32, C.c_uint32, C.POINTER(C.c_float),
      C.c_int32]),
]

_lib = None


class RTError(RuntimeError):
    def __init__(self, status: int, detail: str = ""):
        self.status = status
        msg = f"rt status {status}"
        if _lib is not None:
            msg += f" ({_lib.rt_strerror(status).decode()})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


def load(path: str | None = None) -> C.CDLL:
    """Load librt_amd.so (raises if it was not built — the product has no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{p} not built: run `make -C ray-tracer-from-scratch_amd` (or __graft_entry__.build())")
    lib = C.CDLL(p)
    for name, res, args in SIGNATURES:
        if path is not None and not hasattr(lib, name):
            continue  # an older build loaded side by side (tools/ab.py)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(status: int, ctx=None) -> None:
    if status != RT_OK:
        detail = ""
        if ctx is not None and _lib is not None:
            detail = (_lib.rt_last_hip_error(ctx) or b"").decode()
        raise RTError(status, detail)


def _d3(v) -> C.Array:
    return (C.c_double * 3)(*[float(x) for x in v])


def camera_init(position, lookat, vup, vfov: float, aspect_ratio: float,
                image_width: float) -> rt_camera:
    """Camera::init (scene.cpp:80-106) via the C-ABI host restatement."""
    lib = load()
    cam = rt_camera()
    check(lib.rt_camera_init(_d3(position), _d3(lookat), _d3(vup), float(vfov),
                             float(aspect_ratio), float(image_width), C.byref(cam)))
    return cam


def frame_boxes(prims, cam: rt_camera, row0: int = 0, nrows: int | None = None):
    """rt_frame_boxes (host only) -> (primary [nbox, 4], mirror [.., 4], mir_depth): int16
    {x0, x1, i0, i1} boxes; the mirror array holds the levels back to back (the caller
    knows nW: level L has nW**L sequences of nbox boxes).  See include/rt_capi.h."""
    import numpy as np
    lib = load()
    if nrows is None:
        nrows = cam.height - row0
    arr = (rt_prim * max(1, len(prims)))(*prims)
    nb, md = C.c_int32(), C.c_int32()
    cap = 64 * (1 + 8 + 64 + 512)
    out = np.zeros((cap, 4), np.int16)
    check(lib.rt_frame_boxes(arr, len(prims), C.byref(cam), row0, nrows,
                             out.ctypes.data_as(C.POINTER(C.c_int16)), cap, C.byref(nb),
                             C.byref(md)))
    n = nb.value
    return out[:n], out[n:], md.value


def band_rows(height: int, nranks: int, rank: int) -> tuple[int, int]:
    lib = load()
    r0, nr = C.c_int32(), C.c_int32()
    check(lib.rt_band_rows(height, nranks, rank, C.byref(r0), C.byref(nr)))
    return r0.value, nr.value


def tile_rows_of(height: int) -> int:
    """Tile rows of a frame of `height` pixel rows (rt_tile_rows() rows each)."""
    th = load().rt_tile_rows()
    return (height + th - 1) // th


def weighted_band_rows(height: int, nranks: int, rank: int, weights) -> tuple[int, int]:
    """rt_weighted_band_rows: contiguous band of `rank` cut at tile rows so every band
    carries ~1/nranks of the per-tile-row weights."""
    lib = load()
    w = list(weights)
    arr = (C.c_float * max(1, len(w)))(*w)
    r0, nr = C.c_int32(), C.c_int32()
    check(lib.rt_weighted_band_rows(height, nranks, rank, arr, len(w), C.byref(r0), C.byref(nr)))
    return r0.value, nr.value


def interleaved_rows(height: int, nparts: int, part: int) -> int:
    """rt_interleaved_rows: pixel rows of interleaved part `part` (tile rows part, part +
    nparts, ... of 8 rows)."""
    lib = load()
    n = C.c_int32()
    check(lib.rt_interleaved_rows(height, nparts, part, C.byref(n)))
    return n.value


def interleaved_row_index(height: int, nparts: int, part: int):
    """Frame rows of interleaved part `part`, in the order the part stores them."""
    th = load().rt_tile_rows()
    rows = []
    for t in range(part, (height + th - 1) // th, nparts):
        rows.extend(range(th * t, min(th * t + th, height)))
    return rows


def out_dtype_shape(out_format: int, nrows: int, width: int):
    if out_format == RT_OUT_RGB_F32:
        return np.float32, (nrows, width, 3)
    if out_format == RT_OUT_RGB_F64:
        return np.float64, (nrows, width, 3)
    if out_format in (RT_OUT_RGBA8, RT_OUT_RGBA8_WRAP):
        return np.uint8, (nrows, width, 4)
    raise ValueError(out_format)


class Renderer:
    """One rt_ctx on one HIP device (the C-ABI's lifecycle, RAII-style)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        check(self.lib.rt_ctx_create(int(device), C.byref(h)))
        self.ctx = h
        self.device = device
        self._prims = None

    def close(self):
        if self.ctx:
            self.lib.rt_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, prims) -> None:
        arr = (rt_prim * len(prims))(*prims)
        self._prims = arr
        check(self.lib.rt_set_scene(self.ctx, arr, len(prims)), self.ctx)

    def set_option(self, option: int, value: int) -> None:
        check(self.lib.rt_set_option(self.ctx, option, value), self.ctx)

    def set_row_order(self, perm) -> None:
        """rt_set_row_order: explicit tile-row dispatch order (None or [] clears it)."""
        perm = list(perm or [])
        arr = (C.c_int16 * max(1, len(perm)))(*perm)
        check(self.lib.rt_set_row_order(self.ctx, arr if perm else None, len(perm)), self.ctx)

    def selftest(self, test: int, n: int, seed: int = 1) -> int:
        bad = C.c_uint64()
        check(self.lib.rt_selftest(self.ctx, test, n, seed, C.byref(bad)), self.ctx)
        return bad.value

    def render(self, cam: rt_camera, depth: int, precision: int = RT_PREC_F64, flags: int = 0,
               out_format: int = RT_OUT_RGB_F32, row0: int = 0, nrows: int | None = None,
               count_segments: bool = False):
        """Synchronous render into a host numpy array -> (image, stats)."""
        if nrows is None:
            nrows = cam.height - row0
        dt, shape = out_dtype_shape(out_format, nrows, cam.width)
        out = np.empty(shape, dtype=dt)
        st = rt_stats()
        check(self.lib.rt_render(self.ctx, C.byref(cam), row0, nrows, depth, precision, flags,
                                 out_format, out.ctypes.data_as(C.c_void_p),
                                 1 if count_segments else 0, C.byref(st)), self.ctx)
        return out, st

    def render_device(self, cam: rt_camera, depth: int, d_out: int, precision: int = RT_PREC_F64,
                      flags: int = 0, out_format: int = RT_OUT_RGB_F32, row0: int = 0,
                      nrows: int | None = None, d_segments: int = 0, stream: int = 0) -> None:
        """Asynchronous render into device memory `d_out` on `stream` (raw pointers)."""
        if nrows is None:
            nrows = cam.height - row0
        check(self.lib.rt_render_device(self.ctx, C.byref(cam), row0, nrows, depth, precision,
                                        flags, out_format, C.c_void_p(d_out),
                                        C.c_void_p(d_segments or None),
                                        C.c_void_p(stream or None)), self.ctx)

    def tile_row_costs(self, cam: rt_camera, depth: int, precision: int = RT_PREC_PATH64,
                       flags: int = 0):
        """rt_tile_row_costs: measured cost (sum of the waves' shader cycles / 32) of every
        tile row of one render of the whole frame (synchronous) -> numpy float32."""
        n = tile_rows_of(cam.height)
        out = np.zeros(max(1, n), np.float32)
        check(self.lib.rt_tile_row_costs(self.ctx, C.byref(cam), depth, precision, flags,
                                         out.ctypes.data_as(C.POINTER(C.c_float)), n), self.ctx)
        return out[:n]

    def render_device_interleaved(self, cam: rt_camera, depth: int, nparts: int, part: int,
                                  d_out: int, precision: int = RT_PREC_F64, flags: int = 0,
                                  out_format: int = RT_OUT_RGB_F32, out_frame_rows: bool = False,
                                  d_segments: int = 0, stream: int = 0) -> None:
        """rt_render_device_interleaved: interleaved part `part` of `nparts` into device
        memory, back to back (default) or at its frame rows."""
        check(self.lib.rt_render_device_interleaved(
            self.ctx, C.byref(cam), nparts, part, depth, precision, flags, out_format,
            C.c_void_p(d_out), 1 if out_frame_rows else 0, C.c_void_p(d_segments or None),
            C.c_void_p(stream or None)), self.ctx)

    def render_device_frames(self, cams, depth: int, d_outs, precision: int = RT_PREC_F64,
                             flags: int = 0, out_format: int = RT_OUT_RGB_F32, row0: int = 0,
                             nrows: int | None = None, streams=(), nframes: int = 1) -> None:
        """rt_render_device_frames: frame f renders cams[f % len(cams)] into
        d_outs[f % len(d_outs)] on streams[f % len(streams)] (raw pointers), one call."""
        cams = list(cams)
        if nrows is None:
            nrows = cams[0].height - row0
        ca = (rt_camera * len(cams))(*cams)
        outs = (C.c_void_p * len(d_outs))(*[C.c_void_p(o) for o in d_outs])
        sts = (C.c_void_p * max(1, len(streams)))(*[C.c_void_p(x or None) for x in streams])
        check(self.lib.rt_render_device_frames(self.ctx, ca, len(cams), row0, nrows, depth,
                                               precision, flags, out_format, outs, len(d_outs),
                                               sts, len(streams), nframes), self.ctx)


def multi_unique_id() -> bytes:
    """rt_multi_unique_id: a communicator id to share with every process (one-process-per-GPU
    model of rt_multi_create)."""
    lib = load()
    buf = (C.c_uint8 * RT_MULTI_ID_BYTES)()
    check(lib.rt_multi_unique_id(buf))
    return bytes(buf)


class MultiRenderer:
    """One rt_multi: ONE frame split into row bands over `nranks` GPUs and gathered into the
    frame buffer of rank 0 (include/rt_capi.h "multi-GPU frame operator").

    MultiRenderer([0, 1, 2, 3])                         one process drives 4 GPUs (RCCL)
    MultiRenderer([0, 0, 0], transport=RT_TRANSPORT_COPY)  3 ranks on one GPU, peer copies
    MultiRenderer([local], nranks=N, first_rank=rank, unique_id=id)   one process per GPU
    MultiRenderer([0], nranks=N, first_rank=r, unique_id=id, transport=RT_TRANSPORT_THREADS)
        rank r of N handles in this process, each driven from its own thread (rehearsal)
    """

    def __init__(self, devices, nranks: int | None = None, first_rank: int = 0,
                 unique_id: bytes | None = None, transport: int = RT_TRANSPORT_RCCL):
        self.lib = load()
        devs = list(devices)
        self.nranks = len(devs) if nranks is None else int(nranks)
        self.first_rank = int(first_rank)
        self.devices = devs
        arr = (C.c_int32 * len(devs))(*devs)
        uid = None
        if unique_id is not None:
            uid = (C.c_uint8 * RT_MULTI_ID_BYTES)(*unique_id)
        h = C.c_void_p()
        check(self.lib.rt_multi_create(arr, len(devs), self.nranks, self.first_rank, uid,
                                       int(transport), C.byref(h)))
        self.m = h

    def _check(self, st: int) -> None:
        if st != RT_OK:
            raise RTError(st, (self.lib.rt_multi_last_error(self.m) or b"").decode())

    @property
    def has_root(self) -> bool:
        return self.first_rank == 0

    def close(self):
        if getattr(self, "m", None):
            self.lib.rt_multi_destroy(self.m)
            self.m = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, prims) -> None:
        arr = (rt_prim * max(1, len(prims)))(*prims)
        self._prims = arr
        self._check(self.lib.rt_multi_set_scene(self.m, arr, len(prims)))

    def set_option(self, option: int, value: int) -> None:
        self._check(self.lib.rt_multi_set_option(self.m, option, value))

    def render(self, cam: rt_camera, depth: int, precision: int = RT_PREC_PATH64, flags: int = 0,
               out_format: int = RT_OUT_RGB_F32):
        """Synchronous: (frame on the root's process else None, stats)."""
        st = rt_stats()
        out = None
        ptr = None
        if self.has_root:
            dt, shape = out_dtype_shape(out_format, cam.height, cam.width)
            out = np.empty(shape, dtype=dt)
            ptr = out.ctypes.data_as(C.c_void_p)
        self._check(self.lib.rt_multi_render(self.m, C.byref(cam), depth, precision, flags,
                                             out_format, ptr, C.byref(st)))
        return out, st

    def render_device(self, cam: rt_camera, depth: int, d_frame: int, precision: int = RT_PREC_PATH64,
                      flags: int = 0, out_format: int = RT_OUT_RGB_F32, stream: int = 0) -> None:
        self._check(self.lib.rt_multi_render_device(self.m, C.byref(cam), depth, precision, flags,
                                                    out_format, C.c_void_p(d_frame or None),
                                                    C.c_void_p(stream or None)))

    def render_device_frames(self, cams, depth: int, d_frames, precision: int = RT_PREC_PATH64,
                             flags: int = 0, out_format: int = RT_OUT_RGB_F32, streams=(),
                             nframes: int = 1) -> None:
        cams = list(cams)
        ca = (rt_camera * len(cams))(*cams)
        d_frames = list(d_frames)
        outs = (C.c_void_p * max(1, len(d_frames)))(*[C.c_void_p(o or None) for o in d_frames])
        sts = (C.c_void_p * max(1, len(streams)))(*[C.c_void_p(x or None) for x in streams])
        self._check(self.lib.rt_multi_render_device_frames(
            self.m, ca, len(cams), depth, precision, flags, out_format, outs, len(d_frames), sts,
            len(streams), nframes))

    def sync(self) -> None:
        self._check(self.lib.rt_multi_sync(self.m))

    def set_row_weights(self, weights) -> None:
        """rt_multi_set_row_weights: per-tile-row weights of RT_OPT_MULTI_LAYOUT = 2 (the
        same on every rank; None or [] clears them)."""
        w = [float(x) for x in (weights if weights is not None else [])]
        arr = (C.c_float * max(1, len(w)))(*w)
        self._check(self.lib.rt_multi_set_row_weights(self.m, arr, len(w)))
