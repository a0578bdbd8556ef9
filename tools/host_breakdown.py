#!/usr/bin/env python3
"""Host cost of the pieces of one rt_render_device call (µs per call): a trivial ctypes
call, a zero-row render (argument checks, KParams, row order; no boxes, no launch), a full
render with the box memo on, and with it off.  Each timed loop is queued behind a spin
kernel (torch.cuda._sleep) on the same stream, so the GPU cannot throttle the host."""
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
    st = torch.cuda.Stream(dev)
    cfg = scenes.CONFIGS[os.environ.get("CFG", "c2")]
    lib = capi.load(sys.argv[1] if len(sys.argv) > 1 else None)
    prims = scenes.to_prims(cfg.scene())
    arr = (capi.rt_prim * len(prims))(*prims)
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = torch.empty((cam.height, cam.width, 3), device=dev)
    h = C.c_void_p()
    capi.check(lib.rt_ctx_create(0, C.byref(h)))
    capi.check(lib.rt_set_scene(h, arr, len(prims)))
    n = 200
    r0, r1 = C.c_int32(), C.c_int32()
    camp = C.byref(cam)
    optr, sptr = C.c_void_p(out.data_ptr()), C.c_void_p(st.cuda_stream)

    def timed(fn):
        best = 1e9
        for _ in range(5):
            torch.cuda.synchronize()
            with torch.cuda.stream(st):
                torch.cuda._sleep(int(3e8))  # ~0.1 s of GPU spin ahead of the calls
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            best = min(best, (time.perf_counter() - t0) / n * 1e6)
            torch.cuda.synchronize()
        return round(best, 2)

    res = {"cfg": cfg.name}
    res["ctypes_trivial"] = timed(lambda: lib.rt_band_rows(1080, 1, 0, C.byref(r0), C.byref(r1)))
    res["render_0_rows"] = timed(lambda: lib.rt_render_device(h, camp, 0, 0, cfg.depth, 3, 0, 0, optr,
                                                              None, sptr))
    lib.rt_set_option(h, capi.RT_OPT_BOX_CACHE, 1)
    res["render_boxmemo_on"] = timed(lambda: lib.rt_render_device(h, camp, 0, cam.height, cfg.depth, 3, 0, 0,
                                                                  optr, None, sptr))
    lib.rt_set_option(h, capi.RT_OPT_BOX_CACHE, 0)
    res["render_boxmemo_off"] = timed(lambda: lib.rt_render_device(h, camp, 0, cam.height, cfg.depth, 3, 0,
                                                                   0, optr, None, sptr))
    lib.rt_set_option(h, capi.RT_OPT_ROW_FEEDBACK, 0)
    res["render_off_nofeedback"] = timed(lambda: lib.rt_render_device(h, camp, 0, cam.height, cfg.depth, 3,
                                                                      0, 0, optr, None, sptr))
    t = C.c_int16 * 8192
    buf = t()
    nb, md = C.c_int32(), C.c_int32()
    res["frame_boxes_hostonly"] = timed(lambda: lib.rt_frame_boxes(arr, len(prims), camp, 0, cam.height, buf,
                                                                   1024, C.byref(nb), C.byref(md)))
    print(json.dumps(res), flush=True)
    lib.rt_ctx_destroy(h)


if __name__ == "__main__":
    main()
