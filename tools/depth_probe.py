#!/usr/bin/env python3
"""Marginal kernel time per bounce level at c2 (PATH64): the same scene rendered at depth
0..4 (each after enough frames for the measured row order), and depth 4 with the mirror
bins off.  Tells how much of the frame the last, unbinned bounce costs."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():  # depth_probe.py [config] [precision] [lib]
    import torch
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 3:  # an A/B build of librt_amd.so
        capi._lib = capi.load(sys.argv[3])
    cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    prec = capi.PRECISIONS[sys.argv[2] if len(sys.argv) > 2 else "path64"]
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    out = torch.empty((cfg.height, cfg.width, 3), dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    segs = torch.zeros(1, dtype=torch.int64, device=dev)
    with capi.Renderer(0) as r:
        r.set_option(capi.RT_OPT_BOX_CACHE, 0)
        r.set_scene(scenes.to_prims(cfg.scene()))

        def timed(depth, n=200):
            for _ in range(96):
                r.render_device(cam, depth, out.data_ptr(), prec, 0, capi.RT_OUT_RGB_F32,
                                stream=st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(n):
                r.render_device(cam, depth, out.data_ptr(), prec, 0, capi.RT_OUT_RGB_F32,
                                stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            segs.zero_()
            r.render_device(cam, depth, out.data_ptr(), prec, 0, capi.RT_OUT_RGB_F32,
                            d_segments=segs.data_ptr(), stream=st.cuda_stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n * 1e3, int(segs.item())

        for rep in range(2):
            for d in range(cfg.depth + 1):
                us, s = timed(d)
                print(f"rep {rep} depth {d}: {us:.1f} us, {s} segments", flush=True)
            r.set_option(capi.RT_OPT_MIRROR_BINS, 0)
            us, s = timed(cfg.depth)
            print(f"rep {rep} depth {cfg.depth} mirror bins off: {us:.1f} us", flush=True)
            r.set_option(capi.RT_OPT_MIRROR_BINS, 1)


if __name__ == "__main__":
    main()
