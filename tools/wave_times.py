#!/usr/bin/env python3
"""Per-wave timeline of one render from a diagnostic build (-DRT_WAVE_TIMES=1):
occupancy over time, the tail after the last wave starts, heavy tiles.

    tools/build_variant.sh wt -DRT_WAVE_TIMES=1
    python tools/wave_times.py --lib ray-tracer-from-scratch_amd/lib/ab/wt.so --setups c2:4:path64
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--setups", default="c2:4:path64")
    ap.add_argument("--save", default="")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    lib = capi.load(args.lib)
    h = C.c_void_p()
    capi.check(lib.rt_ctx_create(0, C.byref(h)))
    stream = torch.cuda.Stream(dev)
    saved = {}
    for su in args.setups.split(","):
        name, depth, prec = su.split(":")
        cfg = scenes.CONFIGS[name]
        prims = scenes.to_prims(cfg.scene())
        arr = (capi.rt_prim * len(prims))(*prims)
        capi.check(lib.rt_set_scene(h, arr, len(prims)))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        W, H = cam.width, cam.height
        tx, ty = (W + 7) // 8, (H + 7) // 8
        nw = tx * ty
        buf = torch.zeros(3 * nw, dtype=torch.int64, device=dev)
        out = torch.empty((H, W, 3), dtype=torch.float32, device=dev)
        pc = capi.PRECISIONS[prec]

        def launch():
            capi.check(lib.rt_render_device(h, C.byref(cam), 0, H, int(depth), pc, 0, 0,
                                            C.c_void_p(out.data_ptr()), None,
                                            C.c_void_p(stream.cuda_stream)))
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, 0))
        for _ in range(3):
            launch()
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, buf.data_ptr()))
        launch()
        torch.cuda.synchronize()
        capi.check(lib.rt_set_option(h, capi.RT_OPT_STATS_DEVICE_PTR, 0))
        a = buf.view(nw, 3).cpu().numpy()
        t0, t1 = a[:, 0].astype(np.float64), a[:, 1].astype(np.float64)
        segs = (a[:, 2] >> 32).astype(np.int64)
        base = t0.min()
        t0 = (t0 - base) * 0.01   # 100 MHz ticks -> us
        t1 = (t1 - base) * 0.01
        dur = t1 - t0
        span = t1.max()
        grid = np.linspace(0, span, 200)
        conc = np.array([((t0 <= g) & (t1 > g)).sum() for g in grid])
        last_start = t0.max()
        order = np.argsort(t0)
        r = dict(setup=su, waves=int(nw), span_us=round(span, 2), last_start_us=round(last_start, 2),
                 tail_us=round(span - last_start, 2),
                 dur_us_mean=round(dur.mean(), 3), dur_us_p50=round(float(np.median(dur)), 3),
                 dur_us_p99=round(float(np.percentile(dur, 99)), 3), dur_us_max=round(dur.max(), 3),
                 conc_max=int(conc.max()), conc_mean=round(float(conc.mean()), 1),
                 conc_at_10pct=[int(c) for c in conc[::20]],
                 wave_us_sum_over_span=round(dur.sum() / span, 1),
                 dur_vs_segs_corr=round(float(np.corrcoef(dur, segs)[0, 1]), 3),
                 first_quarter_dur=round(float(dur[order[: nw // 4]].mean()), 3),
                 last_quarter_dur=round(float(dur[order[-nw // 4:]].mean()), 3),
                 starts_per_us_by_decile=[round(float(((t0 >= a0) & (t0 < a0 + span / 10)).sum()
                                                      / (span / 10)), 1)
                                          for a0 in np.arange(10) * span / 10],
                 dur_mean_by_start_decile=[round(float(dur[(t0 >= a0) & (t0 < a0 + span / 10)]
                                                       .mean()), 2) if ((t0 >= a0) & (t0 < a0 + span / 10)).any() else None
                                           for a0 in np.arange(10) * span / 10])
        print(json.dumps(r), flush=True)
        cu = (a[:, 2] & 0xffffffff).astype(np.int64)
        top = np.argsort(-dur)[:12]
        print(json.dumps({"longest_waves": [
            dict(tile=[int(w % tx), int(w // tx)], start_us=round(float(t0[w]), 2),
                 dur_us=round(float(dur[w]), 2), segs=int(segs[w]), hw=int(cu[w])) for w in top]}))
        # how many of the 1% longest waves share a hardware slot id with another one
        k = max(1, nw // 100)
        heavy = np.argsort(-dur)[:k]
        vals, counts = np.unique(cu[heavy], return_counts=True)
        print(json.dumps({"heavy_1pct": k, "distinct_hw_ids": int(len(vals)),
                          "max_per_hw_id": int(counts.max()),
                          "heavy_start_us_p50": round(float(np.median(t0[heavy])), 2),
                          "heavy_end_us_p50": round(float(np.median(t1[heavy])), 2)}), flush=True)
        saved[su] = dict(tx=tx, ty=ty, t0=t0.round(3).tolist(), t1=t1.round(3).tolist(), segs=segs.tolist(),
                         hw=cu.tolist())
    if args.save:
        json.dump(saved, open(args.save, "w"))
    lib.rt_ctx_destroy(h)


if __name__ == "__main__":
    main()
