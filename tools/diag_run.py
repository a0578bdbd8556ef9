#!/usr/bin/env python3
"""Branch-entry counters of a diagnostic build (tools/build_variant.sh diag -DRT_DIAG=1):
per setup, how many wave-iterations enter each branch body and with how many lanes.

    python tools/diag_run.py --lib ray-tracer-from-scratch_amd/lib/ab/diag.so --setups c2:4:path64
"""
import argparse
import ctypes as C
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402

NAMES = {0: "scan", 2: "sphere_hit_body", 4: "wall_sign_pass", 6: "wall_bounds_body",
         12: "bounce_scan_binned", 14: "bounce_scan_unbinned",
         8: "shade_nonterminal", 10: "terminal_f32"}
# the cull kernels' counters (c3, c5: --cull)
NAMES_CULL = {0: "cull_scan", 2: "sphere_hit_body", 4: "clusters_scan", 6: "cluster_walk_step",
              14: "cluster_visit_unpruned", 12: "cone_survivor_test", 8: "shade_nonterminal",
              10: "terminal_f32"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--setups", default="c2:4:path64")
    ap.add_argument("--cull", action="store_true", help="name the cull kernels' counters")
    args = ap.parse_args()
    names = NAMES_CULL if args.cull else NAMES
    lib = capi.load(args.lib)
    lib.rt_diag_read.argtypes = [C.POINTER(C.c_ulonglong)]
    h = C.c_void_p()
    capi.check(lib.rt_ctx_create(0, C.byref(h)))
    # the row feedback's sampled frames run the stamped build, which has no counters
    capi.check(lib.rt_set_option(h, capi.RT_OPT_ROW_FEEDBACK, 0))
    buf = (C.c_ulonglong * 16)()
    for su in args.setups.split(","):
        name, depth, prec = su.split(":")
        m = re.fullmatch(r"s(\d+)w(\d+)", name)
        if m:
            sc, w, hh = scenes.synthetic_scene(int(m.group(1)), int(m.group(2))), 1920, 1080
        else:
            cfg = scenes.CONFIGS[name]
            sc, w, hh = cfg.scene(), cfg.width, cfg.height
        prims = scenes.to_prims(sc)
        arr = (capi.rt_prim * len(prims))(*prims)
        capi.check(lib.rt_set_scene(h, arr, len(prims)))
        cam = capi.camera_init(**scenes.camera_args(w, hh))
        lib.rt_diag_read(buf)  # reset
        out = (C.c_float * (w * hh * 3))()
        st = capi.rt_stats()
        capi.check(lib.rt_render(h, C.byref(cam), 0, hh, int(depth), capi.PRECISIONS[prec], 0,
                                 capi.RT_OUT_RGB_F32, C.cast(out, C.c_void_p), 1, C.byref(st)))
        lib.rt_diag_read(buf)
        waves = (w + 7) // 8 * ((hh + 7) // 8)
        r = {"setup": su, "segments": st.segments, "waves": waves}
        for i, n in names.items():
            r[n] = {"wave_entries_per_wave": round(buf[i] / waves, 3),
                    "lanes_per_entry": round(buf[i + 1] / max(buf[i], 1), 2)}
        print(json.dumps(r), flush=True)
    lib.rt_ctx_destroy(h)


if __name__ == "__main__":
    main()
