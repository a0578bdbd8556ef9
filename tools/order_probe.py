#!/usr/bin/env python3
"""Kernel time of a cull config (c5, c3) with the scene's spheres in other orders: the
scene's, nearest to the camera first, kd-split chunks of 64, and those chunks nearest
first.  Only the tie-break order of equal distances differs between the frames (the cull
kernels compare scene indices on ties), so this prices a sphere permutation for the cull
kernels' 64-sphere chunks before building one.

    python tools/order_probe.py c5

Caveat: the orders are timed one after another on re-uploaded scenes, not interleaved; the
built variant's interleaved A/B (tools/ab.py) disagreed with it.
"""
import json, os, sys, ctypes as C
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes
import torch
dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c5"]
sc = cfg.scene()
sph = [o for o in sc if o.kind == capi.RT_PRIM_SPHERE]
rest = [o for o in sc if not o.kind == capi.RT_PRIM_SPHERE]
def key_dist(s): return sum(c * c for c in s.position)
def kd(lst, depth=0):
    if len(lst) <= 64: return lst
    ax = max(range(3), key=lambda a: max(s.position[a] for s in lst) - min(s.position[a] for s in lst))
    lst = sorted(lst, key=lambda s: s.position[ax]); h = len(lst) // 2
    return kd(lst[:h]) + kd(lst[h:])
def kd_near(lst):
    # kd chunks of 64, chunks ordered by distance of their centroid from the camera
    ch = kd(lst); chunks = [ch[i:i + 64] for i in range(0, len(ch), 64)]
    chunks.sort(key=lambda c: sum(key_dist(s) for s in c) / len(c))
    return [s for c in chunks for s in c]
orders = {"scene": sph, "near_first": sorted(sph, key=key_dist), "kd64": kd(sph), "kd64_near": kd_near(sph)}
cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
out = torch.empty((cfg.height, cfg.width, 3), device=dev)
r = capi.Renderer(0)
res = {}
for rep in range(2):
    for name, o in orders.items():
        r.set_scene(scenes.to_prims(o + rest))
        for _ in range(2):
            r.render_device(cam, cfg.depth, out.data_ptr(), capi.RT_PREC_PATH64, stream=st.cuda_stream)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        n = 10 if cfg.name == "c5" else 40
        for _ in range(n):
            r.render_device(cam, cfg.depth, out.data_ptr(), capi.RT_PREC_PATH64, stream=st.cuda_stream)
        e1.record(st); torch.cuda.synchronize()
        res.setdefault(name, []).append(round(e0.elapsed_time(e1) / n, 4))
print(json.dumps({"config": cfg.name, "ms": res}))
