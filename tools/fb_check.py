#!/usr/bin/env python3
"""Row-order / row-feedback invariance check: renders a config many times with feedback on
(sampling every frame) and with random explicit row orders, and reports any pixel that
differs from a render with both off (which rows / columns, first frame)."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
from rtamd import capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2")
    ap.add_argument("--precisions", default="path64,f64,f32")
    ap.add_argument("--frames", type=int, default=40)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    rend = capi.Renderer(0)
    bad = 0
    for cname in args.configs.split(","):
        cfg = scenes.CONFIGS[cname]
        rend.set_scene(scenes.to_prims(cfg.scene()))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        H, W = cam.height, cam.width
        for pname in args.precisions.split(","):
            pc = capi.PRECISIONS[pname]
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
            rend.set_row_order(None)
            ref = torch.full((H, W, 3), -1.0, dtype=torch.float32, device=dev)
            torch.cuda.synchronize()
            rend.render_device(cam, cfg.depth, ref.data_ptr(), pc, 0, 0)
            torch.cuda.synchronize()
            rng = np.random.default_rng(1)
            for mode in ("feedback", "explicit"):
                if mode == "feedback":
                    rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 1)
                for f in range(args.frames):
                    if mode == "explicit":
                        rend.set_row_order(rng.permutation((H + 7) // 8).tolist())
                    out = torch.full((H, W, 3), -1.0, dtype=torch.float32, device=dev)
                    torch.cuda.synchronize()  # the fill runs on torch's stream, not the ctx's
                    rend.render_device(cam, cfg.depth, out.data_ptr(), pc, 0, 0)
                    torch.cuda.synchronize()
                    d = (out - ref).abs().amax(dim=2)
                    if bool((d > 0).any()):
                        rows = torch.nonzero(d.amax(dim=1) > 0).flatten().tolist()
                        cols = torch.nonzero(d.amax(dim=0) > 0).flatten().tolist()
                        unr = int((out[..., 0] == -1.0).sum())
                        print(json.dumps({"config": cname, "precision": pname, "mode": mode,
                                          "frame": f, "max": float(d.max()), "npx": int((d > 0).sum()),
                                          "unrendered": unr, "rows": rows[:20], "nrows": len(rows),
                                          "cols": cols[:20], "ncols": len(cols)}), flush=True)
                        bad += 1
                        break
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
                rend.set_row_order(None)
            print(json.dumps({"config": cname, "precision": pname, "done": True}), flush=True)
    rend.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
