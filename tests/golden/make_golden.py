"""Generate the committed golden fixtures from the REFERENCE's own compiled code.

Runs only where /root/reference exists (this container): `make -C oracle ref` compiles
/root/reference/{vec,scene}.cpp and the hot-path functions of main.cpp (lines 1-139,
SDL include dropped) into oracle/_ref/libref.so; this script calls them through
oracle/ref_harness.cpp and writes DATA only (inputs + expected outputs):

  tests/golden/kat.json       known-answer values per reference function
                              (Sphere/Wall::intersect, out_color, diffuse_shading,
                              specular, reflect, normalize, Camera::init, find_closest_hit)
  tests/golden/frames.npz     fp64 frames rendered by the reference's recursive_ray_tracing
                              (rt_scene's loop; depth 10 = rt_scene itself), small sizes
  tests/golden/rays.npz       single-ray traces (random origins/directions, all depths)
  tests/golden/surface.npz    main.cpp:345's surface bytes (SDL_MapRGB(val*255) through its
                              implicit double->Uint8 conversion, g++ -O3 x86-64) of every
                              frame in frames.npz, plus edge values (wrap above 1.0, NaN)

Usage:  python tests/golden/make_golden.py [--only surface]
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))

import oracle as orc_mod  # noqa: E402
from rtamd import scenes  # noqa: E402

FRAME_SCENES = {
    "default": lambda: scenes.default_scene(),
    "s8w4": lambda: scenes.synthetic_scene(8, 4),
    "s64w6": lambda: scenes.synthetic_scene(64, 6),
    "s256w0": lambda: scenes.synthetic_scene(256, 0),
}
FRAME_DEPTHS = [0, 1, 2, 4, 8, 10]
FRAME_SIZES = [(64, 36)]
EXTRA_FRAMES = [((96, 54), d) for d in (4,)] + [((48, 48), d) for d in (10,)]


def f(x):
    return float(x)


def make_surface(ref) -> None:
    """Surface bytes of the committed frames (inputs = frames.npz) and of edge values."""
    frames = np.load(os.path.join(HERE, "frames.npz"))
    out = {k: ref.surface_u8(frames[k]) for k in frames.files}
    edge = np.array([[0.0, 0.5, 1.0], [1.0001, 1.084, 1.3423], [2.0, 1.0 + 1 / 255, -0.001],
                     [-1.5, np.nan, 1e12], [0.999999, 255.0 / 255, 3.99]], np.float64)
    out["edge__in"] = edge
    out["edge__u8"] = ref.surface_u8(edge)
    np.savez_compressed(os.path.join(HERE, "surface.npz"), **out)


def main() -> None:
    orc_mod.build(ref=True)
    ref = orc_mod.Reference()
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "surface":
        make_surface(ref)
        return
    L = ref.lib
    A = orc_mod._arr
    kat: dict = {"source": "reference vec.cpp/scene.cpp/main.cpp:1-139 compiled by oracle/Makefile"}

    # ---- Sphere::intersect (scene.cpp:40-78) -------------------------------
    import ctypes as C
    sph_cases = [
        ("front", (3, 0, 0), 1.0, (0, 0, 0), (1, 0, 0)),
        ("unnormalised_dir_world_distance", (3, 0, 0), 1.0, (0, 0, 0), (2, 0, 0)),
        ("origin_inside", (3, 0, 0), 1.0, (3, 0, 0), (1, 0, 0)),
        ("behind", (3, 0, 0), 1.0, (0, 0, 0), (-1, 0, 0)),
        ("tangent_det0", (3, 0, 0), 1.0, (0, 1, 0), (1, 0, 0)),
        ("miss", (3, 0, 0), 1.0, (0, 2, 0), (1, 0, 0)),
        ("oblique", (2.5, -0.3, 0.7), 0.6, (0.1, 0.2, -0.1), (1.0, -0.2, 0.3)),
    ]
    out = []
    for name, c, r, o, d in sph_cases:
        dist, n, hit = C.c_double(), (C.c_double * 3)(), C.c_int()
        L.ref_sphere_intersect(A(c), r, A(o), A(d), C.byref(dist), n, C.byref(hit))
        out.append(dict(name=name, center=c, radius=r, o=o, d=d, dist=f(dist.value),
                        normal=[f(v) for v in n], hit=hit.value))
    kat["sphere_intersect"] = out

    # ---- Wall::intersect (scene.cpp:4-35) -----------------------------------
    wall_cases = [
        ("front", (3, -1, -1), (-1, 0, 0), 2, 2, (0, 0, 0), (1, 0, 0)),
        ("parametric_t", (3, -1, -1), (-1, 0, 0), 2, 2, (0, 0, 0), (2, 0, 0)),
        ("back_side_not_flipped", (3, -1, -1), (-1, 0, 0), 2, 2, (5, 0, 0), (-1, 0, 0)),
        ("parallel", (3, -1, -1), (-1, 0, 0), 2, 2, (0, 0, 0), (0, 1, 0)),
        ("z_normal_never_hits", (-1, -1, 3), (0, 0, 1), 2, 2, (0, 0, 0), (0, 0, 1)),
        ("outside_bounds", (3, -1, -1), (-1, 0, 0), 2, 2, (0, 0, 0), (1, 2, 0)),
        ("unnormalised_normal", (3, 2, 0), (0, -3, 0), 1, 1, (0, 0, 0), (1, 1.2, -0.4)),
        ("diagonal", (8, 3, -1), (-.70710678, -.70710678, 0), 8, 4, (0, 0, 0), (1, 0.4, 0.1)),
    ]
    out = []
    for name, p, n_raw, ln, wd, o, d in wall_cases:
        dist, n, hit = C.c_double(), (C.c_double * 3)(), C.c_int()
        L.ref_wall_intersect(A(p), A(n_raw), ln, wd, A(o), A(d), C.byref(dist), n, C.byref(hit))
        out.append(dict(name=name, position=p, raw_normal=n_raw, length=ln, width=wd, o=o, d=d,
                        dist=f(dist.value), normal=[f(v) for v in n], hit=hit.value))
    kat["wall_intersect"] = out

    # ---- shading helpers (main.cpp:28-62), reflect/normalize (vec.cpp) ------
    oc_in = [(1, 0, 0.5), (0, 0, -1), (0.3, -0.2, 0.0), (-1.0, 2.0, 3.0), (1e-3, 0, 1e-9),
             (0.5, 0.5, 0.70710678)]
    out = []
    for v in oc_in:
        rgb = (C.c_double * 3)()
        L.ref_out_color(A(v), rgb)
        out.append(dict(v=v, rgb=[f(x) for x in rgb]))
    kat["out_color"] = out
    out = []
    for pos, n, lp in [((2, 0, 0), (-1, 0, 0), (0, 0, 0)), ((1.2, 0.3, -0.4), (-0.3, 0.4, 0.1), (0, 0, 0)),
                       ((3, 2, 1), (0, -1, 0), (0, 0, 0)), ((1, 1, 1), (1, 1, 1), (0, 0, 0))]:
        out.append(dict(pos=pos, normal=n, light=lp, value=f(L.ref_diffuse_shading(A(pos), A(n), A(lp)))))
    kat["diffuse_shading"] = out
    out = []
    for pos, n, lp, view in [((2, 1, 0), (-1, 0, 0), (0, 0, 0), (-2, -1, 0)),
                             ((1.2, 0.3, -0.4), (-0.3, 0.4, 0.1), (0, 0, 0), (-1, -0.2, 0.1)),
                             ((3, 2, 1), (0, -1, 0), (0, 0, 0), (1, 1, 1))]:
        out.append(dict(pos=pos, normal=n, light=lp, view=view,
                        value=f(L.ref_specular(A(pos), A(n), A(lp), A(view)))))
    kat["specular"] = out
    out = []
    for v, n in [((1, -1, 0), (0, 2, 0)), ((0.3, 0.2, -0.9), (-0.1, 0.5, 0.2)), ((1, 0, 0), (-1, 0, 0))]:
        r = (C.c_double * 3)()
        L.ref_reflect(A(v), A(n), r)
        out.append(dict(v=v, n=n, out=[f(x) for x in r]))
    kat["reflect"] = out

    # ---- Camera::init (scene.cpp:80-106) ------------------------------------
    out = []
    cams = [("c1_640x480", scenes.camera_args(640, 480)),
            ("app_640x640_aspect_int_div", dict(position=(0, 0, 0), lookat=(-1, 0, 0), vup=(0, 0, -1),
                                                vfov=90.0, aspect_ratio=1.0, image_width=640.0)),
            ("c2_1920x1080", scenes.camera_args(1920, 1080)),
            ("c3_3840x2160", scenes.camera_args(3840, 2160)),
            ("c5_7680x4320", scenes.camera_args(7680, 4320)),
            ("moved", dict(position=(0.3, -0.2, 0.1), lookat=(-1, 0.5, 0.2), vup=(0, 0, -1), vfov=70.0,
                           aspect_ratio=16 / 9, image_width=320.0))]
    for name, ca in cams:
        h, v = ref.camera_init(**ca)
        out.append(dict(name=name, args={k: (list(x) if isinstance(x, tuple) else x) for k, x in ca.items()},
                        height=h, position=v[0].tolist(), image_top_left=v[1].tolist(),
                        pixel_delta_x=v[2].tolist(), pixel_delta_y=v[3].tolist()))
    kat["camera_init"] = out

    # ---- reference framebuffer allocation quirk (main.cpp:243) --------------
    sc = scenes.default_scene()
    prims = scenes.to_prims(sc)
    raw = scenes.raw_normals(sc)
    res = {}
    for (w, h) in [(64, 48), (48, 48)]:
        ca = scenes.camera_args(w, h)
        res[f"{w}x{h}"] = int(L.ref_rt_scene_wh_alloc(
            orc_mod.Oracle.prim_array(prims), A(raw, len(raw)), len(prims), A(ca["position"]),
            A(ca["lookat"]), A(ca["vup"]), ca["vfov"], ca["aspect_ratio"], ca["image_width"]))
    kat["rt_scene_WxH_alloc_throws"] = res

    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)

    # ---- frames --------------------------------------------------------------
    frames = {}
    jobs = [(s, d) for s in FRAME_SIZES for d in FRAME_DEPTHS]
    for scene_name, mk in FRAME_SCENES.items():
        sc = mk()
        prims, raw = scenes.to_prims(sc), scenes.raw_normals(sc)
        for (w, h), depth in jobs + EXTRA_FRAMES:
            ca = scenes.camera_args(w, h)
            img = ref.render(prims, raw, ca, depth)
            frames[f"{scene_name}__{w}x{h}__d{depth}"] = img
    np.savez_compressed(os.path.join(HERE, "frames.npz"), **frames)

    # ---- single rays: random origins / directions through every branch ------
    rng = np.random.default_rng(20261015)
    rays = {}
    for scene_name in ("default", "s8w4", "s64w6"):
        sc = FRAME_SCENES[scene_name]()
        prims, raw = scenes.to_prims(sc), scenes.raw_normals(sc)
        n = 400
        o = rng.uniform([-2, -5, -2], [9, 5, 3], size=(n, 3))
        d = rng.normal(size=(n, 3)) * rng.choice([0.3, 1.0, 2.0], size=(n, 1))
        depth = rng.integers(0, 9, size=n)
        rgb = np.empty((n, 3))
        arr = orc_mod.Oracle.prim_array(prims)
        rawa = A(raw, len(raw))
        for k in range(n):
            out3 = (C.c_double * 3)()
            L.ref_trace(arr, rawa, len(prims), A(o[k]), A(d[k]), int(depth[k]), out3)
            rgb[k] = list(out3)
        rays[f"{scene_name}__o"] = o
        rays[f"{scene_name}__d"] = d
        rays[f"{scene_name}__depth"] = depth
        rays[f"{scene_name}__rgb"] = rgb
    np.savez_compressed(os.path.join(HERE, "rays.npz"), **rays)
    make_surface(ref)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
