"""Pin the oracle (oracle/rt_oracle.c) against the reference's own outputs.

The fixtures under tests/golden/ were produced by the reference's compiled vec.cpp,
scene.cpp and main.cpp hot-path functions (tests/golden/make_golden.py).  The oracle is
a quirk-faithful fp64 restatement, so every comparison here is BIT-EXACT.
"""
import math

import numpy as np
import pytest

from conftest import parse_frame_key, scene_by_name
from rtamd import capi, scenes


def _prim_sphere(center, radius):
    return scenes.to_prims([scenes.Sphere(scenes.Material((1, 1, 1)), center, radius)])[0]


def _prim_wall(position, raw_normal, length, width):
    return scenes.to_prims([scenes.Wall(scenes.Material((1, 1, 1)), position, raw_normal,
                                        length, width)])[0]


def _same(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b)


def test_sphere_intersect_kat(oracle, kat):
    for c in kat["sphere_intersect"]:
        dist, n, hit = oracle.sphere_intersect(_prim_sphere(c["center"], c["radius"]), c["o"], c["d"])
        assert dist == c["dist"], c["name"]
        assert _same(n, c["normal"]), c["name"]
        assert hit == c["hit"], c["name"]


def test_sphere_quirks_pinned(kat):
    by = {c["name"]: c for c in kat["sphere_intersect"]}
    # world distance for |d| != 1, det == 0 uses /a (6 instead of 3)
    assert by["unnormalised_dir_world_distance"]["dist"] == 2.0
    assert by["tangent_det0"]["dist"] == 6.0
    assert by["origin_inside"]["hit"] == 1 and by["origin_inside"]["dist"] == -1.0
    assert by["behind"]["dist"] == -4.0


def test_wall_intersect_kat(oracle, kat):
    for c in kat["wall_intersect"]:
        w = _prim_wall(c["position"], c["raw_normal"], c["length"], c["width"])
        dist, n, hit = oracle.wall_intersect(w, c["o"], c["d"])
        assert dist == c["dist"], c["name"]
        assert _same(n, c["normal"]), c["name"]
        assert hit == c["hit"], c["name"]
    by = {c["name"]: c for c in kat["wall_intersect"]}
    assert by["parametric_t"]["dist"] == 1.5            # parametric, not world
    assert by["z_normal_never_hits"]["hit"] == 0         # NaN basis
    assert by["back_side_not_flipped"]["normal"] == [-1.0, 0.0, 0.0]


def test_shading_kats(oracle, kat):
    for c in kat["out_color"]:
        got = oracle.out_color(c["v"])
        exp = c["rgb"]
        assert all((math.isnan(g) and math.isnan(e)) or g == e for g, e in zip(got, exp)), c
    for c in kat["diffuse_shading"]:
        assert oracle.diffuse_shading(c["pos"], c["normal"], c["light"]) == c["value"]
    for c in kat["specular"]:
        assert oracle.specular(c["pos"], c["normal"], c["light"], c["view"]) == c["value"]
    for c in kat["reflect"]:
        assert _same(oracle.reflect(c["v"], c["n"]), c["out"])
    # SURVEY §4 probe values
    assert kat["specular"][0]["value"] == 0.89442719099991597
    assert kat["diffuse_shading"][0]["value"] == 1.0


def test_camera_init_kat(oracle, kat):
    for c in kat["camera_init"]:
        a = c["args"]
        cam = oracle.camera_init(a["position"], a["lookat"], a["vup"], a["vfov"],
                                 a["aspect_ratio"], a["image_width"])
        assert cam.height == c["height"], c["name"]
        assert _same(list(cam.image_top_left), c["image_top_left"]), c["name"]
        assert _same(list(cam.pixel_delta_x), c["pixel_delta_x"]), c["name"]
        assert _same(list(cam.pixel_delta_y), c["pixel_delta_y"]), c["name"]
    app = [c for c in kat["camera_init"] if c["name"].startswith("app_640")][0]
    # ASPECT_RATIO = 4/3 == 1 -> the app renders 640x640
    assert app["height"] == 640
    assert abs(app["pixel_delta_x"][1] + 0.00312251) < 1e-8


def test_reference_framebuffer_alloc_quirk(kat):
    # main.cpp:243 allocates [W][H] but rt_scene indexes [row][col]: non-square throws
    assert kat["rt_scene_WxH_alloc_throws"] == {"64x48": 1, "48x48": 0}


def test_frames_bit_exact(oracle, golden_frames):
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        sc = scene_by_name(name)
        cam = oracle.camera_init(**scenes.camera_args(w, h))
        o64, _, _ = oracle.render(scenes.to_prims(sc), cam, depth, nthreads=4)
        assert _same(o64, golden_frames[key]), key


def test_rays_bit_exact(oracle, golden_rays):
    for name in ("default", "s8w4", "s64w6"):
        prims = scenes.to_prims(scene_by_name(name))
        o, d = golden_rays[f"{name}__o"], golden_rays[f"{name}__d"]
        depth, rgb = golden_rays[f"{name}__depth"], golden_rays[f"{name}__rgb"]
        for k in range(len(o)):
            got, _ = oracle.trace(prims, o[k], d[k], int(depth[k]))
            assert _same(got, rgb[k]), (name, k)


def test_oracle_thread_invariance(oracle):
    sc = scenes.synthetic_scene(8, 4)
    cam = oracle.camera_init(**scenes.camera_args(96, 54))
    a, _, s1 = oracle.render(scenes.to_prims(sc), cam, 4, nthreads=1)
    b, _, s2 = oracle.render(scenes.to_prims(sc), cam, 4, nthreads=8)
    assert _same(a, b) and s1 == s2


def test_oracle_row_bands_compose(oracle):
    sc = scenes.synthetic_scene(8, 4)
    cam = oracle.camera_init(**scenes.camera_args(64, 36))
    full, _, sfull = oracle.render(scenes.to_prims(sc), cam, 4)
    parts, stot = [], 0
    for r0 in range(0, 36, 10):
        p, _, s = oracle.render(scenes.to_prims(sc), cam, 4, row0=r0, nrows=min(10, 36 - r0))
        parts.append(p)
        stot += s
    assert _same(np.concatenate(parts), full) and stot == sfull


def test_segments_per_pixel_calibration(oracle):
    # c1 scene at 640x480 depth 2 -> 1.141 segments/pixel
    cam = oracle.camera_init(**scenes.camera_args(640, 480))
    _, _, segs = oracle.render(scenes.to_prims(scenes.default_scene()), cam, 2, want64=False)
    assert abs(segs / (640 * 480) - 1.141) < 0.001


def test_sun_extension_changes_only_lit_pixels(oracle):
    sc = scenes.synthetic_scene(8, 4)
    cam = oracle.camera_init(**scenes.camera_args(64, 36))
    a, _, _ = oracle.render(scenes.to_prims(sc), cam, 2)
    b, _, _ = oracle.render(scenes.to_prims(sc), cam, 2, flags=capi.RT_FLAG_SUN)
    assert (b >= a - 1e-15).all() and (b > a).any()


@pytest.mark.skipif(not __import__("oracle").Reference.available(),
                    reason="reference build only exists where /root/reference does")
def test_against_live_reference_random_scenes(oracle):
    import oracle as orc_mod
    ref = orc_mod.Reference()
    for seed in (1, 7, 99):
        sc = scenes.synthetic_scene(12, 6, seed)
        prims, raw = scenes.to_prims(sc), scenes.raw_normals(sc)
        ca = scenes.camera_args(40, 30)
        cam = oracle.camera_init(**ca)
        for depth in (0, 3, 7):
            o64, _, _ = oracle.render(prims, cam, depth)
            assert _same(o64, ref.render(prims, raw, ca, depth)), (seed, depth)


def test_surface_bytes_match_reference_conversion(oracle, golden_frames, golden_surface):
    """main.cpp:345's implicit double->Uint8 (the reference's x86-64 build: truncation,
    highlights above 1.0 wrap mod 256, NaN -> 0) restated in the oracle equals the bytes
    recorded from that conversion compiled by g++ (tests/golden/surface.npz)."""
    for key in golden_frames.files:
        assert np.array_equal(oracle.surface_u8(golden_frames[key]), golden_surface[key]), key
    assert np.array_equal(oracle.surface_u8(golden_surface["edge__in"]), golden_surface["edge__u8"])
    # the fixtures hold out-of-range pixels, so the wrap is pinned, not just truncation
    over = sum(int((golden_frames[k] > 1.0).sum()) for k in golden_frames.files)
    assert over > 100
    assert golden_surface["edge__u8"][1].tolist() == [255, 20, 86]


@pytest.mark.skipif(not __import__("oracle").Reference.available(),
                    reason="reference build only exists where /root/reference does")
def test_surface_bytes_live_reference(oracle):
    import oracle as orc_mod
    ref = orc_mod.Reference()
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.uniform(-3, 3, (4000, 3)), rng.uniform(0, 1.5, (4000, 3))])
    assert np.array_equal(oracle.surface_u8(v), ref.surface_u8(v))
