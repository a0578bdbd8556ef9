"""GPU parity: the HIP path (through the C-ABI) against the reference's golden frames and
the oracle, on an MI355X.  Run with `pytest -m gpu`.

Tolerances (north_star: per-pixel RGB delta <= 1e-4 vs the CPU reference):
  F64    |delta| <= 1e-12 per channel on every pixel of the golden frames (the only
         difference from the reference is libm's last bit in pow: OCML vs glibc);
         at full config sizes the same bound on >= 99.999% of pixels, every other pixel
         on a geometric discontinuity (a 3x3 neighbourhood with differing hit paths).
  MIXED  bit-identical to F64 (the fp32 cull only skips primitives the exact test rejects).
  F32    the throughput variant, not a parity path: |delta| <= 1e-4 on >= 99.5% of pixels
         at depth <= 4 with every outlier on a discontinuity; deeper sphere-to-sphere bounce
         chains amplify fp32 direction error (each bounce off a sphere of radius r scales it
         by ~2|d|/r), so at depth >= 6 the bound is >= 99% of pixels, reported, not gated on
         discontinuities.
"""
import os

import numpy as np
import pytest

from conftest import has_gpu, parse_frame_key, scene_by_name
from rtamd import capi, scenes

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

NTHREADS = min(16, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def rend():
    r = capi.Renderer(0)
    yield r
    r.close()


def render(rend, sc, w, h, depth, prec, flags=0, fmt=capi.RT_OUT_RGB_F64, **kw):
    rend.set_scene(scenes.to_prims(sc))
    cam = capi.camera_init(**scenes.camera_args(w, h))
    img, st = rend.render(cam, depth, prec, flags, fmt, **kw)
    return img, st, cam


def discontinuity_mask(sig):
    """True where any pixel of the 3x3 neighbourhood has a different hit-path signature."""
    h, w = sig.shape
    pad = np.pad(sig, 1, mode="edge")
    m = np.zeros((h, w), bool)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            m |= pad[1 + dy:1 + dy + h, 1 + dx:1 + dx + w] != sig
    return m


def check_f64(img, ref64, sig=None, tol=1e-12, min_frac=1.0, what=""):
    d = np.abs(img - ref64).max(axis=-1)
    bad = d > tol
    frac_ok = 1.0 - bad.mean()
    assert frac_ok >= min_frac, (what, frac_ok, d.max())
    if bad.any():
        assert sig is not None, (what, int(bad.sum()), d.max())
        assert discontinuity_mask(sig)[bad].all(), (what, "outlier off a discontinuity")


# ---------------------------------------------------------------- golden frames
def test_f64_matches_reference_golden_frames(rend, golden_frames):
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        img, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_F64)
        check_f64(img, golden_frames[key], what=key)


def test_mixed_bitwise_equals_f64_on_golden(rend, golden_frames):
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        a, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_F64)
        b, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_MIXED)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), key


def check_f32(img, ref64, sig, depth, what):
    if depth <= 4:
        check_f64(img.astype(np.float64), ref64, sig, tol=1e-4, min_frac=0.995, what=what)
    else:
        frac = (np.abs(img.astype(np.float64) - ref64).max(axis=-1) <= 1e-4).mean()
        assert frac >= 0.99, (what, frac)


def test_f32_within_tolerance_on_golden(rend, golden_frames, oracle):
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        sc = scene_by_name(name)
        img, _, cam = render(rend, sc, w, h, depth, capi.RT_PREC_F32, fmt=capi.RT_OUT_RGB_F32)
        _, _, _, sig = oracle.render(scenes.to_prims(sc), cam, depth, want_sig=True)
        check_f32(img, golden_frames[key], sig, depth, key)


# ---------------------------------------------------------------- output formats
def test_f32_output_is_rounded_f64(rend, oracle):
    sc = scenes.synthetic_scene(8, 4)
    img32, _, cam = render(rend, sc, 96, 54, 4, capi.RT_PREC_F64, fmt=capi.RT_OUT_RGB_F32)
    o64, o32, _ = oracle.render(scenes.to_prims(sc), cam, 4)
    # identical except where a 1e-16 libm difference crosses an fp32 rounding boundary
    ulp = np.abs(img32.view(np.int32).astype(np.int64) - o32.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1 and (ulp == 0).mean() > 0.999


def test_rgba8_epilogue(rend, oracle):
    sc = scenes.synthetic_scene(8, 4)
    img, _, cam = render(rend, sc, 96, 54, 4, capi.RT_PREC_F64, fmt=capi.RT_OUT_RGBA8)
    o64, _, _ = oracle.render(scenes.to_prims(sc), cam, 4)
    exp = np.floor(np.clip(o64, 0.0, 1.0) * 255.0).astype(np.uint8)   # main.cpp:345 truncation
    assert (img[..., 3] == 255).all()
    edge = np.abs(np.clip(o64, 0, 1) * 255.0 - np.round(np.clip(o64, 0, 1) * 255.0)) < 1e-9
    ok = (img[..., :3] == exp) | edge
    assert ok.all()


def test_rgba8_wrap_matches_reference_surface_bytes(rend, golden_frames, golden_surface):
    """RT_OUT_RGBA8_WRAP = main.cpp:345's bytes as the reference's x86-64 build makes them
    (tests/golden/surface.npz, recorded from the compiled conversion): highlights above 1.0
    wrap mod 256.  F64 renders agree with the reference to <= 1e-12, so a byte may differ
    only where v*255 sits on an integer boundary."""
    wrapped = 0
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        img, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_F64,
                           fmt=capi.RT_OUT_RGBA8_WRAP)
        ref64, exp = golden_frames[key], golden_surface[key]
        assert (img[..., 3] == 255).all(), key
        t = ref64 * 255.0
        edge = np.abs(t - np.round(t)) < 1e-9
        assert ((img[..., :3] == exp) | edge).all(), key
        wrapped += int(((ref64 > 1.0) & ~edge).sum())
        # RT_OUT_RGBA8 is the same bytes where the reference is in range, 255 above it
        sat, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_F64,
                           fmt=capi.RT_OUT_RGBA8)
        inr = (ref64 >= 0) & (ref64 <= 1.0) & ~edge
        assert (sat[..., :3][inr] == exp[inr]).all(), key
        assert (sat[..., :3][(ref64 > 1.0) & ~edge] == 255).all(), key
    assert wrapped > 100   # the out-of-range behaviour is exercised, not just truncation


def test_set_scene_waits_for_renders_on_caller_streams(rend):
    """rt_set_scene must not overwrite the device scene under frames still in flight on a
    non-blocking caller stream: queue heavy frames of scene A on a torch
    stream, swap to scene B at once, and every queued frame is still scene A's."""
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(dev)
    sa, sb = scenes.synthetic_scene(64, 6), scenes.synthetic_scene(64, 6, seed=99)
    rend.set_scene(scenes.to_prims(sa))
    cam = capi.camera_init(**scenes.camera_args(1920, 1080))
    ref, _ = rend.render(cam, 6, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32)
    outs = [torch.full((1080, 1920, 3), -1.0, device=dev) for _ in range(4)]
    torch.cuda.synchronize()
    for o in outs:
        rend.render_device(cam, 6, o.data_ptr(), capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32,
                           stream=st.cuda_stream)
    rend.set_scene(scenes.to_prims(sb))   # frames above may still be running
    torch.cuda.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    other, _ = rend.render(cam, 6, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32)
    assert not np.array_equal(other, ref)


def test_calls_keep_the_callers_current_device_and_contexts_are_independent(rend):
    """Entry points run on the ctx's device and restore the caller's current device; two
    contexts interleaved on different streams render their own scenes."""
    import torch
    dev = torch.device("cuda", 0)
    before = torch.cuda.current_device()
    sa, sb = scenes.synthetic_scene(8, 4), scenes.default_scene()
    cam = capi.camera_init(**scenes.camera_args(160, 90))
    with capi.Renderer(0) as r2:
        rend.set_scene(scenes.to_prims(sa))
        r2.set_scene(scenes.to_prims(sb))
        ra, _ = rend.render(cam, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
        rb, _ = r2.render(cam, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        oa = [torch.empty((90, 160, 3), device=dev) for _ in range(3)]
        ob = [torch.empty((90, 160, 3), device=dev) for _ in range(3)]
        torch.cuda.synchronize()
        for a, b in zip(oa, ob):
            rend.render_device(cam, 4, a.data_ptr(), capi.RT_PREC_PATH64, stream=s1.cuda_stream)
            r2.render_device(cam, 4, b.data_ptr(), capi.RT_PREC_PATH64, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        for a, b in zip(oa, ob):
            assert np.array_equal(a.cpu().numpy(), ra) and np.array_equal(b.cpu().numpy(), rb)
    assert torch.cuda.current_device() == before


# ---------------------------------------------------------------- semantics
def test_segment_count_matches_oracle(rend, oracle):
    for sc, depth in ((scenes.default_scene(), 10), (scenes.synthetic_scene(8, 4), 4),
                      (scenes.synthetic_scene(64, 6), 6)):
        for prec in (capi.RT_PREC_F64, capi.RT_PREC_MIXED):
            _, st, cam = render(rend, sc, 96, 54, depth, prec, count_segments=True)
            _, _, segs = oracle.render(scenes.to_prims(sc), cam, depth)
            assert st.segments == segs


def test_row_bands_compose_bitwise(rend):
    sc = scenes.synthetic_scene(8, 4)
    full, _, cam = render(rend, sc, 100, 75, 4, capi.RT_PREC_F64)
    parts = []
    for r0, nr in ((0, 13), (13, 40), (53, 22)):
        img, _ = rend.render(cam, 4, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F64, row0=r0, nrows=nr)
        parts.append(img)
    assert np.array_equal(np.concatenate(parts).view(np.uint64), full.view(np.uint64))


def test_sun_extension_matches_oracle(rend, oracle):
    sc = scenes.synthetic_scene(8, 4)
    for prec in (capi.RT_PREC_F64, capi.RT_PREC_MIXED):
        img, _, cam = render(rend, sc, 96, 54, 4, prec, flags=capi.RT_FLAG_SUN)
        o64, _, _ = oracle.render(scenes.to_prims(sc), cam, 4, flags=capi.RT_FLAG_SUN)
        check_f64(img, o64, what="sun")


def test_deterministic(rend):
    sc = scenes.synthetic_scene(64, 6)
    a, _, _ = render(rend, sc, 160, 90, 6, capi.RT_PREC_MIXED)
    b, _, _ = render(rend, sc, 160, 90, 6, capi.RT_PREC_MIXED)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))


# ---------------------------------------------------------------- edge cases
def test_empty_scene_is_sky(rend, oracle):
    img, _, cam = render(rend, [], 37, 23, 3, capi.RT_PREC_F64)
    o64, _, _ = oracle.render([], cam, 3)
    check_f64(img, o64, what="empty")


def test_ragged_sizes_and_depths(rend, oracle):
    sc = scenes.synthetic_scene(5, 3, seed=11)
    for (w, h) in ((1, 1), (17, 9), (33, 65)):
        for depth in (0, 1, 5, 9, 16):
            for prec in (capi.RT_PREC_F64, capi.RT_PREC_MIXED):
                img, _, cam = render(rend, sc, w, h, depth, prec)
                o64, _, _, sig = oracle.render(scenes.to_prims(sc), cam, depth, want_sig=True)
                check_f64(img, o64, sig, what=(w, h, depth, prec))


def test_dead_wall_and_degenerate_prims(rend, oracle):
    # a z-normal wall (NaN basis, never hit: scene.cpp:18) and a zero-radius sphere
    sc = scenes.synthetic_scene(6, 2, seed=5) + [
        scenes.Wall(scenes.Material((1, 0, 0)), (-2, -2, 4), (0, 0, 1), 8, 8),
        scenes.Sphere(scenes.Material((1, 1, 0)), (3, 0, 0), 0.0),
    ]
    img, _, cam = render(rend, sc, 64, 36, 4, capi.RT_PREC_F64)
    o64, _, _, sig = oracle.render(scenes.to_prims(sc), cam, 4, want_sig=True)
    check_f64(img, o64, sig, what="degenerate")


def test_errors(rend):
    lib = rend.lib
    cam = capi.camera_init(**scenes.camera_args(64, 36))
    fresh = capi.Renderer(0)
    with pytest.raises(capi.RTError) as e:
        fresh.render(cam, 2)
    assert e.value.status == capi.RT_ERR_NO_SCENE
    fresh.close()
    rend.set_scene(scenes.to_prims(scenes.default_scene()))
    with pytest.raises(capi.RTError) as e:
        rend.render(cam, lib.rt_max_depth() + 1)
    assert e.value.status == capi.RT_ERR_UNSUPPORTED
    with pytest.raises(capi.RTError) as e:
        rend.render(cam, 2, row0=30, nrows=10)
    assert e.value.status == capi.RT_ERR_OUT_OF_RANGE


def test_moved_camera_stale_top_left(rend, oracle):
    """Camera moves without init() (main.cpp:265 -> scene.cpp:121): only position shifts."""
    sc = scenes.synthetic_scene(8, 4)
    cam = capi.camera_init(**scenes.camera_args(64, 36))
    for k in range(3):
        cam.position[0] += 0.1   # Camera::forward with direction (1,0,0), speed .1
    rend.set_scene(scenes.to_prims(sc))
    img, _ = rend.render(cam, 4, capi.RT_PREC_MIXED, 0, capi.RT_OUT_RGB_F64)
    o64, _, _, sig = oracle.render(scenes.to_prims(sc), cam, 4, want_sig=True)
    check_f64(img, o64, sig, what="moved")


# ---------------------------------------------------------------- mixed-cull stress
def test_mixed_cull_conservative_random_views(rend):
    rng = np.random.default_rng(7)
    for trial in range(6):
        sc = scenes.synthetic_scene(int(rng.integers(4, 40)), int(rng.integers(0, 7)),
                                    seed=int(rng.integers(1 << 30)))
        rend.set_scene(scenes.to_prims(sc))
        pos = rng.uniform([-1, -3, -1], [6, 3, 2])
        look = pos + rng.normal(size=3)
        cam = capi.camera_init(pos, look, (0, 0, -1), float(rng.uniform(30, 120)), 16 / 9, 256.0)
        depth = int(rng.integers(1, 9))
        a, _ = rend.render(cam, depth, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F64)
        b, _ = rend.render(cam, depth, capi.RT_PREC_MIXED, 0, capi.RT_OUT_RGB_F64)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), trial


# ---------------------------------------------------------------- full config sizes
@pytest.mark.parametrize("cfg_name", ["c1", "c2", "c3"])
def test_full_size_configs_vs_oracle(rend, oracle, cfg_name):
    cfg = scenes.CONFIGS[cfg_name]
    sc = cfg.scene()
    img, st, cam = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_MIXED,
                          count_segments=True)
    o64, _, segs, sig = oracle.render(scenes.to_prims(sc), cam, cfg.depth, nthreads=NTHREADS,
                                      want_sig=True)
    assert st.segments == segs
    check_f64(img, o64, sig, min_frac=0.99999, what=cfg_name)
    f32, _, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_F32,
                       fmt=capi.RT_OUT_RGB_F32)
    check_f32(f32, o64, sig, cfg.depth, cfg_name + "/f32")
    if cfg_name in ("c2", "c3"):
        # the bench precision (PATH64, fp32 RGB: the frame bench.py times) against the oracle
        # at the full headline sizes: the same segment count, EVERY pixel within the
        # north_star's 1e-4 (main.cpp:89-119); how many exceed PATH64_TOL is reported
        p64, sp, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_PATH64,
                            fmt=capi.RT_OUT_RGB_F32, count_segments=True)
        assert sp.segments == segs, (cfg_name, sp.segments, segs)
        d = np.abs(p64.astype(np.float64) - o64).max(axis=-1)
        rep = {"config": cfg_name, "pixels": int(d.size), "max_abs_delta": float(d.max()),
               "above_2e-5": int((d > PATH64_TOL).sum()), "above_1e-4": int((d > 1e-4).sum()),
               "above_2e-5_on_discontinuity": int(discontinuity_mask(sig)[d > PATH64_TOL].sum()),
               "segments": int(segs)}
        print("path64_vs_oracle", rep)
        out = os.environ.get("RT_PARITY_REPORT")
        if out:
            import json
            with open(out, "a") as fh:
                fh.write(json.dumps(rep) + "\n")
        assert d.max() <= 1e-4, rep


def test_c5_sampled_rows_vs_oracle(rend, oracle):
    cfg = scenes.CONFIGS["c5"]
    sc = cfg.scene()
    rend.set_scene(scenes.to_prims(sc))
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    for r0 in (0, 1500, 2200, 4300):
        img, st = rend.render(cam, cfg.depth, capi.RT_PREC_MIXED, 0, capi.RT_OUT_RGB_F64,
                              row0=r0, nrows=8, count_segments=True)
        o64, _, segs, sig = oracle.render(scenes.to_prims(sc), cam, cfg.depth, row0=r0, nrows=8,
                                          nthreads=NTHREADS, want_sig=True)
        assert st.segments == segs
        check_f64(img, o64, sig, min_frac=0.9999, what=("c5", r0))


def test_full_size_c5_properties(rend):
    """Size-independent properties at BASELINE's largest config: the full 8K frame equals
    its row bands rendered separately, MIXED equals F64 on a band, values are finite."""
    cfg = scenes.CONFIGS["c5"]
    rend.set_scene(scenes.to_prims(cfg.scene()))
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    full, st = rend.render(cam, cfg.depth, capi.RT_PREC_MIXED, 0, capi.RT_OUT_RGB_F32,
                           count_segments=True)
    assert np.isfinite(full).all()
    tot = 0
    for r in range(4):
        r0, nr = capi.band_rows(cfg.height, 4, r)
        b, stb = rend.render(cam, cfg.depth, capi.RT_PREC_MIXED, 0, capi.RT_OUT_RGB_F32,
                             row0=r0, nrows=nr, count_segments=True)
        assert np.array_equal(b.view(np.uint32), full[r0:r0 + nr].view(np.uint32))
        tot += stb.segments
    assert tot == st.segments
    a, _ = rend.render(cam, cfg.depth, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32, row0=2000,
                       nrows=64)
    assert np.array_equal(a.view(np.uint32), full[2000:2064].view(np.uint32))


# ---------------------------------------------------------------- exact helpers
def test_selftest_shared_reciprocal_division_is_ieee(rend):
    """rt_trace.hip shares one refined reciprocal across the numerators of a
    normalisation; it must give IEEE `/`'s bits (division over 2^-40..2^40, both signs,
    and the component/|v| pattern)."""
    assert rend.selftest(0, 1 << 24, seed=12345) == 0


def test_selftest_integer_pow(rend):
    assert rend.selftest(1, 1 << 22, seed=777) == 0


def test_selftest_sqrt_sequence_is_ieee(rend):
    assert rend.selftest(2, 1 << 24, seed=4242) == 0


# ---------------------------------------------------------------- PATH64
PATH64_TOL = 2e-5   # fp32 colour arithmetic on the exact fp64 path (north_star bound: 1e-4)


def test_path64_every_pixel_within_tolerance(rend, golden_frames):
    """Exact fp64 ray paths + fp32 colour: no discontinuity flips, so EVERY pixel of every
    golden frame (depth up to 10, 256 spheres) is within PATH64_TOL of the reference."""
    for key in golden_frames.files:
        name, w, h, depth = parse_frame_key(key)
        img, _, _ = render(rend, scene_by_name(name), w, h, depth, capi.RT_PREC_PATH64)
        d = np.abs(img - golden_frames[key]).max()
        assert d <= PATH64_TOL, (key, d)


@pytest.mark.parametrize("cfg_name", ["c2", "c3"])
def test_path64_full_size_vs_f64(rend, cfg_name):
    cfg = scenes.CONFIGS[cfg_name]
    sc = cfg.scene()
    a, sa, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_F64,
                      count_segments=True)
    b, sb, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_PATH64,
                      count_segments=True)
    assert sa.segments == sb.segments
    assert np.abs(a - b).max() <= PATH64_TOL


def test_path64_sun(rend, oracle):
    sc = scenes.synthetic_scene(8, 4)
    img, _, cam = render(rend, sc, 96, 54, 4, capi.RT_PREC_PATH64, flags=capi.RT_FLAG_SUN)
    o64, _, _ = oracle.render(scenes.to_prims(sc), cam, 4, flags=capi.RT_FLAG_SUN)
    assert np.abs(img - o64).max() <= 4 * PATH64_TOL   # sun adds up to 1.64x colour


def test_c2_sun_full_size(rend, oracle):
    """Config 2's literal "+ sun" at full size (1920x1080, 8 spheres + 4 walls, depth 4,
    RT_FLAG_SUN; the sun constants are main.cpp:18-19, unused by the reference, so the bar
    is the oracle's sun): F64 + sun against the oracle on sampled row blocks (top, the
    heavy middle, bottom) to 1e-12 with outliers only on discontinuities; PATH64 + sun
    (the bench precision) against F64 + sun on every pixel, with the same segment count —
    which is also the sun-off count (the sun adds shading terms, never rays)."""
    cfg = scenes.CONFIGS["c2"]
    sc = cfg.scene()
    f64, s64, cam = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_F64,
                           flags=capi.RT_FLAG_SUN, fmt=capi.RT_OUT_RGB_F64, count_segments=True)
    prims = scenes.to_prims(sc)
    for r0 in (0, 536, 1072):
        o64, _, _, sig = oracle.render(prims, cam, cfg.depth, flags=capi.RT_FLAG_SUN, row0=r0,
                                       nrows=8, nthreads=NTHREADS, want_sig=True)
        check_f64(f64[r0:r0 + 8], o64, sig, what=("c2 sun", r0))
    p64, sp, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_PATH64,
                        flags=capi.RT_FLAG_SUN, fmt=capi.RT_OUT_RGB_F32, count_segments=True)
    _, s0, _ = render(rend, sc, cfg.width, cfg.height, cfg.depth, capi.RT_PREC_PATH64,
                      fmt=capi.RT_OUT_RGB_F32, count_segments=True)
    assert sp.segments == s64.segments == s0.segments
    d = np.abs(p64 - f64)
    assert np.isfinite(d).all() and d.max() <= 4 * PATH64_TOL, float(d.max())


def test_non_integer_specular_exponent(rend, oracle):
    """A material with a non-integer exponent selects the general-pow kernel variants: OCML
    pow in fp64 (F64/MIXED: the reference's bar), the fp32 pow (`fpow`, exp2(e*log2 x)) in
    PATH64's colour arithmetic (every pixel within PATH64_TOL, the same ray paths and
    segment count) and in F32 (its discontinuity bar)."""
    sc = scenes.synthetic_scene(6, 3, seed=3)
    sc[0].mat.specular_exponent = 37.5
    sc[2].mat.specular_exponent = 0.0
    sc[4].mat.specular_exponent = 2.25
    for (w, h) in ((64, 36), (192, 108)):
        o64 = None
        for prec in (capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64, capi.RT_PREC_F32):
            fmt = capi.RT_OUT_RGB_F32 if prec == capi.RT_PREC_F32 else capi.RT_OUT_RGB_F64
            img, st, cam = render(rend, sc, w, h, 5, prec, fmt=fmt, count_segments=True)
            if o64 is None:
                o64, _, segs, sig = oracle.render(scenes.to_prims(sc), cam, 5, want_sig=True)
            if prec in (capi.RT_PREC_F64, capi.RT_PREC_MIXED):
                check_f64(img, o64, sig, what=("nonint", prec, w))
                assert st.segments == segs
            elif prec == capi.RT_PREC_PATH64:
                assert st.segments == segs
                assert np.abs(img - o64).max() <= PATH64_TOL, ("nonint path64", w)
            else:
                check_f32(img, o64, sig, 5, ("nonint f32", w))


def test_path64_full_size_c5_vs_oracle_sampled_rows(rend, oracle):
    """The bench precision at BASELINE config 5's full size against the pinned oracle, not
    only against F64: one full 7680x4320 PATH64 frame (depth 8, 256 spheres, the cull +
    sphere-cluster kernels at their defaults), and 32 blocks of 8 rows spread evenly over
    the frame (256 rows, through the sphere cloud) traced by the oracle — every pixel of
    them within PATH64_TOL, and each block's segment count equal to the oracle's."""
    cfg = scenes.CONFIGS["c5"]
    prims = scenes.to_prims(cfg.scene())
    rend.set_scene(prims)
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    full, _ = rend.render(cam, cfg.depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
    starts = [int(round(k * (cfg.height - 8) / 31)) for k in range(32)]
    worst = 0.0
    for r0 in starts:
        o64, _, segs = oracle.render(prims, cam, cfg.depth, row0=r0, nrows=8, nthreads=NTHREADS)
        _, st = rend.render(cam, cfg.depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32,
                            row0=r0, nrows=8, count_segments=True)
        assert st.segments == segs, (r0, st.segments, segs)
        d = float(np.abs(full[r0:r0 + 8] - o64).max())
        worst = max(worst, d)
        assert d <= PATH64_TOL, (r0, d)
    assert worst > 0.0   # fp32 colour: not bit-equal to the fp64 oracle, only within the bar


def test_path64_full_size_c5_vs_f64(rend):
    """BASELINE config 5 (7680x4320, 256 spheres, depth 8) at full size in the bench
    precision with the sphere-cluster path at its default: PATH64's ray paths are F64's
    exactly (equal segment counts; the fp32 colour arithmetic is the only difference) and
    every pixel is within PATH64_TOL of the F64 frame (fp32 output of both)."""
    cfg = scenes.CONFIGS["c5"]
    rend.set_scene(scenes.to_prims(cfg.scene()))
    cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
    a, sa = rend.render(cam, cfg.depth, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32,
                        count_segments=True)
    b, sb = rend.render(cam, cfg.depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32,
                        count_segments=True)
    assert sa.segments == sb.segments
    d = np.abs(a - b)
    assert np.isfinite(d).all() and d.max() <= PATH64_TOL, float(d.max())


# ---------------------------------------------------------------- wave cull
@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64,
                                  capi.RT_PREC_F32])
def test_wave_cull_is_output_invariant(rend, prec):
    """The wave-cooperative cull only skips spheres no live ray of the wave can hit: frames
    with it forced on and forced off are bitwise identical, for every precision."""
    rng = np.random.default_rng(11)
    try:
        # sizes cover the nearest-first traversal (<= 256 spheres) and the chunked one
        for trial, ns in enumerate((20, 97, 256, 300)):
            sc = scenes.synthetic_scene(ns, int(rng.integers(0, 7)),
                                        seed=int(rng.integers(1 << 30)))
            rend.set_scene(scenes.to_prims(sc))
            pos = rng.uniform([-1, -3, -1], [5, 3, 2])
            cam = capi.camera_init(pos, pos + rng.normal(size=3), (0, 0, -1),
                                   float(rng.uniform(40, 110)), 16 / 9, 192.0)
            depth = int(rng.integers(2, 9))
            imgs = []
            for cull in (0, 2**31 - 1):
                rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, cull)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True)
                imgs.append((img, st.segments))
            assert imgs[0][1] == imgs[1][1], trial
            assert np.array_equal(imgs[0][0].view(np.uint64), imgs[1][0].view(np.uint64)), trial
    finally:
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)


@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64,
                                  capi.RT_PREC_F32])
def test_sphere_clusters_are_output_invariant(rend, prec):
    """RT_OPT_CLUSTER_COS: wide-cone waves of the cull kernels test each lane's ray against
    sphere clusters (rt_device.h Clu32) and run the exact test on its own clusters only,
    pruning clusters beyond the lane's best hit.  Forced on for every wave (2000), off
    (-2000) and at the default, frames are bitwise those of the linear scan — with
    duplicated spheres (exact ties across clusters: the lower scene index must win), cameras
    inside the sphere cloud and far outside it (origins past the box margin's range test
    every cluster unpruned), deep bounces.  The fp64 kernels' leaves hold CLU_SIZE_D = 4
    spheres up to 256 spheres (trial 5: 256, 64 full leaves) and fall back to the F32
    kernels' 8 beyond (trial 3: 259)."""
    rng = np.random.default_rng(23)
    try:
        # trial 3: camera far outside the cloud but within the box margin's range (pruned
        # walk); trial 4: beyond 100x the scene extent (clu_oinf), every cluster unpruned
        for trial, ns in enumerate((24, 70, 129, 256, 200, 253)):
            sc = scenes.synthetic_scene(ns, int(rng.integers(0, 7)),
                                        seed=int(rng.integers(1 << 30)))
            sph = [o for o in sc if o.kind == capi.RT_PRIM_SPHERE]
            for k in range(3):  # copies of earlier spheres, another colour, later in order
                o = sph[int(rng.integers(len(sph)))]
                sc.append(scenes.Sphere(scenes.Material(tuple(rng.uniform(0, 1, 3)), .6),
                                        o.position, o.radius))
            rend.set_scene(scenes.to_prims(sc))
            far = trial in (3, 4)
            pos = (np.array([-400.0, 30.0, 10.0]) if trial == 3 else
                   np.array([-5000.0, 40.0, 12.0]) if trial == 4 else
                   rng.uniform([2, -3, -1], [8, 3, 2]))
            look = np.array([5.0, 0.0, 0.5]) if far else pos + rng.normal(size=3)
            vfov = 2.0 if trial == 3 else 0.15 if trial == 4 else 100.0
            cam = capi.camera_init(pos, look, (0, 0, -1), vfov, 16 / 9, 160.0)
            depth = 8
            rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 2**31 - 1)
            ref, rst = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True)
            rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 0)
            for cc in (2000, -2000, 400):
                rend.set_option(capi.RT_OPT_CLUSTER_COS, cc)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True)
                assert st.segments == rst.segments, (trial, cc)
                assert np.array_equal(img.view(np.uint64), ref.view(np.uint64)), (trial, cc)
    finally:
        rend.set_option(capi.RT_OPT_CLUSTER_COS, 400)
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)


# ---------------------------------------------------------------- eye tables
@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64])
def test_eye_tables_are_output_invariant(rend, prec):
    """Primary rays read their camera-origin terms from host-computed tables (rt_device.h
    "eye tables"): for the exact precisions frames with and without them are bitwise
    identical, up to the table limits (32 spheres, 16 walls) and past them (off)."""
    rng = np.random.default_rng(12)
    try:
        for trial, (ns, nw) in enumerate(((1, 0), (5, 3), (8, 4), (23, 7), (32, 16), (33, 2))):
            sc = scenes.synthetic_scene(ns, min(nw, 6), seed=int(rng.integers(1 << 30)))
            for _ in range(nw - 6):  # random extra walls
                nrm = rng.normal(size=3)
                sc.append(scenes.Wall(scenes.Material(tuple(rng.uniform(0, 1, 3)), .5),
                                      tuple(rng.uniform(-6, 6, 3)), tuple(nrm / np.linalg.norm(nrm)),
                                      float(rng.uniform(1, 8)), float(rng.uniform(1, 8))))
            rend.set_scene(scenes.to_prims(sc))
            pos = rng.uniform([-1, -3, -1], [5, 3, 2])
            cam = capi.camera_init(pos, pos + rng.normal(size=3), (0, 0, -1),
                                   float(rng.uniform(40, 110)), 16 / 9, 160.0)
            depth = int(rng.integers(1, 7))
            imgs = []
            for eye in (1, 0):
                rend.set_option(capi.RT_OPT_EYE_TABLES, eye)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True)
                imgs.append((img, st.segments))
            assert imgs[0][1] == imgs[1][1], trial
            assert np.array_equal(imgs[0][0].view(np.uint64), imgs[1][0].view(np.uint64)), trial
    finally:
        rend.set_option(capi.RT_OPT_EYE_TABLES, 1)


# ---------------------------------------------------------------- tile bins
def _random_wall(rng, near=None):
    nrm = rng.normal(size=3)
    nrm /= np.linalg.norm(nrm)
    pos = rng.uniform(-6, 6, 3) if near is None else near + rng.normal(scale=0.05, size=3)
    return scenes.Wall(scenes.Material(tuple(rng.uniform(0, 1, 3)), .5), tuple(pos), tuple(nrm),
                       float(rng.uniform(.5, 8)), float(rng.uniform(.5, 8)))


@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64,
                                  capi.RT_PREC_F32])
def test_tile_bins_are_output_invariant(rend, prec):
    """The primary-ray tile bins (rt_device.h TileBin, k_bin) only skip primitives the
    reference's own test rejects for every ray of a tile, and bounds tests it passes:
    frames with and without them are bitwise identical — random scenes and views, walls
    through the camera and seen edge-on, wide and narrow fields of view, ragged images,
    row bands, up to the 64-primitive limit; the mirror bins of the first bounce off a wall
    (camera reflected in the wall's plane) likewise."""
    rng = np.random.default_rng(31)
    rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 2**31 - 1)  # linear scan up to 64 prims
    try:
        # <= 128 wall x primitive pairs also exercise the mirror (first-bounce) bins
        trials = [(1, 0), (0, 1), (5, 3), (8, 4), (8, 6), (2, 9), (0, 11), (4, 7), (20, 12),
                  (40, 24), (58, 6), (3, 40)]
        for trial, (ns, nw) in enumerate(trials * 2):
            sc = scenes.synthetic_scene(ns, min(nw, 6), seed=int(rng.integers(1 << 30)))
            pos = rng.uniform([-1, -3, -1], [5, 3, 2])
            for k in range(nw - 6):
                # some walls pass (almost) through the camera or contain its position
                sc.append(_random_wall(rng, near=pos if k % 3 == 0 else None))
            rend.set_scene(scenes.to_prims(sc))
            vfov = float(rng.choice([20.0, 60.0, 90.0, 150.0, 178.0]))
            w = int(rng.choice([1, 9, 64, 161, 240]))
            aspect = float(rng.choice([1.0, 16 / 9, 4 / 3, 0.5]))
            look = pos + rng.normal(size=3)
            if trial % 4 == 3:   # axis-aligned view: rays in the walls' planes
                look = pos + np.array([1.0, 0.0, 0.0])
            cam = capi.camera_init(pos, look, (0, 0, -1), vfov, aspect, float(w))
            if cam.height <= 0:
                continue
            depth = int(rng.integers(0, 6))
            r0 = int(rng.integers(0, cam.height))
            n = int(rng.integers(1, cam.height - r0 + 1))
            imgs = []
            for on in (1, 0):
                rend.set_option(capi.RT_OPT_TILE_BINS, on)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True,
                                      row0=r0, nrows=n)
                imgs.append((img, st.segments))
            assert imgs[0][1] == imgs[1][1], trial
            assert np.array_equal(imgs[0][0].view(np.uint64), imgs[1][0].view(np.uint64)), trial
    finally:
        rend.set_option(capi.RT_OPT_TILE_BINS, 1)
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)


@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_MIXED, capi.RT_PREC_PATH64,
                                  capi.RT_PREC_F32])
def test_cull_wall_bins_are_output_invariant(rend, prec):
    """Scenes that use the wave cull keep the cone for their spheres but give their walls
    pixel boxes (KParams::nwbox, RT_CULL_WALL_BINS): the primary segment tests only the walls
    whose box meets the tile, and the bounce segments only the walls whose circumscribed ball
    meets the wave's cone (RT_CULL_WALL_CONE).  Frames with the boxes (RT_OPT_TILE_BINS 1),
    without, and from the linear-scan kernels are bitwise identical, segment counts too —
    random sphere clouds with up to 40 walls, walls through the camera, axis-aligned views,
    ragged images, row bands."""
    rng = np.random.default_rng(47)
    rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 0)  # every scene takes the cull kernels
    try:
        for trial, (ns, nw) in enumerate([(24, 6), (64, 6), (30, 12), (8, 3), (70, 40), (3, 1),
                                          (40, 20), (100, 6)]):
            sc = scenes.synthetic_scene(ns, min(nw, 6), seed=int(rng.integers(1 << 30)))
            pos = rng.uniform([-1, -3, -1], [5, 3, 2])
            for k in range(nw - 6):
                sc.append(_random_wall(rng, near=pos if k % 3 == 0 else None))
            rend.set_scene(scenes.to_prims(sc))
            vfov = float(rng.choice([20.0, 60.0, 90.0, 150.0]))
            w = int(rng.choice([9, 64, 161, 320]))
            aspect = float(rng.choice([1.0, 16 / 9, 4 / 3]))
            look = pos + (np.array([1.0, 0.0, 0.0]) if trial % 4 == 3 else rng.normal(size=3))
            cam = capi.camera_init(pos, look, (0, 0, -1), vfov, aspect, float(w))
            if cam.height <= 0:
                continue
            depth = int(rng.integers(0, 7))
            r0 = int(rng.integers(0, cam.height))
            n = int(rng.integers(1, cam.height - r0 + 1))
            imgs = []
            for on in (1, 0):
                rend.set_option(capi.RT_OPT_TILE_BINS, on)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True,
                                      row0=r0, nrows=n)
                imgs.append((img, st.segments))
            # and the linear scan (no cone: every wall and sphere tested, RT_CULL_WALL_CONE's
            # bounce-segment wall cull included in the comparison)
            rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 2**31 - 1)
            rend.set_option(capi.RT_OPT_TILE_BINS, 0)
            img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True,
                                  row0=r0, nrows=n)
            imgs.append((img, st.segments))
            rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 0)
            for q in (1, 2):
                assert imgs[0][1] == imgs[q][1], (trial, q)
                assert np.array_equal(imgs[0][0].view(np.uint64), imgs[q][0].view(np.uint64)), (trial, q)
        # the configs' own scene and view at a reduced size (c3: 64 spheres + 6 walls)
        cfg = scenes.CONFIGS["c3"]
        rend.set_scene(scenes.to_prims(cfg.scene()))
        cam = capi.camera_init(**scenes.camera_args(640, 360))
        imgs = []
        for on in (1, 0):
            rend.set_option(capi.RT_OPT_TILE_BINS, on)
            imgs.append(rend.render(cam, cfg.depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True))
        assert imgs[0][1].segments == imgs[1][1].segments
        assert np.array_equal(imgs[0][0].view(np.uint64), imgs[1][0].view(np.uint64))
    finally:
        rend.set_option(capi.RT_OPT_TILE_BINS, 1)
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)


@pytest.mark.parametrize("prec", [capi.RT_PREC_F64, capi.RT_PREC_PATH64])
def test_wall_order_is_output_invariant(rend, prec):
    """RT_OPT_WALL_ORDER (the primary scan visits walls nearest to the camera first): the
    reference scans in scene order with a strict `<` (main.cpp:77), so the winner of an
    exact tie is the lower scene index; visiting walls in another order must give the
    same frame bitwise.  Random wall sets and views, plus scenes holding the same wall
    twice (exact ties on every pixel it covers, with different colours) in front of and
    behind others."""
    rng = np.random.default_rng(57)
    try:
        for trial in range(16):
            sc = scenes.synthetic_scene(int(rng.integers(0, 6)), int(rng.integers(0, 7)),
                                        seed=int(rng.integers(1 << 30)))
            for _ in range(int(rng.integers(1, 6))):
                sc.append(_random_wall(rng))
            walls = [o for o in sc if o.kind == capi.RT_PRIM_WALL]
            if trial % 2 == 0 and walls:
                # a duplicate of an earlier wall, later in scene order, another colour
                w = walls[int(rng.integers(len(walls)))]
                sc.append(scenes.Wall(scenes.Material(tuple(rng.uniform(0, 1, 3)), .3),
                                      w.position, w.normal, w.length, w.width))
                if trial % 4 == 0:   # and one before it
                    sc.insert(0, scenes.Wall(scenes.Material((.9, .1, .1), .7), w.position,
                                             w.normal, w.length, w.width))
            rend.set_scene(scenes.to_prims(sc))
            pos = rng.uniform([-2, -3, -1], [4, 3, 2])
            cam = capi.camera_init(pos, pos + rng.normal(size=3), (0, 0, -1),
                                   float(rng.choice([40.0, 90.0, 150.0])), 4 / 3, 160.0)
            depth = int(rng.integers(0, 5))
            imgs = []
            for on in (1, 0):
                rend.set_option(capi.RT_OPT_WALL_ORDER, on)
                img, st = rend.render(cam, depth, prec, 0, capi.RT_OUT_RGB_F64, count_segments=True)
                imgs.append((img, st.segments))
            assert imgs[0][1] == imgs[1][1], trial
            assert np.array_equal(imgs[0][0].view(np.uint64), imgs[1][0].view(np.uint64)), trial
    finally:
        rend.set_option(capi.RT_OPT_WALL_ORDER, 1)


def test_row_order_is_output_invariant(rend):
    """Centre-out tile-row dispatch (RT_OPT_ROW_ORDER) only reorders work: bitwise equal
    frames and segment counts, on full frames and row bands of ragged sizes."""
    sc = scenes.synthetic_scene(8, 4)
    rend.set_scene(scenes.to_prims(sc))
    try:
        # (200, 64): 25 tile columns in 2 dispatch parts of 13, so one workgroup of each
        # tile row lies past the row's end (every lane invalid, no store, no cost stamp)
        for w, h, r0, n in ((160, 90, 0, 90), (203, 117, 13, 71), (64, 36, 35, 1),
                            (200, 64, 0, 64)):
            cam = capi.camera_init(**scenes.camera_args(w, h))
            imgs = []
            for on in (1, 0):
                rend.set_option(capi.RT_OPT_ROW_ORDER, on)
                img, st = rend.render(cam, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32,
                                      count_segments=True, row0=r0, nrows=n)
                imgs.append((img, st.segments))
            assert imgs[0][1] == imgs[1][1]
            assert np.array_equal(imgs[0][0].view(np.uint32), imgs[1][0].view(np.uint32))
    finally:
        rend.set_option(capi.RT_OPT_ROW_ORDER, 1)


def test_row_feedback_and_explicit_orders_are_output_invariant(rend):
    """RT_OPT_ROW_FEEDBACK (measured tile-row order, stamped kernels on sampled frames) and
    rt_set_row_order (any permutation) only reorder work: every frame bitwise equal to the
    top-to-bottom render, on full frames and ragged row bands, F32/PATH64/F64; invalid
    permutations are rejected."""
    sc = scenes.synthetic_scene(8, 4)
    rend.set_scene(scenes.to_prims(sc))
    rng = np.random.default_rng(7)
    try:
        for w, h, r0, n in ((160, 90, 0, 90), (203, 117, 13, 71), (64, 36, 35, 1)):
            cam = capi.camera_init(**scenes.camera_args(w, h))
            for prec in (capi.RT_PREC_PATH64, capi.RT_PREC_F32, capi.RT_PREC_F64):
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
                rend.set_option(capi.RT_OPT_ROW_ORDER, 0)
                ref, st0 = rend.render(cam, 4, prec, 0, capi.RT_OUT_RGB_F32,
                                       count_segments=True, row0=r0, nrows=n)
                rend.set_option(capi.RT_OPT_ROW_ORDER, 1)
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 1)  # sample every other frame
                for _ in range(6):
                    img, st = rend.render(cam, 4, prec, 0, capi.RT_OUT_RGB_F32,
                                          count_segments=True, row0=r0, nrows=n)
                    assert st.segments == st0.segments
                    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
                gy = (n + 7) // 8
                for _ in range(3):
                    rend.set_row_order(rng.permutation(gy).tolist())
                    img, _ = rend.render(cam, 4, prec, 0, capi.RT_OUT_RGB_F32, row0=r0, nrows=n)
                    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
                rend.set_row_order(None)
        for bad in ([0, 0], [1, 2], [-1, 0]):
            with pytest.raises(capi.RTError):
                rend.set_row_order(bad)
    finally:
        rend.set_row_order(None)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 32)
        rend.set_option(capi.RT_OPT_ROW_ORDER, 1)


def test_render_device_frames_equals_per_frame_calls(rend):
    """rt_render_device_frames (the bench's frame loop in one call): frame f renders
    cams[f % 2] into buffer f % 3 on stream f % 3 — each buffer ends bitwise equal to a
    single render of the camera of its last frame; bad arguments are rejected."""
    import torch
    dev = torch.device("cuda", 0)
    sc = scenes.synthetic_scene(8, 4)
    rend.set_scene(scenes.to_prims(sc))
    ca = scenes.camera_args(160, 90)
    cams = [capi.camera_init(**ca)]
    a = dict(ca)
    a["position"] = (ca["position"][0] + 0.3, ca["position"][1], ca["position"][2])
    cams.append(capi.camera_init(**a))
    refs = [rend.render(c, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)[0] for c in cams]
    sts = [torch.cuda.Stream(dev) for _ in range(3)]
    # with the host pipeline (the default: the next frames' arguments on a helper thread) and
    # without it; batches of 1 (no helper), 7 and 40 frames
    for pipe in (1, 0):
        rend.set_option(capi.RT_OPT_HOST_PIPELINE, pipe)
        for nf in (1, 7, 40):
            outs = [torch.zeros((90, 160, 3), dtype=torch.float32, device=dev) for _ in range(3)]
            torch.cuda.synchronize()
            rend.render_device_frames(cams, 4, [o.data_ptr() for o in outs], capi.RT_PREC_PATH64,
                                      streams=[s.cuda_stream for s in sts], nframes=nf)
            torch.cuda.synchronize()
            for b, o in enumerate(outs):
                fr = [f for f in range(nf) if f % 3 == b]
                want = refs[fr[-1] % 2] if fr else np.zeros_like(refs[0])
                assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32)), (pipe, nf, b)
        with pytest.raises(capi.RTError):
            rend.render_device_frames(cams, 4, [], capi.RT_PREC_PATH64, nframes=1)
        # a batch whose second camera is invalid stops there with its status, pipeline or not
        bad = capi.camera_init(**ca)
        bad.height = -1
        with pytest.raises(capi.RTError):
            rend.render_device_frames([cams[0], bad], 4, [o.data_ptr() for o in outs],
                                      capi.RT_PREC_PATH64, streams=[sts[0].cuda_stream], nframes=4)
        torch.cuda.synchronize()
    rend.set_option(capi.RT_OPT_HOST_PIPELINE, 1)


@pytest.mark.parametrize("prec", [capi.RT_PREC_PATH64, capi.RT_PREC_F64, capi.RT_PREC_F32])
def test_frame_batch_launches_equal_per_frame_launches(rend, prec):
    """RT_OPT_FRAME_BATCH (one launch per batch of band frames): consecutive
    frames on one stream go to the GPU as one grid (frame = blockIdx.z, arguments from a
    device table).  A moving camera, 13 frames — into 13 distinct buffers (groups of B = 4,
    the last one short), into 5 buffers (a group breaks at a repeated buffer, in order), and
    over 2 alternating streams (groups of one) — every buffer bitwise equal to the per-frame
    render of its last camera; with the row feedback sampling every second frame (sampled
    frames leave the group and launch alone through the stamped kernels) and off; a full
    frame and a ragged band; the c2 scene in the bench precision and the others."""
    import torch
    dev = torch.device("cuda", 0)
    sc = scenes.CONFIGS["c2"].scene()
    rend.set_scene(scenes.to_prims(sc))
    W, H = 320, 180
    ca = scenes.camera_args(W, H)
    cams = []
    for k in range(6):
        a = dict(ca)
        a["position"] = (ca["position"][0] + 0.04 * k, ca["position"][1], ca["position"][2])
        cams.append(capi.camera_init(**a))
    fmt = capi.RT_OUT_RGB_F32
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    nf = 13
    try:
        for r0, n in ((0, H), (21, 97)):
            rend.set_option(capi.RT_OPT_FRAME_BATCH, 1)
            refs = [rend.render(c, 4, prec, 0, fmt, row0=r0, nrows=n)[0] for c in cams]
            for fb_rows in (2, 0):
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, fb_rows)
                rend.set_option(capi.RT_OPT_FRAME_BATCH, 4)
                for nb, sts in ((13, [s1]), (5, [s1]), (4, [s1, s2])):
                    outs = [torch.full((n, W, 3), -1.0, device=dev) for _ in range(nb)]
                    torch.cuda.synchronize()
                    rend.render_device_frames(cams, 4, [o.data_ptr() for o in outs], prec, 0, fmt,
                                              row0=r0, nrows=n, streams=[s.cuda_stream for s in sts],
                                              nframes=nf)
                    torch.cuda.synchronize()
                    for b, o in enumerate(outs):
                        lf = max(f for f in range(nf) if f % nb == b)
                        assert np.array_equal(o.cpu().numpy().view(np.uint32),
                                              refs[lf % len(cams)].view(np.uint32)), (r0, fb_rows, nb, b)
        for bad in (0, capi.RT_MULTI_BATCH_MAX + 1):
            with pytest.raises(capi.RTError):
                rend.set_option(capi.RT_OPT_FRAME_BATCH, bad)
    finally:
        rend.set_option(capi.RT_OPT_FRAME_BATCH, 1)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 32)


def test_row_feedback_isolated_sampling_in_flight(rend):
    """Row feedback on frames in flight (three caller streams, a snapshot every other
    frame): with RT_OPT_ROW_FEEDBACK_ISOLATE on (default off) the sampled frames are ordered
    between their neighbours on the device, and every frame is still the same frame —
    each buffer bitwise equal to a plain render, isolation on or off, for a full frame and
    a ragged band (the snapshot's per-unit reduction k_unit_max covers both)."""
    import torch
    dev = torch.device("cuda", 0)
    sc = scenes.synthetic_scene(8, 4)
    rend.set_scene(scenes.to_prims(sc))
    cam = capi.camera_init(**scenes.camera_args(200, 117))
    try:
        for r0, n in ((0, 117), (13, 71)):
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 0)
            ref, _ = rend.render(cam, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32, row0=r0, nrows=n)
            for iso in (1, 0):
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK_ISOLATE, iso)
                rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 1)
                outs = [torch.zeros((n, 200, 3), dtype=torch.float32, device=dev) for _ in range(3)]
                sts = [torch.cuda.Stream(dev) for _ in range(3)]
                rend.render_device_frames([cam], 4, [o.data_ptr() for o in outs], capi.RT_PREC_PATH64,
                                          row0=r0, nrows=n, streams=[s.cuda_stream for s in sts],
                                          nframes=24)
                torch.cuda.synchronize()
                for o in outs:
                    assert np.array_equal(o.cpu().numpy().view(np.uint32), ref.view(np.uint32)), (r0, iso)
        with pytest.raises(capi.RTError):
            rend.set_option(capi.RT_OPT_ROW_FEEDBACK_ISOLATE, 2)
    finally:
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK_ISOLATE, 0)   # the product default
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 32)


def _pair_ab(rend, cam, depth, flags=0, **kw):
    """(one pixel per lane, two pixels per lane) PATH64 frames + segment counts."""
    out = []
    for on in (0, 1):
        rend.set_option(capi.RT_OPT_PIXEL_PAIRS, on)
        img, st = rend.render(cam, depth, capi.RT_PREC_PATH64, flags, capi.RT_OUT_RGB_F32,
                              count_segments=True, **kw)
        out.append((img, st.segments))
    return out


def test_pixel_pairs_bitwise(rend):
    """RT_OPT_PIXEL_PAIRS (two pixels per lane, 16x8 pixels per wave) evaluates every test,
    shading step and unwind of the one-pixel PATH64 kernel under shared branches with
    predicated takes: frames and segment counts bitwise equal to the one-pixel kernel —
    random scenes and views up to the 64-primitive tile-bin limit (walls through the camera,
    edge-on views), ragged widths (a lane's second pixel past the row end), row bands,
    every register-stack tier (depth 0-12), the sun extension, bins on and off, and
    full-size c2 under the measured row order."""
    rng = np.random.default_rng(91)
    rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 2**31 - 1)  # linear scan up to 64 prims
    try:
        trials = [(1, 0), (0, 1), (8, 4), (8, 6), (2, 9), (4, 7), (20, 12), (40, 24), (3, 40),
                  (16, 2)]
        for trial, (ns, nw) in enumerate(trials * 2):
            sc = scenes.synthetic_scene(ns, min(nw, 6), seed=int(rng.integers(1 << 30)))
            pos = rng.uniform([-1, -3, -1], [5, 3, 2])
            for k in range(nw - 6):
                sc.append(_random_wall(rng, near=pos if k % 3 == 0 else None))
            rend.set_scene(scenes.to_prims(sc))
            vfov = float(rng.choice([20.0, 60.0, 90.0, 150.0]))
            w = int(rng.choice([1, 9, 15, 64, 161, 240]))
            aspect = float(rng.choice([1.0, 16 / 9, 4 / 3, 0.5]))
            look = pos + rng.normal(size=3)
            if trial % 4 == 3:
                look = pos + np.array([1.0, 0.0, 0.0])
            cam = capi.camera_init(pos, look, (0, 0, -1), vfov, aspect, float(w))
            if cam.height <= 0:
                continue
            depth = int(rng.choice([0, 1, 2, 4, 6, 9, 12]))
            r0 = int(rng.integers(0, cam.height))
            n = int(rng.integers(1, cam.height - r0 + 1))
            flags = capi.RT_FLAG_SUN if trial % 5 == 4 else 0
            rend.set_option(capi.RT_OPT_TILE_BINS, 0 if trial % 7 == 6 else 1)
            (i1, s1), (i2, s2) = _pair_ab(rend, cam, depth, flags, row0=r0, nrows=n)
            assert s1 == s2, trial
            assert np.array_equal(i1.view(np.uint32), i2.view(np.uint32)), trial
        rend.set_option(capi.RT_OPT_TILE_BINS, 1)
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)
        # the bench scene at full size, measured row order (stamped frames included)
        cfg = scenes.CONFIGS["c2"]
        rend.set_scene(scenes.to_prims(cfg.scene()))
        cam = capi.camera_init(**scenes.camera_args(cfg.width, cfg.height))
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 1)
        (ref, s_ref), _ = _pair_ab(rend, cam, cfg.depth)
        rend.set_option(capi.RT_OPT_PIXEL_PAIRS, 1)
        for _ in range(4):
            img, st = rend.render(cam, cfg.depth, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32,
                                  count_segments=True)
            assert st.segments == s_ref
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    finally:
        rend.set_option(capi.RT_OPT_PIXEL_PAIRS, 0)
        rend.set_option(capi.RT_OPT_ROW_FEEDBACK, 32)
        rend.set_option(capi.RT_OPT_TILE_BINS, 1)
        rend.set_option(capi.RT_OPT_WAVE_CULL_MIN_SPHERES, 24)


# ---------------------------------------------------------------- headless frame loop
def _read_ppm(path):
    with open(path, "rb") as fh:
        data = fh.read()
    magic, w, h, mx, rest = data.split(maxsplit=4)
    assert magic == b"P6" and mx == b"255"
    return np.frombuffer(rest, np.uint8).reshape(int(h), int(w), 3)


@pytest.mark.parametrize("scene,width", [("default", 64), ("synthetic:16,6,7", 128)])
def test_frame_loop_binary(tmp_path, oracle, scene, width):
    """bin/rt_frames (host/rt_frames.cpp): main.cpp's loop without SDL — scripted camera
    moves (init() not re-called: stale image_top_left), rt_scene per frame, the
    SDL_MapRGB(val*255) packing, and main.cpp's performance log.  The last frame's surface
    equals main.cpp:345's bytes of the oracle's fp64 frame (x86-64 conversion: highlights
    above 1.0 wrap modulo 256 — the synthetic scene has dozens of them), with rt_scene
    (mixed = fp64 path) and with the kernel's RT_OUT_RGBA8_WRAP epilogue (--gpu-surface)."""
    import re
    import subprocess
    from conftest import PKG
    exe = os.path.join(PKG, "bin", "rt_frames")
    outs = {}
    for mode in ("host", "gpu"):
        ppm = str(tmp_path / f"{mode}.ppm")
        cmd = [exe, "--frames", "3", "--width", str(width), "--keys", "wd", "--precision", "mixed",
               "--scene", scene, "--ppm", ppm] + (["--gpu-surface"] if mode == "gpu" else [])
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        assert res.returncode == 0, res.stderr
        lines = res.stdout.strip().splitlines()
        assert re.fullmatch(r"Number of frames: 3 : \d+ ms average frame time", lines[0]), lines
        for ln, unit, what in zip(lines[1:], ["microseconds"] * 3 + ["milliseconds"] * 2,
                                  ["raytracing", "outpainting", "shading", "surface average update",
                                   "SDL rendering"]):
            assert re.fullmatch(rf"   \d+ {unit} for (average )?{what}", ln), ln
        outs[mode] = _read_ppm(ppm)
    assert np.array_equal(outs["host"], outs["gpu"])
    # expected: frames 'w', 'd', 'w' move the camera (scene.cpp:108-165), init() once
    cam = capi.camera_init((0, 0, 0), (-1, 0, 0), (0, 0, -1), 90.0, 1.0, float(width))
    cam.position[0] = 0.1 + 0.1
    cam.position[1] = 0.1
    if scene == "default":
        sc = scenes.default_scene()
    else:
        ns, nw, seed = (int(v) for v in scene.split(":")[1].split(","))
        sc = scenes.synthetic_scene(ns, nw, seed=seed)
    ref64, _, _ = oracle.render(scenes.to_prims(sc), cam, 10)
    exp = oracle.surface_u8(ref64)
    t = ref64 * 255.0
    edge = np.abs(t - np.round(t)) < 1e-9   # fp64 path within 1e-12: only exact boundaries
    assert ((outs["host"] == exp) | edge).all()
    if scene != "default":
        assert int(((ref64 > 1.0) & ~edge).sum()) >= 20   # the wrap is exercised


# ---------------------------------------------------------------- multi-GPU path (1 rank)
def test_render_tiled_rccl_single_rank(rend):
    """rtamd.tiling.render_tiled over the nccl (RCCL) backend with one rank: the gathered
    frame equals a plain render (the N-rank CPU path is covered by test_dist_gloo.py)."""
    import socket
    import torch
    import torch.distributed as dist
    from rtamd import tiling
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        sc = scenes.synthetic_scene(8, 4)
        rend.set_scene(scenes.to_prims(sc))
        cam = capi.camera_init(**scenes.camera_args(160, 90))
        frame = tiling.render_tiled(rend, cam, 4, capi.RT_PREC_PATH64)
        torch.cuda.synchronize()
        ref, _ = rend.render(cam, 4, capi.RT_PREC_PATH64, 0, capi.RT_OUT_RGB_F32)
        assert np.array_equal(frame.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        # an explicit stream that is NOT the current one: the gather (ordered after the
        # current stream by ProcessGroupNCCL) must still see the finished band
        big = capi.camera_init(**scenes.camera_args(1920, 1080))
        rend.set_scene(scenes.to_prims(scenes.synthetic_scene(64, 6)))
        side = torch.cuda.Stream()
        assert side != torch.cuda.current_stream()
        frame = tiling.render_tiled(rend, big, 6, capi.RT_PREC_F64, stream=side)
        got = frame.cpu().numpy()
        ref, _ = rend.render(big, 6, capi.RT_PREC_F64, 0, capi.RT_OUT_RGB_F32)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    finally:
        dist.destroy_process_group()
