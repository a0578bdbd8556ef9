"""The C++ API mirror (include/rt/vec.h, include/rt/scene.h) compiles against host code
written like the reference's main.cpp and links to the built libraries.  Host-side values
(SceneGeometry::intersect, Camera::init, vec3::reflect) are checked on CPU against the
reference's known answers; rt_scene itself renders on the GPU (marked gpu)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, has_gpu

LIB = os.path.join(REPO, "ray-tracer-from-scratch_amd", "lib")
BIN = os.path.join(REPO, "tests", "cpp", "dropin_main")


@pytest.fixture(scope="module")
def dropin():
    src = os.path.join(REPO, "tests", "cpp", "dropin_main.cpp")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < os.path.getmtime(src):
        subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"), src,
                        "-o", BIN, "-L", LIB, "-lrt_host", "-lrt_amd", f"-Wl,-rpath,{LIB}"],
                       check=True)
    return BIN


def test_host_api_known_answers(dropin, kat):
    out = subprocess.run([dropin, "kat"], capture_output=True, text=True, check=True).stdout
    rows = {ln.split()[0]: [float(x) for x in ln.split()[1:]] for ln in out.strip().splitlines()}
    sph = {c["name"]: c for c in kat["sphere_intersect"]}
    lines = [ln.split() for ln in out.splitlines() if ln.startswith("sphere")]
    assert float(lines[0][1]) == sph["front"]["dist"]
    assert float(lines[1][1]) == sph["unnormalised_dir_world_distance"]["dist"]
    assert float(lines[2][1]) == sph["behind"]["dist"]
    assert rows["tangent"][0] == sph["tangent_det0"]["dist"] == 6.0
    wal = {c["name"]: c for c in kat["wall_intersect"]}
    assert rows["wall"] == [wal["parametric_t"]["dist"], 1.0]
    assert rows["zwall"] == [0.0]
    cam = [c for c in kat["camera_init"] if c["name"] == "c1_640x480"][0]
    assert rows["camera"] == [480.0, cam["image_top_left"][1], cam["image_top_left"][2],
                              cam["pixel_delta_x"][1], cam["pixel_delta_y"][2]]
    assert rows["reflect"] == kat["reflect"][0]["out"]


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
def test_rt_scene_dropin_matches_reference(dropin, golden_frames):
    raw = subprocess.run([dropin, "render", "48", "48"], capture_output=True, check=True).stdout
    img = np.frombuffer(raw, dtype=np.float64).reshape(48, 48, 3)
    ref = golden_frames["default__48x48__d10"]     # the reference's own rt_scene, depth 10
    assert np.abs(img - ref).max() <= 1e-12
    out = subprocess.run([dropin, "throws", "64", "48"], capture_output=True, text=True,
                         check=True).stdout
    assert out.strip() == "1"                       # main.cpp:243's [W][H] buffer throws


def test_reference_style_plugin_compiles_and_is_reported(dropin):
    """A SceneGeometry subclass written against the reference's interface (scene.h:51-60:
    intersect only) compiles against include/rt/scene.h; rt_scene rejects it with
    std::invalid_argument before any device work (so this runs on the CPU)."""
    out = subprocess.run([dropin, "plugin"], capture_output=True, text=True, check=True).stdout
    assert out.startswith("1 ") and "unsupported primitive" in out, out


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")
@pytest.mark.parametrize("n,transport", [(1, 0), (1, 2), (3, 1), (8, 1)])
def test_rt_scene_row_tiled_over_devices(dropin, golden_frames, n, transport):
    """RtSceneOptions::devices: the C++ drop-in renders every frame row-tiled over the listed
    ranks (rt_multi: one device with RCCL is the plain one-GPU renderer; with the loopback
    transport the frame goes through a one-rank RCCL communicator, released by the atexit
    shutdown at process exit; peer copies for several ranks on this box's one GPU) — the
    reference's own depth-10 frame within 1e-12, bitwise the one-GPU drop-in."""
    out = subprocess.run([dropin, "render_multi", "48", "48", str(n), str(transport)],
                         capture_output=True, check=True).stdout
    # RCCL prints its version banner on stdout when a communicator is made (loopback):
    # the frame is the last 48 x 48 x 3 doubles, after text lines only
    nbytes = 48 * 48 * 3 * 8
    raw, banner = out[-nbytes:], out[:-nbytes]
    assert all(ln.isascii() for ln in banner.splitlines()), banner[:200]
    img = np.frombuffer(raw, dtype=np.float64).reshape(48, 48, 3)
    assert np.abs(img - golden_frames["default__48x48__d10"]).max() <= 1e-12
    one = subprocess.run([dropin, "render", "48", "48"], capture_output=True, check=True).stdout
    assert raw == one
