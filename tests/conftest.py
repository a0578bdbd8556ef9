import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ray-tracer-from-scratch_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def has_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc_mod
    return orc_mod.Oracle()


@pytest.fixture(scope="session")
def golden_frames():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "frames.npz"))


@pytest.fixture(scope="session")
def golden_rays():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "rays.npz"))


@pytest.fixture(scope="session")
def kat():
    import json
    with open(os.path.join(GOLDEN, "kat.json")) as fh:
        return json.load(fh)


def parse_frame_key(key: str):
    scene_name, size, depth = key.split("__")
    w, h = (int(v) for v in size.split("x"))
    return scene_name, w, h, int(depth[1:])


def scene_by_name(name: str):
    from rtamd import scenes
    return {
        "default": scenes.default_scene,
        "s8w4": lambda: scenes.synthetic_scene(8, 4),
        "s64w6": lambda: scenes.synthetic_scene(64, 6),
        "s256w0": lambda: scenes.synthetic_scene(256, 0),
    }[name]()


@pytest.fixture(scope="session")
def golden_surface():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "surface.npz"))
