"""Scene and camera construction for the trace/shade path.

* ``default_scene()`` — the reference's own scene (main.cpp:160-163): 1 sphere + 2 walls.
* ``synthetic_scene(n_spheres, n_walls, seed)`` — the build-defined synthetic scenes of
  SURVEY §8d used by BASELINE.json's configs (SplitMix64, U() = (next()>>40)*2^-24).
* ``config(name)`` — BASELINE.json configs c1..c5 as (scene, camera args, depth).

Scenes are lists of ``SceneObject`` (kind, material, position, RAW normal as handed to the
Wall constructor, radius, length, width).  ``to_prims`` flattens them into rt_prim records
holding the OBJECT STATE — Wall's normal normalised exactly as its constructor does
(scene.h:73 → vec.cpp:21: v / sqrt(x*x + y*y + z*z), IEEE double, same order).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

from . import capi


@dataclass
class Material:
    """scene.h:35-49; constructor defaults metallic .5, ambient .1, diffuse .9,
    specular .4, specular_exponent 50 (scene.h:48)."""
    color: tuple
    metallic: float = .5
    ambient: float = .1
    diffuse: float = .9
    specular: float = .4
    specular_exponent: float = 50.0


@dataclass
class SceneObject:
    kind: int
    mat: Material
    position: tuple
    normal: tuple = (0.0, 0.0, 0.0)   # raw (constructor argument) for walls
    radius: float = 0.0
    length: float = 0.0
    width: float = 0.0


def Sphere(mat: Material, center, radius: float) -> SceneObject:
    return SceneObject(capi.RT_PRIM_SPHERE, mat, tuple(map(float, center)), radius=float(radius))


def Wall(mat: Material, position, normal, length: float = 1.0, width: float = 1.0) -> SceneObject:
    return SceneObject(capi.RT_PRIM_WALL, mat, tuple(map(float, position)),
                       normal=tuple(map(float, normal)), length=float(length), width=float(width))


def normalize3(v):
    """vec3::normalize (vec.cpp:21) in IEEE double: v / sqrt(x*x + y*y + z*z)."""
    x, y, z = (float(c) for c in v)
    ln = math.sqrt(x * x + y * y + z * z)
    return (x / ln, y / ln, z / ln) if ln != 0.0 else (math.nan, math.nan, math.nan)


def to_prims(scene) -> list:
    out = []
    for o in scene:
        p = capi.rt_prim()
        p.kind = o.kind
        p.reserved = 0
        m = p.mat
        m.color[:] = [float(c) for c in o.mat.color]
        m.ambient = o.mat.ambient
        m.metallic = o.mat.metallic
        m.diffuse = o.mat.diffuse
        m.specular = o.mat.specular
        m.specular_exponent = o.mat.specular_exponent
        p.position[:] = list(o.position)
        if o.kind == capi.RT_PRIM_WALL:
            p.normal[:] = list(normalize3(o.normal))
        else:
            p.normal[:] = [0.0, 0.0, 0.0]
        p.radius = o.radius
        p.length = o.length
        p.width = o.width
        out.append(p)
    return out


def raw_normals(scene) -> list:
    """Flat list of 3 doubles per object (the Wall constructor arguments; 0 for spheres)."""
    r = []
    for o in scene:
        r.extend(o.normal if o.kind == capi.RT_PRIM_WALL else (0.0, 0.0, 0.0))
    return r


def default_scene():
    """main.cpp:160-163."""
    return [
        Sphere(Material((0, 1, 0), 0.5), (1.5, 0, 0), .5),
        Wall(Material((0, 0, 1)), (3.0, 2, 0), (0, -1, 0), 1, 1),
        Wall(Material((0, 1, 0)), (3.0, -3, 0), (0, 1, 0), 2, 2),
    ]


class SplitMix64:
    MASK = (1 << 64) - 1

    def __init__(self, seed: int):
        self.s = seed & self.MASK

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.MASK
        return z ^ (z >> 31)

    def u(self) -> float:
        return float(self.next() >> 40) * (1.0 / 16777216.0)


WALL_NORMALS = [(0, -1, 0), (0, 1, 0), (-1, 0, 0), (-.70710678, -.70710678, 0),
                (-.70710678, .70710678, 0), (1, 0, 0)]
WALL_POSITIONS = [(3, 4, -1), (3, -4, -1), (10, -4, -1), (8, 3, -1), (8, -6, -1), (-10, -4, -1)]


def synthetic_scene(n_spheres: int, n_walls: int, seed: int = 1234):
    """spheres x=2+6U, y=-3+6U, z=-1+3U, r=.3+.5U, color=(U,U,U), metallic=U
    (drawn in that order); then walls from the fixed table, colour (.2+.6U) grey, 8x4."""
    if not 0 <= n_walls <= 6:
        raise ValueError("n_walls must be in 0..6")
    rng = SplitMix64(seed)
    scene = []
    for _ in range(n_spheres):
        x = 2 + 6 * rng.u()
        y = -3 + 6 * rng.u()
        z = -1 + 3 * rng.u()
        r = .3 + .5 * rng.u()
        cr = rng.u()
        cg = rng.u()
        cb = rng.u()
        metallic = rng.u()
        scene.append(Sphere(Material((cr, cg, cb), metallic), (x, y, z), r))
    for w in range(n_walls):
        g = .2 + .6 * rng.u()
        scene.append(Wall(Material((g, g, g), .5), WALL_POSITIONS[w], WALL_NORMALS[w], 8, 4))
    return scene


# Camera of every config (main.cpp:146-153 with aspect = W/H).
CAM_POSITION = (0.0, 0.0, 0.0)
CAM_LOOKAT = (-1.0, 0.0, 0.0)
CAM_VUP = (0.0, 0.0, -1.0)
CAM_VFOV = 90.0


def camera_args(width: int, height: int):
    aspect = float(width) / float(height)
    if int(width / aspect) != height:
        raise ValueError(f"{width}x{height}: int(W/aspect) != H")
    return dict(position=CAM_POSITION, lookat=CAM_LOOKAT, vup=CAM_VUP, vfov=CAM_VFOV,
                aspect_ratio=aspect, image_width=float(width))


@dataclass
class Config:
    name: str
    width: int
    height: int
    depth: int
    n_spheres: int = -1   # -1: the reference's default scene
    n_walls: int = 0
    seed: int = 1234
    description: str = ""
    extra: dict = field(default_factory=dict)

    def scene(self):
        if self.n_spheres < 0:
            return default_scene()
        return synthetic_scene(self.n_spheres, self.n_walls, self.seed)


# BASELINE.json "configs" (sun is off in parity mode: the reference never uses it).
CONFIGS = {
    "c1": Config("c1", 640, 480, 2, description="default Sprint-3 scene, 640x480, depth 2"),
    "c2": Config("c2", 1920, 1080, 4, 8, 4, description="1920x1080, 8 spheres + 4 walls, depth 4"),
    "c3": Config("c3", 3840, 2160, 6, 64, 6, description="3840x2160, 64 spheres + 6 walls, depth 6"),
    "c4": Config("c4", 1920, 1080, 4, 8, 4, description="c2 row-tiled across GPUs"),
    "c5": Config("c5", 7680, 4320, 8, 256, 0, description="7680x4320, 256 spheres, depth 8"),
}
