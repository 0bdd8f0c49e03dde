"""BASELINE.json configurations C1-C5 as CLI-equivalent settings.

Each config is the reference CLI invocation it names, e.g. C3 =
``shimmer showcase -w 1200 -a 3 2 -s 500 --cam-look-from 478 278 -600
--cam-look-at 278 278 0 --cam-vertical-fov 40 --cam-start-time 0 --cam-end-time 1``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np

Vec3 = Tuple[float, float, float]


@dataclass(frozen=True)
class RenderConfig:
    name: str
    scene: str
    width: int
    aspect: Tuple[float, float]
    spp: int
    depth: int
    look_from: Vec3 = (13.0, 2.0, 3.0)   # src/main.rs:76-90 defaults
    look_at: Vec3 = (0.0, 0.0, 0.0)
    view_up: Vec3 = (0.0, 1.0, 0.0)
    vfov: float = 20.0
    aperture: float = 0.0
    focus_dist: float = 10.0
    time0: float = 0.0
    time1: float = 0.0
    gpus: int = 1
    scene_seed: int = 20231
    render_seed: int = 1

    @property
    def aspect_ratio(self) -> float:
        return float(np.float32(self.aspect[0]) / np.float32(self.aspect[1]))  # main.rs:109, in f32

    @property
    def height(self) -> int:
        return int(np.float32(self.width) / np.float32(self.aspect_ratio))    # renderer.rs:37

    @property
    def samples(self) -> int:
        return self.width * self.height * self.spp

    def camera(self):
        from . import Camera
        return Camera.new(self.look_from, self.look_at, self.view_up, self.vfov, self.aspect_ratio, self.aperture,
                          self.focus_dist, self.time0, self.time1)

    def background(self) -> Vec3:
        from . import scene_background
        return scene_background(self.scene.replace("-nobvh", ""))

    def scaled(self, width: int, spp: int) -> "RenderConfig":
        from dataclasses import replace
        return replace(self, width=width, spp=spp)


_CORNELL = dict(look_from=(278.0, 278.0, -800.0), look_at=(278.0, 278.0, 0.0), vfov=40.0)

CONFIGS = {
    "C1": RenderConfig("C1", "random-spheres", 400, (16.0, 9.0), 50, 50),
    "C2": RenderConfig("C2", "random-spheres-nobvh", 1200, (3.0, 2.0), 500, 50),
    "C3": RenderConfig("C3", "showcase", 1200, (3.0, 2.0), 500, 50, look_from=(478.0, 278.0, -600.0),
                       look_at=(278.0, 278.0, 0.0), vfov=40.0, time0=0.0, time1=1.0),
    "C4": RenderConfig("C4", "bunny", 1920, (16.0, 9.0), 1000, 50, gpus=8, **_CORNELL),
    "C5": RenderConfig("C5", "cornell-smoke", 1920, (16.0, 9.0), 2000, 50, gpus=8, time0=0.0, time1=1.0, **_CORNELL),
}
