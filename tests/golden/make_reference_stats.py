"""Statistics of the reference's own sample renders (/root/reference/images/*.png),
the only outputs of the reference itself available: size, per-channel
mean / standard deviation and 16-bin per-channel histograms of the 8-bit RGB values.

The reference's scenes draw their object placement and every path from OS-seeded
thread_rng, and the spp used for these images is not recorded, so they cannot be
matched pixel for pixel: tests/test_gpu_reference_images.py compares the same
statistics of this build's renders of the same scenes as a sanity check (stated
tolerances, not parity). This script runs where /root/reference exists (the build
container) and writes reference_image_stats.json next to it; the GPU box only reads the JSON.

    python3 tests/golden/make_reference_stats.py
"""
import json
import os

import numpy as np
from PIL import Image

REF = "/root/reference/images"
HERE = os.path.dirname(os.path.abspath(__file__))
# image -> the reference scene (src/main.rs:140-153) and the framing it was rendered with
# (the scenes' book framings; the CLI flags used for the images are not recorded)
IMAGES = {
    "showcase": dict(scene="showcase", look_from=(478.0, 278.0, -600.0), look_at=(278.0, 278.0, 0.0), vfov=40.0,
                     aperture=0.0, time=(0.0, 1.0)),
    "smoke": dict(scene="cornell-smoke", look_from=(278.0, 278.0, -800.0), look_at=(278.0, 278.0, 0.0), vfov=40.0,
                  aperture=0.0, time=(0.0, 1.0)),
    "motion_blur": dict(scene="random-moving-spheres", look_from=(13.0, 2.0, 3.0), look_at=(0.0, 0.0, 0.0), vfov=20.0,
                        aperture=0.1, time=(0.0, 1.0)),
    "spheres_render_checkered": dict(scene="random-spheres", look_from=(13.0, 2.0, 3.0), look_at=(0.0, 0.0, 0.0),
                                     vfov=20.0, aperture=0.1, time=(0.0, 0.0)),
    "lights_and_marble": dict(scene="simple-lights", look_from=(26.0, 3.0, 6.0), look_at=(0.0, 2.0, 0.0), vfov=20.0,
                              aperture=0.0, time=(0.0, 0.0)),
}


def stats(rgb8: np.ndarray) -> dict:
    a = rgb8.reshape(-1, 3).astype(np.float64) / 255.0
    hist = [np.histogram(rgb8.reshape(-1, 3)[:, c], bins=16, range=(0, 256))[0] / len(a) for c in range(3)]
    return {"mean": a.mean(axis=0).tolist(), "std": a.std(axis=0).tolist(), "hist16": [h.tolist() for h in hist]}


def main():
    out = {}
    for name, framing in IMAGES.items():
        im = Image.open(os.path.join(REF, name + ".png")).convert("RGB")
        w, h = im.size
        out[name] = {"width": w, "height": h, **framing, **stats(np.asarray(im))}
    json.dump(out, open(os.path.join(HERE, "reference_image_stats.json"), "w"), indent=1)
    for k, v in out.items():
        print(k, v["width"], v["height"], np.round(v["mean"], 4))


if __name__ == "__main__":
    main()
