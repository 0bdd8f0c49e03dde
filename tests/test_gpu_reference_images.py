"""Statistical link between this build and the reference's OWN renders.

The reference's sample images (images/*.png, decoded once in the build container by
tests/golden/make_reference_stats.py into reference_image_stats.json) are the only
outputs of the reference itself that exist. Its scenes place objects and trace paths
with OS-seeded thread_rng and the spp of the images is not recorded, so the images
cannot be matched pixel for pixel; what must agree is the picture's overall light:
the per-channel mean and the 8-bit value histograms. This test renders the same scene
with the same framing and size on the GPU, quantises it with the output step
(palette 0.6.1, rt_quantize_srgb8) and compares:

  mean:  |mean_ours - mean_ref| per channel (values in [0, 1]) < 0.06
  hist:  total-variation distance of the 16-bin per-channel histograms < 0.35

These are sanity bounds for a statistical comparison, not a parity claim (parity is
bit-exactness against the oracle, test_gpu_parity.py). The measured numbers are
printed and written to gpurun_out/reference_images.json.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STATS = json.load(open(os.path.join(HERE, "golden", "reference_image_stats.json")))
# lights_and_marble.png shows the simple_lights geometry (src/main.rs:377-401) under the book
# camera — the sphere light, the marble sphere and the edge-on XyRect light sit at the oracle
# render's pixel positions — but not its light: main.rs:393's emission 4 gives a u8 mean of 0.079
# (0.148 with a gamma-2 curve) against the image's 0.239, and tests/golden/lights_and_marble_search.py
# finds the image's mean and histogram at emission 16 with gamma 2 (mean 0.246, histogram TV 0.06)
# or emission 32 linear (0.245, TV 0.08): the image was rendered with 4-8x brighter lights than the
# source holds. Reported, not asserted.
STALE = {"lights_and_marble": "image rendered with 4-8x the emission of main.rs:393 (tests/golden/"
                              "lights_and_marble_search.py: emission 16 + gamma 2 matches mean 0.246 vs 0.239, TV 0.06)"}
SPP = {"showcase": 256, "smoke": 512, "motion_blur": 128, "spheres_render_checkered": 128, "lights_and_marble": 512}


def _stats(rgb8):
    a = rgb8.reshape(-1, 3).astype(np.float64) / 255.0
    hist = [np.histogram(rgb8.reshape(-1, 3)[:, c], bins=16, range=(0, 256))[0] / len(a) for c in range(3)]
    return a.mean(axis=0), np.array(hist)


@pytest.mark.parametrize("name", [pytest.param(n, marks=pytest.mark.xfail(reason=STALE[n], strict=False))
                                  if n in STALE else n for n in sorted(STATS)])
def test_render_statistics_match_reference_image(rt, name):
    ref = STATS[name]
    w, h = ref["width"], ref["height"]
    cam = rt.Camera(tuple(ref["look_from"]), tuple(ref["look_at"]), (0.0, 1.0, 0.0), ref["vfov"],
                    float(np.float32(w) / np.float32(h)), ref["aperture"], 10.0, ref["time"][0], ref["time"][1])
    scene = rt.Scene.generate(ref["scene"], 20231)
    p = rt.render_params(w, h, SPP[name], 50, background=rt.scene_background(ref["scene"]))
    ds = rt.DeviceScene(scene)
    try:
        img, _ = ds.render(cam, p)
    finally:
        ds.close()
    mean, hist = _stats(rt.quantize_srgb8(img))
    dmean = np.abs(mean - np.array(ref["mean"]))
    tv = 0.5 * np.abs(hist - np.array(ref["hist16"])).sum(axis=1)
    rec = {"image": name, "scene": ref["scene"], "size": [w, h], "spp": SPP[name], "mean_ours": mean.tolist(),
           "mean_ref": ref["mean"], "abs_mean_diff": dmean.tolist(), "hist_tv_distance": tv.tolist()}
    print(json.dumps(rec))
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.path.join("gpurun_out", "reference_images.json"), "a") as f:
        f.write(json.dumps(rec) + "\n")
    assert (dmean < 0.06).all(), rec
    assert (tv < 0.35).all(), rec
