#!/usr/bin/env python3
"""Cost of C5's Perlin-marble texture (GPU box): the C5 scene at 1920x1080 and
--spp (default 64) as built, and with the NoiseTexture swapped for a solid
colour -- not the same image, a measurement of what the noise evaluation
costs the waves whose shading batches hold a marble hit.
  python scripts/c5_texture_cost.py [spp]"""
import importlib
import json
import os
import sys

import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
pkg = importlib.import_module("raytracer-2025_amd")


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    api = pkg.load()
    torch.cuda.init()
    out = {"spp": spp}
    for variant in ("as_built", "noise_as_solid"):
        s = rt.Scene(api)
        if variant == "noise_as_solid":
            s.NoiseTexture = lambda scale, seed: s.SolidColor((0.5, 0.5, 0.5))
        world, lights, cam = scenes.final_scene(s, 1920, spp, 40, aspect_ratio=16 / 9)
        cam.render(world, lights, seed=1, want_srgb=False)  # warm-up, flatten
        ms = []
        for _ in range(3):
            _, _, st = cam.render(world, lights, seed=1, want_srgb=False)
            ms.append(st.kernel_ms)
        out[variant] = {"kernel_ms": ms, "min": min(ms)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
