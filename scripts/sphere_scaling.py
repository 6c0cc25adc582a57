#!/usr/bin/env python3
"""Sphere-count scaling of the sphere-world tiers (GPU box): book-1-style
worlds -- the ground sphere plus N small spheres drawn with the R28 recipe
 over a square of cells around the book-1 camera's view, three big
spheres -- at 1920x1080, --spp (default 64), depth 50.  Prints per N the
kernel tier the launcher picked, the 4-wide node count and the path-kernel
Msamples/s: where the basic tier's LDS node copy ends and the mesh tier
takes over.
  python scripts/sphere_scaling.py [spp] [N ...]"""
import ctypes
import importlib
import json
import math
import os
import sys

import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
pkg = importlib.import_module("raytracer-2025_amd")


def world(s, n, seed=7):
    g = scenes.SplitMix64(seed)
    objs = s.Hittables()
    objs.add(s.Sphere((0, -1000, 0), 1000, s.Lambertian(s.SolidColor((0.5, 0.5, 0.5)))))
    side = max(1, int(math.ceil(math.sqrt(n))))
    half = side / 2.0
    cell = 22.0 / max(side, 22) if side > 22 else 1.0
    k = 0
    for a in range(side):
        for b in range(side):
            if k >= n:
                break
            k += 1
            cm = g.f64()
            c = ((a - half) * cell + 0.9 * cell * g.f64(), 0.2, (b - half) * cell + 0.9 * cell * g.f64())
            r = 0.2 * min(1.0, cell)
            if cm < 0.8:
                mat = s.Lambertian(s.SolidColor((g.f64() * g.f64(), g.f64() * g.f64(), g.f64() * g.f64())))
            elif cm < 0.95:
                mat = s.Metal((g.range(0.5, 1), g.range(0.5, 1), g.range(0.5, 1)), g.range(0, 0.5))
            else:
                mat = s.Dielectric(s.SolidColor((1, 1, 1)), 1.5)
            objs.add(s.Sphere((c[0], r, c[2]), r, mat))
    objs.add(s.Sphere((0, 1, 0), 1.0, s.Dielectric(s.SolidColor((1, 1, 1)), 1.5)))
    objs.add(s.Sphere((-4, 1, 0), 1.0, s.Lambertian(s.SolidColor((0.4, 0.2, 0.1)))))
    objs.add(s.Sphere((4, 1, 0), 1.0, s.Metal((0.7, 0.6, 0.5), 0.0)))
    w = s.Hittables()
    w.add(s.BVH(objs))
    return w


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    counts = [int(x) for x in sys.argv[2:]] or [100, 485, 900, 1500, 3000, 10000, 50000]
    lib = os.environ.get("RT_LIB")  # another build of the library (A/B), else the product's
    api = capi.Api(ctypes.CDLL(os.path.join(ROOT, "raytracer-2025_amd", lib)), "rt_") if lib else pkg.load()
    torch.cuda.init()
    out = []
    for n in counts:
        s = rt.Scene(api)
        w = world(s, n)
        _, _, cam = scenes.random_spheres(s, 1920, spp)  # the book-1 camera and sky
        info = capi.RtWorldInfo()
        api.check(api.world_info_get(s.s, w.h, -1, cam.background.h, 0, ctypes.byref(info)))
        cam.render(w, None, seed=1, want_srgb=False)  # warm-up + upload
        best = None
        for _ in range(3):
            _, _, st = cam.render(w, None, seed=1, want_srgb=False)
            best = st.kernel_ms if best is None else min(best, st.kernel_ms)
        rec = {"spheres": n + 4, "tier": info.kernel_tier, "bvh4_nodes": info.bvh_nodes, "kernel_ms": round(best, 3),
               "msamples_per_s": round(cam.traced_samples() / (best * 1e-3) / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    print(json.dumps({"spp": spp, "runs": out}))


if __name__ == "__main__":
    main()
