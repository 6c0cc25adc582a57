#!/usr/bin/env python3
"""PCIe-inclusive rate (GPU box): C2 through rt_render with caller-owned HOST
buffers (linear f32 + sRGB bytes), timed from the call to its return, against
the kernel time inside it.  bench.py's `value` keeps the frame in HBM; this is
the rate a host caller of the C ABI sees.  python scripts/host_rate.py [reps]"""
import importlib
import json
import os
import sys
import time

import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("raytracer-2025_amd")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
api = pkg.load()
scene = rt.Scene(api)
world, lights, cam = scenes.random_spheres(scene, 1920, 512)
t0 = time.perf_counter()
_, _, st0 = cam.render(world, lights, seed=1)  # first call: flatten + upload
first_s = time.perf_counter() - t0
runs = []
for _ in range(reps):
    t0 = time.perf_counter()
    lin, srgb, st = cam.render(world, lights, seed=1)
    runs.append((time.perf_counter() - t0, st.kernel_ms, st.render_ms, st.samples))
best = min(runs)
print(json.dumps({
    "workload": "C2 1920x1080, 484 traced spp, rt_render into host buffers (f32 linear + sRGB u8)",
    "first_call_s": round(first_s, 4), "first_flatten_ms": st0.flatten_ms,
    "wall_ms": [round(r[0] * 1e3, 3) for r in runs], "kernel_ms": [round(r[1], 3) for r in runs],
    "render_ms": [round(r[2], 3) for r in runs],
    "msamples_per_s_host_buffers": round(best[3] / best[0] / 1e6, 2),
    "msamples_per_s_kernel": round(best[3] / (best[1] * 1e-3) / 1e6, 2),
}, indent=1))
