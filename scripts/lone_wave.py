#!/usr/bin/env python3
"""Latency of a lone wave (GPU box, lane-trace build): a tiny C2 frame -- a
few pixels, so only a few lanes of the grid get work -- and, per busy lane,
walk steps, rays and wall time: the per-step time of a wave that runs with
the rest of the GPU idle (the end of every launch).
  python scripts/lone_wave.py [width] [spp]"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")

W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(ROOT, "raytracer-2025_amd", "librt_mi355x_trace.so"))
lib.rt_lane_trace.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_uint64]
api = capi.Api(lib, "rt_")
s = rt.Scene(api)
world, lights, cam = scenes.random_spheres(s, W, spp)
cam.render(world, lights, seed=1, want_srgb=False)
n = 1 << 19
buf = (ctypes.c_ulonglong * (n * 10))()
for rep in range(3):
    ctypes.memset(buf, 0, ctypes.sizeof(buf))
    _, _, st = cam.render(world, lights, seed=1 + rep, want_srgb=False)
    assert lib.rt_lane_trace(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 10).astype(np.int64)
    live = a[a[:, 1] > 0]
    t0 = live[:, 0].min()
    busy = live[live[:, 3] > 0]
    idle = live[live[:, 3] == 0]
    life = (busy[:, 1] - busy[:, 0]) / 100.0
    steps = busy[:, 8]
    print(json.dumps({"width": W, "height": cam.image_height, "spp": spp, "kernel_ms": round(st.kernel_ms, 4),
                      "busy_lanes": int(len(busy)), "rays": int(busy[:, 3].sum()), "steps": int(steps.sum()),
                      "us_per_step_max_lane": round(float(life[np.argmax(steps)] / max(1, steps.max())), 3),
                      "max_steps": int(steps.max()), "max_life_us": round(float(life.max()), 1),
                      "memtime_mhz": round(float(busy[np.argmax(steps), 7] / max(1e-9, life[np.argmax(steps)])), 1),
                      # lanes without work: they start, take a queue entry past the end (one
                      # atomicAdd by their wave) and exit -- when, relative to the first start
                      "idle_start_us_pct": {p: round(float(np.percentile((idle[:, 0] - t0) / 100.0, p)), 1) for p in (0, 50, 100)},
                      "idle_exit_us_pct": {p: round(float(np.percentile((idle[:, 1] - t0) / 100.0, p)), 1)
                                           for p in (0, 10, 50, 90, 100)}}))
