#!/usr/bin/env python3
"""Interleaved A/B of kernel variants (raytracer-2025_amd/librt_ab_*.so, built
by `make -C raytracer-2025_amd ab`) in one process on the C2 scene: each
variant renders the same frame; path-kernel time from the library's HIP
events.  Usage: python scripts/ab.py [spp] [reps] [variant ...]; a variant is a library
name (librt_ab_<name>.so) optionally followed by @VAR=val,... (environment
variables set while its world is flattened and its frames render, e.g.
base@RT_PART_SAMPLES=2).
AB_WORKLOAD=c3|c4|c5 renders that config's scene (C5 at 1920 wide) instead of C2."""
import ctypes
import glob
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
names = sys.argv[3:] or sorted(os.path.basename(p)[len("librt_ab_"):-3]
                                for p in glob.glob(os.path.join(ROOT, "raytracer-2025_amd", "librt_ab_*.so")))
torch.cuda.init()
runs = {}
libs = {}
for n in names:
    # "lib@VAR=val,VAR2=val": librt_ab_<lib>.so with those environment
    # variables set while its world is flattened (the first render)
    lib, _, envs = n.partition("@")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    if lib not in libs:
        libs[lib] = capi.Api(ctypes.CDLL(os.path.join(ROOT, "raytracer-2025_amd", f"librt_ab_{lib}.so")), "rt_")
    api = libs[lib]
    scene = rt.Scene(api)
    wl = os.environ.get("AB_WORKLOAD", "c2")
    if wl == "c3":
        world, lights, cam = scenes.cornell_smoke(scene, 800, spp)
    elif wl == "c5":
        world, lights, cam = scenes.final_scene(scene, 1920, spp, 40, aspect_ratio=16 / 9)
    elif wl == "c4":
        import tempfile
        obj = os.path.join(tempfile.gettempdir(), "rt_terrain_707", "terrain.obj")
        if not os.path.exists(obj):
            scenes.write_terrain_obj(os.path.dirname(obj), 707)
        world, lights, cam = scenes.obj_terrain(scene, obj, 1920, spp)
    else:
        world, lights, cam = scenes.random_spheres(scene, 1920, spp)
    print("warm-up", n, file=sys.stderr, flush=True)
    lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)  # warm-up
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    runs[n] = (scene, world, lights, cam, lin)
res = {n: [] for n in names}
for _ in range(reps):
    for n in names:
        scene, world, lights, cam, ref = runs[n]
        env = dict(kv.split("=", 1) for kv in n.partition("@")[2].split(",") if kv)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)  # (knobs read per render, e.g. RT_PART_SAMPLES)
        lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        res[n].append(st.kernel_ms)
        print(n, st.kernel_ms, file=sys.stderr, flush=True)
base = runs[names[0]][4]
out = {}
for n in names:
    d = (runs[n][4].astype("float64") - base).reshape(-1, 3)
    out[n] = {"kernel_ms_min": min(res[n]), "kernel_ms": res[n], "rmse_vs_first": float((d ** 2).mean() ** 0.5),
              "msamples_per_s": cam.traced_samples() / (min(res[n]) * 1e-3) / 1e6}
print(json.dumps(out, indent=1))
