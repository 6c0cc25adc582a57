#!/usr/bin/env python3
"""Diagnostic run (GPU box): renders C2 with librt_mi355x_diag.so (in-kernel
s_memtime stamps + lane work counters, -DRT_DIAG) and prints where the wave
cycles go and how full the lanes are in the traversal loop.  Read the shares,
not the absolute time (stamps cost cycles)."""
import ctypes
import importlib
import json
import os
import sys

import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")

torch.cuda.init()
lib = ctypes.CDLL(os.path.join(ROOT, "raytracer-2025_amd", os.environ.get("DIAG_LIB", "librt_mi355x_diag.so")))
api = capi.Api(lib, "rt_")
lib.rt_diag_counters.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
scene = rt.Scene(api)
wl = os.environ.get("AB_WORKLOAD", "c2")
if wl == "c4":
    import tempfile
    obj = os.path.join(tempfile.gettempdir(), "rt_terrain_707", "terrain.obj")
    if not os.path.exists(obj):
        scenes.write_terrain_obj(os.path.dirname(obj), 707)
    world, lights, cam = scenes.obj_terrain(scene, obj, 1920, spp)
elif wl == "c3":
    world, lights, cam = scenes.cornell_smoke(scene, 800, spp)
elif wl == "c5":
    world, lights, cam = scenes.final_scene(scene, 1920, spp, 40, aspect_ratio=16 / 9)
else:
    world, lights, cam = scenes.random_spheres(scene, 1920, spp)
cam.render(world, lights, seed=1, want_srgb=False)  # warm-up + flatten
buf = (ctypes.c_ulonglong * 61)()
lib.rt_diag_counters(buf, 1)
_, _, st = cam.render(world, lights, seed=1, want_srgb=False)
lib.rt_diag_counters(buf, 0)
c = list(buf)
tot = c[0] + c[1] + c[2]
out = {
    "workload": wl, "spp": spp,
    "kernel_ms": st.kernel_ms,
    "samples": st.samples,
    "rays": st.rays,
    "cycle_share": {"refill+camera": c[0] / tot, "trace": c[1] / tot, "shade": c[2] / tot,
                    "of which media_phase (full tiers)": c[13] / tot},
    "trace_lane_efficiency": c[5] / (64.0 * c[3]) if c[3] else None,
    "trace_iters_per_ray": c[5] / c[8],
    "wave_trace_iters_per_wave_bounce": c[3] / max(1, c[4]),
    "node_visits_per_ray": c[6] / c[8],
    "primitive_tests_per_ray": c[7] / c[8],
    "node_load_wave_cycles": c[9] / c[10] if c[10] else None,
    "stack_reads_per_pop": c[12] / c[11] if c[11] else None,
    "pops_per_ray": c[11] / c[8],
    "big_sphere_exact_tests_per_ray": c[14] / c[8],  # basic tier: spheres with r > 100 (C2's ground)
    "big_sphere_exact_hits_per_ray": c[15] / c[8],
    # mesh / full tiers: unified walk-step loads -- wave steps whose active
    # lanes all read one record (a scalar load could serve them), of them node
    # records, and the mean share of active lanes on the first lane's record
    "uniform_step_share": c[17] / c[16] if c[16] else None,
    "uniform_node_step_share": c[18] / c[16] if c[16] else None,
    "lanes_on_first_record": c[20] / c[19] if c[19] else None,
    "active_lanes_per_step": c[19] / c[16] if c[16] else None,
    # basic / mesh tiers' unified loop: shares of all wave cycles after the
    # walk -- a miss's sky and the sample's end, the queue refill, the
    # iteration's Philox block and sincos (the rest of refill+camera: the
    # walk set-up and the camera rays)
    "after_walk_share": {"miss+finish": c[21] / tot, "queue_refill": c[22] / tot, "draws": c[23] / tot},
    # mesh / full tiers: wave steps whose active lanes all read nodes among the
    # top 5 / 21 / 85 / 341 (levels 0-1 / 0-2 / 0-3 / 0-4 of a full 4-wide
    # tree: rth::bvh4_convert numbers them first), and the share of all node
    # reads that are of those nodes (lane count)
    "top_uniform_step_share": {str(k): (c[24 + i] / c[16] if c[16] else None) for i, k in enumerate((5, 21, 85, 341))},
    "top_node_read_share": {str(k): (c[28 + i] / c[32] if c[32] else None) for i, k in enumerate((5, 21, 85, 341))},
    # full tiers: shading rounds -- lanes per round and distinct shading
    # classes per round (miss, Lambertian x texture kind, Metal, Dielectric,
    # light, Isotropic, other): the branches a round runs one after another,
    # the same whatever the order of the round's lanes
    "shade_lanes_per_round": c[34] / c[33] if c[33] else None,
    "shade_classes_per_round": c[35] / c[33] if c[33] else None,
    # basic tier: wave iterations in which no lane can walk a node (pure
    # sphere rounds: share of the walk's wave iterations), the lanes with a
    # queued sphere in them, and the most any lane still had queued
    "pure_sphere_round_share": c[36] / c[3] if c[3] else None,
    "pure_round_lanes": c[37] / c[36] if c[36] else None,
    "pure_round_max_queued": c[38] / c[36] if c[36] else None,
    # ... per class: the share of shading rounds it is present in, and its
    # lanes per round when present
    "shade_class_presence": {name: {"rounds_share": (c[39 + k] / c[33]) if c[33] else None,
                                    "lanes_when_present": (c[50 + k] / c[39 + k]) if c[39 + k] else None}
                             for k, name in enumerate(("miss", "lambertian_solid", "lambertian_checker",
                                                       "lambertian_image", "lambertian_noise", "lambertian_sky",
                                                       "metal", "dielectric", "diffuse_light", "isotropic", "other"))},
    "raw": c[:61],
}
print(json.dumps(out, indent=1))
