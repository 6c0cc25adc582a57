#!/usr/bin/env python3
"""Host-side scene setup time of the C4 workload (no GPU needed): the
1M-triangle OBJ's load (Wavefont::new: parse + one reference BVH per model)
and the flatten the first render does (rt_world_info_get runs the same
flatten and tier preparation), two repetitions each.
  python scripts/setup_time_box.py"""
import ctypes
import importlib
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
capi = importlib.import_module("raytracer-2025_amd.capi")
pkg = importlib.import_module("raytracer-2025_amd")


def main():
    api = pkg.load()
    obj = os.path.join(tempfile.gettempdir(), "rt_terrain_707", "terrain.obj")
    if not os.path.exists(obj):
        scenes.write_terrain_obj(os.path.dirname(obj), 707)
    reps = []
    for _ in range(2):
        s = rt.Scene(api)
        t0 = time.perf_counter()
        world, _, cam = scenes.obj_terrain(s, obj, 1920, 256)
        t1 = time.perf_counter()
        info = capi.RtWorldInfo()
        api.check(api.world_info_get(s.s, world.h, -1, cam.background.h, 0, ctypes.byref(info)))
        t2 = time.perf_counter()
        reps.append({"load_s": round(t1 - t0, 2), "flatten_s": round(t2 - t1, 2)})
        del s
    print(json.dumps({"workload": "C4 terrain OBJ (999 698 triangles)", "host_cpus": len(os.sched_getaffinity(0)),
                      "reps": reps}))


if __name__ == "__main__":
    main()
