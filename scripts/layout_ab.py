#!/usr/bin/env python3
"""Interleaved A/B of flatten-time settings (GPU box): one scene per setting,
each built and flattened with that setting's environment (e.g.
RT_BVH4_LAYOUT=1: the node / primitive layout, read when the world is
flattened), then rendered in turn, settings interleaved per repetition so
that clock drift hits them alike.  Checks that every setting renders the
first one's frame bit for bit.
  python scripts/layout_ab.py workload spp reps setting [setting ...]"""
import importlib
import json
import os
import statistics
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
pkg = importlib.import_module("raytracer-2025_amd")
import bench  # noqa: E402  (the workloads)


def main():
    wl, spp, reps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    spp = bench.WORKLOADS[wl][1] if spp == "-" else int(spp)
    settings = sys.argv[4:] or [""]
    api = pkg.load()
    torch.cuda.init()
    base_env = dict(os.environ)
    runs = {}
    for k in settings:
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(dict(kv.split("=", 1) for kv in k.split(",") if kv))
        s = rt.Scene(api)
        world, lights, cam, desc = bench.build_workload(scenes, s, wl, bench.WORKLOADS[wl][0], spp)
        lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)  # flatten + upload under k
        runs[k] = (s, world, lights, cam, lin)
        print(json.dumps({"setting": k, "flatten_ms": round(st.flatten_ms, 1)}), flush=True)
    os.environ.clear()
    os.environ.update(base_env)
    ref = runs[settings[0]][4]
    res = {k: [] for k in settings}
    for rep in range(reps):
        for k in settings:
            _, world, lights, cam, _ = runs[k]
            lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)
            res[k].append(st.kernel_ms)
            print(json.dumps({"rep": rep, "setting": k, "kernel_ms": round(st.kernel_ms, 3),
                              "bit_equal": bool(np.array_equal(lin, ref))}), flush=True)
    out = {k: {"min": min(v), "median": statistics.median(v)} for k, v in res.items()}
    print(json.dumps({"workload": desc, "spp": spp, "reps": reps, "settings": out}))


if __name__ == "__main__":
    main()
