#!/usr/bin/env python3
"""Whole-frame parity at a BASELINE config (GPU box): the workload rendered
by the library on the GPU and by the TEST-ONLY oracle (oracle/, the
reference-semantics C++ restatement) on the box's host threads, same scene
script, camera and render seed; prints per-channel RMSE of the linear f32
frames, the largest absolute difference, and the fractions of pixels that are
bit-equal / within 1e-5 relative.  The GPU parity tests check rows of the
full-size configs; this checks every pixel of a whole frame.
  python scripts/full_frame_parity.py c2 [spp]"""
import ctypes
import importlib
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
capi = importlib.import_module("raytracer-2025_amd.capi")
pkg = importlib.import_module("raytracer-2025_amd")


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else bench.WORKLOADS[wl][1]
    threads, _ = bench.usable_cpus()
    so = os.path.join(ROOT, "oracle", "_build", "liboracle_fast.so")  # the timed build: the same bits as liboracle.so (tests/test_oracle_golden.py), faster
    if not os.path.exists(so):
        subprocess.run(["make", "-j", "8", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    torch.cuda.init()
    out = {}
    for name, api in (("gpu", pkg.load()), ("oracle", capi.Api(ctypes.CDLL(so), "orc_", capi.ORACLE_EXTRAS))):
        s = rt.Scene(api)
        world, lights, cam, desc = bench.build_workload(scenes, s, wl, bench.WORKLOADS[wl][0], spp)
        t0 = time.perf_counter()
        if name == "gpu":
            lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)
            samples, panics = int(st.samples), int(st.panics)
        else:  # eight row shards (rows k, k + 8, ...: the same keys), a progress line each
            lin = np.zeros((cam.image_height, cam.image_width, 3), np.float32)
            samples = panics = 0
            for k in range(8):
                part, _, st = cam.render(world, lights, seed=1, row_offset=k, row_stride=8, threads=threads,
                                         want_srgb=False)
                lin[k::8] = part
                samples += int(st.samples)
                panics += int(st.panics)
                print(json.dumps({"oracle_shard": k, "seconds": round(time.perf_counter() - t0, 1)}), flush=True)
        out[name] = (lin.astype(np.float64), time.perf_counter() - t0, samples, panics)
        print(json.dumps({"side": name, "seconds": round(out[name][1], 2), "samples": out[name][2],
                          "panics": out[name][3]}), flush=True)
    g, o = out["gpu"][0], out["oracle"][0]
    d = g - o
    rel = np.abs(d) / np.maximum(np.abs(o), 1e-30)
    res = {
        "workload": desc, "spp": spp, "size": list(g.shape[:2]), "oracle_threads": threads,
        "rmse_per_channel": np.sqrt((d ** 2).mean(axis=(0, 1))).tolist(),
        "max_abs_diff": float(np.abs(d).max()),
        "pixels_bit_equal": float(np.all(d == 0, axis=-1).mean()),
        "pixels_within_1e-5_rel": float(np.all(rel <= 1e-5, axis=-1).mean()),
        "gpu_s": round(out["gpu"][1], 3), "oracle_s": round(out["oracle"][1], 1),
        "panics": [out["gpu"][3], out["oracle"][3]],
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
