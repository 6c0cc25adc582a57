#!/usr/bin/env python3
"""Interleaved A/B of run-time queue settings (GPU box): per repetition and
setting, the whole frame and the 8 row shards of an 8-GPU run (rows r, r + 8,
...) rendered alone, in one process, settings interleaved so that clock drift
hits them alike.  A setting is VAR=val,VAR2=val (environment variables read by
every render, e.g. RT_TAIL_PERMILLE=250).
  python scripts/tail_ab.py workload spp reps setting [setting ...]
Prints per setting the frame's kernel ms (min, median) and the worst shard's
(min over reps of the per-rep worst), and the 8-GPU kernel efficiency
full / (8 x worst shard) from the minima.
TAIL_ORDER=rev renders the shards 7 .. 0 (shards_ms stays indexed by shard);
TAIL_WARM=1 renders one untimed shard first, so that no timed shard follows
the whole frame directly (a rank of an 8-GPU run renders only its shard)."""
import importlib
import json
import os
import statistics
import sys

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
    s = rt.Scene(api)
    world, lights, cam, desc = bench.build_workload(scenes, s, wl, bench.WORKLOADS[wl][0], spp)
    cam.render(world, lights, seed=1, want_srgb=False)  # flatten + upload
    base_env = dict(os.environ)
    res = {k: {"full": [], "worst8": [], "sum8": []} for k in settings}
    ref = None
    for rep in range(reps):
        for k in settings:
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(dict(kv.split("=", 1) for kv in k.split(",") if kv))
            lin, _, st = cam.render(world, lights, seed=1, want_srgb=False)
            if ref is None:
                ref = lin
            rel = float(abs(lin.astype("float64") - ref).max())  # settings may change f64 sum order: ~1 ulp
            res[k]["full"].append(st.kernel_ms)
            shards = [0.0] * 8
            if os.environ.get("TAIL_WARM") == "1":
                cam.render(world, lights, seed=1, row_offset=7, row_stride=8, want_srgb=False)
            order = range(7, -1, -1) if os.environ.get("TAIL_ORDER") == "rev" else range(8)
            for r in order:
                _, _, st8 = cam.render(world, lights, seed=1, row_offset=r, row_stride=8, want_srgb=False)
                shards[r] = st8.kernel_ms
            worst = max(shards)
            res[k]["worst8"].append(worst)
            res[k]["sum8"].append(sum(shards))
            print(json.dumps({"rep": rep, "setting": k, "full_ms": round(st.kernel_ms, 3),
                              "worst8_ms": round(worst, 3), "shards_ms": [round(x, 3) for x in shards],
                              "max_abs_vs_first": rel}), flush=True)
    os.environ.clear()
    os.environ.update(base_env)
    out = {}
    for k, v in res.items():
        out[k] = {"full_min": min(v["full"]), "full_median": statistics.median(v["full"]),
                  "worst8_min": min(v["worst8"]), "worst8_median": statistics.median(v["worst8"]),
                  "eff8": min(v["full"]) / (8 * min(v["worst8"])),
                  # the shards' summed kernel time against the frame's: < 1
                  # when a shard's samples cost more than the frame's (cache
                  # locality, launch ramp and drain), apart from imbalance
                  "sum8_over_full": min(v["sum8"]) / min(v["full"])}
    print(json.dumps({"workload": desc, "spp": spp, "reps": reps, "settings": out}))


if __name__ == "__main__":
    main()
