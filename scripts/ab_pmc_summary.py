#!/usr/bin/env python3
"""Per-variant counters of rt_path_kernel from scripts/ab_pmc.sh: ab.py
dispatches one warm-up render per variant, then one timed render per variant
in the same order; the timed ones are reported."""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abpmc"
names = open(os.path.join(src, "variants.txt")).read().split()
res = {n: {} for n in names}
for f in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "rt_path_kernel" in r["Kernel_Name"]:
            d = per[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    timed = ids[len(names):2 * len(names)]
    for n, i in zip(names, timed):
        res[n].update(per[i])
for n, c in res.items():
    g = c.get
    if g("SQ_WAVE_CYCLES"):
        c["valu_busy_per_simd"] = 4 * g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")
        c["valu_lane_util"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
        c["quad_cycles_per_valu"] = g("SQ_ACTIVE_INST_VALU") / g("SQ_INSTS_VALU")
print(json.dumps(res, indent=1))
