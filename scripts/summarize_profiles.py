#!/usr/bin/env python3
"""Summarise rocprofv3 output (gpurun_out/prof*) into profiles/<round>/:
kernel_stats.csv (copied), pmc_summary.json (per-launch averages of every
counter for rt_path_kernel) and pmc_c2.json (HBM bytes per launch for bench.py)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel="rt_path_kernel"):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {c: v / len(disp[c]) for c, v in agg.items()}


def main(rnd="r01", srcs=("gpurun_out/prof", "gpurun_out/prof2")):
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    counters = {}
    for src in srcs:
        for f in sorted(glob.glob(os.path.join(ROOT, src, "*", "run_counter_collection.csv"))):
            counters.update(per_launch(f))
        ks = os.path.join(ROOT, src, "trace", "run_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(dst, "kernel_stats_c2.csv"))
    out = {"kernel": "rt_path_kernel<false> (C2, 1920x1080x484 spp)", "per_launch": counters}
    c = counters
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
        out["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # rocprofv3 FETCH_SIZE / WRITE_SIZE are KiB; see MI355X_MICROARCH.md §HBM
        out["hbm_bytes_per_launch"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        out["hbm_note"] = ("FETCH_SIZE + WRITE_SIZE (KiB -> B), uncorrected: the ×2 gfx950 FETCH correction is for "
                           "16-B/lane streaming reads; the path kernel's reads are L2/MALL-resident scene gathers")
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    if "hbm_bytes_per_launch" in out:
        json.dump({"hbm_bytes_per_launch": out["hbm_bytes_per_launch"], "source": "profiles/%s/pmc_summary.json" % rnd},
                  open(os.path.join(dst, "pmc_c2.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(sys.argv[1:2] or []))
