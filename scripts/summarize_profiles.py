#!/usr/bin/env python3
"""Summarise one scripts/bench_box.sh run (gpurun_out/box/) into
profiles/<round>/:

  kernel_stats_<w>.csv   rocprofv3 --kernel-trace --stats summary (copied)
  pmc_<w>.json           HBM bytes per launch of rt_path_kernel, for bench.py
  pmc_summary.json       per-launch counters of every workload + derived values
  bench_<w>.json         the bench line of that run

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE (KiB) come
from separate --pmc passes; FETCH_SIZE is doubled (gfx950 tallies 128-B read
requests at 64 B), WRITE_SIZE is taken as is.
  python scripts/summarize_profiles.py [round] [src]"""
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


def kernel_avg_ns(stats_csv, kernel="rt_path_kernel"):
    for r in csv.DictReader(open(stats_csv)):
        if kernel in r["Name"]:
            return float(r["AverageNs"]), r["Name"], int(r["Calls"])
    return None, None, 0


def main(rnd="r01", src="gpurun_out/box"):
    src = os.path.join(ROOT, src)
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    old = os.path.join(dst, "pmc_summary.json")
    summary = json.load(open(old)) if os.path.exists(old) else {}  # workloads this run did not profile keep theirs
    for w in ("c2", "c3", "c4", "c5"):
        entry = {}
        ks = os.path.join(src, "trace_" + w, "run_kernel_stats.csv")
        if os.path.exists(ks):
            shutil.copy(ks, os.path.join(dst, "kernel_stats_%s.csv" % w))
            ns, name, calls = kernel_avg_ns(ks)
            entry.update({"kernel": name, "calls": calls, "avg_ms": ns / 1e6 if ns else None})
        counters = {}
        for f in sorted(glob.glob(os.path.join(src, "*_" + w, "run_counter_collection.csv"))):
            counters.update(per_launch(f))
        entry["per_launch"] = counters
        if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
            fetch = 2.0 * counters["FETCH_SIZE"] * 1024.0
            write = counters["WRITE_SIZE"] * 1024.0
            entry["hbm_read_bytes_per_launch"] = fetch
            entry["hbm_write_bytes_per_launch"] = write
            entry["hbm_bytes_per_launch"] = fetch + write
            json.dump({"hbm_bytes_per_launch": fetch + write, "read": fetch, "write": write,
                       "method": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), separate --pmc passes, MI355X_MICROARCH.md §HBM",
                       "source": "profiles/%s/pmc_summary.json" % rnd},
                      open(os.path.join(dst, "pmc_%s.json" % w), "w"), indent=1)
        bl = os.path.join(src, "bench_%s.log" % w)
        if os.path.exists(bl):
            lines = [l for l in open(bl) if l.startswith("{")]
            if lines:
                line = json.loads(lines[-1])
                # bench.py read the traffic of the previous pmc_<w>.json (its
                # run precedes this job's --pmc passes); the same job's passes
                # measured this code, so their per-launch bytes replace it
                if "hbm_bytes_per_launch" in entry and "roofline" in line:
                    line["roofline"]["traffic"] = entry["hbm_bytes_per_launch"]
                open(os.path.join(dst, "bench_%s.json" % w), "w").write(json.dumps(line) + "\n")
        if entry.get("per_launch") or "kernel" in entry or w not in summary:
            summary[w] = entry
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
