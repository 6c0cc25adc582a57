#!/usr/bin/env python3
"""Summarise one scripts/mem_box.sh run (TA / TD / TCP counters of the path
kernel, three --pmc passes per workload) into profiles/<round>/mem/
mem_summary.json with the derived fractions DESIGN.md §4 cites:

  TA_busy_frac          TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8)       (per-XCD GUI cycles)
  TD_busy_frac          TD_TD_BUSY_sum / (GRBM_GUI_ACTIVE / 8 x 256 CUs)
  TD_TC_stall_frac      TD_TC_STALL_sum / (same)
  TCP_pending_stall_frac TCP_PENDING_STALL_CYCLES_sum / (same)
  L1_to_L2_read_latency_cycles  TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum
  L1_hit_rate           1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum
  python scripts/mem_summary.py [round] [src]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS, XCDS = 256, 8


def main(rnd="r03", src="gpurun_out/mem"):
    src = os.path.join(ROOT, src)
    out = {}
    for w in ("c2", "c3", "c4", "c5"):
        agg = collections.defaultdict(float)
        for f in sorted(glob.glob(os.path.join(src, w + "_p*", "run_counter_collection.csv"))):
            for r in csv.DictReader(open(f)):
                if "rt_path_kernel" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]] += float(r["Counter_Value"])
        if not agg:
            continue
        c = dict(agg)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        cu_cycles = gui * CUS
        d = {}
        if gui:
            d["TA_busy_frac"] = c.get("TA_BUSY_avr", 0.0) / gui
            d["TD_busy_frac"] = c.get("TD_TD_BUSY_sum", 0.0) / cu_cycles
            d["TD_TC_stall_frac"] = c.get("TD_TC_STALL_sum", 0.0) / cu_cycles
            d["TCP_pending_stall_frac"] = c.get("TCP_PENDING_STALL_CYCLES_sum", 0.0) / cu_cycles
        if c.get("TCP_TCC_READ_REQ_sum"):
            d["L1_to_L2_read_latency_cycles"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / c["TCP_TCC_READ_REQ_sum"]
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            d["L1_hit_rate"] = 1.0 - c.get("TCP_TCC_READ_REQ_sum", 0.0) / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        out[w] = {"counters_2_launches": c, "derived": d,
                  "method": "scripts/mem_box.sh: three --pmc passes of bench.py (warmup 1 + 1 step: 2 launches); "
                            "per-XCD GRBM_GUI_ACTIVE as the cycle base; TCP/TD sums over 256 CUs"}
    dst = os.path.join(ROOT, "profiles", rnd, "mem")
    os.makedirs(dst, exist_ok=True)
    old = os.path.join(dst, "mem_summary.json")
    if os.path.exists(old):  # workloads this run did not measure keep theirs
        prev = json.load(open(old))
        out = {**{w: v for w, v in prev.items() if w not in out}, **out}
    json.dump(out, open(os.path.join(dst, "mem_summary.json"), "w"), indent=1)
    print(json.dumps({w: v["derived"] for w, v in out.items()}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
