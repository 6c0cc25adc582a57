#!/usr/bin/env python3
"""Summarise one scripts/prof_box.sh run (gpurun_out/prof/) into
profiles/<round>/:

  kernel_stats_<w>.csv   rocprofv3 --kernel-trace --stats summary (copied)
  pmc_<w>.json           HBM bytes of rt_path_kernel per launch and per traced sample, for bench.py
  valu_<w>.json          executed VALU work per traced sample, for bench.py's frac_executed
  pmc_summary.json       per-launch counters of every workload + derived values
  bench_<w>.json         the bench line of that run

Read bytes (MI355X_MICROARCH.md §HBM): FETCH_SIZE tallies a 128-B fabric read
request at 64 B, and its x2 correction is calibrated only for wide coalesced
16-B/lane streams -- not this kernel's pointer chase.  So reads are counted
from the request counters by size instead: 32 x TCC_EA0_RDREQ_32B + 64 x
TCC_EA0_RDREQ_64B + 128 x TCC_EA0_RDREQ_128B (one --pmc pass; the three sum
to TCC_EA0_RDREQ, checked), and 2 x FETCH_SIZE is kept beside it for
comparison.  Writes: WRITE_SIZE (exact for 16-B streaming stores).  Like
FETCH_SIZE these count L2 -> fabric requests, Infinity-Cache hits included.

Executed VALU work: SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 count wave
instructions; x 64 lanes x the exec density SQ_THREAD_CYCLES_VALU /
(64 x SQ_ACTIVE_INST_VALU) (the VALUUtilization formula, over all VALU) and
FMA x 2 gives executed f64 FLOPs.
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


def bench_line(path):
    try:
        lines = [l for l in open(path) if l.startswith("{")]
    except OSError:
        return None
    return json.loads(lines[-1]) if lines else None


def main(rnd="r02", src="gpurun_out/prof"):
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
            tl = bench_line(os.path.join(src, "trace_%s.log" % w))
            if tl:
                entry["launch_samples"] = tl["config"]["frame_samples"]
                entry["profiled_config"] = tl["config"]["workload"]
                entry["bench_kernel_ms_avg_same_run"] = tl["roofline"]["kernel_ms_avg"]
        counters = {}
        for f in sorted(glob.glob(os.path.join(src, "*_" + w, "run_counter_collection.csv"))):
            counters.update(per_launch(f))
        if not counters and "kernel" not in entry:
            continue
        entry["per_launch"] = counters
        n = entry.get("launch_samples")
        c = counters
        if "FETCH_SIZE" in c:
            entry["fetch_size_x2_bytes_per_launch"] = 2.0 * c["FETCH_SIZE"] * 1024.0
        if "TCC_EA0_RDREQ_32B_sum" in c:
            n32, n64, n128 = c["TCC_EA0_RDREQ_32B_sum"], c["TCC_EA0_RDREQ_64B_sum"], c["TCC_EA0_RDREQ_128B_sum"]
            entry["read_requests"] = {"32B": n32, "64B": n64, "128B": n128, "all": c.get("TCC_EA0_RDREQ_sum")}
            entry["hbm_read_bytes_per_launch"] = 32.0 * n32 + 64.0 * n64 + 128.0 * n128
        if "WRITE_SIZE" in c:
            entry["hbm_write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024.0
        if "hbm_read_bytes_per_launch" in entry and "hbm_write_bytes_per_launch" in entry:
            tot = entry["hbm_read_bytes_per_launch"] + entry["hbm_write_bytes_per_launch"]
            entry["hbm_bytes_per_launch"] = tot
            rec = {"hbm_bytes_per_launch": tot, "read": entry["hbm_read_bytes_per_launch"],
                   "write": entry["hbm_write_bytes_per_launch"],
                   "fetch_size_x2_read": entry.get("fetch_size_x2_bytes_per_launch"),
                   "method": "reads: 32/64/128 x TCC_EA0_RDREQ_{32B,64B,128B}; writes: WRITE_SIZE (KiB -> B); "
                             "separate --pmc passes (MI355X_MICROARCH.md §HBM)",
                   "launch_samples": n, "source": "profiles/%s/pmc_summary.json" % rnd}
            if n:
                rec["hbm_bytes_per_sample"] = tot / n
            json.dump(rec, open(os.path.join(dst, "pmc_%s.json" % w), "w"), indent=1)
        if "SQ_INSTS_VALU_FMA_F64" in c and c.get("SQ_ACTIVE_INST_VALU"):
            dens = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
            f64_inst = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_TRANS_F64"] + \
                2.0 * c["SQ_INSTS_VALU_FMA_F64"]
            flops64 = f64_inst * 64.0 * dens
            rec = {"valu_exec_density": dens, "executed_f64_flops_per_launch": flops64,
                   "valu_insts_per_launch": c.get("SQ_INSTS_VALU"), "salu_insts_per_launch": c.get("SQ_INSTS_SALU"),
                   "launch_samples": n,
                   "method": "(ADD+MUL+TRANS+2 FMA)_F64 wave instructions x 64 x exec density "
                             "SQ_THREAD_CYCLES_VALU/(64 SQ_ACTIVE_INST_VALU)", "source": "profiles/%s/pmc_summary.json" % rnd}
            if "SQ_INSTS_VALU_FMA_F32" in c:
                f32_inst = c["SQ_INSTS_VALU_ADD_F32"] + c["SQ_INSTS_VALU_MUL_F32"] + c["SQ_INSTS_VALU_TRANS_F32"] + \
                    2.0 * c["SQ_INSTS_VALU_FMA_F32"]
                rec["executed_f32_flops_per_launch"] = f32_inst * 64.0 * dens
            if n:
                rec["executed_f64_flops_per_sample"] = flops64 / n
                if "executed_f32_flops_per_launch" in rec:
                    rec["executed_f32_flops_per_sample"] = rec["executed_f32_flops_per_launch"] / n
            if entry.get("avg_ms"):
                rec["executed_f64_tflops"] = flops64 / (entry["avg_ms"] * 1e-3) / 1e12
                if "executed_f32_flops_per_launch" in rec:
                    rec["executed_f32_tflops"] = rec["executed_f32_flops_per_launch"] / (entry["avg_ms"] * 1e-3) / 1e12
            entry["valu"] = rec
            json.dump(rec, open(os.path.join(dst, "valu_%s.json" % w), "w"), indent=1)
        line = bench_line(os.path.join(src, "bench_%s.log" % w))
        if line:
            open(os.path.join(dst, "bench_%s.json" % w), "w").write(json.dumps(line) + "\n")
        summary[w] = entry
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
