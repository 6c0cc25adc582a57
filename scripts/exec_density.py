"""VALU exec density of the path kernel from one rocprofv3 --pmc pass
(box.sh's `density` step): SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU),
the same formula as scripts/summarize_profiles.py, averaged over the
rt_path_kernel dispatches of the run (the last one is the timed frame).
  python scripts/exec_density.py run_counter_collection.csv <workload> <variant>"""
import collections
import csv
import json
import sys


def main(path, workload, variant):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "rt_path_kernel" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        raise SystemExit("no rt_path_kernel dispatch in " + path)
    last = per[max(per, key=int)]
    dens = last["SQ_THREAD_CYCLES_VALU"] / (64.0 * last["SQ_ACTIVE_INST_VALU"])
    out = {"workload": workload, "variant": variant, "valu_exec_density": round(dens, 4),
           "valu_insts": last.get("SQ_INSTS_VALU"), "wave_cycles": last.get("SQ_WAVE_CYCLES"),
           "busy_cycles": last.get("SQ_BUSY_CYCLES"), "waves": last.get("SQ_WAVES"), "dispatches": len(per),
           "method": "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU), last rt_path_kernel dispatch"}
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:4])
