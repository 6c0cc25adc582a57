#!/usr/bin/env python3
"""Per-launch SQ counters of rt_path_kernel from a scripts/sq_box.sh run, with
derived ratios (VALU lane utilisation, stall split, instruction mix).
  python scripts/sq_summary.py [src=gpurun_out/sq] [out.json]"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profiles import per_launch  # noqa: E402


def main(src="gpurun_out/sq", out=None):
    res = {}
    for d in sorted(glob.glob(os.path.join(src, "*_p*"))):
        if not os.path.isdir(d):
            continue
        w = os.path.basename(d).split("_")[0]
        f = os.path.join(d, "run_counter_collection.csv")
        if os.path.exists(f):
            res.setdefault(w, {}).update(per_launch(f))
    for w, c in res.items():
        der = {}
        g = c.get
        if g("SQ_ACTIVE_INST_VALU") and g("SQ_THREAD_CYCLES_VALU"):
            der["valu_lane_util"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
        if g("SQ_WAVE_CYCLES"):
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if g(k) is not None:
                    der[k + "/WAVE_CYCLES"] = g(k) / g("SQ_WAVE_CYCLES")
        if g("SQ_INSTS_VALU"):
            for k in sorted(c):
                if k.startswith("SQ_INSTS_") and k != "SQ_INSTS_VALU":
                    der[k + "/VALU"] = c[k] / g("SQ_INSTS_VALU")
        if g("SQ_WAVES") and g("SQ_INSTS_VALU"):
            der["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
        c["derived"] = der
    s = json.dumps(res, indent=1)
    print(s)
    if out:
        open(out, "w").write(s)


if __name__ == "__main__":
    main(*sys.argv[1:])
