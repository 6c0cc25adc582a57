#!/usr/bin/env python3
"""Summarises rocprofv3 PC-sampling CSVs (scripts/pcs_box.sh): the columns,
then sample counts per instruction (code-object offset + text + source line
where the CSV has them) and per stall / issue reason, for the path kernel.
Usage: python scripts/pcs_summary.py <rocprofv3 output dir> [top N]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 120
files = [f for f in glob.glob(os.path.join(root, "**", "*.csv"), recursive=True) if "pc_sampl" in os.path.basename(f)]
print("files:", files)
for f in files:
    with open(f, newline="") as fh:
        rd = csv.DictReader(fh)
        cols = rd.fieldnames or []
        print("columns:", cols)
        rows = list(rd)
    print("samples:", len(rows))
    if not rows:
        continue
    for r in rows[:3]:
        print("row:", r)

    def pick(*names):
        for n in names:
            for c in cols:
                if c.lower() == n.lower():
                    return c
        for n in names:
            for c in cols:
                if n.lower() in c.lower():
                    return c
        return None
    c_off = pick("Code_Object_Offset", "Offset", "Pc")
    c_ins = pick("Instruction")
    c_cmt = pick("Instruction_Comment", "Comment")
    c_kern = pick("Kernel_Name", "Kernel")
    c_stall = pick("Snapshot_Stall_Reason", "Stall_Reason")
    c_issued = pick("Wave_Issued", "Issued")
    c_type = pick("Inst_Type", "Instruction_Type")
    if c_kern:
        kinds = collections.Counter(r[c_kern][:60] for r in rows)
        print("by kernel:", kinds.most_common(8))
        rows = [r for r in rows if "rt_path_kernel" in r[c_kern]] or rows
    n = len(rows)
    key = lambda r: (r.get(c_off, ""), r.get(c_ins, ""), (r.get(c_cmt, "") or "")[-60:])
    cnt = collections.Counter(key(r) for r in rows)
    print(f"\n== path-kernel samples: {n}; top {top} instructions (share, offset, instruction, source)")
    for (off, ins, cmt), k in cnt.most_common(top):
        print(f"{k / n:7.4f} {off:>10} {ins[:60]:60} {cmt}")
    for c in (c_stall, c_issued, c_type):
        if c:
            print(f"\n== by {c}")
            for v, k in collections.Counter(r[c] for r in rows).most_common(20):
                print(f"{k / n:7.4f} {v}")
    if c_cmt:
        print("\n== by source line")
        for v, k in collections.Counter((r[c_cmt] or "")[-70:] for r in rows).most_common(60):
            print(f"{k / n:7.4f} {v}")
