#!/usr/bin/env python3
"""Summarise a rocprofv3 PC-sampling run (host_trap / stochastic CSV):
samples per source line (the kernel built with -gline-tables-only: the
instruction comment names file:line), per instruction, and per source
region of rt_kernel.hip (REGIONS: line ranges of the path kernel's phases).
  python scripts/pcsample_summary.py <rocprofv3 output dir> [kernel substring] > summary.json
Prints the CSV header on stderr (column names differ between rocprofv3
versions: the script looks for the instruction, comment and kernel columns
by name)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def find_csv(d):
    c = [p for p in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True) if "pc_sampling" in os.path.basename(p)]
    if not c:
        raise SystemExit(f"no *pc_sampling*.csv under {d}: {glob.glob(os.path.join(d, '**', '*'), recursive=True)[:20]}")
    return sorted(c, key=os.path.getsize)[-1]


def col(header, *names):
    low = [h.lower() for h in header]
    for n in names:
        for i, h in enumerate(low):
            if n in h:
                return i
    return None


def main():
    d = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "rt_path_kernel"
    path = find_csv(d)
    with open(path, newline="") as f:
        rd = csv.reader(f)
        header = next(rd)
        print("header:", header, file=sys.stderr)
        i_ins = col(header, "instruction")
        i_com = col(header, "comment")
        i_off = col(header, "offset", "pc")
        i_ker = col(header, "kernel_name", "kernel")
        i_stall = col(header, "stall_reason", "wave_stall", "stall")
        by_line, by_ins, by_stall = collections.Counter(), collections.Counter(), collections.Counter()
        total = kept = 0
        for row in rd:
            total += 1
            if i_ker is not None and want and want not in row[i_ker]:
                continue
            kept += 1
            ins = row[i_ins] if i_ins is not None else "?"
            com = row[i_com] if i_com is not None else ""
            m = re.search(r"([\w./-]+\.(?:hip|h|hpp)):(\d+)", com)
            line = f"{os.path.basename(m.group(1))}:{m.group(2)}" if m else "?"
            by_line[line] += 1
            off = row[i_off] if i_off is not None else ""
            by_ins[(off, ins.strip(), line)] += 1
            if i_stall is not None:
                by_stall[row[i_stall]] += 1
    out = {
        "csv": os.path.relpath(path),
        "samples_total": total,
        "samples_kernel": kept,
        "top_lines": [(k, v, round(v / max(kept, 1), 4)) for k, v in by_line.most_common(80)],
        "top_instructions": [(k[0], k[1], k[2], v) for k, v in by_ins.most_common(80)],
        "stall": dict(by_stall.most_common(20)),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
