#!/usr/bin/env python3
"""Static ISA attribution of the basic tier's path kernel (C2) by phase.

Compiles csrc/rt_kernel.hip for tier 0 as the product does (gfx950, -O3, no
contraction, machine LICM off) with -DRT_ISA_MARKS -- an assembler comment at
each phase boundary of the loop (RT_ISA_MARK: fields, walk / walk_visit /
walk_sphere / walk_tail, park, miss, refill, draws, shade, camera) -- and
counts the instructions of rt_path_kernel<0, false> after each marker, in
layout order, by class: VALU (f64 / f32 / integer+other), SALU, vector
memory, LDS, scalar memory, branches, waits.  It also compiles the unmarked
kernel and reports both totals (the markers' effect on code generation).
A static count is the code of a phase, once; how often each runs is the
diagnostic build's business (scripts/diag.py).
  python scripts/isa_phases.py > profiles/r06/isa_phases_c2.json"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raytracer-2025_amd", "csrc", "rt_kernel.hip")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics",
         "-mllvm", "-disable-machine-licm", "-DRT_TIER_ONLY=0", "--offload-device-only", "-S"]
KERNEL = "_ZN3rtk14rt_path_kernelILi0ELb0EEEvPKNS_7KParamsE"


def asm(extra):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-o", out, SRC], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        text = open(out).read()
    start = text.index(KERNEL + ":")
    end = text.index(".Lfunc_end", start)
    return text[start:end].splitlines()


def klass(op):
    if op.startswith(("v_cmp", "v_cndmask")) or op.startswith("v_") and op.endswith(("_f64", "_f64_e32", "_f64_e64")) is False:
        pass
    if op.startswith("v_"):
        if "_f64" in op:
            return "valu_f64"
        if "_f32" in op or "_f16" in op:
            return "valu_f32"
        return "valu_int_other"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def count(lines):
    phases = collections.OrderedDict()
    cur = "entry"
    total = 0
    for ln in lines:
        m = re.search(r";@@phase (\w+)", ln)
        if m:
            cur = m.group(1)
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        c = phases.setdefault(cur, collections.Counter())
        c[klass(op)] += 1
        c["all"] += 1
        total += 1
    return phases, total


def main():
    marked, total_m = count(asm(["-DRT_ISA_MARKS"]))
    _, total_p = count(asm([]))
    out = {
        "kernel": "rt_path_kernel<0, false> (basic tier, 56-lane shading batches: C1 / C2)",
        "method": "static instruction counts in layout order after each RT_ISA_MARK comment (-DRT_ISA_MARKS); "
                  "a phase's count is its code once, not how often it runs",
        "total_instructions_marked_build": total_m,
        "total_instructions_product_build": total_p,
        "phases": {k: dict(v) for k, v in marked.items()},
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
