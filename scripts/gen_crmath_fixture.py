#!/usr/bin/env python3
"""Writes tests/golden/crmath_args.npz: per function family the arguments
the path feeds it, glibc's results and the correctly rounded results
(tests/cpp/crmath_fixture.cpp, libquadmath).  tests/test_crmath_gpu.py checks
the device functions against it on the GPU box, which then needs neither the
compiler nor libquadmath.

    python scripts/gen_crmath_fixture.py [n_per_family]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["sin_2pi_xi", "cos_2pi_xi", "sin_noise", "cos_noise", "log_xi", "acos_uv", "atan2_uv", "sqrt", "sincos_sin"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    build = os.path.join(ROOT, "tests", "_build")
    os.makedirs(build, exist_ok=True)
    exe = os.path.join(build, "crmath_fixture")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", os.path.join(ROOT, "tests", "cpp", "crmath_fixture.cpp"),
                    "-lquadmath", "-lm", "-o", exe], check=True)
    raw = np.frombuffer(subprocess.run([exe, str(n)], check=True, capture_output=True).stdout, dtype="<f8")
    out, pos = {}, 0
    for name in NAMES:
        fn, m = int(raw[pos]), int(raw[pos + 1])
        pos += 2
        a, b, g, c = (raw[pos + k * m:pos + (k + 1) * m] for k in range(4))
        pos += 4 * m
        out[name + "_fn"] = np.array(fn)
        out[name + "_a"], out[name + "_b"], out[name + "_glibc"], out[name + "_cr"] = a, b, g, c
    assert pos == raw.size
    path = os.path.join(ROOT, "tests", "golden", "crmath_args.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(NAMES)} families x {n}")


if __name__ == "__main__":
    main()
