"""The conservative f32 quad / triangle pre-test
(raytracer-2025_amd/csrc/rt_planar_filter.h, the source the gfx950 kernel
compiles) against the exact f64 Quad::hit / Triangle::hit (quad.rs:71-102,
triangle.rs:69-98, as the kernel's planar_t computes them) on CPU: millions of
random and adversarial (ray, primitive, bound) triples -- Cornell walls,
rotated box faces, terrain-size and tiny / huge / far triangles, slivers;
targets on edges, vertices and the hypotenuse nudged by 1e-12..1e-5; origins
on the plane; grazing rays; bounds at the exact t.  The filter may only reject
primitives the exact test misses (tests/cpp/planar_prop.cpp).  Built with and
without FMA contraction of the f32 code.  The margin is checked to matter: a
zero margin makes the same cases report tens of thousands of violations
(scripts can reproduce with CU = 0)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")


def build(contract):
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "planar_prop_%s.%d" % (contract, os.getpid()))  # one per pytest worker
    flags = ["-mfma", "-ffp-contract=fast"] if contract == "fast" else ["-ffp-contract=off"]
    subprocess.run(["g++", "-O2", "-std=c++17", *flags, os.path.join(HERE, "cpp", "planar_prop.cpp"), "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("contract", ["fast", "off"])
@pytest.mark.parametrize("seed", [2025, 7])
def test_planar_filter_is_conservative(contract, seed):
    exe = build(contract)
    r = subprocess.run([exe, "1500000", str(seed)], capture_output=True, text=True, timeout=300)
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stdout[-3000:]
    n, rejected, bad = map(int, r.stdout.strip().split("\n")[-1].split())
    assert bad == 0
    # the filter decides: a large share of the (mostly adversarial) cases is rejected
    assert rejected > n // 5
