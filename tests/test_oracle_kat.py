"""The oracle against the only golden vectors the reference holds for this
path: its own 34 unit tests (vec3.rs, ray.rs, quaternion.rs, aabb.rs,
sphere.rs), restated in oracle/kat_reference_tests.cpp, plus the Random123
Philox4x32-10 known-answer vectors that pin the RNG contract."""
import os
import subprocess

from conftest import ROOT


def test_reference_unit_tests_restated():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    exe = os.path.join(ROOT, "oracle", "_build", "kat_reference_tests")
    r = subprocess.run([exe], capture_output=True, text=True)
    lines = [l for l in r.stdout.splitlines() if l.startswith(("PASS", "FAIL"))]
    failed = [l for l in lines if l.startswith("FAIL")]
    assert r.returncode == 0 and not failed, r.stdout
    names = {l.split()[1] for l in lines}
    # 16 vec3 + 3 ray + 6 quaternion + 8 aabb + 1 sphere = 34 reference tests, + Philox KAT
    assert sum(n.startswith("vec3::") for n in names) == 16
    assert sum(n.startswith("ray::") for n in names) == 3
    assert sum(n.startswith("quaternion::") for n in names) == 6
    assert sum(n.startswith("aabb::") for n in names) == 8
    assert sum(n.startswith("sphere::") for n in names) == 1
    assert "rng::philox4x32_10_random123_kat" in names
