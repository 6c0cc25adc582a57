"""Host sanitizers: the host code that builds and flattens worlds
-- BVH::from_vec's parallel builder (bvh.rs:16-46), the flatten's parallel
binned SAH, the in-place OBJ / MTL parser (shapes/obj.rs:117-194), the PNG
writer and Camera::from_json -- and the oracle's multithreaded render, each
under AddressSanitizer + UBSan and under ThreadSanitizer.

`make -C raytracer-2025_amd asan tsan` / `make -C oracle asan tsan` link the
test-only driver tests/cpp/host_sanitize.cpp against the sanitized objects
(host code only; nothing here touches a GPU).  The driver checks the parallel
builders against their serial twins (rt_bvh_selftest / rt_world_selftest) on
the book-1 world, a 22 504-sphere list and an OBJ terrain -- the 1M-triangle
C4 terrain for the product under ASan, an 80 000-triangle one otherwise (past
both parallel builders' thresholds) -- and renders a C1-shaped frame on 8
oracle threads.
Each build is first shown to catch a planted heap overflow / data race."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

PKG_DIR = os.path.join(ROOT, "raytracer-2025_amd")
ORC_DIR = os.path.join(ROOT, "oracle")
EXES = {
    ("product", "asan"): os.path.join(PKG_DIR, "_obj", "san", "host_sanitize_asan"),
    ("product", "tsan"): os.path.join(PKG_DIR, "_obj", "san", "host_sanitize_tsan"),
    ("oracle", "asan"): os.path.join(ORC_DIR, "_build", "host_sanitize_asan"),
    ("oracle", "tsan"): os.path.join(ORC_DIR, "_build", "host_sanitize_tsan"),
}


@pytest.fixture(scope="module")
def built():
    for d in (PKG_DIR, ORC_DIR):
        subprocess.run(["make", "-j", "4", "-C", d, "asan", "tsan"], check=True, stdout=subprocess.DEVNULL, timeout=900)
    return EXES


@pytest.fixture(scope="module")
def terrains(tmp_path_factory, scenes):
    base = tmp_path_factory.mktemp("san_terrain")
    return {"c4": scenes.write_terrain_obj(str(base / "t707"), 707),  # C4's 999 698 triangles
            "small": scenes.write_terrain_obj(str(base / "t200"), 200)}  # 79 202 triangles


def _run(exe, obj, out, *extra, timeout=600):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1")
    return subprocess.run([exe, obj, str(out), "8", "4", *extra], capture_output=True, text=True, timeout=timeout,
                          env=env)


@pytest.mark.parametrize("which", ["product", "oracle"])
@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_host_code_is_sanitizer_clean(built, terrains, tmp_path, which, san):
    # the product's loader and builders meet C4's 1M-triangle OBJ under ASan
    r = _run(built[(which, san)], terrains["c4" if (which, san) == ("product", "asan") else "small"], tmp_path)
    sys.stdout.write(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASSED" in r.stdout
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
    # every check of the build ran: selftests (product) / the render (oracle)
    want = ["flatten, parallel SAH == serial (terrain world)", "BVH::from_vec, parallel builder == serial (22 504"] \
        if which == "product" else ["multithreaded oracle render"]
    for w in want:
        assert "ok   " + w in r.stdout, r.stdout


@pytest.mark.parametrize("which", ["product", "oracle"])
@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_sanitizer_is_live(built, terrains, tmp_path, which, san):
    """The driver's planted bug is reported: the build really is instrumented."""
    r = _run(built[(which, san)], terrains["small"], tmp_path, "oob" if san == "asan" else "race", timeout=300)
    assert r.returncode != 0
    if san == "asan":  # UBSan's object-size check or ASan, whichever sees the read first
        assert "heap-buffer-overflow" in r.stderr or "runtime error: load of address" in r.stderr, r.stderr[-2000:]
    else:
        assert "data race" in r.stderr, r.stderr[-2000:]
