"""The oracle against its committed golden frames (tests/golden/, made by
scripts/gen_golden.py) and against analytic properties of the reference
algorithm."""
import ctypes
import importlib
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
gen_golden = importlib.import_module("gen_golden")


@pytest.mark.parametrize("name", sorted(gen_golden.CASES))
def test_oracle_matches_golden(oracle, name):
    """Bit for bit: the oracle is deterministic (counter-based RNG, fixed
    summation order), so any change to a committed frame is a change of the
    restated algorithm."""
    build, seed, off, stride = gen_golden.case(name)
    img = gen_golden.render(oracle, build, seed, off, stride)
    ref = np.load(os.path.join(ROOT, "tests", "golden", name + ".npy"))
    assert img.shape == ref.shape and img.tobytes() == ref.tobytes()


def _furnace(oracle, rt, material):
    scene = rt.Scene(oracle)
    world = scene.Hittables()
    world.add(scene.Sphere((0, 0, -2), 1.0, material(scene)))
    cam = rt.Camera()
    cam.image_width = 24
    cam.samples_per_pixel = 16
    cam.max_depth = 50
    cam.background = scene.SolidColor((1, 1, 1))
    lin, _, _ = cam.render(world, None, seed=3)
    return lin


def test_furnace_lambertian(oracle, rt):
    """CosinePDF weight f/pdf == albedo (pdf.rs:50-57): albedo-1 Lambertian in
    a white environment returns exactly 1 on every pixel."""
    lin = _furnace(oracle, rt, lambda s: s.Lambertian(s.SolidColor((1, 1, 1))))
    np.testing.assert_allclose(lin, 1.0, atol=1e-6)


def test_furnace_glass(oracle, rt):
    """Dielectric with white attenuation never absorbs (material.rs:117-143)."""
    lin = _furnace(oracle, rt, lambda s: s.Dielectric(s.SolidColor((1, 1, 1)), 1.5))
    np.testing.assert_allclose(lin, 1.0, atol=1e-6)


def test_furnace_metal_albedo(oracle, rt):
    """Metal multiplies by its albedo at each bounce and never absorbs
    (material.rs:82-95): a convex metal sphere reflects once -> albedo."""
    lin = _furnace(oracle, rt, lambda s: s.Metal((0.5, 0.25, 0.125), 0.0))
    inside = lin[..., 0] <= 0.5 + 1e-6  # pixels whose every sample hits the sphere (f32 frame)
    assert inside.sum() > 20
    np.testing.assert_allclose(lin[inside], np.broadcast_to([0.5, 0.25, 0.125], lin[inside].shape), atol=1e-12)


def test_sample_count_and_strata(oracle, rt, scenes):
    """spp 10 traces floor(sqrt(10))^2 = 9 strata (camera.rs:212-214)."""
    scene = rt.Scene(oracle)
    world, lights, cam = scenes.random_spheres(scene, 16, 10)
    _, _, st = cam.render(world, lights)
    assert st.samples == 16 * 9 * 9


@pytest.fixture(scope="module")
def oracle_fast(capi, oracle):
    """liboracle_fast.so: the timed CPU baseline (-O3, work counters compiled
    out; oracle/Makefile)."""
    return capi.Api(ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle_fast.so")), "orc_",
                    capi.ORACLE_EXTRAS)


@pytest.mark.parametrize("name", sorted(gen_golden.CASES))
def test_timed_baseline_build_renders_the_same_bits(oracle, oracle_fast, name):
    """bench.py times liboracle_fast.so; it must compute exactly what the
    counting build the tests check computes (same f64 operations: -O3 changes
    no rounding under -ffp-contract=off)."""
    build, seed, off, stride = gen_golden.case(name)
    a = gen_golden.render(oracle, build, seed, off, stride)
    b = gen_golden.render(oracle_fast, build, seed, off, stride)
    assert a.dtype == b.dtype and a.shape == b.shape
    assert a.tobytes() == b.tobytes()


def test_timed_baseline_build_has_no_counts(oracle, oracle_fast, rt, scenes):
    """The counting build reports work per sample; the timed build counts
    nothing (its render loop carries no thread-local increments)."""
    n = oracle.work_count_fields()
    counts = []
    for api in (oracle, oracle_fast):
        scene = rt.Scene(api)
        world, lights, cam = scenes.random_spheres(scene, 16, 4)
        c = cam.to_c()
        opts = rt.Camera._opts(api, 1, 0, 1, 0, 0)[0]
        wc = (ctypes.c_uint64 * n)()
        api.check(api.render_f64(scene.s, world.h, -1 if lights is None else lights.h, ctypes.byref(c),
                                 ctypes.byref(opts), None, None, None, wc))
        counts.append(list(wc))
    assert sum(counts[0]) > 0
    assert sum(counts[1]) == 0
