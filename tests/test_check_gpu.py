"""The check build (`make -C raytracer-2025_amd check`, librt_mi355x_check.so):
every ref the kernel decodes -- walk steps, a node's sphere slots, planar
runs, hit records, lights -- is checked against its array's size
(rt_kernel.hip ref_idx, SceneView::n_ref), and a ref past its array makes the
render fail with RT_EPANIC naming it instead of reading past the array.

Round 3's bvh4_relayout named a record past the triangle array and changed 13
pixels of a C4 frame without a fault; this is the guard that stops such a bug
at its first read.  The whole GPU suite is run once on the check build
(RT_MI355X_LIB=raytracer-2025_amd/librt_mi355x_check.so pytest -m gpu); here
the check build renders each workload kind and a world with an injected bad
ref (RT_CHECK_INJECT=1, compiled into the check build's host only)."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_SO = os.path.join(ROOT, "raytracer-2025_amd", "librt_mi355x_check.so")


@pytest.fixture(scope="module")
def check_api(capi, gpu):
    # a build product (__graft_entry__.build() makes it): absent is a failure
    assert os.path.exists(CHECK_SO), "check build absent: make -C raytracer-2025_amd check (__graft_entry__.build())"
    api = capi.Api(ctypes.CDLL(CHECK_SO), "rt_")
    assert not api.missing, api.missing
    return api


@pytest.fixture(scope="module")
def terrain(scenes, tmp_path_factory):
    return scenes.write_terrain_obj(str(tmp_path_factory.mktemp("check_terrain")), 24)


def _worlds(rt, scenes, api, terrain):
    s = rt.Scene(api)
    yield "spheres", s, *scenes.random_spheres(s, 48, 4)
    s = rt.Scene(api)
    yield "cornell", s, *scenes.cornell_smoke(s, 40, 4)
    s = rt.Scene(api)
    yield "final", s, *scenes.final_scene(s, 48, 4, 8, aspect_ratio=16 / 9)
    s = rt.Scene(api)
    yield "terrain", s, *scenes.obj_terrain(s, terrain, 64, 4)


def test_check_build_renders_like_the_product(check_api, gpu, rt, scenes, capi, terrain):
    """No ref past its array on the basic, mesh (OBJ terrain), flat and full
    tiers, and the same bits as the product library."""
    tiers = set()
    for (name, s, world, lights, cam), (_, s2, world2, lights2, cam2) in zip(_worlds(rt, scenes, check_api, terrain),
                                                                            _worlds(rt, scenes, gpu, terrain)):
        lin, _, st = cam.render(world, lights, seed=3, want_srgb=False)
        ref, _, st2 = cam2.render(world2, lights2, seed=3, want_srgb=False)
        np.testing.assert_array_equal(lin, ref, err_msg=name)
        info = capi.RtWorldInfo()
        bg = cam.background.h if cam.background is not None else -1
        check_api.check(check_api.world_info_get(s.s, world.h, -1 if lights is None else lights.h, bg, 0,
                                                 ctypes.byref(info)))
        tiers.add(info.kernel_tier)
    assert tiers == {0, 1, 2, 3}, tiers


@pytest.mark.parametrize("workload", ["spheres", "final", "terrain"])
def test_check_build_reports_a_bad_ref(check_api, rt, scenes, capi, workload, monkeypatch, terrain):
    """RT_CHECK_INJECT=1: the flattened world's first primitive slot names one
    record past its array (basic tier: a sphere; full tier: a sphere or quad);
    the render must fail with RT_EPANIC and say which ref."""
    monkeypatch.setenv("RT_CHECK_INJECT", "1")
    for name, s, world, lights, cam in _worlds(rt, scenes, check_api, terrain):
        if name != workload:
            continue
        with pytest.raises(capi.RtError) as e:
            cam.render(world, lights, seed=3, want_srgb=False)
        assert e.value.code == -5, e.value
        assert "past their array" in str(e.value) or "past their array" in (check_api.last_error() or b"").decode()
