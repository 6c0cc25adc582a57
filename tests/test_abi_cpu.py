"""CPU-only checks of the product library: it loads, exports every symbol
include/rt_mi355x.h declares, the scene builders keep the reference's
ownership/error semantics, and rendering without a gfx950 device fails loudly
(no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "rt_mi355x.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(product, capi):
    lib = product.lib
    syms = declared_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes table covers exactly the header
    assert sorted("rt_" + k for k in capi.SIGNATURES) == syms


def test_oracle_implements_same_abi(oracle, capi):
    # device-side entry points (stream-ordered render, flattened-world info, device to_rgb) have no CPU
    # meaning; PNG / JSON I/O is checked against Python's zlib / json instead (test_output_cpu.py)
    gpu_only = tuple("orc_" + n for n in capi.GPU_ONLY)
    missing = [m for m in oracle.missing if not m.startswith(("orc_render_device", "orc_world_info", "orc_to_rgb_device",
                                                             "orc_write_png", "orc_camera_from_json") + gpu_only)]
    assert not missing, missing


def test_builders_and_ownership(product, rt, capi):
    s = rt.Scene(product)
    mat = s.Lambertian(s.SolidColor((0.5, 0.5, 0.5)))
    sph = s.Sphere((0, 0, 0), 1.0, mat)
    lst = s.Hittables()
    lst.add(sph)
    with pytest.raises(capi.RtError) as e:  # Box moved into the list
        lst.add(sph)
    assert e.value.code == -3
    bvh = s.BVH(lst)
    with pytest.raises(capi.RtError) as e:
        s.BVH(lst)
    assert e.value.code == -3
    with pytest.raises(capi.RtError) as e:  # BVH over an empty list panics (bvh.rs:26)
        s.BVH(s.Hittables())
    assert e.value.code == -5
    assert s.Triangle((0, 0, 0), (1, 0, 0), (2, 0, 0), mat) is None  # Triangle::new -> None
    assert s.Triangle((0, 0, 0), (1, 0, 0), (0, 1, 0), mat) is not None
    with pytest.raises(capi.RtError) as e:  # Quad::new expect (quad.rs:33)
        s.Quad((0, 0, 0), (1, 0, 0), (2, 0, 0), mat)
    assert e.value.code == -5
    with pytest.raises(capi.RtError):
        s.Lambertian(type("T", (), {"h": 999})())
    box = s.build_box((0, 0, 0), (1, 2, 3), mat)
    t = s.Transform(box, (1, 2, 3), rt.Quaternion.from_axis_angle(product, (0, 1, 0), 15.0), None)
    m = s.ConstantMedium(t, 0.01, s.SolidColor((1, 1, 1)))
    assert bvh.h >= 0 and m.h >= 0


def test_camera_and_shards_match_oracle(product, oracle, capi):
    for api in (product, oracle):
        cam = capi.RtCamera()
        api.camera_default(ctypes.byref(cam))
        assert cam.image_width == 100 and cam.samples_per_pixel == 10 and cam.max_depth == 10
        assert api.camera_image_height(ctypes.byref(cam)) == 100
        cam.aspect_ratio = 16 / 9
        cam.image_width = 1920
        assert api.camera_image_height(ctypes.byref(cam)) == 1080
        opts = capi.RtRenderOpts()
        api.render_opts_default(ctypes.byref(opts))
        opts.row_stride = 8
        total = 0
        for r in range(8):
            opts.row_offset = r
            total += api.shard_rows(ctypes.byref(cam), ctypes.byref(opts))
        assert total == 1080


def test_quaternion_helpers_agree(product, oracle):
    for axis, deg in (((0, 1, 0), 15.0), ((1, 0, 0), 90.0), ((1, 2, 3), -18.0)):
        a = (ctypes.c_double * 4)()
        b = (ctypes.c_double * 4)()
        product.quat_from_axis_angle((ctypes.c_double * 3)(*axis), deg, a)
        oracle.quat_from_axis_angle((ctypes.c_double * 3)(*axis), deg, b)
        assert list(a) == list(b)


def test_render_without_gpu_fails_loudly(product, rt, scenes, capi):
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    s = rt.Scene(product)
    world, lights, cam = scenes.random_spheres(s, 8, 1)
    with pytest.raises(capi.RtError) as e:
        cam.render(world, lights)
    assert e.value.code == -7  # RT_EDEVICE, never a silent CPU fallback


def test_integration_binds_every_symbol():
    """INTEGRATION.md's Rust extern block declares every entry point of the header."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    missing = [s for s in declared_symbols() if "fn " + s + "(" not in text]
    assert not missing, missing


def test_null_camera_is_einval(product, rt, scenes):
    """rt_render / rt_render_device check the camera before touching it or a device."""
    s = rt.Scene(product)
    world, lights, cam = scenes.random_spheres(s, 8, 1)
    assert product.render(s.s, world.h, -1, None, None, None, None, None) == -1
    assert b"camera" in product.last_error()
    assert product.render_device(s.s, world.h, -1, None, None, ctypes.c_void_p(16)) == -1


def test_comm_and_partials_without_render(product, rt):
    """Argument checks of the multi-process and parity-tooling entry points
    (no device needed): bad communicator arguments, partials before a render."""
    assert not product.comm_init(None, 1, 0)
    uid = (ctypes.c_uint8 * 128)()
    assert not product.comm_init(uid, 2, 5)  # rank out of range
    s = rt.Scene(product)
    assert product.render_partials_get(s.s, None, 0) == -1


def test_render_opts_struct_size_checked(product, rt, scenes, capi):
    """rt_render_opts carries its size (ABI 3): options not made by
    rt_render_opts_default (struct_size 0, an older and smaller struct) are
    refused before anything is read past the caller's struct."""
    s = rt.Scene(product)
    world, lights, cam = scenes.random_spheres(s, 8, 1)
    opts = capi.RtRenderOpts()
    product.render_opts_default(ctypes.byref(opts))
    assert opts.struct_size == ctypes.sizeof(capi.RtRenderOpts) and product.abi_version() == 3
    opts.struct_size = 0
    c = cam.to_c()
    assert product.render(s.s, world.h, -1, ctypes.byref(c), ctypes.byref(opts), None, None, None) == -1
    assert b"struct_size" in product.last_error()


def test_product_has_no_test_hooks():
    """The RCCL stand-in override (RT_RCCL_LIB) and the check build's other
    switches are compiled into librt_mi355x_check.so only; the product library
    opens librccl and nothing else."""
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prod = open(os.path.join(here, "raytracer-2025_amd", "librt_mi355x.so"), "rb").read()
    for hook in (b"RT_RCCL_LIB", b"RT_CHECK_RCCL_DUPS", b"RT_CHECK_INJECT"):
        assert hook not in prod, hook
    chk_path = os.path.join(here, "raytracer-2025_amd", "librt_mi355x_check.so")
    if os.path.exists(chk_path):
        chk = open(chk_path, "rb").read()
        assert b"RT_RCCL_LIB" in chk and b"RT_CHECK_RCCL_DUPS" in chk
