"""C4 host side on CPU: the OBJ/MTL loader of the product (rt_wavefront_load)
and of the oracle (orc_wavefront_load) on small hand-written files, with the
reference's Wavefont semantics (shapes/obj.rs:117-345): fan triangulation,
models zipped with materials, degenerate triangles skipped, vanilla MTL ->
Metal / Dielectric, Ke -> DiffuseLight, d -> Mix, panics and unsupported
features as error codes.  tobj itself is absent (parity of the parser
unpinned); the expected counts below follow its documented behaviour.

The oracle's RemappedMaterial is checked against the plain-triangle render
(flat vertex normals = face normal -> identical image) and against a bent
normal (different image)."""
import ctypes
import os

import numpy as np
import pytest

MTL = """newmtl chrome
Kd 0.8 0.8 0.8
Pm 1.0
Pr 0.0
newmtl glass
Kd 1 1 1
Tf 1 1 1
Ni 1.5
newmtl lamp
Kd 0.5 0.5 0.5
Pm 1
Ke 4 4 4
newmtl ghost
Kd 0.5 0.5 0.5
Pm 1
d 0.25
"""

QUAD = """mtllib m.mtl
v -1 0 -1
v 1 0 -1
v 1 0 1
v -1 0 1
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 1 0
o quad
usemtl {mat}
f 1/1/1 4/4/1 3/3/1 2/2/1
"""


def write(tmp_path, obj, mtl=MTL, name="t.obj"):
    (tmp_path / "m.mtl").write_text(mtl)
    p = tmp_path / name
    p.write_text(obj)
    return str(p)


def prims(product, capi, scene, world):
    info = capi.RtWorldInfo()
    rc = product.world_info_get(scene.s, world.h, -1, -1, 0, ctypes.byref(info))
    assert rc == 0, product.last_error()
    return info


def load(api, rt, path, vanilla=True):
    s = rt.Scene(api)
    return s, s.Wavefont(path, vanilla)


def test_fan_triangulation_and_counts(product, oracle, rt, capi, tmp_path):
    p = write(tmp_path, QUAD.format(mat="chrome"))
    s, w = load(product, rt, p)
    info = prims(product, capi, s, w)
    assert info.primitives == 2 and info.features & 128  # F_REMAP
    assert info.kernel_tier == 1
    load(oracle, rt, p)  # loads


def test_negative_indices_and_polygon(product, capi, rt, tmp_path):
    obj = QUAD.format(mat="chrome").replace("f 1/1/1 4/4/1 3/3/1 2/2/1", "f -4/-4/-1 -1/-1/-1 -2/-2/-1 -3/-3/-1")
    s, w = load(product, rt, write(tmp_path, obj))
    assert prims(product, capi, s, w).primitives == 2
    pent = QUAD.format(mat="chrome") + "v 0 0 2\nf 1/1/1 4/4/1 5/3/1 3/3/1 2/2/1\n"
    s, w = load(product, rt, write(tmp_path, pent, name="p.obj"))
    assert prims(product, capi, s, w).primitives == 2 + 3


def test_models_zipped_with_materials(product, oracle, capi, rt, tmp_path):
    one_mtl = "newmtl chrome\nKd 1 1 1\nPm 1\n"
    obj = QUAD.format(mat="chrome") + "o second\nf 1/1/1 2/2/1 3/3/1\no third\nf 1/1/1 3/3/1 4/4/1\n"
    s, w = load(product, rt, write(tmp_path, obj, mtl=one_mtl))
    assert prims(product, capi, s, w).primitives == 2  # only the first model (obj.rs:129)
    s, w = load(product, rt, write(tmp_path, obj, name="u.obj"))
    assert prims(product, capi, s, w).primitives == 4  # six materials: all three models


def test_usemtl_splits_models_and_unknown_material_is_empty(product, capi, rt, tmp_path):
    obj = QUAD.format(mat="chrome") + "usemtl glass\nf 1/1/1 2/2/1 3/3/1\nusemtl nosuch\nf 1/1/1 3/3/1 4/4/1\n"
    s, w = load(product, rt, write(tmp_path, obj))
    info = prims(product, capi, s, w)
    assert info.primitives == 4
    # three models -> three BVHs over 2 + 1 + 1 triangles (a 1-object BVH is one
    # node), and the list of the three is walked as a BVH over them (+3 leaves)
    assert info.bvh_leaves == 4 + 3


def test_missing_mtl_loads_nothing(product, oracle, capi, rt, tmp_path):
    obj = QUAD.format(mat="chrome").replace("mtllib m.mtl", "mtllib absent.mtl")
    load(oracle, rt, write(tmp_path, obj))
    s, w = load(product, rt, write(tmp_path, obj))
    assert prims(product, capi, s, w).primitives == 0


def test_degenerate_triangles_skipped(product, capi, rt, tmp_path):
    obj = QUAD.format(mat="chrome") + "f 1/1/1 2/2/1 2/2/1\n"
    s, w = load(product, rt, write(tmp_path, obj))
    assert prims(product, capi, s, w).primitives == 2


NO_VN = lambda o: o.replace("f 1/1/1 4/4/1 3/3/1 2/2/1", "f 1/1 4/4 3/3 2/2")


@pytest.mark.parametrize("obj_edit,extra_mtl,vanilla,code", [
    (NO_VN, "", True, -5),                                    # face corner without vn: index panic (obj.rs:148-158)
    (None, "newmtl nodiffuse\nPm 1\n", True, -5),            # "should at least have one diffuse" (obj.rs:228)
    (None, "newmtl disney\nKd 0.5 0.5 0.5\n", True, -6),     # Disney BSDF: not on the kernel path
    (None, "", False, -6),                                    # vanilla_material = false -> Disney
])
def test_errors(product, oracle, rt, capi, tmp_path, obj_edit, extra_mtl, vanilla, code):
    obj = QUAD.format(mat="chrome")
    if obj_edit:
        obj = obj_edit(obj)
    p = write(tmp_path, obj, mtl=MTL + extra_mtl)
    for api in (product, oracle):
        s = rt.Scene(api)
        with pytest.raises(capi.RtError) as e:
            s.Wavefont(p, vanilla)
        assert e.value.code == code, (api, e.value)


def test_missing_obj_is_an_error(product, oracle, rt, capi, tmp_path):
    for api in (product, oracle):
        with pytest.raises(capi.RtError) as e:
            rt.Scene(api).Wavefont(str(tmp_path / "absent.obj"))
        assert e.value.code == -1


def test_material_mapping_kinds(product, capi, rt, tmp_path):
    """glass -> Dielectric, lamp -> DiffuseLight(Metal) (full tier), ghost -> Mix (full tier)."""
    for mat, tier in (("chrome", 1), ("glass", 1), ("lamp", 2), ("ghost", 2)):
        s, w = load(product, rt, write(tmp_path, QUAD.format(mat=mat), name=mat + ".obj"))
        assert prims(product, capi, s, w).kernel_tier == tier, mat


def _render_oracle(oracle, rt, build, w=48, spp=4):
    s = rt.Scene(oracle)
    world = build(s)
    cam = rt.Camera()
    cam.aspect_ratio = 1.0
    cam.image_width = w
    cam.samples_per_pixel = spp
    cam.max_depth = 8
    cam.vertical_fov_in_degrees = 50.0
    cam.look_from = (0.3, 2.0, 2.5)
    cam.look_at = (0.0, 0.0, 0.0)
    cam.background = s.SkyGradient((1.0, 1.0, 1.0), (0.5, 0.7, 1.0))
    lin, _, st = cam.render(world, None, seed=5)
    assert st.panics == 0
    return lin


def test_oracle_remap_flat_normals_equal_plain_triangles(oracle, rt, tmp_path):
    mtl_ok = "newmtl chrome\nKd 0.8 0.8 0.8\nPm 1.0\nPr 0.2\n"
    p = write(tmp_path, QUAD.format(mat="chrome"), mtl=mtl_ok)

    def from_obj(s):
        w = s.Hittables()
        w.add(s.Wavefont(p))
        return w

    def plain(s):
        m = s.Metal((0.8, 0.8, 0.8), 0.2)
        lst = s.Hittables()
        # fan (1, 4, 3), (1, 3, 2) of the quad, as Triangle::new(p1, p2 - p1, p3 - p1)
        lst.add(s.Triangle((-1, 0, -1), (0, 0, 2), (2, 0, 2), m))
        lst.add(s.Triangle((-1, 0, -1), (2, 0, 2), (2, 0, 0), m))
        w = s.Hittables()
        w.add(s.BVH(lst))
        return w

    a = _render_oracle(oracle, rt, from_obj)
    b = _render_oracle(oracle, rt, plain)
    np.testing.assert_array_equal(a, b)
    bent = QUAD.format(mat="chrome").replace("vn 0 1 0", "vn 0.3 1 0")
    p2 = write(tmp_path, bent, mtl=mtl_ok, name="bent.obj")

    def from_bent(s):
        w = s.Hittables()
        w.add(s.Wavefont(p2))
        return w

    c = _render_oracle(oracle, rt, from_bent)
    assert np.abs(c - a).max() > 1e-3


def test_terrain_generator_deterministic(scenes, tmp_path):
    a = scenes.write_terrain_obj(str(tmp_path / "a"), 6)
    b = scenes.write_terrain_obj(str(tmp_path / "b"), 6)
    assert open(a).read() == open(b).read()
    text = open(a).read()
    assert text.count("\nf ") == 2 * 6 * 6
    assert text.count("\nv ") == 7 * 7 and text.count("\nvn ") == 7 * 7


def test_terrain_loads_on_both(product, oracle, rt, capi, scenes, tmp_path):
    p = scenes.write_terrain_obj(str(tmp_path), 10)
    s = rt.Scene(product)
    w, _, cam = scenes.obj_terrain(s, p, 32, 4)
    info = prims(product, capi, s, w)
    assert info.primitives == 2 * 10 * 10 + 2 and info.kernel_tier == 1
    lin = None
    so = rt.Scene(oracle)
    w, _, cam = scenes.obj_terrain(so, p, 32, 4)
    lin, _, st = cam.render(w, None, seed=1)
    assert st.panics == 0 and np.isfinite(lin).all() and lin.mean() > 0.05


REF_ASSETS = "/root/reference/assets/Final"


@pytest.mark.skipif(not os.path.isdir(REF_ASSETS), reason="reference assets not present (GPU box)")
@pytest.mark.parametrize("name,tier", [("镜子.obj", 2), ("水面.obj", 2)])
def test_reference_vanilla_assets_load(product, oracle, rt, capi, name, tier):
    """The two OBJs the reference's obj_scene loads with vanilla_material = true
    (main.rs:213, 217): the mirror (Pm 1 -> Metal, Ke 0 0 0 -> DiffuseLight
    around it) and the water (Tf 1 -> Dielectric, map_Bump "-bm 1 file" whose
    file is absent -> cyan normal map).  Read in place, not copied."""
    path = os.path.join(REF_ASSETS, name)
    s, w = load(product, rt, path)
    info = prims(product, capi, s, w)
    assert info.primitives == 2 and info.kernel_tier == tier
    so, wo = load(oracle, rt, path)
    cam = rt.Camera()
    cam.image_width = 24
    cam.samples_per_pixel = 4
    cam.max_depth = 6
    cam.look_from = (0.0, 3.0, 2.0)
    cam.look_at = (-1.5, 2.5, -13.0)
    cam.background = so.SkyGradient((1.0, 1.0, 1.0), (0.5, 0.7, 1.0))
    world = so.Hittables()
    world.add(wo)
    lin, _, st = cam.render(world, None, seed=1)
    assert np.isfinite(lin).all()


NM_MTL = "newmtl water\nKd 1 1 1\nNi 1.33\nTf 1.0 1.0 1.0\nmap_Bump -bm 1.000000 absent_normal.png\n"


def test_missing_normal_map_is_cyan(product, oracle, rt, capi, tmp_path):
    """normal_color = cyan*2 - 1 = (-1, 1, 1): the shading normal tilts to
    -u_vec + v_vec + n (obj.rs:42-51); the oracle image must differ from the
    same quad without the map, and the product must pick the full tier."""
    obj = QUAD.format(mat="water")
    p_nm = write(tmp_path, obj, mtl=NM_MTL, name="nm.obj")
    s, w = load(product, rt, p_nm)
    info = prims(product, capi, s, w)
    assert info.kernel_tier == 2 and info.features & 256  # F_NORMALMAP
    a = _render_oracle(oracle, rt, lambda so: _wrap(so, p_nm))
    (tmp_path / "plain").mkdir()
    p_plain = write(tmp_path / "plain", obj, mtl=NM_MTL.split("map_Bump")[0], name="plain.obj")
    b = _render_oracle(oracle, rt, lambda so: _wrap(so, p_plain))
    assert np.abs(a - b).max() > 1e-3


def _wrap(s, path):
    w = s.Hittables()
    w.add(s.Wavefont(path))
    return w


@pytest.mark.parametrize("names,tier", [(["tile", "glass", "bumpy"], 2), (["lamp", "leaf", "lampleaf"], 4)])
def test_obj_image_maps_load(product, oracle, rt, capi, tmp_path, names, tier):
    """map_Kd / map_Ke / map_d / map_Bump images decode (rt_png.hpp) and load
    in both implementations; wrapper nesting and Mix::from_image select the
    FULL_GL tier; a vanilla Metal over map_Kd takes the pixel at (0, 0)."""
    pytest.importorskip("PIL")
    import ctypes
    import objimg
    p = objimg.write_scene(tmp_path, names)
    for api in (product, oracle):
        s = rt.Scene(api)
        w = s.Hittables()
        w.add(s.Wavefont(p))
    s = rt.Scene(product)
    w = s.Wavefont(p)
    info = capi.RtWorldInfo()
    product.check(product.world_info_get(s.s, w.h, -1, -1, 0, ctypes.byref(info)))
    assert info.kernel_tier == tier and info.primitives == 2 * len(names)


def test_reference_mc_obj_needs_disney(product, oracle, rt, capi):
    """The reference's own assets/Final/mc.obj (read in place) decodes its PNG
    maps (4-bit palette, gray, RGBA) but its materials are Disney BSDFs
    (no Pm / Tf, obj.rs:299-311): out of scope, RT_EUNSUPPORTED in both."""
    path = "/root/reference/assets/Final/mc.obj"
    if not os.path.exists(path):
        pytest.skip("reference assets not mounted")
    for api in (product, oracle):
        s = rt.Scene(api)
        with pytest.raises(capi.RtError) as e:
            s.Wavefont(path)
        assert e.value.code == -6 and b"Disney" in api.last_error()
