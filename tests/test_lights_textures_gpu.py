"""GPU parity for the light and texture breadth of the path (SURVEY §8a R12,
R15, R22, R24): sphere lights, Transform and nested-list lights (tier
FULL_GL), CheckerTexture, decoded ImageTexture (nearest and bilinear) on
objects and as the environment, against the TEST-ONLY oracle on the same
scene script and seed.  Bars as test_parity_gpu.check."""
import numpy as np
import pytest

import objimg
from conftest import rmse_per_channel
from test_parity_gpu import check, render_both

pytestmark = pytest.mark.gpu


def _room(s, rt, width=64, spp=16, depth=10):
    """A small Cornell-style room (main.rs:541-639 proportions, 555 units)."""
    red = s.Lambertian(s.SolidColor((0.65, 0.05, 0.05)))
    white = s.Lambertian(s.SolidColor((0.73, 0.73, 0.73)))
    green = s.Lambertian(s.SolidColor((0.12, 0.45, 0.15)))
    world = s.Hittables()
    world.add(s.Quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green))
    world.add(s.Quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red))
    world.add(s.Quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
    world.add(s.Quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white))
    world.add(s.Quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    cam = rt.Camera()
    cam.aspect_ratio = 1.0
    cam.image_width = width
    cam.samples_per_pixel = spp
    cam.max_depth = depth
    cam.vertical_fov_in_degrees = 40.0
    cam.look_from = (278.0, 278.0, -800.0)
    cam.look_at = (278.0, 278.0, 0.0)
    return world, cam


def _tier(api, capi, scene, world, lights, cam):
    import ctypes
    info = capi.RtWorldInfo()
    bg = cam.background.h if cam.background is not None else -1
    api.check(api.world_info_get(scene.s, world.h, -1 if lights is None else lights.h, bg, 0, ctypes.byref(info)))
    return info.kernel_tier


def test_sphere_light(gpu, oracle, rt, capi):
    """A spherical DiffuseLight sampled through Sphere::pdf_value / random
    (sphere.rs:114-145, cone sampling) in the 50/50 mixture, beside a glass
    sphere the light also shines through (camera inside no sphere, origin
    inside the light for the rays that start on it)."""
    def build(s):
        world, cam = _room(s, rt)
        lm = s.DiffuseLight(s.SolidColor((12.0, 12.0, 10.0)))
        world.add(s.Sphere((278, 470, 278), 60, lm))
        world.add(s.Sphere((190, 90, 190), 90, s.Dielectric(s.SolidColor((1, 1, 1)), 1.5)))
        world.add(s.Sphere((380, 80, 300), 80, s.Metal((0.8, 0.85, 0.9), 0.2)))
        lights = s.Hittables()
        lights.add(s.Sphere((278, 470, 278), 60, s.EmptyMaterial()))
        return world, lights, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) in (2, 3)  # a flat light list: the C3 / C5 tiers' light code


def test_transform_light(gpu, oracle, rt, capi):
    """The ceiling light as a Transform (rotated 25 deg about x, scaled,
    offset): HittablePDF reaches it through Transform::pdf_value / random in
    the light's local frame (shapes.rs:117-132) -- tier FULL_GL."""
    def build(s):
        world, cam = _room(s, rt)
        lm = s.DiffuseLight(s.SolidColor((15.0, 15.0, 15.0)))
        q = rt.Quaternion.from_axis_angle(s.api, (1, 0, 0), 25.0)
        world.add(s.Transform(s.Quad((0, 0, 0), (130, 0, 0), (0, 0, 105), lm), (213, 520, 227), q, (1.2, 1.0, 0.8)))
        world.add(s.Transform(s.build_box((0, 0, 0), (165, 330, 165), s.Lambertian(s.SolidColor((0.73, 0.73, 0.73)))),
                              (265, 0, 295), rt.Quaternion.from_axis_angle(s.api, (0, 1, 0), 15.0), None))
        lights = s.Transform(s.Quad((0, 0, 0), (130, 0, 0), (0, 0, 105), s.EmptyMaterial()), (213, 520, 227), q,
                             (1.2, 1.0, 0.8))
        return world, lights, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) == 4


def test_nested_light_tree(gpu, oracle, rt, capi):
    """lights = [ [quad, triangle], Transform([sphere]), moving sphere ]:
    nested Hittables averages (hits.rs:52-67), a choose per level
    (hits.rs:69-75), a moving sphere sampled at its time-0 center
    (sphere.rs:114-144), all in one mixture."""
    def build(s):
        world, cam = _room(s, rt, depth=8)
        l1 = s.DiffuseLight(s.SolidColor((10.0, 10.0, 10.0)))
        l2 = s.DiffuseLight(s.SolidColor((4.0, 8.0, 12.0)))
        world.add(s.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), l1))
        world.add(s.Triangle((60, 554, 60), (120, 0, 0), (0, 0, 120), l1))
        world.add(s.Transform(s.Sphere((0, 0, 0), 40, l2), (420, 300, 420), None, (1.0, 1.0, 1.0)))
        world.add(s.Sphere_new_with_motion((120, 300, 400), (150, 300, 400), 35, l2))
        world.add(s.Sphere((278, 100, 250), 100, s.Lambertian(s.SolidColor((0.5, 0.5, 0.5)))))
        e = s.EmptyMaterial()
        inner = s.Hittables()
        inner.add(s.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), e))
        inner.add(s.Triangle((60, 554, 60), (120, 0, 0), (0, 0, 120), e))
        sph = s.Hittables()
        sph.add(s.Sphere((0, 0, 0), 40, e))
        lights = s.Hittables()
        lights.add(inner)
        lights.add(s.Transform(sph, (420, 300, 420), None, (1.0, 1.0, 1.0)))
        lights.add(s.Sphere_new_with_motion((120, 300, 400), (150, 300, 400), 35, e))
        return world, lights, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) == 4


@pytest.mark.parametrize("kind", ["bvh", "medium", "empty"])
def test_lights_without_pdf_panic(gpu, oracle, rt, capi, kind):
    """A BVH or a ConstantMedium has no pdf_value / random (hit.rs:52-60
    unimplemented!()), an empty Hittables panics in choose (hits.rs:71-73):
    the reference panics at the first light sample, so do both here."""
    def build(s):
        world, cam = _room(s, rt, width=16, spp=1)
        lst = s.Hittables()
        if kind != "empty":
            lst.add(s.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), s.EmptyMaterial()))
        if kind == "bvh":
            lights = s.BVH(lst)
        elif kind == "medium":
            lights = s.ConstantMedium(lst, 0.1, s.SolidColor((1, 1, 1)))
        else:
            lights = lst
        return world, lights, cam
    for api in (gpu, oracle):
        s = rt.Scene(api)
        w, l, c = build(s)
        with pytest.raises(capi.RtError) as e:
            c.render(w, l)
        assert e.value.code == -5  # RT_EPANIC


def checker_world(rt, s, where):
    """CheckerTexture (texture.rs:39-73) on spheres and a floor; "quad_y0" puts
    the floor on y = 0, the texture's knife edge."""
    even = s.CheckerTexture(0.5, s.SolidColor((0.9, 0.9, 0.9)), s.SolidColor((0.1, 0.3, 0.6)))
    tex = s.CheckerTexture(3.0, even, s.SolidColor((0.8, 0.2, 0.1)))
    world = s.Hittables()
    if where == "sphere":
        world.add(s.Sphere((0, -1000, 0), 1000, s.Lambertian(tex)))
    else:
        y = 0.0 if where == "quad_y0" else 0.25
        world.add(s.Quad((-8, y, -8), (16, 0, 0), (0, 0, 16), s.Lambertian(tex)))
    world.add(s.Sphere((0, 1, 0), 1.0, s.Lambertian(tex)))
    world.add(s.Sphere((2.2, 0.7, 0.5), 0.7, s.Metal((0.8, 0.8, 0.8), 0.05)))
    cam = rt.Camera()
    cam.aspect_ratio = 16 / 9
    cam.image_width = 96
    cam.samples_per_pixel = 16
    cam.max_depth = 20
    cam.vertical_fov_in_degrees = 30.0
    cam.look_from = (6.0, 2.5, 7.0)
    cam.look_at = (0.0, 0.6, 0.0)
    cam.background = s.SkyGradient()
    return world, None, cam


@pytest.mark.parametrize("where", ["sphere", "quad", "quad_y0"])
def test_checker_texture(gpu, oracle, rt, capi, where):
    """CheckerTexture (texture.rs:39-73): floor(scale * p) parity, nested
    (a checker of a checker and a solid), on the basic tier (spheres) and on
    the mesh tier (a quad floor).

    quad_y0 puts the floor on y = 0, a knife edge of the texture: every hit
    point's p.y is 0 +- an ulp, and floor(p.y / 0.5) is 0 or -1 by its sign,
    so an ulp of difference anywhere upstream picks the other square.  With
    ROCm's ocml sin / cos in the kernel 1.3e-3 of its (pixel, s_i) sums
    diverged (RMSE 1.1e-3, round 2); with the kernel's correctly rounded
    functions (rt_crmath.h) only glibc's own misroundings remain, and the
    default bar holds (test_libm_parity_gpu.py: exact against the oracle on
    the same functions)."""
    out, st = render_both(gpu, oracle, rt, lambda s: checker_world(rt, s, where))
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = checker_world(rt, s, where)
    assert _tier(gpu, capi, s, w, l, c) == (0 if where == "sphere" else 1)


def _image(h, w, seed):
    """A decoded linear RGBA image (what Image::pixel_data hands the texture,
    image.rs:63-82): smooth bands plus noise, alpha 1."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    img = np.zeros((h, w, 4), dtype=np.float32)
    img[..., 0] = 0.5 + 0.5 * np.sin(x * 0.7)
    img[..., 1] = (y / max(1, h - 1)).astype(np.float32)
    img[..., 2] = rng.random((h, w)).astype(np.float32)
    img[..., 3] = 1.0
    return img


@pytest.mark.parametrize("linear", [False, True])
def test_image_texture(gpu, oracle, rt, linear):
    """ImageTexture (texture.rs:82-174): u, v wrapped by x - floor(x), v
    flipped, nearest (ImageInterpMethod::None) or bilinear
    (ImageInterpMethod::Linear), on a sphere (uv from sphere.rs:53-61), on a
    quad (alpha/beta as uv) and as the environment (environment.rs:14-24)."""
    def build(s):
        tex = s.ImageTexture(_image(24, 48, 1), linear_interp=linear)
        env = s.ImageTexture(_image(16, 32, 2), linear_interp=linear)
        world = s.Hittables()
        world.add(s.Sphere((0, 1, 0), 1.0, s.Lambertian(tex)))
        world.add(s.Quad((-3, 0, -3), (6, 0, 0), (0, 0, 6), s.Lambertian(tex)))
        world.add(s.Sphere((2.0, 0.6, 0.8), 0.6, s.Dielectric(tex, 1.5)))
        cam = rt.Camera()
        cam.aspect_ratio = 16 / 9
        cam.image_width = 96
        cam.samples_per_pixel = 16
        cam.max_depth = 12
        cam.vertical_fov_in_degrees = 35.0
        cam.look_from = (5.0, 2.0, 6.0)
        cam.look_at = (0.0, 0.7, 0.0)
        cam.background = env
        return world, None, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0


@pytest.mark.parametrize("fmt", ["jpeg420", "jpeg_progressive", "hdr"])
def test_image_texture_file_formats(gpu, oracle, rt, tmp_path, fmt):
    """ImageTexture::new_raw_image(file) (texture.rs:82-97) from a JPEG (4:2:0
    baseline / progressive, rt_jpeg.hpp) or a Radiance HDR (rt_hdr.hpp, linear
    whatever the raw flag: image.rs:76-80) decoded by the library, against the
    oracle given the same pixels decoded independently -- PIL for the JPEG
    (tests/test_jpeg_cpu.py holds the decoder bit-exact against it), the
    RGBE formula for the HDR."""
    PILImage = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(11)
    h, w = 40, 56
    if fmt.startswith("jpeg"):
        a = (_image(h, w, 4)[..., :3] * 255).astype(np.uint8)
        path = tmp_path / "t.jpg"
        PILImage.fromarray(a).save(str(path), quality=85, subsampling=2, progressive=fmt == "jpeg_progressive")
        px = np.asarray(PILImage.open(str(path)).convert("RGB"), dtype=np.float32) / np.float32(255.0)
    else:
        from test_jpeg_cpu import _hdr_bytes, _rgbe_expected
        rgbe = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
        rgbe[..., 3] = rng.integers(125, 131, size=(h, w))
        path = tmp_path / "t.hdr"
        path.write_bytes(_hdr_bytes(rgbe, "new_rle"))
        px = _rgbe_expected(rgbe)
    rgba = np.concatenate([px, np.ones((h, w, 1), np.float32)], axis=-1)

    def build(s):
        if s.api is gpu:
            tex = s.ImageTexture_file(str(path), raw=True, linear_interp=True)
        else:
            tex = s.ImageTexture(rgba, linear_interp=True)
        world = s.Hittables()
        world.add(s.Sphere((0, 1, 0), 1.0, s.Lambertian(tex)))
        world.add(s.Quad((-3, 0, -3), (6, 0, 0), (0, 0, 6), s.Lambertian(tex)))
        cam = rt.Camera()
        cam.aspect_ratio = 16 / 9
        cam.image_width = 96
        cam.samples_per_pixel = 16
        cam.max_depth = 8
        cam.vertical_fov_in_degrees = 35.0
        cam.look_from = (5.0, 2.0, 6.0)
        cam.look_at = (0.0, 0.7, 0.0)
        return world, None, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0


def test_obj_jpeg_maps(gpu, oracle, rt, tmp_path):
    """An OBJ whose map_Kd / map_Ke / map_Bump images are JPEGs (4:2:0, one
    progressive): the library decodes them (rt_jpeg.hpp) on the GPU side; the
    oracle, which reads PNG only, gets the same scene with each JPEG replaced
    by a PNG of PIL's decode of it (tests/test_jpeg_cpu.py holds the two
    decodes bit-equal) -- so the JPEG path through the OBJ loader is checked
    against the oracle at the default bar."""
    PILImage = pytest.importorskip("PIL.Image")
    names = ["tile", "glass", "lamp", "bumpy"]
    dirs = {}
    for side in ("gpu", "oracle"):
        d = tmp_path / side
        d.mkdir()
        objimg.write_scene(d, names)
        dirs[side] = d
    mtl = (dirs["gpu"] / "m.mtl").read_text()
    for k, img in enumerate(("albedo", "emit", "normal")):
        src = dirs["gpu"] / f"{img}.png"
        jpg = dirs["gpu"] / f"{img}.jpg"
        PILImage.open(str(src)).convert("RGB").save(str(jpg), quality=88, subsampling=2, progressive=k == 1)
        mtl = mtl.replace(f"{img}.png", f"{img}.jpg")
        # the oracle's PNG: PIL's decode of that JPEG, lossless
        PILImage.open(str(jpg)).convert("RGB").save(str(dirs["oracle"] / f"{img}.png"))
    (dirs["gpu"] / "m.mtl").write_text(mtl)

    def build(s):
        d = dirs["gpu"] if s.api is gpu else dirs["oracle"]
        world = s.Hittables()
        world.add(s.Wavefont(str(d / "scene.obj")))
        world.add(s.Sphere((0, -100.2, 0), 100, s.Lambertian(s.SolidColor((0.4, 0.45, 0.4)))))
        cam = rt.Camera()
        cam.aspect_ratio = 16 / 9
        cam.image_width = 96
        cam.samples_per_pixel = 16
        cam.max_depth = 12
        cam.vertical_fov_in_degrees = 50.0
        cam.look_from = (0.0, 1.2, 4.0)
        cam.look_at = (-0.4, 0.6, 0.0)
        cam.background = s.SkyGradient((1.0, 1.0, 1.0), (0.5, 0.7, 1.0))
        return world, None, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == st["oracle"].panics == 0


@pytest.mark.parametrize("names", [["tile", "glass", "bumpy"], ["lamp", "leaf", "lampleaf"]])
def test_obj_image_materials(gpu, oracle, rt, capi, tmp_path, names):
    """map_Kd -> ImageTexture (a vanilla Metal takes its pixel at (0, 0), a
    Dielectric the texture), map_Ke -> DiffuseLight(image, mat), map_d ->
    Mix::from_image(Transparent, mat) (the alpha as the ratio), map_Bump ->
    a raw bilinear normal map; PNGs decoded by the library (rt_png.hpp).  The
    second case nests wrappers (Mix of DiffuseLight(image, DiffuseLight(Ke,
    Metal))) -- the FULL_GL tier."""
    pytest.importorskip("PIL")
    objimg.write_scene(tmp_path, names)

    def build(s):
        world = s.Hittables()
        world.add(s.Wavefont(str(tmp_path / "scene.obj")))
        world.add(s.Sphere((0, -100.2, 0), 100, s.Lambertian(s.SolidColor((0.4, 0.45, 0.4)))))
        cam = rt.Camera()
        cam.aspect_ratio = 16 / 9
        cam.image_width = 96
        cam.samples_per_pixel = 16
        cam.max_depth = 12
        cam.vertical_fov_in_degrees = 50.0
        cam.look_from = (0.0, 1.2, 4.0)
        cam.look_at = (-0.4, 0.6, 0.0)
        cam.background = s.SkyGradient((1.0, 1.0, 1.0), (0.5, 0.7, 1.0))
        return world, None, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == st["oracle"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) == (4 if "leaf" in names else 2)
