"""GPU parity for the full-flat tier's shortcuts (tier 3, worlds without BVH
nodes), against the TEST-ONLY oracle, which walks lists element by element and
medium boundaries twice (volume.rs:44-48):

* planar runs: a list step tests up to 8 consecutive quads / triangles at once
  (rt_scene.cpp DBoxF::run) -- runs of quads, of triangles, mixed, a list
  longer than one run, a run inside a Transform;
* one-pass medium boundaries (rt_kernel.hip boundary_onepass): a box of quads
  inside one and two Transforms, a triangle boundary, a sphere boundary bare
  and inside a Transform, a camera inside a medium, and a 7-quad boundary that
  is longer than the one-pass limit (the two-walk path).
Bars as test_parity_gpu.check."""
import pytest

from test_lights_textures_gpu import _room, _tier
from test_parity_gpu import check, render_both

pytestmark = pytest.mark.gpu


def _light(s, world):
    lm = s.DiffuseLight(s.SolidColor((15.0, 15.0, 15.0)))
    world.add(s.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), lm))
    lights = s.Hittables()
    lights.add(s.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), s.EmptyMaterial()))
    return lights


def _pyramid(s, apex, base, half, mat):
    """Four triangles (a square pyramid's sides) in one list: a triangle run."""
    x, y, z = base
    corners = [(x - half, y, z - half), (x + half, y, z - half), (x + half, y, z + half), (x - half, y, z + half)]
    lst = s.Hittables()
    for k in range(4):
        a, b = corners[k], corners[(k + 1) % 4]
        lst.add(s.Triangle(a, tuple(b[i] - a[i] for i in range(3)), tuple(apex[i] - a[i] for i in range(3)), mat))
    return lst


def test_flat_planar_runs(gpu, oracle, rt, capi):
    """Room walls (a 5-quad run, then the light), a pyramid (triangle run), a
    rotated box (a 6-quad run inside a Transform), a 10-quad staircase (runs of
    8 + 2) and a list mixing quads and triangles."""
    def build(s, rt=rt):
        world, cam = _room(s, rt, width=64, spp=16, depth=8)
        lights = _light(s, world)
        white = s.Lambertian(s.SolidColor((0.73, 0.73, 0.73)))
        metal = s.Metal((0.8, 0.85, 0.9), 0.1)
        world.add(_pyramid(s, (150, 260, 380), (150, 0, 380), 90, metal))
        q = rt.Quaternion.from_axis_angle(s.api, (0, 1, 0), 15.0)
        world.add(s.Transform(s.build_box((0, 0, 0), (120, 200, 120), white), (330, 0, 300), q, None))
        stairs = s.Hittables()
        for k in range(10):
            stairs.add(s.Quad((40 + 18 * k, 20 * k, 60), (18, 0, 0), (0, 0, 90), white))
        world.add(stairs)
        mixed = s.Hittables()
        mixed.add(s.Quad((400, 40, 120), (80, 0, 0), (0, 80, 0), s.Dielectric(s.SolidColor((1, 1, 1)), 1.5)))
        mixed.add(s.Triangle((420, 150, 140), (60, 0, 0), (0, 60, 0), metal))
        mixed.add(s.Quad((420, 230, 160), (60, 0, 0), (0, 0, 60), white))
        world.add(mixed)
        return world, lights, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) == 3


@pytest.mark.parametrize("variant", ["boxes", "spheres", "inside_fog"])
def test_flat_medium_boundaries(gpu, oracle, rt, capi, variant):
    """ConstantMedium over the boundaries the one-pass test covers and one it
    does not (a 7-quad list)."""
    def build(s, rt=rt):
        world, cam = _room(s, rt, width=64, spp=16, depth=8)
        lights = _light(s, world)
        q1 = rt.Quaternion.from_axis_angle(s.api, (0, 1, 0), -18.0)
        q2 = rt.Quaternion.from_axis_angle(s.api, (1, 0, 0), 10.0)
        if variant == "boxes":
            box = s.build_box((0, 0, 0), (150, 150, 150), s.EmptyMaterial())
            world.add(s.ConstantMedium(s.Transform(box, (100, 0, 60), q1, None), 0.01, s.SolidColor((0.9, 0.9, 0.9))))
            box2 = s.build_box((0, 0, 0), (120, 240, 120), s.EmptyMaterial())
            inner = s.Transform(box2, (0, 0, 0), q2, (1.0, 0.9, 1.1))
            world.add(s.ConstantMedium(s.Transform(inner, (320, 10, 280), q1, None), 0.02, s.SolidColor((0.2, 0.3, 0.8))))
            world.add(s.ConstantMedium(_pyramid(s, (450, 200, 120), (450, 0, 120), 80, s.EmptyMaterial()), 0.05,
                                       s.SolidColor((0.9, 0.5, 0.1))))
            seven = s.build_box((0, 0, 0), (100, 100, 100), s.EmptyMaterial())
            seven_l = s.Hittables()
            seven_l.add(seven)
            seven_l.add(s.Quad((0, 50, 0), (100, 0, 0), (0, 0, 100), s.EmptyMaterial()))
            world.add(s.ConstantMedium(s.Transform(seven_l, (60, 300, 300), None, None), 0.02,
                                       s.SolidColor((0.1, 0.9, 0.3))))
        elif variant == "spheres":
            world.add(s.ConstantMedium(s.Sphere((170, 120, 200), 110, s.EmptyMaterial()), 0.02,
                                       s.SolidColor((0.9, 0.9, 0.9))))
            world.add(s.ConstantMedium(s.Transform(s.Sphere((0, 0, 0), 80, s.EmptyMaterial()), (380, 150, 300), q2,
                                                   (1.3, 0.8, 1.0)), 0.03, s.SolidColor((0.8, 0.2, 0.2))))
        else:  # camera and room inside one fog sphere (C5's atmosphere)
            world.add(s.ConstantMedium(s.Sphere((0, 0, 0), 5000, s.EmptyMaterial()), 0.0001,
                                       s.SolidColor((1.0, 1.0, 1.0))))
            box = s.build_box((0, 0, 0), (150, 150, 150), s.EmptyMaterial())
            world.add(s.ConstantMedium(s.Transform(box, (250, 0, 250), q1, None), 0.01, s.SolidColor((0.3, 0.3, 0.3))))
        return world, lights, cam
    out, st = render_both(gpu, oracle, rt, build)
    check(out)
    assert st["gpu"].panics == 0
    s = rt.Scene(gpu)
    w, l, c = build(s)
    assert _tier(gpu, capi, s, w, l, c) == 3
