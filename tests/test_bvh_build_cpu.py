"""BVH::from_vec (bvh.rs:16-46) as rt_bvh_new builds it: over a compact (box,
id) array, both halves of a large node at once (rt_scene.cpp bvh_build).  The
C-ABI hook rt_bvh_selftest builds the tree that way and with the plain serial
recursion on copies of a scene and compares every node (ids, children, boxes
bit for bit); here on worlds sized around the parallel threshold, with equal
box minima (the stable sort's ties), signed zeros and mixed primitives."""
import os
import random

import pytest


def _world(rt, product, n, kind, seed):
    rng = random.Random(seed)
    s = rt.Scene(product)
    mat = s.Lambertian(s.SolidColor((0.5, 0.5, 0.5)))
    lst = s.Hittables()
    for i in range(n):
        if kind == "ties":  # a coarse grid: many equal box minima on every axis
            c = (float(rng.randrange(8)), float(rng.randrange(8)), float(rng.randrange(8)))
        elif kind == "zeros":
            c = (rng.choice((0.0, -0.0, 1.0)), rng.choice((0.0, -0.0)), rng.uniform(-1, 1))
        else:
            c = (rng.uniform(-50, 50), rng.uniform(-5, 5), rng.uniform(-50, 50))
        if kind == "mixed" and i % 3 == 0:
            lst.add(s.Triangle(c, (rng.uniform(0.1, 1), 0.0, 0.0), (0.0, 0.0, rng.uniform(0.1, 1)), mat))
        elif kind == "mixed" and i % 3 == 1:
            lst.add(s.Quad(c, (0.0, rng.uniform(0.1, 1), 0.0), (0.0, 0.0, rng.uniform(0.1, 1)), mat))
        else:
            r = 0.0 if kind == "zeros" else rng.uniform(0.05, 0.5)
            lst.add(s.Sphere(c, r, mat))
    return s, lst


@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 1000, 16384, 16385, 40000])
def test_parallel_bvh_equals_serial(product, rt, n):
    s, lst = _world(rt, product, n, "random", n)
    assert product.bvh_selftest(s.s, lst.h) == 1


@pytest.mark.parametrize("kind", ["ties", "zeros", "mixed"])
def test_parallel_bvh_equals_serial_edge_boxes(product, rt, kind):
    s, lst = _world(rt, product, 50000, kind, 7)
    assert product.bvh_selftest(s.s, lst.h) == 1


def test_bvh_selftest_rejects_bad_handles(product, rt):
    s = rt.Scene(product)
    assert product.bvh_selftest(s.s, 12345) < 0
    assert product.bvh_selftest(s.s, s.Hittables().h) < 0


def test_parallel_sah_flatten_equals_serial_mesh(product, rt, scenes, tmp_path):
    """The binned-SAH rebuild at flatten (rt_scene.cpp Flattener::sah): both
    halves of large nodes at once, spliced in preorder -- the same flattened
    world as the serial build, on a C4-style terrain (80 000 triangles in
    two model BVHs beside two spheres)."""
    scenes.write_terrain_obj(str(tmp_path), 200)
    s = rt.Scene(product)
    world, lights, cam = scenes.obj_terrain(s, str(tmp_path / "terrain.obj"), 64, 1)
    assert product.world_selftest(s.s, world.h, -1, cam.background.h) == 1


def test_parallel_sah_flatten_equals_serial_spheres(product, rt):
    rng = random.Random(3)
    s = rt.Scene(product)
    mat = s.Lambertian(s.SolidColor((0.5, 0.5, 0.5)))
    lst = s.Hittables()
    for i in range(70000):
        c = (float(rng.randrange(200)) * 0.5, rng.uniform(-1, 1), float(rng.randrange(200)) * 0.5)
        lst.add(s.Sphere(c, 0.2, mat))
    world = s.Hittables()
    world.add(s.BVH(lst))
    world.add(s.Sphere((0.0, -1000.0, 0.0), 1000.0, mat))
    assert product.world_selftest(s.s, world.h, -1, -1) == 1
