"""The benchmark scenes of BASELINE.json `configs`, built through the
reference-mirroring API (raytracer.py).  Each builder takes a `Scene` (on any
implementation of the ABI) and returns (world, lights, camera).

  C1  random_spheres(scene, 400, 100)     book-1 final scene, reference CPU size
  C2  random_spheres(scene, 1920, 512)    the headline benchmark (484 traced spp)
  C3  cornell_smoke(scene, 800, 1024)     reference cornell_box + a smoke box
  C4  obj_terrain(scene, path, 1920, 256) synthetic 1M-triangle OBJ (write_terrain_obj)
  C5  final_scene(scene, 3840, 4096, 40)  reference final_scene, aspect 16/9

Scene-construction randomness (the reference calls Random:: while building,
src/main.rs:395-400, 491-499) is drawn from SplitMix64(seed) here so every
implementation receives identical objects.
"""
import json
import os

from .raytracer import Camera, Quaternion

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
MASK = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed):
        self.state = seed & MASK

    def next_u64(self):
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        return z ^ (z >> 31)

    def f64(self):
        return (self.next_u64() >> 11) * (1.0 / 9007199254740992.0)

    def range(self, lo, hi):
        return lo + (hi - lo) * self.f64()


def load_random_spheres():
    with open(os.path.join(DATA, "random_spheres_seed2025.json")) as f:
        return json.load(f)


def random_spheres(scene, image_width=400, samples_per_pixel=100, max_depth=None, spheres=None):
    """Book-1 random spheres: world = Hittables{ BVH::new(spheres) }."""
    data = load_random_spheres()
    objs = scene.Hittables()
    mats = {}
    sph = data["spheres"] if spheres is None else data["spheres"][:spheres]
    for s in sph:
        m = s["material"]
        key = json.dumps(m, sort_keys=True)
        if key not in mats:
            if m["type"] == "lambertian":
                mats[key] = scene.Lambertian(scene.SolidColor(m["albedo"]))
            elif m["type"] == "metal":
                mats[key] = scene.Metal(m["albedo"], m["fuzz"])
            else:
                mats[key] = scene.Dielectric(scene.SolidColor(m["albedo"]), m["ior"])
        objs.add(scene.Sphere(s["center"], s["radius"], mats[key]))
    world = scene.Hittables()
    world.add(scene.BVH(objs))
    c = data["camera"]
    cam = Camera()
    cam.aspect_ratio = c["aspect_ratio"]
    cam.image_width = image_width
    cam.samples_per_pixel = samples_per_pixel
    cam.max_depth = c["max_depth"] if max_depth is None else max_depth
    cam.vertical_fov_in_degrees = c["vertical_fov_in_degrees"]
    cam.look_from = tuple(c["look_from"])
    cam.look_at = tuple(c["look_at"])
    cam.vec_up = tuple(c["vec_up"])
    cam.defocus_angle_in_degrees = c["defocus_angle_in_degrees"]
    cam.focus_distance = c["focus_distance"]
    cam.background = scene.SkyGradient(data["sky"]["horizon"], data["sky"]["zenith"])
    return world, None, cam


def cornell_smoke(scene, image_width=800, samples_per_pixel=1024, max_depth=10, smoke=True):
    """src/main.rs:541-639 cornell_box(), plus (C3) a 165^3 smoke box rotated
    -18 deg about y at (130,0,65) as ConstantMedium::new_with_tex(box, 0.01,
    white) (volume.rs:23-33)."""
    api = scene.api
    red = scene.Lambertian(scene.SolidColor((0.65, 0.05, 0.05)))
    white = scene.Lambertian(scene.SolidColor((0.73, 0.73, 0.73)))
    green = scene.Lambertian(scene.SolidColor((0.12, 0.45, 0.15)))
    light = scene.DiffuseLight(scene.SolidColor((15.0, 15.0, 15.0)))
    world = scene.Hittables()
    world.add(scene.Quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green))
    world.add(scene.Quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red))
    world.add(scene.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light))
    world.add(scene.Quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white))
    world.add(scene.Quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white))
    world.add(scene.Quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    box1 = scene.build_box((0, 0, 0), (165, 330, 165), white)
    box1 = scene.Transform(box1, (265, 0, 295), Quaternion.from_axis_angle(api, (0, 1, 0), 15.0), None)
    world.add(box1)
    if smoke:
        box2 = scene.build_box((0, 0, 0), (165, 165, 165), white)
        box2 = scene.Transform(box2, (130, 0, 65), Quaternion.from_axis_angle(api, (0, 1, 0), -18.0), None)
        world.add(scene.ConstantMedium(box2, 0.01, scene.SolidColor((1.0, 1.0, 1.0))))
    lights = scene.Hittables()
    lights.add(scene.Quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light))
    cam = Camera()
    cam.aspect_ratio = 1.0
    cam.image_width = image_width
    cam.samples_per_pixel = samples_per_pixel
    cam.max_depth = max_depth
    cam.vertical_fov_in_degrees = 40.0
    cam.look_from = (278.0, 278.0, -800.0)
    cam.look_at = (278.0, 278.0, 0.0)
    cam.vec_up = (0.0, 1.0, 0.0)
    cam.defocus_angle_in_degrees = 0.0
    return world, lights, cam


def final_scene(scene, image_width=800, samples_per_pixel=5000, max_depth=40, aspect_ratio=1.0, seed=2025):
    """src/main.rs:384-539 final_scene.  The earth texture file is missing from
    the mount -> ImageTexture cyan fallback (texture.rs:167-169)."""
    api = scene.api
    g = SplitMix64(seed)
    boxes1 = scene.Hittables()
    ground = scene.Lambertian(scene.SolidColor((0.48, 0.83, 0.53)))
    for i in range(20):
        for j in range(20):
            w = 100.0
            x0 = -1000.0 + i * w
            z0 = -1000.0 + j * w
            y1 = g.range(1.0, 101.0)
            boxes1.add(scene.build_box((x0, 0.0, z0), (x0 + w, y1, z0 + w), ground))
    world = scene.Hittables()
    world.add(scene.Sphere((400, 200, 400), 100, scene.Lambertian(scene.ImageTexture(None))))
    world.add(scene.BVH(boxes1))
    light_mat = scene.DiffuseLight(scene.SolidColor((7, 7, 7)))
    world.add(scene.Quad((123, 554, 147), (300, 0, 0), (0, 0, 265), light_mat))
    world.add(scene.Sphere_new_with_motion((400, 400, 200), (430, 400, 200), 50,
                                           scene.Lambertian(scene.SolidColor((0.7, 0.3, 0.1)))))
    glass = scene.Dielectric(scene.SolidColor((1, 1, 1)), 1.5)
    world.add(scene.Sphere((260, 150, 45), 50, glass))
    world.add(scene.Sphere((0, 150, 145), 50, scene.Metal((0.8, 0.8, 0.9), 1.0)))
    world.add(scene.Sphere((360, 150, 145), 70, glass))
    boundary = scene.Sphere((360, 150, 145), 70, scene.EmptyMaterial())
    world.add(scene.ConstantMedium(boundary, 0.2, scene.SolidColor((0.2, 0.4, 0.9))))
    boundary = scene.Sphere((0, 0, 0), 5000, scene.EmptyMaterial())
    world.add(scene.ConstantMedium(boundary, 0.0001, scene.SolidColor((1, 1, 1))))
    world.add(scene.Sphere((220, 280, 300), 80, scene.Lambertian(scene.NoiseTexture(0.2, seed))))
    boxes2 = scene.Hittables()
    white = scene.Lambertian(scene.SolidColor((0.73, 0.73, 0.73)))
    for _ in range(1000):
        c = (g.range(0.0, 165.0), g.range(0.0, 165.0), g.range(0.0, 165.0))
        boxes2.add(scene.Sphere(c, 10, white))
    world.add(scene.Transform(scene.BVH(boxes2), (-100, 270, 395),
                              Quaternion.from_axis_angle(api, (0, 1, 0), 15.0), None))
    lights = scene.Hittables()
    lights.add(scene.Quad((123, 554, 147), (300, 0, 0), (0, 0, 265), scene.EmptyMaterial()))
    cam = Camera()
    cam.aspect_ratio = aspect_ratio
    cam.image_width = image_width
    cam.samples_per_pixel = samples_per_pixel
    cam.max_depth = max_depth
    cam.vertical_fov_in_degrees = 40.0
    cam.look_from = (478.0, 278.0, -600.0)
    cam.look_at = (278.0, 278.0, 0.0)
    cam.vec_up = (0.0, 1.0, 0.0)
    cam.defocus_angle_in_degrees = 0.0
    return world, lights, cam


# ---------------------------------------------------------------- C4: synthetic OBJ mesh
TERRAIN_MTL = """# two vanilla materials (obj.rs:289-298): Pm 1 -> Metal(Kd, Pr)
newmtl chrome
Kd 0.8 0.85 0.9
Pm 1.0
Pr 0.15
newmtl gold
Kd 0.9 0.7 0.3
Pm 1.0
Pr 0.45
"""


def terrain_height(x, z):
    """Displacement of the C4 terrain and its analytic gradient."""
    import numpy as np

    h = 0.35 * np.sin(1.3 * x) * np.cos(1.1 * z) + 0.12 * np.sin(3.7 * x + 1.3) * np.sin(2.9 * z) \
        + 0.04 * np.cos(9.0 * x - 7.0 * z)
    hx = 0.35 * 1.3 * np.cos(1.3 * x) * np.cos(1.1 * z) + 0.12 * 3.7 * np.cos(3.7 * x + 1.3) * np.sin(2.9 * z) \
        - 0.04 * 9.0 * np.sin(9.0 * x - 7.0 * z)
    hz = -0.35 * 1.1 * np.sin(1.3 * x) * np.sin(1.1 * z) + 0.12 * 2.9 * np.sin(3.7 * x + 1.3) * np.cos(2.9 * z) \
        + 0.04 * 7.0 * np.sin(9.0 * x - 7.0 * z)
    return h, hx, hz


def write_terrain_obj(directory, cells=707, extent=4.0):
    """Writes terrain.obj + terrain.mtl: a (cells x cells)-quad displaced grid
    over [-extent, extent]^2 (2*cells^2 triangles; cells=707 -> 999 698), every
    corner `v/vt/vn` with one shared index, analytic vertex normals, texture
    coordinates (i/cells, j/cells).  Two objects (x < 0: `chrome`, x >= 0:
    `gold`) so the loader's per-model BVHs and usemtl handling are exercised.
    Deterministic: the same cells give the same bytes."""
    import numpy as np

    os.makedirs(directory, exist_ok=True)
    n = cells + 1
    g = np.linspace(-extent, extent, n)
    X, Z = np.meshgrid(g, g, indexing="ij")  # [i, j] -> (x_i, z_j)
    H, HX, HZ = terrain_height(X, Z)
    N = np.stack([-HX, np.ones_like(HX), -HZ], axis=-1)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    U, V = np.meshgrid(np.arange(n) / cells, np.arange(n) / cells, indexing="ij")
    obj = os.path.join(directory, "terrain.obj")
    with open(os.path.join(directory, "terrain.mtl"), "w") as f:
        f.write(TERRAIN_MTL)
    with open(obj, "w") as f:
        f.write("# synthetic C4 terrain: %d x %d cells, %d triangles\nmtllib terrain.mtl\n" % (cells, cells, 2 * cells * cells))
        np.savetxt(f, np.stack([X.ravel(), H.ravel(), Z.ravel()], 1), fmt="v %.6f %.6f %.6f")
        np.savetxt(f, np.stack([U.ravel(), V.ravel()], 1), fmt="vt %.6f %.6f")
        np.savetxt(f, N.reshape(-1, 3), fmt="vn %.6f %.6f %.6f")
        idx = np.arange(n * n).reshape(n, n) + 1  # 1-based
        a, b, c, d = idx[:-1, :-1], idx[1:, :-1], idx[1:, 1:], idx[:-1, 1:]
        half = cells // 2
        for name, sl in (("chrome", slice(0, half)), ("gold", slice(half, cells))):
            f.write("o terrain_%s\nusemtl %s\n" % (name, name))
            # two counter-clockwise (seen from +y) triangles per cell
            t1 = np.stack([a[sl], d[sl], c[sl]], -1).reshape(-1, 3)
            t2 = np.stack([a[sl], c[sl], b[sl]], -1).reshape(-1, 3)
            tris = np.stack([t1, t2], 1).reshape(-1, 3)
            np.savetxt(f, np.repeat(tris, 3, axis=1), fmt="f %d/%d/%d %d/%d/%d %d/%d/%d")
    return obj


def obj_terrain(scene, obj_path, image_width=1920, samples_per_pixel=256, max_depth=50):
    """C4: world = Hittables{ Wavefont(terrain.obj) (one BVH per
    model), a glass and a diffuse sphere }, sky background."""
    world = scene.Hittables()
    world.add(scene.Wavefont(obj_path, True))
    world.add(scene.Sphere((-0.9, 1.0, 0.6), 0.45, scene.Dielectric(scene.SolidColor((1.0, 1.0, 1.0)), 1.5)))
    world.add(scene.Sphere((1.1, 0.95, -0.3), 0.4, scene.Lambertian(scene.SolidColor((0.7, 0.2, 0.15)))))
    cam = Camera()
    cam.aspect_ratio = 16.0 / 9.0
    cam.image_width = image_width
    cam.samples_per_pixel = samples_per_pixel
    cam.max_depth = max_depth
    cam.vertical_fov_in_degrees = 40.0
    cam.look_from = (0.0, 3.4, 6.8)
    cam.look_at = (0.0, 0.0, 0.0)
    cam.vec_up = (0.0, 1.0, 0.0)
    cam.defocus_angle_in_degrees = 0.0
    cam.focus_distance = 10.0
    cam.background = scene.SkyGradient((1.0, 1.0, 1.0), (0.5, 0.7, 1.0))
    return world, None, cam
