"""Test data (not a test module): a small OBJ / MTL whose materials use every
image map obj.rs:212-345 reads -- map_Kd on a vanilla Metal and a Dielectric,
map_Ke, map_d (Mix::from_image), map_Bump -- with PNGs written by PIL."""
import numpy as np

IMG_MTL = """newmtl tile
Kd 0.5 0.5 0.5
Pm 1
Pr 0.2
map_Kd albedo.png
newmtl glass
Tf 1 1 1
Ni 1.5
map_Kd albedo.png
newmtl lamp
Kd 0.6 0.6 0.6
Pm 1
Pr 0.4
map_Ke emit.png
newmtl leaf
Kd 0.3 0.8 0.3
Pm 1
Pr 0.6
map_d alpha.png
newmtl lampleaf
Kd 0.8 0.8 0.8
Pm 1
Pr 0.3
Ke 0.5 0.2 0.1
map_Ke emit.png
map_d alpha.png
newmtl bumpy
Kd 0.7 0.7 0.9
Pm 1
Pr 0.1
map_Bump -bm 1.000000 normal.png
"""


def _img_obj(names):
    """One quad per model (two triangles, v/vt/vn), side by side."""
    lines = ["mtllib m.mtl"]
    vi = 0
    for k, name in enumerate(names):
        x0 = -3.0 + 1.2 * k
        y0 = 0.2 + 0.3 * (k % 2)
        for (x, y, z) in ((x0, y0, -0.5), (x0 + 1.0, y0, -0.5), (x0 + 1.0, y0 + 1.0, -0.3), (x0, y0 + 1.0, -0.3)):
            lines.append(f"v {x} {y} {z}")
        for (u, v) in ((0.05, 0.1), (1.9, 0.0), (2.1, 1.7), (-0.2, 1.1)):  # wraps past [0, 1]
            lines.append(f"vt {u} {v}")
        for (a, b, c) in ((0.1, 0.2, 1.0), (-0.1, 0.1, 1.0), (0.0, -0.2, 1.0), (0.2, 0.0, 1.0)):
            lines.append(f"vn {a} {b} {c}")
        lines.append(f"o {name}")
        lines.append(f"usemtl {name}")
        i = vi + 1
        lines.append(f"f {i}/{i}/{i} {i + 1}/{i + 1}/{i + 1} {i + 2}/{i + 2}/{i + 2} {i + 3}/{i + 3}/{i + 3}")
        vi += 4
    return "\n".join(lines) + "\n"


def _write_images(d):
    from PIL import Image
    rng = np.random.default_rng(5)
    Image.fromarray(rng.integers(0, 256, size=(12, 20, 3), dtype=np.uint8), "RGB").save(str(d / "albedo.png"))
    e = np.zeros((8, 8, 3), dtype=np.uint8)
    e[::2, :, 0] = 255
    e[:, ::3, 2] = 200
    Image.fromarray(e, "RGB").save(str(d / "emit.png"))
    a = rng.integers(0, 256, size=(10, 10, 4), dtype=np.uint8)
    a[..., 3] = np.where(a[..., 3] > 128, 255, 0)  # alpha 0 / 1 regions plus the interpolation-free middle
    a[4:6, :, 3] = 100
    Image.fromarray(a, "RGBA").save(str(d / "alpha.png"))
    n = np.zeros((16, 16, 3), dtype=np.uint8)
    n[..., 0] = 128 + (np.arange(16)[None, :] * 6)
    n[..., 1] = 128
    n[..., 2] = 230
    Image.fromarray(n, "RGB").save(str(d / "normal.png"))




def write_scene(d, names):
    """scene.obj with one quad per model in `names`, m.mtl with their
    materials in model order (obj.rs:129 zips models with materials), PNGs."""
    blocks = {b.split("\n", 1)[0]: "newmtl " + b for b in IMG_MTL.split("newmtl ")[1:]}
    (d / "m.mtl").write_text("".join(blocks[n] for n in names))
    (d / "scene.obj").write_text(_img_obj(names))
    _write_images(d)
    return str(d / "scene.obj")
