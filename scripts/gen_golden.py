#!/usr/bin/env python3
"""Golden render vectors from the TEST-ONLY oracle (reference-semantics CPU
restatement): small frames of the C1 / C3 / C4 / C5 scenes and two full-width
rows of the headline C2 frame at fixed seeds, stored as linear f64 (npy) in
tests/golden/.  They pin the oracle against itself
across changes (regression) and give GPU tests a fixture that does not need
the oracle at run time.  The reference itself cannot produce them (no Rust
toolchain; unseedable RNG) -- see DESIGN.md §2."""
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")

def terrain(cells):
    """The C4 synthetic OBJ at `cells` (deterministic bytes), cached under TMPDIR."""
    import tempfile
    d = os.path.join(tempfile.gettempdir(), "rt_terrain_%d" % cells)
    p = os.path.join(d, "terrain.obj")
    if not os.path.exists(p):
        scenes.write_terrain_obj(d, cells)
    return p


# name -> (scene builder, render seed[, (row_offset, row_stride)]: a row shard
# of the frame, rows y = row_offset + k * row_stride)
CASES = {
    "c1_64x36_s16_seed7": (lambda s: scenes.random_spheres(s, 64, 16), 7),
    "c3_48x48_s16_seed7": (lambda s: scenes.cornell_smoke(s, 48, 16), 7),
    "c5_64x36_s16_seed7": (lambda s: scenes.final_scene(s, 64, 16, 40, aspect_ratio=16 / 9), 7),
    "c4_64x36_s16_seed7": (lambda s: scenes.obj_terrain(s, terrain(16), 64, 16), 7),
    # the headline C2 geometry (BASELINE configs[1]): two full-width rows of
    # the 1920x1080 frame (y = 270 and 810) at 16 spp, depth 50
    "c2_1920x1080_rows270_810_s16_seed7": (lambda s: scenes.random_spheres(s, 1920, 16), 7, (270, 540)),
}


def case(name):
    """(build, seed, row_offset, row_stride) of a golden case."""
    c = CASES[name]
    off, stride = c[2] if len(c) > 2 else (0, 1)
    return c[0], c[1], off, stride


def render(api, build, seed, row_offset=0, row_stride=1):
    scene = rt.Scene(api)
    world, lights, cam = build(scene)
    c = cam.to_c()
    opts = capi.RtRenderOpts()
    api.render_opts_default(ctypes.byref(opts))
    opts.seed = seed
    opts.row_offset = row_offset
    opts.row_stride = row_stride
    rows = api.shard_rows(ctypes.byref(c), ctypes.byref(opts))
    out = np.zeros((rows, cam.image_width, 3), dtype=np.float64)
    api.check(api.render_f64(scene.s, world.h, -1 if lights is None else lights.h, ctypes.byref(c), ctypes.byref(opts),
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), None, None, None))
    return out


def main():
    api = capi.Api(ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle.so")), "orc_", capi.ORACLE_EXTRAS)
    os.makedirs(os.path.join(ROOT, "tests", "golden"), exist_ok=True)
    only = set(sys.argv[1:])  # names to (re)write; default all
    for name in CASES:
        if only and name not in only:
            continue
        build, seed, off, stride = case(name)
        img = render(api, build, seed, off, stride)
        np.save(os.path.join(ROOT, "tests", "golden", name + ".npy"), img)
        print(name, img.shape, img.mean(axis=(0, 1)))


if __name__ == "__main__":
    main()
