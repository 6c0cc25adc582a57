#!/usr/bin/env python3
"""Generate the book-1 random-spheres scene fixture.

The reference has no book-1 final scene in src/main.rs, so the
build assembles it through the reference constructors (Sphere::new,
Lambertian, Metal, Dielectric; src/shapes/sphere.rs:25, src/material.rs).  The
scene generator draws random numbers, and the reference RNG is unseedable
(src/utils/random.rs:8-14), so the scene is drawn once from SplitMix64(2025)
and committed as raytracer-2025_amd/data/random_spheres_seed2025.json.

Draw order follows "Ray Tracing in One Weekend" §14.1 (the scene this config
names): per cell choose_mat, centre.x, centre.z; Lambertian albedo =
Color::random() * Color::random(); Metal albedo = Color::random_range(0.5..1),
fuzz = random_range(0..0.5).  U[0,1) = (u64 >> 11) * 2^-53.
"""
import json
import os
import sys

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


def generate(seed=2025):
    g = SplitMix64(seed)
    spheres = [{"center": [0.0, -1000.0, 0.0], "radius": 1000.0, "material": {"type": "lambertian", "albedo": [0.5, 0.5, 0.5]}}]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose_mat = g.f64()
            cx = a + 0.9 * g.f64()
            cz = b + 0.9 * g.f64()
            center = [cx, 0.2, cz]
            d = ((cx - 4.0) ** 2 + (0.2 - 0.2) ** 2 + (cz - 0.0) ** 2) ** 0.5
            if d <= 0.9:
                continue
            if choose_mat < 0.8:
                c1 = [g.f64(), g.f64(), g.f64()]
                c2 = [g.f64(), g.f64(), g.f64()]
                mat = {"type": "lambertian", "albedo": [c1[i] * c2[i] for i in range(3)]}
            elif choose_mat < 0.95:
                albedo = [g.range(0.5, 1.0), g.range(0.5, 1.0), g.range(0.5, 1.0)]
                mat = {"type": "metal", "albedo": albedo, "fuzz": g.range(0.0, 0.5)}
            else:
                mat = {"type": "dielectric", "albedo": [1.0, 1.0, 1.0], "ior": 1.5}
            spheres.append({"center": center, "radius": 0.2, "material": mat})
    spheres.append({"center": [0.0, 1.0, 0.0], "radius": 1.0, "material": {"type": "dielectric", "albedo": [1.0, 1.0, 1.0], "ior": 1.5}})
    spheres.append({"center": [-4.0, 1.0, 0.0], "radius": 1.0, "material": {"type": "lambertian", "albedo": [0.4, 0.2, 0.1]}})
    spheres.append({"center": [4.0, 1.0, 0.0], "radius": 1.0, "material": {"type": "metal", "albedo": [0.7, 0.6, 0.5], "fuzz": 0.0}})
    return {
        "generator": "scripts/gen_random_spheres.py SplitMix64",
        "seed": seed,
        "camera": {
            "aspect_ratio": 16.0 / 9.0,
            "vertical_fov_in_degrees": 20.0,
            "look_from": [13.0, 2.0, 3.0],
            "look_at": [0.0, 0.0, 0.0],
            "vec_up": [0.0, 1.0, 0.0],
            "defocus_angle_in_degrees": 0.6,
            "focus_distance": 10.0,
            "max_depth": 50,
        },
        "sky": {"horizon": [1.0, 1.0, 1.0], "zenith": [0.5, 0.7, 1.0]},
        "spheres": spheres,
    }


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "raytracer-2025_amd", "data", "random_spheres_seed2025.json")
    scene = generate()
    with open(out, "w") as f:
        json.dump(scene, f, indent=1)
    print(f"{len(scene['spheres'])} spheres -> {out}")
