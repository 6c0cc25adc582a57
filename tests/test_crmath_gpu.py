"""Device f64 transcendentals against glibc (what Rust's f64::sin / cos / ln /
acos / atan2 call on Linux, and what the oracle calls): the render kernel's
correctly rounded functions (rt_crmath.h, impl 0 of rt_math_selftest) and
ROCm's device libm (ocml, impl 1, what the kernel used before), on the
committed argument sets of tests/golden/crmath_args.npz -- the ranges the path
feeds them: 2 pi xi (vec3.rs:313-343), NoiseTexture arguments
(texture.rs:191-196), ln xi (volume.rs:58), sphere / environment uv
(sphere.rs:53-61, environment.rs:14-24), square roots.

Bar: the kernel's functions return the correctly rounded value bit for bit on
every argument (so they disagree with glibc exactly where glibc is not
correctly rounded, ~0.1 %); the per-function disagreement rates of both
implementations with glibc are printed and written to
gpurun_out/crmath_rates.json."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

FAMILIES = ["sin_2pi_xi", "cos_2pi_xi", "sincos_sin", "sin_noise", "cos_noise", "log_xi", "acos_uv", "atan2_uv", "sqrt"]


def _eval(gpu, fn, impl, a, b):
    out = np.empty_like(a)
    P = ctypes.POINTER(ctypes.c_double)
    bp = b.ctypes.data_as(P) if fn == 6 else None
    gpu.check(gpu.math_selftest(fn, impl, a.ctypes.data_as(P), bp, out.ctypes.data_as(P), a.size))
    return out


def test_device_math_vs_glibc(gpu):
    d = np.load(os.path.join(ROOT, "tests", "golden", "crmath_args.npz"))
    rates, bad = {}, {}
    for name in FAMILIES:
        fn = int(d[name + "_fn"])
        a = np.ascontiguousarray(d[name + "_a"])
        b = np.ascontiguousarray(d[name + "_b"])
        g, cr = d[name + "_glibc"], d[name + "_cr"]
        ours = _eval(gpu, fn, 0, a, b)
        ocml = _eval(gpu, fn, 1, a, b)
        rates[name] = {
            "n": int(a.size),
            "kernel_ne_glibc": float((ours != g).mean()),
            "ocml_ne_glibc": float((ocml != g).mean()),
            "glibc_not_correctly_rounded": float((g != cr).mean()),
            "ocml_not_correctly_rounded": float((ocml != cr).mean()),
        }
        miss = int((ours != cr).sum())
        if miss:
            i = int(np.argmax(ours != cr))
            bad[name] = (miss, float(a[i]).hex(), float(ours[i]).hex(), float(cr[i]).hex())
        print("%-11s kernel!=glibc %.2e  ocml!=glibc %.2e  (glibc misrounded %.2e, ocml misrounded %.2e)" %
              (name, rates[name]["kernel_ne_glibc"], rates[name]["ocml_ne_glibc"],
               rates[name]["glibc_not_correctly_rounded"], rates[name]["ocml_not_correctly_rounded"]))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "crmath_rates.json"), "w") as f:
        json.dump(rates, f, indent=1)
    assert not bad, bad


def test_device_math_specials(gpu):
    """IEEE specials through the kernel's functions, as glibc returns them."""
    import math

    cases = {
        0: [0.0, -0.0, math.inf, -math.inf, math.nan, 1e300, -3e22, 2.0 ** 20, 2.0 ** 20 + 1],
        1: [0.0, -0.0, math.inf, math.nan, 1e300, 2.0 ** 600],
        4: [0.0, -0.0, -1.0, 1.0, math.inf, math.nan, 5e-324, 1.7976931348623157e308],
        5: [1.0, -1.0, 0.0, -0.0, 1.0000000000000002, -1.0000000000000002, math.nan],
    }
    libm = ctypes.CDLL("libm.so.6")
    for fn, name in ((0, "sin"), (1, "cos"), (4, "log"), (5, "acos")):
        f = getattr(libm, name)
        f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double]
        a = np.array(cases[fn], dtype=np.float64)
        ours = _eval(gpu, fn, 0, a, a)
        want = np.array([f(x) for x in a])
        same = (ours == want) | (np.isnan(ours) & np.isnan(want))
        assert same.all(), (name, a[~same], ours[~same], want[~same])
    f = libm.atan2
    f.restype, f.argtypes = ctypes.c_double, [ctypes.c_double, ctypes.c_double]
    sp = [0.0, -0.0, 1.0, -1.0, math.inf, -math.inf, 1e-300, -1e300]
    ys = np.array([y for y in sp for _ in sp]), np.array([x for _ in sp for x in sp])
    ours = _eval(gpu, 6, 0, np.ascontiguousarray(ys[0]), np.ascontiguousarray(ys[1]))
    want = np.array([f(y, x) for y, x in zip(*ys)])
    assert (np.signbit(ours) == np.signbit(want)).all() and (ours == want).all()


def test_device_sincos_2pi_matches_sincos(gpu):
    """rtcr::sincos_2pi(xi) -- what every sincos of the kernel calls, the
    argument 2.0 * PI * xi formed inside -- returns the same doubles as
    rtcr::sincos(2.0 * PI * xi) (pinned above against the correctly rounded
    values) on the path's draws and on xi stepped ulp by ulp around every
    k / 256 (x next to each k pi/128 of its reduction), 0 and 1."""
    rng = np.random.default_rng(2025)
    xi = [(rng.integers(0, 1 << 53, 200000, dtype=np.int64) * 2.0 ** -53)]
    near = []
    for k in range(257):
        c = k / 256.0
        lo = hi = c
        near.append(c)
        for _ in range(24):
            lo, hi = np.nextafter(lo, -1.0), np.nextafter(hi, 2.0)
            if lo >= 0.0:
                near.append(lo)
            if hi <= 1.0:
                near.append(hi)
    xi.append(np.array(near + [0.0, 1.0, 2.0 ** -53, 1.0 - 2.0 ** -53]))
    xi = np.ascontiguousarray(np.concatenate(xi))
    x = 2.0 * np.pi * xi  # the same double as the kernel's 2.0 * PI * xi
    for fn2, fn in ((8, 2), (9, 3)):
        got, want = _eval(gpu, fn2, 0, xi, xi), _eval(gpu, fn, 0, x, x)
        diff = got != want
        assert not diff.any(), (fn2, int(diff.sum()), float(xi[np.argmax(diff)]).hex())
