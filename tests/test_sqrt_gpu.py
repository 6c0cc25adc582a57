"""The kernel's f64 square root (rt_math.h k_sqrt, every sqrt of the path)
against IEEE sqrt (numpy: correctly rounded), bit for bit, through
rt_math_selftest (fn 7, impl 0).  With RT_FAST_SQRT a wave whose arguments are
all in [2^-767, inf) runs the Newton sequence without LLVM's scaling and
special-case steps, and any other wave runs sqrt(); so the arguments come in
64-lane groups (one wave each): groups wholly in range (every binade, the
binades next to 2^-767, the path's [0, 1] draws), and groups with one lane out
of range (0, -0, subnormals, 2^-800, just below 2^-767, inf, NaN, negatives) at
varied positions."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LO = 2.0 ** -767


def _sqrt_gpu(gpu, a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    P = ctypes.POINTER(ctypes.c_double)
    gpu.check(gpu.math_selftest(7, 0, a.ctypes.data_as(P), None, out.ctypes.data_as(P), a.size))
    return out


def _same_bits(x, y):
    both_nan = np.isnan(x) & np.isnan(y)
    return both_nan | (x.view(np.uint64) == y.view(np.uint64))


def _in_range_groups(rng):
    groups = []
    # every binade from 2^-767 up: random mantissas
    e = rng.integers(-767, 1024, size=64 * 400)
    m = rng.random(64 * 400) + 1.0
    groups.append(np.ldexp(m, e).clip(LO, np.finfo(np.float64).max))
    # the binades next to the threshold, and the threshold's neighbours above it
    groups.append(np.ldexp(rng.random(64 * 50) + 1.0, rng.integers(-767, -760, size=64 * 50)))
    groups.append(np.nextafter(np.full(64, LO), np.inf) * (1.0 + np.arange(64) * 2.0 ** -52))
    groups.append(np.full(64, LO))
    # the path's arguments: unit draws and 1 - x^2 style values, |d|^2 of directions
    xi = (rng.integers(1, 2 ** 53, size=64 * 400) >> 0).astype(np.float64) * 2.0 ** -53
    groups.append(xi)
    groups.append(1.0 - xi * xi)
    groups.append(xi * (1.0 - xi))
    d = rng.normal(size=(64 * 200, 3))
    groups.append((d * d).sum(axis=1))
    groups.append(np.full(64, np.finfo(np.float64).max))
    a = np.concatenate(groups)
    a = a[a >= LO]
    return a[: (a.size // 64) * 64]


def test_sqrt_in_range_waves(gpu):
    a = _in_range_groups(np.random.default_rng(11))
    ours = _sqrt_gpu(gpu, a)
    ok = _same_bits(ours, np.sqrt(a))
    assert ok.all(), (int((~ok).sum()), float(a[~ok][0]).hex(), float(ours[~ok][0]).hex())


def test_sqrt_mixed_waves(gpu):
    rng = np.random.default_rng(12)
    specials = [0.0, -0.0, 5e-324, 2.0 ** -1030, 2.0 ** -800, np.nextafter(LO, 0.0), LO / 2, np.inf, -np.inf,
                np.nan, -1.0, -LO, -5e-324, 2.0 ** -1022]
    groups = []
    for k, s in enumerate(specials):
        for pos in (0, 1, 31, 32, 63, (7 * k) % 64):
            g = np.ldexp(rng.random(64) + 1.0, rng.integers(-767, 1000, size=64))
            g[pos] = s
            groups.append(g)
    groups.append(np.array(specials * 5)[:64])  # a wave of specials only
    a = np.concatenate(groups)
    with np.errstate(invalid="ignore"):
        ref = np.sqrt(a)
    ours = _sqrt_gpu(gpu, a)
    ok = _same_bits(ours, ref)
    assert ok.all(), (int((~ok).sum()), float(a[~ok][0]).hex(), float(ours[~ok][0]).hex())
    # IEEE: sqrt(-0) = -0, sqrt(+inf) = +inf
    z = _sqrt_gpu(gpu, np.array([-0.0] + [1.0] * 63))
    assert np.signbit(z[0]) and z[0] == 0.0
