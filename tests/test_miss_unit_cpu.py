"""The basic tier's miss under a sky gradient (rt_kernel.hip shade, miss
branch) makes only the unit direction's y quotient.  Its panic flag must be
the one unit() gives (rt_math.h: u = v / |v|, ok = every u_i finite), which
the kernel states as: |v| not NaN, not 0, and every v_i finite.  This checks
the two statements agree over random, scaled and special directions in IEEE
double (numpy rounds each operation as the device code does: -ffp-contract=off),
and that the y quotient is the same double either way."""
import numpy as np


def _len(v):
    return np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2])


def _ok_unit(v):  # unit() = divs(v, |v|) = (1 / |v|) * v (rt_math.h, vec3.rs:225-232): every product finite
    l = _len(v)
    u = (1.0 / l)[:, None] * v
    return np.isfinite(u).all(axis=1), u[:, 1]


def _ok_sky(v):  # the kernel's statement (rt_kernel.hip shade, basic tier's sky miss)
    l = _len(v)
    return ~(np.isnan(l) | (l == 0.0) | ~np.isfinite(v).all(axis=1)), ((1.0 / l) * v[:, 1])


def test_division_form_differs_from_reciprocal_form():
    """d.y / l is not (1 / l) * d.y: the y the gradient reads must be made the
    reference's way, and this shows the check can tell them apart."""
    rng = np.random.default_rng(7)
    v = rng.standard_normal((20000, 3))
    l = _len(v)
    assert ((v[:, 1] / l) != ((1.0 / l) * v[:, 1])).mean() > 0.05


def _cases():
    rng = np.random.default_rng(2025)
    out = [rng.standard_normal((20000, 3))]
    for e in list(range(-330, -290, 2)) + list(range(-170, -140, 2)) + list(range(140, 170, 2)) + list(range(290, 309)):
        out.append(rng.standard_normal((400, 3)) * 10.0 ** e)
    specials = [0.0, -0.0, 5e-324, -5e-324, 1e-310, 1e-160, 1e154, 1e300, 1.7976931348623157e308,
                np.inf, -np.inf, np.nan, 1.0, -1.0]
    s = np.array(specials)
    grid = np.array(np.meshgrid(s, s, s)).reshape(3, -1).T
    out.append(grid)
    # one component dominating, the others tiny or zero
    big = rng.standard_normal((2000, 3))
    big[:, 0] *= 1e200
    big[:, 1:] *= 1e-200
    out.append(big)
    return np.concatenate(out)


def test_sky_miss_panic_flag_matches_unit():
    with np.errstate(all="ignore"):
        v = _cases()
        ok_u, y_u = _ok_unit(v)
        ok_s, y_s = _ok_sky(v)
    assert (ok_u == ok_s).all(), v[ok_u != ok_s][:5]
    # the y the gradient reads: the same double (NaN where both are NaN)
    same = (y_u == y_s) | (np.isnan(y_u) & np.isnan(y_s))
    assert same.all()
    # both outcomes occur among the cases
    assert ok_u.any() and (~ok_u).any()
