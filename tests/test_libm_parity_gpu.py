"""Where the remaining GPU-vs-oracle divergence comes from.  The kernel's
transcendentals are correctly rounded (rt_crmath.h); glibc's -- what the
oracle and Rust's f64 functions call -- are correctly rounded on ~99.9 % of
arguments (tests/test_crmath_cpu.py).  Against liboracle_cr.so (the same
oracle with its path libm calls on rt_crmath.h) the kernel must be exact: RMSE
0 and no diverged (pixel, s_i) sum, on the knife-edge checker (a floor on
y = 0, where an ulp anywhere upstream picks the other square) and on C5 /
C3 rows (40-bounce paths, media, Perlin).  Against the default glibc oracle
the residual is then glibc's own misrounding, printed per test."""
import pytest

from test_lights_textures_gpu import checker_world
from test_parity_gpu import check, render_both, rows_vs_oracle

pytestmark = pytest.mark.gpu


def _exact(out):
    # the kernel's loop (beta * L) and the oracle's recursion agree to ~1e-15
    # relative on equal paths: every pixel within 1e-5, no diverged sum
    check(out, tol=1e-9, min_exact=1.0, max_div=0.0)


def test_knife_edge_checker_exact(gpu, oracle_cr, rt):
    out, st = render_both(gpu, oracle_cr, rt, lambda s: checker_world(rt, s, "quad_y0"))
    _exact(out)


def test_c5_rows_exact(gpu, oracle_cr, rt, scenes):
    def build(s):
        return scenes.final_scene(s, 3840, 64, 40, aspect_ratio=16 / 9)
    g, o, gp, op = rows_vs_oracle(gpu, oracle_cr, rt, build, 1, [(1080, 2160)])
    _exact({"gpu": (g, None, gp), "oracle": (o, None, op)})


def test_c3_rows_exact(gpu, oracle_cr, rt, scenes):
    def build(s):
        return scenes.cornell_smoke(s, 800, 256)
    g, o, gp, op = rows_vs_oracle(gpu, oracle_cr, rt, build, 1, [(400, 800)])
    _exact({"gpu": (g, None, gp), "oracle": (o, None, op)})


def test_c5_small_exact(gpu, oracle_cr, rt, scenes):
    out, _ = render_both(gpu, oracle_cr, rt, lambda s: scenes.final_scene(s, 128, 16, 40, aspect_ratio=16 / 9))
    _exact(out)
