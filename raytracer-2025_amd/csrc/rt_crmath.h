// rt_crmath.h -- correctly rounded f64 sin, cos, sincos, log, atan2, acos,
// one source for the gfx950 kernel and for host code (g++ / hipcc host pass).
//
// Why: the reference calls Rust's f64::sin / cos / ln / acos / atan2, which on
// Linux are glibc's libm.  ROCm's ocml versions differ from glibc
// by an ulp on a sizeable fraction of arguments, and one ulp in a bounce
// direction is enough to flip a knife-edge decision downstream (a checker
// square on the y = 0 plane, an edge between two boxes).  glibc is correctly
// rounded on ~99.9 % of arguments (tests/test_crmath_cpu.py measures it
// against libquadmath), so a correctly rounded device function agrees with
// glibc wherever glibc is correctly rounded.
//
// How (Ziv's strategy): a fast path evaluates the function as a double-double
// yh + yl with a rigorous error bound err, and returns yh when yh +- err round
// alike; otherwise (about 1 call in 10^4-10^5) a slow path evaluates it in
// double-double arithmetic to ~2^-100 and rounds that.  Reductions:
//   sin / cos: x = k pi/128 + r, |r| <= pi/256 (Cody-Waite with a 26-bit first
//     constant below 2^20, Payne-Hanek with the 128/pi bits above), then
//     sin x = S cos r + C sin r with S, C = sin / cos(k pi/128) from a
//     256-record table (8 KiB, L1-resident); sincos_2pi(xi) for the path's
//     x = 2 pi xi in [0, 2pi] with 44-bit constants and no range branches.
//   log: x = 2^e z, r = z c - 1 exact as a double-double (|r| < 2^-7), then
//     log x = e ln2 - log c + log1p(r); c = 1 around 1, so log x near 1 is
//     log1p(r) without cancellation.
//   atan2 / acos: t = min/max (double-double quotient), t = j/64 + ...,
//     atan t = atan(j/64) + atan((t - c)/(1 + t c)); acos y = atan2(sqrt((1-y)
//     (1+y)), y) with the square root as a double-double.
// Tables: rt_crmath_tables.h (scripts/gen_crmath_tables.py, 160-digit decimal).
// Needs FMA contraction off for its own plain operations (the kernel and the
// oracle are built with -ffp-contract=off; the functions also say so).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTCR_FN __host__ __device__ inline
#if defined(RTCR_SLOW_NOINLINE)
#define RTCR_SLOW __host__ __device__ __attribute__((noinline))
#else
#define RTCR_SLOW __host__ __device__ inline
#endif
#else
#define RTCR_FN static inline
#define RTCR_SLOW static inline
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define RTCR_TABLE static __constant__ const
#else
#define RTCR_TABLE static const
#endif
#if defined(__clang__)
#define RTCR_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define RTCR_NOCONTRACT
#endif

#include "rt_crmath_tables.h"
#if defined(RTCR_SLOW_COUNTER) && !defined(__HIP_DEVICE_COMPILE__)
#define RTCR_COUNT_SLOW() (++(RTCR_SLOW_COUNTER))
#else
#define RTCR_COUNT_SLOW() ((void)0)
#endif

namespace rtcr {

struct DD {
    double h, l;
};

RTCR_FN double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
RTCR_FN double abs_(double a) { return __builtin_fabs(a); }
RTCR_FN uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
RTCR_FN double from_bits(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}
RTCR_FN DD two_sum(double a, double b) {
    RTCR_NOCONTRACT
    const double s = a + b, bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
RTCR_FN DD fast_two_sum(double a, double b) {  // |a| >= |b| (or a = 0)
    RTCR_NOCONTRACT
    const double s = a + b;
    return DD{s, b - (s - a)};
}
RTCR_FN DD two_prod(double a, double b) {
    const double p = a * b;
    return DD{p, fma_(a, b, -p)};
}
RTCR_FN DD dd_neg(DD a) { return DD{-a.h, -a.l}; }
// a + b, no massive cancellation between a and b
RTCR_FN DD dd_add(DD a, DD b) {
    RTCR_NOCONTRACT
    const DD s = two_sum(a.h, b.h);
    return fast_two_sum(s.h, s.l + a.l + b.l);
}
// a + b, any cancellation
RTCR_FN DD dd_add_acc(DD a, DD b) {
    RTCR_NOCONTRACT
    DD s = two_sum(a.h, b.h);
    const DD t = two_sum(a.l, b.l);
    s = fast_two_sum(s.h, s.l + t.h);
    return fast_two_sum(s.h, s.l + t.l);
}
RTCR_FN DD dd_mul(DD a, DD b) {
    RTCR_NOCONTRACT
    DD p = two_prod(a.h, b.h);
    p.l = fma_(a.h, b.l, fma_(a.l, b.h, p.l));
    return fast_two_sum(p.h, p.l);
}
RTCR_FN DD dd_mul_d(DD a, double b) {
    DD p = two_prod(a.h, b);
    p.l = fma_(a.l, b, p.l);
    return fast_two_sum(p.h, p.l);
}
// round-to-nearest of every value within err of yh + yl is the same double
RTCR_FN bool rounds_ok(double yh, double yl, double err) {
    RTCR_NOCONTRACT
    return yh + (yl + err) == yh + (yl - err);
}

// ------------------------------------------------------------------ sin / cos
// sin / cos (k pi/128) from the table: S = sin, C = cos (double-doubles)
RTCR_FN void sc_table(int k, DD& S, DD& C) {
    const double* e = RTCR_SC_PIO128[k & 255];  // one 32-B record: no quadrant folding
    S = DD{e[0], e[1]};
    C = DD{e[2], e[3]};
}

// |x| <= 2^20: x = k pi/128 + (rh + rl), |error| < 2^-108
RTCR_FN void reduce_fast(double x, double& rh, double& rl, int& k) {
    RTCR_NOCONTRACT
    const double kd = __builtin_rint(x * RTCR_INV_PIO128);
    const double y1 = fma_(-kd, RTCR_PIO128_1, x);  // exact (k C1 has <= 53 bits, Sterbenz)
    const DD p2 = two_prod(kd, RTCR_PIO128_2);
    const DD s = two_sum(y1, -p2.h);
    const double lo = (s.l - p2.l) - kd * RTCR_PIO128_3;
    const DD r = two_sum(s.h, lo);
    rh = r.h;
    rl = r.l;
    k = (int)(int64_t)kd;
}

// |x| <= 2^20, four constants: |error| < 2^-150 + 2^-105 |r|
RTCR_FN void reduce_slow(double x, DD& r, int& k) {
    RTCR_NOCONTRACT
    const double kd = __builtin_rint(x * RTCR_INV_PIO128);
    const double y1 = fma_(-kd, RTCR_PIO128_1, x);
    const DD p2 = two_prod(kd, RTCR_PIO128_2), p3 = two_prod(kd, RTCR_PIO128_3);
    const double p4 = kd * RTCR_PIO128_4;
    const DD s = two_sum(y1, -p2.h);
    const DD u = two_sum(s.l, -p2.l);
    const DD v = two_sum(u.h, -p3.h);
    const double lo = ((u.l + v.l) - p3.l) - p4;
    DD w = two_sum(s.h, v.h);
    w = two_sum(w.h, w.l + lo);
    r = w;
    k = (int)(int64_t)kd;
}

RTCR_FN void mul64(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    lo = a * b;
    hi = __umul64hi(a, b);
#else
    const unsigned __int128 p = (unsigned __int128)a * b;
    lo = (uint64_t)p;
    hi = (uint64_t)(p >> 64);
#endif
}

// Payne-Hanek for 2^20 < ax < inf: ax = k pi/128 + r, k mod 256
RTCR_SLOW void reduce_ph(double ax, DD& r, int& k) {
    RTCR_NOCONTRACT
    const uint64_t ib = bits(ax);
    const int E = (int)(ib >> 52) - 1075;  // ax = M 2^E
    const uint64_t M = (ib & 0x000fffffffffffffull) | 0x0010000000000000ull;
    // 192-bit window of 128/pi from the bit of weight 2^(7 - E) (bit index E +
    // 64 of the zero-prefixed table): ax 128/pi mod 256 = M * window * 2^-184
    const int G = E + 64, jw = G >> 6, sh = G & 63;
    uint64_t U[3];
    for (int i = 0; i < 3; ++i) {
        const uint64_t a = RTCR_128_OVER_PI[jw + i], b = RTCR_128_OVER_PI[jw + i + 1];
        U[i] = sh ? (a << sh) | (b >> (64 - sh)) : a;
    }
    uint64_t l0, c0, l1, c1, l2, h2;
    mul64(M, U[2], l0, c0);
    mul64(M, U[1], l1, c1);
    l1 += c0;
    c1 += (l1 < c0);
    mul64(M, U[0], l2, h2);
    l2 += c1;
    // P mod 2^192 = l2:l1:l0; k = bits 184..191, fraction = bits 183..0
    k = (int)(l2 >> 56);
    uint64_t f2 = l2 & 0x00ffffffffffffffull, f1 = l1;  // fraction * 2^184, top 120 bits kept
    bool neg = false;
    if (f2 >> 55) {  // fraction >= 1/2: round k up, fraction - 1
        k += 1;
        // two's complement of the 120-bit fixed-point fraction (f2:f1)
        f1 = ~f1 + 1;
        f2 = (~f2 + (f1 == 0 ? 1 : 0)) & 0x00ffffffffffffffull;
        neg = true;
    }
    // |fraction| = (f2 2^64 + f1) 2^-120 (f2 < 2^56), as four exact pieces
    const double p0 = (double)(f2 >> 28) * 0x1p-28, p1 = (double)(f2 & 0xfffffffull) * 0x1p-56;
    const double p2 = (double)(f1 >> 32) * 0x1p-88, p3 = (double)(f1 & 0xffffffffull) * 0x1p-120;
    DD f = dd_add_acc(two_sum(p0, p1), two_sum(p2, p3));
    if (neg) f = dd_neg(f);
    r = dd_mul(f, DD{RTCR_PIO128_H, RTCR_PIO128_L});
}

// sin r, cos r as double-doubles (|r| <= pi/256 + tiny): ~2^-104 relative
RTCR_FN void sincos_r_dd(DD r, DD& sr, DD& cr) {
    RTCR_NOCONTRACT
    const DD r2 = dd_mul(r, r);
    const double q = r2.h;
    const double ps = RTCR_S7_H + q * (RTCR_S9_H + q * (RTCR_S11_H + q * RTCR_S13_H));
    DD P = fast_two_sum(RTCR_S5_H, q * ps);
    P.l += RTCR_S5_L;
    const DD Q = dd_add(DD{RTCR_S3_H, RTCR_S3_L}, dd_mul(r2, P));
    sr = dd_add(r, dd_mul(r, dd_mul(r2, Q)));
    const double pc = RTCR_C6_H + q * (RTCR_C8_H + q * (RTCR_C10_H + q * RTCR_C12_H));
    DD PC = fast_two_sum(RTCR_C4_H, q * pc);
    PC.l += RTCR_C4_L;
    const DD QC = dd_add(DD{-0.5, 0.0}, dd_mul(r2, PC));
    cr = dd_add(DD{1.0, 0.0}, dd_mul(r2, QC));
}

// sin and cos to ~2^-100, rounded once: the slow path (and |x| > 2^20, inf, nan)
RTCR_SLOW void sincos_slow(double x, double* s, double* c) {
    RTCR_NOCONTRACT
    RTCR_COUNT_SLOW();
    const double ax = abs_(x);
    if (!(ax < __builtin_huge_val())) {  // inf, nan
        *s = *c = x - x;
        return;
    }
    if (ax < 0x1p-500) {  // sin x = x, cos x = 1 (x^2/2 below half an ulp of 1)
        *s = x;
        *c = 1.0;
        return;
    }
    DD r;
    int k;
    if (ax <= 0x1p20) {
        reduce_slow(x, r, k);
    } else {
        reduce_ph(ax, r, k);
        if (x < 0) {
            r = dd_neg(r);
            k = -k;
        }
    }
    DD S, C, sr, cr;
    sc_table(k, S, C);
    sincos_r_dd(r, sr, cr);
    const DD ys = dd_add_acc(dd_mul(S, cr), dd_mul(C, sr));
    const DD yc = dd_add_acc(dd_mul(C, cr), dd_neg(dd_mul(S, sr)));
    *s = ys.h + ys.l;
    *c = yc.h + yc.l;
}

// A cos r + B sin r (fast path); false when the result's rounding is not certain.
// A + B rh exactly (|A| >= sin(pi/128) > |B rh| unless A = 0), then the
// small terms, the two largest of them -- A hq = -A rh^2/2 and B t = B (sin r
// - r) -- last, so that the others round at a finer scale; the bound covers
// their roundings (2^-53 each) and t's own error (~2^-50.2 relative: r^2 from
// rh alone, the polynomial, the products) adaptively, everything else stays
// under 2^-75 |y| or 2^-108 absolute.
RTCR_FN bool sc_combine(DD A, DD B, double rh, double rl, double hq, double cmr, double t, double& y) {
    RTCR_NOCONTRACT
    const DD b = two_prod(B.h, rh);
    const DD u = fast_two_sum(A.h, b.h);
    double sm = (A.l + u.l) + b.l;
    sm = fma_(B.h, rl, sm);
    sm = fma_(B.l, rh, sm);
    sm = fma_(A.h, cmr, sm);
    sm = fma_(A.l, hq, sm);
    sm = fma_(B.l, t, sm);
    const double ah = A.h * hq, bt = B.h * t;
    sm = fma_(A.h, hq, sm);
    sm = fma_(B.h, t, sm);
    const DD yy = fast_two_sum(u.h, sm);
    const double err = fma_(abs_(bt), 0x1p-49, fma_(abs_(ah), 0x1p-51, fma_(abs_(yy.h), 0x1p-68, 0x1p-105)));
    y = yy.h;
    return rounds_ok(yy.h, yy.l, err);
}

// shared fast-path pieces of sin r / cos r
struct ScR {
    double rh, rl, hq, cmr, t;
    int k;
};
// the polynomial pieces from p.rh, p.rl
RTCR_FN void sc_poly(ScR& p) {
    RTCR_NOCONTRACT
    const double rh = p.rh;
    const double q2 = rh * rh;
    const double eq = fma_(2.0 * rh, p.rl, fma_(rh, rh, -q2));  // r^2 = q2 + eq
    const double ps = q2 * (RTCR_S3_H + q2 * (RTCR_S5_H + q2 * RTCR_S7_H));  // r^8/9! < 2^-69 r: inside the bound
    p.t = rh * ps;  // sin r - r
    p.hq = -0.5 * q2;
    p.cmr = fma_(q2 * q2, RTCR_C4_H + q2 * (RTCR_C6_H + q2 * RTCR_C8_H), -0.5 * eq);  // cos r - 1 - hq
}
RTCR_FN bool sc_prep(double x, ScR& p) {
    if (!(abs_(x) <= 0x1p20) || abs_(x) < 0x1p-500) return false;
    reduce_fast(x, p.rh, p.rl, p.k);
    sc_poly(p);
    return true;
}

RTCR_FN double sin(double x) {
    ScR p;
    if (sc_prep(x, p)) {
        DD S, C;
        sc_table(p.k, S, C);
        double y;
        if (sc_combine(S, C, p.rh, p.rl, p.hq, p.cmr, p.t, y)) return y;
    }
    double s, c;
    sincos_slow(x, &s, &c);
    return s;
}
RTCR_FN double cos(double x) {
    ScR p;
    if (sc_prep(x, p)) {
        DD S, C;
        sc_table(p.k, S, C);
        double y;
        if (sc_combine(C, dd_neg(S), p.rh, p.rl, p.hq, p.cmr, p.t, y)) return y;
    }
    double s, c;
    sincos_slow(x, &s, &c);
    return c;
}
RTCR_FN void sincos(double x, double* s, double* c) {
    ScR p;
    if (sc_prep(x, p)) {
        DD S, C;
        sc_table(p.k, S, C);
        double ys, yc;
        const bool oks = sc_combine(S, C, p.rh, p.rl, p.hq, p.cmr, p.t, ys);
        const bool okc = sc_combine(C, dd_neg(S), p.rh, p.rl, p.hq, p.cmr, p.t, yc);
        if (oks && okc) {
            *s = ys;
            *c = yc;
            return;
        }
    }
    sincos_slow(x, s, c);
}

// sin and cos of x = 2pi xi for 0 <= xi <= 1 (a unit draw: every sincos of
// the path, vec3.rs:63-69 / 313-343, pdf.rs, camera.rs:263-266) -- the same
// correctly rounded doubles as sincos(2.0 * PI * xi), with the argument's range
// known: no range branches, and a reduction whose constants have 44 bits, so
// that k C1 and k C2 are exact for k <= 256 (rt_crmath_tables.h): x - k C1
// exact (Sterbenz, or one binade for k = 1), x - k C1 - k C2 as an exact two-sum,
// lo = RN(s.l - k C3) (|error| < 2^-112), then a fast two-sum -- valid because
// every double x lies >= 9.7e-21 from the k pi/128 it reduces to, far above
// |lo| (scripts/gen_crmath_tables.py checks it).  x = 0 fails the rounding test
// (err > 0) and takes the slow path, which returns sin 0 = 0, cos 0 = 1.
RTCR_FN void reduce_2pi(double x, double& rh, double& rl, int& k) {
    RTCR_NOCONTRACT
    const double kd = __builtin_rint(x * RTCR_INV_PIO128);
    const double y1 = fma_(-kd, RTCR_PIO128S_1, x);
    const double p2 = kd * RTCR_PIO128S_2;
    const DD s = two_sum(y1, -p2);
    const double lo = fma_(-kd, RTCR_PIO128S_3, s.l);
    const DD r = fast_two_sum(s.h, lo);
    rh = r.h;
    rl = r.l;
    k = (int)kd;
}
RTCR_FN void sincos_2pi(double xi, double* s, double* c) {
    RTCR_NOCONTRACT
    const double x = 2.0 * 0x1.921fb54442d18p+1 * xi;  // 2.0 * PI * xi, PI = RN(pi)
    ScR p;
    reduce_2pi(x, p.rh, p.rl, p.k);
    sc_poly(p);
    DD S, C;
    sc_table(p.k, S, C);
    double ys, yc;
    const bool oks = sc_combine(S, C, p.rh, p.rl, p.hq, p.cmr, p.t, ys);
    const bool okc = sc_combine(C, dd_neg(S), p.rh, p.rl, p.hq, p.cmr, p.t, yc);
    if (oks && okc) {
        *s = ys;
        *c = yc;
        return;
    }
    sincos_slow(x, s, c);
}

// ------------------------------------------------------------------ log
struct LogR {
    double ed, rh, rl;
    int j;
};
// x > 0 finite: x = 2^e z, r = z c_j - 1 (exact double-double)
RTCR_FN void log_reduce(double x, LogR& p) {
    RTCR_NOCONTRACT
    uint64_t ix = bits(x);
    int e = (int)(ix >> 52) - 1023;
    if ((ix >> 52) == 0) {  // subnormal
        ix = bits(x * 0x1p54);
        e = (int)(ix >> 52) - 1023 - 54;
    }
    const int j = (int)((ix >> 45) & 127);
    double z = from_bits((ix & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (j >= 53) {
        z *= 0.5;
        e += 1;
    }
    const DD pz = two_prod(z, RTCR_LOG_T[j][0]);
    const DD r = fast_two_sum(pz.h - 1.0, pz.l);  // pz.h - 1 exact (Sterbenz)
    p.ed = (double)e;
    p.rh = r.h;
    p.rl = r.l;
    p.j = j;
}

RTCR_SLOW double log_slow(double x) {
    RTCR_NOCONTRACT
    RTCR_COUNT_SLOW();
    if (!(x > 0.0)) return x == 0.0 ? -__builtin_huge_val() : (x - x) / (x - x);
    if (!(x < __builtin_huge_val())) return x;
    LogR p;
    log_reduce(x, p);
    const DD r{p.rh, p.rl};
    const double q = p.rh;
    // log1p(r) = r + r^2 (-1/2 + r (1/3 + r (-1/4 + ...))): terms 9.. in double
    double tail = 0.0;
    for (int k = 20; k >= 9; --k) tail = fma_(q, tail, ((k & 1) ? 1.0 : -1.0) / (double)k);
    const double invh[9] = {0, 0, 0, RTCR_INV3_H, 0, RTCR_INV5_H, RTCR_INV6_H, RTCR_INV7_H, 0};
    const double invl[9] = {0, 0, 0, RTCR_INV3_L, 0, RTCR_INV5_L, RTCR_INV6_L, RTCR_INV7_L, 0};
    DD acc{tail, 0.0};
    for (int k = 8; k >= 2; --k) {
        const double sg = (k & 1) ? 1.0 : -1.0;
        const DD ck = (k == 2 || k == 4 || k == 8) ? DD{sg / (double)k, 0.0} : DD{sg * invh[k], sg * invl[k]};
        acc = dd_add(ck, dd_mul(r, acc));
    }
    const DD l1p = dd_add(r, dd_mul(dd_mul(r, r), acc));
    // e ln2 - log c + log1p(r)
    const DD e2 = dd_add_acc(DD{p.ed * RTCR_LN2_H, 0.0}, dd_add(two_prod(p.ed, RTCR_LN2_M), DD{p.ed * RTCR_LN2_L, 0.0}));
    const DD y = dd_add_acc(dd_add_acc(e2, DD{-RTCR_LOG_T[p.j][1], -RTCR_LOG_T[p.j][2]}), l1p);
    return y.h + y.l;
}

RTCR_FN double log(double x) {
    RTCR_NOCONTRACT
    if (x > 0.0 && x < __builtin_huge_val()) {
        LogR p;
        log_reduce(x, p);
        const double rh = p.rh;
        const DD a = two_sum(p.ed * RTCR_LN2_H, -RTCR_LOG_T[p.j][1]);  // e LN2_H exact
        const DD b = two_sum(a.h, rh);
        const DD q = two_prod(rh, rh);
        const DD s = two_sum(b.h, -0.5 * q.h);
        // r^3 (1/3 - r/4 + r^2/5 - ... - r^9/12)
        double P = -RTCR_INV12_H;
        P = fma_(rh, P, RTCR_INV11_H);
        P = fma_(rh, P, -RTCR_INV10_H);
        P = fma_(rh, P, RTCR_INV9_H);
        P = fma_(rh, P, -0.125);
        P = fma_(rh, P, RTCR_INV7_H);
        P = fma_(rh, P, -RTCR_INV6_H);
        P = fma_(rh, P, RTCR_INV5_H);
        P = fma_(rh, P, -0.25);
        P = fma_(rh, P, RTCR_INV3_H);
        const double p3 = (rh * q.h) * P;
        double lo = ((a.l + b.l) + s.l) + p.rl;
        lo = fma_(p.ed, RTCR_LN2_M, lo);
        lo -= RTCR_LOG_T[p.j][2];
        lo = fma_(-0.5, q.l, lo);
        lo = fma_(-rh, p.rl, lo);
        lo += p3;
        const DD y = fast_two_sum(s.h, lo);
        const double err = fma_(abs_(p3), 0x1p-49, abs_(y.h) * 0x1p-70);
        if (rounds_ok(y.h, y.l, err)) return y.h;
    }
    return log_slow(x);
}

// ------------------------------------------------------------------ atan2 / acos
// atan(n / d) for 0 <= n, 0 < d as double-doubles, plus the octant: result =
// K + sg * atan(min/max), K in {0, pi/2, pi}; fast path with error bound, or
// slow (ok = false -> caller reruns with slow = true)
RTCR_FN bool atan_core(DD n, DD d, bool xneg, bool slow, double& out) {
    RTCR_NOCONTRACT
    const bool sw = n.h > d.h;
    const DD num = sw ? d : n, den = sw ? n : d;
    // t = num / den as a double-double
    const double th = num.h / den.h;
    const double tl = (fma_(-th, den.h, num.h) + num.l - th * den.l) / den.h;
    const double jd = __builtin_rint(th * 64.0);
    const int j = (int)jd;
    const double c = jd * 0.015625;
    // u = (t - c) / (1 + t c)
    const DD nn = two_sum(th - c, tl);  // th - c exact (Sterbenz / c = 0)
    const DD pc = two_prod(th, c);
    DD dd = two_sum(1.0, pc.h);
    dd = fast_two_sum(dd.h, dd.l + fma_(tl, c, pc.l));
    const double uh = nn.h / dd.h;
    const double ul = (fma_(-uh, dd.h, nn.h) + nn.l - uh * dd.l) / dd.h;
    const DD A{RTCR_ATAN_T[j][0], RTCR_ATAN_T[j][1]};
    // octant constant K and sign sg: result = K + sg * (A + atan u)
    DD K{0.0, 0.0};
    double sg = 1.0;
    if (!sw && xneg) K = DD{RTCR_PI_H, RTCR_PI_L}, sg = -1.0;
    if (sw && !xneg) K = DD{RTCR_PIO2_H, RTCR_PIO2_L}, sg = -1.0;
    if (sw && xneg) K = DD{RTCR_PIO2_H, RTCR_PIO2_L};
    const double u2 = uh * uh;
    if (!slow) {
        // atan u - u = u^3 (-1/3 + u^2/5 - ... ), |u| <= 2^-7
        double P = RTCR_INV11_H;
        P = fma_(u2, P, -RTCR_INV9_H);
        P = fma_(u2, P, RTCR_INV7_H);
        P = fma_(u2, P, -RTCR_INV5_H);
        P = fma_(u2, P, RTCR_INV3_H);
        const double tail = -(uh * u2) * P;
        const DD v = two_sum(A.h, uh);
        const double vl = ((A.l + ul) + v.l) + tail;
        const DD w = two_sum(K.h, sg * v.h);
        const double wl = (w.l + K.l) + sg * vl;
        const DD y = fast_two_sum(w.h, wl);
        const double err = fma_(abs_(tail), 0x1p-49, abs_(y.h) * 0x1p-70);
        out = y.h;
        return rounds_ok(y.h, y.l, err);
    }
    // slow: atan u = u + u^3 P(u^2) in double-double, P to u^16
    RTCR_COUNT_SLOW();
    const DD u{uh, ul};
    const DD w2 = dd_mul(u, u);
    double tail = 0.0;
    for (int k = 17; k >= 9; k -= 2) tail = fma_(w2.h, tail, (((k - 1) / 2) & 1 ? -1.0 : 1.0) / (double)k);
    DD acc{tail, 0.0};
    acc = dd_add(DD{-RTCR_INV7_H, -RTCR_INV7_L}, dd_mul(w2, acc));
    acc = dd_add(DD{RTCR_INV5_H, RTCR_INV5_L}, dd_mul(w2, acc));
    acc = dd_add(DD{-RTCR_INV3_H, -RTCR_INV3_L}, dd_mul(w2, acc));
    const DD at = dd_add(u, dd_mul(dd_mul(u, w2), acc));
    const DD v = dd_add(A, at);
    const DD y = dd_add_acc(K, DD{sg * v.h, sg * v.l});
    out = y.h + y.l;
    return true;
}

RTCR_FN double atan2(double y, double x) {
    RTCR_NOCONTRACT
    const double ay = abs_(y), ax = abs_(x);
    const bool xneg = __builtin_signbit(x) != 0;
    if (y != y || x != x) return x + y;
    double r;
    if (ay == 0.0) {
        r = xneg ? RTCR_PI_H : 0.0;  // atan2(+-0, -0 / x<0) = +-pi
    } else if (ax == __builtin_huge_val() || ay == __builtin_huge_val()) {
        if (ax == __builtin_huge_val() && ay == __builtin_huge_val())
            r = xneg ? dd_mul_d(DD{0.5 * RTCR_PIO2_H, 0.5 * RTCR_PIO2_L}, 3.0).h : 0.5 * RTCR_PIO2_H;  // 3pi/4, pi/4
        else if (ay == __builtin_huge_val())
            r = RTCR_PIO2_H;
        else
            r = xneg ? RTCR_PI_H : 0.0;
    } else if (ax == 0.0) {
        r = RTCR_PIO2_H;
    } else {
        double sy = ay, sx = ax;
        const int ey = (int)(bits(ay) >> 52), ex = (int)(bits(ax) >> 52);
        if (ey - ex < -200) {  // t < 2^-199: atan t = t (1 - t^2/3) rounds as t; pi - t as pi
            r = xneg ? RTCR_PI_H : ay / ax;
            return __builtin_copysign(r, y);
        }
        if (ey - ex > 200) return __builtin_copysign(RTCR_PIO2_H, y);  // pi/2 +- t
        if (ey > 1800 || ex > 1800 || ey < 300 || ex < 300) {
            // scale both (the quotient is scale-free) so that the double-double
            // remainders below stay normal
            const int m = ey > ex ? ey : ex;
            const double sc = from_bits((uint64_t)(2046 - m) << 52);  // 2^(1023 - m): the larger to [1, 2)
            sy *= sc;
            sx *= sc;
        }
        if (!atan_core(DD{sy, 0.0}, DD{sx, 0.0}, xneg, false, r)) atan_core(DD{sy, 0.0}, DD{sx, 0.0}, xneg, true, r);
    }
    return __builtin_copysign(r, y);
}

RTCR_FN double acos(double y) {
    RTCR_NOCONTRACT
    const double ay = abs_(y);
    if (!(ay <= 1.0)) return (y - y) / (y - y);  // nan, |y| > 1
    if (y == 1.0) return 0.0;
    if (y == -1.0) return RTCR_PI_H;
    // acos y = atan2(sqrt((1 - y)(1 + y)), y)
    const DD a = two_sum(1.0, -y), b = two_sum(1.0, y);
    const DD w = dd_mul(a, b);
    const double sh = __builtin_sqrt(w.h);
    const double sl = (fma_(-sh, sh, w.h) + w.l) / (2.0 * sh);
    const DD n = fast_two_sum(sh, sl);
    const bool xneg = y < 0.0;
    double r;
    if (!atan_core(n, DD{ay, 0.0}, xneg, false, r)) atan_core(n, DD{ay, 0.0}, xneg, true, r);
    return r;
}

}  // namespace rtcr
