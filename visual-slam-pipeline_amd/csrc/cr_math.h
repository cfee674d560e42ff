// cr_math.h — correctly rounded (round-to-nearest) sin, cos, acos, log and pow for the fp64
// geometry shared by the kernels and their host-side callers.
//
// Why: the reference computes Rodrigues (OpenCV: std::sin / std::cos / std::acos), the 7-point
// cubic (std::acos / std::cos / std::pow) and RANSACUpdateNumIters (std::pow / std::log) with
// glibc, whose results are within 1 ulp but not correctly rounded on ~0.15 % of inputs; the
// device's libm differs from glibc on a similar fraction.  A last-ulp difference inside the PnP
// Levenberg-Marquardt (central differences with step 1e-6 amplify it a million-fold) is enough to
// move a pose by 1e-9 and, hundreds of frames later, a keyframe decision.  Both sides therefore use
// the one function that has a definition independent of any implementation: the correctly rounded
// one.  Against glibc (the reference) these differ by at most 1 ulp on the rare non-correctly-
// rounded glibc results — inside the stated pose tolerance.
//
// Implementation (device and the product's host code): double-double arithmetic (fma-exact
// products) with ~2^-100 relative error before the final rounding, so the rounded result is the
// correctly rounded one except within 2^-100 of a rounding midpoint (probability ~2^-47 per call).
//   sin / cos: x - k pi/2 with a triple-double pi/2, Taylor series of degree 29 / 28 on |r| <= pi/4;
//   acos: pi/2 - asin(c) for |c| <= 1/2, 2 asin(sqrt((1 -+ c) / 2)) beyond, asin by one
//         double-double Newton step on sin from the libm estimate;
//   log: one Newton step on exp from the libm estimate; pow(y, p) = exp(p log y);
//   exp: k ln2 reduction (triple-double ln2), /32, degree-14 Taylor, five squarings.
// The oracle (oracle/, test infrastructure) compiles this header with VS_CR_QUADMATH: the same
// functions from libquadmath's binary128 routines rounded to double — an independent
// implementation of the same correctly rounded values (tests compare the two bit for bit).
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define VS_CR_HD __host__ __device__
#else
#define VS_CR_HD
#endif

#if defined(VS_CR_QUADMATH) && !defined(__HIP_DEVICE_COMPILE__)
#include <quadmath.h>
namespace vs_cr {
inline double sin(double x) { return (double)sinq((__float128)x); }
inline double cos(double x) { return (double)cosq((__float128)x); }
inline double acos(double x) { return (double)acosq((__float128)x); }
inline double log(double x) { return (double)logq((__float128)x); }
inline double pow(double y, double p) { return (double)powq((__float128)y, (__float128)p); }
}  // namespace vs_cr
#else
namespace vs_cr {

struct dd {
    double hi, lo;
};

VS_CR_HD inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
VS_CR_HD inline dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
    const double s = a + b;
    return {s, b - (s - a)};
}
VS_CR_HD inline dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, ::fma(a, b, -p)};
}
VS_CR_HD inline dd add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fast_two_sum(s.hi, s.lo);
}
VS_CR_HD inline dd neg(dd a) { return {-a.hi, -a.lo}; }
VS_CR_HD inline dd sub(dd a, dd b) { return add(a, neg(b)); }
VS_CR_HD inline dd mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return fast_two_sum(p.hi, p.lo);
}
VS_CR_HD inline dd mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return fast_two_sum(p.hi, p.lo);
}
VS_CR_HD inline double round_dd(dd a) { return a.hi + a.lo; }  // RN of the double-double value

// 1/n! as double-doubles, n = 0..29 (exact rationals rounded twice)
#define VS_CR_INV_FACT                                                                                          \
    {                                                                                                           \
        {0x1p+0, 0x0p+0}, {0x1p+0, 0x0p+0}, {0x1p-1, 0x0p+0}, {0x1.5555555555555p-3, 0x1.5555555555555p-57},     \
            {0x1.5555555555555p-5, 0x1.5555555555555p-59}, {0x1.1111111111111p-7, 0x1.1111111111111p-63},       \
            {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65}, {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73},    \
            {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76}, {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},    \
            {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76}, {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80},    \
            {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83}, {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},    \
            {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92}, {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97},     \
            {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101}, {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},   \
            {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107}, {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112},   \
            {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120}, {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},  \
            {0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124}, {0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130}, \
            {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135}, {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139}, \
            {0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143}, {0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149},  \
            {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153}, {                                                 \
            0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157                                                      \
        }                                                                                                       \
    }

constexpr double kPio2[3] = {0x1.921fb54442d18p+0, 0x1.1a62633145c07p-54, -0x1.f1976b7ed8fbcp-110};
constexpr double kLn2[3] = {0x1.62e42fefa39efp-1, 0x1.abc9e3b39803fp-56, 0x1.7b57a079a1934p-111};

VS_CR_HD inline dd inv_fact(int n) {
    const double t[30][2] = VS_CR_INV_FACT;
    return {t[n][0], t[n][1]};
}

// sin(r), cos(r) for |r| <= pi/4 (+ rounding slack): Horner in u = r^2 with signs (-1)^k
VS_CR_HD inline dd sin_poly(dd r) {  // r * sum_{k=0}^{14} (-1)^k u^k / (2k+1)!
    const dd u = mul(r, r);
    dd p = inv_fact(29);
    for (int k = 13; k >= 0; k--) {
        p = mul(p, u);
        p = (k & 1) ? sub(p, inv_fact(2 * k + 1)) : add(p, inv_fact(2 * k + 1));
    }
    return mul(p, r);
}
VS_CR_HD inline dd cos_poly(dd r) {  // sum_{k=0}^{14} (-1)^k u^k / (2k)!
    const dd u = mul(r, r);
    dd p = inv_fact(28);
    for (int k = 13; k >= 0; k--) {
        p = mul(p, u);
        p = (k & 1) ? sub(p, inv_fact(2 * k)) : add(p, inv_fact(2 * k));
    }
    return p;
}

// x = k pi/2 + r, |r| <= pi/4; valid for |x| < 2^20
VS_CR_HD inline dd reduce_pio2(double x, int& q) {
    const double k = ::rint(x * 0x1.45f306dc9c883p-1);  // 2/pi
    dd r = sub(dd{x, 0.0}, two_prod(k, kPio2[0]));
    r = sub(r, two_prod(k, kPio2[1]));
    r = sub(r, dd{k * kPio2[2], 0.0});
    q = (int)((int64_t)k & 3);
    return r;
}

VS_CR_HD inline dd sin_dd(double x) {
    int q;
    const dd r = reduce_pio2(x, q);
    switch (q) {
        case 0: return sin_poly(r);
        case 1: return cos_poly(r);
        case 2: return neg(sin_poly(r));
        default: return neg(cos_poly(r));
    }
}
VS_CR_HD inline dd cos_dd(double x) {
    int q;
    const dd r = reduce_pio2(x, q);
    switch (q) {
        case 0: return cos_poly(r);
        case 1: return neg(sin_poly(r));
        case 2: return neg(cos_poly(r));
        default: return sin_poly(r);
    }
}
VS_CR_HD inline double sin(double x) { return round_dd(sin_dd(x)); }
VS_CR_HD inline double cos(double x) { return round_dd(cos_dd(x)); }

// sqrt of a double as a double-double
VS_CR_HD inline dd sqrt_dd(double s) {
    const double q0 = ::sqrt(s);
    if (q0 == 0.0) return {0.0, 0.0};
    const double e = ::fma(-q0, q0, s);
    return fast_two_sum(q0, e / (2.0 * q0));
}
// asin of a double-double q, |q| <= 0.75: one Newton step on sin from the libm estimate
VS_CR_HD inline dd asin_dd(dd q) {
    const double t0 = ::asin(q.hi);
    const dd res = sub(q, sin_dd(t0));
    return add(dd{t0, 0.0}, dd{res.hi / ::cos(t0), 0.0});
}
VS_CR_HD inline double acos(double c) {
    if (!(c >= -1.0 && c <= 1.0)) return (c > 1.0) ? 0.0 : (c < -1.0 ? 0x1.921fb54442d18p+1 : c);  // NaN passes
    if (c == 1.0) return 0.0;
    const dd pio2{kPio2[0], kPio2[1]};
    if (::fabs(c) <= 0.5) return round_dd(sub(pio2, asin_dd(dd{c, 0.0})));
    if (c > 0.0) {
        const dd t = asin_dd(sqrt_dd((1.0 - c) * 0.5));
        return round_dd(dd{2.0 * t.hi, 2.0 * t.lo});
    }
    const dd t = asin_dd(sqrt_dd((1.0 + c) * 0.5));
    return round_dd(sub(dd{2.0 * kPio2[0], 2.0 * kPio2[1]}, dd{2.0 * t.hi, 2.0 * t.lo}));
}

// exp of a double-double z, |z.hi| < 700
VS_CR_HD inline dd exp_dd(dd z) {
    const double k = ::rint(z.hi * 0x1.71547652b82fep+0);  // 1/ln2
    dd r = sub(z, two_prod(k, kLn2[0]));
    r = sub(r, two_prod(k, kLn2[1]));
    r = sub(r, dd{k * kLn2[2], 0.0});
    r = dd{r.hi * 0x1p-5, r.lo * 0x1p-5};
    dd p = inv_fact(14);
    for (int n = 13; n >= 0; n--) p = add(mul(p, r), inv_fact(n));
    for (int i = 0; i < 5; i++) p = mul(p, p);
    return {::ldexp(p.hi, (int)k), ::ldexp(p.lo, (int)k)};
}
// log of a positive double as a double-double: one Newton step on exp from the libm estimate
VS_CR_HD inline dd log_dd(double y) {
    const double l0 = ::log(y);
    const dd t = sub(mul_d(exp_dd(dd{-l0, 0.0}), y), dd{1.0, 0.0});  // y e^-l0 - 1 = log correction
    return add(dd{l0, 0.0}, sub(t, dd{0.5 * t.hi * t.hi, 0.0}));
}
VS_CR_HD inline double log(double y) {
    if (!(y > 0.0) || y == 1.0 || y > 1.7976931348623157e308) return ::log(y);
    return round_dd(log_dd(y));
}
// y^p for y > 0 (the callers' domain: RANSACUpdateNumIters, the 7-point cubic's real root)
VS_CR_HD inline double pow(double y, double p) {
    if (y == 1.0 || p == 0.0) return 1.0;
    if (!(y > 0.0) || y > 1.7976931348623157e308) return ::pow(y, p);
    const dd z = mul_d(log_dd(y), p);
    if (z.hi > 709.0 || z.hi < -708.0) return ::pow(y, p);
    return round_dd(exp_dd(z));
}

}  // namespace vs_cr
#endif
