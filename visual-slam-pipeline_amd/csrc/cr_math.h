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
//   sin / cos: x - k pi/2 with a triple-double pi/2, then r = j/64 + b with a 53-entry double-double
//         table of sin / cos (j/64), Taylor series of degree 13 / 12 on |b| <= 1/128 (terms past
//         u^3 in plain double) and the addition formulas (sincos shares the reduction);
//   acos: pi/2 - asin(c) for |c| <= 1/2, 2 asin(sqrt((1 -+ c) / 2)) beyond, asin by one
//         double-double Newton step on sin from the libm estimate;
//   log: one Newton step on exp from the libm estimate; pow(y, p) = exp(p log y), integer
//         exponents 2..8 by binary powering;
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
inline void sincos(double x, double& sn, double& cs) {
    sn = sin(x);
    cs = cos(x);
}
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

// sin(j/64), cos(j/64) as double-doubles, j = 0..52 (libquadmath: hi = RN(q), lo = RN(q - hi))
#define VS_CR_SINCOS64 \
    { \
    {0x0p+0, 0x0p+0, 0x1p+0, 0x0p+0}, \
    {0x1.fffaaaaeeeed5p-7, -0x1.2ab639a9f0776p-63, 0x1.fff000155549fp-1, 0x1.28a28a03a5ef3p-55}, \
    {0x1.ffeaaaeeee86fp-6, -0x1.cd406fb224ae2p-60, 0x1.ffc00155527d3p-1, -0x1.3b54492d89b5bp-55}, \
    {0x1.7fdc01032fba9p-5, -0x1.599bdf46e997ap-59, 0x1.ff7006bfdf99fp-1, -0x1.8b3b560648d5fp-56}, \
    {0x1.ffaaaeeed4edbp-5, -0x1.2d16d32684b69p-59, 0x1.ff0015549f4d3p-1, 0x1.328387b99426fp-55}, \
    {0x1.3facb12d1755bp-4, -0x1.921915299468bp-58, 0x1.fe7034129ef6fp-1, -0x1.cbf4337c96f96p-57}, \
    {0x1.7f701032550e4p-4, 0x1.afc2d1800501ap-60, 0x1.fdc06bf7e6b9bp-1, 0x1.31902b535f8dbp-55}, \
    {0x1.bf1b78568391dp-4, 0x1.e91841dea4cc8p-58, 0x1.fcf0c800e99b1p-1, 0x1.ea3d786d186acp-57}, \
    {0x1.feaaeee86ee36p-4, -0x1.afcb2bcc6f03bp-59, 0x1.fc015527d5bd3p-1, 0x1.b68f35094efb8p-55}, \
    {0x1.1f0d3d7afceafp-3, -0x1.6ef95099769a5p-57, 0x1.faf22263c4bd3p-1, -0x1.52ace133a2769p-58}, \
    {0x1.3eb312c5d66cbp-3, 0x1.47d666b66cb91p-57, 0x1.f9c340a7cc428p-1, 0x1.c5b6b063b7462p-55}, \
    {0x1.5e44fcfa126f3p-3, -0x1.6f443063f89b6p-57, 0x1.f874c2e1eecf6p-1, -0x1.c6514e1332b16p-55}, \
    {0x1.7dc102fbaf2b5p-3, 0x1.5ab50e23c97c3p-59, 0x1.f706bdf9ece1cp-1, -0x1.698c80c36dcb4p-55}, \
    {0x1.9d252d0cec312p-3, 0x1.9c43d80b1137dp-58, 0x1.f57948cff6797p-1, 0x1.e3a0d3e03b1d4p-57}, \
    {0x1.bc6f84edc6199p-3, 0x1.9c1a56a7b0cabp-57, 0x1.f3cc7c3b3d16ep-1, -0x1.21a3ad28a3494p-57}, \
    {0x1.db9e15fb5a5dp-3, -0x1.32e20d6cc6fc2p-57, 0x1.f20073086649fp-1, 0x1.b940416c1984bp-56}, \
    {0x1.faaeed4f31577p-3, -0x1.15d88508e32b8p-57, 0x1.f01549f7deea1p-1, 0x1.d3c1e99e5cafdp-55}, \
    {0x1.0cd00cef36436p-2, -0x1.9fb0a0c93e2b4p-56, 0x1.ee0b1fbc0f11cp-1, -0x1.bfd2380bbc3b1p-59}, \
    {0x1.1c37d64c6b876p-2, 0x1.46076fe0dcff4p-56, 0x1.ebe214f76efa8p-1, -0x1.02f9f12ba543ep-55}, \
    {0x1.2b8ddc43eb49fp-2, 0x1.1553899f2d807p-57, 0x1.e99a4c3a7cd83p-1, -0x1.2264b1bc53ce8p-55}, \
    {0x1.3ad129769d3d8p-2, 0x1.03d550487839ap-63, 0x1.e733ea0193d4p-1, -0x1.6428b3546ce13p-55}, \
    {0x1.4a00c9b0f3d2p-2, 0x1.823ba6bb08eadp-56, 0x1.e4af14b2a449cp-1, -0x1.68ca02e8a6833p-55}, \
    {0x1.591bc9fa2f597p-2, 0x1.7c74bac3fe0cbp-57, 0x1.e20bf49acd6c1p-1, -0x1.660aec7ef636cp-58}, \
    {0x1.682138a38d7f7p-2, -0x1.d889202444aadp-56, 0x1.df4ab3ebd875ep-1, -0x1.e2d8a7e6736c4p-55}, \
    {0x1.7710255764214p-2, -0x1.6ead7314bb6cep-57, 0x1.dc6b7eb995912p-1, 0x1.4b364776dcd35p-58}, \
    {0x1.85e7a12826949p-2, 0x1.8a40e9b5facep-56, 0x1.d96e82f71a9dcp-1, 0x1.ff61bd5d2039dp-55}, \
    {0x1.94a6be9f546c5p-2, -0x1.69ce13e683f58p-56, 0x1.d653f073e404p-1, -0x1.76236434bec37p-55}, \
    {0x1.a34c91cc50ccap-2, -0x1.a310e3b50cecdp-58, 0x1.d31bf8d8d7c06p-1, 0x1.e60dd3089cbddp-56}, \
    {0x1.b1d8305321617p-2, -0x1.ae242cb99f519p-56, 0x1.cfc6cfa52ad9fp-1, 0x1.8b5b5508f2a0dp-55}, \
    {0x1.c048b17b140a3p-2, 0x1.19fe6757e9fa6p-57, 0x1.cc54aa2b2972ep-1, 0x1.4ee162ba83a98p-57}, \
    {0x1.ce9d2e3d4a51fp-2, -0x1.2fc8a12dae298p-57, 0x1.c8c5bf8ce1a84p-1, 0x1.ab3d1a1590123p-56}, \
    {0x1.dcd4c15329c9ap-2, 0x1.0d4c6e171fd9ap-56, 0x1.c51a48b8b175ep-1, -0x1.1bbb43b9aa88p-57}, \
    {0x1.eaee8744b05fp-2, -0x1.789b43c9b027cp-58, 0x1.c1528065b7d5p-1, -0x1.892111312e828p-55}, \
    {0x1.f8e99e76abc97p-2, 0x1.9d950af2d00a3p-58, 0x1.bd6ea310294f5p-1, 0x1.31bbcc88c109dp-56}, \
    {0x1.0362939c69955p-1, -0x1.2d8cd78397b01p-55, 0x1.b96eeef58840ep-1, 0x1.45a3cc78fadep-58}, \
    {0x1.0a4021e9e1001p-1, -0x1.6f643a13914f6p-55, 0x1.b553a410c104ep-1, 0x1.8ff7947027a16p-58}, \
    {0x1.110d0c4b69c3bp-1, 0x1.d918998809981p-55, 0x1.b11d04162a4c6p-1, 0x1.1dd561efbc0c2p-56}, \
    {0x1.17c8e5f2eedbp-1, 0x1.35e57102e2488p-57, 0x1.accb526f69de5p-1, 0x1.8fb6a8dd6b6ccp-55}, \
    {0x1.1e7343236574cp-1, 0x1.22a3fa4f41d5ap-56, 0x1.a85ed4373e02dp-1, 0x1.9be06385ec792p-57}, \
    {0x1.250bb93788bbbp-1, 0x1.ea3d02457bccep-56, 0x1.a3d7d0352bdcfp-1, -0x1.68dbaeca19669p-55}, \
    {0x1.2b91dea88421ep-1, -0x1.fa371db216abp-55, 0x1.9f368ed912f85p-1, -0x1.1d200c5791606p-55}, \
    {0x1.32054b148bc4fp-1, 0x1.f6b42095a135bp-55, 0x1.9a7b5a36a6514p-1, 0x1.722cfcc9fa7a9p-55}, \
    {0x1.386597456282bp-1, -0x1.10fada93b07a8p-56, 0x1.95a67e00cb1fdp-1, -0x1.0befda21f862dp-55}, \
    {0x1.3eb25d36cd53ap-1, -0x1.be570e1570fcp-58, 0x1.90b84784ddaf7p-1, -0x1.0feb10ab93b87p-56}, \
    {0x1.44eb381cf386bp-1, -0x1.3ed6c1e6a5505p-55, 0x1.8bb105a5dc9p-1, 0x1.863e03e9474c1p-55}, \
    {0x1.4b0fc46aab761p-1, 0x1.0da05738cc59cp-61, 0x1.869108d77a6c6p-1, 0x1.338ffe2bfe9ddp-56}, \
    {0x1.511f9fd7b351cp-1, -0x1.5c0e861c48831p-55, 0x1.8158a31916d5dp-1, -0x1.de8b90b8228dep-57}, \
    {0x1.571a6966d59b3p-1, 0x1.c843b4d0fb197p-58, 0x1.7c0827f09e54fp-1, -0x1.c73d6d72aee68p-57}, \
    {0x1.5cffc16bf8f0dp-1, 0x1.96cb370eb578ap-55, 0x1.769fec655211fp-1, -0x1.827d5cf8c68c5p-57}, \
    {0x1.62cf49921ac79p-1, -0x1.edd9855b6241ap-55, 0x1.712046fa77678p-1, 0x1.425b0a5029c81p-55}, \
    {0x1.6888a4e134b2fp-1, -0x1.6b7d37644d5e6p-55, 0x1.6b898fa9efb5dp-1, 0x1.15ac786ccf4b2p-56}, \
    {0x1.6e2b77c40bde1p-1, -0x1.0e729857fad53p-56, 0x1.65dc1fdeb8cbap-1, -0x1.97c1b47337c77p-58}, \
    {0x1.73b7680dea578p-1, -0x1.2248306dc12a2p-56, 0x1.6018526f563dfp-1, 0x1.46ca5e0e432dp-55} \
    }
#if defined(__HIPCC__)
__device__ __constant__ const double kSinCos64Dev[53][4] = VS_CR_SINCOS64;
#endif
inline constexpr double kSinCos64[53][4] = VS_CR_SINCOS64;

// sin(b), cos(b) for |b| <= 1/128 (+ slack): Taylor to b^13 / b^12.  With u = b^2 <= 2^-14 the
// terms from u^4 on are below 2^-68 relative, so they are summed in plain double (error < 2^-120)
// and only the first four steps of the Horner chain run in double-double.
VS_CR_HD inline dd sin_small(dd b) {  // b * sum_{k=0}^{6} (-1)^k u^k / (2k+1)!
    const dd u = mul(b, b);
    const double ud = u.hi;
    const double tl = inv_fact(9).hi + ud * (-inv_fact(11).hi + ud * inv_fact(13).hi);
    dd p = sub(mul_d(u, tl), inv_fact(7));
    p = add(mul(p, u), inv_fact(5));
    p = sub(mul(p, u), inv_fact(3));
    p = add(mul(p, u), dd{1.0, 0.0});
    return mul(p, b);
}
VS_CR_HD inline dd cos_small(dd b) {  // sum_{k=0}^{6} (-1)^k u^k / (2k)!
    const dd u = mul(b, b);
    const double ud = u.hi;
    const double tl = inv_fact(8).hi + ud * (-inv_fact(10).hi + ud * inv_fact(12).hi);
    dd p = sub(mul_d(u, tl), inv_fact(6));
    p = add(mul(p, u), inv_fact(4));
    p = sub(mul(p, u), inv_fact(2));
    return add(mul(p, u), dd{1.0, 0.0});
}
// sin(r), cos(r) for |r| <= pi/4: r = a + b with a = j/64 (table), |b| <= 1/128 (the subtraction
// r.hi - a is exact), then the addition formulas in double-double
VS_CR_HD inline void sincos_poly(dd r, dd& sn, dd& cs) {
    const double j = ::rint(r.hi * 64.0);
    const int ji = (int)::fabs(j);
#if defined(__HIP_DEVICE_COMPILE__)
    const double* t = kSinCos64Dev[ji];
#else
    const double* t = kSinCos64[ji];
#endif
    const dd sa{j < 0 ? -t[0] : t[0], j < 0 ? -t[1] : t[1]}, ca{t[2], t[3]};
    const dd b = two_sum(r.hi - j * 0x1p-6, r.lo);
    const dd sb = sin_small(b), cb = cos_small(b);
    sn = add(mul(sa, cb), mul(ca, sb));
    cs = sub(mul(ca, cb), mul(sa, sb));
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

VS_CR_HD inline void sincos_dd(double x, dd& sn, dd& cs) {
    int q;
    const dd r = reduce_pio2(x, q);
    dd s0, c0;
    sincos_poly(r, s0, c0);
    switch (q) {
        case 0: sn = s0, cs = c0; break;
        case 1: sn = c0, cs = neg(s0); break;
        case 2: sn = neg(s0), cs = neg(c0); break;
        default: sn = neg(c0), cs = s0; break;
    }
}
VS_CR_HD inline dd sin_dd(double x) {
    dd s, c;
    sincos_dd(x, s, c);
    return s;
}
VS_CR_HD inline double sin(double x) { return round_dd(sin_dd(x)); }
VS_CR_HD inline double cos(double x) {
    dd s, c;
    sincos_dd(x, s, c);
    return round_dd(c);
}
VS_CR_HD inline void sincos(double x, double& sn, double& cs) {
    dd s, c;
    sincos_dd(x, s, c);
    sn = round_dd(s);
    cs = round_dd(c);
}

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
    if (p >= 2.0 && p <= 8.0 && p == ::rint(p) && y > 0x1p-100 && y < 0x1p100) {
        // small integer powers (RANSACUpdateNumIters' (1 - ep)^model_points) by binary powering in
        // double-double: relative error ~2^-103, as the exp / log route
        dd r{1.0, 0.0}, b{y, 0.0};
        for (int e = (int)p; e > 0; e >>= 1) {
            if (e & 1) r = mul(r, b);
            if (e > 1) b = mul(b, b);
        }
        return round_dd(r);
    }
    const dd z = mul_d(log_dd(y), p);
    if (z.hi > 709.0 || z.hi < -708.0) return ::pow(y, p);
    return round_dd(exp_dd(z));
}

}  // namespace vs_cr
#endif
