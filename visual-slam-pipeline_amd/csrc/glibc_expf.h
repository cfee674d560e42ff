// glibc_expf.h — bit-exact restatement of glibc's single-precision expf for host and device.
//
// The reference computes the SuperPoint softmax with std::exp(float) (FeatureExtractor.cpp:137),
// i.e. glibc's expf, which is NOT correctly rounded (about 1e-4 of inputs in [-110, 0] differ
// from (float)exp((double)x)).  Keypoint scores are only bit-exact if the GPU reproduces glibc's
// own algorithm: the ARM optimized-routines expf that glibc >= 2.27 ships (table of 2^(i/32),
// cubic polynomial in double).  x86-64 glibc selects its FMA variant (__expf_fma) on every CPU
// with FMA+AVX2 (any MI355X host); the operation sequence below is that variant's, instruction
// for instruction (constants and table as in glibc 2.35 e_exp2f_data.c).  The exhaustive host
// test (tests/test_oracle.py::test_glibc_expf_restatement_exhaustive) compares it with the
// running libm over every float in [-110, 0].
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define VS_HD __host__ __device__
#else
#define VS_HD
#endif

namespace vs_expf {

#if defined(__HIP_DEVICE_COMPILE__)
__device__ static const uint64_t kTab[32] = {
#else
static const uint64_t kTab[32] = {
#endif
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

VS_HD inline double as_double(uint64_t u) { return __builtin_bit_cast(double, u); }
VS_HD inline uint64_t as_u64(double d) { return __builtin_bit_cast(uint64_t, d); }
VS_HD inline uint32_t as_u32(float f) { return __builtin_bit_cast(uint32_t, f); }
VS_HD inline float as_float(uint32_t u) { return __builtin_bit_cast(float, u); }

// use_fma = 1: __expf_fma (FMA+AVX2 hosts); 0: the SSE2 variant, for completeness.
VS_HD inline float glibc_expf(float x, int use_fma = 1) {
    const double kShift = as_double(0x4338000000000000ull);    // 0x1.8p52
    const double kInvLn2N = as_double(0x40471547652b82feull);  // 32/ln2
    const double kC0 = as_double(0x3ebc6af84b912394ull);
    const double kC1 = as_double(0x3f2ebfce50fac4f3ull);
    const double kC2 = as_double(0x3f962e42ff0c52d6ull);
    const uint32_t ux = as_u32(x);
    const uint32_t abstop = (ux >> 20) & 0x7ff;
    if (abstop > 0x42a) {                              // |x| >= 88 or nan
        if (ux == 0xff800000u) return 0.0f;            // -inf
        if (abstop > 0x7f7) return x + x;              // inf, nan
        if (x > as_float(0x42b17217u)) return as_float(0x7f800000u);   // __math_oflowf
        if (x < as_float(0xc2cff1b4u)) return 0.0f;                    // __math_uflowf
        if (x < as_float(0xc2ce8ecfu)) return as_float(0x00000001u);   // __math_may_uflowf
    }
    const double xd = (double)x;
    double kd, r, z, y;
    uint64_t ki;
    if (use_fma) {
        kd = fma(kInvLn2N, xd, kShift);
        ki = as_u64(kd);
        kd -= kShift;
        r = fma(kInvLn2N, xd, -kd);
    } else {
        z = xd * kInvLn2N;
        kd = kShift + z;
        ki = as_u64(kd);
        kd -= kShift;
        r = z - kd;
    }
    uint64_t t = kTab[ki & 31];
    t += ki << 47;
    const double s = as_double(t);
    if (use_fma) {
        z = fma(r, kC0, kC1);
        const double r2 = r * r;
        y = fma(r, kC2, 1.0);
        y = fma(z, r2, y);
    } else {
        double a = kC2 * r;
        z = kC0 * r;
        a = a + 1.0;
        const double r2 = r * r;
        z = z + kC1;
        z = z * r2;
        y = z + a;
    }
    y = y * s;
    return (float)y;
}

}  // namespace vs_expf
