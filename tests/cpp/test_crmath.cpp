// CPU check of csrc/cr_math.h's double-double implementation (the code the device runs) against
// libquadmath's binary128 functions rounded to double: both must give the correctly rounded
// result, so they must agree bit for bit.  Built by oracle/Makefile (crmath_test), run by
// tests/test_crmath.py.  Prints the mismatch count per function; exit status 1 on any mismatch.
#include <quadmath.h>

#include <cmath>
#include <cstdio>
#include <random>

#include "../../visual-slam-pipeline_amd/csrc/cr_math.h"

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 200000;
    std::mt19937_64 g(20261016);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad[5] = {0, 0, 0, 0, 0};
    auto chk = [&](int k, double got, __float128 want) { bad[k] += got != (double)want; };
    for (int i = 0; i < N; i++) {
        const double x = (U(g) * 2 - 1) * 8;  // Rodrigues angles, the cubic's angles
        const double tiny = std::ldexp(U(g), -(int)(U(g) * 60));
        const double c = U(g) * 2 - 1, c1 = 1 - std::ldexp(U(g), -(int)(U(g) * 50));
        const double y = std::exp((U(g) * 2 - 1) * 40), p = U(g) * 10 - 3, u = U(g);
        chk(0, vs_cr::sin(x), sinq(x));
        chk(0, vs_cr::sin(tiny), sinq(tiny));
        chk(1, vs_cr::cos(x), cosq(x));
        chk(1, vs_cr::cos(tiny), cosq(tiny));
        chk(2, vs_cr::acos(c), acosq(c));
        chk(2, vs_cr::acos(c1), acosq(c1));
        chk(2, vs_cr::acos(-c1), acosq(-c1));
        chk(3, vs_cr::log(y), logq(y));
        chk(4, vs_cr::pow(y, p * 0.5), powq(y, p * 0.5));
        chk(4, vs_cr::pow(u, 5.0), powq(u, 5.0));  // RANSACUpdateNumIters: (1 - ep)^modelPoints
        chk(4, vs_cr::pow(u, 7.0), powq(u, 7.0));  // the F-matrix registrator's 7-point subsets
        chk(4, vs_cr::pow(y, (double)(2 + i % 7)), powq(y, (double)(2 + i % 7)));
        double sn, cs;  // sincos = (sin, cos); arguments near the table knots j/64 and near k pi/4
        const double knot = std::ldexp(std::floor(U(g) * 100) - 50, -6) + (U(g) - 0.5) * 1e-12;
        vs_cr::sincos(knot, sn, cs);
        chk(0, sn, sinq(knot));
        chk(1, cs, cosq(knot));
        const double q4 = (std::floor(U(g) * 16) - 8) * 0.7853981633974483 + (U(g) - 0.5) * 1e-9;
        vs_cr::sincos(q4, sn, cs);
        chk(0, sn, sinq(q4));
        chk(1, cs, cosq(q4));
    }
    std::printf("mismatches sin %ld cos %ld acos %ld log %ld pow %ld over %d draws\n", bad[0], bad[1], bad[2], bad[3],
                bad[4], N);
    return (bad[0] | bad[1] | bad[2] | bad[3] | bad[4]) ? 1 : 0;
}
