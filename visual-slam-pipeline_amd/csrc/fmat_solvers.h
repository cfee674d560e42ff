// fmat_solvers.h — host/device numerical kernels behind the F-matrix verification of
// Slam::process_frame (reference src/Slam.cpp:880-910, 930-948: cv::findFundamentalMat(pts1,
// pts2, FM_RANSAC, 3.0, RANSAC_PROB = 0.999) and compute_epipolar_error :1217-1240).
//
// OpenCV 4.x (external, unpinned) restated from its published algorithm (fundam.cpp,
// ptsetreg.cpp):
//   * n < 7: no model; n == 7: a single 7-point solve (first root here; OpenCV stacks all roots);
//   * n >= 15: RANSACPointSetRegistrator(7 points, thr, conf, maxIters = 1000);
//     8 <= n < 15: LMeDSPointSetRegistrator(7 points, conf, maxIters) — outlier ratio 0.45,
//     niters = max(RANSACUpdateNumIters(conf, 0.45, 7, maxIters), 3), smallest median error
//     wins, inliers within sigma = max(2.5 * 1.4826 * (1 + 5 / (n - 7)) * sqrt(median), 0.001);
//   * subsets: cv::RNG((uint64)-1), 7 distinct indices, rejected as a whole (up to the
//     registrator's attempt limit) when the 7th point of either image lies on a line through
//     two earlier ones (haveCollinearPoints, checkPartialSubsets = false);
//   * run7Point with Hartley normalisation (centroid, mean distance sqrt(2)), the 2-D null space
//     of the 7 x 9 system, the cubic det(lambda f1 + (1 - lambda) f2) = 0 (cv::solveCubic), each
//     root de-normalised and scaled so F(3,3) = 1;
//   * error: max(d1^2 s1, d2^2 s2) as float (FMEstimatorCallback::computeError), inlier iff
//     err <= (float)(thr^2); the RANSAC path returns the best 7-point model without a refit.
// All fp64 with identical operation order on host (oracle/orc_fmat.cpp) and device (fmat.hip).
#pragma once

#include "pnp_solvers.h"

namespace vs_fm {

using vs_pnp::CvRng;

constexpr int kModelPoints = 7;

// haveCollinearPoints(m, count) for the last point of a subset (x[i], y[i] fp32)
VS_HD inline bool have_collinear(const float* x, const float* y, int count) {
    const int i = count - 1;
    for (int j = 0; j < i; j++) {
        const double dx1 = (double)x[j] - (double)x[i], dy1 = (double)y[j] - (double)y[i];
        for (int k = 0; k < j; k++) {
            const double dx2 = (double)x[k] - (double)x[i], dy2 = (double)y[k] - (double)y[i];
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

// getSubset (checkPartialSubsets = false) for the F-matrix callback; p1/p2 interleaved xy fp32.
// Returns false when every attempt was degenerate.
VS_HD inline bool get_subset(CvRng& rng, const float* p1, const float* p2, int n, int max_attempts, int* idx) {
    for (int attempt = 0; attempt < max_attempts; attempt++) {
        for (int i = 0; i < kModelPoints; i++)
            for (;;) {
                idx[i] = rng.uniform(0, n);
                int j = 0;
                while (j < i && idx[j] != idx[i]) j++;
                if (j == i) break;
            }
        float x1[kModelPoints], y1[kModelPoints], x2[kModelPoints], y2[kModelPoints];
        for (int i = 0; i < kModelPoints; i++) {
            x1[i] = p1[2 * idx[i]];
            y1[i] = p1[2 * idx[i] + 1];
            x2[i] = p2[2 * idx[i]];
            y2[i] = p2[2 * idx[i] + 1];
        }
        if (!have_collinear(x1, y1, kModelPoints) && !have_collinear(x2, y2, kModelPoints)) return true;
    }
    return false;
}

// cv::solveCubic for c[0] x^3 + c[1] x^2 + c[2] x + c[3] = 0; returns the root count (-1: any x)
VS_HD inline int solve_cubic(const double* c, double* x) {
    double a0 = c[0], a1 = c[1], a2 = c[2], a3 = c[3];
    int n = 0;
    if (a0 == 0) {
        if (a1 == 0) {
            if (a2 == 0)
                n = a3 == 0 ? -1 : 0;
            else {
                x[0] = -a3 / a2;
                n = 1;
            }
        } else {
            double d = a2 * a2 - 4 * a1 * a3;
            if (d >= 0) {
                d = sqrt(d);
                const double q1 = (-a2 + d) * 0.5, q2 = (a2 + d) * -0.5;
                if (fabs(q1) > fabs(q2)) {
                    x[0] = q1 / a1;
                    x[1] = a3 / q1;
                } else {
                    x[0] = q2 / a1;
                    x[1] = a3 / q2;
                }
                n = d > 0 ? 2 : 1;
            }
        }
    } else {
        a0 = 1. / a0;
        a1 *= a0;
        a2 *= a0;
        a3 *= a0;
        const double Q = (a1 * a1 - 3 * a2) * (1. / 9);
        const double R = (a1 * (2 * a1 * a1 - 9 * a2) + 27 * a3) * (1. / 54);
        const double Qcubed = Q * Q * Q;
        double d = Qcubed - R * R;
        if (d >= 0) {
            const double theta = vs_cr::acos(R / sqrt(Qcubed));
            const double sqrtQ = sqrt(Q);
            const double t0 = -2 * sqrtQ, t1 = theta * (1. / 3), t2 = a1 * (1. / 3);
            x[0] = t0 * vs_cr::cos(t1) - t2;
            x[1] = t0 * vs_cr::cos(t1 + (2. * M_PI / 3)) - t2;
            x[2] = t0 * vs_cr::cos(t1 + (4. * M_PI / 3)) - t2;
            n = 3;
        } else {
            d = sqrt(-d);
            double e = vs_cr::pow(d + fabs(R), 1. / 3);
            if (R > 0) e = -e;
            x[0] = (e + Q / e) - a1 * (1. / 3);
            n = 1;
        }
    }
    return n;
}

// run7Point: up to 3 fundamental matrices (row-major) from 7 correspondences.
VS_HD inline int run_7point(const float* x1, const float* y1, const float* x2, const float* y2, double (*F)[9]) {
    double m1cx = 0, m1cy = 0, m2cx = 0, m2cy = 0;
    for (int i = 0; i < 7; i++) {
        m1cx += (double)x1[i];
        m1cy += (double)y1[i];
        m2cx += (double)x2[i];
        m2cy += (double)y2[i];
    }
    const double t = 1. / 7;
    m1cx *= t;
    m1cy *= t;
    m2cx *= t;
    m2cy *= t;
    double scale1 = 0, scale2 = 0;
    for (int i = 0; i < 7; i++) {
        const double ax = (double)x1[i] - m1cx, ay = (double)y1[i] - m1cy;
        const double bx = (double)x2[i] - m2cx, by = (double)y2[i] - m2cy;
        scale1 += sqrt(ax * ax + ay * ay);
        scale2 += sqrt(bx * bx + by * by);
    }
    scale1 *= t;
    scale2 *= t;
    if (scale1 < FLT_EPSILON || scale2 < FLT_EPSILON) return 0;
    scale1 = sqrt(2.) / scale1;
    scale2 = sqrt(2.) / scale2;
    double a[7][9];
    for (int i = 0; i < 7; i++) {
        const double X0 = ((double)x1[i] - m1cx) * scale1, Y0 = ((double)y1[i] - m1cy) * scale1;
        const double X1 = ((double)x2[i] - m2cx) * scale2, Y1 = ((double)y2[i] - m2cy) * scale2;
        a[i][0] = X1 * X0;
        a[i][1] = X1 * Y0;
        a[i][2] = X1;
        a[i][3] = Y1 * X0;
        a[i][4] = Y1 * Y0;
        a[i][5] = Y1;
        a[i][6] = X0;
        a[i][7] = Y0;
        a[i][8] = 1;
    }
    // 2-D null space of A by Gaussian elimination with partial pivoting (OpenCV takes the last two
    // right singular vectors; any basis spans the same pencil and the F(3,3) = 1 normalisation
    // below removes the basis).  Row swaps are selects so the unrolled matrix stays in registers.
    VS_UNROLL
    for (int k = 0; k < 7; k++) {
        int p = k;
        double big = fabs(a[k][k]);
    VS_UNROLL
        for (int r = k + 1; r < 7; r++) {
            const double v = fabs(a[r][k]);
            if (v > big) {
                big = v;
                p = r;
            }
        }
        if (!(big > 1e-300)) return 0;  // rank-deficient subset
    VS_UNROLL
        for (int r = k + 1; r < 7; r++) {
            const bool sw = r == p;
    VS_UNROLL
            for (int j = k; j < 9; j++) {
                const double ak = a[k][j], ar = a[r][j];
                a[k][j] = sw ? ar : ak;
                a[r][j] = sw ? ak : ar;
            }
        }
        const double inv = 1.0 / a[k][k];
    VS_UNROLL
        for (int r = k + 1; r < 7; r++) {
            const double f = a[r][k] * inv;
    VS_UNROLL
            for (int j = k + 1; j < 9; j++) a[r][j] -= f * a[k][j];
        }
    }
    // back substitution with the free unknowns (f[7], f[8]) = (1, 0) and (0, 1)
    double f1[9], f2[9];
    f1[7] = 1;
    f1[8] = 0;
    f2[7] = 0;
    f2[8] = 1;
    VS_UNROLL
    for (int k = 6; k >= 0; k--) {
        double s1 = a[k][7], s2 = a[k][8];
    VS_UNROLL
        for (int j = k + 1; j < 7; j++) {
            s1 += a[k][j] * f1[j];
            s2 += a[k][j] * f2[j];
        }
        f1[k] = -s1 / a[k][k];
        f2[k] = -s2 / a[k][k];
    }
    for (int i = 0; i < 9; i++) f1[i] -= f2[i];
    double c[4];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    double r[3] = {0, 0, 0};
    const int n = solve_cubic(c, r);
    if (n < 1 || n > 3) return n < 0 ? 0 : n;
    // T1 = [s1 0 -s1 m1cx; 0 s1 -s1 m1cy; 0 0 1], T2 likewise; F = T2^T Fn T1
    VS_UNROLL
    for (int k = 0; k < 3; k++) {  // unrolled with a guard: constant indices keep F, r in registers
        if (k < n) {
            double lambda = r[k], mu = 1.;
            double s = f1[8] * r[k] + f2[8];
            double Fn[9];
            if (fabs(s) > DBL_EPSILON) {
                mu = 1. / s;
                lambda *= mu;
                Fn[8] = 1.;
            } else {
                Fn[8] = 0.;
            }
            for (int i = 0; i < 8; i++) Fn[i] = f1[i] * lambda + f2[i] * mu;
            const double T1[9] = {scale1, 0, -scale1 * m1cx, 0, scale1, -scale1 * m1cy, 0, 0, 1};
            const double T2[9] = {scale2, 0, -scale2 * m2cx, 0, scale2, -scale2 * m2cy, 0, 0, 1};
            double tmp[9];
            VS_UNROLL
            for (int i = 0; i < 3; i++)  // tmp = T2^T Fn
                VS_UNROLL
                for (int j = 0; j < 3; j++)
                    tmp[i * 3 + j] = T2[0 * 3 + i] * Fn[0 * 3 + j] + T2[1 * 3 + i] * Fn[1 * 3 + j] + T2[2 * 3 + i] * Fn[2 * 3 + j];
            VS_UNROLL
            for (int i = 0; i < 3; i++)  // F = tmp T1
                VS_UNROLL
                for (int j = 0; j < 3; j++)
                    F[k][i * 3 + j] = tmp[i * 3 + 0] * T1[0 * 3 + j] + tmp[i * 3 + 1] * T1[1 * 3 + j] + tmp[i * 3 + 2] * T1[2 * 3 + j];
            if (fabs(F[k][8]) > FLT_EPSILON) {
                const double sc = 1. / F[k][8];
                for (int i = 0; i < 9; i++) F[k][i] *= sc;
            }
        }
    }
    return n;
}

// FMEstimatorCallback::computeError for one correspondence
VS_HD inline float fm_error(const double* F, float x1, float y1, float x2, float y2) {
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1. / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1. / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 > e2 ? e1 : e2);
}

// fm_error(F, ...) <= thr2, decided without the two divisions except within 1e-6 (relative) of
// the gate, where the exact OpenCV rounding (double error, float cast) is evaluated.  Outside
// that band the products' rounding (~1e-16) and the float cast (<= 6e-8) cannot change the
// outcome, so the result is identical to the exact comparison for every input.
VS_HD inline bool fm_inlier(const double* F, float x1, float y1, float x2, float y2, float thr2) {
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double q2 = a * a + b * b, d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double q1 = a * a + b * b, d1 = x1 * a + y1 * b + c;
    if (q1 > 0 && q2 > 0 && q1 < 1e300 && q2 < 1e300) {
        const double e1 = d1 * d1, e2 = d2 * d2, t = thr2;
        const double lo = t * (1.0 - 1e-6), hi = t * (1.0 + 1e-6);
        if (e1 <= lo * q1 && e2 <= lo * q2) return true;
        if (e1 >= hi * q1 || e2 >= hi * q2) return false;
    }
    return fm_error(F, x1, y1, x2, y2) <= thr2;
}

// one term of Slam::compute_epipolar_error (Slam.cpp:1226-1236); returns false when skipped
VS_HD inline bool epipolar_term(const double* F, float x1, float y1, float x2, float y2, double& term) {
    const double fx0 = F[0] * x1 + F[1] * y1 + F[2] * 1.0;
    const double fx1 = F[3] * x1 + F[4] * y1 + F[5] * 1.0;
    const double fx2 = F[6] * x1 + F[7] * y1 + F[8] * 1.0;
    const double num = fabs((double)x2 * fx0 + (double)y2 * fx1 + 1.0 * fx2);
    const double denom = sqrt(fx0 * fx0 + fx1 * fx1);
    if (!(denom > 1e-10)) return false;
    term = num / denom;
    return true;
}

}  // namespace vs_fm
