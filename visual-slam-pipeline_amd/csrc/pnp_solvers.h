// pnp_solvers.h — host/device numerical kernels behind Slam::solve_pnp (reference
// src/Slam.cpp:505-529 -> cv::solvePnPRansac, SOLVEPNP_ITERATIVE, useExtrinsicGuess = false).
//
// OpenCV 4.x semantics restated from its published algorithm (external, unpinned):
//   * RANSAC registrator: cv::RNG((uint64)-1), 5-point subsets drawn with rejection of repeats,
//     EPnP hypotheses, inlier iff the float squared reprojection error <= (float)(thr^2),
//     a model replaces the best when its count exceeds max(best, modelPoints-1), iteration budget
//     shrunk by RANSACUpdateNumIters(confidence, outlier ratio, 5, niters);
//   * EPnP (Lepetit, Moreno-Noguer, Fua 2009): four control points from the PCA of the object
//     points, barycentric coordinates, the 12x12 M^T M null space, the N = 4 / 2 / 3 beta
//     approximations refined by 5 Gauss-Newton steps, the lowest reprojection error wins;
//   * final refinement on the RANSAC inliers: Levenberg-Marquardt over (rvec, tvec) from the
//     RANSAC model, Marquardt-scaled diagonal, lambda 1e-3 (/10 on success, x10 on failure),
//     at most 20 iterations.
// Everything is fp64 and written once for host (oracle/, the CPU restatement) and device
// (pnp.hip) with identical operation order; the solver's correctness is pinned by known-answer
// tests (tests/test_oracle_pnp.py), not by the oracle.
#pragma once

#include <float.h>
#include <math.h>
#include <stdint.h>

#include "cr_math.h"  // correctly rounded sin / cos / acos / log / pow (host == device)

#if defined(__HIPCC__)
#define VS_HD __host__ __device__
#define VS_UNROLL _Pragma("unroll")
#define VS_NOUNROLL _Pragma("unroll 1")
#else
#define VS_HD
#define VS_UNROLL
#define VS_NOUNROLL
#endif

namespace vs_pnp {

// ---------------------------------------------------------------------------- cv::RNG
struct CvRng {
    uint64_t state;
    VS_HD explicit CvRng(uint64_t s) : state(s ? s : (uint64_t)-1) {}
    VS_HD unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    VS_HD int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a)) + a; }
};

// Jump-ahead for cv::RNG.  One step s' = lo32(s) * A + hi32(s) is multiplication by A modulo
// M = A * 2^32 - 1 (A * 2^32 == 1 mod M), for every state 1 <= s < M (all states after the first
// step of (uint64)-1; the representation is the residue).  k steps = multiplication by A^k mod M,
// done in Montgomery form (R = 2^64): kMwcR1 = 2^64 mod M is the Montgomery one, stepping the
// generator k times from it gives Mont(A^k), and mwc_mont_mul(s, Mont(A^k)) = s * A^k mod M.
constexpr uint64_t kMwcA = 4164903690u;
constexpr uint64_t kMwcM = (kMwcA << 32) - 1;
constexpr uint64_t kMwcR1 = 0 - kMwcM;  // 2^64 - M (M > 2^63)
constexpr uint64_t mwc_neg_inv() {      // -M^-1 mod 2^64 by Newton's iteration
    uint64_t x = kMwcM;                 // correct to 3 bits (M odd)
    for (int i = 0; i < 6; i++) x *= 2 - kMwcM * x;
    return 0 - x;
}
constexpr uint64_t kMwcMInv = mwc_neg_inv();

VS_HD constexpr uint64_t mwc_step(uint64_t s) { return (uint64_t)(unsigned)s * kMwcA + (unsigned)(s >> 32); }

VS_HD inline uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// x * y / 2^64 mod M for x, y < M (REDC; the 65-bit intermediate is < 2M)
VS_HD inline uint64_t mwc_mont_mul(uint64_t x, uint64_t y) {
    const uint64_t lo = x * y, hi = mulhi64(x, y);
    const uint64_t q = lo * kMwcMInv;
    const uint64_t qh = mulhi64(q, kMwcM);  // lo + q * M == 0 mod 2^64: carry iff lo != 0
    const uint64_t u = hi + qh;
    const bool c1 = u < hi;
    const uint64_t v = u + (lo != 0);
    const bool c2 = v < u;
    return (c1 || c2 || v >= kMwcM) ? v - kMwcM : v;
}

// The state k steps after s, given mont_pow_k = Mont(A^k).  s may be any state reached by at least
// one step (the first step of (uint64)-1 lands on M + 2^32 - A, above M: its residue is used; every
// later state is its own residue).
VS_HD inline uint64_t mwc_jump(uint64_t s, int k, uint64_t mont_pow_k) {
    return k == 0 ? s : mwc_mont_mul(s >= kMwcM ? s - kMwcM : s, mont_pow_k);
}

// cv::RANSACUpdateNumIters
// log(max(1 - p, DBL_MIN)) of RANSACUpdateNumIters (p clamped to [0, 1]): constant per caller,
// so replay loops compute it once
VS_HD inline double ransac_log_num(double p) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    return vs_cr::log((1. - p) > DBL_MIN ? (1. - p) : DBL_MIN);
}
// RANSACUpdateNumIters in two parts: the outlier-ratio term log(1 - (1 - ep)^m), which does not
// depend on the running budget (a device evaluates it for every hypothesis at once; +inf marks
// OpenCV's denom < DBL_MIN exit), and the budget update from it.
VS_HD inline double ransac_log_denom(double ep, int model_points) {
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    const double denom = 1. - vs_cr::pow(1. - ep, model_points);
    if (denom < DBL_MIN) return HUGE_VAL;
    return vs_cr::log(denom);
}
VS_HD inline int ransac_update_from_denom(double log_num, double denom, int max_iters) {
    if (denom == HUGE_VAL) return 0;
    const double num = log_num;
    if (denom >= 0 || -num >= max_iters * (-denom)) return max_iters;
    return (int)lrint(num / denom);  // cvRound
}
VS_HD inline int ransac_update_num_iters_ln(double log_num, double ep, int model_points, int max_iters) {
    return ransac_update_from_denom(log_num, ransac_log_denom(ep, model_points), max_iters);
}
VS_HD inline int ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    return ransac_update_num_iters_ln(ransac_log_num(p), ep, model_points, max_iters);
}

// ------------------------------------------------------------- small dense linear algebra
// The Jacobi rotation (c, s) that zeroes A[p][q]: with d = A[q][q] - A[p][p], h = 2 A[p][q],
// r = |(d, h)|, the classic t = tan = sgn(d) h / (|d| + r) gives c = 1 / sqrt(1 + t^2) =
// (|d| + r) / w and s = t c = sgn(d) h / w with w = sqrt(2 r (|d| + r)): two square roots and two
// independent divisions (the textbook form chains three divisions and two roots; on the device
// that chain is each Jacobi round's latency).  No cancellation: every sum adds non-negative terms.
// Rotations with |A[p][q]| < 1e-150 are skipped (h^2 stays a normal number).
VS_HD inline bool jacobi_angle(double app, double aqq, double apq, double& c, double& s) {
    if (fabs(apq) < 1e-150) return false;
    const double d = aqq - app, h = 2.0 * apq;
    const double r = sqrt(d * d + h * h);
    const double u = fabs(d) + r;
    const double w = sqrt(2.0 * r * u);
    c = u / w;
    s = (d >= 0 ? h : -h) / w;
    return true;
}
// The same arithmetic without the early exit, for the device's parallel rounds: (c, s) are
// computed unconditionally (meaningless when the rotation is skipped — the caller selects on the
// flag), so a lane's two angles compile to one straight-line pair of interleaved chains instead of
// two serialised branches.  Where the rotation runs, (c, s) are bit-identical to jacobi_angle's.
VS_HD inline bool jacobi_angle_nb(double app, double aqq, double apq, double& c, double& s) {
    const double d = aqq - app, h = 2.0 * apq;
    const double r = sqrt(d * d + h * h);
    const double u = fabs(d) + r;
    const double w = sqrt(2.0 * r * u);
    c = u / w;
    s = (d >= 0 ? h : -h) / w;
    return !(fabs(apq) < 1e-150);
}

// Cyclic Jacobi eigen-decomposition of the symmetric n x n matrix A (row-major, destroyed):
// w[k] eigenvalues in descending order, V[i*n + k] the k-th eigenvector (columns).
template <int N>
VS_HD void sym_eig(double* A, double* w, double* V) {
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) V[i * N + j] = (i == j) ? 1.0 : 0.0;
    double total = 0;
    for (int i = 0; i < N * N; i++) total += A[i] * A[i];
    for (int sweep = 0; sweep < 30; sweep++) {
        double off = 0;
        for (int p = 0; p < N; p++)
            for (int q = p + 1; q < N; q++) off += A[p * N + q] * A[p * N + q];
        if (!(off > 1e-32 * total)) break;
        for (int p = 0; p < N - 1; p++)
            for (int q = p + 1; q < N; q++) {
                double c, s;
                if (!jacobi_angle(A[p * N + p], A[q * N + q], A[p * N + q], c, s)) continue;
                for (int k = 0; k < N; k++) {
                    const double akp = A[k * N + p], akq = A[k * N + q];
                    A[k * N + p] = c * akp - s * akq;
                    A[k * N + q] = s * akp + c * akq;
                }
                for (int k = 0; k < N; k++) {
                    const double apk = A[p * N + k], aqk = A[q * N + k];
                    A[p * N + k] = c * apk - s * aqk;
                    A[q * N + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < N; k++) {
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = c * vkp - s * vkq;
                    V[k * N + q] = s * vkp + c * vkq;
                }
            }
    }
    for (int i = 0; i < N; i++) w[i] = A[i * N + i];
    for (int i = 0; i < N - 1; i++) {  // selection sort, descending
        int m = i;
        for (int j = i + 1; j < N; j++)
            if (w[j] > w[m]) m = j;
        if (m != i) {
            const double tw = w[i];
            w[i] = w[m];
            w[m] = tw;
            for (int k = 0; k < N; k++) {
                const double tv = V[k * N + i];
                V[k * N + i] = V[k * N + m];
                V[k * N + m] = tv;
            }
        }
    }
}

// sym_eig with every index static once unrolled (the device keeps A, V and w in registers instead of
// a private array indexed at run time): the same rotations in the same order, the same selection sort
// (the running maximum's value tracked beside its position; the swaps as selects), the same results.
template <int N>
VS_HD void sym_eig_static(double* A, double* w, double* V) {
    VS_UNROLL
    for (int i = 0; i < N; i++)
        VS_UNROLL
        for (int j = 0; j < N; j++) V[i * N + j] = (i == j) ? 1.0 : 0.0;
    double total = 0;
    VS_UNROLL
    for (int i = 0; i < N * N; i++) total += A[i] * A[i];
    VS_NOUNROLL
    for (int sweep = 0; sweep < 30; sweep++) {
        double off = 0;
        VS_UNROLL
        for (int p = 0; p < N; p++)
            VS_UNROLL
            for (int q = p + 1; q < N; q++) off += A[p * N + q] * A[p * N + q];
        if (!(off > 1e-32 * total)) break;
        VS_UNROLL
        for (int p = 0; p < N - 1; p++)
            VS_UNROLL
            for (int q = p + 1; q < N; q++) {
                double c, s;
                if (!jacobi_angle(A[p * N + p], A[q * N + q], A[p * N + q], c, s)) continue;
                VS_UNROLL
                for (int k = 0; k < N; k++) {
                    const double akp = A[k * N + p], akq = A[k * N + q];
                    A[k * N + p] = c * akp - s * akq;
                    A[k * N + q] = s * akp + c * akq;
                }
                VS_UNROLL
                for (int k = 0; k < N; k++) {
                    const double apk = A[p * N + k], aqk = A[q * N + k];
                    A[p * N + k] = c * apk - s * aqk;
                    A[q * N + k] = s * apk + c * aqk;
                }
                VS_UNROLL
                for (int k = 0; k < N; k++) {
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = c * vkp - s * vkq;
                    V[k * N + q] = s * vkp + c * vkq;
                }
            }
    }
    VS_UNROLL
    for (int i = 0; i < N; i++) w[i] = A[i * N + i];
    VS_UNROLL
    for (int i = 0; i < N - 1; i++) {  // selection sort, descending
        int m = i;
        double wm = w[i];
        VS_UNROLL
        for (int j = i + 1; j < N; j++)
            if (w[j] > wm) {
                wm = w[j];
                m = j;
            }
        if (m != i) {
            const double tw = w[i];
            w[i] = wm;
            VS_UNROLL
            for (int j = i + 1; j < N; j++)
                if (j == m) w[j] = tw;
            VS_UNROLL
            for (int k = 0; k < N; k++) {
                const double tv = V[k * N + i];
                double vm = tv;
                VS_UNROLL
                for (int j = i + 1; j < N; j++) vm = j == m ? V[k * N + j] : vm;
                V[k * N + i] = vm;
                VS_UNROLL
                for (int j = i + 1; j < N; j++)
                    if (j == m) V[k * N + j] = tv;
            }
        }
    }
}

// Parallel-order Jacobi (even N): each sweep is N - 1 rounds of N / 2 disjoint rotations in the
// round-robin (circle) order; a round takes every angle from the matrix as the round starts, then
// applies all column rotations of A, all row rotations of A, and all column rotations of V.
// Every element receives at most one column and one row update per round, so the device can run
// a round's rotations in parallel and stay bit-identical to this sequential statement.  Same
// stopping rule and output convention as sym_eig (used for the EPnP 12 x 12 MtM).
VS_HD inline void rr_pair(int N, int r, int k, int& p, int& q) {
    const int a = k == 0 ? N - 1 : (r + k) % (N - 1);
    const int b = k == 0 ? r : (r - k + (N - 1)) % (N - 1);
    p = a < b ? a : b;
    q = a < b ? b : a;
}


template <int N>
VS_HD void sym_eig_rr(double* A, double* w, double* V) {
    static_assert(N % 2 == 0, "round-robin Jacobi needs an even order");
    constexpr int H = N / 2;
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) V[i * N + j] = (i == j) ? 1.0 : 0.0;
    double total = 0;
    for (int i = 0; i < N * N; i++) total += A[i] * A[i];
    for (int sweep = 0; sweep < 30; sweep++) {
        double off = 0;
        for (int p = 0; p < N; p++)
            for (int q = p + 1; q < N; q++) off += A[p * N + q] * A[p * N + q];
        if (!(off > 1e-32 * total)) break;
        for (int r = 0; r < N - 1; r++) {
            int P[H], Q[H];
            double C[H], S[H];
            bool act[H];
            for (int k = 0; k < H; k++) {
                rr_pair(N, r, k, P[k], Q[k]);
                act[k] = jacobi_angle(A[P[k] * N + P[k]], A[Q[k] * N + Q[k]], A[P[k] * N + Q[k]], C[k], S[k]);
            }
            for (int k = 0; k < H; k++) {
                if (!act[k]) continue;
                const int p = P[k], q = Q[k];
                for (int i = 0; i < N; i++) {
                    const double aip = A[i * N + p], aiq = A[i * N + q];
                    A[i * N + p] = C[k] * aip - S[k] * aiq;
                    A[i * N + q] = S[k] * aip + C[k] * aiq;
                }
            }
            for (int k = 0; k < H; k++) {
                if (!act[k]) continue;
                const int p = P[k], q = Q[k];
                for (int j = 0; j < N; j++) {
                    const double apj = A[p * N + j], aqj = A[q * N + j];
                    A[p * N + j] = C[k] * apj - S[k] * aqj;
                    A[q * N + j] = S[k] * apj + C[k] * aqj;
                }
            }
            for (int k = 0; k < H; k++) {
                if (!act[k]) continue;
                const int p = P[k], q = Q[k];
                for (int i = 0; i < N; i++) {
                    const double vip = V[i * N + p], viq = V[i * N + q];
                    V[i * N + p] = C[k] * vip - S[k] * viq;
                    V[i * N + q] = S[k] * vip + C[k] * viq;
                }
            }
        }
    }
    for (int i = 0; i < N; i++) w[i] = A[i * N + i];
    for (int i = 0; i < N - 1; i++) {  // selection sort, descending
        int m = i;
        for (int j = i + 1; j < N; j++)
            if (w[j] > w[m]) m = j;
        if (m != i) {
            const double tw = w[i];
            w[i] = w[m];
            w[m] = tw;
            for (int k = 0; k < N; k++) {
                const double tv = V[k * N + i];
                V[k * N + i] = V[k * N + m];
                V[k * N + m] = tv;
            }
        }
    }
}

// cv::triangulatePoints for one correspondence (OpenCV's icvTriangulatePoints restated: the 4x4
// DLT system, its right singular vector of the smallest singular value -- here the eigenvector of
// A^T A -- stored as float like the CV_32F pts4D of Slam.cpp:1276-1277).  Shared by the host
// tracker restatement and the GPU back end's per-match kernel.
VS_HD inline void dlt_point(const double P1[12], const double P2[12], float x1, float y1, float x2, float y2,
                            float X[4]);

// Pairwise sum of t[0..N) in a fixed tree (halves, the first one rounded up): the same order on
// host and device, log2(N) dependent additions instead of N - 1.  Callers pad skipped terms with
// -0.0 (x + -0.0 == x for every x, so padding never changes a sum and the device folds it away).
template <int N>
VS_HD inline double tsum(const double* t) {
    if constexpr (N == 1) {
        return t[0];
    } else {
        constexpr int H = (N + 1) / 2;
        return tsum<H>(t) + tsum<N - H>(t + H);
    }
}

// Least squares min ||A x - b|| for an M x N (M >= N) matrix by Householder QR (A, b destroyed).
// Column k's reflector u = (a_kk - alpha, a_k+1,k, ...) has u^T u = 2 |a| (|a| + |a_kk|), so one
// division per column (tau = 2 / u^T u) replaces one per updated column; R_kk = alpha exactly and
// back substitution multiplies by 1 / alpha.  A zero column is skipped (x = 0 for it): trailing zero
// columns leave the other unknowns bit-identical (epnp_betas_init_uniform relies on this).
template <int M, int N>
VS_HD void lstsq(double* A, double* b, double* x) {
    double inv[N];
    VS_UNROLL
    for (int k = 0; k < N; k++) {
        double t[M];
        VS_UNROLL
        for (int i = 0; i < M; i++) t[i] = i >= k ? A[i * N + k] * A[i * N + k] : -0.0;
        const double s = tsum<M>(t);
        inv[k] = 0.0;
        if (!(s > 0)) continue;
        const double nrm = sqrt(s), akk = A[k * N + k];
        const double alpha = akk > 0 ? -nrm : nrm;
        const double tau = 1.0 / (nrm * (nrm + fabs(akk)));
        double u[M];
        VS_UNROLL
        for (int i = 0; i < M; i++) u[i] = i > k ? A[i * N + k] : i == k ? akk - alpha : 0.0;
        VS_UNROLL
        for (int j = k + 1; j < N; j++) {
            VS_UNROLL
            for (int i = 0; i < M; i++) t[i] = i >= k ? u[i] * A[i * N + j] : -0.0;
            const double f = tau * tsum<M>(t);
            VS_UNROLL
            for (int i = k; i < M; i++) A[i * N + j] = A[i * N + j] - f * u[i];
        }
        VS_UNROLL
        for (int i = 0; i < M; i++) t[i] = i >= k ? u[i] * b[i] : -0.0;
        const double f = tau * tsum<M>(t);
        VS_UNROLL
        for (int i = k; i < M; i++) b[i] = b[i] - f * u[i];
        A[k * N + k] = alpha;
        inv[k] = 1.0 / alpha;
    }
    VS_UNROLL
    for (int k = N - 1; k >= 0; k--) {
        double s = b[k];
        VS_UNROLL
        for (int j = k + 1; j < N; j++) s = s - A[k * N + j] * x[j];
        x[k] = s * inv[k];
    }
}

VS_HD inline double det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// R = argmin ||R A + t - B|| (Kabsch with reflection fix) from ABt = sum (b - cb)(a - ca)^T:
// SVD: V from the symmetric eigen-decomposition of ABt^T ABt, u0 and u1 from ABt v0 and ABt v1
// (Gram-Schmidt), u2 = u0 x u1.  With that u2, R = u0 v0^T + u1 v1^T + det(V) u2 v2^T is exactly
// U diag(1, 1, det(U V^T)) V^T, and it never divides by the smallest singular value.
VS_HD inline void rotation_from_cross(const double* ABt, double* R) {
    double AtA[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += ABt[k * 3 + i] * ABt[k * 3 + j];
            AtA[i * 3 + j] = s;
        }
    double w[3], V[9];
    sym_eig<3>(AtA, w, V);
    double u[3][3];
    for (int k = 0; k < 2; k++)
        for (int i = 0; i < 3; i++)
            u[k][i] = ABt[i * 3 + 0] * V[0 * 3 + k] + ABt[i * 3 + 1] * V[1 * 3 + k] + ABt[i * 3 + 2] * V[2 * 3 + k];
    double n0 = sqrt(u[0][0] * u[0][0] + u[0][1] * u[0][1] + u[0][2] * u[0][2]);
    n0 = n0 > 0 ? n0 : 1.0;
    for (int i = 0; i < 3; i++) u[0][i] /= n0;
    const double pr = u[0][0] * u[1][0] + u[0][1] * u[1][1] + u[0][2] * u[1][2];
    for (int i = 0; i < 3; i++) u[1][i] -= pr * u[0][i];
    double n1 = sqrt(u[1][0] * u[1][0] + u[1][1] * u[1][1] + u[1][2] * u[1][2]);
    n1 = n1 > 0 ? n1 : 1.0;
    for (int i = 0; i < 3; i++) u[1][i] /= n1;
    u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
    u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
    u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
    const double d = det3(V) < 0 ? -1.0 : 1.0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[i * 3 + j] = u[0][i] * V[j * 3 + 0] + u[1][i] * V[j * 3 + 1] + d * u[2][i] * V[j * 3 + 2];
}

// ----------------------------------------------------------------------------- Rodrigues
VS_HD inline void rod_v2m(const double r[3], double R[9]) {
    const double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < DBL_EPSILON) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double s, c;
    vs_cr::sincos(theta, s, c);  // one reduction for both (correctly rounded each)
    const double c1 = 1.0 - c;
    const double it = 1.0 / theta;
    const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int i = 0; i < 9; i++) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx[i];
}

VS_HD inline void rod_m2v(const double R[9], double r[3]) {
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = vs_cr::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            r[0] = r[1] = r[2] = 0;
            return;
        }
        double t = (R[0] + 1) * 0.5;
        rx = sqrt(fmax(t, 0.));
        t = (R[4] + 1) * 0.5;
        ry = sqrt(fmax(t, 0.)) * (R[1] < 0 ? -1. : 1.);
        t = (R[8] + 1) * 0.5;
        rz = sqrt(fmax(t, 0.)) * (R[2] < 0 ? -1. : 1.);
        if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
        theta /= sqrt(rx * rx + ry * ry + rz * rz);
        r[0] = rx * theta;
        r[1] = ry * theta;
        r[2] = rz * theta;
        return;
    }
    double vth = 1 / (2 * s);
    vth *= theta;
    r[0] = rx * vth;
    r[1] = ry * vth;
    r[2] = rz * vth;
}

// projection (world -> camera R, t; cv::projectPoints without distortion, double then float)
struct Cam {
    double fx, fy, cx, cy;
};

VS_HD inline void project(const double* R, const double* t, const Cam& K, double X, double Y, double Z, double& u,
                          double& v) {
    const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    const double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    const double iz = z ? 1.0 / z : 1.0;
    u = K.fx * (x * iz) + K.cx;
    v = K.fy * (y * iz) + K.cy;
}

// float squared reprojection error (PnPRansacCallback::computeError)
VS_HD inline float reproj_err2(const double* R, const double* t, const Cam& K, float X, float Y, float Z, float u,
                               float v) {
    double pu, pv;
    project(R, t, K, X, Y, Z, pu, pv);
    const float du = u - (float)pu, dv = v - (float)pv;
    return du * du + dv * dv;
}

// ----------------------------------------------------------------------------------- EPnP
// stage marks for the device's profiling build (cycle counters); everything else passes NoMark
struct NoMark {
    VS_HD void operator()(int) const {}
};
// Written as stages so the device can spread one hypothesis over a wave (pnp.hip): control
// points and barycentric coordinates, one M^T M entry at a time (each entry's sum runs over the
// points in order, as the host's row-pair accumulation does), the 12 x 12 eigen-decomposition,
// the L_6x10 / rho system, and one beta approximation (N = 4 / 2 / 3) refined and turned into a
// pose per call.  epnp() composes them sequentially; the device composes the same functions.

// Control points cw (centroid + principal axes) and barycentric coordinates; false if degenerate.
// MAXN bounds n at compile time (the point loops run to MAXN with an i < n guard, the same
// operations in the same order), so on the device they unroll over a register copy of the points.
template <int MAXN, class Mark = NoMark>
VS_HD inline bool epnp_control(const double* X, int n, double cw[4][3], double (*alphas)[4], Mark mark = Mark()) {
    for (int j = 0; j < 3; j++) {
        double s = 0;
        VS_UNROLL
        for (int i = 0; i < MAXN; i++)
            if (i < n) s += X[3 * i + j];
        cw[0][j] = s / n;
    }
    double C[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0;
            VS_UNROLL
            for (int i = 0; i < MAXN; i++)
                if (i < n) s += (X[3 * i + a] - cw[0][a]) * (X[3 * i + b] - cw[0][b]);
            C[a * 3 + b] = s;
        }
    mark(0);
    double dc[3], uc[9];
    sym_eig<3>(C, dc, uc);
    mark(1);
    // Each principal axis with its largest-magnitude component positive (the first on ties): the
    // control points, hence M and the QR basis of its null space (epnp_small_eig), stop depending
    // on the eigen-solver's arbitrary signs.
    for (int i = 0; i < 3; i++) {
        int r = 0;
        for (int q = 1; q < 3; q++)
            if (fabs(uc[q * 3 + i]) > fabs(uc[r * 3 + i])) r = q;
        if (uc[r * 3 + i] < 0)
            for (int q = 0; q < 3; q++) uc[q * 3 + i] = -uc[q * 3 + i];
    }
    for (int i = 1; i < 4; i++) {
        const double k = sqrt((dc[i - 1] > 0 ? dc[i - 1] : 0.0) / n);
        for (int j = 0; j < 3; j++) cw[i][j] = cw[0][j] + k * uc[j * 3 + (i - 1)];
    }
    // barycentric coordinates: CC a = p - cw0 with CC columns cw_i - cw0
    double CC[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) CC[r * 3 + c] = cw[c + 1][r] - cw[0][r];
    mark(2);
    const double det = det3(CC);
    if (fabs(det) < 1e-300) return false;
    double CI[9];
    CI[0] = (CC[4] * CC[8] - CC[5] * CC[7]) / det;
    CI[1] = (CC[2] * CC[7] - CC[1] * CC[8]) / det;
    CI[2] = (CC[1] * CC[5] - CC[2] * CC[4]) / det;
    CI[3] = (CC[5] * CC[6] - CC[3] * CC[8]) / det;
    CI[4] = (CC[0] * CC[8] - CC[2] * CC[6]) / det;
    CI[5] = (CC[2] * CC[3] - CC[0] * CC[5]) / det;
    CI[6] = (CC[3] * CC[7] - CC[4] * CC[6]) / det;
    CI[7] = (CC[1] * CC[6] - CC[0] * CC[7]) / det;
    CI[8] = (CC[0] * CC[4] - CC[1] * CC[3]) / det;
    VS_UNROLL
    for (int i = 0; i < MAXN; i++) {
        if (i >= n) continue;
        const double p[3] = {X[3 * i] - cw[0][0], X[3 * i + 1] - cw[0][1], X[3 * i + 2] - cw[0][2]};
        double a1 = CI[0] * p[0] + CI[1] * p[1] + CI[2] * p[2];
        double a2 = CI[3] * p[0] + CI[4] * p[1] + CI[5] * p[2];
        double a3 = CI[6] * p[0] + CI[7] * p[1] + CI[8] * p[2];
        alphas[i][1] = a1;
        alphas[i][2] = a2;
        alphas[i][3] = a3;
        alphas[i][0] = 1.0 - a1 - a2 - a3;
    }
    mark(3);
    return true;
}

// Row a of the two M rows of point i (M = [alpha_j fx, 0, alpha_j (cx - u)] / [0, alpha_j fy, ...]).
VS_HD inline double epnp_m0(const double* al, double u, const Cam& K, int a) {
    const double x = al[a / 3];
    return (a % 3 == 0) ? x * K.fx : (a % 3 == 1) ? 0.0 : x * (K.cx - u);
}
VS_HD inline double epnp_m1(const double* al, double v, const Cam& K, int a) {
    const double x = al[a / 3];
    return (a % 3 == 0) ? 0.0 : (a % 3 == 1) ? x * K.fy : x * (K.cy - v);
}
// (M^T M)[a][b], accumulated over the points in order
// (MAXN bounds n at compile time so the device unrolls the point loop, as in epnp_variant)
template <int MAXN>
VS_HD inline double epnp_mtm(const double (*alphas)[4], const double* uv, int n, const Cam& K, int a, int b) {
    double s = 0;
    VS_UNROLL
    for (int i = 0; i < MAXN; i++)
        if (i < n)
            s += epnp_m0(alphas[i], uv[2 * i], K, a) * epnp_m0(alphas[i], uv[2 * i], K, b) +
             epnp_m1(alphas[i], uv[2 * i + 1], K, a) * epnp_m1(alphas[i], uv[2 * i + 1], K, b);
    return s;
}

// ------------------------------------------- the four smallest eigenvectors for m = 4 / 5 points
// A RANSAC subset has m <= 5 points, so M (2m x 12) has rank <= 2m and M^T M a null space of
// dimension >= 12 - 2m.  Instead of diagonalising the 12 x 12 M^T M:
//   1. Householder QR of M^T (12 x 2m) = Q [R; 0]: M^T M = Q diag(R R^T, 0) Q^T, so the last
//      12 - 2m columns of Q span the null space exactly (m = 4: all four vectors, nothing else);
//   2. m = 5: the two smallest eigenpairs of B = R R^T (10 x 10): Householder tridiagonalisation
//      T = H_7..H_0 B H_0..H_7 (scaled by a power of two to ||T|| in [1, 2)), the two smallest
//      eigenvalues of T by 33-way multisection of the Sturm count, their vectors by inverse
//      iteration (LU with partial pivoting of T - lambda I, kEpInvIters solves from a fixed start,
//      the second made orthogonal to the first after every solve when the two are closer than
//      1e-3 ||T||, as LAPACK's dstein does), mapped back through the tridiagonal and QR reflectors.
// v[0], v[1] = null vectors (Q e_10, Q e_11), v[2], v[3] = eigenvectors of the smallest and the
// second smallest nonzero eigenvalue (m = 4: v[k] = Q e_{8+k}).  The null space is as accurate as M
// (not M^T M) allows; within it the basis is the QR's, which numpy's QR of the same M^T reproduces
// (tests/indep.py) -- any solver's basis there is arbitrary, and EPnP's N = 2 / 3 approximations
// depend on it.  Every step is a fixed sequence of IEEE operations (sums in tsum's tree order);
// pnp.hip spreads each over a wave (one lane per column / row / multisection point) without
// changing any value.
constexpr int kEpMsSteps = 10;  // multisection steps: 33^10 > 1.5e15, the interval at the rounding of ||T||
constexpr int kEpMsPts = 32;    // interior points per step and eigenvalue
constexpr int kEpInvIters = 3;  // inverse iteration solves
constexpr double kEpTiny = 0x1p-200;

// Householder reflector H = I - tau u u^T taking x (sum of squares s, leading entry x0) to alpha e_0;
// u = (x0 - alpha, x_1, ...), tau = 1 / (|x| (|x| + |x0|)) = 2 / u^T u (0 when x = 0).
VS_HD inline void ep_householder(double s, double x0, double& alpha, double& u0, double& tau) {
    const double nrm = sqrt(s);
    alpha = x0 >= 0 ? -nrm : nrm;
    u0 = x0 - alpha;
    tau = s > 0 ? 1.0 / (nrm * (nrm + fabs(x0))) : 0.0;
}

// entry r of column j of M^T (= row j of M)
VS_HD inline double ep_mt(const double (*al)[4], const double* uv, const Cam& K, int j, int r) {
    const int i = j >> 1;
    return (j & 1) ? epnp_m1(al[i], uv[2 * i + 1], K, r) : epnp_m0(al[i], uv[2 * i], K, r);
}

// Sturm count of the 10 x 10 tridiagonal (d, e2 = e^2, ||T|| < 2): the number of eigenvalues < x,
// from the sign changes of the leading principal minors p_i = (d_i - x) p_{i-1} - e2_{i-1} p_{i-2}.
// A zero minor becomes -2^-200 p_{i-1} (a tiny pivot of the other sign, as an LDL^T count treats
// it).  With ||T|| < 2 and x inside the Gershgorin interval |p_i| < 6^10, so no rescaling.
VS_HD inline int ep_sturm(const double* d, const double* e2, double x) {
    double pp = 1.0, pc = d[0] - x;
    if (pc == 0) pc = -kEpTiny;
    int cnt = pc < 0;
    VS_UNROLL
    for (int i = 1; i < 10; i++) {
        double pn = (d[i] - x) * pc - e2[i - 1] * pp;
        if (pn == 0) pn = -kEpTiny * pc;
        cnt += (pn < 0) != (pc < 0);
        pp = pc;
        pc = pn;
    }
    return cnt;
}

VS_HD inline double ep_frac(int j) { return (double)(j + 1) / (double)(kEpMsPts + 1); }

// LU with partial pivoting of the tridiagonal T - lam I (dgttrf's elimination, one division per
// step); pivots below tiny in magnitude are set to +-tiny, inv[i] = 1 / U_ii.
struct EpLu {
    double dd[10], du[9], du2[8], dl[9], inv[10];
    bool sw[9];
};
VS_HD inline void ep_lu(const double* d, const double* e, double lam, double tiny, EpLu& f) {
    VS_UNROLL
    for (int i = 0; i < 10; i++) f.dd[i] = d[i] - lam;
    VS_UNROLL
    for (int i = 0; i < 9; i++) f.du[i] = f.dl[i] = e[i];
    VS_UNROLL
    for (int i = 0; i < 8; i++) f.du2[i] = 0.0;
    VS_UNROLL
    for (int i = 0; i < 9; i++) {
        const double a = f.dd[i], l = f.dl[i], u = f.du[i], a1 = f.dd[i + 1];
        const bool sw = !(fabs(a) >= fabs(l));  // row interchange
        double fact = (sw ? a : l) / (sw ? l : a);
        if (!sw && a == 0) fact = 0.0;
        f.sw[i] = sw;
        f.dd[i] = sw ? l : a;
        f.dl[i] = fact;
        f.du[i] = sw ? a1 : u;
        f.dd[i + 1] = (sw ? u : a1) - fact * (sw ? a1 : u);
        if (i < 8) {
            const double u1 = f.du[i + 1];
            f.du2[i] = sw ? u1 : 0.0;
            f.du[i + 1] = sw ? -fact * u1 : u1;
        }
    }
    VS_UNROLL
    for (int i = 0; i < 10; i++) {
        const double a = f.dd[i];
        f.dd[i] = fabs(a) < tiny ? (a < 0 ? -tiny : tiny) : a;
        f.inv[i] = 1.0 / f.dd[i];
    }
}
VS_HD inline void ep_lu_solve(const EpLu& f, double* b) {
    VS_UNROLL
    for (int i = 0; i < 9; i++) {
        const double b0 = b[i], b1 = b[i + 1];
        b[i] = f.sw[i] ? b1 : b0;
        b[i + 1] = (f.sw[i] ? b0 : b1) - f.dl[i] * (f.sw[i] ? b1 : b0);
    }
    b[9] = b[9] * f.inv[9];
    b[8] = (b[8] - f.du[8] * b[9]) * f.inv[8];
    VS_UNROLL
    for (int i = 7; i >= 0; i--) b[i] = (b[i] - f.du[i] * b[i + 1] - f.du2[i] * b[i + 2]) * f.inv[i];
}
VS_HD inline double ep_dot10(const double* a, const double* b) {
    double t[10];
    VS_UNROLL
    for (int i = 0; i < 10; i++) t[i] = a[i] * b[i];
    return tsum<10>(t);
}
VS_HD inline void ep_normalize10(double* y) {
    const double inv = 1.0 / sqrt(ep_dot10(y, y));
    VS_UNROLL
    for (int i = 0; i < 10; i++) y[i] *= inv;
}
// fixed start vector of the inverse iteration (no structure a tridiagonal eigenvector shares)
VS_HD inline double ep_start(int i) {
    constexpr double s[10] = {0.53, -0.41, 0.37, 0.61, -0.29, 0.47, -0.33, 0.59, 0.43, -0.51};
    return s[i];
}
// y1 -= (y0 . y1 / y0 . y0) y0 (the solves' growth, at most ~2^52 each, is never normalised away
// in between: kEpInvIters solves stay far inside the double range)
VS_HD inline void ep_orth10(const double* y0, double* y1) {
    const double c = ep_dot10(y0, y1) / ep_dot10(y0, y0);
    VS_UNROLL
    for (int i = 0; i < 10; i++) y1[i] = y1[i] - c * y0[i];
}
// 2^-e with ||T|| * 2^-e in [1, 2) (exact; 1 for ||T|| = 0 or not finite)
VS_HD inline double ep_scale(double tnorm) {
    if (!(tnorm > 0) || !(tnorm <= DBL_MAX)) return 1.0;
    int e;
    frexp(tnorm, &e);  // tnorm = f 2^e, f in [0.5, 1)
    return ldexp(1.0, 1 - e);
}

// Sequential statement (host oracle; the device's parallel version in pnp.hip is bit-identical).
// dbg (test hook): when non-null, the stage results land in dbg[0..215]: alpha[10],
// tau[10], B[100] (before tridiagonalisation), d[10] and e[9] after it, the scale, lo, hi, the
// multisection brackets a[2] / b[2], lambda[2], y[2][10] after inverse iteration, v[48].
VS_HD inline void epnp_small_eig(const double (*al)[4], const double* uv, int m, const Cam& K, double v[4][12],
                                 double* dbg = nullptr) {
    const int nc = 2 * m;  // 8 or 10
    double C[10][12], alpha[10], tau[10], t[12];
    for (int j = 0; j < nc; j++)
        for (int r = 0; r < 12; r++) C[j][r] = ep_mt(al, uv, K, j, r);
    // 1. QR of M^T: column k keeps its reflector u (rows k..11), alpha[k] = R_kk
    for (int k = 0; k < nc; k++) {
        for (int r = 0; r < 12; r++) t[r] = r >= k ? C[k][r] * C[k][r] : -0.0;
        double u0;
        ep_householder(tsum<12>(t), C[k][k], alpha[k], u0, tau[k]);
        C[k][k] = u0;
        for (int j = k + 1; j < nc; j++) {
            for (int r = 0; r < 12; r++) t[r] = r >= k ? C[k][r] * C[j][r] : -0.0;
            const double f = tau[k] * tsum<12>(t);
            for (int r = k; r < 12; r++) C[j][r] = C[j][r] - f * C[k][r];
        }
    }
    double x[4][12];
    const int nz = nc == 10 ? 2 : 4;  // null vectors
    for (int q = 0; q < 4; q++)
        for (int r = 0; r < 12; r++) x[q][r] = (q < nz && r == nc + q) ? 1.0 : 0.0;
    if (nc == 10) {
        // 2. B = R R^T (R_ak = C[k][a] above the diagonal, alpha[a] on it), upper triangle then mirrored.
        // The diagonal factor is substituted by assignment, not by `k == a ? alpha[a] : C[k][a]`: in a
        // non-inlined gfx950 copy of this function that select between the two private arrays came out
        // as C[k][a] (tools/r06/epnp_b_repro.hip modes 10-17).
        double B[10][10];
        for (int a = 0; a < 10; a++)
            for (int b = a; b < 10; b++) {
                for (int k = 0; k < 10; k++) {
                    double fa = C[k][a], fb = C[k][b];
                    if (k == a) fa = alpha[a];
                    if (k == b) fb = alpha[b];
                    t[k] = k >= b ? fa * fb : -0.0;
                }
                B[a][b] = B[b][a] = tsum<10>(t);
            }
        if (dbg)
            for (int i = 0; i < 10; i++) {
                dbg[i] = alpha[i];
                dbg[10 + i] = tau[i];
                for (int j = 0; j < 10; j++) dbg[20 + 10 * i + j] = B[i][j];
            }
        // tridiagonalisation: reflector k (indices k+1..9) in U[k], tau in tt[k]
        double d[10], e[9], U[8][10], tt[8];
        for (int k = 0; k < 8; k++) {
            for (int j = 0; j < 10; j++) t[j] = j > k ? B[k][j] * B[k][j] : -0.0;
            double u0, tk;
            ep_householder(tsum<10>(t), B[k][k + 1], e[k], u0, tk);
            d[k] = B[k][k];
            tt[k] = tk;
            for (int j = 0; j < 10; j++) U[k][j] = j > k + 1 ? B[k][j] : j == k + 1 ? u0 : 0.0;
            double p[10], w[10];
            for (int i = k + 1; i < 10; i++) {
                for (int j = 0; j < 10; j++) t[j] = j > k ? B[i][j] * U[k][j] : -0.0;
                p[i] = tk * tsum<10>(t);
            }
            for (int i = 0; i < 10; i++) t[i] = i > k ? p[i] * U[k][i] : -0.0;
            const double Kc = (0.5 * tk) * tsum<10>(t);
            for (int i = k + 1; i < 10; i++) w[i] = p[i] - Kc * U[k][i];
            for (int i = k + 1; i < 10; i++)
                for (int j = k + 1; j < 10; j++) B[i][j] = B[i][j] - (U[k][i] * w[j] + w[i] * U[k][j]);
        }
        d[8] = B[8][8];
        d[9] = B[9][9];
        e[8] = B[8][9];
        if (dbg) {
            for (int i = 0; i < 10; i++) dbg[120 + i] = d[i];
            for (int i = 0; i < 9; i++) dbg[130 + i] = e[i];
        }
        // 3. scaled to ||T|| in [1, 2) (Gershgorin bound); the two smallest eigenvalues by multisection
        double lo = 0, hi = 0;
        for (int i = 0; i < 10; i++) {
            const double rad = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < 9 ? fabs(e[i]) : 0.0);
            const double l = d[i] - rad, h = d[i] + rad;
            lo = (i == 0 || l < lo) ? l : lo;
            hi = (i == 0 || h > hi) ? h : hi;
        }
        const double sc = ep_scale(fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi));
        double e2[9];
        for (int i = 0; i < 10; i++) d[i] *= sc;
        for (int i = 0; i < 9; i++) {
            e[i] *= sc;
            e2[i] = e[i] * e[i];
        }
        lo *= sc;
        hi *= sc;
        double a_t[2] = {lo, lo}, b_t[2] = {hi, hi};
        for (int st = 0; st < kEpMsSteps; st++)
            for (int q = 0; q < 2; q++) {
                const double a = a_t[q], wd = b_t[q] - a_t[q];
                int js = kEpMsPts;
                for (int j = 0; j < kEpMsPts; j++)
                    if (ep_sturm(d, e2, a + wd * ep_frac(j)) > q) {
                        js = j;
                        break;
                    }
                a_t[q] = js > 0 ? a + wd * ep_frac(js - 1) : a;
                b_t[q] = js < kEpMsPts ? a + wd * ep_frac(js) : b_t[q];
            }
        if (dbg) {
            dbg[139] = sc;
            dbg[140] = lo;
            dbg[141] = hi;
            for (int q = 0; q < 2; q++) dbg[142 + q] = a_t[q], dbg[144 + q] = b_t[q];
        }
        // 4. inverse iteration
        const double tnorm = fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi);
        const double tiny = tnorm > 0 ? DBL_EPSILON * tnorm : DBL_MIN;
        double lam[2], y[2][10];
        EpLu f[2];
        for (int q = 0; q < 2; q++) {
            lam[q] = 0.5 * (a_t[q] + b_t[q]);
            ep_lu(d, e, lam[q], tiny, f[q]);
            for (int i = 0; i < 10; i++) y[q][i] = ep_start(i);
        }
        const bool cluster = lam[1] - lam[0] <= 1e-3 * tnorm;
        for (int it = 0; it < kEpInvIters; it++) {
            for (int q = 0; q < 2; q++) ep_lu_solve(f[q], y[q]);
            if (cluster) ep_orth10(y[0], y[1]);
        }
        if (dbg)
            for (int q = 0; q < 2; q++) {
                dbg[146 + q] = lam[q];
                for (int i = 0; i < 10; i++) dbg[148 + 10 * q + i] = y[q][i];
            }
        // 5. normalised, back through the tridiagonal reflectors (H_7 first), into the QR basis
        for (int q = 0; q < 2; q++) {
            ep_normalize10(y[q]);
            for (int k = 7; k >= 0; k--) {
                for (int i = 0; i < 10; i++) t[i] = i > k ? U[k][i] * y[q][i] : -0.0;
                const double fk = tt[k] * tsum<10>(t);
                for (int i = k + 1; i < 10; i++) y[q][i] = y[q][i] - fk * U[k][i];
            }
            for (int r = 0; r < 10; r++) x[2 + q][r] = y[q][r];
        }
    }
    // 6. v = Q x (Q = H_0 .. H_{nc-1}: H_{nc-1} first)
    for (int q = 0; q < 4; q++) {
        for (int k = nc - 1; k >= 0; k--) {
            for (int r = 0; r < 12; r++) t[r] = r >= k ? C[k][r] * x[q][r] : -0.0;
            const double fk = tau[k] * tsum<12>(t);
            for (int r = k; r < 12; r++) x[q][r] = x[q][r] - fk * C[k][r];
        }
        for (int r = 0; r < 12; r++) v[q][r] = x[q][r];
    }
    if (dbg)
        for (int q = 0; q < 4; q++)
            for (int r = 0; r < 12; r++) dbg[168 + 12 * q + r] = v[q][r];
}

// From the eigenvectors um (columns, descending eigenvalues): v[k] = eigenvector of the k-th
// smallest eigenvalue, the L_6x10 matrix and the squared control point distances rho.
VS_HD inline void epnp_L_rho_v(const double v[4][12], const double cw[4][3], double L[6][10], double rho[6]);
VS_HD inline void epnp_L_rho(const double* um, const double cw[4][3], double v[4][12], double L[6][10], double rho[6]) {
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 12; i++) v[k][i] = um[i * 12 + (11 - k)];
    epnp_L_rho_v(v, cw, L, rho);
}
// L and rho from the four eigenvectors v[k] (k-th smallest eigenvalue)
// Entry (j, c) of L_6x10 (pair j of control points, product c of the betas) and rho[j]: one
// expression per entry, so the device computes each on its own lane with the same arithmetic.
VS_HD inline double epnp_L_entry(const double v[4][12], int j, int c) {
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    constexpr int ka[10] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3}, kb[10] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3};
    const int a = ka[c], b = kb[c], p = 3 * pa[j], q = 3 * pb[j];
    const double d0 = (v[a][p] - v[a][q]) * (v[b][p] - v[b][q]);
    const double d1 = (v[a][p + 1] - v[a][q + 1]) * (v[b][p + 1] - v[b][q + 1]);
    const double d2 = (v[a][p + 2] - v[a][q + 2]) * (v[b][p + 2] - v[b][q + 2]);
    const double dt = d0 + d1 + d2;
    return a == b ? dt : 2.0 * dt;
}
VS_HD inline double epnp_rho_entry(const double cw[4][3], int j) {
    constexpr int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
    const double dx = cw[pa[j]][0] - cw[pb[j]][0], dy = cw[pa[j]][1] - cw[pb[j]][1], dz = cw[pa[j]][2] - cw[pb[j]][2];
    return dx * dx + dy * dy + dz * dz;
}
VS_HD inline void epnp_L_rho_v(const double v[4][12], const double cw[4][3], double L[6][10], double rho[6]) {
    for (int j = 0; j < 6; j++) {
        for (int c = 0; c < 10; c++) L[j][c] = epnp_L_entry(v, j, c);
        rho[j] = epnp_rho_entry(cw, j);
    }
}

// Beta approximation s (0: N = 4, 1: N = 2, 2: N = 3), 5 Gauss-Newton steps on the 6 distance
// constraints, pose by Kabsch on the camera-frame points; returns the mean reprojection error.
// MAXN bounds n at compile time: the point loops run to MAXN with an i < n guard (the same
// operations in the same order), so on the device (MAXN = 5) they unroll and the arrays stay in
// registers instead of scratch.
// The initial betas of approximation s (least squares on the selected L columns).
VS_HD inline void epnp_betas_init(int s, const double L[6][10], const double rho[6], double be[4]) {
    if (s == 0) {  // N = 4: B11 B12 B13 B14
        double A[24], b[6], x[4];
        for (int j = 0; j < 6; j++) {
            A[j * 4 + 0] = L[j][0];
            A[j * 4 + 1] = L[j][1];
            A[j * 4 + 2] = L[j][3];
            A[j * 4 + 3] = L[j][6];
            b[j] = rho[j];
        }
        lstsq<6, 4>(A, b, x);
        if (x[0] < 0) {
            const double b0 = sqrt(-x[0]);
            be[0] = b0;
            be[1] = b0 ? -x[1] / b0 : 0.0;
            be[2] = b0 ? -x[2] / b0 : 0.0;
            be[3] = b0 ? -x[3] / b0 : 0.0;
        } else {
            const double b0 = sqrt(x[0]);
            be[0] = b0;
            be[1] = b0 ? x[1] / b0 : 0.0;
            be[2] = b0 ? x[2] / b0 : 0.0;
            be[3] = b0 ? x[3] / b0 : 0.0;
        }
    } else if (s == 1) {  // N = 2: B11 B12 B22
        double A[18], b[6], x[3];
        for (int j = 0; j < 6; j++) {
            A[j * 3 + 0] = L[j][0];
            A[j * 3 + 1] = L[j][1];
            A[j * 3 + 2] = L[j][2];
            b[j] = rho[j];
        }
        lstsq<6, 3>(A, b, x);
        double b0, b1;
        if (x[0] < 0) {
            b0 = sqrt(-x[0]);
            b1 = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
        } else {
            b0 = sqrt(x[0]);
            b1 = (x[2] > 0) ? sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b0 = -b0;
        be[0] = b0;
        be[1] = b1;
        be[2] = 0.0;
        be[3] = 0.0;
    } else {  // N = 3: B11 B12 B22 B13 B23
        double A[30], b[6], x[5];
        for (int j = 0; j < 6; j++) {
            for (int c = 0; c < 5; c++) A[j * 5 + c] = L[j][c];
            b[j] = rho[j];
        }
        lstsq<6, 5>(A, b, x);
        double b0, b1;
        if (x[0] < 0) {
            b0 = sqrt(-x[0]);
            b1 = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
        } else {
            b0 = sqrt(x[0]);
            b1 = (x[2] > 0) ? sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b0 = -b0;
        be[0] = b0;
        be[1] = b1;
        be[2] = b0 ? x[3] / b0 : 0.0;
        be[3] = 0.0;
    }
}

// The same initial betas with one lstsq<6, 5> for every s (the selected columns first, zero columns
// after them): Householder QR skips a zero column (nrm == 0), leaves it zero (d = 0 in every
// update), and back substitution gives it x = 0 and subtracts exact zeros for it, so the result is
// bit-identical to epnp_betas_init's lstsq<6, N>; on the device the three approximations then run
// the same code on three lanes instead of three divergent solves.
VS_HD inline void epnp_betas_init_uniform(int s, const double L[6][10], const double rho[6], double be[4]) {
    double A[30], b[6], x[5];
    const int c3 = s == 0 ? 3 : 2, c4 = s == 0 ? 6 : 3;  // s = 0: L0 L1 L3 L6; s = 1: L0 L1 L2; s = 2: L0..L4
    const int ncol = s == 0 ? 4 : s == 1 ? 3 : 5;
    for (int j = 0; j < 6; j++) {
        A[j * 5 + 0] = L[j][0];
        A[j * 5 + 1] = L[j][1];
        A[j * 5 + 2] = L[j][c3 == 3 ? 3 : 2];
        A[j * 5 + 3] = ncol > 3 ? L[j][c4] : 0.0;
        A[j * 5 + 4] = ncol > 4 ? L[j][4] : 0.0;
        b[j] = rho[j];
    }
    lstsq<6, 5>(A, b, x);
    if (s == 0) {
        const double sg = x[0] < 0 ? -1.0 : 1.0;
        const double b0 = sqrt(sg * x[0]);
        be[0] = b0;
        be[1] = b0 ? (sg * x[1]) / b0 : 0.0;
        be[2] = b0 ? (sg * x[2]) / b0 : 0.0;
        be[3] = b0 ? (sg * x[3]) / b0 : 0.0;
    } else {
        double b0, b1;
        if (x[0] < 0) {
            b0 = sqrt(-x[0]);
            b1 = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
        } else {
            b0 = sqrt(x[0]);
            b1 = (x[2] > 0) ? sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b0 = -b0;
        be[0] = b0;
        be[1] = b1;
        be[2] = (s == 2 && b0) ? x[3] / b0 : 0.0;
        be[3] = 0.0;
    }
}

// Gauss-Newton on the betas, then the pose by Kabsch; returns the mean reprojection error.
// mark(k) at the stage ends (0: Gauss-Newton, 1: control points + cross-covariance, 2: Kabsch,
// 3: reprojection error): the device's profiling build counts cycles there, everything else
// passes NoMark
template <int MAXN, class Mark = NoMark>
VS_HD inline double epnp_refine(double be[4], const double L[6][10], const double rho[6], const double v[4][12],
                                const double (*alphas)[4], const double* X, const double* uv, int n, const Cam& K,
                                double* R, double* t, Mark mark = Mark()) {
    double Lr[6][10], rr[6];  // register copies (the device passes LDS arrays)
    VS_UNROLL
    for (int j = 0; j < 6; j++) {
        rr[j] = rho[j];
        VS_UNROLL
        for (int c = 0; c < 10; c++) Lr[j][c] = L[j][c];
    }
    VS_NOUNROLL  // one copy of the body: the device's instruction cache, not its ALUs, bounds this code
    for (int it = 0; it < 5; it++) {  // Gauss-Newton on the 6 distance constraints
        double A[24], b[6], x[4];
        // the beta products once; every sum in tsum's tree order
        const double q[10] = {be[0] * be[0], be[0] * be[1], be[1] * be[1], be[0] * be[2], be[1] * be[2],
                              be[2] * be[2], be[0] * be[3], be[1] * be[3], be[2] * be[3], be[3] * be[3]};
        VS_UNROLL
        for (int j = 0; j < 6; j++) {
            const double* l = Lr[j];
            const double a0[4] = {(2 * l[0]) * be[0], l[1] * be[1], l[3] * be[2], l[6] * be[3]};
            const double a1[4] = {l[1] * be[0], (2 * l[2]) * be[1], l[4] * be[2], l[7] * be[3]};
            const double a2[4] = {l[3] * be[0], l[4] * be[1], (2 * l[5]) * be[2], l[8] * be[3]};
            const double a3[4] = {l[6] * be[0], l[7] * be[1], l[8] * be[2], (2 * l[9]) * be[3]};
            A[j * 4 + 0] = tsum<4>(a0);
            A[j * 4 + 1] = tsum<4>(a1);
            A[j * 4 + 2] = tsum<4>(a2);
            A[j * 4 + 3] = tsum<4>(a3);
            double lq[10];
            VS_UNROLL
            for (int k = 0; k < 10; k++) lq[k] = l[k] * q[k];
            b[j] = rr[j] - tsum<10>(lq);
        }
        lstsq<6, 4>(A, b, x);
        for (int k = 0; k < 4; k++) be[k] += x[k];
    }
    mark(0);
    // camera coordinates of control and object points
    double ccs[4][3];
    for (int i = 0; i < 4; i++)
        for (int c = 0; c < 3; c++)
            ccs[i][c] = be[0] * v[0][3 * i + c] + be[1] * v[1][3 * i + c] + be[2] * v[2][3 * i + c] +
                        be[3] * v[3][3 * i + c];
    double pcs0z = alphas[0][0] * ccs[0][2] + alphas[0][1] * ccs[1][2] + alphas[0][2] * ccs[2][2] +
                   alphas[0][3] * ccs[3][2];
    const double sgn = pcs0z < 0 ? -1.0 : 1.0;
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    VS_UNROLL
    for (int i = 0; i < MAXN; i++)
        if (i < n)
            for (int c = 0; c < 3; c++) {
            pc0[c] += sgn * (alphas[i][0] * ccs[0][c] + alphas[i][1] * ccs[1][c] + alphas[i][2] * ccs[2][c] +
                             alphas[i][3] * ccs[3][c]);
            pw0[c] += X[3 * i + c];
        }
    for (int c = 0; c < 3; c++) {
        pc0[c] /= n;
        pw0[c] /= n;
    }
    double ABt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    VS_UNROLL
    for (int i = 0; i < MAXN; i++) {
        if (i >= n) continue;
        double pc[3];
        for (int c = 0; c < 3; c++)
            pc[c] = sgn * (alphas[i][0] * ccs[0][c] + alphas[i][1] * ccs[1][c] + alphas[i][2] * ccs[2][c] +
                           alphas[i][3] * ccs[3][c]) - pc0[c];
        const double pw[3] = {X[3 * i] - pw0[0], X[3 * i + 1] - pw0[1], X[3 * i + 2] - pw0[2]};
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) ABt[a * 3 + b] += pc[a] * pw[b];
    }
    mark(1);
    rotation_from_cross(ABt, R);
    for (int c = 0; c < 3; c++) t[c] = pc0[c] - (R[c * 3] * pw0[0] + R[c * 3 + 1] * pw0[1] + R[c * 3 + 2] * pw0[2]);
    mark(2);
    double err = 0;
    VS_UNROLL
    for (int i = 0; i < MAXN; i++) {
        if (i >= n) continue;
        double u, vv;
        project(R, t, K, X[3 * i], X[3 * i + 1], X[3 * i + 2], u, vv);
        const double du = uv[2 * i] - u, dvv = uv[2 * i + 1] - vv;
        err += sqrt(du * du + dvv * dvv);
    }
    mark(3);
    return err / n;
}

template <int MAXN>
VS_HD inline double epnp_variant(int s, const double L[6][10], const double rho[6], const double v[4][12],
                                 const double (*alphas)[4], const double* X, const double* uv, int n, const Cam& K,
                                 double* R, double* t) {
    double be[4];
    epnp_betas_init(s, L, rho, be);
    return epnp_refine<MAXN>(be, L, rho, v, alphas, X, uv, n, K, R, t);
}

// n >= 4 correspondences (object points X[3i..], image points u[2i..]).  Returns R (world ->
// camera) and t; false if degenerate.  The lowest-error approximation wins (first on ties).
template <int MAXN>
VS_HD bool epnp(const double* X, const double* uv, int n, const Cam& K, double* Rout, double* tout) {
    if (n < 4 || n > MAXN) return false;
    double cw[4][3], alphas[MAXN][4];
    if (!epnp_control<MAXN>(X, n, cw, alphas)) return false;
    double v[4][12], L[6][10], rho[6];
    if (n <= 5) {  // RANSAC subsets: the null space by QR, two eigenpairs of R R^T
        epnp_small_eig(alphas, uv, n, K, v);
        epnp_L_rho_v(v, cw, L, rho);
    } else {
        double MtM[144];
        for (int a = 0; a < 12; a++)
            for (int b = 0; b < 12; b++) MtM[a * 12 + b] = epnp_mtm<MAXN>(alphas, uv, n, K, a, b);
        double dm[12], um[144];
        sym_eig_rr<12>(MtM, dm, um);
        epnp_L_rho(um, cw, v, L, rho);
    }
    double best_err = 0;
    bool have = false;
    for (int s = 0; s < 3; s++) {
        double R[9], t[3];
        const double err = epnp_variant<MAXN>(s, L, rho, v, alphas, X, uv, n, K, R, t);
        if (!have || err < best_err) {
            have = true;
            best_err = err;
            for (int k = 0; k < 9; k++) Rout[k] = R[k];
            for (int k = 0; k < 3; k++) tout[k] = t[k];
        }
    }
    return have;
}

// ------------------------------------------------------------ Levenberg-Marquardt refinement
// Parameters p = (rvec, tvec), world -> camera.  Residuals r_i = project(X_i) - uv_i (double).
// Rotation columns of J by central differences (step kLmStep) from seven shared rotations,
// translation columns analytic.
constexpr double kLmStep = 1e-6;
constexpr int kLmMaxIters = 20;
constexpr int kLmTerms = 28;  // 21 upper-triangular J^T J, 6 J^T r, 1 cost

struct LmRots {
    double R[7][9];  // R(r), R(r + h e0), R(r - h e0), R(r + h e1), ...
};

VS_HD inline void lm_rotations(const double* p, LmRots& L) {
    rod_v2m(p, L.R[0]);
    for (int k = 0; k < 3; k++) {
        double rp[3] = {p[0], p[1], p[2]}, rm[3] = {p[0], p[1], p[2]};
        rp[k] += kLmStep;
        rm[k] -= kLmStep;
        rod_v2m(rp, L.R[1 + 2 * k]);
        rod_v2m(rm, L.R[2 + 2 * k]);
    }
}

// Adds one correspondence's terms to acc[kLmTerms].
VS_HD inline void lm_point(const LmRots& L, const double* t, const Cam& K, double X, double Y, double Z, double u,
                           double v, double* acc) {
    const double* R = L.R[0];
    const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    const double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    const double iz = z ? 1.0 / z : 1.0;
    const double pu = K.fx * (x * iz) + K.cx, pv = K.fy * (y * iz) + K.cy;
    const double ru = pu - u, rv = pv - v;
    double ju[6], jv[6];
    for (int k = 0; k < 3; k++) {
        double up, vp, um, vm;
        project(L.R[1 + 2 * k], t, K, X, Y, Z, up, vp);
        project(L.R[2 + 2 * k], t, K, X, Y, Z, um, vm);
        ju[k] = (up - um) / (2.0 * kLmStep);
        jv[k] = (vp - vm) / (2.0 * kLmStep);
    }
    ju[3] = K.fx * iz;
    ju[4] = 0.0;
    ju[5] = -K.fx * x * iz * iz;
    jv[3] = 0.0;
    jv[4] = K.fy * iz;
    jv[5] = -K.fy * y * iz * iz;
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) acc[k++] += ju[a] * ju[c] + jv[a] * jv[c];
    for (int a = 0; a < 6; a++) acc[21 + a] += ju[a] * ru + jv[a] * rv;
    acc[27] += ru * ru + rv * rv;
}

// Solves (J^T J with its diagonal scaled by 1 + lambda) d = -J^T r by Cholesky; false if not SPD.
// Each pivot's reciprocal is taken once: the factor's column and both substitutions multiply by it,
// so the substitutions' chains are products, not divisions (the device's latency).
VS_HD inline bool lm_solve(const double* acc, double lambda, double* d) {
    double A[36];
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int c = a; c < 6; c++) {
            A[a * 6 + c] = acc[k];
            A[c * 6 + a] = acc[k];
            k++;
        }
    for (int a = 0; a < 6; a++) {
        A[a * 6 + a] *= 1.0 + lambda;
        d[a] = -acc[21 + a];
    }
    double inv[6];
    for (int j = 0; j < 6; j++) {
        double s = A[j * 6 + j];
        for (int q = 0; q < j; q++) s -= A[j * 6 + q] * A[j * 6 + q];
        if (!(s > 0)) return false;
        const double r = sqrt(s);
        A[j * 6 + j] = r;
        inv[j] = 1.0 / r;
        for (int i = j + 1; i < 6; i++) {
            double w = A[i * 6 + j];
            for (int q = 0; q < j; q++) w -= A[i * 6 + q] * A[j * 6 + q];
            A[i * 6 + j] = w * inv[j];
        }
    }
    for (int i = 0; i < 6; i++) {
        double w = d[i];
        for (int q = 0; q < i; q++) w -= A[i * 6 + q] * d[q];
        d[i] = w * inv[i];
    }
    for (int i = 5; i >= 0; i--) {
        double w = d[i];
        for (int q = i + 1; q < 6; q++) w -= A[q * 6 + i] * d[q];
        d[i] = w * inv[i];
    }
    return true;
}

// LM control shared by the sequential (oracle) and workgroup (device) drivers.  The caller
// evaluates acc at `cand` whenever step() returns 1 and then calls accept_or_reject().
struct LmState {
    double p[6], cand[6];
    double acc[kLmTerms];  // terms at p
    double lambda;
    int iters, accepted, done;

    VS_HD void init(const double* p0, const double* acc0) {
        for (int i = 0; i < 6; i++) p[i] = cand[i] = p0[i];
        for (int i = 0; i < kLmTerms; i++) acc[i] = acc0[i];
        lambda = 1e-3;
        iters = accepted = done = 0;
    }
    // 1: evaluate cand; 0: finished
    VS_HD int step() {
        while (!done && iters < kLmMaxIters) {
            iters++;
            double d[6];
            if (!lm_solve(acc, lambda, d)) {
                lambda *= 10;
                continue;
            }
            double dn = 0, pn = 0;
            for (int i = 0; i < 6; i++) {
                dn += d[i] * d[i];
                pn += p[i] * p[i];
            }
            if (sqrt(dn) <= DBL_EPSILON * sqrt(pn)) {
                done = 1;
                break;
            }
            for (int i = 0; i < 6; i++) cand[i] = p[i] + d[i];
            return 1;
        }
        done = 1;
        return 0;
    }
    VS_HD void accept_or_reject(const double* acc_cand) {
        if (acc_cand[27] < acc[27]) {
            double dn = 0, pn = 0;
            for (int i = 0; i < 6; i++) {
                dn += (cand[i] - p[i]) * (cand[i] - p[i]);
                pn += cand[i] * cand[i];
            }
            for (int i = 0; i < 6; i++) p[i] = cand[i];
            for (int i = 0; i < kLmTerms; i++) acc[i] = acc_cand[i];
            lambda = lambda / 10 > 1e-15 ? lambda / 10 : 1e-15;
            accepted++;
            if (sqrt(dn) <= FLT_EPSILON * sqrt(pn)) done = 1;
        } else {
            lambda *= 10;
            if (lambda > 1e16) done = 1;
        }
    }
};

VS_HD inline void dlt_point(const double P1[12], const double P2[12], float x1, float y1, float x2, float y2,
                            float X[4]) {
    double A[16];
    const double* Ps[2] = {P1, P2};
    const double xs[2] = {x1, x2}, ys[2] = {y1, y2};
    for (int j = 0; j < 2; j++)
        for (int k = 0; k < 4; k++) {
            A[(2 * j) * 4 + k] = xs[j] * Ps[j][8 + k] - Ps[j][k];
            A[(2 * j + 1) * 4 + k] = ys[j] * Ps[j][8 + k] - Ps[j][4 + k];
        }
    double AtA[16], w[4], V[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += A[k * 4 + i] * A[k * 4 + j];
            AtA[i * 4 + j] = s;
        }
    sym_eig<4>(AtA, w, V);
    for (int i = 0; i < 4; i++) X[i] = (float)V[i * 4 + 3];
}

}  // namespace vs_pnp
