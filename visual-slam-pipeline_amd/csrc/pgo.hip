// pgo.hip — F4 pose graph optimisation, Optimizer::pose_graph_optimize (reference
// src/Optimizer.cpp:654-863): g2o SE3 vertices (one per keyframe, the first fixed), EdgeSE3
// odometry edges between consecutive keyframes (measurement from the old poses, information
// diag(1/0.05^2 x3, 1/0.02^2 x3)), EdgeSE3 loop edges (diag(1/sigma_t^2, 1/sigma_r^2)), optional
// EdgeHeightPrior unary edges (g . t - h, 1/0.005^2), solved by g2o's Levenberg-Marquardt
// (OptimizationAlgorithmLevenberg: lambda0 = 1e-5 max diag H, rho = dchi / (x.(lambda x + b) + 1e-3),
// lambda *= max(1/3, min(2/3, 1 - (2 rho - 1)^3)) on success, lambda *= ni, ni *= 2 on failure, at most
// 10 trials per iteration) for `iterations` iterations.  g2o conventions restated: vertex update
// T <- T * exp(dx) with dx = (translation, quaternion xyz; w = sqrt(1 - |q|^2)), error =
// (translation, normalised quaternion xyz with w >= 0) of Z^-1 Ta^-1 Tb, Jacobians by central
// differences (step 1e-6) of that error in dx.  g2o itself is not in this image: "parity unpinned"
// against it; the oracle (oracle/orc_pgo.cpp, dense Cholesky) is an independent restatement.
//
// Device design: the whole LM runs in ONE workgroup (a persistent 256-thread kernel).  The normal
// matrix of a keyframe chain is block tridiagonal plus one "spike" per loop edge; it is factorised
// as a block skyline (envelope) Cholesky H = U^T U whose column j holds blocks rows f_j .. j, so a
// loop from keyframe a to b fills only rows a .. b of column b and nothing else.  Per column: the
// 6 x 6 block products on 36 lanes, triangular solves on 6 lanes, the diagonal Cholesky on one.
// Edge linearisation runs one edge per lane; every sum has a fixed order (per-block contribution
// lists built on the host), so a run is deterministic.  fp64 throughout; latency-bound by design
// (n sequential 6 x 6 steps per factorisation), so the figure of merit is ms per call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "vs_internal.h"

namespace vs {

constexpr int kPgoThreads = 256;
constexpr double kPgoStep = 1e-6;  // central-difference step of the numeric Jacobians

struct PgoArgs {
    int N, n, E, L, iters, has_h;  // vertices, unknown blocks (N - 1), binary edges, loop edges
    double tau, height, hinfo;
    double g[3];
    double* P;       // [N][12] current poses (R row-major, t)
    double* Pt;      // [N][12] trial poses
    const int* ea;   // [E] edge vertices (a, b)
    const int* eb;
    double* Zinv;    // [E][12] inverse measurements (odometry ones filled by the kernel)
    const double* om;  // [E][6] information diagonal
    double* EB;      // [E][120] Haa | Hab | Hbb | ba | bb
    double* HB;      // [N][8] height-prior blocks per vertex: d e / d t (3, in the update frame) ...
    const int* colf;   // [n] envelope start of block column j
    const int* colp;   // [n + 1] first skyline block of column j (row colf[j])
    const int* clist_p;  // [nblk + 1] contribution list per skyline block
    const int* clist;    // entries: 4 * edge + kind (0 aa, 1 bb, 2 ab, 3 ab^T)
    const int* vinc_p;   // [N + 1] incident edges per vertex
    const int* vinc;     // entries: 2 * edge + side (0 a, 1 b)
    double* H;       // [nblk][36] assembled upper blocks
    double* U;       // [nblk][36] factor
    double* b;       // [n][6]
    double* x;       // [n][6]
    double* y;       // [n][6]
    int* stats;      // {iterations, accepted steps, trials, ok}
    double* chi_out; // {chi2 before, chi2 after, final lambda}
};

// ---- SE3 helpers (row-major R, t) -------------------------------------------------------------
__device__ inline void iso_mul(const double* A, const double* B, double* C) {  // C = A B
    double R[9], t[3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
        t[i] = A[i * 3] * B[9] + A[i * 3 + 1] * B[10] + A[i * 3 + 2] * B[11] + A[9 + i];
    }
    for (int k = 0; k < 9; k++) C[k] = R[k];
    for (int k = 0; k < 3; k++) C[9 + k] = t[k];
}
__device__ inline void iso_inv(const double* A, double* C) {
    double R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = A[j * 3 + i];
    const double t0 = -(R[0] * A[9] + R[1] * A[10] + R[2] * A[11]);
    const double t1 = -(R[3] * A[9] + R[4] * A[10] + R[5] * A[11]);
    const double t2 = -(R[6] * A[9] + R[7] * A[10] + R[8] * A[11]);
    for (int k = 0; k < 9; k++) C[k] = R[k];
    C[9] = t0;
    C[10] = t1;
    C[11] = t2;
}
// Eigen's Quaterniond(Matrix3d) (trace / largest-diagonal branches), normalised, w >= 0: xyz
__device__ inline void rot_to_qvec(const double* R, double q[3]) {
    double w, x, y, z;
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        double s = sqrt(tr + 1.0);
        w = 0.5 * s;
        s = 0.5 / s;
        x = (R[7] - R[5]) * s;
        y = (R[2] - R[6]) * s;
        z = (R[3] - R[1]) * s;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[i * 4]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
        double c[3];
        c[i] = 0.5 * s;
        s = 0.5 / s;
        w = (R[k * 3 + j] - R[j * 3 + k]) * s;
        c[j] = (R[j * 3 + i] + R[i * 3 + j]) * s;
        c[k] = (R[k * 3 + i] + R[i * 3 + k]) * s;
        x = c[0];
        y = c[1];
        z = c[2];
    }
    const double nrm = sqrt(w * w + x * x + y * y + z * z);
    const double sg = w < 0 ? -1.0 : 1.0;
    q[0] = sg * x / nrm;
    q[1] = sg * y / nrm;
    q[2] = sg * z / nrm;
}
// g2o fromVectorMQT: translation v[0..2], quaternion (w = sqrt(1 - |v[3..5]|^2), v[3..5])
__device__ inline void mqt_to_iso(const double* v, double* T) {
    const double qx = v[3], qy = v[4], qz = v[5];
    double w = 1.0 - (qx * qx + qy * qy + qz * qz);
    double x = qx, y = qy, z = qz;
    if (w < 0) {
        w = 1.0;
        x = y = z = 0.0;
    } else {
        w = sqrt(w);
    }
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    T[0] = 1 - (tyy + tzz);
    T[1] = txy - twz;
    T[2] = txz + twy;
    T[3] = txy + twz;
    T[4] = 1 - (txx + tzz);
    T[5] = tyz - twx;
    T[6] = txz - twy;
    T[7] = tyz + twx;
    T[8] = 1 - (txx + tyy);
    T[9] = v[0];
    T[10] = v[1];
    T[11] = v[2];
}
// EdgeSE3::computeError: MQT(Zinv * Ta^-1 * Tb)
__device__ inline void se3_error(const double* Zinv, const double* Ta, const double* Tb, double e[6]) {
    double ia[12], d[12], d2[12];
    iso_inv(Ta, ia);
    iso_mul(Zinv, ia, d);
    iso_mul(d, Tb, d2);
    e[0] = d2[9];
    e[1] = d2[10];
    e[2] = d2[11];
    rot_to_qvec(d2, e + 3);
}
__device__ inline void oplus(const double* T, const double* dx, double* out) {
    double inc[12];
    mqt_to_iso(dx, inc);
    iso_mul(T, inc, out);
}

// chi2 of the active edges at poses Q (deterministic: strided per-lane sums, then a fixed tree)
__device__ double pgo_chi2(const PgoArgs& a, const double* Q, double* red) {
    double acc = 0;
    for (int k = threadIdx.x; k < a.E; k += kPgoThreads) {
        double e[6];
        se3_error(a.Zinv + 12 * k, Q + 12 * a.ea[k], Q + 12 * a.eb[k], e);
        for (int r = 0; r < 6; r++) acc += e[r] * a.om[6 * k + r] * e[r];
    }
    if (a.has_h)
        for (int v = 1 + threadIdx.x; v < a.N; v += kPgoThreads) {  // unary edges on the fixed vertex are inactive
            const double* T = Q + 12 * v;
            const double e = a.g[0] * T[9] + a.g[1] * T[10] + a.g[2] * T[11] - a.height;
            acc += e * a.hinfo * e;
        }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = kPgoThreads / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

// one edge's blocks: J (6 x 12, numeric), then Haa, Hab, Hbb (J^T Omega J) and ba, bb (-J^T Omega e)
__device__ void pgo_linearize_edge(const PgoArgs& a, int k) {
    const double* Ta = a.P + 12 * a.ea[k];
    const double* Tb = a.P + 12 * a.eb[k];
    const double* Zi = a.Zinv + 12 * k;
    const double* w = a.om + 6 * k;
    double e0[6], J[6][12];
    se3_error(Zi, Ta, Tb, e0);
    for (int c = 0; c < 12; c++) {
        double dx[6] = {0, 0, 0, 0, 0, 0}, Tp[12], Tm[12], ep[6], em[6];
        const double* T = c < 6 ? Ta : Tb;
        dx[c % 6] = kPgoStep;
        oplus(T, dx, Tp);
        dx[c % 6] = -kPgoStep;
        oplus(T, dx, Tm);
        if (c < 6) {
            se3_error(Zi, Tp, Tb, ep);
            se3_error(Zi, Tm, Tb, em);
        } else {
            se3_error(Zi, Ta, Tp, ep);
            se3_error(Zi, Ta, Tm, em);
        }
        for (int r = 0; r < 6; r++) J[r][c] = (ep[r] - em[r]) / (2.0 * kPgoStep);
    }
    double* out = a.EB + 120 * k;
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            double aa = 0, ab = 0, bb = 0;
            for (int r = 0; r < 6; r++) {
                aa += J[r][i] * w[r] * J[r][j];
                ab += J[r][i] * w[r] * J[r][6 + j];
                bb += J[r][6 + i] * w[r] * J[r][6 + j];
            }
            out[i * 6 + j] = aa;
            out[36 + i * 6 + j] = ab;
            out[72 + i * 6 + j] = bb;
        }
    for (int i = 0; i < 6; i++) {
        double sa = 0, sb = 0;
        for (int r = 0; r < 6; r++) {
            sa += J[r][i] * w[r] * e0[r];
            sb += J[r][6 + i] * w[r] * e0[r];
        }
        out[108 + i] = -sa;
        out[114 + i] = -sb;
    }
}

// height prior on vertex v: e = g . t - h; J (1 x 6, numeric) -> HB[v] = {J (6), e}
__device__ void pgo_linearize_height(const PgoArgs& a, int v) {
    const double* T = a.P + 12 * v;
    double* out = a.HB + 8 * v;
    for (int c = 0; c < 6; c++) {
        double dx[6] = {0, 0, 0, 0, 0, 0}, Tp[12], Tm[12];
        dx[c] = kPgoStep;
        oplus(T, dx, Tp);
        dx[c] = -kPgoStep;
        oplus(T, dx, Tm);
        const double ep = a.g[0] * Tp[9] + a.g[1] * Tp[10] + a.g[2] * Tp[11] - a.height;
        const double em = a.g[0] * Tm[9] + a.g[1] * Tm[10] + a.g[2] * Tm[11] - a.height;
        out[c] = (ep - em) / (2.0 * kPgoStep);
    }
    out[6] = a.g[0] * T[9] + a.g[1] * T[10] + a.g[2] * T[11] - a.height;
}

__global__ __launch_bounds__(kPgoThreads) void k_pgo(PgoArgs a) {
    __shared__ double red[kPgoThreads];
    __shared__ double S[36], v6[6];
    __shared__ int s_ok;
    const int tid = threadIdx.x, n = a.n;
    // measurements: odometry from the initial poses, Z = Ta^-1 Tb (Optimizer.cpp:715), loops as
    // given (slots hold Z on entry); EdgeSE3::setMeasurement keeps Z^-1
    for (int k = tid; k < a.E; k += kPgoThreads) {
        double z[12];
        if (k < a.E - a.L) {
            double ia[12];
            iso_inv(a.P + 12 * a.ea[k], ia);
            iso_mul(ia, a.P + 12 * a.eb[k], z);
        } else {
            for (int q = 0; q < 12; q++) z[q] = a.Zinv[12 * k + q];
        }
        iso_inv(z, a.Zinv + 12 * k);
    }
    __syncthreads();
    double chi = pgo_chi2(a, a.P, red);
    if (tid == 0) a.chi_out[0] = chi;
    double lambda = 0, ni = 2;
    int it = 0, accepted = 0, trials = 0;
    bool go = true;
    for (; it < a.iters && go; it++) {
        // ---- linearise and assemble ----
        for (int k = tid; k < a.E; k += kPgoThreads) pgo_linearize_edge(a, k);
        if (a.has_h)
            for (int v = 1 + tid; v < a.N; v += kPgoThreads) pgo_linearize_height(a, v);
        __syncthreads();
        const int nblk = a.colp[n];
        for (int q = tid; q < nblk * 36; q += kPgoThreads) {
            const int blk = q / 36, el = q - blk * 36, r = el / 6, c = el - r * 6;
            double s = 0;
            for (int m = a.clist_p[blk]; m < a.clist_p[blk + 1]; m++) {
                const int e = a.clist[m] >> 2, kind = a.clist[m] & 3;
                const double* B = a.EB + 120 * e;
                s += kind == 0 ? B[el] : kind == 1 ? B[72 + el] : kind == 2 ? B[36 + el] : B[36 + c * 6 + r];
            }
            a.H[(size_t)blk * 36 + el] = s;
        }
        for (int q = tid; q < n * 6; q += kPgoThreads) {
            const int j = q / 6, r = q - j * 6, v = j + 1;
            double s = 0;
            for (int m = a.vinc_p[v]; m < a.vinc_p[v + 1]; m++) {
                const int e = a.vinc[m] >> 1, side = a.vinc[m] & 1;
                s += a.EB[120 * e + 108 + 6 * side + r];
            }
            a.b[q] = s;
        }
        __syncthreads();
        if (a.has_h) {  // the unary blocks on the diagonal (after the binary ones: a fixed order)
            for (int q = tid; q < n * 36; q += kPgoThreads) {
                const int j = q / 36, el = q - j * 36, r = el / 6, c = el - r * 6;
                const double* hb = a.HB + 8 * (j + 1);
                a.H[(size_t)(a.colp[j + 1] - 1) * 36 + el] += hb[r] * a.hinfo * hb[c];
            }
            for (int q = tid; q < n * 6; q += kPgoThreads) {
                const double* hb = a.HB + 8 * (q / 6 + 1);
                a.b[q] -= hb[q % 6] * a.hinfo * hb[6];
            }
            __syncthreads();
        }
        if (it == 0) {  // computeLambdaInit: tau * max |H_ii|
            double m = 0;
            for (int q = tid; q < n * 6; q += kPgoThreads) {
                const int j = q / 6, r = q - j * 6;
                m = fmax(m, fabs(a.H[(size_t)(a.colp[j + 1] - 1) * 36 + r * 7]));
            }
            red[tid] = m;
            __syncthreads();
            for (int o = kPgoThreads / 2; o > 0; o >>= 1) {
                if (tid < o) red[tid] = fmax(red[tid], red[tid + o]);
                __syncthreads();
            }
            lambda = a.tau * red[0];
            ni = 2;
            __syncthreads();
        }
        // ---- LM trials ----
        double rho = 0;
        int qmax = 0;
        do {
            // factorise H + lambda I = U^T U (block skyline, column by column)
            if (tid == 0) s_ok = 1;
            __syncthreads();
            for (int j = 0; j < n; j++) {
                const int f = a.colf[j];
                for (int i = f; i <= j; i++) {
                    const size_t bij = (size_t)(a.colp[j] + i - f) * 36;
                    if (tid < 36) {
                        const int r = tid / 6, c = tid - (tid / 6) * 6;
                        double s = a.H[bij + tid] + (i == j && r == c ? lambda : 0.0);
                        const int k0 = max(a.colf[i], f);
                        for (int k = k0; k < i; k++) {
                            const double* Uki = a.U + (size_t)(a.colp[i] + k - a.colf[i]) * 36;
                            const double* Ukj = a.U + (size_t)(a.colp[j] + k - f) * 36;
                            for (int m = 0; m < 6; m++) s -= Uki[m * 6 + r] * Ukj[m * 6 + c];
                        }
                        S[tid] = s;
                    }
                    __syncthreads();
                    if (i < j) {
                        if (tid < 6) {  // U_ij[:, c] = U_ii^-T S[:, c] (forward substitution)
                            const double* Uii = a.U + (size_t)(a.colp[i + 1] - 1) * 36;
                            double yv[6];
                            for (int r = 0; r < 6; r++) {
                                double s = S[r * 6 + tid];
                                for (int m = 0; m < r; m++) s -= Uii[m * 6 + r] * yv[m];
                                yv[r] = s / Uii[r * 6 + r];
                            }
                            for (int r = 0; r < 6; r++) a.U[bij + r * 6 + tid] = yv[r];
                        }
                    } else if (tid == 0) {  // U_jj = chol(S), upper
                        double Uj[36];
                        for (int q = 0; q < 36; q++) Uj[q] = 0;
                        for (int c = 0; c < 6 && s_ok; c++) {
                            double s = S[c * 6 + c];
                            for (int k = 0; k < c; k++) s -= Uj[k * 6 + c] * Uj[k * 6 + c];
                            if (!(s > 0)) {
                                s_ok = 0;
                                break;
                            }
                            const double d = sqrt(s);
                            Uj[c * 6 + c] = d;
                            for (int r2 = c + 1; r2 < 6; r2++) {
                                double t = S[c * 6 + r2];
                                for (int k = 0; k < c; k++) t -= Uj[k * 6 + c] * Uj[k * 6 + r2];
                                Uj[c * 6 + r2] = t / d;
                            }
                        }
                        for (int q = 0; q < 36; q++) a.U[bij + q] = Uj[q];
                    }
                    __syncthreads();
                }
                if (!s_ok) break;
            }
            const bool ok = s_ok != 0;
            if (ok) {
                // U^T y = b (forward), U x = y (backward), column-oriented over the envelope
                for (int j = 0; j < n; j++) {
                    const int f = a.colf[j];
                    if (tid < 6) {
                        double s = a.b[6 * j + tid];
                        for (int k = f; k < j; k++) {
                            const double* Ukj = a.U + (size_t)(a.colp[j] + k - f) * 36;
                            for (int m = 0; m < 6; m++) s -= Ukj[m * 6 + tid] * a.y[6 * k + m];
                        }
                        v6[tid] = s;
                    }
                    __syncthreads();
                    if (tid == 0) {
                        const double* Ujj = a.U + (size_t)(a.colp[j + 1] - 1) * 36;
                        for (int r = 0; r < 6; r++) {
                            double s = v6[r];
                            for (int m = 0; m < r; m++) s -= Ujj[m * 6 + r] * a.y[6 * j + m];
                            a.y[6 * j + r] = s / Ujj[r * 6 + r];
                        }
                    }
                    __syncthreads();
                }
                for (int j = n - 1; j >= 0; j--) {
                    const int f = a.colf[j];
                    if (tid == 0) {
                        const double* Ujj = a.U + (size_t)(a.colp[j + 1] - 1) * 36;
                        for (int r = 5; r >= 0; r--) {
                            double s = a.y[6 * j + r];
                            for (int m = r + 1; m < 6; m++) s -= Ujj[r * 6 + m] * a.x[6 * j + m];
                            a.x[6 * j + r] = s / Ujj[r * 6 + r];
                        }
                    }
                    __syncthreads();
                    for (int q = tid; q < (j - f) * 6; q += kPgoThreads) {  // y_k -= U_kj x_j
                        const int k = f + q / 6, r = q % 6;
                        const double* Ukj = a.U + (size_t)(a.colp[j] + k - f) * 36;
                        double s = 0;
                        for (int m = 0; m < 6; m++) s += Ukj[r * 6 + m] * a.x[6 * j + m];
                        a.y[6 * k + r] -= s;
                    }
                    __syncthreads();
                }
            }
            // trial poses
            for (int v = tid; v < a.N; v += kPgoThreads) {
                if (v == 0 || !ok) {
                    for (int q = 0; q < 12; q++) a.Pt[12 * v + q] = a.P[12 * v + q];
                } else {
                    oplus(a.P + 12 * v, a.x + 6 * (v - 1), a.Pt + 12 * v);
                }
            }
            __syncthreads();
            double tchi = pgo_chi2(a, a.Pt, red);
            if (!ok) tchi = DBL_MAX;
            // computeScale: sum x (lambda x + b), + 1e-3
            double sc = 0;
            if (ok)
                for (int q = tid; q < n * 6; q += kPgoThreads) sc += a.x[q] * (lambda * a.x[q] + a.b[q]);
            red[tid] = sc;
            __syncthreads();
            for (int o = kPgoThreads / 2; o > 0; o >>= 1) {
                if (tid < o) red[tid] += red[tid + o];
                __syncthreads();
            }
            const double scale = red[0] + 1e-3;
            __syncthreads();
            rho = (chi - tchi) / scale;
            trials++;
            if (rho > 0 && isfinite(tchi) && ok) {
                double alpha = 1.0 - pow(2 * rho - 1, 3);
                alpha = fmin(alpha, 2.0 / 3.0);
                lambda *= fmax(1.0 / 3.0, alpha);
                ni = 2;
                chi = tchi;
                accepted++;
                for (int q = tid; q < 12 * a.N; q += kPgoThreads) a.P[q] = a.Pt[q];
                __syncthreads();
            } else {
                lambda *= ni;
                ni *= 2;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0 || !isfinite(lambda)) go = false;
    }
    if (tid == 0) {
        a.stats[0] = it;
        a.stats[1] = accepted;
        a.stats[2] = trials;
        a.stats[3] = 1;
        a.chi_out[1] = chi;
        a.chi_out[2] = lambda;
    }
}

// map points: p <- delta_k p with delta_k = new_k * old_k^-1 for the point's keyframe k
__global__ void k_pgo_points(const double* __restrict__ delta, const int* __restrict__ kf, int M, double* pos) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const int k = kf[i];
    if (k < 0) return;
    const double* D = delta + 12 * k;
    const double x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
    pos[3 * i] = D[0] * x + D[1] * y + D[2] * z + D[9];
    pos[3 * i + 1] = D[3] * x + D[4] * y + D[5] * z + D[10];
    pos[3 * i + 2] = D[6] * x + D[7] * y + D[8] * z + D[11];
}

__global__ void k_pgo_deltas(const double* __restrict__ Pnew, const double* __restrict__ Pold, int N, double* delta) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= N) return;
    double io[12];
    iso_inv(Pold + 12 * v, io);
    iso_mul(Pnew + 12 * v, io, delta + 12 * v);
}

}  // namespace vs

using namespace vs;

extern "C" {

int vs_pose_graph_optimize(vs_ctx* ctx, int N, double* R, double* t, int L, const int* lc_from, const int* lc_to,
                           const double* lc_R, const double* lc_t, const double* lc_sigma, const double* gravity,
                           double height, int iterations, int stats[4], double chi2[3]) {
    VS_ARG(ctx && R && t && N >= 0 && L >= 0 && iterations >= 0, "vs_pose_graph_optimize: bad arguments");
    VS_ARG(L == 0 || (lc_from && lc_to && lc_R && lc_t && lc_sigma), "vs_pose_graph_optimize: null loop arrays");
    if (stats) std::memset(stats, 0, 4 * sizeof(int));
    if (chi2) chi2[0] = chi2[1] = chi2[2] = 0;
    for (int l = 0; l < L; l++)
        VS_ARG(lc_from[l] >= 0 && lc_from[l] < N && lc_to[l] >= 0 && lc_to[l] < N && lc_from[l] != lc_to[l],
               "vs_pose_graph_optimize: loop vertex out of range");
    if (N < 3 || (L == 0 && !gravity)) return VS_OK;  // Optimizer.cpp:670, 775
    VS_HIP(hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    const int n = N - 1, E = N - 1 + L;
    // edges: odometry (i, i + 1), then loops; envelope of each block column (unknown j = vertex j + 1)
    std::vector<int> ea(E), eb(E);
    std::vector<double> Zinv((size_t)E * 12, 0.0), om((size_t)E * 6);
    const double ot = 1.0 / (0.05 * 0.05), orr = 1.0 / (0.02 * 0.02);  // PGO_ODOM_*_SIGMA (Config.h:133-134)
    for (int i = 0; i < N - 1; i++) {
        ea[i] = i;
        eb[i] = i + 1;
        for (int r = 0; r < 6; r++) om[6 * i + r] = r < 3 ? ot : orr;
    }
    std::vector<int> colf(n);
    for (int j = 0; j < n; j++) colf[j] = j > 0 ? j - 1 : 0;
    for (int l = 0; l < L; l++) {
        const int k = N - 1 + l;
        ea[k] = lc_from[l];
        eb[k] = lc_to[l];
        std::memcpy(Zinv.data() + 12 * k, lc_R + 9 * l, 9 * sizeof(double));  // Z; inverted on the device
        std::memcpy(Zinv.data() + 12 * k + 9, lc_t + 3 * l, 3 * sizeof(double));
        const double st = lc_sigma[2 * l], sr = lc_sigma[2 * l + 1];
        for (int r = 0; r < 6; r++) om[6 * k + r] = r < 3 ? 1.0 / (st * st) : 1.0 / (sr * sr);
        const int lo = std::min(ea[k], eb[k]), hi = std::max(ea[k], eb[k]);
        if (lo >= 1) colf[hi - 1] = std::min(colf[hi - 1], lo - 1);
    }
    std::vector<int> colp(n + 1, 0);
    for (int j = 0; j < n; j++) colp[j + 1] = colp[j] + (j - colf[j] + 1);
    const int nblk = colp[n];
    // contribution lists per skyline block (fixed order: odometry edges, then loops)
    std::vector<std::vector<int>> contrib(nblk);
    auto blk = [&](int vi, int vj) { return colp[vj - 1] + (vi - 1) - colf[vj - 1]; };  // vi <= vj, both >= 1
    for (int k = 0; k < E; k++) {
        const int va = ea[k], vb = eb[k];
        if (va >= 1) contrib[blk(va, va)].push_back(4 * k + 0);
        if (vb >= 1) contrib[blk(vb, vb)].push_back(4 * k + 1);
        if (va >= 1 && vb >= 1) {
            if (va < vb)
                contrib[blk(va, vb)].push_back(4 * k + 2);
            else
                contrib[blk(vb, va)].push_back(4 * k + 3);
        }
    }
    std::vector<int> clist_p(nblk + 1, 0), clist;
    for (int q = 0; q < nblk; q++) {
        clist.insert(clist.end(), contrib[q].begin(), contrib[q].end());
        clist_p[q + 1] = (int)clist.size();
    }
    std::vector<std::vector<int>> inc(N);
    for (int k = 0; k < E; k++) {
        inc[ea[k]].push_back(2 * k);
        inc[eb[k]].push_back(2 * k + 1);
    }
    std::vector<int> vinc_p(N + 1, 0), vinc;
    for (int v = 0; v < N; v++) {
        vinc.insert(vinc.end(), inc[v].begin(), inc[v].end());
        vinc_p[v + 1] = (int)vinc.size();
    }
    if (clist.empty()) clist.push_back(0);
    // one device block: doubles first, then ints
    std::vector<double> P0((size_t)N * 12);
    for (int v = 0; v < N; v++) {
        std::memcpy(&P0[12 * v], R + 9 * (size_t)v, 9 * sizeof(double));
        std::memcpy(&P0[12 * v + 9], t + 3 * (size_t)v, 3 * sizeof(double));
    }
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (bytes + 255) & ~(size_t)255;
        return o;
    };
    const size_t oP = take((size_t)N * 12 * 8), oPt = take((size_t)N * 12 * 8), oP0 = take((size_t)N * 12 * 8);
    const size_t oZ = take((size_t)E * 12 * 8), oOm = take((size_t)E * 6 * 8), oEB = take((size_t)E * 120 * 8);
    const size_t oHB = take((size_t)N * 8 * 8), oH = take((size_t)nblk * 36 * 8), oU = take((size_t)nblk * 36 * 8);
    const size_t ob = take((size_t)n * 6 * 8), ox = take((size_t)n * 6 * 8), oy = take((size_t)n * 6 * 8);
    const size_t ochi = take(3 * 8);
    const size_t oea = take((size_t)E * 4), oeb = take((size_t)E * 4), ocf = take((size_t)n * 4);
    const size_t ocp = take((size_t)(n + 1) * 4), oclp = take((size_t)(nblk + 1) * 4), ocl = take(clist.size() * 4);
    const size_t ovp = take((size_t)(N + 1) * 4), ov = take(vinc.size() * 4 + 4), ost = take(4 * 4);
    DevBuf buf;
    VS_CHECK(buf.ensure(off));
    char* d = buf.as<char>();
    auto up = [&](size_t o, const void* src, size_t bytes) -> int {
        if (bytes) VS_HIP(hipMemcpyAsync(d + o, src, bytes, hipMemcpyHostToDevice, s));
        return VS_OK;
    };
    int rc = VS_OK;
    if (rc == VS_OK) rc = up(oP, P0.data(), P0.size() * 8);
    if (rc == VS_OK) rc = up(oP0, P0.data(), P0.size() * 8);
    if (rc == VS_OK) rc = up(oZ, Zinv.data(), Zinv.size() * 8);
    if (rc == VS_OK) rc = up(oOm, om.data(), om.size() * 8);
    if (rc == VS_OK) rc = up(oea, ea.data(), ea.size() * 4);
    if (rc == VS_OK) rc = up(oeb, eb.data(), eb.size() * 4);
    if (rc == VS_OK) rc = up(ocf, colf.data(), colf.size() * 4);
    if (rc == VS_OK) rc = up(ocp, colp.data(), colp.size() * 4);
    if (rc == VS_OK) rc = up(oclp, clist_p.data(), clist_p.size() * 4);
    if (rc == VS_OK) rc = up(ocl, clist.data(), clist.size() * 4);
    if (rc == VS_OK) rc = up(ovp, vinc_p.data(), vinc_p.size() * 4);
    if (rc == VS_OK) rc = up(ov, vinc.data(), vinc.size() * 4);
    if (rc != VS_OK) {
        (void)hipStreamSynchronize(s);
        return rc;
    }
    PgoArgs a{};
    a.N = N;
    a.n = n;
    a.E = E;
    a.L = L;
    a.iters = iterations;
    a.has_h = gravity != nullptr;
    a.tau = 1e-5;  // g2o OptimizationAlgorithmLevenberg _tau
    a.height = height;
    a.hinfo = 1.0 / (0.005 * 0.005);  // PGO_HEIGHT_SIGMA (Config.h:137)
    if (gravity)
        for (int k = 0; k < 3; k++) a.g[k] = gravity[k];
    a.P = reinterpret_cast<double*>(d + oP);
    a.Pt = reinterpret_cast<double*>(d + oPt);
    a.ea = reinterpret_cast<const int*>(d + oea);
    a.eb = reinterpret_cast<const int*>(d + oeb);
    a.Zinv = reinterpret_cast<double*>(d + oZ);
    a.om = reinterpret_cast<const double*>(d + oOm);
    a.EB = reinterpret_cast<double*>(d + oEB);
    a.HB = reinterpret_cast<double*>(d + oHB);
    a.colf = reinterpret_cast<const int*>(d + ocf);
    a.colp = reinterpret_cast<const int*>(d + ocp);
    a.clist_p = reinterpret_cast<const int*>(d + oclp);
    a.clist = reinterpret_cast<const int*>(d + ocl);
    a.vinc_p = reinterpret_cast<const int*>(d + ovp);
    a.vinc = reinterpret_cast<const int*>(d + ov);
    a.H = reinterpret_cast<double*>(d + oH);
    a.U = reinterpret_cast<double*>(d + oU);
    a.b = reinterpret_cast<double*>(d + ob);
    a.x = reinterpret_cast<double*>(d + ox);
    a.y = reinterpret_cast<double*>(d + oy);
    a.stats = reinterpret_cast<int*>(d + ost);
    a.chi_out = reinterpret_cast<double*>(d + ochi);
    {
        ProfScope ps(ctx, "pose_graph", s);
        hipLaunchKernelGGL(k_pgo, dim3(1), dim3(kPgoThreads), 0, s, a);
    }
    VS_HIP(hipGetLastError());
    std::vector<double> Pn((size_t)N * 12);
    int st[4];
    double ch[3];
    VS_HIP(hipMemcpyAsync(Pn.data(), d + oP, Pn.size() * 8, hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(st, d + ost, sizeof(st), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(ch, d + ochi, sizeof(ch), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    for (int v = 0; v < N; v++) {
        std::memcpy(R + 9 * (size_t)v, &Pn[12 * v], 9 * sizeof(double));
        std::memcpy(t + 3 * (size_t)v, &Pn[12 * v + 9], 3 * sizeof(double));
    }
    if (stats) {
        stats[0] = st[0];
        stats[1] = st[1];
        stats[2] = st[2];
        stats[3] = L;
    }
    if (chi2) std::memcpy(chi2, ch, sizeof(ch));
    return VS_OK;
}

int vs_pgo_transform_points(vs_ctx* ctx, int N, const double* R_old, const double* t_old, const double* R_new,
                            const double* t_new, int M, const int* kf, double* pos) {
    VS_ARG(ctx && N >= 0 && M >= 0, "vs_pgo_transform_points: bad arguments");
    if (N == 0 || M == 0) return VS_OK;
    VS_ARG(R_old && t_old && R_new && t_new && kf && pos, "vs_pgo_transform_points: null argument");
    VS_HIP(hipSetDevice(ctx->device));
    const hipStream_t s = ctx->stream;
    std::vector<double> Po((size_t)N * 12), Pn((size_t)N * 12);
    for (int v = 0; v < N; v++) {
        std::memcpy(&Po[12 * v], R_old + 9 * (size_t)v, 72);
        std::memcpy(&Po[12 * v + 9], t_old + 3 * (size_t)v, 24);
        std::memcpy(&Pn[12 * v], R_new + 9 * (size_t)v, 72);
        std::memcpy(&Pn[12 * v + 9], t_new + 3 * (size_t)v, 24);
    }
    const size_t b1 = (size_t)N * 12 * 8, b3 = (size_t)M * 3 * 8, b4 = (size_t)M * 4;
    DevBuf buf;
    VS_CHECK(buf.ensure(3 * b1 + b3 + b4 + 1024));
    double* dPo = buf.as<double>();
    double* dPn = dPo + (size_t)N * 12;
    double* dD = dPn + (size_t)N * 12;
    double* dpos = dD + (size_t)N * 12;
    int* dkf = reinterpret_cast<int*>(dpos + (size_t)M * 3);
    VS_HIP(hipMemcpyAsync(dPo, Po.data(), b1, hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dPn, Pn.data(), b1, hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dpos, pos, b3, hipMemcpyHostToDevice, s));
    VS_HIP(hipMemcpyAsync(dkf, kf, b4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_pgo_deltas, dim3((N + 127) / 128), dim3(128), 0, s, dPn, dPo, N, dD);
    hipLaunchKernelGGL(k_pgo_points, dim3((M + 255) / 256), dim3(256), 0, s, dD, dkf, M, dpos);
    VS_HIP(hipGetLastError());
    VS_HIP(hipMemcpyAsync(pos, dpos, b3, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    return VS_OK;
}

}  // extern "C"
