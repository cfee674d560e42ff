// Reduced repro of the round-5 device/host EPnP divergence, isolated by the stage dump of
// tests/test_gpu_pnp.py::test_epnp_eig_stages_out_of_line to step 2 of epnp_small_eig (B = R R^T from the
// QR's alpha and C): the QR results are equal, B is not, when the function runs out of line.
//
// This program computes the QR inputs (alpha[10], C[10][12]) of 2,000 five-point EPnP problems on the host
// with pnp_solvers.h, then B from them on the host and on the device in several forms:
//   0  the product's statement, inlined into the kernel
//   1  the same statement in a noinline device function (arguments: pointers into the caller's stack)
//   2  noinline, alpha / C passed through global memory instead of the caller's private arrays
//   3  noinline, the statement without the ternary selects (the two factors read by index)
// and prints how many problems differ bit for bit from the host in each form; then the QR itself (step 1)
// on the device, inline (4) and out of line (5), entry by entry against the host's.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I visual-slam-pipeline_amd/csrc \
//         tools/r06/epnp_b_repro.hip -o tools/r06/epnp_b_repro && tools/r06/epnp_b_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "pnp_solvers.h"

using namespace vs_pnp;

struct QrIn {
    double alpha[10];
    double C[10][12];
};

// epnp_small_eig step 2, verbatim
__host__ __device__ inline void b_product(const double* alpha, const double (*C)[12], double* Bout) {
    double t[12];
    double B[10][10];
    for (int a = 0; a < 10; a++)
        for (int b = a; b < 10; b++) {
            for (int k = 0; k < 10; k++)
                t[k] = k >= b ? (k == a ? alpha[a] : C[k][a]) * (k == b ? alpha[b] : C[k][b]) : -0.0;
            B[a][b] = B[b][a] = tsum<10>(t);
        }
    for (int i = 0; i < 100; i++) Bout[i] = B[i / 10][i % 10];
}
// the same products and order without the selects
__host__ __device__ inline void b_product_idx(const double* alpha, const double (*C)[12], double* Bout) {
    double t[12];
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
    for (int i = 0; i < 100; i++) Bout[i] = B[i / 10][i % 10];
}

__device__ __attribute__((noinline)) void b_out_of_line(const double* alpha, const double (*C)[12], double* Bout) {
    b_product(alpha, C, Bout);
}
__device__ __attribute__((noinline)) void b_out_of_line_idx(const double* alpha, const double (*C)[12], double* Bout) {
    b_product_idx(alpha, C, Bout);
}

__global__ void k_b(const QrIn* in, int n, int mode, double* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    double alpha[10], C[10][12];  // private copies, as epnp_small_eig holds them
    for (int i = 0; i < 10; i++) alpha[i] = in[p].alpha[i];
    for (int i = 0; i < 10; i++)
        for (int r = 0; r < 12; r++) C[i][r] = in[p].C[i][r];
    double* o = out + (size_t)p * 100;
    if (mode == 0)
        b_product(alpha, C, o);
    else if (mode == 1)
        b_out_of_line(alpha, C, o);
    else if (mode == 2)
        b_out_of_line(in[p].alpha, in[p].C, o);
    else
        b_out_of_line_idx(alpha, C, o);
}

// epnp_small_eig's step 1 (QR of M^T): alpha and C from the control-point weights al and the pixels
struct QrSrc {
    double al[5][4];
    double uv[10];
};
__host__ __device__ inline void qr_of(const double (*al)[4], const double* uv, QrIn& q) {
    const Cam K{525.0, 525.0, 319.5, 239.5};
    double t[12], tau[10];
    for (int j = 0; j < 10; j++)
        for (int r = 0; r < 12; r++) q.C[j][r] = ep_mt(al, uv, K, j, r);
    for (int k = 0; k < 10; k++) {
        for (int r = 0; r < 12; r++) t[r] = r >= k ? q.C[k][r] * q.C[k][r] : -0.0;
        double u0;
        ep_householder(tsum<12>(t), q.C[k][k], q.alpha[k], u0, tau[k]);
        q.C[k][k] = u0;
        for (int j = k + 1; j < 10; j++) {
            for (int r = 0; r < 12; r++) t[r] = r >= k ? q.C[k][r] * q.C[j][r] : -0.0;
            const double f = tau[k] * tsum<12>(t);
            for (int r = k; r < 12; r++) q.C[j][r] = q.C[j][r] - f * q.C[k][r];
        }
    }
}

__device__ __attribute__((noinline)) void qr_out_of_line(const double (*al)[4], const double* uv, QrIn& q) {
    qr_of(al, uv, q);
}

// modes 4 / 5: the QR itself on the device (inline / out of line); out = C[10][12] then alpha[10]
__global__ void k_qr(const QrSrc* src, int n, int mode, double* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    double al[5][4], uv[10];
    for (int i = 0; i < 5; i++)
        for (int c = 0; c < 4; c++) al[i][c] = src[p].al[i][c];
    for (int i = 0; i < 10; i++) uv[i] = src[p].uv[i];
    QrIn q;
    if (mode == 4)
        qr_of(al, uv, q);
    else
        qr_out_of_line(al, uv, q);
    double* o = out + (size_t)p * 130;
    for (int j = 0; j < 10; j++)
        for (int r = 0; r < 12; r++) o[12 * j + r] = q.C[j][r];
    for (int i = 0; i < 10; i++) o[120 + i] = q.alpha[i];
}

// the whole eigen stage (the product's epnp_small_eig, templated copies): VAR 0 verbatim, 1 with m fixed at 5
// (compile-time loop bounds), 2 returning right after B
template <int VAR>
__host__ __device__ inline void eig_copy(const double (*al)[4], const double* uv, int m_in, const Cam& K, double v[4][12],
                                        double* dbg) {
    const int m = VAR == 1 ? 5 : m_in;
    const int nc = 2 * m;  // 8 or 10
    double C[10][12], alpha[10], tau[10], t[12];
    for (int j = 0; j < nc; j++)
        for (int r = 0; r < 12; r++) C[j][r] = ep_mt(al, uv, K, j, r);
    if (VAR == 3) {  // C as ep_mt builds it
        for (int j = 0; j < 10; j++)
            for (int r = 0; r < 12; r++) dbg[12 * j + r] = C[j][r];
        return;
    }
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
    if (VAR == 4) {  // C and alpha after the QR
        for (int j = 0; j < 10; j++)
            for (int r = 0; r < 12; r++) dbg[12 * j + r] = C[j][r];
        for (int i = 0; i < 10; i++) dbg[120 + i] = alpha[i];
        return;
    }
    if (VAR == 5) __asm__ volatile("" : : "r"(&C[0][0]), "r"(&alpha[0]) : "memory");  // C, alpha to memory here
    double x[4][12];
    const int nz = nc == 10 ? 2 : 4;  // null vectors
    for (int q = 0; q < 4; q++)
        for (int r = 0; r < 12; r++) x[q][r] = (q < nz && r == nc + q) ? 1.0 : 0.0;
    if (nc == 10) {
        // 2. B = R R^T (R_ak = C[k][a] above the diagonal, alpha[a] on it), upper triangle then mirrored
        double B[10][10], t2[10];
        double* tb = VAR == 6 ? t2 : t;  // VAR 6: B's products in an array of their own
        if (VAR == 7) {  // the factors by if-assignment instead of the two selects
            for (int a = 0; a < 10; a++)
                for (int b = a; b < 10; b++) {
                    for (int k = 0; k < 10; k++) {
                        double fa = C[k][a], fb = C[k][b];
                        if (k == a) fa = alpha[a];
                        if (k == b) fb = alpha[b];
                        tb[k] = k >= b ? fa * fb : -0.0;
                    }
                    B[a][b] = B[b][a] = tsum<10>(tb);
                }
        } else if (VAR == 8) {  // R^T (R_ak in Rt[k][a], alpha on the diagonal) copied out first
            double Rt[10][10];
            for (int k = 0; k < 10; k++)
                for (int a = 0; a < 10; a++) Rt[k][a] = k == a ? alpha[a] : k > a ? C[k][a] : 0.0;
            for (int a = 0; a < 10; a++)
                for (int b = a; b < 10; b++) {
                    for (int k = 0; k < 10; k++) tb[k] = k >= b ? Rt[k][a] * Rt[k][b] : -0.0;
                    B[a][b] = B[b][a] = tsum<10>(tb);
                }
        } else {
        for (int a = 0; a < 10; a++)
            for (int b = a; b < 10; b++) {
                for (int k = 0; k < 10; k++)
                    tb[k] = k >= b ? (k == a ? alpha[a] : C[k][a]) * (k == b ? alpha[b] : C[k][b]) : -0.0;
                B[a][b] = B[b][a] = tsum<10>(tb);
            }
        }
        if (dbg)
            for (int i = 0; i < 10; i++) {
                dbg[i] = alpha[i];
                dbg[10 + i] = tau[i];
                for (int j = 0; j < 10; j++) dbg[20 + 10 * i + j] = B[i][j];
            }
        if (VAR == 2 || VAR >= 5) return;
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

template <int VAR>
__device__ __attribute__((noinline)) void eig_ool(const double (*al)[4], const double* uv, int m, const Cam& K,
                                                  double v[4][12], double* dbg) {
    eig_copy<VAR>(al, uv, m, K, v, dbg);
}
__device__ __attribute__((noinline)) void eig_product_ool(const double (*al)[4], const double* uv, int m, const Cam& K,
                                                          double v[4][12], double* dbg) {
    epnp_small_eig(al, uv, m, K, v, dbg);
}

// modes 6..10: the whole eigen stage, B dumped (dbg[20..120)): 6 the product's function out of line,
// 7 inline, 8 / 9 / 10 the copy VAR 0 / 1 / 2 out of line
__global__ void k_eig(const QrSrc* src, int n, int mode, double* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    double al[5][4], uv[10], v[4][12];
    for (int i = 0; i < 5; i++)
        for (int c = 0; c < 4; c++) al[i][c] = src[p].al[i][c];
    for (int i = 0; i < 10; i++) uv[i] = src[p].uv[i];
    const Cam K{525.0, 525.0, 319.5, 239.5};
    double* o = out + (size_t)p * 216;
    for (int i = 0; i < 216; i++) o[i] = 0.0;
    if (mode == 6) eig_product_ool(al, uv, 5, K, v, o);
    if (mode == 7) epnp_small_eig(al, uv, 5, K, v, o);
    if (mode == 8) eig_ool<0>(al, uv, 5, K, v, o);
    if (mode == 9) eig_ool<1>(al, uv, 5, K, v, o);
    if (mode == 10) eig_ool<2>(al, uv, 5, K, v, o);
    if (mode == 11) eig_ool<3>(al, uv, 5, K, v, o);
    if (mode == 12) eig_ool<4>(al, uv, 5, K, v, o);
    if (mode == 14) eig_ool<5>(al, uv, 5, K, v, o);
    if (mode == 15) eig_ool<6>(al, uv, 5, K, v, o);
    if (mode == 16) eig_ool<7>(al, uv, 5, K, v, o);
    if (mode == 17) eig_ool<8>(al, uv, 5, K, v, o);
    if (mode == 13) {  // the camera built in the callee's caller from kernel arguments (as the library's hook)
        const Cam K2{src[p].uv[0] * 0.0 + 525.0, 525.0, 319.5, 239.5};
        eig_ool<2>(al, uv, 5, K2, v, o);
    }
}

int main() {
    const int n = 2000;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<QrIn> in(n);
    std::vector<QrSrc> qs(n);
    for (int p = 0; p < n; p++) {
        double X[15], cw[4][3];
        for (int j = 0; j < 5; j++) {
            X[3 * j] = 2 * U(rng), X[3 * j + 1] = 1.5 * U(rng), X[3 * j + 2] = 4 + 2 * U(rng);
            qs[p].uv[2 * j] = 319.5 + 525.0 * X[3 * j] / X[3 * j + 2] + 0.5 * U(rng);
            qs[p].uv[2 * j + 1] = 239.5 + 525.0 * X[3 * j + 1] / X[3 * j + 2] + 0.5 * U(rng);
        }
        epnp_control<5>(X, 5, cw, qs[p].al);
        qr_of(qs[p].al, qs[p].uv, in[p]);
    }
    std::vector<double> host((size_t)n * 100), dev((size_t)n * 100);
    for (int p = 0; p < n; p++) b_product(in[p].alpha, in[p].C, host.data() + (size_t)p * 100);
    QrIn* d_in;
    double* d_out;
    if (hipMalloc(&d_in, sizeof(QrIn) * n) != hipSuccess || hipMalloc(&d_out, sizeof(double) * 100 * n) != hipSuccess)
        return 1;
    (void)hipMemcpy(d_in, in.data(), sizeof(QrIn) * n, hipMemcpyHostToDevice);
    const char* what[4] = {"inline", "noinline, private arrays", "noinline, global arrays", "noinline, no selects"};
    for (int mode = 0; mode < 4; mode++) {
        (void)hipMemset(d_out, 0, sizeof(double) * 100 * n);
        hipLaunchKernelGGL(k_b, dim3((n + 63) / 64), dim3(64), 0, 0, d_in, n, mode, d_out);
        if (hipMemcpy(dev.data(), d_out, sizeof(double) * 100 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int bad = 0, first = -1, fe = -1;
        for (int p = 0; p < n; p++)
            for (int i = 0; i < 100; i++)
                if (std::memcmp(&host[(size_t)p * 100 + i], &dev[(size_t)p * 100 + i], 8) != 0) {
                    if (first < 0) first = p, fe = i;
                    bad++;
                    break;
                }
        std::printf("mode %d (%s): %d of %d problems differ", mode, what[mode], bad, n);
        if (first >= 0)
            std::printf("; first: problem %d entry %d host %.17g dev %.17g", first, fe, host[(size_t)first * 100 + fe],
                        dev[(size_t)first * 100 + fe]);
        std::printf("\n");
    }
    // the QR on the device
    QrSrc* d_src;
    double* d_q;
    if (hipMalloc(&d_src, sizeof(QrSrc) * n) != hipSuccess || hipMalloc(&d_q, sizeof(double) * 130 * n) != hipSuccess)
        return 1;
    (void)hipMemcpy(d_src, qs.data(), sizeof(QrSrc) * n, hipMemcpyHostToDevice);
    std::vector<double> qd((size_t)n * 130);
    for (int mode = 4; mode < 6; mode++) {
        hipLaunchKernelGGL(k_qr, dim3((n + 63) / 64), dim3(64), 0, 0, d_src, n, mode, d_q);
        if (hipMemcpy(qd.data(), d_q, sizeof(double) * 130 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int bad_r = 0, bad_u = 0, bad_a = 0, fj = -1, fr = -1, fp = -1;
        for (int p = 0; p < n; p++) {
            bool br = false, bu = false, ba = false;
            for (int j = 0; j < 10; j++)
                for (int r = 0; r < 12; r++)
                    if (std::memcmp(&qd[(size_t)p * 130 + 12 * j + r], &in[p].C[j][r], 8) != 0) {
                        if (r < j) {  // above the diagonal: R
                            if (!br && fp < 0) fp = p, fj = j, fr = r;
                            br = true;
                        } else {
                            bu = true;
                        }
                    }
            for (int i = 0; i < 10; i++)
                if (std::memcmp(&qd[(size_t)p * 130 + 120 + i], &in[p].alpha[i], 8) != 0) ba = true;
            bad_r += br, bad_u += bu, bad_a += ba;
        }
        std::printf("mode %d (QR %s): problems with R entries (C[j][r], r < j) differing: %d, reflector entries: %d, "
                    "alpha: %d of %d", mode, mode == 4 ? "inline" : "noinline", bad_r, bad_u, bad_a, n);
        if (fp >= 0)
            std::printf("; first: problem %d C[%d][%d] host %.17g dev %.17g", fp, fj, fr, in[fp].C[fj][fr],
                        qd[(size_t)fp * 130 + 12 * fj + fr]);
        std::printf("\n");
    }
    // the whole eigen stage
    double* d_e;
    if (hipMalloc(&d_e, sizeof(double) * 216 * n) != hipSuccess) return 1;
    std::vector<double> eh((size_t)n * 216, 0.0), ed((size_t)n * 216);
    const Cam Kh{525.0, 525.0, 319.5, 239.5};
    for (int p = 0; p < n; p++) {
        double v[4][12];
        epnp_small_eig(qs[p].al, qs[p].uv, 5, Kh, v, eh.data() + (size_t)p * 216);
    }
    const char* ewhat[5] = {"product's function, noinline", "product's function, inline", "copy, noinline",
                            "copy with m = 5 at compile time, noinline", "copy stopping after B, noinline"};
    for (int mode = 6; mode < 11; mode++) {
        hipLaunchKernelGGL(k_eig, dim3((n + 63) / 64), dim3(64), 0, 0, d_src, n, mode, d_e);
        if (hipMemcpy(ed.data(), d_e, sizeof(double) * 216 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int bad_b = 0, bad_all = 0, fp = -1, fi = -1;
        for (int p = 0; p < n; p++) {
            bool bb = false, ba = false;
            const int lim = mode == 10 ? 120 : 216;
            for (int i = 0; i < lim; i++)
                if (std::memcmp(&ed[(size_t)p * 216 + i], &eh[(size_t)p * 216 + i], 8) != 0) {
                    ba = true;
                    if (i >= 20 && i < 120) {
                        if (!bb && fp < 0) fp = p, fi = i;
                        bb = true;
                    }
                }
            bad_b += bb, bad_all += ba;
        }
        std::printf("mode %d (%s): B differs in %d, any stage in %d of %d problems", mode, ewhat[mode - 6], bad_b,
                    bad_all, n);
        if (fp >= 0)
            std::printf("; first: problem %d B[%d] host %.17g dev %.17g", fp, fi - 20, eh[(size_t)fp * 216 + fi],
                        ed[(size_t)fp * 216 + fi]);
        std::printf("\n");
    }
    // where it starts: C from ep_mt (11), C and alpha after the QR (12), against the host's copies
    for (int mode = 11; mode < 18; mode++) {
        std::vector<double> hh((size_t)n * 216, 0.0);
        for (int p = 0; p < n; p++) {
            double v[4][12];
            if (mode == 11) eig_copy<3>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 12) eig_copy<4>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 13) eig_copy<2>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 14) eig_copy<5>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 15) eig_copy<6>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 16) eig_copy<7>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
            if (mode == 17) eig_copy<8>(qs[p].al, qs[p].uv, 5, Kh, v, hh.data() + (size_t)p * 216);
        }
        hipLaunchKernelGGL(k_eig, dim3((n + 63) / 64), dim3(64), 0, 0, d_src, n, mode, d_e);
        if (hipMemcpy(ed.data(), d_e, sizeof(double) * 216 * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        int bad = 0, fp = -1, fi = -1;
        for (int p = 0; p < n; p++)
            for (int i = 0; i < 216; i++)
                if (std::memcmp(&ed[(size_t)p * 216 + i], &hh[(size_t)p * 216 + i], 8) != 0) {
                    if (fp < 0) fp = p, fi = i;
                    bad++;
                    break;
                }
        const char* w = mode == 11   ? "C from ep_mt"
                         : mode == 12 ? "C, alpha after the QR"
                         : mode == 13 ? "stop after B, camera from the kernel"
                         : mode == 14 ? "stop after B, compiler memory barrier between the QR and B"
                         : mode == 15 ? "stop after B, B's products in their own array"
                         : mode == 16 ? "stop after B, the factors by if-assignment"
                                      : "stop after B, R^T copied out first";
        std::printf("mode %d (%s, noinline): %d of %d differ", mode, w, bad, n);
        if (fp >= 0) std::printf("; first: problem %d entry %d host %.17g dev %.17g", fp, fi, hh[(size_t)fp * 216 + fi], ed[(size_t)fp * 216 + fi]);
        std::printf("\n");
    }
    (void)hipFree(d_e);
    (void)hipFree(d_src);
    (void)hipFree(d_q);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return 0;
}
