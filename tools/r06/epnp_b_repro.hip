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
    (void)hipFree(d_src);
    (void)hipFree(d_q);
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return 0;
}
