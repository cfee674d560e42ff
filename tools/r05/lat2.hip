// latency probe of pnp_solvers.h pieces on one wave (round 5): lanes 0..2 active like the EPnP variants
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../visual-slam-pipeline_amd/csrc/pnp_solvers.h"
using namespace vs_pnp;
__global__ void k(double* io, long long* cyc) {
    const int l = threadIdx.x;
    if (l >= 3) return;
    double A[24], b[6], x[4];
    for (int i = 0; i < 24; i++) A[i] = io[i] + l * 1e-3;
    for (int i = 0; i < 6; i++) b[i] = io[24 + i];
    long long t0 = clock64();
    lstsq<6, 4>(A, b, x);
    long long t1 = clock64();
    double C[9] = {x[0] + 2, 0.3, 0.1, 0.3, x[1] + 1, 0.2, 0.1, 0.2, x[2] + 0.5}, w[3], V[9];
    sym_eig<3>(C, w, V);
    long long t2 = clock64();
    double ABt[9] = {w[0], 0.1, 0.2, 0.3, w[1], 0.1, V[0], 0.2, w[2]}, R[9];
    rotation_from_cross(ABt, R);
    long long t3 = clock64();
    double rv[3], R2[9];
    rod_m2v(R, rv);
    long long t4 = clock64();
    rod_v2m(rv, R2);
    long long t5 = clock64();
    double c, s;
    double acc = R2[0];
    for (int i = 0; i < 8; i++) { jacobi_angle(acc, 1.0, 0.3, c, s); acc = c + s; }
    long long t6 = clock64();
    io[64 + l] = acc + R2[4] + x[3];
    if (l == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4; cyc[5] = (t6 - t5) / 8; }
}
int main() {
    double* io; long long* c;
    (void)hipMalloc(&io, 128 * 8); (void)hipMalloc(&c, 64);
    double h[128]; for (int i = 0; i < 128; i++) h[i] = 0.5 + ((i * 37) % 11) * 0.1;
    (void)hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, io, c);
        long long hc[6]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("cycles: lstsq<6,4> %lld  sym_eig<3> %lld  rotation_from_cross %lld  rod_m2v %lld  rod_v2m %lld  jacobi_angle %lld\n",
               hc[0], hc[1], hc[2], hc[3], hc[4], hc[5]);
    }
    return 0;
}
