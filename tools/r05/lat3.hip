// latency probe of emat_solvers.h five_point on one lane (round 5)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../visual-slam-pipeline_amd/csrc/emat_solvers.h"
using namespace vs_em;
__global__ void k(const double* q, double* out, long long* cyc) {
    __shared__ double ws[kWsSize * 32];
    __shared__ double E[32 * kMaxModels * 9];
    const int l = threadIdx.x;
    if (l >= 32) return;
    double q1[10], q2[10];
    for (int i = 0; i < 10; i++) { q1[i] = q[20 * l + i]; q2[i] = q[20 * l + 10 + i]; }
    long long t0 = clock64();
    const int nm = five_point(q1, q2, &E[l * kMaxModels * 9], &ws[l], 32);
    long long t1 = clock64();
    long long t2 = clock64();
    out[l] = nm + E[l * kMaxModels * 9];
    if (l == 0) { cyc[0] = t1 - t0; cyc[1] = nm; }
}
int main() {
    double *q, *o; long long* c;
    (void)hipMalloc(&q, 640 * 8); (void)hipMalloc(&o, 64 * 8); (void)hipMalloc(&c, 64);
    double h[640];
    unsigned s = 12345;
    for (int i = 0; i < 640; i++) { s = s * 1103515245u + 12345u; h[i] = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    (void)hipMemcpy(q, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, q, o, c);
        long long hc[2]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("five_point cycles %lld (models %lld)\n", hc[0], hc[1]);
    }
    return 0;
}
