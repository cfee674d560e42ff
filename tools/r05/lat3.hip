// latency probe of emat_solvers.h five_point on one lane (round 5)
#include <hip/hip_runtime.h>
#include <cstdio>
#ifndef NL
#define NL 32
#endif
#include "../../visual-slam-pipeline_amd/csrc/emat_solvers.h"
using namespace vs_em;
__global__ void k(const double* q, double* out, long long* cyc) {
    __shared__ double ws[kWsSize * 32];
    __shared__ double E[32 * kMaxModels * 9];
    const int l = threadIdx.x;
    if (l >= NL) return;
    double q1[10], q2[10];
    for (int i = 0; i < 10; i++) { q1[i] = q[20 * l + i]; q2[i] = q[20 * l + 10 + i]; }
    long long st[6];
    int ns = 0;
    long long t0 = clock64();
    auto mark = [&](int k) { st[k] = clock64(); ns = k + 1; };
    const int nm = five_point(q1, q2, &E[l * kMaxModels * 9], &ws[l], 32, mark);
    long long t1 = clock64();
    out[l] = nm + E[l * kMaxModels * 9];
    if (l == 0) {
        cyc[0] = t1 - t0; cyc[1] = nm;
        long long prev = t0;
        for (int k = 0; k < 5; k++) { cyc[2 + k] = k < ns ? st[k] - prev : 0; if (k < ns) prev = st[k]; }
        cyc[7] = t1 - prev;
    }
}
int main() {
    double *q, *o; long long* c;
    (void)hipMalloc(&q, 640 * 8); (void)hipMalloc(&o, 64 * 8); (void)hipMalloc(&c, 128);
    double h[640];
    unsigned s = 12345;
    for (int i = 0; i < 640; i++) { s = s * 1103515245u + 12345u; h[i] = ((s >> 8) & 0xffff) / 65536.0 - 0.5; }
    (void)hipMemcpy(q, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, q, o, c);
        long long hc[8]; (void)hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("five_point cycles %lld (models %lld): basis %lld, AA %lld, Gauss-Jordan %lld, det poly %lld, roots %lld, E %lld\n",
               hc[0], hc[1], hc[2], hc[3], hc[4], hc[5], hc[6], hc[7]);
    }
    return 0;
}
