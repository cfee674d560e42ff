// Single-lane latency of the correctly rounded fp64 functions (csrc/cr_math.h) on gfx950: N
// dependent calls timed with clock64 (s_memtime) on lane 0, printed as cycles per call.
//   hipcc -O3 --offload-arch=gfx950 -I visual-slam-pipeline_amd/csrc tools/crmath_latency.hip -o /tmp/crlat
#include <hip/hip_runtime.h>

#include <cstdio>

#include "cr_math.h"

__global__ void k_lat(int op, int n, double x0, double* out, long long* cyc) {
    double x = x0, acc = 0;
    const long long t0 = clock64();
    for (int i = 0; i < n; i++) {
        double r;
        switch (op) {
            case 0: r = vs_cr::sin(x); break;
            case 1: r = vs_cr::cos(x); break;
            case 2: r = vs_cr::acos(x * 0.5); break;
            case 3: r = vs_cr::log(x + 1.5); break;
            default: r = vs_cr::pow(x * 0.5 + 0.25, 5.0); break;
        }
        acc += r;
        x = 0.3 + 1e-3 * r;  // dependent chain
    }
    cyc[op] = clock64() - t0;
    out[op] = acc;
}

int main() {
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, 8 * sizeof(double));
    (void)hipMalloc(&cyc, 8 * sizeof(long long));
    const char* names[5] = {"sin", "cos", "acos", "log", "pow"};
    const int n = 200;
    for (int op = 0; op < 5; op++) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, op, n, 0.7, out, cyc);
        (void)hipDeviceSynchronize();
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, op, n, 0.7, out, cyc);
        long long c[8];
        (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
        std::printf("%-5s %8.0f cycles per call\n", names[op], (double)c[op] / n);
    }
    return 0;
}
