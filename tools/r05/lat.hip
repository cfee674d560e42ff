// fp64 dependent-latency probe (round 5): one wave, lane-0 clock64 around 256-long dependent chains
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* io, long long* cyc) {
    double x = io[threadIdx.x], y = io[64 + threadIdx.x];
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 256; i++) x = x * y + 0.25;  // mul then add (contract off): 2 dependent ops
    long long t1 = clock64();
#pragma unroll 1
    for (int i = 0; i < 256; i++) x = sqrt(x + 1.0);
    long long t2 = clock64();
#pragma unroll 1
    for (int i = 0; i < 256; i++) x = y / (x + 1.0);
    long long t3 = clock64();
    double z = x;
#pragma unroll 1
    for (int i = 0; i < 256; i++) z = __builtin_fma(z, y, 0.25);
    long long t4 = clock64();
    float f = (float)z;
#pragma unroll 1
    for (int i = 0; i < 256; i++) f = f * 0.999f + 0.25f;
    long long t5 = clock64();
    io[threadIdx.x] = x + z + f;
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; cyc[4] = t5 - t4;
    }
}
int main() {
    double* io; long long* c;
    hipMalloc(&io, 128 * 8); hipMalloc(&c, 64);
    double h[128]; for (int i = 0; i < 128; i++) h[i] = 0.5 + i * 1e-3;
    hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, io, c);
        long long hc[5]; hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
        printf("per iteration cycles: mul+add %.1f  sqrt(+1) %.1f  div(+1) %.1f  fma %.1f  f32 mul+add %.1f\n",
               hc[0] / 256.0, hc[1] / 256.0, hc[2] / 256.0, hc[3] / 256.0, hc[4] / 256.0);
    }
    // wall-clock vs clock64 rate
    return 0;
}
