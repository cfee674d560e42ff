// Round-5 probe: the band Cholesky's 1/sqrt(x) without the range scaling of the compiler's sqrt and
// division expansions (ba.hip recip_sqrt_rn) against the compiler's 1.0 / sqrt(x), bit for bit, over
// random x in [2^-700, 2^700] (log-uniform) and near-1 / near-pivot ranges.  Prints the mismatch count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
__device__ __forceinline__ double recip_sqrt_rn(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    const double s = fma(d, h, g);
    double z = __builtin_amdgcn_rcp(s);
    double e = fma(-s, z, 1.0);
    z = fma(z, e, z);
    e = fma(-s, z, 1.0);
    z = fma(z, e, z);
    const double rr = fma(-s, z, 1.0);
    return fma(rr, z, z);
}
__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__global__ void k(uint64_t seed, long per, unsigned long long* bad, double* ex) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long nb = 0;
    for (long i = 0; i < per; i++) {
        const uint64_t u = mix(seed + (uint64_t)(t * per + i));
        double x;
        const int mode = (int)(u & 3);
        if (mode == 0) x = ldexp(1.0 + (double)(u >> 12) * 0x1p-52, (int)((u >> 2) % 1400) - 700);  // log-uniform
        else if (mode == 1) x = 1.0 + (double)(u >> 11) * 0x1p-53;                               // [1, 2)
        else if (mode == 2) x = ldexp(1.0 + (double)(u >> 12) * 0x1p-52, (int)((u >> 2) % 80) - 52); // pivots
        else x = __longlong_as_double((long long)((u >> 2) & 0x000fffffffffffffull) | 0x3ff0000000000000ll) * ldexp(1.0, (int)((u >> 54) % 60) - 30);
        const double a = recip_sqrt_rn(x), b = 1.0 / sqrt(x);
        if (__double_as_longlong(a) != __double_as_longlong(b)) {
            nb++;
            ex[0] = x;
        }
    }
    if (nb) atomicAdd(bad, nb);
}
int main() {
    unsigned long long* bad; double* ex;
    (void)hipMalloc(&bad, 8); (void)hipMalloc(&ex, 8);
    (void)hipMemset(bad, 0, 8); (void)hipMemset(ex, 0, 8);
    const long blocks = 4096, threads = 256, per = 512;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, 12345ull, per, bad, ex);
    unsigned long long h; double hx;
    (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost); (void)hipMemcpy(&hx, ex, 8, hipMemcpyDeviceToHost);
    printf("tested %ld values, mismatches %llu (example x = %.17g)\n", blocks * threads * per, h, hx);
    return h != 0;
}
