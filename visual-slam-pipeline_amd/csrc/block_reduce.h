// block_reduce.h — deterministic workgroup sums for the one-workgroup-per-problem solvers
// (optimize.hip, pnp.hip).  256 lanes = 4 wave64s.
#pragma once

#include <hip/hip_runtime.h>

namespace vs {

// Sum of N doubles per lane over NW wave64s: xor-shuffle tree inside each wave, then the wave
// partials in a fixed order.  Every lane receives the totals in out[].  s_red holds NW * N doubles.
template <int N, int NW = 4>
__device__ inline void block_sum(double (&v)[N], double* s_red, double (&out)[N]) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < N; k++) {
        double x = v[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        v[k] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < N; k++) s_red[wv * N + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; k++) {
        double s = s_red[k];
#pragma unroll
        for (int w = 1; w < NW; w++) s += s_red[w * N + k];
        out[k] = s;
    }
    __syncthreads();
}

}  // namespace vs
