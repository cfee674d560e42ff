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

// The same totals as block_sum (bit for bit), delivered to thread 0 only, for N <= 32 terms.  The
// in-wave butterfly is transposed: at the xor-32 step a lane keeps half of the (padded) 32 terms and
// sends the other half to its partner, at xor-16 a quarter, ... so a wave exchanges 16 + 8 + 4 + 2 +
// 1 + 1 values instead of 6 N.  Every partial sum is the one block_sum forms (the same lane groups
// are added level by level; a two-operand add is commutative), so the result is identical.  After
// the reduction lane l holds term l >> 1; the wave partials are added in wave order by thread 0.
// s_red holds NW * N doubles; contains one barrier.
template <int N, int NW = 4>
__device__ inline void block_sum_to0(const double (&v)[N], double* s_red, double (&out)[N]) {
    static_assert(N <= 32, "block_sum_to0: at most 32 terms");
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double x[32];
#pragma unroll
    for (int k = 0; k < 32; k++) x[k] = k < N ? v[k] : 0.0;
#pragma unroll
    for (int m = 32, h = 16; m >= 2; m >>= 1, h >>= 1) {
        const bool hi = (lane & m) != 0;
#pragma unroll
        for (int j = 0; j < h; j++) {
            const double keep = hi ? x[j + h] : x[j], send = hi ? x[j] : x[j + h];
            x[j] = keep + __shfl_xor(send, m);
        }
    }
    x[0] += __shfl_xor(x[0], 1);
    if ((lane & 1) == 0 && (lane >> 1) < N) s_red[wv * N + (lane >> 1)] = x[0];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < N; k++) {
            double s = s_red[k];
#pragma unroll
            for (int w = 1; w < NW; w++) s += s_red[w * N + k];
            out[k] = s;
        }
    }
}

}  // namespace vs
