// match.hip — Slam::match_features for float descriptors on gfx950 (reference src/Slam.cpp:1140-1172).
//
// Exact L2 2-NN + Lowe ratio test.  The reference's FLANN kd-tree search is approximate; the
// exact 2-NN it approximates is the only definable semantics (DESIGN.md "Matching"):
//   dot(q, t) on the fp32 matrix cores: v_mfma_f32_32x32x2_f32 accumulates k = 2s, 2s+1 per
//   instruction as a k-ordered fp32 fmaf chain, so chaining s = 0..127 gives exactly the
//   sequential fmaf chain over k = 0..255 that the CPU oracle computes;
//   d2 = max((na + nb) - 2*dot, 0) with the row norms as sequential fmaf chains;
//   best / second = the two smallest (d2, train index) pairs; distance = sqrtf(d2);
//   good iff sqrtf(d0) < ratio * sqrtf(d1).
// Pair lists are therefore bit-identical to the oracle.
//
// Mapping: A operand = 32 train rows (M), B operand = 32 query rows (N).  A workgroup owns 128
// query rows (one 32-row N block per wave, its K = 256 values held in 128 VGPRs) and one slice of
// 64 train rows staged through LDS (k-major, conflict free); the grid is pairs x query blocks x
// train slices, so even a single pair spreads over tens of CUs.  The accumulator puts one query
// per lane and 16 train rows per register set, so the slice's top-2 is per-lane register work,
// merged with the partner half-wave by one shuffle.  The compaction kernel merges the slices'
// top-2 per query (a total order on (d2, train index), so the merge order cannot matter), then
// applies the ratio test and compacts in query order.
#include <hip/hip_runtime.h>

#include <climits>

#include "vs_internal.h"

namespace vs {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Best2 {
    float d0, d1;
    int j0, j1;
    __device__ void init() {
        d0 = d1 = __int_as_float(0x7f800000);
        j0 = j1 = INT_MAX;
    }
    __device__ void push(float d, int j) {
        if (d < d0 || (d == d0 && j < j0)) {
            d1 = d0; j1 = j0; d0 = d; j0 = j;
        } else if (d < d1 || (d == d1 && j < j1)) {
            d1 = d; j1 = j;
        }
    }
};

// Sequential fmaf-chain squared norm of every descriptor row of F frames.
__global__ __launch_bounds__(256) void k_desc_norms(const float* __restrict__ desc, const int* __restrict__ n,
                                                    int F, int cap, float* __restrict__ norms) {
    long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= (long)F * cap) return;
    int f = (int)(r / cap), i = (int)(r - (long)f * cap);
    if (i >= n[f]) return;
    const float4* p = reinterpret_cast<const float4*>(desc + (size_t)r * 256);
    float s = 0.0f;
    for (int k4 = 0; k4 < 64; k4++) {
        float4 v = p[k4];
        s = fmaf(v.x, v.x, s);
        s = fmaf(v.y, v.y, s);
        s = fmaf(v.z, v.z, s);
        s = fmaf(v.w, v.w, s);
    }
    norms[r] = s;
}

constexpr int kTrainChunk = 64;

struct Part2 {  // a train slice's top-2 for one query
    float d0, d1;
    int j0, j1;
};

__global__ __launch_bounds__(256) void k_match(const int* __restrict__ pairs, const float* __restrict__ descq,
                                               const float* __restrict__ desct, const float* __restrict__ normsq,
                                               const float* __restrict__ normst, const int* __restrict__ n,
                                               int qstride, int tstride, int cap, int nslices,
                                               Part2* __restrict__ part) {
    __shared__ float s_t[256 * kTrainChunk];  // [k][m]
    __shared__ float s_nb[kTrainChunk];
    const int p = blockIdx.x;
    const int qf = pairs[2 * p], tf = pairs[2 * p + 1];
    const int n1 = n[qf], n2 = n[tf];
    const int q0 = blockIdx.y * 128, t0 = blockIdx.z * kTrainChunk;
    if (q0 >= n1 || n2 < 2 || t0 >= n2) return;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
    const int qj = q0 + wv * 32 + li;
    const bool qvalid = qj < n1;
    const float* T = desct + (size_t)tf * tstride * 256;
    // stage the slice's train rows, k-major; lanes walk rows so LDS writes are conflict free
    for (int idx = tid; idx < kTrainChunk * 64; idx += 256) {
        int m = idx & (kTrainChunk - 1), k4 = idx / kTrainChunk;
        float4 v = {0.f, 0.f, 0.f, 0.f};
        if (t0 + m < n2) v = reinterpret_cast<const float4*>(T + (size_t)(t0 + m) * 256)[k4];
        s_t[(4 * k4 + 0) * kTrainChunk + m] = v.x;
        s_t[(4 * k4 + 1) * kTrainChunk + m] = v.y;
        s_t[(4 * k4 + 2) * kTrainChunk + m] = v.z;
        s_t[(4 * k4 + 3) * kTrainChunk + m] = v.w;
    }
    if (tid < kTrainChunk) s_nb[tid] = (t0 + tid < n2) ? normst[(size_t)tf * tstride + t0 + tid] : 0.0f;
    const float* Q = descq + ((size_t)qf * qstride + (qvalid ? qj : 0)) * 256;
    float qreg[128];
    const bool wlive = q0 + wv * 32 < n1;  // wave-uniform
#pragma unroll
    for (int s = 0; s < 128; s++) qreg[s] = (qvalid && wlive) ? Q[2 * s + lh] : 0.0f;
    const float na = qvalid ? normsq[(size_t)qf * qstride + qj] : 0.0f;
    __syncthreads();
    // padding is not computed: a wave whose 32 queries are all past n1 leaves (no barrier follows),
    // and the upper 32 train rows of a slice are skipped when all of them are past n2
    if (q0 + wv * 32 >= n1) return;
    Best2 best;
    best.init();
    f32x16 acc0, acc1;
#pragma unroll
    for (int e = 0; e < 16; e++) acc0[e] = acc1[e] = 0.0f;
    if (t0 + 32 < n2) {
#pragma unroll
        for (int s = 0; s < 128; s++) {
            const float a0 = s_t[(2 * s + lh) * kTrainChunk + li];
            const float a1 = s_t[(2 * s + lh) * kTrainChunk + 32 + li];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, qreg[s], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, qreg[s], acc1, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int s = 0; s < 128; s++) {
            const float a0 = s_t[(2 * s + lh) * kTrainChunk + li];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, qreg[s], acc0, 0, 0, 0);
        }
    }
    // C/D: col = query (lane&31), row = train (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
        const int mr = (reg & 3) + 8 * (reg >> 2) + 4 * lh;
        if (t0 + mr < n2) {
            float s = na + s_nb[mr];
            float d = s - 2.0f * acc0[reg];
            best.push(d < 0.0f ? 0.0f : d, t0 + mr);
        }
        if (t0 + 32 + mr < n2) {
            float s = na + s_nb[32 + mr];
            float d = s - 2.0f * acc1[reg];
            best.push(d < 0.0f ? 0.0f : d, t0 + 32 + mr);
        }
    }
    // merge the two half-waves that saw disjoint train rows of the same query
    Best2 other;
    other.d0 = __shfl_xor(best.d0, 32);
    other.d1 = __shfl_xor(best.d1, 32);
    other.j0 = __shfl_xor(best.j0, 32);
    other.j1 = __shfl_xor(best.j1, 32);
    best.push(other.d0, other.j0);
    best.push(other.d1, other.j1);
    if (lh == 0 && qvalid) part[((size_t)p * nslices + blockIdx.z) * cap + qj] = {best.d0, best.d1, best.j0, best.j1};
}

// Per query: merge the train slices' top-2, distance = sqrtf(d2), ratio test (Slam.cpp:1151-1157);
// then the order-preserving compaction of the good rows (query order).
__global__ __launch_bounds__(1024) void k_match_compact(const int* __restrict__ pairs, const int* __restrict__ n,
                                                        int cap, int nslices, float ratio,
                                                        const Part2* __restrict__ part, vs_match* __restrict__ raw,
                                                        int* __restrict__ nraw, vs_match* __restrict__ good,
                                                        int* __restrict__ ngood) {
    __shared__ int s_wave[16];
    __shared__ int s_base;
    const int p = blockIdx.x;
    const int n1 = n[pairs[2 * p]], n2 = n[pairs[2 * p + 1]];
    const int rows = (n2 >= 2) ? n1 : 0;
    const int used = (n2 + kTrainChunk - 1) / kTrainChunk;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    for (int c0 = 0; c0 < rows; c0 += 1024) {
        const int i = c0 + threadIdx.x;
        bool f = false;
        vs_match m;
        if (i < rows) {
            Best2 best;
            best.init();
            for (int z = 0; z < used; z++) {
                const Part2 q = part[((size_t)p * nslices + z) * cap + i];
                best.push(q.d0, q.j0);
                best.push(q.d1, q.j1);
            }
            const float dist0 = sqrt_rn(best.d0), dist1 = sqrt_rn(best.d1);
            m.query_idx = i;
            m.train_idx = best.j0;
            m.img_idx = 0;
            m.distance = dist0;
            raw[(size_t)p * cap + i] = m;
            f = dist0 < ratio * dist1;
        }
        const unsigned long long bal = __ballot(f);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) s_wave[wv] = __popcll(bal);
        __syncthreads();
        int off = s_base;
        for (int k = 0; k < wv; k++) off += s_wave[k];
        if (f) good[(size_t)p * cap + off + before] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int k = 0; k < 16; k++) tot += s_wave[k];
            s_base += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        nraw[p] = rows;
        ngood[p] = s_base;
    }
}

// Norms of only the frames the P pairs reference (a pair out of a large frame pool): row r of
// the 2P*cap grid is row r % cap of frame pairs[r / cap]; a frame named twice is written twice
// with the same value.
__global__ __launch_bounds__(256) void k_desc_norms_sel(const float* __restrict__ desc, const int* __restrict__ n,
                                                        const int* __restrict__ pairs, int P, int cap,
                                                        float* __restrict__ norms) {
    long r = (long)blockIdx.x * 256 + threadIdx.x;
    if (r >= (long)2 * P * cap) return;
    const int f = pairs[r / cap], i = (int)(r % cap);
    if (i >= n[f]) return;
    const float4* p = reinterpret_cast<const float4*>(desc + ((size_t)f * cap + i) * 256);
    float s = 0.0f;
    for (int k4 = 0; k4 < 64; k4++) {
        float4 v = p[k4];
        s = fmaf(v.x, v.x, s);
        s = fmaf(v.y, v.y, s);
        s = fmaf(v.z, v.z, s);
        s = fmaf(v.w, v.w, s);
    }
    norms[(size_t)f * cap + i] = s;
}

__global__ void k_set_meta(int* meta, int n1, int n2) {
    meta[0] = 0;  // pairs = {0, 1}
    meta[1] = 1;
    meta[2] = n1;  // n = {n1, n2}
    meta[3] = n2;
}

int desc_norms(vs_ctx* ctx, int F, const float* d_desc, const int* d_n, int cap, float* d_norms, hipStream_t s) {
    (void)ctx;
    const long rows = (long)F * cap;
    if (rows <= 0) return VS_OK;
    hipLaunchKernelGGL(k_desc_norms, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, d_desc, d_n, F, cap, d_norms);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int match_pairs(vs_ctx* ctx, int P, const int* d_pairs, int F, const float* d_desc, const int* d_n, int cap,
                float ratio, vs_match* d_raw, int* d_nraw, vs_match* d_good, int* d_ngood, hipStream_t s,
                const float* d_norms) {
    if (P <= 0) return VS_OK;
    const int nslices = (cap + kTrainChunk - 1) / kTrainChunk;
    const size_t norm_bytes = ((size_t)F * cap * sizeof(float) + 255) & ~(size_t)255;
    VS_CHECK(ctx->norms.ensure(norm_bytes + (size_t)P * nslices * cap * sizeof(Part2)));
    float* norms = ctx->norms.as<float>();
    Part2* part = reinterpret_cast<Part2*>(ctx->norms.as<uint8_t>() + norm_bytes);
    ProfScope ps(ctx, "match", s);
    if (d_norms) {  // the caller keeps the frames' row norms
        norms = const_cast<float*>(d_norms);
    } else if (2 * P < F) {  // a few pairs out of a frame pool: only the referenced frames' norms
        long rows = (long)2 * P * cap;
        hipLaunchKernelGGL(k_desc_norms_sel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, d_desc, d_n,
                           d_pairs, P, cap, norms);
    } else {
        long rows = (long)F * cap;
        hipLaunchKernelGGL(k_desc_norms, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, d_desc, d_n, F, cap,
                           norms);
    }
    hipLaunchKernelGGL(k_match, dim3(P, (cap + 127) / 128, nslices), dim3(256), 0, s, d_pairs, d_desc, d_desc, norms,
                       norms, d_n, cap, cap, cap, nslices, part);
    hipLaunchKernelGGL(k_match_compact, dim3(P), dim3(1024), 0, s, d_pairs, d_n, cap, nslices, ratio, part, d_raw,
                       d_nraw, d_good, d_ngood);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

// One query set against one train set held in separate arrays (PnP recovery: a frame's
// descriptors against every valid map point, Slam.cpp:560-575).  Outputs are indexed by query
// row (d_raw / d_good have n1 entries); d_counts = {n_raw, n_good}.
int match_sets(vs_ctx* ctx, const float* d_q, int n1, const float* d_t, int n2, float ratio, vs_match* d_raw,
               vs_match* d_good, int* d_counts, hipStream_t s) {
    if (n1 <= 0) return VS_OK;
    const int nslices = (n2 + kTrainChunk - 1) / kTrainChunk;
    const size_t head = (((size_t)n1 + n2) * sizeof(float) + 4 * sizeof(int) + 255) & ~(size_t)255;
    VS_CHECK(ctx->norms_sets.ensure(head + (size_t)(nslices > 0 ? nslices : 1) * n1 * sizeof(Part2)));
    float* nq = ctx->norms_sets.as<float>();
    float* nt = nq + n1;
    int* meta = reinterpret_cast<int*>(nt + n2);
    Part2* part = reinterpret_cast<Part2*>(ctx->norms_sets.as<uint8_t>() + head);
    ProfScope ps(ctx, "match_map", s);
    hipLaunchKernelGGL(k_set_meta, dim3(1), dim3(1), 0, s, meta, n1, n2);
    // norms: query rows as "frame 0" of stride n1, train rows as "frame 1" read with stride 0
    hipLaunchKernelGGL(k_desc_norms, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, s, d_q, meta + 2, 1, n1, nq);
    if (n2 > 0)
        hipLaunchKernelGGL(k_desc_norms, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, s, d_t, meta + 3, 1, n2,
                           nt);
    if (nslices > 0)
        hipLaunchKernelGGL(k_match, dim3(1, (n1 + 127) / 128, nslices), dim3(256), 0, s, meta, d_q, d_t, nq, nt,
                           meta + 2, n1, 0, n1, nslices, part);
    hipLaunchKernelGGL(k_match_compact, dim3(1), dim3(1024), 0, s, meta, meta + 2, n1, nslices, ratio, part, d_raw,
                       d_counts, d_good, d_counts + 1);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
