// match.hip — Slam::match_features for float descriptors on gfx950 (reference src/Slam.cpp:1140-1172).
//
// Exact L2 2-NN + Lowe ratio test.  The reference's FLANN kd-tree search is approximate; the
// exact 2-NN it approximates is the only definable semantics (DESIGN.md "Matching"):
//   dot(q, t) on the fp32 matrix cores: v_mfma_f32_16x16x4_f32 accumulates k = 4s .. 4s+3 per
//   instruction as a k-ordered fp32 fmaf chain, so chaining s = 0..63 gives exactly the
//   sequential fmaf chain over k = 0..255 that the CPU oracle computes;
//   d2 = max((na + nb) - 2*dot, 0) with the row norms as sequential fmaf chains;
//   best / second = the two smallest (d2, train index) pairs; distance = sqrtf(d2);
//   good iff sqrtf(d0) < ratio * sqrtf(d1).
// Pair lists are therefore bit-identical to the oracle.
//
// One launch per call (any number of pairs):
//   * grid = pairs x query blocks x train blocks, linearised so that the 8-block round-robin XCD
//     placement gives each XCD a contiguous range of pairs (one pair's descriptors stay in one L2);
//   * a workgroup (4 waves, 2 x 2) owns 2WQ queries x 2WT train rows and stages them through LDS in
//     k-chunks of 64 with one-chunk register prefetch: coalesced 16 B global loads of 16
//     consecutive k per thread, a 4 x 4 register transpose, and 16 B LDS stores into rows padded to
//     72 floats, so every MFMA fragment (lane i, k-group g) is one conflict-free ds_read_b128 that
//     carries four consecutive MFMA steps;
//   * each wave chains (WQ/16) x (WT/16) independent 16x16 accumulators over the 64 steps (the
//     16x16x4 MFMA issues every 32 cycles with a 40-cycle dependent latency, so >= 2 chains per
//     wave, or >= 2 waves per SIMD, keep the matrix pipe busy);
//   * row norms: either the caller's (computed once per frame) or sequential fmaf chains over the
//     staged chunks, one thread per row, interleaved with the MFMAs;
//   * the per-query top-2 of a wave is merged across train blocks with 64-bit atomicMin on keys
//     (d2 bits << 32 | train index; d2 >= +0 so the bits order like the floats, and the index
//     breaks ties toward the lower index): best0 keeps the minimum and the key it displaces (or
//     the rejected candidate) goes to best1, so best1 ends as the minimum over everything except
//     best0 — the exact top-2 of the union, independent of arrival order;
//   * the last workgroup of a pair to arrive (a device-scope counter; every atomic of the earlier
//     workgroups has returned before their arrival) reads and resets the keys with atomicExch,
//     applies the ratio test and compacts the good rows in query order: NTH queries per pass,
//     per-wave ballots and one barrier per pass (several chunks per pass raised the whole kernel's
//     VGPR count and cost the 64 x 64 main loop an occupancy step).  Keys and counters are left
//     reset for the next launch.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "vs_internal.h"

namespace vs {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// f(integral_constant<int, I>) for I = B .. E-1, unrolled at compile time
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

constexpr unsigned long long kNoKey = ~0ull;
constexpr int kTailChunks = 1;  // last arrival: query chunks of NTH per pass (more raise the kernel's VGPR count)

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

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const unsigned lo = __shfl_xor((unsigned)v, m), hi = __shfl_xor((unsigned)(v >> 32), m);
    return ((unsigned long long)hi << 32) | lo;
}

// top-2 of a set of distinct keys (k0 < k1), branch-free
__device__ __forceinline__ void push2(unsigned long long& k0, unsigned long long& k1, unsigned long long k) {
    const unsigned long long lo = k < k0 ? k : k0, hi = k < k0 ? k0 : k;
    k1 = hi < k1 ? hi : k1;
    k0 = lo;
}

struct MatchArgs {
    const int* pairs;      // [P][2] (query frame, train frame)
    const float* descq;    // query frames, row stride 256 floats, frame stride qstride rows
    const float* desct;    // train frames (tstride 0: one set)
    const float* normsq;   // optional caller norms, same indexing as the rows
    const float* normst;
    const int* n;          // rows per frame
    int qstride, tstride;
    int qblocks, tblocks;  // grid extents per pair (capacity)
    int qfull, tfull;      // blocks whole at capacity (largest-first order; 0: pair-major order)
    int npairs;
    int work, per_xcd;     // P * qblocks * tblocks; blocks per XCD range
    float ratio;
    unsigned long long* keys;  // [P][2][kcap]
    int kcap;
    unsigned* cnt;             // [P] arrival counters
    vs_match* raw;             // [P][ostride]
    int* nraw;
    vs_match* good;
    int* ngood;
    int ostride;
};

// Workgroup = NWQ x NWT waves, each owning WQ queries x WT train rows (FQ x FT 16 x 16 MFMA
// chains), so a workgroup covers TQ = NWQ WQ queries x TT = NWT WT train rows.
// ABL: phase ablation for latency studies (VS_MATCH_ABLATE; results are not matches): 0 = the
// product kernel, 1 = stop after the k-loop, 2 = no MFMAs in the k-loop, 3 = stop after the
// prologue's first chunk.
template <int NWQ, int NWT, int WQ, int WT, int KC, int NBUF, int PD, bool NORMS, int ABL = 0>
__global__ __launch_bounds__(64 * NWQ * NWT) void k_match(MatchArgs a) {
    constexpr int NW = NWQ * NWT, NTH = 64 * NW;
    constexpr int TQ = NWQ * WQ, TT = NWT * WT, R = TQ + TT;
    constexpr int FQ = WQ / 16, FT = WT / 16;
    constexpr int NC = 256 / KC;           // staged chunks
    constexpr int NB = NC > 1 ? NBUF : 1;  // LDS buffers (1: a second barrier per chunk, half the LDS)
    constexpr int RS4 = KC / 4 + 2;        // row stride in float4 (KC + 8 floats)
    constexpr int GR = KC / 16;            // 16-k groups per row and chunk
    constexpr int GPT = (R * GR + NTH - 1) / NTH;  // groups per thread and chunk (the last may be partial)
    constexpr bool GPART = GPT * NTH != R * GR;
    constexpr int NR = R / NW;             // norm rows per wave
    static_assert(NR * NW == R && NR <= 64, "norm split");
    __shared__ float4 sbuf[NB][R * RS4];
    __shared__ float s_norm[R];
    __shared__ unsigned long long s_top[NWT > 1 ? NWT : 1][TQ][2];
    __shared__ int s_cnt[kTailChunks][NW];
    __shared__ int s_last;

    // linear work index: XCD x (= blockIdx % 8 under round-robin placement) takes a contiguous range
    const int L = (blockIdx.x & 7) * a.per_xcd + (blockIdx.x >> 3);
    if (L >= a.work) return;
    // largest first (round 5): the workgroups whose tiles are whole at capacity come first, pair by
    // pair, and the edge tiles (the last query / train block of a 400-row frame holds 16 rows) after
    // them, so that the grid's last dispatch wave is made of short workgroups and the launch's tail is
    // shorter; a.qfull / a.tfull = 0 keeps the plain pair-major order
    const int per_pair = a.qblocks * a.tblocks;
    int p, qb, tb;
    const int nfull = a.qfull * a.tfull;
    if (nfull == 0) {
        p = L / per_pair;
        const int r0 = L - p * per_pair;
        qb = r0 / a.tblocks, tb = r0 - qb * a.tblocks;
    } else if (L < a.npairs * nfull) {
        p = L / nfull;
        const int r0 = L - p * nfull;
        qb = r0 / a.tfull, tb = r0 - qb * a.tfull;
    } else {
        const int edges = per_pair - nfull, L2 = L - a.npairs * nfull;
        p = L2 / edges;
        const int e = L2 - p * edges, rows = (a.qblocks - a.qfull) * a.tblocks;
        if (e < rows) {
            qb = a.qfull + e / a.tblocks, tb = e - (e / a.tblocks) * a.tblocks;
        } else {
            const int e2 = e - rows, tw = a.tblocks - a.tfull;
            qb = e2 / tw, tb = a.tfull + e2 - (e2 / tw) * tw;
        }
    }
    const int qf = a.pairs[2 * p], tf = a.pairs[2 * p + 1];
    const int n1 = a.n[qf], n2 = a.n[tf];
    const int tid = threadIdx.x;
    if (n1 <= 0 || n2 < 2) {  // empty Mat / fewer than k = 2 neighbours: no matches (Slam.cpp:1151-1153)
        if (qb == 0 && tb == 0 && tid == 0) {
            a.nraw[p] = 0;
            a.ngood[p] = 0;
        }
        return;
    }
    const int nq = (n1 + TQ - 1) / TQ, nt = (n2 + TT - 1) / TT;
    if (qb >= nq || tb >= nt) return;
    const int q0 = qb * TQ, t0 = tb * TT;
    const float* Q = a.descq + (size_t)qf * a.qstride * 256;
    const float* T = a.desct + (size_t)tf * a.tstride * 256;

    // staging: group G = tid + NTH u -> LDS row G / GR, 16 consecutive k at (G % GR) * 16 of the
    // chunk.  Rows past n1 / n2 re-read the last valid row (their results are never used), so every
    // load is unconditional and the compiler keeps all of them in flight together.
    const float4* src[GPT];
#pragma unroll
    for (int u = 0; u < GPT; u++) {
        const int G = min(tid + NTH * u, R * GR - 1), row = G / GR, q4 = G % GR;
        const float* base = row < TQ ? Q + (size_t)min(q0 + row, n1 - 1) * 256
                                     : T + (size_t)min(t0 + row - TQ, n2 - 1) * 256;
        src[u] = reinterpret_cast<const float4*>(base) + 4 * q4;
    }
    // PD chunks in flight in registers (slot c % PD holds chunk c): PD = 1 overlaps one chunk's
    // loads with the previous chunk's MFMAs; PD = NC issues every load of the tile up front
    // (compile-time chunk indices throughout — static_for — so the ring stays in registers).
    float4 reg[PD][GPT][4];
    auto load = [&](auto cc) {
        constexpr int c = decltype(cc)::value;
#pragma unroll
        for (int u = 0; u < GPT; u++)
#pragma unroll
            for (int j = 0; j < 4; j++) reg[c % PD][u][j] = src[u][(KC / 4) * c + j];
    };
    // position 4g + j of a 16-k group holds k = 4j + g: the fragment of lane group g is one float4
    auto store = [&](auto cc, int buf) {
        constexpr int c = decltype(cc)::value;
        const float4(&r)[GPT][4] = reg[c % PD];
#pragma unroll
        for (int u = 0; u < GPT; u++) {
            const int G = tid + NTH * u, row = G / GR, q4 = G % GR;
            if (GPART && u == GPT - 1 && G >= R * GR) continue;  // (loaded a duplicate group; not stored)
            float4* d = &sbuf[buf][row * RS4 + 4 * q4];
            d[0] = make_float4(r[u][0].x, r[u][1].x, r[u][2].x, r[u][3].x);
            d[1] = make_float4(r[u][0].y, r[u][1].y, r[u][2].y, r[u][3].y);
            d[2] = make_float4(r[u][0].z, r[u][1].z, r[u][2].z, r[u][3].z);
            d[3] = make_float4(r[u][0].w, r[u][1].w, r[u][2].w, r[u][3].w);
        }
    };

    const int wv = tid >> 6, lane = tid & 63, li = lane & 15, lg = lane >> 4;
    const int wq = wv % NWQ, wt = wv / NWQ;
    const int qrow0 = wq * WQ, trow0 = TQ + wt * WT;  // LDS rows of this wave's fragments
    // fragments entirely past n1 / n2 are not computed (wave-uniform)
    bool vq[FQ], vt[FT];
#pragma unroll
    for (int y = 0; y < FQ; y++) vq[y] = q0 + qrow0 + 16 * y < n1;
#pragma unroll
    for (int x = 0; x < FT; x++) vt[x] = t0 + wt * WT + 16 * x < n2;
    const bool full = q0 + qrow0 + WQ <= n1 && t0 + wt * WT + WT <= n2;
    f32x4 acc[FT][FQ];
#pragma unroll
    for (int x = 0; x < FT; x++)
#pragma unroll
        for (int y = 0; y < FQ; y++) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    // NORMS == false: lane < NR of each wave chains the squared norm of LDS row wv * NR + lane (the
    // same share per wave, so no wave reaches the chunk barrier late)
    const int nrow = wv * NR + lane;
    const bool nthread = !NORMS && lane < NR;
    float nrm = 0.0f;

    // caller's norms: loaded before the staging loads, stored to LDS after them (vmcnt is in order)
    float cnorm = 0.0f;
    if (NORMS && tid < R) {
        const float* nsrc = tid < TQ ? a.normsq + (size_t)qf * a.qstride + min(q0 + tid, n1 - 1)
                                     : a.normst + (size_t)tf * a.tstride + min(t0 + tid - TQ, n2 - 1);
        cnorm = *nsrc;
    }
    static_for<0, (PD < NC ? PD : NC)>([&](auto cc) { load(cc); });
    store(std::integral_constant<int, 0>{}, 0);
    if (NORMS && tid < R) s_norm[tid] = cnorm;
    __syncthreads();
    if constexpr (ABL == 3) {
        if (sbuf[0][tid].x == 1234.5f) a.raw[0].distance = sbuf[0][tid].y;
        return;
    }
    static_for<0, NC>([&](auto cc) {  // unrolled: no loop-carried copies of the prefetch registers
        constexpr int c = decltype(cc)::value;
        const int buf = NB > 1 ? (c & 1) : 0;
        if constexpr (c + PD < NC) load(std::integral_constant<int, c + PD>{});
        // keep the transposing register moves of store() below the MFMAs: hoisted here they would
        // wait for the loads just issued
        __builtin_amdgcn_sched_barrier(0);
        const float4* sb = sbuf[buf];
#pragma unroll
        for (int qd = 0; qd < KC / 16; qd++) {
            float4 fa[FT], fb[FQ];
#pragma unroll
            for (int x = 0; x < FT; x++) fa[x] = sb[(trow0 + 16 * x + li) * RS4 + 4 * qd + lg];
#pragma unroll
            for (int y = 0; y < FQ; y++) fb[y] = sb[(qrow0 + 16 * y + li) * RS4 + 4 * qd + lg];
            // all fragments valid (every interior workgroup): straight-line MFMAs; else per-fragment
            if constexpr (ABL == 2) {
#pragma unroll
                for (int x = 0; x < FT; x++)
#pragma unroll
                    for (int y = 0; y < FQ; y++) acc[x][y][0] += fa[x][0] * fb[y][0];
            } else if (full) {
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int x = 0; x < FT; x++)
#pragma unroll
                        for (int y = 0; y < FQ; y++)
                            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[x][j], fb[y][j], acc[x][y], 0, 0, 0);
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int x = 0; x < FT; x++)
#pragma unroll
                        for (int y = 0; y < FQ; y++)
                            if (vt[x] && vq[y])
                                acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[x][j], fb[y][j], acc[x][y], 0, 0, 0);
            }
            if (nthread) {
                // k = 16 qd + m sits at float4 (m & 3), component (m >> 2)
                float4 v[4];
#pragma unroll
                for (int g = 0; g < 4; g++) v[g] = sb[nrow * RS4 + 4 * qd + g];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    nrm = fmaf(v[0][j], v[0][j], nrm);
                    nrm = fmaf(v[1][j], v[1][j], nrm);
                    nrm = fmaf(v[2][j], v[2][j], nrm);
                    nrm = fmaf(v[3][j], v[3][j], nrm);
                }
            }
        }
        if constexpr (c + 1 < NC) {
            __builtin_amdgcn_sched_barrier(0);
            if (NB == 1) __syncthreads();
            store(std::integral_constant<int, c + 1>{}, NB > 1 ? (buf ^ 1) : 0);
        } else {
            if (nthread) s_norm[nrow] = nrm;
        }
        __syncthreads();
    });
    if constexpr (ABL == 1) {
        float t = 0.0f;
#pragma unroll
        for (int x = 0; x < FT; x++)
#pragma unroll
            for (int y = 0; y < FQ; y++) t += acc[x][y][0] + acc[x][y][1] + acc[x][y][2] + acc[x][y][3];
        if (t == 1234.5f) a.raw[0].distance = t;
        return;
    }

    // ---- per-wave top-2 per query over the wave's WT train rows: D[train 4 lg + e][query li] of
    // each 16 x 16 fragment, merged over e, x and (shuffles) the lane groups; NWT > 1 merges the
    // waves of a query block through LDS ----
    unsigned long long w0[FQ], w1[FQ];
#pragma unroll
    for (int y = 0; y < FQ; y++) {
        const float na = s_norm[qrow0 + 16 * y + li];
        unsigned long long k0 = kNoKey, k1 = kNoKey;
#pragma unroll
        for (int x = 0; x < FT; x++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int tr = wt * WT + 16 * x + 4 * lg + e;  // train row within the block
                const float s = na + s_norm[TQ + tr];
                float d = s - 2.0f * acc[x][y][e];
                d = d < 0.0f ? 0.0f : d;
                const unsigned long long key = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)(t0 + tr);
                push2(k0, k1, t0 + tr < n2 ? key : kNoKey);
            }
#pragma unroll
        for (int m = 16; m <= 32; m <<= 1) {
            const unsigned long long o0 = shfl_xor_u64(k0, m), o1 = shfl_xor_u64(k1, m);
            const unsigned long long lo = k0 < o0 ? k0 : o0, hi = k0 < o0 ? o0 : k0;
            const unsigned long long m1 = k1 < o1 ? k1 : o1;
            k0 = lo;
            k1 = hi < m1 ? hi : m1;
        }
        w0[y] = k0;
        w1[y] = k1;
    }
    unsigned long long mine0 = kNoKey, mine1 = kNoKey;  // the query this thread publishes
    int ql = -1;                                        // its row within the query block
    if constexpr (NWT == 1) {
        // lane group lg publishes fragments y = lg, lg + 4, ... (one query per lane and pass)
#pragma unroll
        for (int y = 0; y < FQ; y++)
            if ((y & 3) == lg && y < 4) {
                mine0 = w0[y];
                mine1 = w1[y];
                ql = qrow0 + 16 * y + li;
            }
    } else {
        if (lg == 0) {
#pragma unroll
            for (int y = 0; y < FQ; y++) {
                s_top[wt][qrow0 + 16 * y + li][0] = w0[y];
                s_top[wt][qrow0 + 16 * y + li][1] = w1[y];
            }
        }
        __syncthreads();
        if (tid < TQ) {
            unsigned long long k0 = s_top[0][tid][0], k1 = s_top[0][tid][1];
#pragma unroll
            for (int w = 1; w < NWT; w++) {
                const unsigned long long o0 = s_top[w][tid][0], o1 = s_top[w][tid][1];
                const unsigned long long lo = k0 < o0 ? k0 : o0, hi = k0 < o0 ? o0 : k0;
                const unsigned long long m1 = k1 < o1 ? k1 : o1;
                k0 = lo;
                k1 = hi < m1 ? hi : m1;
            }
            mine0 = k0;
            mine1 = k1;
            ql = tid;
        }
    }
    unsigned long long* B0 = a.keys + (size_t)p * 2 * a.kcap;
    unsigned long long* B1 = B0 + a.kcap;
    auto publish = [&](int qloc, unsigned long long m0, unsigned long long m1) {
        const int qi = q0 + qloc;
        if (qloc >= 0 && qi < n1 && m0 != kNoKey) {
            if (m1 != kNoKey) atomicMin(B1 + qi, m1);
            const unsigned long long old = atomicMin(B0 + qi, m0);
            atomicMin(B1 + qi, old > m0 ? old : m0);
        }
    };
    publish(ql, mine0, mine1);
    if constexpr (NWT == 1 && FQ > 4) {  // fragments 4.. (one more pass)
#pragma unroll
        for (int y = 4; y < FQ; y++)
            if ((y & 3) == lg) publish(qrow0 + 16 * y + li, w0[y], w1[y]);
    }
    // every atomic of this workgroup has been performed (acknowledged) before it arrives
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(a.cnt + p, 1u) == (unsigned)(nq * nt - 1);
    __syncthreads();
    if (!s_last) return;

    // ---- last arrival: ratio test + order-preserving compaction (Slam.cpp:1151-1157) ----
    // kTailChunks x NTH queries per pass: the pass's key exchanges in flight together, per-wave
    // ballots, one barrier, then each thread's slot from the per-(chunk, wave) counts
    if (tid == 0) atomicExch(a.cnt + p, 0u);
    vs_match* raw = a.raw + (size_t)p * a.ostride;
    vs_match* good = a.good + (size_t)p * a.ostride;
    int base = 0;
    for (int c0 = 0; c0 < n1; c0 += kTailChunks * NTH) {
        unsigned long long k0[kTailChunks], k1[kTailChunks];
#pragma unroll
        for (int u = 0; u < kTailChunks; u++) {
            const int i = c0 + u * NTH + tid;
            k0[u] = k1[u] = kNoKey;
            if (i < n1) {
                k0[u] = atomicExch(B0 + i, kNoKey);
                k1[u] = atomicExch(B1 + i, kNoKey);
            }
        }
        bool f[kTailChunks];
        vs_match m[kTailChunks];
        int before[kTailChunks];
#pragma unroll
        for (int u = 0; u < kTailChunks; u++) {
            const int i = c0 + u * NTH + tid;
            f[u] = false;
            if (i < n1) {
                const float dist0 = sqrt_rn(__uint_as_float((unsigned)(k0[u] >> 32)));
                const float dist1 = sqrt_rn(__uint_as_float((unsigned)(k1[u] >> 32)));
                m[u].query_idx = i;
                m[u].train_idx = (int)(unsigned)k0[u];
                m[u].img_idx = 0;
                m[u].distance = dist0;
                raw[i] = m[u];
                f[u] = dist0 < a.ratio * dist1;
            }
            const unsigned long long bal = __ballot(f[u]);
            before[u] = __popcll(bal & ((1ull << lane) - 1ull));
            if (lane == 0) s_cnt[u][wv] = __popcll(bal);
        }
        __syncthreads();
        int run = base;
#pragma unroll
        for (int u = 0; u < kTailChunks; u++) {
            int off = run;
#pragma unroll
            for (int w = 0; w < NW; w++) {
                const int cw = s_cnt[u][w];
                off += w < wv ? cw : 0;
                run += cw;
            }
            if (f[u]) good[off + before[u]] = m[u];
        }
        base = run;
        if (c0 + kTailChunks * NTH < n1) __syncthreads();  // s_cnt is rewritten by the next pass
    }
    if (tid == 0) {
        a.nraw[p] = n1;
        a.ngood[p] = base;
    }
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

// Keys ([P][2][kcap], all ones) and arrival counters ([P], zero) that every k_match launch leaves
// reset; (re)initialised only when a buffer grows.  Growth is detected on the size: a freed and
// reallocated buffer can come back at the same address with an uninitialised tail.
static int match_state(vs_ctx* ctx, int P, int kcap, unsigned long long** keys, unsigned** cnt, hipStream_t s) {
    const size_t kb = ctx->match_keys.bytes;
    VS_CHECK(ctx->match_keys.ensure((size_t)P * 2 * kcap * sizeof(unsigned long long)));
    if (ctx->match_keys.bytes != kb) VS_HIP(hipMemsetAsync(ctx->match_keys.p, 0xFF, ctx->match_keys.bytes, s));
    const size_t cb = ctx->match_cnt.bytes;
    VS_CHECK(ctx->match_cnt.ensure((size_t)P * sizeof(unsigned)));
    if (ctx->match_cnt.bytes != cb) VS_HIP(hipMemsetAsync(ctx->match_cnt.p, 0, ctx->match_cnt.bytes, s));
    *keys = ctx->match_keys.as<unsigned long long>();
    *cnt = ctx->match_cnt.as<unsigned>();
    return VS_OK;
}

int match_reserve(vs_ctx* ctx, int P, int cap, hipStream_t s) {
    unsigned long long* keys;
    unsigned* cnt;
    return match_state(ctx, P, cap, &keys, &cnt, s);
}

template <int NWQ, int NWT, int WQ, int WT, int KC, int NBUF, int PD = 1>
static void launch_tile(MatchArgs& a, int P, int cap_q, int cap_t, bool norms, hipStream_t s) {
    constexpr int TQ = NWQ * WQ, TT = NWT * WT, NTH = 64 * NWQ * NWT;
    a.qblocks = (cap_q + TQ - 1) / TQ;
    a.tblocks = (cap_t + TT - 1) / TT;
    a.work = P * a.qblocks * a.tblocks;
    a.npairs = P;
    // largest-first order for multi-pair launches whose capacity leaves edge tiles: opt-in
    // (VS_MATCH_ORDER=1), measured slower -- 318 pairs 0.463 vs 0.495 of peak pair-major, 512 pairs
    // 0.485 vs 0.524 (profiles/r05h_match_order_ab.txt): the edge tiles' short blocks interleaved with
    // whole ones fill the CUs better than a tail of edge tiles alone
    static const bool lf = [] {
        const char* e = std::getenv("VS_MATCH_ORDER");
        return e && e[0] == '1';
    }();
    const int qf = cap_q / TQ, tf = cap_t / TT;
    const bool edges = qf * tf < a.qblocks * a.tblocks;
    a.qfull = (lf && P > 2 && edges && qf > 0 && tf > 0) ? qf : 0;
    a.tfull = a.qfull ? tf : 0;
    a.per_xcd = (a.work + 7) / 8;
    const unsigned blocks = (unsigned)(8 * a.per_xcd);
    static const char* abl = std::getenv("VS_MATCH_ABLATE");  // latency study only
    if (abl && PD == 1) {
        const int m = std::atoi(abl);
        if (m == 1) hipLaunchKernelGGL((k_match<NWQ, NWT, WQ, WT, KC, NBUF, PD, false, 1>), dim3(blocks), dim3(NTH), 0, s, a);
        if (m == 2) hipLaunchKernelGGL((k_match<NWQ, NWT, WQ, WT, KC, NBUF, PD, false, 2>), dim3(blocks), dim3(NTH), 0, s, a);
        if (m == 3) hipLaunchKernelGGL((k_match<NWQ, NWT, WQ, WT, KC, NBUF, PD, false, 3>), dim3(blocks), dim3(NTH), 0, s, a);
        if (m >= 1 && m <= 3) return;
    }
    if (norms)
        hipLaunchKernelGGL((k_match<NWQ, NWT, WQ, WT, KC, NBUF, PD, true>), dim3(blocks), dim3(NTH), 0, s, a);
    else
        hipLaunchKernelGGL((k_match<NWQ, NWT, WQ, WT, KC, NBUF, PD, false>), dim3(blocks), dim3(NTH), 0, s, a);
}

// Tile (r02 sweeps, profiles/r02_match_variants.jsonl): 64 x 64 workgroups of 2 x 2 waves, each
// wave 32 x 32 (four 16 x 16 chains), k staged in 32-wide chunks through one LDS buffer (23 KB,
// seven waves per SIMD).  Fragments wholly past n are skipped, so 400 keypoints cost no padded
// MFMA work.  Measured against: all of k in LDS at once (32 x 32 workgroups), 64-wide chunks,
// double buffering, every chunk's loads issued up front (PD = 8: no faster at one pair, so the
// lone-pair time is not per-chunk load latency), and 80 x 80 workgroups of five waves (no padding
// and 5 instead of 7 stagings per row, but five waves on four SIMDs: 13-16 % slower).
// VS_MATCH_TILE = small | k64 | k64d | k32d | deep | t80 selects those (experiments).
// r03 sweep (profiles/r03b_match_sweep.json, kernel durations alone on the chip, 400 x 400 pairs):
// one pair 16.3 us with 64 x 64 tiles vs 10.9 us with 32 x 32 (q32t32, four 16 x 16 waves), which
// loses at 32 pairs (52.3 vs 43.0 us) and 512 (0.39 vs 0.51 of the fp32 MFMA peak); 32 x 64 /
// 64 x 32 tiles and 8-wave 64 x 64 workgroups sit in between.  So P <= 2 takes 32 x 32 tiles.
static void launch(MatchArgs& a, int P, int cap_q, int cap_t, bool norms, hipStream_t s) {
    static const char* force = std::getenv("VS_MATCH_TILE");
    if (force && std::strcmp(force, "small") == 0)
        launch_tile<2, 2, 16, 16, 256, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "k64") == 0)
        launch_tile<2, 2, 32, 32, 64, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "k64d") == 0)
        launch_tile<2, 2, 32, 32, 64, 2>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "k32d") == 0)
        launch_tile<2, 2, 32, 32, 32, 2>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "deep") == 0)
        launch_tile<2, 2, 32, 32, 32, 1, 8>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "t80") == 0)
        launch_tile<5, 1, 16, 80, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "q32t64") == 0)
        launch_tile<1, 4, 32, 16, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "q32t32") == 0)
        launch_tile<2, 2, 16, 16, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "q64t32") == 0)
        launch_tile<2, 2, 32, 16, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "w8") == 0)
        launch_tile<2, 4, 32, 16, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "w8k64") == 0)
        launch_tile<2, 4, 32, 16, 64, 1>(a, P, cap_q, cap_t, norms, s);
    else if (force && std::strcmp(force, "default") == 0)
        launch_tile<2, 2, 32, 32, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else if (P <= 2)  // one or two pairs: 32 x 32 tiles (169 workgroups per 400 x 400 pair) fill the CUs
        launch_tile<2, 2, 16, 16, 32, 1>(a, P, cap_q, cap_t, norms, s);
    else
        launch_tile<2, 2, 32, 32, 32, 1>(a, P, cap_q, cap_t, norms, s);
}

int match_pairs(vs_ctx* ctx, int P, const int* d_pairs, int F, const float* d_desc, const int* d_n, int cap,
                float ratio, vs_match* d_raw, int* d_nraw, vs_match* d_good, int* d_ngood, hipStream_t s,
                const float* d_norms, unsigned long long* d_keys, unsigned* d_cnt) {
    if (P <= 0) return VS_OK;
    MatchArgs a{};
    if (d_keys && d_cnt) {  // the caller's own key / counter state (all ones / zero, left reset)
        a.keys = d_keys;
        a.cnt = d_cnt;
    } else {
        VS_CHECK(match_state(ctx, P, cap, &a.keys, &a.cnt, s));
    }
    // the tracker's speculative chain (its own key state) is timed apart from the tracking stream's matches
    ProfScope ps(ctx, (d_keys && d_cnt) ? "match_spec" : "match", s);
    static const bool pre_norms = std::getenv("VS_MATCH_NORMS") != nullptr;  // experiment: norms first
    if (!d_norms && pre_norms) {
        VS_CHECK(ctx->norms_sets.ensure(((size_t)F * cap * sizeof(float) + 255) & ~(size_t)255));
        VS_CHECK(desc_norms(ctx, F, d_desc, d_n, cap, ctx->norms_sets.as<float>(), s));
        d_norms = ctx->norms_sets.as<float>();
    }
    a.pairs = d_pairs;
    a.descq = a.desct = d_desc;
    a.normsq = a.normst = d_norms;
    a.n = d_n;
    a.qstride = a.tstride = cap;
    a.ratio = ratio;
    a.kcap = cap;
    a.raw = d_raw;
    a.nraw = d_nraw;
    a.good = d_good;
    a.ngood = d_ngood;
    a.ostride = cap;
    launch(a, P, cap, cap, d_norms != nullptr, s);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

// One query set against one train set held in separate arrays (PnP recovery: a frame's
// descriptors against every valid map point, Slam.cpp:560-575).  Outputs are indexed by query
// row (d_raw / d_good have n1 entries); d_counts = {n_raw, n_good}.
int match_sets(vs_ctx* ctx, const float* d_q, int n1, const float* d_t, int n2, float ratio, vs_match* d_raw,
               vs_match* d_good, int* d_counts, hipStream_t s) {
    if (n1 <= 0) return VS_OK;
    VS_CHECK(ctx->norms_sets.ensure(256));
    int* meta = ctx->norms_sets.as<int>();
    MatchArgs a{};
    VS_CHECK(match_state(ctx, 1, n1, &a.keys, &a.cnt, s));
    ProfScope ps(ctx, "match_map", s);
    hipLaunchKernelGGL(k_set_meta, dim3(1), dim3(1), 0, s, meta, n1, n2);
    // query rows as "frame 0" of stride n1, train rows as "frame 1" read with stride 0
    a.pairs = meta;
    a.descq = d_q;
    a.desct = d_t;
    a.n = meta + 2;
    a.qstride = n1;
    a.tstride = 0;
    a.ratio = ratio;
    a.kcap = n1;
    a.raw = d_raw;
    a.nraw = d_counts;
    a.good = d_good;
    a.ngood = d_counts + 1;
    a.ostride = n1;
    launch(a, 1, n1, n2 > 0 ? n2 : 1, false, s);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
