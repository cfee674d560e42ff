// sp_net.hip — SuperPoint network forward on gfx950 (replaces ONNX Runtime's Session::Run,
// reference src/FeatureExtractor.cpp:107-124; topology SURVEY.md 8(a) A3).
//
// Layout: NHWC fp32 activations, frames batched along N.  Every 3x3 / 1x1 conv is an implicit
// GEMM on the fp32 matrix cores (v_mfma_f32_32x32x2_f32, exact fp32 products, fp32 accumulate):
//   M = output pixels (tiles of 8 rows x 32 columns, one 32-pixel row segment per MFMA block),
//   N = output channels (64 per workgroup), K = k*k*Cin (Cin staged through LDS 16 at a time).
// Bias, ReLU and the 2x2 max-pool are fused into the epilogue: the 32x32 accumulator keeps
// horizontally adjacent pixels in adjacent registers of one lane and the two image rows of a
// pool window in the same wave, so pooling never leaves registers.  conv1a (1 -> 64) is fused
// into conv1b's input staging.
//
// Pipeline per channel chunk: the next chunk's input / weights are fetched into registers
// (global loads, or the fused conv1a recompute) before the current chunk's MFMAs so their
// latency hides under 288 MFMAs; the MFMA loop reads its LDS operands one k-step ahead.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "vs_internal.h"

namespace vs {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// A2: BGR u8 -> gray u8 (OpenCV fixed point) -> fp32 * (float)(1/255.0), zero-padded to Hp x Wp
// (FeatureExtractor.cpp:63-67, 90-105).
__global__ void k_gray_norm(const uint8_t* __restrict__ img, int channels, int h, int w, int Hp,
                            int Wp, float* __restrict__ out, int total) {
    int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    int x = idx % Wp;
    int t = idx / Wp;
    int y = t % Hp;
    int b = t / Hp;
    float v = 0.0f;
    if (x < w && y < h) {
        const uint8_t* p = img + ((size_t)b * h * w + (size_t)y * w + x) * channels;
        unsigned g;
        if (channels == 3)
            g = ((unsigned)p[0] * 1868u + (unsigned)p[1] * 9617u + (unsigned)p[2] * 4899u + (1u << 13)) >> 14;
        else
            g = p[0];
        v = (float)g * (float)(1.0 / 255.0);
    }
    out[idx] = v;
}

// XCD-aware work order.  Workgroups are dealt round-robin to the 8 XCDs (block b and b + 8 share
// one, and each XCD has its own L2), so the flat block index is remapped so that every XCD walks a
// contiguous range of work items w = tile * ntiles + output-channel tile: the ntiles workgroups of
// one spatial tile run back to back on one XCD and read its input patch through one L2 instead of
// ntiles times from the fabric.  Falls back to the plain order when the grid is not a multiple of 8.
__device__ inline void xcd_work_at(int w, int nblk, int ntiles, int& tile, int& nt) {
    if ((nblk & 7) == 0) w = (w & 7) * (nblk >> 3) + (w >> 3);
    tile = w / ntiles;
    nt = w - tile * ntiles;
}
__device__ inline void xcd_work(int ntiles, int& tile, int& nt) { xcd_work_at(blockIdx.x, gridDim.x, ntiles, tile, nt); }

// Generic conv (KS = 3: 3x3 pad 1 over 8x32 spatial tiles; KS = 1: 1x1 over linear 256-pixel
// tiles) on v_mfma_f32_32x32x2_f32.  256 threads = 4 waves; wave wv owns tile rows 2wv, 2wv+1
// (two 32-pixel M blocks) x 64 output channels (two N blocks): four 32x32 accumulators.
// LDS: s_in[CK][pixels] (channel-major: a half-wave reads 32 consecutive pixels, conflict free)
//      s_w [k*k*CK][64] (a half-wave reads 32 consecutive output channels, conflict free).
template <int KS, int CKV = (KS == 3 ? 16 : 32)>
struct ConvGeom {
    static constexpr int CK = CKV;
    static constexpr int TW = 32, TH = 8;
    static constexpr int PW = (KS == 3) ? TW + 2 : TW;
    static constexpr int PH = (KS == 3) ? TH + 2 : TH;
    static constexpr int NPIX = PW * PH;
};

// FUSE1A (conv1b only): `in` is the fp32 gray plane [B][H][W]; the kernel recomputes conv1a
// (1 -> 64, 3x3, ReLU) for each 16-channel chunk of its 10x34 input patch from a 12x36 gray patch
// in LDS, so the 64-channel full-resolution conv1a activation never goes through HBM.  Patch
// positions outside the image are conv1b's zero padding (0, not conv1a evaluated there).
// The body, for workgroup w_blk of an n_blk-workgroup grid (k_conv_mfma: blockIdx.x of gridDim.x;
// k_conv1x1_pair: its sub-grid's own index and size).
template <int KS, bool POOL, bool FUSE1A, int CKV>
__device__ __forceinline__ void conv_mfma_body(
    const float* __restrict__ in, int in_cstride, int in_coff, const float* __restrict__ wt,
    const float* __restrict__ bias, int cin, int cout, int cout_pad, float* __restrict__ out,
    int out_cstride, int out_coff, int B, int H, int W, int tiles_x, int tiles_y, int relu,
    const float* __restrict__ w1a, const float* __restrict__ b1a, int w_blk, int n_blk) {
    using G = ConvGeom<KS, CKV>;
    constexpr int CK = G::CK;
    constexpr int Q = CK / 4;                                  // float4 per pixel and chunk
    constexpr int NQ = (G::NPIX * Q + 255) / 256;              // input float4 per thread
    constexpr int NW = (KS * KS * CK * 16 + 255) / 256;        // weight float4 per thread
    constexpr int S = KS * KS * CK / 2;                        // MFMA k-steps per chunk
    __shared__ float s_in[CK * G::NPIX];
    __shared__ __attribute__((aligned(16))) float s_w[KS * KS * CK * 64];
    constexpr int GW = G::PW + 2, GH = G::PH + 2;  // gray patch for the fused conv1a
    __shared__ float s_g[FUSE1A ? GW * GH : 1];
    __shared__ float s_w1a[FUSE1A ? 10 * 64 : 1];   // 9 taps x 64 + bias

    const int tid = threadIdx.x;
    const int wv = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
    int tile, nt;
    xcd_work_at(w_blk, n_blk, cout_pad >> 6, tile, nt);
    const int n0 = nt * 64;
    int b = 0, y0 = 0, x0 = 0;
    long m0 = 0;  // KS == 1: first linear pixel of the tile
    const long M = (long)B * H * W;
    if constexpr (KS == 3) {
        int t = tile;
        int tx = t % tiles_x;
        t /= tiles_x;
        int ty = t % tiles_y;
        b = t / tiles_y;
        y0 = ty * G::TH;
        x0 = tx * G::TW;
    } else {
        m0 = (long)tile * 256;
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int nb = 0; nb < 2; nb++)
#pragma unroll
            for (int e = 0; e < 16; e++) acc[r][nb][e] = 0.0f;

    if constexpr (FUSE1A) {
        const float* g = in + (size_t)b * H * W;
        for (int i = tid; i < GW * GH; i += 256) {
            const int yy = i / GW, xx = i - yy * GW;
            const int gy = y0 - 2 + yy, gx = x0 - 2 + xx;
            s_g[i] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? g[(size_t)gy * W + gx] : 0.0f;
        }
        for (int i = tid; i < 9 * 64; i += 256) s_w1a[i] = w1a[i];
        if (tid < 64) s_w1a[9 * 64 + tid] = b1a[tid];
        __syncthreads();
    }

    f32x4 rin[FUSE1A ? 1 : NQ];
    f32x4 rw[NW];
    constexpr int NF = FUSE1A ? (G::NPIX * CK + 255) / 256 : 1;  // fused conv1a values per thread
    float rf[NF];
    // fused conv1a output j of this thread for the chunk starting at channel c0 (0 = zero padding)
    auto conv1a_val = [&](int j, int c0) -> float {
        const int idx = tid + 256 * j;
        const int c = idx / G::NPIX, p = idx - c * G::NPIX;
        const int py = p / G::PW, px = p - py * G::PW;
        const int gy = y0 - 1 + py, gx = x0 - 1 + px;
        float a = 0.0f;
        if (idx < G::NPIX * CK && gy >= 0 && gy < H && gx >= 0 && gx < W) {
            a = s_w1a[9 * 64 + c0 + c];
#pragma unroll
            for (int ky = 0; ky < 3; ky++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++)
                    a += s_g[(py + ky) * GW + px + kx] * s_w1a[(ky * 3 + kx) * 64 + c0 + c];
            a = a > 0.0f ? a : 0.0f;
        }
        return a;
    };

    // global -> registers for the chunk starting at channel c0 (the fused conv1a input is computed
    // at commit time instead: holding it in registers would spill)
    auto fetch = [&](int c0) {
        if constexpr (!FUSE1A) {
#pragma unroll
            for (int j = 0; j < NQ; j++) {
                const int idx = tid + 256 * j;
                const int p = idx / Q, q = idx - p * Q;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (idx < G::NPIX * Q) {
                    if constexpr (KS == 3) {
                        const int py = p / G::PW, px = p - py * G::PW;
                        const int gy = y0 - 1 + py, gx = x0 - 1 + px;
                        if (gy >= 0 && gy < H && gx >= 0 && gx < W)
                            v = *reinterpret_cast<const f32x4*>(in + (((size_t)b * H + gy) * W + gx) * in_cstride +
                                                                in_coff + c0 + 4 * q);
                    } else {
                        const long m = m0 + p;
                        if (m < M) v = *reinterpret_cast<const f32x4*>(in + (size_t)m * in_cstride + in_coff + c0 + 4 * q);
                    }
                }
                rin[j] = v;
            }
        }
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int idx = tid + 256 * j;
            if (idx < KS * KS * CK * 16) {
                const int r = idx >> 4, q = idx & 15;
                const int kk = r / CK, c = r - kk * CK;
                rw[j] = *reinterpret_cast<const f32x4*>(wt + ((size_t)kk * cin + c0 + c) * cout_pad + n0 + 4 * q);
            }
        }
    };
    // registers -> LDS (fused: the conv1a values computed into rf during the previous MFMA loop)
    auto commit = [&](int c0) {
        (void)c0;
        if constexpr (FUSE1A) {
#pragma unroll
            for (int j = 0; j < NF; j++) {
                const int idx = tid + 256 * j;
                if (idx < G::NPIX * CK) s_in[idx] = rf[j];  // idx = c * NPIX + p
            }
        } else {
#pragma unroll
            for (int j = 0; j < NQ; j++) {
                const int idx = tid + 256 * j;
                if (idx < G::NPIX * Q) {
                    const int p = idx / Q, q = idx - p * Q;
#pragma unroll
                    for (int e = 0; e < 4; e++) s_in[(4 * q + e) * G::NPIX + p] = rin[j][e];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int idx = tid + 256 * j;
            if (idx < KS * KS * CK * 16) {
                const int r = idx >> 4, q = idx & 15;
                *reinterpret_cast<f32x4*>(&s_w[r * 64 + 4 * q]) = rw[j];
            }
        }
    };
    // LDS operands of k-step s (s = kk * CK/2 + cp; lane half lh supplies channel 2cp + lh)
    auto operands = [&](int s, float& a0, float& a1, float& b0, float& b1) {
        const int kk = s / (CK / 2), cp = s - kk * (CK / 2);
        const int ky = kk / KS, kx = kk - ky * KS;
        const int c = 2 * cp + lh;
        const float* si = &s_in[c * G::NPIX];
        if constexpr (KS == 3) {
            a0 = si[(2 * wv + 0 + ky) * G::PW + li + kx];
            a1 = si[(2 * wv + 1 + ky) * G::PW + li + kx];
        } else {
            a0 = si[(2 * wv + 0) * 32 + li];
            a1 = si[(2 * wv + 1) * 32 + li];
        }
        b0 = s_w[(kk * CK + c) * 64 + li];
        b1 = s_w[(kk * CK + c) * 64 + 32 + li];
    };

    fetch(0);
    if constexpr (FUSE1A) {
#pragma unroll
        for (int j = 0; j < NF; j++) rf[j] = conv1a_val(j, 0);
    }
    commit(0);
    __syncthreads();
    for (int c0 = 0; c0 < cin; c0 += CK) {
        const bool more = c0 + CK < cin;
        if (more) fetch(c0 + CK);
        const int cnext = more ? c0 + CK : 0;  // fused conv1a: the next chunk, computed between MFMAs
        float A0[2], A1[2], B0[2], B1[2];
        operands(0, A0[0], A1[0], B0[0], B1[0]);
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int cur = s & 1, nxt = cur ^ 1;
            if (s + 1 < S) operands(s + 1, A0[nxt], A1[nxt], B0[nxt], B1[nxt]);
            if constexpr (FUSE1A) {
                if (s % 3 == 1 && s / 3 < NF) rf[s / 3] = conv1a_val(s / 3, cnext);
            }
            // keep the next step's LDS reads ahead of this step's MFMAs (the scheduler otherwise
            // sinks them to just before their consumers and exposes the LDS latency)
            __builtin_amdgcn_sched_barrier(0);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[cur], B0[cur], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[cur], B1[cur], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[cur], B0[cur], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[cur], B1[cur], acc[1][1], 0, 0, 0);
        }
        __syncthreads();
        if (more) {
            commit(c0 + CK);
            __syncthreads();
        }
    }

    // ---- epilogue: C/D map of 32x32 blocks: col (out channel) = lane&31,
    //      row (pixel in the 32-segment) = (reg&3) + 8*(reg>>2) + 4*(lane>>5) ----
#pragma unroll
    for (int nb = 0; nb < 2; nb++) {
        const int n = n0 + nb * 32 + li;
        if (n >= cout) continue;
        const float bv = bias[n];
        if constexpr (POOL) {
            const int y = y0 + 2 * wv;  // pool window rows y, y+1 live in acc[0], acc[1]
            if (y >= H) continue;
            const int Wo = W >> 1;
#pragma unroll
            for (int reg = 0; reg < 16; reg += 2) {
                const int px = (reg & 3) + 8 * (reg >> 2) + 4 * lh;
                const int x = x0 + px;
                if (x >= W) continue;
                float m = fmaxf(fmaxf(acc[0][nb][reg], acc[0][nb][reg + 1]), fmaxf(acc[1][nb][reg], acc[1][nb][reg + 1]));
                m += bv;
                if (relu) m = fmaxf(m, 0.0f);
                out[(((size_t)b * (H >> 1) + (y >> 1)) * Wo + (x >> 1)) * out_cstride + out_coff + n] = m;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 2; r++) {
#pragma unroll
                for (int reg = 0; reg < 16; reg++) {
                    const int px = (reg & 3) + 8 * (reg >> 2) + 4 * lh;
                    float v = acc[r][nb][reg] + bv;
                    if (relu) v = fmaxf(v, 0.0f);
                    if constexpr (KS == 3) {
                        const int y = y0 + 2 * wv + r, x = x0 + px;
                        if (y < H && x < W)
                            out[(((size_t)b * H + y) * W + x) * out_cstride + out_coff + n] = v;
                    } else {
                        const long m = m0 + (2 * wv + r) * 32 + px;
                        if (m < M) out[(size_t)m * out_cstride + out_coff + n] = v;
                    }
                }
            }
        }
    }
}

template <int KS, bool POOL, int LAYER, bool FUSE1A = false, int CKV = (KS == 3 ? 16 : 32)>
__global__ __launch_bounds__(256, (KS == 3 && CKV == 32) ? 1 : ((CKV == 8 || (KS == 1 && CKV == 16)) ? 3 : 2)) void k_conv_mfma(
    const float* __restrict__ in, int in_cstride, int in_coff, const float* __restrict__ wt,
    const float* __restrict__ bias, int cin, int cout, int cout_pad, float* __restrict__ out,
    int out_cstride, int out_coff, int B, int H, int W, int tiles_x, int tiles_y, int relu,
    const float* __restrict__ w1a, const float* __restrict__ b1a) {
    conv_mfma_body<KS, POOL, FUSE1A, CKV>(in, in_cstride, in_coff, wt, bias, cin, cout, cout_pad, out, out_cstride,
                                          out_coff, B, H, W, tiles_x, tiles_y, relu, w1a, b1a, blockIdx.x, gridDim.x);
}

// Two 1x1 convolutions in one grid (round 6: SuperPoint's convDb and convPb, which read different channel
// ranges of head_a's output): the first n_first workgroups run the first, the rest the second, each
// with its own XCD-aware order — one launch, the second layer's workgroups filling the first's tail.
struct Conv1x1Args {
    const float* in;
    int in_cstride, in_coff;
    const float* wt;
    const float* bias;
    int cin, cout, cout_pad;
    float* out;
    int out_cstride, out_coff;
};
template <int CKV>
__global__ __launch_bounds__(256, CKV == 16 ? 3 : 2) void k_conv1x1_pair(Conv1x1Args a, Conv1x1Args b, int n_first,
                                                                          int B, int H, int W) {
    const bool first = (int)blockIdx.x < n_first;
    const Conv1x1Args& c = first ? a : b;
    const int w = first ? (int)blockIdx.x : (int)blockIdx.x - n_first;
    const int n = first ? n_first : (int)gridDim.x - n_first;
    conv_mfma_body<1, false, false, CKV>(c.in, c.in_cstride, c.in_coff, c.wt, c.bias, c.cin, c.cout, c.cout_pad, c.out,
                                         c.out_cstride, c.out_coff, B, H, W, 1, 1, 0, nullptr, nullptr, w, n);  // no ReLU after the heads
}

// Double-buffered 3x3 conv: 8-channel chunks, s_in / s_w in two LDS buffers (63 KB with the fused
// conv1a, two workgroups per CU), ONE barrier per chunk.  While chunk k's 36 k-steps run on the
// matrix cores, chunk k+1 is staged into the other buffer: global loads issued at the top of the
// chunk and written to LDS six k-steps before its end, or (FUSE1A) conv1a evaluated straight into
// the buffer, one channel every four k-steps.  Nothing staged is held across the MFMA loop except
// 8 float4 of loads, so the kernel fits two waves per SIMD without spilling.  Tiles, wave roles
// and the epilogue (bias, ReLU, in-register 2x2 pool) are those of k_conv_mfma.
//
// LIN (layers whose width is not a multiple of 32, e.g. the 80 x 60 conv4 / head layers of a
// 640 x 480 frame): a tile is 256 CONSECUTIVE pixels of the image in raster order instead of an
// 8 x 32 block, so no MFMA row is spent on columns past the image edge (8 x 32 tiles waste 22% of
// the grid at W = 80).  The LDS patch holds the rows those pixels span plus the halo, full width
// (tiles_y = patch rows, <= 640 patch pixels), and every lane addresses its own pixel in it.
// MB = 32-pixel M blocks per wave: 2 (256-pixel tiles), or 1 for linear tiles of 128 pixels
// (the 60 x 80 conv4 layers: 152 tiles of 256 pixels x 2 channel tiles per 8 frames fill only
// 45 % of the workgroup slots of 224 CUs; half-height tiles double the grid).
template <bool POOL, int LAYER, bool FUSE1A, bool LIN = false, int CKT = 8, int MB = 2>
__global__ __launch_bounds__(256, CKT == 4 ? (MB == 1 ? 4 : 3) : 2) void k_conv3_db(
    const float* __restrict__ in, int in_cstride, int in_coff, const float* __restrict__ wt,
    const float* __restrict__ bias, int cin, int cout, int cout_pad, float* __restrict__ out,
    int out_cstride, int out_coff, int B, int H, int W, int tiles_x, int tiles_y, int relu,
    const float* __restrict__ w1a, const float* __restrict__ b1a) {
    // CKT input channels per chunk: 8 (two workgroups per CU), or 4 (about half the LDS, three
    // workgroups per CU, twice the chunk barriers)
    constexpr int CK = CKT, TW = 32, TH = 8, PW = TW + 2, PH = TH + 2, NPIX = PW * PH;
    constexpr int TPIX = 128 * MB;                  // linear tile pixels
    constexpr int NPIXC = LIN ? (MB == 2 ? 640 : 448) : NPIX;  // patch capacity
    constexpr int Q = CK / 4;                       // float4 per pixel and chunk
    constexpr int NQ = (NPIXC * Q + 255) / 256;     // input float4 per thread
    constexpr int NWV = 9 * CK * 16;                // weight float4 per chunk
    constexpr int NW = (NWV + 255) / 256;           // weight float4 per thread
    constexpr int S = 9 * CK / 2;                   // MFMA k-steps per chunk
    constexpr int GW = PW + 2, GH = PH + 2;         // gray patch for the fused conv1a
    constexpr int SW = S - 6;                       // k-step at which staged loads go to LDS
    static_assert(NPIX > 256 && NPIX <= 512 && 4 * (CK - 1) + 2 < S, "conv3_db geometry");
    static_assert(!LIN || (!POOL && !FUSE1A), "linear tiles: plain 3x3 layers only");
    static_assert(MB == 2 || (MB == 1 && LIN), "half-height tiles: linear layers only");
    __shared__ float s_in[2][CK * NPIXC];
    __shared__ __attribute__((aligned(16))) float s_w[2][9 * CK * 64];
    __shared__ float s_g[FUSE1A ? GW * GH : 1];
    __shared__ __attribute__((aligned(16))) float s_w1a[FUSE1A ? 12 * 64 : 4];  // [channel][9 taps, bias, 0, 0]
    __shared__ float s_trash[FUSE1A ? 256 : 1];      // sink of the masked second-pixel stores

    const int tid = threadIdx.x;
    const int wv = tid >> 6, lane = tid & 63, li = lane & 31, lh = lane >> 5;
    int tile, nt;
    xcd_work(cout_pad >> 6, tile, nt);
    const int n0 = nt * 64;
    const int HW = H * W;
    int b, y0, x0, m0 = 0;
    if constexpr (LIN) {  // tiles_x = tiles per image, tiles_y = patch rows
        b = tile / tiles_x;
        m0 = (tile - b * tiles_x) * TPIX;
        y0 = m0 / W;  // first image row of the tile
        x0 = 0;
    } else {
        int t = tile;
        const int tx = t % tiles_x;
        t /= tiles_x;
        const int ty = t % tiles_y;
        b = t / tiles_y;
        y0 = ty * TH;
        x0 = tx * TW;
    }
    const int pw = LIN ? W + 2 : PW;           // patch row pitch
    const int npix = LIN ? pw * tiles_y : NPIX;  // patch pixels (per channel)
    // A-operand base of this lane's pixel in the two M blocks (patch position of tap (0, 0))
    int abase[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < MB; r++) {
        if constexpr (LIN) {
            int m = m0 + (MB * wv + r) * 32 + li;
            m = m < HW ? m : HW - 1;  // past the image end: any in-patch pixel, never stored
            const int y = m / W, x = m - y * W;
            abase[r] = (y - y0) * pw + x;
        } else {
            abase[r] = (2 * wv + r) * PW + li;
        }
    }

    f32x16 acc[2][2];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int nb = 0; nb < 2; nb++)
#pragma unroll
            for (int e = 0; e < 16; e++) acc[r][nb][e] = 0.0f;

    // fused conv1a: thread tid owns patch pixels tid and tid + 256 (< NPIX)
    int gbase[2] = {0, 0};
    bool gin[2] = {false, false};
    if constexpr (FUSE1A) {
        const float* g = in + (size_t)b * H * W;
        for (int i = tid; i < GW * GH; i += 256) {
            const int yy = i / GW, xx = i - yy * GW;
            const int gy = y0 - 2 + yy, gx = x0 - 2 + xx;
            s_g[i] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? g[(size_t)gy * W + gx] : 0.0f;
        }
        for (int i = tid; i < 12 * 64; i += 256) {
            const int c = i / 12, k = i - c * 12;
            s_w1a[i] = k < 9 ? w1a[k * 64 + c] : k == 9 ? b1a[c] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int p = tid + 256 * i < NPIX ? tid + 256 * i : 0;
            const int py = p / PW, px = p - py * PW;
            const int gy = y0 - 1 + py, gx = x0 - 1 + px;
            gin[i] = tid + 256 * i < NPIX && gy >= 0 && gy < H && gx >= 0 && gx < W;  // else zero padding
            gbase[i] = py * GW + px;
        }
        __syncthreads();
    }
    // the two pixels' 3x3 gray windows, in registers for the whole kernel
    float gnb[2][9];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int k = 0; k < 9; k++) gnb[i][k] = FUSE1A ? s_g[gbase[i] + (k / 3) * GW + k % 3] : 0.0f;
    // conv1a channel c0 + c (ReLU) at pixel i from the taps + bias in wq (one broadcast 3 x 16 B
    // read of s_w1a, issued two k-steps ahead of its use) -> s_in[buf][c]
    auto w1a_load = [&](int c, int c0, f32x4* wq) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(&s_w1a[(c0 + c) * 12]);
        wq[0] = wp[0];
        wq[1] = wp[1];
        wq[2] = wp[2];
    };
    auto conv1a_px = [&](int i, int c, int buf, const f32x4* wq) {
        const float wk[10] = {wq[0][0], wq[0][1], wq[0][2], wq[0][3], wq[1][0],
                              wq[1][1], wq[1][2], wq[1][3], wq[2][0], wq[2][1]};
        float a = wk[9];
#pragma unroll
        for (int k = 0; k < 9; k++) a = __builtin_fmaf(gnb[i][k], wk[k], a);
        a = a > 0.0f ? a : 0.0f;
        float* dst = (i == 0 || tid + 256 < NPIX) ? &s_in[buf][c * NPIX + tid + 256 * i] : &s_trash[tid];
        *dst = gin[i] ? a : 0.0f;
    };
    auto conv1a_chan = [&](int c, int c0, int buf) {
        f32x4 wq[3];
        w1a_load(c, c0, wq);
        conv1a_px(0, c, buf, wq);
        conv1a_px(1, c, buf, wq);
    };

    f32x4 rin[FUSE1A ? 1 : NQ];
    f32x4 rw[NW];
    auto fetch = [&](int c0) {
        if constexpr (!FUSE1A) {
#pragma unroll
            for (int j = 0; j < NQ; j++) {
                const int idx = tid + 256 * j;
                const int p = idx / Q, q = idx - p * Q;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (idx < npix * Q) {
                    const int py = p / pw, px = p - py * pw;
                    const int gy = y0 - 1 + py, gx = x0 - 1 + px;
                    if (gy >= 0 && gy < H && gx >= 0 && gx < W)
                        v = *reinterpret_cast<const f32x4*>(in + (((size_t)b * H + gy) * W + gx) * in_cstride + in_coff +
                                                            c0 + 4 * q);
                }
                rin[j] = v;
            }
        }
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int idx = tid + 256 * j;
            if (idx < NWV) {
                const int r = idx >> 4, q = idx & 15;
                const int kk = r / CK, c = r - kk * CK;
                rw[j] = *reinterpret_cast<const f32x4*>(wt + ((size_t)kk * cin + c0 + c) * cout_pad + n0 + 4 * q);
            }
        }
    };
    auto stage = [&](int buf) {
        if constexpr (!FUSE1A) {
#pragma unroll
            for (int j = 0; j < NQ; j++) {
                const int idx = tid + 256 * j;
                if (idx < npix * Q) {
                    const int p = idx / Q, q = idx - p * Q;
#pragma unroll
                    for (int e = 0; e < 4; e++) s_in[buf][(4 * q + e) * npix + p] = rin[j][e];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NW; j++) {
            const int idx = tid + 256 * j;
            if (idx < NWV) {
                const int r = idx >> 4, q = idx & 15;
                *reinterpret_cast<f32x4*>(&s_w[buf][r * 64 + 4 * q]) = rw[j];
            }
        }
    };

    fetch(0);
    if constexpr (FUSE1A) {
#pragma unroll
        for (int c = 0; c < CK; c++) conv1a_chan(c, 0, 0);
    }
    stage(0);
    __syncthreads();
    const int nchunk = cin / CK;
    for (int k = 0; k < nchunk; k++) {
        const int cur = k & 1, nxt = cur ^ 1;
        const bool more = k + 1 < nchunk;
        const int cn = (k + 1) * CK;
        if (more) fetch(cn);
        const float* si = s_in[cur];
        const float* sw = s_w[cur];
        auto operands = [&](int s, float& a0, float& a1, float& b0, float& b1) {
            const int kk = s / (CK / 2), cp = s - kk * (CK / 2);
            const int ky = kk / 3, kx = kk - ky * 3;
            const int c = 2 * cp + lh;
            a0 = si[c * npix + abase[0] + ky * pw + kx];
            a1 = si[c * npix + abase[1] + ky * pw + kx];
            b0 = sw[(kk * CK + c) * 64 + li];
            b1 = sw[(kk * CK + c) * 64 + 32 + li];
        };
        float A0[2], A1[2], B0[2], B1[2];
        operands(0, A0[0], A1[0], B0[0], B1[0]);
        f32x4 wq[3];
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int c_ = s & 1, n_ = c_ ^ 1;
            if (s + 1 < S) operands(s + 1, A0[n_], A1[n_], B0[n_], B1[n_]);
            // fused conv1a of the next chunk: channel s/4's taps are read at s % 4 == 0 and its two
            // pixels evaluated at s % 4 == 2, each FMA chain issued behind an MFMA so it runs while
            // the matrix core is busy
            const bool c1a = FUSE1A && more && s / 4 < CK;
            if (c1a && s % 4 == 0) w1a_load(s / 4, cn, wq);
            if (more && s == SW) stage(nxt);
            __builtin_amdgcn_sched_barrier(0);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[c_], B0[c_], acc[0][0], 0, 0, 0);
            if (c1a && s % 4 == 2) conv1a_px(0, s / 4, nxt, wq);
            __builtin_amdgcn_sched_barrier(0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0[c_], B1[c_], acc[0][1], 0, 0, 0);
            if (c1a && s % 4 == 2) conv1a_px(1, s / 4, nxt, wq);
            if constexpr (MB == 2) {
                __builtin_amdgcn_sched_barrier(0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[c_], B0[c_], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1[c_], B1[c_], acc[1][1], 0, 0, 0);
            }
        }
        __syncthreads();
    }

#pragma unroll
    for (int nb = 0; nb < 2; nb++) {
        const int n = n0 + nb * 32 + li;
        if (n >= cout) continue;
        const float bv = bias[n];
        if constexpr (POOL) {
            const int y = y0 + 2 * wv;
            if (y >= H) continue;
            const int Wo = W >> 1;
#pragma unroll
            for (int reg = 0; reg < 16; reg += 2) {
                const int px = (reg & 3) + 8 * (reg >> 2) + 4 * lh;
                const int x = x0 + px;
                if (x >= W) continue;
                float m = fmaxf(fmaxf(acc[0][nb][reg], acc[0][nb][reg + 1]), fmaxf(acc[1][nb][reg], acc[1][nb][reg + 1]));
                m += bv;
                if (relu) m = fmaxf(m, 0.0f);
                out[(((size_t)b * (H >> 1) + (y >> 1)) * Wo + (x >> 1)) * out_cstride + out_coff + n] = m;
            }
        } else {
#pragma unroll
            for (int r = 0; r < MB; r++) {
#pragma unroll
                for (int reg = 0; reg < 16; reg++) {
                    const int px = (reg & 3) + 8 * (reg >> 2) + 4 * lh;
                    float v = acc[r][nb][reg] + bv;
                    if (relu) v = fmaxf(v, 0.0f);
                    if constexpr (LIN) {
                        const int m = m0 + (MB * wv + r) * 32 + px;
                        if (m < HW) out[((size_t)b * HW + m) * out_cstride + out_coff + n] = v;
                    } else {
                        const int y = y0 + 2 * wv + r, x = x0 + px;
                        if (y < H && x < W) out[(((size_t)b * H + y) * W + x) * out_cstride + out_coff + n] = v;
                    }
                }
            }
        }
    }
}

// Winograd F(2x2, 3x3) conv on v_mfma_f32_16x16x4_f32 (round 3).  Each 2 x 2 output tile is
//   Y = A^T [ (G g G^T) (.) (B^T d B) ] A      (d: the tile's 4 x 4 input window, g: the 3 x 3 kernel)
// so the 9 multiply-adds per output pixel, input channel and output channel of the direct conv
// become 16 per 2 x 2 tile (2.25x fewer matrix-core FLOPs), all in fp32: the transforms are
// additions (input, output) or precomputed in fp64 and rounded once (weights, DevLayer::wu), and
// the 16 per-element products are accumulated over the input channels by the matrix cores —
// 16 independent GEMMs M[xi][tile][cout] = sum_c V[xi][tile][c] U[xi][c][cout].  The parity bar is
// the fp32 tolerance of the network tests (tests/test_gpu_parity.py), as for the direct conv.
//
// Workgroup = 4 x 8 tiles (8 x 16 output pixels, a 10 x 18 input patch) x 64 output channels,
// 4 waves; wave w owns tiles 16 (w & 1) .. + 15 and output channels 32 (w >> 1) .. + 31 for ALL 16
// transform elements (32 accumulators of 16 x 16), so the output transform, bias, ReLU and the
// 2 x 2 max-pool (POOL: a tile IS a pool window) stay in the lane's registers.  MFMA operands:
// A = V[xi][c0 + lane / 16][tile lane % 16], B = U[xi][c0 + lane / 16][cout lane % 16].
// LDS images (MI355X_MICROARCH.md, LDS banking): V as [row i][channel][tile][j] so one
// ds_read_b128 gives a lane the A operands of the 4 elements of a row (conflict-free lane groups);
// U with the columns of each 32-channel half permuted on the host (position 2i + nb = channel
// 16 nb + i: both B operands of a lane in one ds_read_b64) and the halves swapped for odd channels
// (the two 32-lane groups of a read hit different banks).
// Input channels go in chunks of 4 (one float4 per patch pixel) through a three-stage pipeline
// with ONE barrier per chunk: during chunk k's 32 MFMAs per wave, the raw patch of chunk k + 2 and
// the weights of chunk k + 1 go from registers (loaded a chunk earlier) to LDS, and chunk k + 1's
// patch (in LDS since chunk k - 1) is transformed into the other V buffer (32 tiles x 4 channels x
// 2 row halves on the 256 lanes); each row's LDS operands are read one row ahead of its MFMAs.
// FUSE1A: the patch channels are conv1a (1 -> 64, ReLU) evaluated from a 12 x 20 gray patch.
// MiDaS (midas.hip) runs its stride-1 3x3 convs through the same kernel (WinoArgs: input-side ReLU,
// ReLU / ReLU6 / none, residual adds after the activation, as k_mid_conv's epilogue).
// C32 (cout <= 32, MiDaS's head at 128^2 / 256^2): the wave pair of a tile half splits the 16
// transform elements instead of the 64 output channels (wave ch takes rows 2 ch, 2 ch + 1 of the 4 x 4
// domain for channels 0..31), so no MFMA multiplies a zero weight column; the two partial output
// transforms are added through LDS (Y = A^T (M_rows01 + M_rows23) A) before bias and activation.
// SPLIT: input-channel split-K (WinoArgs::part / splits, MiDaS's 8^2-16^2 decoder convs); a template
// parameter so that the unsplit instantiations keep their code (runtime split support had cost them
// 5-13 %, r03an).
#ifndef VS_WINO_SCHED
#define VS_WINO_SCHED 1  // main-loop schedule (A/B builds): 0 fenced segments, 1 interleaved, 2 free
#endif
#ifndef VS_WINO_PRIO
#define VS_WINO_PRIO 0   // 1: s_setprio(1) over each MFMA row region (A/B)
#endif
#ifndef VS_WINO_ABL
#define VS_WINO_ABL 0    // latency ablation (results are wrong): 1 no weight staging after the prologue,
                         // 2 no input transform, 3 no patch staging / conv1a, 4 no chunk barrier
#endif
template <bool POOL, bool FUSE1A, bool C32 = false, bool SPLIT = false>
__global__ __launch_bounds__(256, 2) void k_wino3(WinoArgs wa) {
    static_assert(!(C32 && (POOL || FUSE1A)), "C32 is the plain (MiDaS) variant");
    static_assert(!(SPLIT && (POOL || FUSE1A)), "SPLIT is the plain (MiDaS) variant");
    const float* __restrict__ in = wa.in;
    const float* __restrict__ wu = wa.wu;
    const float* __restrict__ bias = wa.bias;
    float* __restrict__ out = wa.out;
    const float* __restrict__ w1a = wa.w1a;  // FUSE1A: [64][9 taps, bias, 0, 0], read as scalar loads
    const int in_cstride = wa.in_cstride, in_coff = wa.in_coff, cin = wa.cin, cout = wa.cout, cout_pad = wa.cout_pad;
    const int out_cstride = wa.out_cstride, out_coff = wa.out_coff, H = wa.H, W = wa.W, nbx = wa.nbx, nby = wa.nby;
    const int act = wa.act;
    const bool pre_relu = wa.pre_relu != 0;
    constexpr int CK = 4, TBX = 8, NT = 32, PX = 2 * TBX + 2, PY = 10, NP = PX * PY;  // 18 x 10 patch
    constexpr int GX = PX + 2, GY = PY + 2;                                            // 20 x 12 gray
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    // one slot per thread (NP = 180 patch pixels used): every thread stores its chunk value without a
    // branch (threads past the patch write slots nobody reads), so the staging code has no basic-block
    // boundaries and interleaves with the MFMAs
    __shared__ __attribute__((aligned(16))) float s_x[2][CK][256];
    __shared__ __attribute__((aligned(16))) float s_v[2][4][CK][NT][4];
    __shared__ __attribute__((aligned(16))) float s_u[2][16][CK][64];
    __shared__ float s_g[FUSE1A ? GX * GY : 1];

    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
    const int th = wv & 1, ch = wv >> 1;
    int blk, nt;
    xcd_work(cout_pad >> 6, blk, nt);
    const int n0 = nt * 64;
    const int b = blk / (nbx * nby), r0 = blk - b * (nbx * nby);
    const int y0 = (r0 / nbx) * 8, x0 = (r0 % nbx) * 16;
    // split-K: this workgroup's input-channel chunks [cb, cb + nchunk)
    const int split = SPLIT ? (int)blockIdx.y : 0, nsplit = SPLIT ? wa.splits : 1;
    const int cb = SPLIT ? (int)((long)(cin / CK) * split / nsplit) : 0;
    const int nchunk = SPLIT ? (int)((long)(cin / CK) * (split + 1) / nsplit) - cb : cin / CK;
    constexpr bool raw = SPLIT;

    // raw patch pixel of this thread (tid < NP): patch (py, px) = input (y0 - 1 + py, x0 - 1 + px)
    const bool own_px = tid < NP;
    const int ppy = tid / PX, ppx = tid - (tid / PX) * PX;
    const int gy = y0 - 1 + ppy, gx = x0 - 1 + ppx;
    const bool pin = own_px && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const float* src = in + (((size_t)b * H + (pin ? gy : 0)) * W + (pin ? gx : 0)) * in_cstride + in_coff;

    float gnb[FUSE1A ? 9 : 1];
    if constexpr (FUSE1A) {
        const float* g = in + (size_t)b * H * W;
        for (int i = tid; i < GX * GY; i += 256) {
            const int yy = i / GX, xx = i - yy * GX;
            const int sy = y0 - 2 + yy, sx = x0 - 2 + xx;
            s_g[i] = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? g[(size_t)sy * W + sx] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 9; k++) gnb[k] = own_px ? s_g[(ppy + k / 3) * GX + ppx + k % 3] : 0.0f;
    }

    // registers: chunk c's patch in rx[c & 1] (loaded two chunks ahead of its LDS write), the next
    // chunk's weights in ru (loaded one chunk ahead)
    f32x4 rx[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    f32x4 ru[4];
    // G (guarded): the chunk index may run past the last chunk (the pipeline's tail); the steady
    // state below runs unguarded instantiations (no per-chunk branches around the staging code)
    auto fetch_x = [&](auto sl_c, auto g_c, int c) {
        constexpr int sl = decltype(sl_c)::value;
        if constexpr (!FUSE1A) {
            // src is clamped in the image (pin == false: pixel 0 of the frame), so the load needs no
            // branch; put_x zeroes what lies outside
            if (!decltype(g_c)::value || c < nchunk) rx[sl] = *reinterpret_cast<const f32x4*>(src + (cb + c) * CK);
        }
    };
    auto fetch_u = [&](auto g_c, int c) {
        if (decltype(g_c)::value && c >= nchunk) return;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int idx = tid + 256 * j, xi = idx >> 6, cc = (idx >> 4) & 3, q = idx & 15;
            ru[j] = *reinterpret_cast<const f32x4*>(wu + ((size_t)xi * cin + (cb + c) * CK + cc) * cout_pad + n0 + 4 * q);
        }
    };
    // chunk c's patch -> s_x[c & 1] (fused: conv1a of its 4 channels at this pixel, 0 outside the image)
    // channels [LO, HI) of the chunk (the schedule may split a chunk's conv1a over two MFMA rows)
    auto put_x_part = [&](auto sl_c, auto g_c, auto lo_c, auto hi_c, int c) {
        constexpr int sl = decltype(sl_c)::value;
        constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
        if (decltype(g_c)::value && c >= nchunk) return;
        if constexpr (FUSE1A) {
            // the chunk's 4 x (9 taps + bias) are wave-uniform: scalar loads into SGPRs, v_fma_f32 with an
            // SGPR operand (no LDS staging, no operand moves); same fmaf chain as before
            const f32x4* wp = reinterpret_cast<const f32x4*>(w1a + (size_t)(c * CK) * 12);
            f32x4 q[3 * CK];
#pragma unroll
            for (int i = 3 * LO; i < 3 * HI; i++) q[i] = wp[i];
#pragma unroll
            for (int cc = LO; cc < HI; cc++) {
                const f32x4 q0 = q[3 * cc], q1 = q[3 * cc + 1], q2 = q[3 * cc + 2];
                const float wk[9] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3], q2[0]};
                float a = q2[1];
#pragma unroll
                for (int k = 0; k < 9; k++) a = __builtin_fmaf(gnb[k], wk[k], a);
                s_x[sl][cc][tid] = pin ? (a > 0.0f ? a : 0.0f) : 0.0f;
            }
        } else {
#pragma unroll
            for (int cc = LO; cc < HI; cc++) {
                const float v = pin ? rx[sl][cc] : 0.0f;
                s_x[sl][cc][tid] = pre_relu ? fmaxf(v, 0.0f) : v;
            }
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I2 [[maybe_unused]] = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, CK>;
    auto put_x = [&](auto sl_c, auto g_c, int c) { put_x_part(sl_c, g_c, I0{}, I4{}, c); };
    // chunk c's weights -> s_u[c & 1] (channel cc's 32-column halves swapped when cc is odd)
    auto put_u = [&](auto sl_c, auto g_c, int c) {
        constexpr int sl = decltype(sl_c)::value;
        if (decltype(g_c)::value && c >= nchunk) return;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int idx = tid + 256 * j, xi = idx >> 6, cc = (idx >> 4) & 3, q = idx & 15;
            *reinterpret_cast<f32x4*>(&s_u[sl][xi][cc][4 * (q ^ (8 * (cc & 1)))]) = ru[j];
        }
    };
    // B^T d B of chunk c (s_x[c & 1] -> s_v[c & 1]) on all 64 lanes: lane = (tile t, channel cc)
    // of a channel pair, and the wave's half (wave-uniform: no divergence) takes V rows 2 half and
    // 2 half + 1, which need input rows half .. half + 2 only
    auto transform = [&](auto sl_c, auto g_c, int c) {
        constexpr int sl = decltype(sl_c)::value;
        if (decltype(g_c)::value && c >= nchunk) return;
        const int t = lane & 31, cc = 2 * (wv & 1) + (lane >> 5), tr = t >> 3, tc = t & 7;
        const int half = wv >> 1;
        const float* xp = &s_x[sl][cc][(2 * tr + half) * PX + 2 * tc];
        float e[3][4];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const f32x2 p0 = *reinterpret_cast<const f32x2*>(xp + i * PX);
            const f32x2 p1 = *reinterpret_cast<const f32x2*>(xp + i * PX + 2);
            e[i][0] = p0[0];
            e[i][1] = p0[1];
            e[i][2] = p1[0];
            e[i][3] = p1[1];
        }
        // rows 2 half, 2 half + 1 of B^T d without a branch (the selects are wave-uniform):
        //   half 0: ua = d0 - d2 = e0 - e2, ub = d1 + d2 = e1 + e2
        //   half 1: ua = d2 - d1 = e1 - e0, ub = d1 - d3 = e0 - e2
        // i.e. ua = y - x, ub = r + sg e2 (fmaf(+-1, e2, r) == r +- e2 exactly)
        const bool h1 = half != 0;
        const float sg = h1 ? -1.0f : 1.0f;
        float ua[4], ub[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float y = h1 ? e[1][j] : e[0][j], x = h1 ? e[0][j] : e[2][j], r = h1 ? e[0][j] : e[1][j];
            ua[j] = y - x;
            ub[j] = __builtin_fmaf(sg, e[2][j], r);
        }
        *reinterpret_cast<f32x4*>(&s_v[sl][2 * half][cc][t][0]) =
            f32x4{ua[0] - ua[2], ua[1] + ua[2], ua[2] - ua[1], ua[1] - ua[3]};
        *reinterpret_cast<f32x4*>(&s_v[sl][2 * half + 1][cc][t][0]) =
            f32x4{ub[0] - ub[2], ub[1] + ub[2], ub[2] - ub[1], ub[1] - ub[3]};
    };

    f32x4 acc[16][2];
#pragma unroll
    for (int x = 0; x < 16; x++) acc[x][0] = acc[x][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: V / U of chunk 0 and the patch of chunk 1 in LDS, chunk 1's weights and chunk 2's
    // patch in registers
    using GY_ = std::true_type;
    using GN_ = std::false_type;
    fetch_x(S0{}, GY_{}, 0);
    fetch_x(S1{}, GY_{}, 1);
    fetch_u(GY_{}, 0);
    put_x(S0{}, GY_{}, 0);
    put_x(S1{}, GY_{}, 1);
    put_u(S0{}, GY_{}, 0);
    fetch_u(GY_{}, 1);
    __syncthreads();
    transform(S0{}, GY_{}, 0);
    fetch_x(S0{}, GY_{}, 2);
    __syncthreads();
    const int ucol = (C32 ? 0 : 32 * ch) ^ (32 * (lk & 1));  // this lane's 32-column half in s_u (swizzled)
    f32x4 opa[2];      // A operands of a row (4 elements)
    f32x2 opb[2][4];   // B operands of a row (2 x 16 channels per element)
    auto read_row = [&](int buf, int i, int o) {
        opa[o] = *reinterpret_cast<const f32x4*>(&s_v[buf][i][lk][16 * th + li][0]);
#pragma unroll
        for (int j = 0; j < 4; j++) opb[o][j] = *reinterpret_cast<const f32x2*>(&s_u[buf][4 * i + j][lk][ucol + 2 * li]);
    };
    auto mfma_row = [&](int i, int o) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int xi = 4 * i + j;
            acc[xi][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(opa[o][j], opb[o][j][0], acc[xi][0], 0, 0, 0);
            acc[xi][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(opa[o][j], opb[o][j][1], acc[xi][1], 0, 0, 0);
        }
    };
    // C32: this wave's row r (domain row 2 ch + r) into accumulators 4 r .. 4 r + 3
    auto mfma_row_c32 = [&](int r, int o) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            acc[4 * r + j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(opa[o][j], opb[o][j][0], acc[4 * r + j][0], 0, 0, 0);
            acc[4 * r + j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(opa[o][j], opb[o][j][1], acc[4 * r + j][1], 0, 0, 0);
        }
    };
    // chunk k (P = k & 1): slots / buffers of chunk k + 1 are P ^ 1, of chunk k + 2 are P
    auto chunk = [&](auto par, auto g_c, int k) {
        constexpr int P = decltype(par)::value;
        using SP = std::integral_constant<int, P>;
        using SN = std::integral_constant<int, P ^ 1>;
        if constexpr (C32) {
            read_row(P, 2 * ch, 0);
            read_row(P, 2 * ch + 1, 1);
            put_u(SN{}, g_c, k + 1);
            fetch_u(g_c, k + 2);
            fetch_x(SN{}, g_c, k + 3);
            __builtin_amdgcn_sched_barrier(0);
            mfma_row_c32(0, 0);
            __builtin_amdgcn_sched_barrier(0);
            put_x(SP{}, g_c, k + 2);
            __builtin_amdgcn_sched_barrier(0);
            mfma_row_c32(1, 1);
            __builtin_amdgcn_sched_barrier(0);
            transform(SN{}, g_c, k + 1);
            __syncthreads();
            return;
        }
#if VS_WINO_SCHED == 0
        read_row(P, 0, 0);
        read_row(P, 1, 1);
        put_u(SN{}, g_c, k + 1);    // loaded during chunk k - 1; its buffer's last reader was chunk k - 1
        fetch_u(g_c, k + 2);
        fetch_x(SN{}, g_c, k + 3);  // slot of chunk k + 1, whose patch went to LDS during chunk k - 1
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(0, 0);
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(1, 1);
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 3, 1);
        put_x(SP{}, g_c, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(2, 0);
        __builtin_amdgcn_sched_barrier(0);
        transform(SN{}, g_c, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(3, 1);
#elif VS_WINO_SCHED == 1
        // interleaved: each row's 8 MFMAs carry the staging / conv1a / transform work between them
        // (sched_group_barrier: MFMA=0x8 VALU=0x2 VMEM=0x10 DS_READ=0x100 DS_WRITE=0x200)
        read_row(P, 0, 0);
        read_row(P, 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (VS_WINO_PRIO) __builtin_amdgcn_s_setprio(1);
        mfma_row(0, 0);
        if (VS_WINO_ABL != 1) {
            put_u(SN{}, g_c, k + 1);
            fetch_u(g_c, k + 2);
        }
        if (VS_WINO_ABL != 3) fetch_x(SN{}, g_c, k + 3);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 2, 0);
        mfma_row(1, 1);
        if (VS_WINO_ABL != 3) put_x(SP{}, g_c, k + 2);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 1);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 3, 1);
        mfma_row(2, 0);
        if (VS_WINO_ABL != 2) transform(SN{}, g_c, k + 1);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 2);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 2);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(3, 1);
        if (VS_WINO_PRIO) __builtin_amdgcn_s_setprio(0);
#elif VS_WINO_SCHED == 3
        // as 1, with conv1a split over rows 0 and 1 and the transform over rows 2 and 3
        read_row(P, 0, 0);
        read_row(P, 1, 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(0, 0);
        put_u(SN{}, g_c, k + 1);
        fetch_u(g_c, k + 2);
        fetch_x(SN{}, g_c, k + 3);
        put_x_part(SP{}, g_c, I0{}, I2{}, k + 2);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 2, 0);
        mfma_row(1, 1);
        put_x_part(SP{}, g_c, I2{}, I4{}, k + 2);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 1);
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        read_row(P, 3, 1);
        transform(SN{}, g_c, k + 1);
        mfma_row(2, 0);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 2);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 2);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_row(3, 1);
#else
        // no scheduling fences: the compiler's own interleave
        read_row(P, 0, 0);
        read_row(P, 1, 1);
        put_u(SN{}, g_c, k + 1);
        fetch_u(g_c, k + 2);
        fetch_x(SN{}, g_c, k + 3);
        mfma_row(0, 0);
        read_row(P, 2, 0);
        mfma_row(1, 1);
        read_row(P, 3, 1);
        put_x(SP{}, g_c, k + 2);
        mfma_row(2, 0);
        transform(SN{}, g_c, k + 1);
        mfma_row(3, 1);
#endif
        if (VS_WINO_ABL != 4) __syncthreads();  // chunk k + 1's V / U and chunk k + 2's patch complete; chunk k's buffers free
    };
    // steady state: a chunk pair (k, k + 1) touches chunks up to k + 4, so it runs unguarded while
    // k + 4 < nchunk; the tail pairs keep the guards
    int k = 0;
    for (; k + 4 < nchunk; k += 2) {
        chunk(S0{}, GN_{}, k);
        chunk(S1{}, GN_{}, k + 1);
    }
    for (; k < nchunk; k += 2) {
        chunk(S0{}, GY_{}, k);
        if (k + 1 < nchunk) chunk(S1{}, GY_{}, k + 1);
    }

    // A^T M A per (tile, output channel); C/D: cout = lane % 16, tile row 4 (lane / 16) + reg.
    // Results go through LDS (the staging buffers are free after the last barrier) so that every
    // global store is a float4 of 4 consecutive channels and a pixel's 32 channels of this wave
    // form one 128-byte segment (scalar stores of 16 channels per pixel wrote half lines).
    float* so = &s_u[0][0][0][0] + wv * 2048;  // this wave: [16 tiles x (POOL ? 1 : 4) pixels][32 channels]
    if constexpr (C32) {
        // waves ch = 1 (domain rows 2, 3) leave their partial transforms in their LDS region; the
        // ch = 0 partner (rows 0, 1) adds them below
        if (ch == 1) {
#pragma unroll
            for (int nb = 0; nb < 2; nb++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int tl = 4 * lk + r;
                    float m2[4], m3[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        m2[j] = acc[j][nb][r];
                        m3[j] = acc[4 + j][nb][r];
                    }
                    float s0[4], s1[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        s0[j] = m2[j];
                        s1[j] = -m2[j] - m3[j];
                    }
                    so[(4 * tl + 0) * 32 + 16 * nb + li] = s0[0] + s0[1] + s0[2];
                    so[(4 * tl + 1) * 32 + 16 * nb + li] = s0[1] - s0[2] - s0[3];
                    so[(4 * tl + 2) * 32 + 16 * nb + li] = s1[0] + s1[1] + s1[2];
                    so[(4 * tl + 3) * 32 + 16 * nb + li] = s1[1] - s1[2] - s1[3];
                }
        }
        __syncthreads();
    }
    const float* sp = so + 2 * 2048;  // C32: the ch = 1 partner's partials (read by ch = 0 waves only)
#pragma unroll
    for (int nb = 0; nb < 2; nb++) {
        const int n = n0 + (C32 ? 0 : 32 * ch) + 16 * nb + li;
        const float bv = (n < cout && !raw) ? bias[n] : 0.0f;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int tl = 4 * lk + r;  // tile within the wave's 16
            float m[4][4];
            if constexpr (C32) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    m[0][j] = acc[j][nb][r];
                    m[1][j] = acc[4 + j][nb][r];
                    m[2][j] = m[3][j] = 0.0f;
                }
            } else {
#pragma unroll
                for (int xi = 0; xi < 16; xi++) m[xi >> 2][xi & 3] = acc[xi][nb][r];
            }
            float s0[4], s1[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                s0[j] = m[0][j] + m[1][j] + m[2][j];
                s1[j] = m[1][j] - m[2][j] - m[3][j];
            }
            const float y00 = s0[0] + s0[1] + s0[2], y01 = s0[1] - s0[2] - s0[3];
            const float y10 = s1[0] + s1[1] + s1[2], y11 = s1[1] - s1[2] - s1[3];
            // act: 0 none, 1 ReLU, 2 ReLU6 (v > 0 ? min(v, 6) : 0, as midas.hip activate()); raw
            // split-K partials take neither bias nor activation
            auto actf = [&](float v) {
                return (act == 0 || raw) ? v : v > 0.0f ? (act == 2 && !(v < 6.0f) ? 6.0f : v) : 0.0f;
            };
            if constexpr (POOL) {
                so[tl * 32 + 16 * nb + li] = actf(fmaxf(fmaxf(y00, y01), fmaxf(y10, y11)) + bv);
            } else if constexpr (C32) {
                if (ch == 0) {
                    const int o0 = (4 * tl) * 32 + 16 * nb + li;
                    so[o0] = actf(y00 + sp[o0] + bv);
                    so[o0 + 32] = actf(y01 + sp[o0 + 32] + bv);
                    so[o0 + 64] = actf(y10 + sp[o0 + 64] + bv);
                    so[o0 + 96] = actf(y11 + sp[o0 + 96] + bv);
                }
            } else {
                so[(4 * tl + 0) * 32 + 16 * nb + li] = actf(y00 + bv);
                so[(4 * tl + 1) * 32 + 16 * nb + li] = actf(y01 + bv);
                so[(4 * tl + 2) * 32 + 16 * nb + li] = actf(y10 + bv);
                so[(4 * tl + 3) * 32 + 16 * nb + li] = actf(y11 + bv);
            }
        }
    }
    __syncthreads();
    constexpr int NV = POOL ? 2 : 8;  // float4 per lane: 16 (POOL) or 64 pixels x 8 float4
#pragma unroll
    for (int u = 0; u < NV; u++) {
        const int e = lane + 64 * u, pix = e >> 3, q = e & 7;
        const int n = n0 + 32 * ch + 4 * q;  // C32: the ch = 1 waves' n >= 32 >= cout (nothing to store)
        if (n >= cout) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(&so[pix * 32 + 4 * q]);
        const int tl = POOL ? pix : pix >> 2, t = 16 * th + tl, tr = t >> 3, tc = t & 7;
        if constexpr (POOL) {
            const int oy = y0 + 2 * tr, ox = x0 + 2 * tc;
            if (oy >= H || ox >= W) continue;  // H, W even: a tile inside is a whole window
            *reinterpret_cast<f32x4*>(out + (((size_t)b * (H >> 1) + (oy >> 1)) * (W >> 1) + (ox >> 1)) * out_cstride +
                                      out_coff + n) = v;
        } else {
            const int oy = y0 + 2 * tr + ((pix >> 1) & 1), ox = x0 + 2 * tc + (pix & 1);
            if (oy >= H || ox >= W) continue;
            if constexpr (raw) {
                const size_t pp = (size_t)split * wa.B * H * W + ((size_t)b * H + oy) * W + ox;
                *reinterpret_cast<f32x4*>(wa.part + pp * cout + n) = v;
                continue;
            }
            const size_t o = (((size_t)b * H + oy) * W + ox) * out_cstride + out_coff + n;
            f32x4 r = v;
            if (wa.res1) r = r + *reinterpret_cast<const f32x4*>(wa.res1 + o);
            if (wa.res2) r = *reinterpret_cast<const f32x4*>(wa.res2 + o) + r;
            *reinterpret_cast<f32x4*>(out + o) = r;
        }
    }
}

namespace {

template <int KS, bool POOL, int LAYER, bool FUSE1A = false, int CKV = (KS == 3 ? 16 : 32)>
int launch_conv(const DevLayer& L, const float* in, int in_cstride, int in_coff, float* out,
                int out_cstride, int out_coff, int B, int H, int W, int relu, hipStream_t s,
                const DevLayer* L1a = nullptr) {
    using G = ConvGeom<KS, CKV>;
    if (L.cin % G::CK != 0 || L.cout_pad % 64 != 0 || (!FUSE1A && (in_cstride % 4 || in_coff % 4)) ||
        (FUSE1A && !L1a)) {
        set_error("conv: unsupported channel geometry");
        return VS_ERR_ARG;
    }
    int tiles_x = 1, tiles_y = 1;
    long nblk;
    if (KS == 3) {
        tiles_x = (W + G::TW - 1) / G::TW;
        tiles_y = (H + G::TH - 1) / G::TH;
        nblk = (long)B * tiles_x * tiles_y;
    } else {
        nblk = ((long)B * H * W + 255) / 256;
    }
    if (POOL && ((H | W) & 1)) {
        set_error("conv: pooled layer needs even H, W");
        return VS_ERR_ARG;
    }
    dim3 grid((unsigned)(nblk * (L.cout_pad / 64)));
    hipLaunchKernelGGL((k_conv_mfma<KS, POOL, LAYER, FUSE1A, CKV>), grid, dim3(256), 0, s, in, in_cstride, in_coff, L.w,
                       L.b, L.cin, L.cout, L.cout_pad, out, out_cstride, out_coff, B, H, W, tiles_x, tiles_y, relu,
                       L1a ? L1a->w : nullptr, L1a ? L1a->b : nullptr);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

// 3x3 layers use a 16-channel chunk: 58.6 KB of LDS, two workgroups per CU, so one workgroup's
// staging overlaps the other's MFMAs.  (A 32-channel chunk at one workgroup per CU measured
// 1.5x slower end to end: 1306 vs 1952 frames/s, round 1.)
// conv1 (fused conv1a) runs the double-buffered kernel: 6.56 vs 6.84 ms per 32 frames (round 1
// A/B); the other 3x3 layers measured the same or 1-2% slower with it and keep the single-buffered
// 16-channel kernel.  VS_CONV3=single selects the single-buffered conv1 too (A/B measurements).
inline bool conv3_db_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VS_CONV3");
        return !(e && std::strcmp(e, "single") == 0);
    }();
    return on;
}

// Winograd F(2x2, 3x3) for every 3x3 layer with a transformed weight copy (round 3; VS_WINO=0
// selects the direct implicit-GEMM kernels below, for A/B measurements).
inline bool wino_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VS_WINO");
        return !(e && e[0] == '0');
    }();
    return on;
}

inline bool wino4_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VS_WINO4");
        return !(e && e[0] == '0');
    }();
    return on;
}

inline long wino4_min_wg() {
    static const long n = [] {
        const char* e = std::getenv("VS_WINO4_MIN_WG");
        return e ? std::atol(e) : 32L;
    }();
    return n;
}

// VS_WINO_C32=0: cout <= 32 layers on the 64-channel variant (A/B measurements)
bool wino_c32_on() {
    static const bool on = [] {
        const char* e = std::getenv("VS_WINO_C32");
        return !(e && e[0] == '0');
    }();
    return on;
}

}  // namespace

int wino3_launch(WinoArgs a, bool pool, bool fuse1a, hipStream_t s) {
    a.nbx = (a.W + 15) / 16;
    a.nby = (a.H + 7) / 8;
    if (a.splits < 1) a.splits = 1;
    if (a.splits > 1 && (pool || fuse1a || !a.part || a.cout % 4 != 0 || a.splits > a.cin / 4)) return VS_ERR_ARG;
    dim3 grid((unsigned)((long)a.B * a.nbx * a.nby * (a.cout_pad / 64)), (unsigned)a.splits);
    if (pool && fuse1a)
        hipLaunchKernelGGL((k_wino3<true, true>), grid, dim3(256), 0, s, a);
    else if (pool)
        hipLaunchKernelGGL((k_wino3<true, false>), grid, dim3(256), 0, s, a);
    else if (fuse1a)
        return VS_ERR_ARG;
    else if (a.cout <= 32 && wino_c32_on() && a.splits > 1)
        hipLaunchKernelGGL((k_wino3<false, false, true, true>), grid, dim3(256), 0, s, a);
    else if (a.cout <= 32 && wino_c32_on())
        hipLaunchKernelGGL((k_wino3<false, false, true>), grid, dim3(256), 0, s, a);
    else if (a.splits > 1)
        hipLaunchKernelGGL((k_wino3<false, false, false, true>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_wino3<false, false>), grid, dim3(256), 0, s, a);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

namespace {

template <bool POOL, bool FUSE1A>
int launch_wino(const DevLayer& L, const float* in, int in_cstride, int in_coff, float* out, int out_cstride,
                int out_coff, int B, int H, int W, hipStream_t s, const DevLayer* L1a) {
    if (!L.wu || L.cin % 4 != 0 || L.cout_pad % 64 != 0 || L.cout % 4 != 0 || out_cstride % 4 || out_coff % 4 ||
        (!FUSE1A && (in_cstride % 4 || in_coff % 4)) ||
        (FUSE1A && (!L1a || L1a->cout != 64 || L.cin != 64 || !L1a->w1a_rows)) || (POOL && ((H | W) & 1))) {
        set_error("conv3 (Winograd): unsupported geometry");
        return VS_ERR_ARG;
    }
    WinoArgs a{};
    a.in = in;
    a.in_cstride = in_cstride;
    a.in_coff = in_coff;
    a.wu = L.wu;
    a.bias = L.b;
    a.cin = L.cin;
    a.cout = L.cout;
    a.cout_pad = L.cout_pad;
    a.out = out;
    a.out_cstride = out_cstride;
    a.out_coff = out_coff;
    a.B = B;
    a.H = H;
    a.W = W;
    a.w1a = L1a ? L1a->w1a_rows : nullptr;  // [64][9 taps, bias, 0, 0]
    a.b1a = nullptr;
    a.act = 1;  // every SuperPoint 3x3 conv is followed by ReLU
    // F(4x4, 3x3) (round 5, wino4.hip) on the layers whose 16 x 16-pixel workgroups are many per frame:
    // at least VS_WINO4_MIN_WG (default 32: conv4a/b's 40 included — alone on the chip they run 5 %
    // slower than F(2x2), beside the tracker 14 % faster, +2.5 % frames/s) per frame — a property of the layer's geometry alone, so a
    // frame's result never depends on the batch it is extracted in; VS_WINO4=0 keeps every layer on
    // F(2x2, 3x3) (A/B)
    if (L.wu4 && wino4_enabled() && (long)((H + 15) / 16) * ((W + 15) / 16) * (L.cout_pad / 64) >= wino4_min_wg()) {
        a.wu = L.wu4;
        a.wu3 = L.wu4x3;
        return wino4_launch(a, POOL, FUSE1A, s);
    }
    return wino3_launch(a, POOL, FUSE1A, s);
}

template <bool POOL, int LAYER, bool FUSE1A = false>
int conv3(vs_ctx* ctx, const DevLayer& L, const float* in, int in_cstride, int in_coff, float* out, int out_cstride,
          int out_coff, int B, int H, int W, hipStream_t s, const DevLayer* L1a = nullptr) {
    (void)ctx;
    if (wino_enabled() && L.wu)
        return launch_wino<POOL, FUSE1A>(L, in, in_cstride, in_coff, out, out_cstride, out_coff, B, H, W, s, L1a);
    if constexpr (!FUSE1A) {
        // linear tiles when 8 x 32 tiles would waste columns and the patch fits
        const int lin_rows = (W - 1 + 255) / W + 1 + 2;
        if (!POOL && W % 32 != 0 && lin_rows * (W + 2) <= 640 && conv3_db_enabled() && L.cin % 8 == 0 &&
            L.cout_pad % 64 == 0 && in_cstride % 4 == 0 && in_coff % 4 == 0) {
            const int ntn = L.cout_pad / 64;
            // conv4a / conv4b / the fused head: 4-channel chunks, three workgroups per CU (39 KB LDS, 134
            // VGPRs; same-box A/B over 3 runs each: the three layers 0.1051 -> 0.0993 ms per frame).
            // VS_CONV_LIN_CK=8 restores 8-channel chunks.  A grid of fewer than 1024 256-pixel
            // workgroups (conv4a / conv4b: 304 per 8 frames) runs 128-pixel tiles instead
            // (VS_CONV_LIN_MB = 1 / 2 forces one size).
            static const int ck = [] {
                const char* e = std::getenv("VS_CONV_LIN_CK");
                return e ? std::atoi(e) : 4;
            }();
            static const int mb_env = [] {
                const char* e = std::getenv("VS_CONV_LIN_MB");
                return e ? std::atoi(e) : 0;
            }();
            const int tiles256 = (H * W + 255) / 256;
            const int mb = mb_env == 1 || mb_env == 2 ? mb_env : ((long)B * tiles256 * ntn < 1024 ? 1 : 2);
            const int lin_rows1 = (W - 1 + 127) / W + 1 + 2;
            if (ck == 4 && mb == 1 && lin_rows1 * (W + 2) <= 448) {
                const int tiles = (H * W + 127) / 128;
                dim3 grid((unsigned)(B * tiles * ntn));
                hipLaunchKernelGGL((k_conv3_db<false, LAYER, false, true, 4, 1>), grid, dim3(256), 0, s, in,
                                   in_cstride, in_coff, L.w, L.b, L.cin, L.cout, L.cout_pad, out, out_cstride,
                                   out_coff, B, H, W, tiles, lin_rows1, 1, nullptr, nullptr);
                VS_HIP(hipGetLastError());
                return VS_OK;
            }
            const int tiles = tiles256;
            dim3 grid((unsigned)(B * tiles * ntn));
            if (ck == 4)
                hipLaunchKernelGGL((k_conv3_db<false, LAYER, false, true, 4>), grid, dim3(256), 0, s, in, in_cstride,
                                   in_coff, L.w, L.b, L.cin, L.cout, L.cout_pad, out, out_cstride, out_coff, B, H, W,
                                   tiles, lin_rows, 1, nullptr, nullptr);
            else
                hipLaunchKernelGGL((k_conv3_db<false, LAYER, false, true>), grid, dim3(256), 0, s, in, in_cstride,
                                   in_coff, L.w, L.b, L.cin, L.cout, L.cout_pad, out, out_cstride, out_coff, B, H, W,
                                   tiles, lin_rows, 1, nullptr, nullptr);
            VS_HIP(hipGetLastError());
            return VS_OK;
        }
        // conv2a / conv2b / conv3a / conv3b: 8-channel chunks, three workgroups per CU (29 KB LDS, 146
        // VGPRs) instead of 16-channel chunks at two (same-box A/B over 4 runs each: the four layers
        // 0.1997 -> 0.1920 ms per frame).  VS_CONV_CK=16 restores 16-channel chunks.
        static const int ck = [] {
            const char* e = std::getenv("VS_CONV_CK");
            return e ? std::atoi(e) : 8;
        }();
        if (ck == 8)
            return launch_conv<3, POOL, LAYER, FUSE1A, 8>(L, in, in_cstride, in_coff, out, out_cstride, out_coff, B, H,
                                                          W, 1, s, L1a);
        return launch_conv<3, POOL, LAYER, FUSE1A, 16>(L, in, in_cstride, in_coff, out, out_cstride, out_coff, B, H,
                                                       W, 1, s, L1a);
    } else {
    if (!conv3_db_enabled())
        return launch_conv<3, POOL, LAYER, FUSE1A, 16>(L, in, in_cstride, in_coff, out, out_cstride, out_coff, B, H,
                                                       W, 1, s, L1a);
    if (L.cin % 8 != 0 || L.cout_pad % 64 != 0 || (!FUSE1A && (in_cstride % 4 || in_coff % 4)) || (FUSE1A && !L1a) ||
        (POOL && ((H | W) & 1))) {
        set_error("conv3: unsupported geometry");
        return VS_ERR_ARG;
    }
    const int tiles_x = (W + 31) / 32, tiles_y = (H + 7) / 8;
    dim3 grid((unsigned)(B * tiles_x * tiles_y * (L.cout_pad / 64)));
    // The fused conv1 runs with 4-channel chunks: three workgroups per CU instead of two (35 KB of
    // LDS, 145 VGPRs) hide its chunk barriers and prologue better (same-box A/B over 5 + 3 runs: conv1
    // 97.6-99.5 -> 102.4-103.1 TFLOP/s, 0.63 -> 0.65-0.66 of the whole-chip fp32 MFMA peak; end to end
    // equal).  VS_CONV1_CK=8 restores 8-channel chunks.
    static const int ck = [] {
        const char* e = std::getenv("VS_CONV1_CK");
        return e ? std::atoi(e) : 4;
    }();
    if (FUSE1A && ck == 4)
        hipLaunchKernelGGL((k_conv3_db<POOL, LAYER, FUSE1A, false, 4>), grid, dim3(256), 0, s, in, in_cstride, in_coff,
                           L.w, L.b, L.cin, L.cout, L.cout_pad, out, out_cstride, out_coff, B, H, W, tiles_x, tiles_y,
                           1, L1a ? L1a->w : nullptr, L1a ? L1a->b : nullptr);
    else
        hipLaunchKernelGGL((k_conv3_db<POOL, LAYER, FUSE1A>), grid, dim3(256), 0, s, in, in_cstride, in_coff, L.w, L.b,
                           L.cin, L.cout, L.cout_pad, out, out_cstride, out_coff, B, H, W, tiles_x, tiles_y, 1,
                           L1a ? L1a->w : nullptr, L1a ? L1a->b : nullptr);
    VS_HIP(hipGetLastError());
    return VS_OK;
    }
}

}  // namespace

int sp_forward(vs_ctx* ctx, int B, const uint8_t* d_img, int channels, int h, int w, hipStream_t s, float* semi_out,
               float* dgrid_out, bool grid_raw) {
    VS_CHECK(scratch_order(ctx, s));
    ScratchUse scratch_use(ctx, s);
    const int Hp = ((h + 7) / 8) * 8, Wp = ((w + 7) / 8) * 8;
    const int hc = Hp / 8, wc = Wp / 8;
    const size_t full = (size_t)B * Hp * Wp;
    VS_CHECK(ctx->gray.ensure(full * sizeof(float)));
    // largest activations: the half-resolution 64-channel maps (conv1b+pool and conv2a outputs)
    VS_CHECK(ctx->act0.ensure(full / 4 * 64 * sizeof(float)));
    VS_CHECK(ctx->act1.ensure(full / 4 * 64 * sizeof(float)));
    if (!semi_out) {
        VS_CHECK(ctx->semi.ensure((size_t)B * hc * wc * kSemiCh * sizeof(float)));
        semi_out = ctx->semi.as<float>();
    }
    if (!dgrid_out) {
        VS_CHECK(ctx->dgrid.ensure((size_t)B * hc * wc * kDescDim * sizeof(float)));
        dgrid_out = ctx->dgrid.as<float>();
    }
    float* gray = ctx->gray.as<float>();
    float* a0 = ctx->act0.as<float>();
    float* a1 = ctx->act1.as<float>();
    const DevLayer* L = ctx->layers;
    if (d_img) {
        ProfScope ps(ctx, "gray_norm", s);
        int total = (int)full;
        hipLaunchKernelGGL(k_gray_norm, dim3((total + 255) / 256), dim3(256), 0, s, d_img, channels, h, w, Hp, Wp,
                           gray, total);
        VS_HIP(hipGetLastError());
    }
    int H = Hp, W = Wp;
    {
        ProfScope ps(ctx, "conv1_fused", s);  // conv1a + conv1b + ReLU + 2x2 pool in one kernel
        VS_CHECK((conv3<true, 1, true>(ctx, L[1], gray, 1, 0, a1, 64, 0, B, H, W, s, &L[0])));
    }
    H /= 2; W /= 2;
    {
        ProfScope ps(ctx, "conv2a", s);
        VS_CHECK((conv3<false, 2>(ctx, L[2], a1, 64, 0, a0, 64, 0, B, H, W, s)));
    }
    {
        ProfScope ps(ctx, "conv2b_pool", s);
        VS_CHECK((conv3<true, 3>(ctx, L[3], a0, 64, 0, a1, 64, 0, B, H, W, s)));
    }
    H /= 2; W /= 2;
    {
        ProfScope ps(ctx, "conv3a", s);
        VS_CHECK((conv3<false, 4>(ctx, L[4], a1, 64, 0, a0, 128, 0, B, H, W, s)));
    }
    {
        ProfScope ps(ctx, "conv3b_pool", s);
        VS_CHECK((conv3<true, 5>(ctx, L[5], a0, 128, 0, a1, 128, 0, B, H, W, s)));
    }
    H /= 2; W /= 2;
    {
        ProfScope ps(ctx, "conv4a", s);
        VS_CHECK((conv3<false, 6>(ctx, L[6], a1, 128, 0, a0, 128, 0, B, H, W, s)));
    }
    {
        ProfScope ps(ctx, "conv4b", s);
        VS_CHECK((conv3<false, 7>(ctx, L[7], a0, 128, 0, a1, 128, 0, B, H, W, s)));
    }
    {
        ProfScope ps(ctx, "head_a", s);  // convPa | convDa, 128 -> 512
        VS_CHECK((conv3<false, 8>(ctx, ctx->head_a, a1, 128, 0, a0, 512, 0, B, H, W, s)));
    }
    {
        ProfScope ps(ctx, "head_b", s);  // convPb 256 -> 65 and convDb 256 -> 256 (1x1)
        // the 1x1 heads (convPb, convDb) with 16-channel chunks, three workgroups per CU (20 KB LDS, 130
        // VGPRs; same-box A/B over 3 runs each: 0.0191-0.0206 -> 0.0162 ms per frame).
        // VS_CONV1X1_CK=32 restores 32-channel chunks.
        static const int ck1 = [] {
            const char* e = std::getenv("VS_CONV1X1_CK");
            return e ? std::atoi(e) : 16;
        }();
        // round 6: both in one grid (convDb's workgroups first: both sub-grids keep an 8-aligned XCD order);
        // VS_HEADB_PAIR=0: two launches
        static const bool pair = [] {
            const char* e = std::getenv("VS_HEADB_PAIR");
            return !(e && e[0] == '0');
        }();
        if (ck1 == 16 && pair) {
            const DevLayer& P = L[9];
            const DevLayer& D = L[11];
            if (P.cin % 16 || D.cin % 16 || P.cout_pad % 64 || D.cout_pad % 64) return VS_ERR_ARG;
            const long nb = ((long)B * H * W + 255) / 256;
            const Conv1x1Args d{a0, 512, 256, D.w, D.b, D.cin, D.cout, D.cout_pad, dgrid_out, kDescDim, 0};
            const Conv1x1Args p{a0, 512, 0, P.w, P.b, P.cin, P.cout, P.cout_pad, semi_out, kSemiCh, 0};
            const int n_first = (int)(nb * (D.cout_pad / 64));
            hipLaunchKernelGGL(k_conv1x1_pair<16>, dim3((unsigned)(n_first + nb * (P.cout_pad / 64))), dim3(256), 0, s,
                               d, p, n_first, B, H, W);
            VS_HIP(hipGetLastError());
        } else if (ck1 == 16) {
            VS_CHECK((launch_conv<1, false, 9, false, 16>(L[9], a0, 512, 0, semi_out, kSemiCh, 0, B, H, W, 0, s)));
            VS_CHECK((launch_conv<1, false, 11, false, 16>(L[11], a0, 512, 256, dgrid_out, kDescDim, 0, B, H, W, 0, s)));
        } else {
            VS_CHECK((launch_conv<1, false, 9>(L[9], a0, 512, 0, semi_out, kSemiCh, 0, B, H, W, 0, s)));
            VS_CHECK((launch_conv<1, false, 11>(L[11], a0, 512, 256, dgrid_out, kDescDim, 0, B, H, W, 0, s)));
        }
    }
    // the model's "desc" output is normalised (a raw-"desc" ONNX export skips it); grid_raw: the
    // caller's post-processing normalises the sampled corners instead (sp_postprocess)
    if (ctx->desc_l2 && !grid_raw) VS_CHECK(desc_grid_l2norm(ctx, (long)B * H * W, dgrid_out, s));
    return VS_OK;
}

}  // namespace vs
