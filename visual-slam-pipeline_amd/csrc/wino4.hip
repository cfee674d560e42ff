// wino4.hip — Winograd F(4x4, 3x3) convolution on v_mfma_f32_16x16x4_f32 for SuperPoint's large
// stride-1 3x3 layers (round 5; replaces ONNX Runtime's Conv inside Session::Run, reference
// src/FeatureExtractor.cpp:116-124, topology SURVEY.md 8(a) A3).
//
// Each 4 x 4 output tile is  Y = A^T [ (G g G^T) (.) (B^T d B) ] A  over its 6 x 6 input window d
// (points 0, +-1, +-2 and infinity; Lavin & Gray's matrices):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0; 0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// 36 products per tile, input channel and output channel instead of the direct form's 144 (the
// F(2x2) kernel k_wino3 does 64 per four 2 x 2 tiles): 2.25 per output pixel against 4 (F(2x2)) and
// 9 (direct).  Everything is fp32: G g G^T is computed in fp64 at weight upload and rounded once
// (winograd4_weights, vs_ctx.hip), the input and output transforms are fp32 adds / fmas, and the 36
// element-wise products are accumulated over the input channels by the matrix cores as 36
// independent GEMMs  M[xi][tile][cout] = sum_c V[xi][tile][c] U[xi][c][cout].  Parity bar: the
// network's fp32 tolerance against torch fp64 (tests/test_gpu_parity.py, stated there).
//
// Workgroup = 16 x 16 output pixels (4 x 4 tiles, an 18 x 18 input patch) x 64 output channels,
// 4 XG waves.  Wave w owns output channels 16 (w & 3) .. + 15 of all 16 tiles for the transform
// elements of domain rows RG (w >> 2) .. + RG - 1 (RG = 6 / XG: 6 RG sixteen-by-sixteen accumulators), so
// each wave's partial output transform A^T M_rows A stays in registers and the XG parts are added once,
// through LDS, in the epilogue.  XG = 3 (round 6, the default): 12 waves of 12 accumulators, ~144 VGPRs,
// 3 waves per SIMD — the kernel is bound by the latency of its staging chain (profiles/r05c ablation), so
// the third wave per SIMD is what pays (+3.6 % headline, profiles/r06xg_headline_ab.txt); XG = 2 (round 5):
// 8 waves of 18.  Per 4-channel k-step a wave issues 6 RG MFMAs; its operands are one 6-float row of V and
// of U per domain row (3 ds_read_b64 each, conflict-free images).
//
// Per k-step k (one barrier), while the MFMAs of k run on buffers k & 1:
//   * each lane's B operands of k + 1 (U, prearranged on the host in MFMA operand order, 20 floats
//     per lane and domain-row half) are read from L2 straight into registers one step ahead (no LDS
//     image and no barrier for U; the first version staged U through LDS with global_load_lds and
//     was slower);
//   * the patch of k + 1 (in LDS since step k - 1) is transformed into V of k + 1: thread
//     (domain row i = its wave, channel, tile) forms row i of B^T d from four patch rows and
//     applies the row transform (the row index is wave-uniform, so its coefficients are scalars);
//   * the patch of k + 2 is written to LDS — from registers loaded one step earlier, or (FUSE1A,
//     conv1) evaluated as conv1a (1 -> 64, 3 x 3, ReLU) from a 20 x 20 gray patch.
// POOL: a 4 x 4 tile holds four whole 2 x 2 pool windows; bias, ReLU and the pool are applied to
// the summed halves before the results go through LDS to float4 stores.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "vs_internal.h"

namespace vs {

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kW4Patch = 18;                 // 18 x 18 input patch
constexpr int kW4NP = kW4Patch * kW4Patch;   // 324
// The patch in LDS: rows kW4RS floats apart, channels W4Geo::CS apart.  A transform lane (channel tc,
// tile row a, tile column b) reads at tc CS + 4 a kW4RS + 4 b (+ the same row / column offset in every
// lane): with 4 kW4RS = 16 mod 64 and CS = 2 mod 64 the 32 lanes of a ds_read_b64 group fall on 32
// distinct bank pairs (row stride 18 and channel stride 512 gave up to 4-way conflicts).
constexpr int kW4RS = 20;
constexpr int kW4PadSlot = kW4Patch * kW4RS;  // 360: 16 dummy slots after the patch (a partly real wave's rest)
// per k-step of 4 SUB channels (SUB 4-channel MFMA sub-steps between two barriers)
template <int SUB> struct W4Geo {
    static constexpr int CH = 4 * SUB;
    static constexpr int V = 8 * CH * 16 * 6;   // V image: [row 8][ch][tile 16][col 6] (rows 6, 7: dummy)
    static constexpr int CS = 386;              // patch channel stride: 18 rows x kW4RS + 16 dummy slots + 10, = 2 mod 64
    static constexpr int X = CH * CS;           // patch: [ch][CS]
    static constexpr int OffV = 0;
    static constexpr int OffX = 2 * V;
    static constexpr int OffG = OffX + 2 * X;
    static constexpr int Main = OffG + 400;     // + the FUSE1A gray patch (20 x 20)
    static constexpr int YS = 16 * 16 + 4;       // epilogue: a tile's 16 px x 16 ch of a half, 4 floats of skew
    static constexpr int Epi = 64 * YS > 16384 ? 64 * YS : 16384;
    static constexpr int Lds = Main > Epi ? Main : Epi;  // epilogue: partial halves, then the outputs
    static_assert(Lds * 4 <= 160 * 1024, "LDS");
};

__device__ inline void w4_xcd_work(int ntiles, int& tile, int& nt) {
    const int nblk = gridDim.x;
    int w = blockIdx.x;
    if ((nblk & 7) == 0) w = (w & 7) * (nblk >> 3) + (w >> 3);
    tile = w / ntiles;
    nt = w - tile * ntiles;
}

// row transform of a 6-vector by B (V[i][:] = T_i B): the factored F(4, 3) input transform
__device__ inline void w4_rowB(const float t[6], float o[6]) {
    const float a = t[1] + t[2], b = t[3] + t[4];
    const float c = t[1] - t[2], e = t[4] - t[3];
    const float f = t[3] - t[1], g = t[4] - t[2];
    o[0] = __builtin_fmaf(4.0f, t[0], __builtin_fmaf(-5.0f, t[2], t[4]));
    o[1] = __builtin_fmaf(-4.0f, a, b);
    o[2] = __builtin_fmaf(4.0f, c, e);
    o[3] = __builtin_fmaf(2.0f, f, g);
    o[4] = __builtin_fmaf(-2.0f, f, g);
    o[5] = __builtin_fmaf(4.0f, t[1], __builtin_fmaf(-5.0f, t[3], t[5]));
}

// R = m A (4 outputs from a 6-vector): the factored F(4, 3) output transform
__device__ inline void w4_rowA(const float m[6], float r[4]) {
    const float a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], e = m[3] - m[4];
    r[0] = m[0] + a + c;
    r[1] = __builtin_fmaf(2.0f, e, b);
    r[2] = __builtin_fmaf(4.0f, c, a);
    r[3] = __builtin_fmaf(8.0f, e, b) + m[5];
}

}  // namespace

#ifndef VS_W4_ABL
#define VS_W4_ABL 0  // latency ablation (results are wrong): 1 no transform, 2 no patch staging, 3 no MFMA,
                     // 4 no barrier in the k-loop, 5 no B loads, 6 half the k-steps, 7 two k-steps only
                     // (6 and 7 separate the per-workgroup fixed cost from the per-k-step cost)
#endif
// one lane's B operands of a 4-channel sub-step: U[6 RG xh + x][ch][cout] for x < 6 RG (XG = 2: 18 = 4 x 16 B
// + 8 B; XG = 3: 12 = 3 x 16 B)
template <int XG> struct W4B;
template <> struct W4B<2> {
    f32x4 q[4];
    f32x2 r;
    __device__ float operator[](int x) const { return x < 16 ? q[x >> 2][x & 3] : r[x - 16]; }
};
template <> struct W4B<3> {
    f32x4 q[3];
    __device__ float operator[](int x) const { return q[x >> 2][x & 3]; }
};

// XG: domain-row groups per workgroup — 2: rows 0-2 | 3-5 on 8 waves (18 accumulators each, 2 waves per
// SIMD); 3 (round 6): rows 0-1 | 2-3 | 4-5 on 12 waves (12 accumulators each, 3 waves per SIMD to hide the
// staging chain's latency; the same A operand traffic in total)
template <bool POOL, bool FUSE1A, int SUB, int XG>
__global__ __launch_bounds__(256 * XG, 1) void k_wino4(WinoArgs wa) {
    static_assert(XG == 2 || (XG == 3 && SUB == 1), "XG");
    using Geo = W4Geo<SUB>;
    constexpr int CH = Geo::CH;
    constexpr int RG = 6 / XG;         // domain rows per wave
    constexpr int NT = 256 * XG;       // threads
    constexpr int NW = NT / 64;        // waves
    constexpr int BS = XG == 2 ? 20 : 12;  // B operand floats per lane in the weight image
    constexpr int BK = 4 * XG * 64 * BS;   // B operands per 4 channels
    const float* __restrict__ in = wa.in;
    const float* __restrict__ bias = wa.bias;
    float* __restrict__ out = wa.out;
    const float* __restrict__ w1a = wa.w1a;  // FUSE1A: [64][9 taps, bias, 0, 0]
    const int in_cstride = wa.in_cstride, in_coff = wa.in_coff, cin = wa.cin, cout = wa.cout;
    const int out_cstride = wa.out_cstride, out_coff = wa.out_coff, H = wa.H, W = wa.W, nbx = wa.nbx, nby = wa.nby;
    const int ntn = wa.cout_pad >> 6;
    // XG = 3: the epilogue holds both other groups' partial transforms at once (one pass; 133 KB, within
    // the CU's 160 KB: a workgroup fills its CU's VGPRs anyway)
    constexpr int kEpiParts = XG == 3 ? 2 : 1;
    constexpr int kLds = Geo::Lds > kEpiParts * 64 * Geo::YS ? Geo::Lds : kEpiParts * 64 * Geo::YS;
    static_assert(kLds * 4 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[kLds];

    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
    const int cg = wv & 3, xh = wv >> 2;
    int blk, nt;
    w4_xcd_work(ntn, blk, nt);
    const int b = blk / (nbx * nby), r0 = blk - b * (nbx * nby);
    const int y0 = (r0 / nbx) * 16, x0 = (r0 % nbx) * 16;
    const int nk = VS_W4_ABL == 6 ? cin / CH / 2 : VS_W4_ABL == 7 ? 2 : cin / CH;  // k-steps
    // this lane's B operands: [nt][4-channel chunk][cg][xh][lane][20]
    const float* __restrict__ wb = wa.wu + ((size_t)nt * (cin >> 2) * (4 * XG) + cg * XG + xh) * (64 * BS) + lane * BS;

    // ---- patch role: slot p of the 18 x 18 patch, every thread (slots >= 324 are written, never read).
    // XG = 2: waves 6, 7, 0, 1, 2, 3 hold the 324 real pixels, so the patch work lands beside the transform
    // work on the other waves of the SIMD pairs; XG = 3: waves 6-11 (the transform is on waves 0-5).
    constexpr int PW = XG == 2 ? 2 : 6;
    const int pslot = (wv + PW) % NW;
    const int p = pslot * 64 + lane;
    const bool own_px = p < kW4NP;
    const bool dummy_wave = pslot * 64 >= kW4NP;  // wave-uniform: no patch pixel at all
    const int ppy = p / kW4Patch, ppx = p - (p / kW4Patch) * kW4Patch;
    const int pq = own_px ? ppy * kW4RS + ppx : kW4PadSlot + (lane & 15);  // the slot's place in the LDS patch
    const int gy = y0 - 1 + ppy, gx = x0 - 1 + ppx;
    const bool pin = own_px && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const float* src = in + (((size_t)b * H + (pin ? gy : 0)) * W + (pin ? gx : 0)) * in_cstride + in_coff;
    // +0 outside the image (conv padding) by a bit mask: a select between two stores became a branch
    const uint32_t pmask = pin ? ~0u : 0u;
    auto masked = [&](float v) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & pmask); };
    float gnb[FUSE1A ? 9 : 1];
    if constexpr (FUSE1A) {
        const float* g = in + (size_t)b * H * W;
        for (int i = tid; i < 400; i += NT) {
            const int yy = i / 20, xx = i - (i / 20) * 20;
            const int sy = y0 - 2 + yy, sx = x0 - 2 + xx;
            lds[Geo::OffG + i] = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? g[(size_t)sy * W + sx] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 9; k++) gnb[k] = own_px ? lds[Geo::OffG + (ppy + k / 3) * 20 + ppx + k % 3] : 0.0f;
    }
    using GY_ = std::true_type;   // guarded: the k-step index may run past the last one (pipeline tail)
    using GN_ = std::false_type;  // steady state: no guards, so no basic-block boundaries around the work
    f32x4 rx[SUB];
#pragma unroll
    for (int u = 0; u < SUB; u++) rx[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto fetch_x = [&](auto g_c, int c) {
        if (dummy_wave) return;
        if constexpr (!FUSE1A) {
            // src is clamped into the image (pin == false: pixel 0 of the frame); put_x zeroes what lies outside
            if (!decltype(g_c)::value || c < nk)
#pragma unroll
                for (int u = 0; u < SUB; u++) rx[u] = *reinterpret_cast<const f32x4*>(src + CH * c + 4 * u);
        }
    };
    // patch of k-step c -> lds[X slot]: [ch][slot]
    auto put_x = [&](int slot, auto g_c, int c) {
        if (decltype(g_c)::value && c >= nk) return;
        if (VS_W4_ABL == 2 || dummy_wave) return;
        float* xs = lds + Geo::OffX + slot * Geo::X + pq;
        if constexpr (FUSE1A) {
            // the k-step's channels' 9 taps + bias are wave-uniform: scalar loads, v_fma_f32 with SGPR operands
            const f32x4* wp = reinterpret_cast<const f32x4*>(w1a + (size_t)(CH * c) * 12);
#pragma unroll
            for (int cc = 0; cc < CH; cc++) {
                const f32x4 q0 = wp[3 * cc], q1 = wp[3 * cc + 1], q2 = wp[3 * cc + 2];
                const float wk[9] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3], q2[0]};
                float a = q2[1];
#pragma unroll
                for (int k = 0; k < 9; k++) a = __builtin_fmaf(gnb[k], wk[k], a);
                xs[cc * Geo::CS] = masked(a > 0.0f ? a : 0.0f);
            }
        } else {
#pragma unroll
            for (int cc = 0; cc < CH; cc++) xs[cc * Geo::CS] = masked(rx[cc >> 2][cc & 3]);
        }
    };

    // ---- transform role: SUB items per thread, item u = (domain row i, channel, tile) of index
    // tid + 512 u over [row][ch][tile]; rows 6 and 7 are dummy rows of the image (waves past the six
    // real rows repeat rows 0 and 1 there), so that the code has no branch
    struct TrItem {
        int rr[4];
        float kc[4];
        int xbase, vbase;
    };
    TrItem tri[SUB];
#pragma unroll
    for (int u = 0; u < SUB; u++) {
        const int idx = tid + 512 * u, ti = idx / (16 * CH), tc = (idx >> 4) % CH, tt = idx & 15;
        TrItem& T = tri[u];
        // row i of B^T: four patch rows and their coefficients (wave-uniform)
        T.rr[0] = 1, T.rr[1] = 2, T.rr[2] = 3, T.rr[3] = 4;
        switch (ti) {
            case 0: case 6: T.rr[0] = 0, T.rr[1] = 2, T.rr[2] = 4, T.rr[3] = 4;
                T.kc[0] = 4.f, T.kc[1] = -5.f, T.kc[2] = 1.f, T.kc[3] = 0.f; break;
            case 1: case 7: T.kc[0] = -4.f, T.kc[1] = -4.f, T.kc[2] = 1.f, T.kc[3] = 1.f; break;
            case 2: T.kc[0] = 4.f, T.kc[1] = -4.f, T.kc[2] = -1.f, T.kc[3] = 1.f; break;
            case 3: T.kc[0] = -2.f, T.kc[1] = -1.f, T.kc[2] = 2.f, T.kc[3] = 1.f; break;
            case 4: T.kc[0] = 2.f, T.kc[1] = -1.f, T.kc[2] = -2.f, T.kc[3] = 1.f; break;
            default: T.rr[0] = 1, T.rr[1] = 3, T.rr[2] = 5, T.rr[3] = 5;
                T.kc[0] = 4.f, T.kc[1] = -5.f, T.kc[2] = 1.f, T.kc[3] = 0.f; break;
        }
        T.xbase = tc * Geo::CS + (4 * (tt >> 2)) * kW4RS + 4 * (tt & 3);
        T.vbase = ((ti * CH + tc) * 16 + tt) * 6;
    }
    auto transform = [&](int u, int slot, auto g_c, int c) {
        if (decltype(g_c)::value && c >= nk) return;
        if (VS_W4_ABL == 1) return;
        if (XG == 3 && wv >= 6) return;  // the six real rows on waves 0-5
        const TrItem& T = tri[u];
        const float* xs = lds + Geo::OffX + slot * Geo::X + T.xbase;
        float e[4][6];
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int h = 0; h < 3; h++) {
                const f32x2 v = *reinterpret_cast<const f32x2*>(xs + T.rr[r] * kW4RS + 2 * h);
                e[r][2 * h] = v[0];
                e[r][2 * h + 1] = v[1];
            }
        }
        float t[6], o[6];
#pragma unroll
        for (int j = 0; j < 6; j++)
            t[j] = __builtin_fmaf(T.kc[3], e[3][j],
                                  __builtin_fmaf(T.kc[2], e[2][j], __builtin_fmaf(T.kc[1], e[1][j], T.kc[0] * e[0][j])));
        w4_rowB(t, o);
        float* vs = lds + Geo::OffV + slot * Geo::V + T.vbase;
#pragma unroll
        for (int h = 0; h < 3; h++) *reinterpret_cast<f32x2*>(vs + 2 * h) = f32x2{o[2 * h], o[2 * h + 1]};
    };
    // ---- B operands straight from L2 into registers, one k-step ahead (no LDS image, no barrier)
    // one W4B per 4-channel sub-step
    struct W4BS {
        W4B<XG> s[SUB];
    };
    auto fetch_b = [&](W4BS& bq, auto g_c, int c) {
        if (decltype(g_c)::value && c >= nk) return;
        if (VS_W4_ABL == 5) return;
#pragma unroll
        for (int u = 0; u < SUB; u++) {
            const float* q = wb + (size_t)(SUB * c + u) * BK;
#pragma unroll
            for (int j = 0; j < (XG == 2 ? 4 : 3); j++) bq.s[u].q[j] = *reinterpret_cast<const f32x4*>(q + 4 * j);
            if constexpr (XG == 2) bq.s[u].r = *reinterpret_cast<const f32x2*>(q + 16);
        }
    };

    f32x4 acc[6 * RG];
#pragma unroll
    for (int x = 0; x < 6 * RG; x++) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: patches 0, 1 in LDS, patch 2 and the B operands of step 0 in registers, V 0 transformed
    W4BS bA, bB;
    fetch_b(bA, GY_{}, 0);
    fetch_x(GY_{}, 0);
    put_x(0, GY_{}, 0);
    fetch_x(GY_{}, 1);
    put_x(1, GY_{}, 1);
    fetch_x(GY_{}, 2);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SUB; u++) transform(u, 0, GY_{}, 0);
    __syncthreads();

    // A operands of sub-step s: V[RG xh + rr][4 s + lk][li][0..5]
    const int aoff = Geo::OffV + (lk * 16 + li) * 6 + RG * xh * (CH * 16 * 6);
    // k-step k on buffers P = k & 1 with B operands bc, loading the next step's into bn
    auto step = [&](auto par, auto g_c, int k, const W4BS& bc, W4BS& bn) {
        constexpr int P = decltype(par)::value;
        fetch_b(bn, g_c, k + 1);
#pragma unroll
        for (int sb = 0; sb < SUB; sb++) {
            const float* av = lds + aoff + P * Geo::V + sb * (4 * 16 * 6);
            f32x2 a2[RG][3];
#pragma unroll
            for (int rr = 0; rr < RG; rr++)
#pragma unroll
                for (int h = 0; h < 3; h++)
                    a2[rr][h] = *reinterpret_cast<const f32x2*>(av + rr * (CH * 16 * 6) + 2 * h);
#pragma unroll
            for (int rr = 0; rr < RG; rr++) {
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    if (VS_W4_ABL == 3) {
                        acc[6 * rr + j][0] += a2[rr][j >> 1][j & 1] * bc.s[sb][6 * rr + j];
                        continue;
                    }
                    acc[6 * rr + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2[rr][j >> 1][j & 1], bc.s[sb][6 * rr + j],
                                                                           acc[6 * rr + j], 0, 0, 0);
                }
                if (rr == 0) transform(sb, P ^ 1, g_c, k + 1);
                if (rr == 1 && sb == 0) {
                    put_x(P, g_c, k + 2);
                    fetch_x(g_c, k + 3);
                }
            }
        }
        if (VS_W4_ABL != 4) __syncthreads();  // V of k + 1 and the patch of k + 2 complete; the buffers of k free
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    int k = 0;
    for (; k + 4 < nk; k += 2) {  // a pair touches k-steps up to k + 4
        step(S0{}, GN_{}, k, bA, bB);
        step(S1{}, GN_{}, k + 1, bB, bA);
    }
    for (; k < nk; k += 2) {
        step(S0{}, GY_{}, k, bA, bB);
        if (k + 1 < nk) step(S1{}, GY_{}, k + 1, bB, bA);
    }

    // ---- epilogue: partial output transforms, the groups' parts added through LDS
    // acc[6 rr + j][r]: tile 4 lk + r, channel 16 cg + li, domain (RG xh + rr, j)
    float y[4][16];  // [r][4 p + q]
#pragma unroll
    for (int r = 0; r < 4; r++) {
        float R[RG][4];
#pragma unroll
        for (int rr = 0; rr < RG; rr++) {
            float m[6];
#pragma unroll
            for (int j = 0; j < 6; j++) m[j] = acc[6 * rr + j][r];
            w4_rowA(m, R[rr]);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if constexpr (XG == 2) {
                if (xh == 0) {  // rows 0, 1, 2: A^T columns (1,0,0,0), (1,1,1,1), (1,-1,1,-1)
                    const float s = R[1][q] + R[2][q], d = R[1][q] - R[2][q];
                    y[r][q] = R[0][q] + s;
                    y[r][4 + q] = d;
                    y[r][8 + q] = s;
                    y[r][12 + q] = d;
                } else {        // rows 3, 4, 5: (1,2,4,8), (1,-2,4,-8), (0,0,0,1)
                    const float s = R[0][q] + R[1][q], d = R[0][q] - R[1][q];
                    y[r][q] = s;
                    y[r][4 + q] = 2.0f * d;
                    y[r][8 + q] = 4.0f * s;
                    y[r][12 + q] = __builtin_fmaf(8.0f, d, R[2][q]);
                }
            } else {
                if (xh == 0) {         // rows 0, 1: (1,0,0,0), (1,1,1,1)
                    y[r][q] = R[0][q] + R[1][q];
                    y[r][4 + q] = R[1][q];
                    y[r][8 + q] = R[1][q];
                    y[r][12 + q] = R[1][q];
                } else if (xh == 1) {  // rows 2, 3: (1,-1,1,-1), (1,2,4,8)
                    y[r][q] = R[0][q] + R[1][q];
                    y[r][4 + q] = __builtin_fmaf(2.0f, R[1][q], -R[0][q]);
                    y[r][8 + q] = __builtin_fmaf(4.0f, R[1][q], R[0][q]);
                    y[r][12 + q] = __builtin_fmaf(8.0f, R[1][q], -R[0][q]);
                } else {               // rows 4, 5: (1,-2,4,-8), (0,0,0,1)
                    y[r][q] = R[0][q];
                    y[r][4 + q] = -2.0f * R[0][q];
                    y[r][8 + q] = 4.0f * R[0][q];
                    y[r][12 + q] = __builtin_fmaf(-8.0f, R[0][q], R[1][q]);
                }
            }
        }
    }
    // [cg][tile][16 px][16 ch] with tiles YS floats apart: a group's parts (4 YS = 16 mod 32, so lanes
    // lk = 0 and 1 of a ds_read_b32 group land on different banks), all written at once, added by group 0
    float* yp = lds;
    float* so = lds;  // then [pixel][64 ch]: the outputs (after every part has been read)
    if (xh > 0) {  // group xh's part into region xh - 1
        float* yq = yp + (xh - 1) * (64 * Geo::YS);
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int e = 0; e < 16; e++) yq[(cg * 16 + 4 * lk + r) * Geo::YS + e * 16 + li] = y[r][e];
    }
    __syncthreads();
    if (xh == 0) {  // group 0 adds the parts in group order
#pragma unroll
        for (int gx = 1; gx < XG; gx++) {
            const float* yq = yp + (gx - 1) * (64 * Geo::YS);
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int e = 0; e < 16; e++) y[r][e] += yq[(cg * 16 + 4 * lk + r) * Geo::YS + e * 16 + li];
        }
    }
    __syncthreads();
    if (xh == 0) {
        const int n = 16 * cg + li;
        const float bv = (nt * 64 + n < cout) ? bias[nt * 64 + n] : 0.0f;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int t = 4 * lk + r, ty = t >> 2, tx = t & 3;
            if constexpr (POOL) {
#pragma unroll
                for (int pp = 0; pp < 2; pp++)
#pragma unroll
                    for (int qq = 0; qq < 2; qq++) {
                        const int e0 = 8 * pp + 2 * qq;
                        float m = fmaxf(fmaxf(y[r][e0], y[r][e0 + 1]), fmaxf(y[r][e0 + 4], y[r][e0 + 5])) + bv;
                        m = m > 0.0f ? m : 0.0f;
                        so[((2 * ty + pp) * 8 + 2 * tx + qq) * 64 + n] = m;
                    }
            } else {
#pragma unroll
                for (int e = 0; e < 16; e++) {
                    float m = y[r][e] + bv;
                    m = m > 0.0f ? m : 0.0f;
                    so[((4 * ty + (e >> 2)) * 16 + 4 * tx + (e & 3)) * 64 + n] = m;
                }
            }
        }
    }
    __syncthreads();
    constexpr int NE = POOL ? 64 * 16 : 256 * 16;  // float4s: 64 (POOL) or 256 pixels x 16
#pragma unroll
    for (int e = tid; e < NE; e += NT) {
        const int pix = e >> 4, q = e & 15;
        const int n = nt * 64 + 4 * q;
        if (n >= cout) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(&so[pix * 64 + 4 * q]);
        if constexpr (POOL) {
            const int oy = (y0 >> 1) + (pix >> 3), ox = (x0 >> 1) + (pix & 7);
            if (oy >= (H >> 1) || ox >= (W >> 1)) continue;
            *reinterpret_cast<f32x4*>(out + (((size_t)b * (H >> 1) + oy) * (W >> 1) + ox) * out_cstride + out_coff + n) = v;
        } else {
            const int oy = y0 + (pix >> 4), ox = x0 + (pix & 15);
            if (oy >= H || ox >= W) continue;
            *reinterpret_cast<f32x4*>(out + (((size_t)b * H + oy) * W + ox) * out_cstride + out_coff + n) = v;
        }
    }
}

// F(4x4, 3x3) launch: SuperPoint layers (bias + ReLU; POOL: 2 x 2 max-pool; FUSE1A: conv1a fused).
// wa.wu = winograd4_weights(...) images; cin % 4 == 0, cout_pad % 64 == 0, cout % 4 == 0.
int wino4_launch(WinoArgs a, bool pool, bool fuse1a, hipStream_t s) {
    if (a.cin % 4 || a.cout_pad % 64 || a.cout % 4 || a.out_cstride % 4 || a.out_coff % 4 ||
        (!fuse1a && (a.in_cstride % 4 || a.in_coff % 4)) || (pool && ((a.H | a.W) & 1)) ||
        (fuse1a && (!a.w1a || a.cin != 64)) || a.res1 || a.res2 || a.splits > 1 || a.pre_relu || a.act != 1)
        return VS_ERR_ARG;
    a.nbx = (a.W + 15) / 16;
    a.nby = (a.H + 15) / 16;
    dim3 grid((unsigned)((long)a.B * a.nbx * a.nby * (a.cout_pad / 64)));
    // 4-channel k-steps; VS_WINO4_SUB=2 runs 8-channel steps (two MFMA sub-steps per barrier: 256 VGPRs,
    // measured 5 % slower over the network, profiles/r05e_wino4_sub_ab.txt)
    static const int sub = [] {
        const char* e = std::getenv("VS_WINO4_SUB");
        return e && e[0] == '2' ? 2 : 1;
    }();
    // VS_WINO4_XG=2: the 8-wave variant (domain halves) instead of the 12-wave one (row pairs)
    static const int xg_env = [] {
        const char* e = std::getenv("VS_WINO4_XG");
        return e && e[0] == '2' ? 2 : 3;
    }();
    const int xg = (sub == 1 && a.wu3) ? xg_env : 2;
#define VS_W4_LAUNCH(S_, X_)                                                                              \
    do {                                                                                                \
        if (pool && fuse1a)                                                                             \
            hipLaunchKernelGGL((k_wino4<true, true, S_, X_>), grid, dim3(256 * X_), 0, s, a);           \
        else if (pool)                                                                                  \
            hipLaunchKernelGGL((k_wino4<true, false, S_, X_>), grid, dim3(256 * X_), 0, s, a);          \
        else if (fuse1a)                                                                                \
            hipLaunchKernelGGL((k_wino4<false, true, S_, X_>), grid, dim3(256 * X_), 0, s, a);          \
        else                                                                                            \
            hipLaunchKernelGGL((k_wino4<false, false, S_, X_>), grid, dim3(256 * X_), 0, s, a);         \
    } while (0)
    if (sub == 2 && a.cin % 8 == 0) {
        VS_W4_LAUNCH(2, 2);
    } else if (xg == 3) {
        a.wu = a.wu3;
        VS_W4_LAUNCH(1, 3);
    } else {
        VS_W4_LAUNCH(1, 2);
    }
#undef VS_W4_LAUNCH
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
