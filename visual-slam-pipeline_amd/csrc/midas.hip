// midas.hip — DepthEstimator::estimate (reference src/DepthEstimator.cpp:39-112) on gfx950: the
// MiDaS v2.1-small network (the published midas_v21_small_256 topology: MidasNet_small with an
// EfficientNet-Lite3 encoder, features = 64, expand = True, non-negative output) as hand-written
// NHWC fp32 kernels, with the reference's pre- and post-processing around it.
//
//   pre   cv::resize(image, 256 x 256) (INTER_LINEAR, 8-bit fixed point: the SIMD row formula of
//         OpenCV's VResizeLinearVec_32s8u, which covers whole 256-pixel rows), convertTo(1/255),
//         (c - mean[c]) / std[c] per BGR channel as the reference writes it (:54-67)
//   net   encoder: TF-"same"-padded stem and depthwise stride-2 convolutions (timm tf_ models),
//         inverted residual blocks (1x1 expand + ReLU6, depthwise k x k + ReLU6, 1x1 project,
//         identity skip), BatchNorm folded into the convolutions; decoder: 3x3 "rn" projections,
//         four FeatureFusionBlock_custom (two residual conv units, x2 bilinear align_corners,
//         1x1 out conv), output head (3x3 conv, x2 bilinear, 3x3 conv + ReLU, 1x1 conv + ReLU)
//   post  cv::resize back to the frame size (INTER_LINEAR, float), minMaxLoc, (d - min) / (max -
//         min) when the range exceeds 1e-6 (:96-109)
//
// Dense convolutions (3x3 and 1x1, 99 % of the FLOPs) are implicit GEMMs on the fp32 matrix cores:
// a workgroup computes 64 output pixels x 64 output channels with v_mfma_f32_16x16x4_f32 (2 x 2
// waves, four 16 x 16 chains each) over K = k*k*Cin in chunks of 16 input channels of one tap,
// staged through LDS; bias, activation, an input-side ReLU (residual conv units) and up to two
// residual adds are fused.  Depthwise convolutions and the resizes are HBM/L2-bound elementwise
// kernels with channel-vectorised (float4) NHWC accesses.
//
// The reference never consumes this output (Frame::estimate_depth has no caller);
// it is built for BASELINE config[4].  Weights: seeded He-normal (no checkpoint ships with the
// reference, README.md:43) or a VSMW file written by tools/midas_to_vsmw.py from a MiDaS
// state_dict (BatchNorm folded there).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "vs_internal.h"
#include "../host/onnx_weights.h"

#include <functional>
#include <set>

namespace vs {
namespace midas {

constexpr int kIn = 256;  // Config::MIDAS_INPUT_SIZE (Config.h:45)
enum Kind : int { K_CONV = 0, K_DW = 1, K_UP = 2 };
enum Act : int { A_NONE = 0, A_RELU = 1, A_RELU6 = 2 };

// Canonical weights per layer: conv [cout][cin][k][k] then [cout] bias; depthwise [c][k][k] then
// [c] bias (BatchNorm folded).
struct LayerDef {
    int kind, cin, cout, k;
    bool bias;  // the scratch "rn" projections have none
};

struct Step {
    int kind;
    int layer = -1;
    int in = -1, out = -1, res1 = -1, res2 = -1;
    int H = 0, W = 0, C = 0, Ho = 0, Wo = 0, Co = 0;
    int k = 1, stride = 1, pad_t = 0, pad_l = 0;
    int act = A_NONE;
    bool pre_relu = false, align_corners = false;
    bool tf_same = false;  // TF "same" padding (an explicit Pad node in the ONNX export)
};

// The network as data: layer definitions (canonical weight order) and the step program over
// SSA tensors (tensor t has tdims[t] = {H, W, C}).
struct Net {
    std::vector<LayerDef> layers;
    std::vector<Step> steps;
    std::vector<int> tdims;  // 3 per tensor
    int input = -1, output = -1;

    int tensor(int H, int W, int C) {
        tdims.insert(tdims.end(), {H, W, C});
        return (int)tdims.size() / 3 - 1;
    }
    int Hof(int t) const { return tdims[3 * t]; }
    int Wof(int t) const { return tdims[3 * t + 1]; }
    int Cof(int t) const { return tdims[3 * t + 2]; }
    // TF "same" padding (timm Conv2dSame): total = max((ceil(i/s) - 1) s + k - i, 0), begin = total / 2
    static int same_begin(int i, int k, int s) {
        const int o = (i + s - 1) / s;
        const int total = std::max((o - 1) * s + k - i, 0);
        return total / 2;
    }
    int conv(int in, int cout, int k, int stride, int act, bool tf_same, bool bias = true, int res1 = -1,
             int res2 = -1, bool pre_relu = false) {
        Step st;
        st.kind = K_CONV;
        st.layer = (int)layers.size();
        layers.push_back({K_CONV, Cof(in), cout, k, bias});
        st.in = in;
        st.H = Hof(in), st.W = Wof(in), st.C = Cof(in);
        st.k = k, st.stride = stride;
        st.Ho = (st.H + stride - 1) / stride, st.Wo = (st.W + stride - 1) / stride, st.Co = cout;
        st.tf_same = tf_same;
        st.pad_t = tf_same ? same_begin(st.H, k, stride) : k / 2;
        st.pad_l = tf_same ? same_begin(st.W, k, stride) : k / 2;
        st.act = act, st.res1 = res1, st.res2 = res2, st.pre_relu = pre_relu;
        st.out = tensor(st.Ho, st.Wo, cout);
        steps.push_back(st);
        return st.out;
    }
    int dw(int in, int k, int stride) {
        Step st;
        st.kind = K_DW;
        st.layer = (int)layers.size();
        layers.push_back({K_DW, Cof(in), Cof(in), k, true});
        st.in = in;
        st.H = Hof(in), st.W = Wof(in), st.C = st.Co = Cof(in);
        st.k = k, st.stride = stride;
        st.Ho = (st.H + stride - 1) / stride, st.Wo = (st.W + stride - 1) / stride;
        st.tf_same = true;
        st.pad_t = same_begin(st.H, k, stride);
        st.pad_l = same_begin(st.W, k, stride);
        st.act = A_RELU6;
        st.out = tensor(st.Ho, st.Wo, st.C);
        steps.push_back(st);
        return st.out;
    }
    int up(int in, bool align_corners) {
        Step st;
        st.kind = K_UP;
        st.in = in;
        st.H = Hof(in), st.W = Wof(in), st.C = st.Co = Cof(in);
        st.Ho = 2 * st.H, st.Wo = 2 * st.W;
        st.align_corners = align_corners;
        st.out = tensor(st.Ho, st.Wo, st.C);
        steps.push_back(st);
        return st.out;
    }
    // timm InvertedResidual (exp ratio 6, no SE in the Lite models): 1x1 expand + BN + ReLU6,
    // depthwise + BN + ReLU6, 1x1 project + BN, identity skip when stride 1 and cin == cout
    int ir(int in, int cout, int k, int stride) {
        const int cin = Cof(in);
        int x = conv(in, cin * 6, 1, 1, A_RELU6, false);
        x = dw(x, k, stride);
        return conv(x, cout, 1, 1, A_NONE, false, true, stride == 1 && cin == cout ? in : -1);
    }
    // ResidualConvUnit_custom (bn = False): conv2(relu(conv1(relu(x)))) + x  [+ extra]
    int rcu(int x, int extra = -1) {
        const int c = Cof(x);
        const int h = conv(x, c, 3, 1, A_RELU, false, true, -1, -1, /*pre_relu=*/true);
        return conv(h, c, 3, 1, A_NONE, false, true, x, extra);
    }
    // FeatureFusionBlock_custom: out = xs0 [+ rcu1(xs1)]; rcu2; x2 bilinear (align_corners); 1x1 out
    int fusion(int xs0, int xs1, int out_ch) {
        int o = xs1 >= 0 ? rcu(xs1, xs0) : xs0;
        o = rcu(o);
        o = up(o, true);
        return conv(o, out_ch, 1, 1, A_NONE, false);
    }

    void build() {
        input = tensor(kIn, kIn, 3);
        // EfficientNet-Lite3 (tf_efficientnet_lite3): stem 32, stages
        // DS(24) | IR k3 s2 32 x3 | IR k5 s2 48 x3 | IR k3 s2 96 x5 | IR k5 s1 136 x5 | IR k5 s2 232 x6 | IR k3 s1 384 x1
        int x = conv(input, 32, 3, 2, A_RELU6, true);
        x = dw(x, 3, 1);  // DepthwiseSeparable: dw 3x3 + BN + ReLU6, pw 1x1 + BN (no act, no skip 32 -> 24)
        x = conv(x, 24, 1, 1, A_NONE, false);
        struct Stage {
            int c, k, s, n;
        };
        const Stage stages[6] = {{32, 3, 2, 3}, {48, 5, 2, 3}, {96, 3, 2, 5}, {136, 5, 1, 5}, {232, 5, 2, 6}, {384, 3, 1, 1}};
        int skip[4];
        for (int si = 0; si < 6; si++) {
            for (int r = 0; r < stages[si].n; r++) x = ir(x, stages[si].c, stages[si].k, r == 0 ? stages[si].s : 1);
            if (si == 0) skip[0] = x;  // layer1 = stem + blocks[0:2]   (32 @ 64^2)
            if (si == 1) skip[1] = x;  // layer2 = blocks[2:3]          (48 @ 32^2)
            if (si == 3) skip[2] = x;  // layer3 = blocks[3:5]          (136 @ 16^2)
            if (si == 5) skip[3] = x;  // layer4 = blocks[5:9]          (384 @ 8^2)
        }
        // scratch.layerN_rn: 3x3, no bias, to 64 / 128 / 256 / 512 (expand)
        const int rn1 = conv(skip[0], 64, 3, 1, A_NONE, false, false);
        const int rn2 = conv(skip[1], 128, 3, 1, A_NONE, false, false);
        const int rn3 = conv(skip[2], 256, 3, 1, A_NONE, false, false);
        const int rn4 = conv(skip[3], 512, 3, 1, A_NONE, false, false);
        const int p4 = fusion(rn4, -1, 256);
        const int p3 = fusion(p4, rn3, 128);
        const int p2 = fusion(p3, rn2, 64);
        const int p1 = fusion(p2, rn1, 64);  // refinenet1: no expand
        // output_conv: 3x3 64 -> 32, x2 bilinear (align_corners False), 3x3 32 -> 32 + ReLU, 1x1 32 -> 1 + ReLU
        int o = conv(p1, 32, 3, 1, A_NONE, false);
        o = up(o, false);
        o = conv(o, 32, 3, 1, A_RELU, false);
        output = conv(o, 1, 1, 1, A_RELU, false);
    }
    size_t num_params() const {
        size_t n = 0;
        for (const auto& L : layers)
            n += (size_t)(L.kind == K_DW ? L.cout * L.k * L.k : L.cout * L.cin * L.k * L.k) + (L.bias ? L.cout : 0);
        return n;
    }
    double flops() const {  // per frame (2 x MACs of the convolutions)
        double f = 0;
        for (const auto& st : steps) {
            if (st.kind == K_CONV) f += 2.0 * st.Ho * st.Wo * st.Co * st.C * st.k * st.k;
            if (st.kind == K_DW) f += 2.0 * st.Ho * st.Wo * st.C * st.k * st.k;
        }
        return f;
    }
};

const Net& net() {
    static Net n = [] {
        Net m;
        m.build();
        return m;
    }();
    return n;
}

// ---- kernels --------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float activate(float v, int act) {
    if (act == A_RELU) return v > 0.f ? v : 0.f;
    if (act == A_RELU6) return v > 0.f ? (v < 6.f ? v : 6.f) : 0.f;
    return v;
}

// OpenCV resize coefficient (resizeGeneric_, INTER_LINEAR): f = (float)((d + 0.5) * scale - 0.5),
// s = floor(f), f -= s, clamped to the source; fixed point saturate_cast<short>(f * 2048)
struct Lin {
    int s0, s1;
    float f;
};
__device__ __forceinline__ Lin lin_coef(int d, double scale, int n) {
    float f = (float)((d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) {
        f = 0.f;
        s = 0;
    }
    if (s >= n - 1) {
        f = 0.f;
        s = n - 1;
    }
    return {s, s + 1 < n ? s + 1 : n - 1, f};
}
__device__ __forceinline__ int fix11(float v) {  // saturate_cast<short>(v * INTER_RESIZE_COEF_SCALE)
    return (int)rintf(v * 2048.0f);
}

// pre: B BGR u8 frames (h x w) -> B x 256 x 256 x 3 fp32, normalised (DepthEstimator.cpp:54-67)
__global__ __launch_bounds__(256) void k_mid_pre(const uint8_t* __restrict__ bgr, int h, int w, int B,
                                                 float* __restrict__ out) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= B * kIn * kIn) return;
    const int b = idx / (kIn * kIn), p = idx - b * kIn * kIn, y = p / kIn, x = p - y * kIn;
    const Lin cx = lin_coef(x, 1.0 / ((double)kIn / w), w), cy = lin_coef(y, 1.0 / ((double)kIn / h), h);
    const int a0 = fix11(1.f - cx.f), a1 = fix11(cx.f), b0 = fix11(1.f - cy.f), b1 = fix11(cy.f);
    const uint8_t* im = bgr + (size_t)b * h * w * 3;
    const uint8_t* r0 = im + (size_t)cy.s0 * w * 3;
    const uint8_t* r1 = im + (size_t)cy.s1 * w * 3;
    // (float)(1/255.0); 1/std and -mean/std in double, then float (MatExpr -> convertTo, fma)
    const float mean[3] = {0.485f, 0.456f, 0.406f}, sd[3] = {0.229f, 0.224f, 0.225f};
    float* o = out + (size_t)idx * 3;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const int h0 = r0[cx.s0 * 3 + c] * a0 + r0[cx.s1 * 3 + c] * a1;
        const int h1 = r1[cx.s0 * 3 + c] * a0 + r1[cx.s1 * 3 + c] * a1;
        // VResizeLinearVec_32s8u: (mulhi16(h0 >> 4, b0) + mulhi16(h1 >> 4, b1) + 2) >> 2, saturated
        int v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
        const float f = (float)v * (float)(1.0 / 255.0);
        const double is = 1.0 / (double)sd[c];
        o[c] = fmaf(f, (float)is, (float)(-(double)mean[c] * is));
    }
}

// Dense convolution as an implicit GEMM on the fp32 matrix cores (see file header).
// in [B][H][W][C], w [k*k][C][CoP] (CoP = Co rounded up to 64), out / res [B][Ho][Wo][Co].
struct ConvArgs {
    const float* in;
    const float* w;
    const float* bias;  // nullptr: none
    const float* res1;
    const float* res2;
    float* out;
    float* part;  // split-K: raw partial sums [split][pixel][Co] instead of out (k_mid_splitk finishes)
    int B, H, W, C, Ho, Wo, Co, CoP, k, stride, pad_t, pad_l, act, pre_relu;
    int splits;   // K splits (blockIdx.z), 1 = none
};

constexpr int kCT = 64;  // output pixels x channels per workgroup
constexpr int kCK = 16;  // input channels per K chunk
constexpr int kAS = kCK + 4;  // LDS row stride of the pixel operand (floats)
constexpr int kOS = kCT + 4;  // LDS row stride of the staged output tile (floats)
static_assert(kCT * kOS <= 4 * kCT * kAS, "output tile must fit the operand buffers");

__global__ __launch_bounds__(256) void k_mid_conv(ConvArgs a) {
    // sA [2][pixel][16 k] (k permuted for float4 fragments), double-buffered; sB [2][cout][16 k]; after
    // the K loop the same LDS holds the output tile [pixel][64 channels] (row stride kOS)
    __shared__ __attribute__((aligned(16))) float smem[4 * kCT * kAS];
    float(*sA)[kCT * kAS] = reinterpret_cast<float(*)[kCT * kAS]>(smem);
    float(*sB)[kCT * kAS] = reinterpret_cast<float(*)[kCT * kAS]>(smem + 2 * kCT * kAS);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, li = lane & 15, lg = lane >> 4;
    const int npix = a.B * a.Ho * a.Wo;
    const int p0 = blockIdx.x * kCT, n0 = blockIdx.y * kCT;
    // staging roles.  Pixel operand: pixel r = tid / 4 reads 4 consecutive channels (quad q = tid % 4),
    // so 4 neighbouring threads cover 16 contiguous channels of one pixel.  Weight operand: cout
    // co = tid % 64 for channel quad kq = tid / 64, so neighbouring threads read neighbouring couts
    // of one [tap][channel] row (coalesced).
    const int r = tid >> 2, q = tid & 3;
    const int co = tid & 63, kq = tid >> 6;
    const int gp = p0 + r;
    int b = 0, oy = 0, ox = 0;
    const bool pvalid = gp < npix;
    if (pvalid) {
        b = gp / (a.Ho * a.Wo);
        const int rem = gp - b * a.Ho * a.Wo;
        oy = rem / a.Wo;
        ox = rem - oy * a.Wo;
    }
    const bool vec = (a.C & 3) == 0;
    const int wq = wv & 1, wt = wv >> 1;  // wave: pixels wq*32.., couts wt*32..
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nchunk = (a.C + kCK - 1) / kCK;
    const int T = a.k * a.k * nchunk;  // (tap, channel chunk) steps
    // split-K: this workgroup's contiguous range of steps
    const int t0 = (int)((long)T * blockIdx.z / a.splits), t1 = (int)((long)T * (blockIdx.z + 1) / a.splits);
    float v[4], u[4];
    // operands of step t into registers (global loads; issued one step ahead of their MFMAs)
    auto fetch = [&](int t) {
        const int tap = t / nchunk, ch = t - tap * nchunk;
        const int ky = tap / a.k, kx = tap - ky * a.k;
        const int iy = oy * a.stride - a.pad_t + ky, ix = ox * a.stride - a.pad_l + kx;
        const bool inb = pvalid && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const float* src = a.in + (((size_t)b * a.H + (inb ? iy : 0)) * a.W + (inb ? ix : 0)) * a.C;
        const int c0 = ch * kCK + 4 * q;
        if (vec) {
            const float4 t4 = (inb && c0 < a.C) ? *reinterpret_cast<const float4*>(src + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
            v[0] = t4.x;
            v[1] = t4.y;
            v[2] = t4.z;
            v[3] = t4.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = (inb && c0 + j < a.C) ? src[c0 + j] : 0.f;
        }
        if (a.pre_relu)
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = v[j] > 0.f ? v[j] : 0.f;
        const int cw = ch * kCK + 4 * kq;
#pragma unroll
        for (int j = 0; j < 4; j++) u[j] = (cw + j < a.C) ? a.w[((size_t)tap * a.C + cw + j) * a.CoP + n0 + co] : 0.f;
    };
    // k = 4 q + j -> position 4 j + q (a lane group g reads k = g, 4 + g, 8 + g, 12 + g)
    auto stage = [&](int buf) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            sA[buf][r * kAS + 4 * j + q] = v[j];
            sB[buf][co * kAS + 4 * j + kq] = u[j];
        }
    };
    fetch(t0);
    stage(t0 & 1);
    __syncthreads();
    for (int t = t0; t < t1; t++) {
        const int cur = t & 1;
        if (t + 1 < t1) fetch(t + 1);
        float4 fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; i++) {
            fa[i] = *reinterpret_cast<const float4*>(&sA[cur][(wq * 32 + 16 * i + li) * kAS + 4 * lg]);
            fb[i] = *reinterpret_cast<const float4*>(&sB[cur][(wt * 32 + 16 * i + li) * kAS + 4 * lg]);
        }
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int m = 0; m < 2; m++)
                    acc[i][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i][j], fb[m][j], acc[i][m], 0, 0, 0);
        // the other buffer was last read in step t - 1, which every wave finished before the
        // barrier that ended it
        if (t + 1 < t1) stage(cur ^ 1);
        __syncthreads();
    }
    if ((a.Co & 3) == 0) {
        // through LDS so that every global access is a float4 of 4 channels and a pixel's 64 channels
        // form whole 256-byte rows (the direct stores below write 64-byte pieces per pixel: partial
        // lines on the HBM-bound expand / project layers).  The K loop's last barrier freed the LDS.
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int m = 0; m < 2; m++)
#pragma unroll
                for (int e = 0; e < 4; e++) smem[(wq * 32 + 16 * i + 4 * lg + e) * kOS + wt * 32 + 16 * m + li] = acc[i][m][e];
        __syncthreads();
        float* dst = a.part ? a.part + (size_t)blockIdx.z * npix * a.Co : a.out;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int idx = tid + 256 * j, px = idx >> 4, c4 = 4 * (idx & 15);
            const int gpix = p0 + px, c = n0 + c4;
            if (gpix >= npix || c >= a.Co) continue;
            f32x4 ov = *reinterpret_cast<const f32x4*>(&smem[px * kOS + c4]);
            const size_t o = (size_t)gpix * a.Co + c;
            if (!a.part) {
                const f32x4 bv = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
                f32x4 r1 = {0.f, 0.f, 0.f, 0.f}, r2 = {0.f, 0.f, 0.f, 0.f};
                if (a.res1) r1 = *reinterpret_cast<const f32x4*>(a.res1 + o);
                if (a.res2) r2 = *reinterpret_cast<const f32x4*>(a.res2 + o);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    float t = activate(ov[e] + bv[e], a.act);
                    if (a.res1) t = t + r1[e];
                    if (a.res2) t = r2[e] + t;
                    ov[e] = t;
                }
            }
            *reinterpret_cast<f32x4*>(dst + o) = ov;
        }
        return;
    }
    if (a.part) {  // split-K partials, finished by k_mid_splitk
        float* dst = a.part + (size_t)blockIdx.z * npix * a.Co;
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int m = 0; m < 2; m++) {
                const int co = n0 + wt * 32 + 16 * m + li;
                if (co >= a.Co) continue;
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const int gpix = p0 + wq * 32 + 16 * i + 4 * lg + e;
                    if (gpix < npix) dst[(size_t)gpix * a.Co + co] = acc[i][m][e];
                }
            }
        return;
    }
    // D[pixel 4 lg + e][cout li] of fragment (i, m)
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const int co = n0 + wt * 32 + 16 * m + li;
            if (co >= a.Co) continue;
            const float bv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int gpix = p0 + wq * 32 + 16 * i + 4 * lg + e;
                if (gpix >= npix) continue;
                const size_t o = (size_t)gpix * a.Co + co;
                float v = activate(acc[i][m][e] + bv, a.act);
                if (a.res1) v = v + a.res1[o];
                if (a.res2) v = a.res2[o] + v;
                a.out[o] = v;
            }
        }
}

// 1 x 1 convolution to a single output channel (the head's last layer, 32 -> 1 at the full
// 256 x 256): one thread per pixel, a plain dot product over the channels.  On the implicit GEMM it
// would occupy a 64-wide output tile for one channel (63/64 of the MFMA work padding).  The
// workgroup's 256 pixel rows (C floats each, contiguous in HBM) are staged through LDS with
// coalesced float4 loads, rows padded to C + 4 floats so that the per-pixel float4 reads are
// conflict-free (round 3: direct per-thread row loads at a 4C-byte lane stride reached 0.9 TB/s).
constexpr int kCo1MaxC = 32;
__global__ __launch_bounds__(256) void k_mid_conv_co1(ConvArgs a) {
    __shared__ float sx[256 * (kCo1MaxC + 4)];
    const int tid = threadIdx.x;
    const int npix = a.B * a.Ho * a.Wo;
    const int p0 = blockIdx.x * 256, p = p0 + tid;
    const int C = a.C, C4 = C >> 2, RS = C + 4;
    const int nv = (min(256, npix - p0)) * C4;  // float4s of this workgroup's rows
    const float4* src = reinterpret_cast<const float4*>(a.in + (size_t)p0 * C);
    for (int i = tid; i < nv; i += 256) {
        const int r = i / C4, q = i - r * C4;
        *reinterpret_cast<float4*>(&sx[r * RS + 4 * q]) = src[i];
    }
    __syncthreads();
    if (p >= npix) return;
    float s = 0.f;
    auto term = [&](float t, int c) {
        if (a.pre_relu) t = t > 0.f ? t : 0.f;
        s = fmaf(t, a.w[(size_t)c * a.CoP], s);
    };
    for (int c = 0; c < C; c += 4) {
        const float4 t = *reinterpret_cast<const float4*>(&sx[tid * RS + c]);
        term(t.x, c);
        term(t.y, c + 1);
        term(t.z, c + 2);
        term(t.w, c + 3);
    }
    float v = activate(s + (a.bias ? a.bias[0] : 0.f), a.act);
    if (a.res1) v = v + a.res1[p];
    if (a.res2) v = a.res2[p] + v;
    a.out[p] = v;
}

// The stem (3 -> 32, 3 x 3, stride 2 at 256^2): K = 27 would fill 27 of the implicit GEMM's 16 x 9
// K slots per tap and 8192 workgroups of 9 barriers each; here a thread computes one output pixel's
// 32 channels on the vector ALUs (weights broadcast from LDS, the 3 x 3 x C window from L1) and the
// workgroup's 256 x 32 outputs leave through LDS as coalesced float4 rows.  C <= 4, Co == 32.
constexpr int kStemCo = 32, kStemMaxC = 4;
__global__ __launch_bounds__(256) void k_mid_stem(ConvArgs a) {
    __shared__ float sw[9 * kStemMaxC * kStemCo];
    __shared__ __attribute__((aligned(16))) float so[256 * (kStemCo + 4)];
    const int tid = threadIdx.x, C = a.C, kk = a.k * a.k;
    for (int i = tid; i < kk * C * kStemCo; i += 256) {
        const int co = i % kStemCo, tc = i / kStemCo;  // tc = tap * C + channel
        sw[i] = a.w[(size_t)tc * a.CoP + co];
    }
    __syncthreads();
    const int npix = a.B * a.Ho * a.Wo, p0 = blockIdx.x * 256, p = p0 + tid;
    float acc[kStemCo];
#pragma unroll
    for (int co = 0; co < kStemCo; co++) acc[co] = 0.f;
    if (p < npix) {
        const int b = p / (a.Ho * a.Wo), rem = p - b * a.Ho * a.Wo, oy = rem / a.Wo, ox = rem - oy * a.Wo;
        for (int ky = 0; ky < a.k; ky++) {
            const int iy = oy * a.stride - a.pad_t + ky;
            if (iy < 0 || iy >= a.H) continue;
            for (int kx = 0; kx < a.k; kx++) {
                const int ix = ox * a.stride - a.pad_l + kx;
                if (ix < 0 || ix >= a.W) continue;
                const float* src = a.in + (((size_t)b * a.H + iy) * a.W + ix) * C;
                const float* wt = sw + (ky * a.k + kx) * C * kStemCo;
                for (int c = 0; c < C; c++) {
                    const float x = src[c];
#pragma unroll
                    for (int co = 0; co < kStemCo; co++) acc[co] = fmaf(x, wt[c * kStemCo + co], acc[co]);
                }
            }
        }
    }
#pragma unroll
    for (int co = 0; co < kStemCo; co++) so[tid * (kStemCo + 4) + co] = activate(acc[co] + (a.bias ? a.bias[co] : 0.f), a.act);
    __syncthreads();
    const int nv = min(256, npix - p0) * (kStemCo / 4);
    f32x4* dst = reinterpret_cast<f32x4*>(a.out + (size_t)p0 * kStemCo);
    for (int i = tid; i < nv; i += 256) {
        const int r = i / (kStemCo / 4), q = i - r * (kStemCo / 4);
        dst[i] = *reinterpret_cast<const f32x4*>(&so[r * (kStemCo + 4) + 4 * q]);
    }
}

// Split-K finish: out = epilogue(sum of the S partials in split order), the epilogue of
// k_mid_conv (bias, activation, then the residual adds); Co % 4 == 0, 4 channels per thread.
__global__ __launch_bounds__(256) void k_mid_splitk(ConvArgs a) {
    const int npix = a.B * a.Ho * a.Wo, C4 = a.Co >> 2;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)npix * C4) return;
    const int c = 4 * (int)(idx % C4);
    const float4* P = reinterpret_cast<const float4*>(a.part);
    const size_t plane = (size_t)npix * C4;
    float4 acc = P[idx];
    for (int z = 1; z < a.splits; z++) {
        const float4 t = P[z * plane + idx];
        acc.x += t.x;
        acc.y += t.y;
        acc.z += t.z;
        acc.w += t.w;
    }
    float o[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int e = 0; e < 4; e++) {
        float v = activate(o[e] + (a.bias ? a.bias[c + e] : 0.f), a.act);
        if (a.res1) v = v + a.res1[4 * idx + e];
        if (a.res2) v = a.res2[4 * idx + e] + v;
        o[e] = v;
    }
    reinterpret_cast<float4*>(a.out)[idx] = make_float4(o[0], o[1], o[2], o[3]);
}

// Depthwise k x k, stride s, TF-same padding, bias + ReLU6; one thread per (pixel, 4 channels).
// (Round 3: four outputs per thread sharing each kernel row's loads measured the same, 1.02 ms per
// 32-frame batch; not kept.)
__global__ __launch_bounds__(256) void k_mid_dw(const float* __restrict__ in, const float* __restrict__ w,
                                                const float* __restrict__ bias, float* __restrict__ out, int B, int H,
                                                int W, int C, int Ho, int Wo, int k, int stride, int pad_t, int pad_l) {
    const int C4 = C / 4;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)B * Ho * Wo * C4) return;
    const int c4 = (int)(idx % C4);
    const long pix = idx / C4;
    const int ox = (int)(pix % Wo), oy = (int)((pix / Wo) % Ho), b = (int)(pix / ((long)Wo * Ho));
    float4 s = reinterpret_cast<const float4*>(bias)[c4];
    for (int ky = 0; ky < k; ky++) {
        const int iy = oy * stride - pad_t + ky;
        if (iy < 0 || iy >= H) continue;
        for (int kx = 0; kx < k; kx++) {
            const int ix = ox * stride - pad_l + kx;
            if (ix < 0 || ix >= W) continue;
            const float4 v = reinterpret_cast<const float4*>(in + (((size_t)b * H + iy) * W + ix) * C)[c4];
            const float4 g = reinterpret_cast<const float4*>(w + (size_t)(ky * k + kx) * C)[c4];
            s.x = fmaf(v.x, g.x, s.x);
            s.y = fmaf(v.y, g.y, s.y);
            s.z = fmaf(v.z, g.z, s.z);
            s.w = fmaf(v.w, g.w, s.w);
        }
    }
    s.x = activate(s.x, A_RELU6);
    s.y = activate(s.y, A_RELU6);
    s.z = activate(s.z, A_RELU6);
    s.w = activate(s.w, A_RELU6);
    reinterpret_cast<float4*>(out)[idx] = s;
}

// Stride-1 depthwise K x K for PX consecutive output pixels of a row per thread (4 channels): each
// kernel row's K weights and PX + K - 1 input pixels are loaded once for the PX outputs (the
// per-output kernel above re-reads 2 K^2 float4 per output: L2-bandwidth-bound on the 16^2 / 8^2
// layers).  Every output's taps are summed in the same (ky, kx) order as k_mid_dw.
// ST = 2: the stride-2 layers, PX outputs from 2 PX + K - 2 input pixels per kernel row.
template <int K, int PX, int ST = 1>
__global__ __launch_bounds__(256) void k_mid_dw_row(const float* __restrict__ in, const float* __restrict__ w,
                                                    const float* __restrict__ bias, float* __restrict__ out, int B,
                                                    int H, int W, int C, int Ho, int Wo, int pad_t, int pad_l) {
    constexpr int NR = ST * (PX - 1) + K;  // input pixels per kernel row
    const int C4 = C / 4, nxg = (Wo + PX - 1) / PX;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)B * Ho * nxg * C4) return;
    const int c4 = (int)(idx % C4);
    const long g = idx / C4;
    const int xg = (int)(g % nxg), oy = (int)((g / nxg) % Ho), b = (int)(g / ((long)nxg * Ho));
    const int x0 = xg * PX;
    const float4* in4 = reinterpret_cast<const float4*>(in);
    const float4* w4 = reinterpret_cast<const float4*>(w);
    const float4 bv = reinterpret_cast<const float4*>(bias)[c4];
    float4 acc[PX];
#pragma unroll
    for (int p = 0; p < PX; p++) acc[p] = bv;
    for (int ky = 0; ky < K; ky++) {
        const int iy = oy * ST - pad_t + ky;
        if (iy < 0 || iy >= H) continue;
        float4 wr[K], row[NR];
#pragma unroll
        for (int kx = 0; kx < K; kx++) wr[kx] = w4[(size_t)(ky * K + kx) * C4 + c4];
        const size_t rbase = ((size_t)b * H + iy) * W;
#pragma unroll
        for (int j = 0; j < NR; j++) {
            const int ix = x0 * ST - pad_l + j;
            row[j] = (ix >= 0 && ix < W) ? in4[(rbase + ix) * C4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int p = 0; p < PX; p++)
#pragma unroll
            for (int kx = 0; kx < K; kx++) {
                // taps outside the image are skipped (not added as zero), as in k_mid_dw
                const int ix = (x0 + p) * ST - pad_l + kx;
                if (ix < 0 || ix >= W) continue;
                acc[p].x = fmaf(row[ST * p + kx].x, wr[kx].x, acc[p].x);
                acc[p].y = fmaf(row[ST * p + kx].y, wr[kx].y, acc[p].y);
                acc[p].z = fmaf(row[ST * p + kx].z, wr[kx].z, acc[p].z);
                acc[p].w = fmaf(row[ST * p + kx].w, wr[kx].w, acc[p].w);
            }
    }
    float4* o4 = reinterpret_cast<float4*>(out) + (((size_t)b * Ho + oy) * Wo) * C4 + c4;
#pragma unroll
    for (int p = 0; p < PX; p++) {
        if (x0 + p >= Wo) continue;
        float4 v = acc[p];
        v.x = activate(v.x, A_RELU6);
        v.y = activate(v.y, A_RELU6);
        v.z = activate(v.z, A_RELU6);
        v.w = activate(v.w, A_RELU6);
        o4[(size_t)(x0 + p) * C4] = v;
    }
}

// x2 bilinear upsampling (torch interpolate, mode "bilinear"), NHWC, 4 channels per thread.
__global__ __launch_bounds__(256) void k_mid_up(const float* __restrict__ in, float* __restrict__ out, int B, int H,
                                                int W, int C, int align_corners) {
    const int C4 = C / 4, Ho = 2 * H, Wo = 2 * W;
    const long idx = (long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long)B * Ho * Wo * C4) return;
    const int c4 = (int)(idx % C4);
    const long pix = idx / C4;
    const int ox = (int)(pix % Wo), oy = (int)((pix / Wo) % Ho), b = (int)(pix / ((long)Wo * Ho));
    float sy, sx;
    if (align_corners) {
        sy = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) * oy : 0.f;
        sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) * ox : 0.f;
    } else {
        sy = fmaxf((oy + 0.5f) * 0.5f - 0.5f, 0.f);
        sx = fmaxf((ox + 0.5f) * 0.5f - 0.5f, 0.f);
    }
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
    const float ly = sy - y0, lx = sx - x0, hy = 1.f - ly, hx = 1.f - lx;
    const float4* p = reinterpret_cast<const float4*>(in) + (size_t)b * H * W * C4;
    const float4 v00 = p[((size_t)y0 * W + x0) * C4 + c4], v01 = p[((size_t)y0 * W + x1) * C4 + c4];
    const float4 v10 = p[((size_t)y1 * W + x0) * C4 + c4], v11 = p[((size_t)y1 * W + x1) * C4 + c4];
    float4 o;
    o.x = hy * (hx * v00.x + lx * v01.x) + ly * (hx * v10.x + lx * v11.x);
    o.y = hy * (hx * v00.y + lx * v01.y) + ly * (hx * v10.y + lx * v11.y);
    o.z = hy * (hx * v00.z + lx * v01.z) + ly * (hx * v10.z + lx * v11.z);
    o.w = hy * (hx * v00.w + lx * v01.w) + ly * (hx * v10.w + lx * v11.w);
    reinterpret_cast<float4*>(out)[idx] = o;
}

// post: the 1-channel 256^2 output resized to h x w (float INTER_LINEAR, the same coefficients
// without fixed point) with per-block min / max partials.
__global__ __launch_bounds__(256) void k_mid_post(const float* __restrict__ d, int B, int h, int w,
                                                  float* __restrict__ out, float* __restrict__ part) {
    __shared__ float smin[256], smax[256];
    const int b = blockIdx.y;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    float mn = INFINITY, mx = -INFINITY;
    if (idx < h * w) {
        const int y = idx / w, x = idx - y * w;
        const Lin cx = lin_coef(x, 1.0 / ((double)w / kIn), kIn), cy = lin_coef(y, 1.0 / ((double)h / kIn), kIn);
        const float* s = d + (size_t)b * kIn * kIn;
        const float a0 = 1.f - cx.f, a1 = cx.f, b0 = 1.f - cy.f, b1 = cy.f;
        const float r0 = s[cy.s0 * kIn + cx.s0] * a0 + s[cy.s0 * kIn + cx.s1] * a1;
        const float r1 = s[cy.s1 * kIn + cx.s0] * a0 + s[cy.s1 * kIn + cx.s1] * a1;
        const float v = r0 * b0 + r1 * b1;
        out[(size_t)b * h * w + idx] = v;
        mn = mx = v;
    }
    smin[threadIdx.x] = mn;
    smax[threadIdx.x] = mx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + o]);
            smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + o]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[((size_t)b * gridDim.x + blockIdx.x) * 2] = smin[0];
        part[((size_t)b * gridDim.x + blockIdx.x) * 2 + 1] = smax[0];
    }
}

// minMaxLoc over the partials, then (d - min) / (max - min) when max - min > 1e-6 (convertTo with
// alpha = 1 / range, beta = -min / range, as the MatExpr evaluates): one workgroup row per frame.
__global__ __launch_bounds__(256) void k_mid_norm(float* __restrict__ out, const float* __restrict__ part, int nparts,
                                                  int n) {
    __shared__ float smin[256], smax[256];
    const int b = blockIdx.y;
    float mn = INFINITY, mx = -INFINITY;
    for (int i = threadIdx.x; i < nparts; i += 256) {
        mn = fminf(mn, part[((size_t)b * nparts + i) * 2]);
        mx = fmaxf(mx, part[((size_t)b * nparts + i) * 2 + 1]);
    }
    smin[threadIdx.x] = mn;
    smax[threadIdx.x] = mx;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            smin[threadIdx.x] = fminf(smin[threadIdx.x], smin[threadIdx.x + o]);
            smax[threadIdx.x] = fmaxf(smax[threadIdx.x], smax[threadIdx.x + o]);
        }
        __syncthreads();
    }
    const double lo = smin[0], hi = smax[0];
    if (!(hi - lo > 1e-6)) return;
    const double sc = 1.0 / (hi - lo);
    const float al = (float)sc, be = (float)(-lo * sc);
    float* o = out + (size_t)b * n;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) o[i] = fmaf(o[i], al, be);
}

// ---- weights --------------------------------------------------------------------------------
std::vector<float> synth(uint64_t seed) {
    uint64_t st = seed;
    auto next = [&]() {
        uint64_t z = (st += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    auto normal = [&]() {
        double u1 = ((next() >> 11) + 1) * (1.0 / 9007199254740992.0);
        double u2 = (next() >> 11) * (1.0 / 9007199254740992.0);
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    };
    std::vector<float> w;
    for (const auto& L : net().layers) {
        const int fan_in = (L.kind == K_DW ? 1 : L.cin) * L.k * L.k;
        const double sd = std::sqrt(2.0 / fan_in);
        const size_t nw = (size_t)(L.kind == K_DW ? L.cout : L.cout * L.cin) * L.k * L.k;
        for (size_t i = 0; i < nw; i++) w.push_back((float)(normal() * sd));
        if (L.bias)
            for (int i = 0; i < L.cout; i++) w.push_back((float)(normal() * 0.05));
    }
    return w;
}

// The canonical weights from an ONNX export of midas_v21_small_256: the graph's convolutions in
// node order (BatchNormalization folded) checked layer by layer against the network's definition.
bool from_onnx(const char* path, std::vector<float>& w, std::string& err) {
    const Net& N = net();
    std::vector<vs_onnx::LayerSpec> spec(N.layers.size());
    // structural input of every layer: the layers whose outputs reach its data input through the
    // step program (residual adds and upsampling included), -1 for the network input
    std::vector<int> producer(N.tdims.size() / 3, -2);  // tensor -> producing step
    for (size_t i = 0; i < N.steps.size(); i++) producer[N.steps[i].out] = (int)i;
    std::function<void(int, std::set<int>&)> sources = [&](int t, std::set<int>& acc) {
        if (t == N.input) {
            acc.insert(-1);
            return;
        }
        const Step& st = N.steps[producer[t]];
        if (st.layer >= 0) {
            acc.insert(st.layer);
            if (st.res1 >= 0) sources(st.res1, acc);
            if (st.res2 >= 0) sources(st.res2, acc);
        } else {
            sources(st.in, acc);  // upsampling
        }
    };
    for (const Step& st : N.steps) {
        if (st.layer < 0) continue;
        const LayerDef& L = N.layers[st.layer];
        vs_onnx::LayerSpec& sp = spec[st.layer];
        sp.depthwise = L.kind == K_DW;
        sp.cin = L.cin, sp.cout = L.cout, sp.k = L.k, sp.stride = st.stride, sp.bias = L.bias;
        sp.tf_same = st.tf_same;
        sources(st.in, sp.from);
    }
    vs_onnx::Model model;
    if (!vs_onnx::load(path, model, err)) return false;
    if (!vs_onnx::midas_weights(model, spec, w, err)) return false;
    if (w.size() != N.num_params()) {
        err = "MiDaS graph: parameter count mismatch";
        return false;
    }
    return true;
}

struct DevW {
    float* w = nullptr;
    float* b = nullptr;
    int cop = 0;
    float* wu = nullptr;  // 3x3 convs: Winograd F(2x2, 3x3) weights (stride-1 steps run k_wino3)
    float* bz = nullptr;  // their bias, zeros for the bias-free "rn" projections
};

}  // namespace midas
}  // namespace vs

struct vs_midas {
    vs_ctx* ctx = nullptr;
    std::vector<float> h_weights;
    std::vector<vs::midas::DevW> dev;
    std::vector<vs::DevBuf> slots;  // activation slots (reused by last use)
    std::vector<int> slot_of;       // tensor -> slot
    std::vector<size_t> slot_elems; // floats per frame per slot
    vs::DevBuf input, post_part;
    vs::DevBuf splitk;  // k_mid_conv split-K partials (largest step's S x pixels x Co)
    int batch_cap = 0;
};

namespace vs {
namespace midas {

static int upload(vs_midas* m) {
    const Net& N = net();
    const float* p = m->h_weights.data();
    m->dev.resize(N.layers.size());
    for (size_t i = 0; i < N.layers.size(); i++) {
        const LayerDef& L = N.layers[i];
        DevW& D = m->dev[i];
        const int kk = L.k * L.k;
        if (L.kind == K_DW) {
            std::vector<float> w((size_t)kk * L.cout), b(L.cout, 0.f);
            for (int c = 0; c < L.cout; c++)
                for (int t = 0; t < kk; t++) w[(size_t)t * L.cout + c] = p[(size_t)c * kk + t];
            p += (size_t)L.cout * kk;
            for (int c = 0; c < L.cout; c++) b[c] = p[c];
            p += L.cout;
            VS_HIP(hipMalloc(&D.w, w.size() * sizeof(float)));
            VS_HIP(hipMalloc(&D.b, b.size() * sizeof(float)));
            VS_HIP(hipMemcpy(D.w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice));
            VS_HIP(hipMemcpy(D.b, b.data(), b.size() * sizeof(float), hipMemcpyHostToDevice));
        } else {
            D.cop = (L.cout + kCT - 1) / kCT * kCT;
            std::vector<float> w((size_t)kk * L.cin * D.cop, 0.f), b(D.cop, 0.f);
            for (int co = 0; co < L.cout; co++)
                for (int ci = 0; ci < L.cin; ci++)
                    for (int t = 0; t < kk; t++) w[((size_t)t * L.cin + ci) * D.cop + co] = p[((size_t)co * L.cin + ci) * kk + t];
            p += (size_t)L.cout * L.cin * kk;
            if (L.bias) {
                for (int c = 0; c < L.cout; c++) b[c] = p[c];
                p += L.cout;
            }
            VS_HIP(hipMalloc(&D.w, w.size() * sizeof(float)));
            VS_HIP(hipMemcpy(D.w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice));
            if (L.bias) {
                VS_HIP(hipMalloc(&D.b, b.size() * sizeof(float)));
                VS_HIP(hipMemcpy(D.b, b.data(), b.size() * sizeof(float), hipMemcpyHostToDevice));
            }
            if (L.k == 3 && L.cin % 4 == 0 && L.cout % 4 == 0) {
                const std::vector<float> u = winograd_weights(w.data(), L.cin, D.cop);
                VS_HIP(hipMalloc(&D.wu, u.size() * sizeof(float)));
                VS_HIP(hipMemcpy(D.wu, u.data(), u.size() * sizeof(float), hipMemcpyHostToDevice));
                if (L.bias) {
                    D.bz = D.b;
                } else {
                    VS_HIP(hipMalloc(&D.bz, b.size() * sizeof(float)));
                    VS_HIP(hipMemcpy(D.bz, b.data(), b.size() * sizeof(float), hipMemcpyHostToDevice));
                }
            }
        }
    }
    return VS_OK;
}

// tensor -> slot assignment by last use (a slot is reused once its tensor is dead)
static void plan(vs_midas* m) {
    const Net& N = net();
    const int nt = (int)N.tdims.size() / 3;
    std::vector<int> last(nt, -1);
    for (int i = 0; i < (int)N.steps.size(); i++) {
        const Step& s = N.steps[i];
        for (int t : {s.in, s.res1, s.res2})
            if (t >= 0) last[t] = i;
    }
    last[N.output] = (int)N.steps.size();
    m->slot_of.assign(nt, -1);
    std::vector<int> free_slots;
    m->slot_of[N.input] = -2;  // the input lives in m->input
    auto grab = [&](int t) {
        const size_t need = (size_t)N.Hof(t) * N.Wof(t) * N.Cof(t);
        int best = -1;
        for (size_t j = 0; j < free_slots.size(); j++)
            if (best < 0 || m->slot_elems[free_slots[j]] < m->slot_elems[free_slots[best]]) best = (int)j;
        int slot;
        if (best >= 0) {
            slot = free_slots[best];
            free_slots.erase(free_slots.begin() + best);
        } else {
            slot = (int)m->slot_elems.size();
            m->slot_elems.push_back(0);
        }
        m->slot_elems[slot] = std::max(m->slot_elems[slot], need);
        m->slot_of[t] = slot;
    };
    const bool keep_all = std::getenv("VS_MIDAS_KEEP_TENSORS") != nullptr;  // debugging: every tensor its own slot
    for (int i = 0; i < (int)N.steps.size(); i++) {
        const Step& s = N.steps[i];
        grab(s.out);
        if (keep_all) continue;
        for (int t : {s.in, s.res1, s.res2})
            if (t >= 0 && last[t] == i && m->slot_of[t] >= 0) free_slots.push_back(m->slot_of[t]);
    }
    m->slots.resize(m->slot_elems.size());
}

static float* tensor_ptr(vs_midas* m, int t) {
    const int s = m->slot_of[t];
    return s == -2 ? m->input.as<float>() : m->slots[s].as<float>();
}

// K splits of an implicit-GEMM step: the encoder's 1x1 projections at 8^2-16^2 (K up to 1392, 64 x 64
// tiles over 2k-8k pixels: 128-384 workgroups, each walking up to 87 K steps) fill the chip only when
// K is split.  S raises the workgroup count toward VS_MIDAS_SPLITK_WGS (default 1024; 0 = never
// split) with at least 3 K steps per split; the partials are summed in split order by k_mid_splitk.
// S is sized for a nominal 32-frame batch whatever B is, so that a frame's depth does not depend on
// the batch it was computed in (the summation order follows S).
static int splitk_of(const Step& st, int /*B*/) {
    constexpr int B = 32;
    static const int target = [] {
        const char* e = std::getenv("VS_MIDAS_SPLITK_WGS");
        return e ? std::atoi(e) : 1024;
    }();
    if (target <= 0 || st.Co % 4 != 0 || st.Co == 1) return 1;
    const long npix = (long)B * st.Ho * st.Wo;
    const long nwg = (npix + kCT - 1) / kCT * ((st.Co + kCT - 1) / kCT);
    const int T = st.k * st.k * ((st.C + kCK - 1) / kCK);
    long S = (target + nwg - 1) / nwg;
    S = std::min<long>(S, T / 3);
    S = std::min<long>(S, 16);
    return S > 1 ? (int)S : 1;
}

// Input-channel splits of a Winograd step (k_wino3 split-K): the 8^2 / 16^2 decoder convs (256-512
// channels) are one workgroup per 8 x 16 tile block and 64 output channels — 256 workgroups walking
// 64-128 channel chunks each, one wave per SIMD — so S raises the count toward 1024 with at least
// 8 chunks per split, for steps of at most 256 workgroups (VS_MIDAS_WINO_SPLITK=0: never).  Sized
// for a nominal 32-frame batch, as splitk_of.
static int wino_splits_of(const Step& st) {
    static const bool on = [] {
        const char* e = std::getenv("VS_MIDAS_WINO_SPLITK");
        return !(e && e[0] == '0');
    }();
    if (!on || st.Co % 4 != 0 || st.C % 4 != 0) return 1;
    constexpr long B = 32;
    const long nwg = B * ((st.W + 15) / 16) * ((st.H + 7) / 8) * ((st.Co + kCT - 1) / kCT);
    if (nwg > 256) return 1;  // 512 workgroups (the 32^2 convs) measured slower split in two (r03am)
    long S = (1024 + nwg - 1) / nwg;
    S = std::min<long>(S, (st.C / 4) / 8);
    return S > 1 ? (int)S : 1;
}

static int ensure_batch(vs_midas* m, int B) {
    if (B <= m->batch_cap) return VS_OK;
    for (size_t i = 0; i < m->slots.size(); i++) VS_CHECK(m->slots[i].ensure((size_t)B * m->slot_elems[i] * sizeof(float)));
    VS_CHECK(m->input.ensure((size_t)B * kIn * kIn * 3 * sizeof(float)));
    size_t part = 0;
    for (const Step& st : net().steps)
        if (st.kind == K_CONV) {
            const int S = std::max(splitk_of(st, B), st.k == 3 && st.stride == 1 ? wino_splits_of(st) : 1);
            if (S > 1) part = std::max(part, (size_t)S * B * st.Ho * st.Wo * st.Co);
        }
    if (part) VS_CHECK(m->splitk.ensure(part * sizeof(float)));
    m->batch_cap = B;
    return VS_OK;
}

// VS_WINO=0: every conv on k_mid_conv (A/B measurements)
static bool wino_on() {
    static const bool on = [] {
        const char* e = std::getenv("VS_WINO");
        return !(e && e[0] == '0');
    }();
    return on;
}

// VS_MIDAS_DW_ROW=0: the depthwise layers on the per-output k_mid_dw (A/B measurements)
static bool dw_row_on() {
    static const bool on = [] {
        const char* e = std::getenv("VS_MIDAS_DW_ROW");
        return !(e && e[0] == '0');
    }();
    return on;
}

// network: m->input [B][256][256][3] -> returns the output tensor pointer [B][256][256]
static int forward(vs_midas* m, int B, hipStream_t s, float** out) {
    const Net& N = net();
    VS_CHECK(ensure_batch(m, B));
    ProfScope ps(m->ctx, "midas_net", s);
    for (const Step& st : N.steps) {
        if (st.kind == K_CONV) {
            ConvArgs a{};
            a.in = tensor_ptr(m, st.in);
            a.w = m->dev[st.layer].w;
            a.bias = m->dev[st.layer].b;
            a.res1 = st.res1 >= 0 ? tensor_ptr(m, st.res1) : nullptr;
            a.res2 = st.res2 >= 0 ? tensor_ptr(m, st.res2) : nullptr;
            a.out = tensor_ptr(m, st.out);
            a.B = B, a.H = st.H, a.W = st.W, a.C = st.C, a.Ho = st.Ho, a.Wo = st.Wo, a.Co = st.Co;
            a.CoP = m->dev[st.layer].cop, a.k = st.k, a.stride = st.stride, a.pad_t = st.pad_t, a.pad_l = st.pad_l;
            a.act = st.act, a.pre_relu = st.pre_relu;
            a.splits = 1;
            const int npix = B * st.Ho * st.Wo;
            const DevW& D = m->dev[st.layer];
            if (D.wu && st.k == 3 && st.stride == 1 && st.pad_t == 1 && st.pad_l == 1 && wino_on()) {
                // stride-1 3x3 (the refinenet residual units, the rn projections, the head): Winograd
                WinoArgs wa{};
                wa.in = a.in;
                wa.in_cstride = st.C;
                wa.wu = D.wu;
                wa.bias = D.bz;
                wa.cin = st.C;
                wa.cout = st.Co;
                wa.cout_pad = D.cop;
                wa.out = a.out;
                wa.out_cstride = st.Co;
                wa.B = B;
                wa.H = st.H;
                wa.W = st.W;
                wa.res1 = a.res1;
                wa.res2 = a.res2;
                wa.act = st.act;
                wa.pre_relu = st.pre_relu ? 1 : 0;
                const int S = wino_splits_of(st);
                if (S > 1) {
                    wa.part = m->splitk.as<float>();
                    wa.splits = S;
                }
                VS_CHECK(wino3_launch(wa, false, false, s));
                if (S > 1) {  // bias, activation and the residual adds on the summed partials
                    a.part = m->splitk.as<float>();
                    a.splits = S;
                    const long n = (long)npix * (st.Co / 4);
                    hipLaunchKernelGGL(k_mid_splitk, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
                }
            } else if (st.Co == 1 && st.k == 1 && st.stride == 1) {
                VS_ARG(st.C % 4 == 0 && st.C <= kCo1MaxC, "midas: 1x1 single-channel conv needs C % 4 == 0, C <= 32");
                hipLaunchKernelGGL(k_mid_conv_co1, dim3((npix + 255) / 256), dim3(256), 0, s, a);
            } else if (st.Co == kStemCo && st.C <= kStemMaxC && st.k <= 3 && !st.pre_relu && st.res1 < 0 && st.res2 < 0) {
                hipLaunchKernelGGL(k_mid_stem, dim3((npix + 255) / 256), dim3(256), 0, s, a);
            } else {
                const int S = splitk_of(st, B);
                if (S > 1) {
                    a.part = m->splitk.as<float>();
                    a.splits = S;
                }
                hipLaunchKernelGGL(k_mid_conv, dim3((npix + kCT - 1) / kCT, a.CoP / kCT, S), dim3(256), 0, s, a);
                if (S > 1) {
                    const long n = (long)npix * (st.Co / 4);
                    hipLaunchKernelGGL(k_mid_splitk, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
                }
            }
        } else if (st.kind == K_DW && (st.stride == 1 || st.stride == 2) && (st.k == 3 || st.k == 5) && dw_row_on()) {
            constexpr int PX = 8;
            const long n = (long)B * st.Ho * ((st.Wo + PX - 1) / PX) * (st.C / 4);
            const dim3 grid((unsigned)((n + 255) / 256));
            const float* din = tensor_ptr(m, st.in);
            float* dout = tensor_ptr(m, st.out);
            const float* dw = m->dev[st.layer].w;
            const float* db = m->dev[st.layer].b;
#define VS_DW_ROW(K_, S_)                                                                                          \
    hipLaunchKernelGGL((k_mid_dw_row<K_, PX, S_>), grid, dim3(256), 0, s, din, dw, db, dout, B, st.H, st.W, st.C, st.Ho, \
                       st.Wo, st.pad_t, st.pad_l)
            if (st.k == 3 && st.stride == 1)
                VS_DW_ROW(3, 1);
            else if (st.k == 5 && st.stride == 1)
                VS_DW_ROW(5, 1);
            else if (st.k == 3)
                VS_DW_ROW(3, 2);
            else
                VS_DW_ROW(5, 2);
#undef VS_DW_ROW
        } else if (st.kind == K_DW) {
            const long n = (long)B * st.Ho * st.Wo * (st.C / 4);
            hipLaunchKernelGGL(k_mid_dw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tensor_ptr(m, st.in),
                               m->dev[st.layer].w, m->dev[st.layer].b, tensor_ptr(m, st.out), B, st.H, st.W, st.C,
                               st.Ho, st.Wo, st.k, st.stride, st.pad_t, st.pad_l);
        } else {
            const long n = (long)B * st.Ho * st.Wo * (st.C / 4);
            hipLaunchKernelGGL(k_mid_up, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tensor_ptr(m, st.in),
                               tensor_ptr(m, st.out), B, st.H, st.W, st.C, st.align_corners ? 1 : 0);
        }
    }
    VS_HIP(hipGetLastError());
    *out = tensor_ptr(m, N.output);
    return VS_OK;
}

static int preprocess(vs_midas* m, int B, const uint8_t* d_bgr, int h, int w, hipStream_t s) {
    VS_CHECK(ensure_batch(m, B));
    ProfScope ps(m->ctx, "midas_pre", s);
    const int n = B * kIn * kIn;
    hipLaunchKernelGGL(k_mid_pre, dim3((n + 255) / 256), dim3(256), 0, s, d_bgr, h, w, B, m->input.as<float>());
    VS_HIP(hipGetLastError());
    return VS_OK;
}

static int postprocess(vs_midas* m, int B, const float* d_small, int h, int w, float* d_out, hipStream_t s) {
    ProfScope ps(m->ctx, "midas_post", s);
    const int nb = (h * w + 255) / 256;
    VS_CHECK(m->post_part.ensure((size_t)B * nb * 2 * sizeof(float)));
    hipLaunchKernelGGL(k_mid_post, dim3(nb, B), dim3(256), 0, s, d_small, B, h, w, d_out, m->post_part.as<float>());
    hipLaunchKernelGGL(k_mid_norm, dim3(64, B), dim3(256), 0, s, d_out, m->post_part.as<float>(), nb, h * w);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace midas
}  // namespace vs

using namespace vs;

extern "C" {

size_t vs_midas_num_params(void) { return midas::net().num_params(); }

int vs_midas_onnx_weights(const char* path, float* out, size_t count) {
    VS_ARG(path && out && count == midas::net().num_params(), "vs_midas_onnx_weights: bad arguments");
    std::vector<float> w;
    std::string err;
    if (!midas::from_onnx(path, w, err)) {
        set_error("vs_midas_onnx_weights: " + err);
        return VS_ERR_IO;
    }
    std::memcpy(out, w.data(), count * sizeof(float));
    return VS_OK;
}

int vs_midas_synth_weights(float* out, size_t count) {
    VS_ARG(out && count == midas::net().num_params(), "vs_midas_synth_weights: bad arguments");
    const std::vector<float> w = midas::synth(VS_SYNTH_WEIGHT_SEED + 1);
    std::memcpy(out, w.data(), count * sizeof(float));
    return VS_OK;
}

double vs_midas_flops_per_frame(void) { return midas::net().flops(); }

int vs_midas_create(vs_ctx* ctx, const char* weights_path, vs_midas** out) {
    VS_ARG(ctx && out, "vs_midas_create: null argument");
    *out = nullptr;
    VS_HIP(hipSetDevice(ctx->device));
    auto* m = new (std::nothrow) vs_midas();
    if (!m) return VS_ERR_NOMEM;
    m->ctx = ctx;
    const size_t np = midas::net().num_params();
    if (weights_path && vs_onnx::looks_like_onnx(weights_path)) {
        // the reference's own model file (DepthEstimator.cpp:15-36: models/midas_v21_small_256.onnx)
        std::string err;
        if (!midas::from_onnx(weights_path, m->h_weights, err)) {
            delete m;
            set_error("vs_midas_create: " + err);
            return VS_ERR_IO;
        }
    } else if (weights_path) {
        FILE* f = std::fopen(weights_path, "rb");
        if (!f) {
            delete m;
            set_error(std::string("cannot open MiDaS weights ") + weights_path);
            return VS_ERR_IO;
        }
        uint32_t magic = 0, version = 0;
        uint64_t count = 0;
        const bool okh = std::fread(&magic, 4, 1, f) == 1 && std::fread(&version, 4, 1, f) == 1 &&
                         std::fread(&count, 8, 1, f) == 1;
        if (!okh || magic != 0x574D5356u || version != 1 || count != np) {  // "VSMW"
            std::fclose(f);
            delete m;
            set_error("malformed VSMW weight file");
            return VS_ERR_IO;
        }
        m->h_weights.resize(np);
        const bool okd = std::fread(m->h_weights.data(), sizeof(float), np, f) == np;
        std::fclose(f);
        if (!okd) {
            delete m;
            set_error("truncated VSMW weight file");
            return VS_ERR_IO;
        }
    } else {
        m->h_weights = midas::synth(VS_SYNTH_WEIGHT_SEED + 1);
    }
    int rc = midas::upload(m);
    if (rc != VS_OK) {
        vs_midas_destroy(m);
        return rc;
    }
    midas::plan(m);
    *out = m;
    return VS_OK;
}

void vs_midas_destroy(vs_midas* m) {
    if (!m) return;
    (void)hipDeviceSynchronize();
    for (auto& D : m->dev) {
        if (D.w) (void)hipFree(D.w);
        if (D.b) (void)hipFree(D.b);
        if (D.wu) (void)hipFree(D.wu);
        if (D.bz && D.bz != D.b) (void)hipFree(D.bz);
    }
    for (auto& b : m->slots) b.release();
    m->input.release();
    m->post_part.release();
    m->splitk.release();
    delete m;
}

int vs_midas_get_weights(vs_midas* m, float* out, size_t count) {
    VS_ARG(m && out && count == m->h_weights.size(), "vs_midas_get_weights: bad arguments");
    std::memcpy(out, m->h_weights.data(), count * sizeof(float));
    return VS_OK;
}

int vs_midas_estimate_dev(vs_midas* m, int B, const uint8_t* d_bgr, int h, int w, float* d_depth, void* stream) {
    VS_ARG(m && d_bgr && d_depth && B >= 1 && h >= 2 && w >= 2, "vs_midas_estimate_dev: bad arguments");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : m->ctx->stream;
    VS_CHECK(midas::preprocess(m, B, d_bgr, h, w, s));
    float* small = nullptr;
    VS_CHECK(midas::forward(m, B, s, &small));
    return midas::postprocess(m, B, small, h, w, d_depth, s);
}

int vs_midas_preprocess_dev(vs_midas* m, int B, const uint8_t* d_bgr, int h, int w, float* d_input, void* stream) {
    VS_ARG(m && d_bgr && d_input && B >= 1 && h >= 2 && w >= 2, "vs_midas_preprocess_dev: bad arguments");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : m->ctx->stream;
    VS_CHECK(midas::preprocess(m, B, d_bgr, h, w, s));
    VS_HIP(hipMemcpyAsync(d_input, m->input.p, (size_t)B * 256 * 256 * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
    return VS_OK;
}

int vs_midas_forward_dev(vs_midas* m, int B, const float* d_input, float* d_out, void* stream) {
    VS_ARG(m && d_input && d_out && B >= 1, "vs_midas_forward_dev: bad arguments");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : m->ctx->stream;
    VS_CHECK(midas::ensure_batch(m, B));
    VS_HIP(hipMemcpyAsync(m->input.p, d_input, (size_t)B * 256 * 256 * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
    float* small = nullptr;
    VS_CHECK(midas::forward(m, B, s, &small));
    VS_HIP(hipMemcpyAsync(d_out, small, (size_t)B * 256 * 256 * sizeof(float), hipMemcpyDeviceToDevice, s));
    return VS_OK;
}

// Debugging (VS_MIDAS_KEEP_TENSORS set at create): frame 0 of the output tensor of step i after
// the last forward ([Ho][Wo][Co] floats); returns the element count, or < 0.
long vs_midas_debug_step(vs_midas* m, int i, float* out) {
    const auto& N = midas::net();
    if (!m || i < 0 || i >= (int)N.steps.size()) return VS_ERR_ARG;
    const auto& st = N.steps[i];
    const long n = (long)st.Ho * st.Wo * st.Co;
    if (out) {
        VS_HIP(hipDeviceSynchronize());
        VS_HIP(hipMemcpy(out, midas::tensor_ptr(m, st.out), n * sizeof(float), hipMemcpyDeviceToHost));
    }
    return n;
}

int vs_midas_postprocess_dev(vs_midas* m, int B, const float* d_small, int h, int w, float* d_depth, void* stream) {
    VS_ARG(m && d_small && d_depth && B >= 1 && h >= 2 && w >= 2, "vs_midas_postprocess_dev: bad arguments");
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : m->ctx->stream;
    return midas::postprocess(m, B, d_small, h, w, d_depth, s);
}

}  // extern "C"
