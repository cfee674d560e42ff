// orc_superpoint.cpp — fp32 CPU forward of the SuperPoint network that the reference runs through
// ONNX Runtime (FeatureExtractor.cpp:107-124; topology SURVEY.md 8(a) A3, MagicLeap
// SuperPointNet: VGG encoder + detector / descriptor heads, descriptor L2-normalised over
// channels).  TEST INFRASTRUCTURE ONLY (see oracle.h): it is the cpu_baseline's network and an
// independent check of the GPU network next to the torch F.conv2d reference in tests/.
// Direct NHWC convolution, OpenMP over output rows; FMA contraction allowed (tolerance-checked).
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

struct LayerDef {
    int cin, cout, k;
};
// Canonical blob order (== vs_superpoint_get_weights): conv1a conv1b conv2a conv2b conv3a conv3b
// conv4a conv4b convPa convPb convDa convDb.
const LayerDef kLayers[12] = {{1, 64, 3},    {64, 64, 3},   {64, 64, 3},    {64, 64, 3},
                              {64, 128, 3},  {128, 128, 3}, {128, 128, 3},  {128, 128, 3},
                              {128, 256, 3}, {256, 65, 1},  {128, 256, 3},  {256, 256, 1}};

struct Layer {
    int cin, cout, k;
    std::vector<float> wt;  // [ky][kx][cin][cout]
    std::vector<float> b;
};

// NHWC conv, stride 1, pad k/2, optional ReLU.
void conv(const Layer& L, const float* in, int H, int W, float* out, bool relu) {
    const int C = L.cin, N = L.cout, pad = L.k / 2;
#pragma omp parallel
    {
        std::vector<float> acc((size_t)W * N);
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++) {
            for (int x = 0; x < W; x++)
                std::memcpy(&acc[(size_t)x * N], L.b.data(), sizeof(float) * N);
            for (int ky = 0; ky < L.k; ky++) {
                int iy = y + ky - pad;
                if (iy < 0 || iy >= H) continue;
                for (int kx = 0; kx < L.k; kx++) {
                    const float* wk = &L.wt[(size_t)(ky * L.k + kx) * C * N];
                    for (int x = 0; x < W; x++) {
                        int ix = x + kx - pad;
                        if (ix < 0 || ix >= W) continue;
                        const float* ip = in + ((size_t)iy * W + ix) * C;
                        float* ap = &acc[(size_t)x * N];
                        for (int c = 0; c < C; c++) {
                            const float v = ip[c];
                            const float* wr = wk + (size_t)c * N;
#pragma omp simd
                            for (int n = 0; n < N; n++) ap[n] += v * wr[n];
                        }
                    }
                }
            }
            float* op = out + (size_t)y * W * N;
            for (size_t i = 0; i < (size_t)W * N; i++) op[i] = relu ? (acc[i] > 0.f ? acc[i] : 0.f) : acc[i];
        }
    }
}

void pool2(const float* in, int H, int W, int C, float* out) {
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H / 2; y++)
        for (int x = 0; x < W / 2; x++)
            for (int c = 0; c < C; c++) {
                const float* p = in + ((size_t)(2 * y) * W + 2 * x) * C + c;
                float m = p[0];
                m = std::max(m, p[C]);
                m = std::max(m, p[(size_t)W * C]);
                m = std::max(m, p[(size_t)W * C + C]);
                out[((size_t)y * (W / 2) + x) * C + c] = m;
            }
}

}  // namespace

extern "C" {

size_t orc_superpoint_num_params(void) {
    size_t n = 0;
    for (const auto& l : kLayers) n += (size_t)l.cout * l.cin * l.k * l.k + l.cout;
    return n;
}

int orc_superpoint_forward(const float* weights, const float* img, int H, int W, float* semi,
                           float* desc, int nthreads) {
    if (H % 8 || W % 8) return -1;
#ifdef _OPENMP
    int saved = omp_get_max_threads();
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    std::vector<Layer> L(12);
    const float* p = weights;
    for (int i = 0; i < 12; i++) {
        const LayerDef& d = kLayers[i];
        L[i].cin = d.cin;
        L[i].cout = d.cout;
        L[i].k = d.k;
        L[i].wt.resize((size_t)d.k * d.k * d.cin * d.cout);
        for (int co = 0; co < d.cout; co++)
            for (int ci = 0; ci < d.cin; ci++)
                for (int ky = 0; ky < d.k; ky++)
                    for (int kx = 0; kx < d.k; kx++)
                        L[i].wt[((size_t)(ky * d.k + kx) * d.cin + ci) * d.cout + co] =
                            p[(((size_t)co * d.cin + ci) * d.k + ky) * d.k + kx];
        p += (size_t)d.cout * d.cin * d.k * d.k;
        L[i].b.assign(p, p + d.cout);
        p += d.cout;
    }
    std::vector<float> a((size_t)H * W * 64), b((size_t)H * W * 64);
    int h = H, w = W;
    conv(L[0], img, h, w, a.data(), true);
    conv(L[1], a.data(), h, w, b.data(), true);
    pool2(b.data(), h, w, 64, a.data());
    h /= 2; w /= 2;
    conv(L[2], a.data(), h, w, b.data(), true);
    conv(L[3], b.data(), h, w, a.data(), true);
    pool2(a.data(), h, w, 64, b.data());
    h /= 2; w /= 2;
    conv(L[4], b.data(), h, w, a.data(), true);
    conv(L[5], a.data(), h, w, b.data(), true);
    pool2(b.data(), h, w, 128, a.data());
    h /= 2; w /= 2;
    conv(L[6], a.data(), h, w, b.data(), true);
    conv(L[7], b.data(), h, w, a.data(), true);  // a = encoder output [h][w][128]
    const size_t P = (size_t)h * w;
    std::vector<float> pa(P * 256), s(P * 65), da(P * 256), dd(P * 256);
    conv(L[8], a.data(), h, w, pa.data(), true);
    conv(L[9], pa.data(), h, w, s.data(), false);
    conv(L[10], a.data(), h, w, da.data(), true);
    conv(L[11], da.data(), h, w, dd.data(), false);
    for (size_t i = 0; i < P; i++) {
        for (int c = 0; c < 65; c++) semi[(size_t)c * P + i] = s[i * 65 + c];
        double nrm = 0;
        for (int c = 0; c < 256; c++) nrm += (double)dd[i * 256 + c] * dd[i * 256 + c];
        float inv = (float)(1.0 / std::sqrt(nrm));
        for (int c = 0; c < 256; c++) desc[(size_t)c * P + i] = dd[i * 256 + c] * inv;
    }
#ifdef _OPENMP
    omp_set_num_threads(saved);
#endif
    return 0;
}

}  // extern "C"
