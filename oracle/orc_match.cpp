// orc_match.cpp — CPU restatement of Slam::match_features for float descriptors
// (reference src/Slam.cpp:1140-1172).  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// The reference calls cv::FlannBasedMatcher::knnMatch(desc1, desc2, k=2) (Slam.cpp:1149), an
// approximate randomized kd-tree search (external, unpinned).  The only definable oracle is the
// exact 2-NN it approximates; DESIGN.md "Matching" fixes its fp32 arithmetic:
//     dot, na, nb = fp32 fmaf chains over k = 0..255 (start 0)
//     d2 = max((na + nb) - 2*dot, 0)            (no contraction; 2*dot is exact)
//     best/second = the two smallest (d2, train index) pairs, lexicographic
//     DMatch.distance = sqrtf(d2); good iff d0 < ratio * d1 (Slam.cpp:1154).
// Rows produce a raw match only when n2 >= 2 (knnMatch returns min(k, n2) neighbours and the
// reference keeps rows with m.size() >= 2, Slam.cpp:1152).
#include "oracle.h"

#include <immintrin.h>

#include <cmath>
#include <limits>
#include <vector>

namespace {

struct Best2 {
    float d0 = std::numeric_limits<float>::infinity(), d1 = std::numeric_limits<float>::infinity();
    int j0 = -1, j1 = -1;
    void push(float d, int j) {
        if (d < d0 || (d == d0 && j < j0)) {
            d1 = d0; j1 = j0; d0 = d; j0 = j;
        } else if (d < d1 || (d == d1 && j < j1)) {
            d1 = d; j1 = j;
        }
    }
};

float fma_norm(const float* a) {
    float s = 0.0f;
    for (int k = 0; k < 256; k++) s = std::fmaf(a[k], a[k], s);
    return s;
}

// The same fmaf chains, eight train rows per AVX2 register (one independent chain per lane, k in
// order, vfmadd = one rounding like fmaf): bit-identical to the scalar loops above, ~50x faster
// than libm's software fmaf the -march=x86-64 parity build otherwise calls.  Train rows are
// transposed once per call to tT[k][j] (n2p = n2 rounded up to 32, zero padded).
__attribute__((target("avx2,fma"))) void dots_avx2(const float* a, const float* tT, int n2p, float* dot) {
    for (int j = 0; j < n2p; j += 32) {
        __m256 c0 = _mm256_setzero_ps(), c1 = _mm256_setzero_ps(), c2 = _mm256_setzero_ps(), c3 = _mm256_setzero_ps();
        for (int k = 0; k < 256; k++) {
            const __m256 x = _mm256_set1_ps(a[k]);
            const float* r = tT + (size_t)k * n2p + j;
            c0 = _mm256_fmadd_ps(x, _mm256_loadu_ps(r), c0);
            c1 = _mm256_fmadd_ps(x, _mm256_loadu_ps(r + 8), c1);
            c2 = _mm256_fmadd_ps(x, _mm256_loadu_ps(r + 16), c2);
            c3 = _mm256_fmadd_ps(x, _mm256_loadu_ps(r + 24), c3);
        }
        _mm256_storeu_ps(dot + j, c0);
        _mm256_storeu_ps(dot + j + 8, c1);
        _mm256_storeu_ps(dot + j + 16, c2);
        _mm256_storeu_ps(dot + j + 24, c3);
    }
}
__attribute__((target("avx2,fma"))) void norms_avx2(const float* tT, int n2p, float* nrm) {
    for (int j = 0; j < n2p; j += 8) {
        __m256 c = _mm256_setzero_ps();
        for (int k = 0; k < 256; k++) {
            const __m256 x = _mm256_loadu_ps(tT + (size_t)k * n2p + j);
            c = _mm256_fmadd_ps(x, x, c);
        }
        _mm256_storeu_ps(nrm + j, c);
    }
}
__attribute__((target("fma"))) float fma_norm_hw(const float* a) {
    float s = 0.0f;
    for (int k = 0; k < 256; k++) s = __builtin_fmaf(a[k], a[k], s);
    return s;
}
bool have_avx2_fma() {
    static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
    return ok;
}

}  // namespace

extern "C" {

void orc_match_ratio(const float* d1, int n1, const float* d2, int n2, float ratio, orc_match* raw,
                     int* n_raw, orc_match* good, int* n_good) {
    *n_raw = 0;
    *n_good = 0;
    if (n1 <= 0 || n2 < 2) return;
    if (have_avx2_fma()) {  // the same arithmetic, vectorised across train rows
        const int n2p = (n2 + 31) / 32 * 32;
        std::vector<float> tT((size_t)256 * n2p, 0.0f), nb(n2p), dot(n2p);
        for (int j = 0; j < n2; j++)
            for (int k = 0; k < 256; k++) tT[(size_t)k * n2p + j] = d2[(size_t)j * 256 + k];
        norms_avx2(tT.data(), n2p, nb.data());
        for (int i = 0; i < n1; i++) {
            const float* a = d1 + (size_t)i * 256;
            const float na = fma_norm_hw(a);
            dots_avx2(a, tT.data(), n2p, dot.data());
            Best2 b;
            for (int j = 0; j < n2; j++) {
                float s = na + nb[j];
                float dd = s - 2.0f * dot[j];
                if (dd < 0.0f) dd = 0.0f;
                b.push(dd, j);
            }
            const float dist0 = std::sqrt(b.d0), dist1 = std::sqrt(b.d1);
            raw[(*n_raw)++] = {i, b.j0, 0, dist0};
            if (dist0 < ratio * dist1) good[(*n_good)++] = {i, b.j0, 0, dist0};
        }
        return;
    }
    std::vector<float> nb(n2);
    for (int j = 0; j < n2; j++) nb[j] = fma_norm(d2 + (size_t)j * 256);
    for (int i = 0; i < n1; i++) {
        const float* a = d1 + (size_t)i * 256;
        const float na = fma_norm(a);
        Best2 b;
        for (int j = 0; j < n2; j++) {
            const float* t = d2 + (size_t)j * 256;
            float dot = 0.0f;
            for (int k = 0; k < 256; k++) dot = std::fmaf(a[k], t[k], dot);
            float s = na + nb[j];
            float dd = s - 2.0f * dot;
            if (dd < 0.0f) dd = 0.0f;
            b.push(dd, j);
        }
        const float dist0 = std::sqrt(b.d0), dist1 = std::sqrt(b.d1);
        raw[(*n_raw)++] = {i, b.j0, 0, dist0};
        if (dist0 < ratio * dist1) good[(*n_good)++] = {i, b.j0, 0, dist0};
    }
}

// The scalar loops only (the reference statement of the vectorised path; tests compare the two).
void orc_match_ratio_scalar(const float* d1, int n1, const float* d2, int n2, float ratio, orc_match* raw,
                            int* n_raw, orc_match* good, int* n_good) {
    *n_raw = 0;
    *n_good = 0;
    if (n1 <= 0 || n2 < 2) return;
    std::vector<float> nb(n2);
    for (int j = 0; j < n2; j++) nb[j] = fma_norm(d2 + (size_t)j * 256);
    for (int i = 0; i < n1; i++) {
        const float* a = d1 + (size_t)i * 256;
        const float na = fma_norm(a);
        Best2 b;
        for (int j = 0; j < n2; j++) {
            const float* t = d2 + (size_t)j * 256;
            float dot = 0.0f;
            for (int k = 0; k < 256; k++) dot = std::fmaf(a[k], t[k], dot);
            float s = na + nb[j];
            float dd = s - 2.0f * dot;
            if (dd < 0.0f) dd = 0.0f;
            b.push(dd, j);
        }
        const float dist0 = std::sqrt(b.d0), dist1 = std::sqrt(b.d1);
        raw[(*n_raw)++] = {i, b.j0, 0, dist0};
        if (dist0 < ratio * dist1) good[(*n_good)++] = {i, b.j0, 0, dist0};
    }
}

void orc_match_ratio_f64(const float* d1, int n1, const float* d2, int n2, float ratio,
                         orc_match* raw, int* n_raw, orc_match* good, int* n_good) {
    *n_raw = 0;
    *n_good = 0;
    if (n1 <= 0 || n2 < 2) return;
    for (int i = 0; i < n1; i++) {
        const float* a = d1 + (size_t)i * 256;
        double b0 = INFINITY, b1 = INFINITY;
        int j0 = -1, j1 = -1;
        for (int j = 0; j < n2; j++) {
            const float* t = d2 + (size_t)j * 256;
            double s = 0;
            for (int k = 0; k < 256; k++) {
                double df = (double)a[k] - (double)t[k];
                s += df * df;
            }
            if (s < b0 || (s == b0 && j < j0)) {
                b1 = b0; j1 = j0; b0 = s; j0 = j;
            } else if (s < b1 || (s == b1 && j < j1)) {
                b1 = s; j1 = j;
            }
        }
        (void)j1;
        const float dist0 = (float)std::sqrt(b0), dist1 = (float)std::sqrt(b1);
        raw[(*n_raw)++] = {i, j0, 0, dist0};
        if (dist0 < ratio * dist1) good[(*n_good)++] = {i, j0, 0, dist0};
    }
}

}  // extern "C"
