// orc_extract.cpp — CPU restatement of FeatureExtractor::extract / extract_superpoint / nms
// (reference src/FeatureExtractor.cpp).  TEST INFRASTRUCTURE ONLY (see oracle.h).
// Compiled with -ffp-contract=off: the reference is a plain -O3 x86-64 build with no FMA
// contraction, and every float expression below keeps the reference's evaluation order.
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

extern "C" {

// FeatureExtractor.cpp:63-67 -> cv::cvtColor(BGR2GRAY) on CV_8UC3.  External (OpenCV 4.x,
// unpinned) semantics: fixed-point Y = (1868*B + 9617*G + 4899*R + 2^13) >> 14.
void orc_bgr_to_gray(const uint8_t* bgr, int h, int w, size_t stride, uint8_t* gray) {
    for (int y = 0; y < h; y++) {
        const uint8_t* row = bgr + (size_t)y * stride;
        for (int x = 0; x < w; x++) {
            unsigned b = row[3 * x], g = row[3 * x + 1], r = row[3 * x + 2];
            gray[(size_t)y * w + x] = (uint8_t)((b * 1868u + g * 9617u + r * 4899u + (1u << 13)) >> 14);
        }
    }
}

// FeatureExtractor.cpp:96 -> gray.convertTo(CV_32F, 1.0/255.0).  External semantics: OpenCV
// converts the double scale to float and computes src * scale (+ 0 shift) in fp32.
void orc_gray_to_f32(const uint8_t* gray, int h, int w, float* out) {
    const float scale = (float)(1.0 / 255.0);
    for (size_t i = 0; i < (size_t)h * w; i++) out[i] = (float)gray[i] * scale;
}

// FeatureExtractor.cpp:126-151: per-cell softmax over 65 channels (std::exp is glibc expf,
// the sum is a sequential float sum, IEEE division), channel c<64 -> pixel (8hc+c/8, 8wc+c%8).
void orc_decode_heatmap(const float* semi, int hc, int wc, float* heatmap) {
    const int Hp = hc * 8, Wp = wc * 8;
    std::memset(heatmap, 0, sizeof(float) * (size_t)Hp * Wp);
    for (int y = 0; y < hc; y++) {
        for (int x = 0; x < wc; x++) {
            float cell[65];
            for (int c = 0; c < 65; c++) cell[c] = semi[(size_t)c * hc * wc + (size_t)y * wc + x];
            float max_val = *std::max_element(cell, cell + 65);
            float sum = 0;
            for (int c = 0; c < 65; c++) {
                cell[c] = std::exp(cell[c] - max_val);
                sum += cell[c];
            }
            for (int c = 0; c < 65; c++) cell[c] /= sum;
            for (int c = 0; c < 64; c++) {
                int py = y * 8 + c / 8, px = x * 8 + c % 8;
                heatmap[(size_t)py * Wp + px] = cell[c];
            }
        }
    }
}

struct Candidate {
    float score;
    int x, y;
};

// FeatureExtractor.cpp:219-259 (nms) followed by the border erase at :155-160.
int orc_nms(const float* heatmap, int hp, int wp, int h, int w, float thr, int radius, int max_kp,
            int order_mode, orc_keypoint* out, int* n_candidates, int* n_tied) {
    std::vector<Candidate> candidates;
    for (int y = 0; y < hp; y++)
        for (int x = 0; x < wp; x++) {
            float val = heatmap[(size_t)y * wp + x];
            if (val > thr) candidates.push_back({val, x, y});
        }
    if (n_candidates) *n_candidates = (int)candidates.size();
    auto cmp = [](const Candidate& a, const Candidate& b) { return a.score > b.score; };
    if (order_mode == 0)
        std::sort(candidates.begin(), candidates.end(), cmp);
    else
        std::stable_sort(candidates.begin(), candidates.end(), cmp);
    if (n_tied) {
        int tied = 0;
        for (size_t i = 0; i < candidates.size(); i++) {
            bool t = (i > 0 && candidates[i - 1].score == candidates[i].score) ||
                     (i + 1 < candidates.size() && candidates[i + 1].score == candidates[i].score);
            tied += t;
        }
        *n_tied = tied;
    }
    std::vector<uint8_t> suppressed((size_t)hp * wp, 0);
    std::vector<orc_keypoint> kps;
    for (const auto& c : candidates) {
        if ((int)kps.size() >= max_kp) break;
        if (suppressed[(size_t)c.y * wp + c.x]) continue;
        // cv::KeyPoint(Point2f(x, y), size 8, angle -1, response score): octave 0, class_id -1
        kps.push_back({(float)c.x, (float)c.y, 8.0f, -1.0f, c.score, 0, -1});
        for (int dy = -radius; dy <= radius; dy++)
            for (int dx = -radius; dx <= radius; dx++) {
                int ny = c.y + dy, nx = c.x + dx;
                if (ny >= 0 && ny < hp && nx >= 0 && nx < wp) suppressed[(size_t)ny * wp + nx] = 1;
            }
    }
    int n = 0;
    for (const auto& k : kps)
        if (!(k.x >= w || k.y >= h)) out[n++] = k;  // FeatureExtractor.cpp:155-160
    return n;
}

// The ties that can make std::sort's output (FeatureExtractor.cpp:238-239, unstable) differ from
// the raster-order tie break used here (sp_post.hip header): over the stable greedy's kept sequence
// (uncapped), out[0] = selected pixels (the first min(max_kp, kept) of it) with an equal-score
// candidate in their (2 radius + 1)^2 window, out[1] = 1 when the max_kp-th and the next kept pixel
// score the same, out[2] = selected keypoints sharing their score with another selected one.
// out[0] = out[1] = 0 => every order of equal scores gives the same keypoint set; all three zero =>
// the same list.
void orc_nms_ties(const float* heatmap, int hp, int wp, float thr, int radius, int max_kp, int* out) {
    std::vector<Candidate> candidates;
    for (int y = 0; y < hp; y++)
        for (int x = 0; x < wp; x++) {
            float val = heatmap[(size_t)y * wp + x];
            if (val > thr) candidates.push_back({val, x, y});
        }
    std::stable_sort(candidates.begin(), candidates.end(),
                     [](const Candidate& a, const Candidate& b) { return a.score > b.score; });
    std::vector<uint8_t> suppressed((size_t)hp * wp, 0);
    std::vector<Candidate> kept;
    for (const auto& c : candidates) {
        if (suppressed[(size_t)c.y * wp + c.x]) continue;
        kept.push_back(c);
        for (int dy = -radius; dy <= radius; dy++)
            for (int dx = -radius; dx <= radius; dx++) {
                int ny = c.y + dy, nx = c.x + dx;
                if (ny >= 0 && ny < hp && nx >= 0 && nx < wp) suppressed[(size_t)ny * wp + nx] = 1;
            }
    }
    const int K = std::min<int>(max_kp, (int)kept.size());
    int window = 0;
    for (int i = 0; i < K; i++) {
        const Candidate& c = kept[i];
        bool tie = false;
        for (int dy = -radius; dy <= radius; dy++)
            for (int dx = -radius; dx <= radius; dx++) {
                int ny = c.y + dy, nx = c.x + dx;
                if ((dx || dy) && ny >= 0 && ny < hp && nx >= 0 && nx < wp && heatmap[(size_t)ny * wp + nx] == c.score)
                    tie = true;
            }
        window += tie;
    }
    out[0] = window;
    out[1] = (K > 0 && (int)kept.size() > K && kept[K - 1].score == kept[K].score) ? 1 : 0;
    // order ties: selected keypoints sharing their exact score with another selected one — the
    // set is order-independent, their order in the output list is not
    int order = 0;
    for (int i = 0; i < K; i++)
        order += (i > 0 && kept[i - 1].score == kept[i].score) || (i + 1 < K && kept[i + 1].score == kept[i].score);
    out[2] = order;
}

// FeatureExtractor.cpp:167-206: bilinear sample of the coarse descriptor grid, expression
// order kept, then sequential sum of squares, sqrtf, divide when norm > 1e-8f.
void orc_sample_descriptors(const float* desc_data, int Hc, int Wc, const orc_keypoint* kps,
                            int n, float* out) {
    for (int i = 0; i < n; i++) {
        float sx = kps[i].x / 8.0f;
        float sy = kps[i].y / 8.0f;
        int x0 = std::max(0, std::min((int)std::floor(sx), Wc - 1));
        int y0 = std::max(0, std::min((int)std::floor(sy), Hc - 1));
        int x1 = std::min(x0 + 1, Wc - 1);
        int y1 = std::min(y0 + 1, Hc - 1);
        float wx = sx - x0;
        float wy = sy - y0;
        float* row = out + (size_t)i * 256;
        for (int c = 0; c < 256; c++) {
            float v00 = desc_data[(size_t)c * Hc * Wc + y0 * Wc + x0];
            float v01 = desc_data[(size_t)c * Hc * Wc + y0 * Wc + x1];
            float v10 = desc_data[(size_t)c * Hc * Wc + y1 * Wc + x0];
            float v11 = desc_data[(size_t)c * Hc * Wc + y1 * Wc + x1];
            float val = (1 - wy) * ((1 - wx) * v00 + wx * v01) + wy * ((1 - wx) * v10 + wx * v11);
            row[c] = val;
        }
        float norm = 0;
        for (int c = 0; c < 256; c++) {
            float v = row[c];
            norm += v * v;
        }
        norm = std::sqrt(norm);
        if (norm > 1e-8f)
            for (int c = 0; c < 256; c++) row[c] /= norm;
    }
}

int orc_postprocess(const float* semi, const float* desc_grid, int hc, int wc, int h, int w,
                    int max_kp, int order_mode, orc_keypoint* kps, float* desc) {
    const int Hp = hc * 8, Wp = wc * 8;
    std::vector<float> heat((size_t)Hp * Wp);
    orc_decode_heatmap(semi, hc, wc, heat.data());
    // SP_CONFIDENCE_THRESHOLD 0.005f, SP_NMS_RADIUS 4 (Config.h:40-41)
    int n = orc_nms(heat.data(), Hp, Wp, h, w, 0.005f, 4, max_kp, order_mode, kps, nullptr, nullptr);
    if (n > 0) orc_sample_descriptors(desc_grid, hc, wc, kps, n, desc);
    return n;
}

int orc_extract(const float* weights, const uint8_t* bgr, int h, int w, size_t stride,
                int max_kp, int nthreads, orc_keypoint* kps, float* desc) {
    // FeatureExtractor.cpp:90-105: pad to a multiple of 8 with zeros.
    const int Hp = ((h + 7) / 8) * 8, Wp = ((w + 7) / 8) * 8;
    std::vector<uint8_t> gray((size_t)h * w);
    orc_bgr_to_gray(bgr, h, w, stride, gray.data());
    std::vector<float> f((size_t)h * w), padded((size_t)Hp * Wp, 0.0f);
    orc_gray_to_f32(gray.data(), h, w, f.data());
    for (int y = 0; y < h; y++) std::memcpy(&padded[(size_t)y * Wp], &f[(size_t)y * w], sizeof(float) * w);
    const int hc = Hp / 8, wc = Wp / 8;
    std::vector<float> semi((size_t)65 * hc * wc), dgrid((size_t)256 * hc * wc);
    int rc = orc_superpoint_forward(weights, padded.data(), Hp, Wp, semi.data(), dgrid.data(), nthreads);
    if (rc) return rc;
    return orc_postprocess(semi.data(), dgrid.data(), hc, wc, h, w, max_kp, 1, kps, desc);
}

void orc_expf_array(const float* x, int n, float* out) {
    for (int i = 0; i < n; i++) out[i] = std::exp(x[i]);
}

}  // extern "C"
