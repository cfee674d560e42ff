// spcf.hip — the SPCF feature cache (reference src/FeatureExtractor.cpp:261-381: save_cache /
// load_cache) as the interchange between batch extraction (vs_extract_batch_dev, DevicePipeline)
// and sequential tracking (vs_slam_process_features).  Host code; the device variant only stages
// the extractor's outputs through pinned memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "vs_internal.h"

namespace {

constexpr uint32_t kMagic = 0x53504346u;  // "SPCF"
constexpr uint32_t kVersion = 1;
constexpr int32_t kCV32F = 5;
constexpr int kDim = VS_DESC_DIM;

struct File {
    FILE* f = nullptr;
    ~File() {
        if (f) std::fclose(f);
    }
};

bool put(FILE* f, const void* p, size_t bytes) { return bytes == 0 || std::fwrite(p, 1, bytes, f) == bytes; }
bool get(FILE* f, void* p, size_t bytes) { return bytes == 0 || std::fread(p, 1, bytes, f) == bytes; }

int write_entries(const char* path, int F, const int* frame_idx, const vs_keypoint* kps, const float* desc,
                  const int* n, int cap, int append) {
    if (!path || F < 0 || (F > 0 && (!frame_idx || !n)) || cap < 0) return VS_ERR_ARG;
    for (int f = 0; f < F; f++) {
        if (n[f] < 0 || n[f] > cap) {
            vs::set_error("vs_spcf_write: keypoint count out of range");
            return VS_ERR_ARG;
        }
        if (n[f] > 0 && (!kps || !desc)) return VS_ERR_ARG;  // empty frames need no feature buffers
    }
    File out;
    uint32_t hdr[3] = {kMagic, kVersion, 0};
    if (append && (out.f = std::fopen(path, "r+b"))) {
        if (!get(out.f, hdr, sizeof(hdr)) || hdr[0] != kMagic || hdr[1] != kVersion) {
            vs::set_error("vs_spcf_write: existing file is not an SPCF v1 cache");
            return VS_ERR_IO;
        }
        if (std::fseek(out.f, 0, SEEK_END) != 0) return VS_ERR_IO;
    } else {
        if (!(out.f = std::fopen(path, "wb"))) {
            vs::set_error("vs_spcf_write: cannot create file");
            return VS_ERR_IO;
        }
        if (!put(out.f, hdr, sizeof(hdr))) return VS_ERR_IO;
    }
    for (int f = 0; f < F; f++) {
        const int32_t head[2] = {frame_idx[f], n[f]};
        // FeatureExtractor.cpp:162-165: no keypoints -> descriptors = cv::Mat() (0 x 0, type 0)
        const int32_t mat[3] = {n[f], n[f] > 0 ? kDim : 0, n[f] > 0 ? kCV32F : 0};
        if (!put(out.f, head, sizeof(head)) || !put(out.f, kps + (size_t)f * cap, (size_t)n[f] * sizeof(vs_keypoint)) ||
            !put(out.f, mat, sizeof(mat)) || !put(out.f, desc + (size_t)f * cap * kDim, (size_t)n[f] * kDim * sizeof(float))) {
            vs::set_error("vs_spcf_write: write failed");
            return VS_ERR_IO;
        }
    }
    hdr[2] += (uint32_t)F;
    if (std::fseek(out.f, 8, SEEK_SET) != 0 || !put(out.f, &hdr[2], 4)) return VS_ERR_IO;
    if (std::fclose(out.f) != 0) {
        out.f = nullptr;
        return VS_ERR_IO;
    }
    out.f = nullptr;
    return VS_OK;
}

struct Entry {
    std::vector<vs_keypoint> kps;
    std::vector<float> desc;
};

}  // namespace

extern "C" {

int vs_spcf_write(const char* path, int F, const int* frame_idx, const vs_keypoint* kps, const float* desc,
                  const int* n, int cap, int append) {
    return write_entries(path, F, frame_idx, kps, desc, n, cap, append);
}

int vs_spcf_write_dev(vs_ctx* ctx, const char* path, int F, const int* frame_idx, const vs_keypoint* d_kps,
                      const float* d_desc, const int* d_n, int cap, int append, void* stream) {
    if (!ctx || F < 0 || cap < 0) return VS_ERR_ARG;
    if (F == 0) return write_entries(path, 0, frame_idx, nullptr, nullptr, nullptr, cap, append);
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    std::vector<int> n(F);
    VS_HIP(hipMemcpyAsync(n.data(), d_n, F * sizeof(int), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    std::vector<vs_keypoint> kps((size_t)F * cap);
    std::vector<float> desc((size_t)F * cap * kDim);
    // only each frame's live rows cross PCIe
    for (int f = 0; f < F; f++) {
        if (n[f] < 0 || n[f] > cap) {
            vs::set_error("vs_spcf_write_dev: keypoint count out of range (extraction error?)");
            return n[f] == VS_ERR_NOTCONV ? VS_ERR_NOTCONV : VS_ERR_ARG;
        }
        VS_HIP(hipMemcpyAsync(kps.data() + (size_t)f * cap, d_kps + (size_t)f * cap, (size_t)n[f] * sizeof(vs_keypoint),
                              hipMemcpyDeviceToHost, s));
        VS_HIP(hipMemcpyAsync(desc.data() + (size_t)f * cap * kDim, d_desc + (size_t)f * cap * kDim,
                              (size_t)n[f] * kDim * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    VS_HIP(hipStreamSynchronize(s));
    return write_entries(path, F, frame_idx, kps.data(), desc.data(), n.data(), cap, append);
}

int vs_spcf_read(const char* path, int max_frames, int cap, int* frame_idx, vs_keypoint* kps, float* desc, int* n,
                 int* count) {
    if (!path || !count) return VS_ERR_ARG;
    File in;
    if (!(in.f = std::fopen(path, "rb"))) {
        vs::set_error("vs_spcf_read: cannot open file");
        return VS_ERR_IO;
    }
    uint32_t hdr[3];
    if (!get(in.f, hdr, sizeof(hdr)) || hdr[0] != kMagic || hdr[1] != kVersion) {
        vs::set_error("vs_spcf_read: not an SPCF v1 cache");
        return VS_ERR_IO;
    }
    std::map<int32_t, Entry> cache;  // FeatureExtractor.cpp:310: cache_[frame_idx] = ... (last wins)
    for (uint32_t e = 0; e < hdr[2]; e++) {
        int32_t head[2], mat[3];
        if (!get(in.f, head, sizeof(head)) || head[1] < 0) {
            vs::set_error("vs_spcf_read: truncated entry");
            return VS_ERR_IO;
        }
        Entry en;
        en.kps.resize(head[1]);
        if (!get(in.f, en.kps.data(), (size_t)head[1] * sizeof(vs_keypoint)) || !get(in.f, mat, sizeof(mat))) {
            vs::set_error("vs_spcf_read: truncated entry");
            return VS_ERR_IO;
        }
        if (mat[0] > 0 && mat[1] > 0) {
            if (mat[1] != kDim || mat[2] != kCV32F || mat[0] != head[1]) {
                vs::set_error("vs_spcf_read: descriptors are not num_kp x 256 CV_32F");
                return VS_ERR_IO;
            }
            en.desc.resize((size_t)mat[0] * kDim);
            if (!get(in.f, en.desc.data(), en.desc.size() * sizeof(float))) {
                vs::set_error("vs_spcf_read: truncated descriptors");
                return VS_ERR_IO;
            }
        } else if (head[1] > 0) {
            vs::set_error("vs_spcf_read: keypoints without descriptors");
            return VS_ERR_IO;
        }
        cache[head[0]] = std::move(en);
    }
    *count = (int)cache.size();
    if (!kps && !desc && !n && !frame_idx) return VS_OK;
    if (!kps || !desc || !n || !frame_idx) return VS_ERR_ARG;
    if ((int)cache.size() > max_frames) {
        vs::set_error("vs_spcf_read: more entries than max_frames");
        return VS_ERR_CAPACITY;
    }
    int f = 0;
    for (const auto& kv : cache) {
        const int m = (int)kv.second.kps.size();
        if (m > cap) {
            vs::set_error("vs_spcf_read: more keypoints than cap");
            return VS_ERR_CAPACITY;
        }
        frame_idx[f] = kv.first;
        n[f] = m;
        std::memcpy(kps + (size_t)f * cap, kv.second.kps.data(), (size_t)m * sizeof(vs_keypoint));
        std::memcpy(desc + (size_t)f * cap * kDim, kv.second.desc.data(), (size_t)m * kDim * sizeof(float));
        f++;
    }
    return VS_OK;
}

}  // extern "C"
