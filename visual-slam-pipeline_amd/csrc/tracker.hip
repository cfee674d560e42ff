// tracker.hip — the GPU back end of the host tracking loop (host/tracker.hpp, a restatement of
// Slam::process_frame, reference src/Slam.cpp:809-1135) and its C ABI (vs_slam_*).
//
// Device residency.  Every frame's features and depth live in HBM in a slot of a frame pool
// ([slot][400] keypoints, [slot][400][256] descriptors, [slot][h][w] depth): two batch regions of
// B slots each (a batch's frames are extracted straight into one region) plus persistent slots
// that the tracker's live frames (last frame, last keyframe, reference frame) move into when
// their batch region is about to be reused.  The map's point positions, validity bytes and
// 256-d descriptors are mirrored in HBM and appended in place (descriptor rows are gathered
// device-side from the creating frame's slot), so the per-frame O(map) work never crosses PCIe.
//
// Per processed frame the host issues: one fused chain (match -> F verification -> 3D-3D
// RANSAC -> E-matrix fallback, one D2H of a packed 13 KB result block), local-map tracking
// (one D2H of the index / observation block), PnP refinement, and for keyframes the keyframe
// match, the visibility sweep and the map appends.  Everything runs on the context's stream.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <functional>
#include <thread>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "../host/tracker.hpp"
#include "vs_internal.h"

namespace vs {

int match_sets(vs_ctx* ctx, const float* d_q, int n1, const float* d_t, int n2, float ratio, vs_match* d_raw,
               vs_match* d_good, int* d_counts, hipStream_t s);

static_assert(sizeof(vs_trk::Keypoint) == sizeof(vs_keypoint), "keypoint layouts differ");
static_assert(sizeof(vs_trk::Match) == sizeof(vs_match), "match layouts differ");

constexpr int kCap = VS_SP_MAX_KEYPOINTS;
constexpr int kPersist = 8;
constexpr int kArchInit = 512;   // keyframes the feature archive holds before it first grows
constexpr int kLoopPairs = 128;  // loop candidates reserved up front (kArchInit / 5 + slack)

// Loop-closure candidate pool: frame f of the pool = the keypoints / descriptors / count at src[f]
// (archive rows or pool slots); grid (F, slices), float4 copies.
struct FrameSrc {
    const vs_keypoint* k;
    const float* d;
    const int* n;
};
__global__ __launch_bounds__(256) void k_gather_frames(const FrameSrc* __restrict__ src, vs_keypoint* __restrict__ kps,
                                                       float* __restrict__ desc, int* __restrict__ n) {
    const int f = blockIdx.x;
    const FrameSrc S = src[f];
    const float4* sd = reinterpret_cast<const float4*>(S.d);
    float4* dd = reinterpret_cast<float4*>(desc + (size_t)f * kCap * 256);
    for (int i = blockIdx.y * 256 + threadIdx.x; i < kCap * 64; i += gridDim.y * 256) dd[i] = sd[i];
    if (blockIdx.y == 0) {
        constexpr int kw = kCap * (int)sizeof(vs_keypoint) / 4;
        const int* sk = reinterpret_cast<const int*>(S.k);
        int* dk = reinterpret_cast<int*>(kps + (size_t)f * kCap);
        for (int i = threadIdx.x; i < kw; i += 256) dk[i] = sk[i];
        if (threadIdx.x == 0) n[f] = *S.n;
    }
}

// Triangulation inputs (Slam::triangulate_points, Slam.cpp:1265-1277): the DLT solution of every
// good match of a keyframe match, one lane per match, right behind the matcher.
struct DltProj {
    double P1[12], P2[12];
};
__global__ __launch_bounds__(64) void k_dlt(const vs_match* __restrict__ good, const int* __restrict__ ng,
                                            const vs_keypoint* __restrict__ ka, const vs_keypoint* __restrict__ kb,
                                            DltProj P, float4* __restrict__ X) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= *ng) return;
    const vs_match m = good[i];
    float x[4];
    vs_pnp::dlt_point(P.P1, P.P2, ka[m.query_idx].x, ka[m.query_idx].y, kb[m.train_idx].x, kb[m.train_idx].y, x);
    X[i] = make_float4(x[0], x[1], x[2], x[3]);
}

// dst[i] = src row rows[i] (256 floats), one 64-lane wave per row, float4 per lane
__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ src, const int* __restrict__ rows,
                                                     int k, float* __restrict__ dst) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= k) return;
    reinterpret_cast<float4*>(dst + (size_t)r * 256)[lane] =
        reinterpret_cast<const float4*>(src + (size_t)rows[r] * 256)[lane];
}

// Slam's map-point insertion mirrored in HBM (map_append): for the k new points, the position (3
// doubles from the staging upload), the descriptor row of the source frame and the valid flag, one
// 64-lane wave per point
__global__ __launch_bounds__(256) void k_map_append(const double* __restrict__ pos_in, const int* __restrict__ rows,
                                                    int k, const float* __restrict__ desc_src, double* __restrict__ pos,
                                                    float* __restrict__ desc, uint8_t* __restrict__ valid) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= k) return;
    reinterpret_cast<float4*>(desc + (size_t)r * 256)[lane] =
        reinterpret_cast<const float4*>(desc_src + (size_t)rows[r] * 256)[lane];
    if (lane < 3) pos[3 * (size_t)r + lane] = pos_in[3 * (size_t)r + lane];
    if (lane == 3) valid[r] = 1;
}

// A list of device-to-device copies in one launch (the settle step's keyframe archiving and slot
// moves: tens of small hipMemcpyAsync per batch, each a blit kernel and a host round of its own).
// blockIdx.y = job; 16-byte words when source, destination and size allow, else 4-byte words (every
// size here is a multiple of 4).
struct CopyJob {
    const void* src;
    void* dst;
    unsigned long long bytes;
};
__global__ __launch_bounds__(256) void k_copy_jobs(const CopyJob* __restrict__ jobs) {
    const CopyJob J = jobs[blockIdx.y];
    const size_t t0 = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
    if ((((uintptr_t)J.src | (uintptr_t)J.dst | (uintptr_t)J.bytes) & 15) == 0) {
        const uint4* a = reinterpret_cast<const uint4*>(J.src);
        uint4* b = reinterpret_cast<uint4*>(J.dst);
        for (size_t i = t0; i < J.bytes / 16; i += stride) b[i] = a[i];
    } else {
        const unsigned* a = reinterpret_cast<const unsigned*>(J.src);
        unsigned* b = reinterpret_cast<unsigned*>(J.dst);
        for (size_t i = t0; i < J.bytes / 4; i += stride) b[i] = a[i];
    }
}

// The tracking stream's small host <-> device transfers through coherent (fine-grained) mapped pinned
// memory, as a kernel: results go straight into host memory (the kernel's stores cross the fabric
// themselves, so the host's stream synchronisation sees them) and inputs are read from it, without a
// copy command in the stream (a hipMemcpyAsync D2H started ~11 us after the kernel before it in the
// kernel trace, profiles/r04n_tracker_chain_trace.txt).  16-, 4- or 1-byte words as the alignment
// allows.
__global__ __launch_bounds__(256) void k_copy_bytes(const char* __restrict__ src, char* __restrict__ dst, size_t bytes) {
    const size_t t0 = (size_t)blockIdx.x * 256 + threadIdx.x, stride = (size_t)gridDim.x * 256;
    const uintptr_t al = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)bytes;
    if ((al & 15) == 0) {
        for (size_t i = t0; i < bytes / 16; i += stride)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else if ((al & 3) == 0) {
        for (size_t i = t0; i < bytes / 4; i += stride)
            reinterpret_cast<unsigned*>(dst)[i] = reinterpret_cast<const unsigned*>(src)[i];
    } else {
        for (size_t i = t0; i < bytes; i += stride) dst[i] = src[i];
    }
}

// The reference frame of a speculative chain two frames ahead: the keyframe rule chain() predicts with
// (Slam.cpp:1061-1072, is_keyframe :1360) on the ratio-test count of the chain before it (prev[4], the
// same stream, so already final): kf_slot when that frame becomes a keyframe, else base_slot.  Written
// into the chain's header (the pair every kernel of the chain reads) and into its result block (int 28)
// for the host's check.
__global__ void k_pick_ref(const int* __restrict__ prev, int kf_slot, int base_slot, int gap, int* __restrict__ hdr,
                           int* __restrict__ res) {
    if (threadIdx.x != 0) return;
    const int ng = prev[4];
    const bool kf = (gap >= vs_trk::cfg::KF_MIN_FRAME_GAP && ng >= vs_trk::cfg::KF_MIN_MATCHES) ||
                    (ng < 2 * vs_trk::cfg::MIN_MATCHES && gap >= 5);
    const int slot = kf ? kf_slot : base_slot;
    hdr[0] = slot;
    res[28] = slot;
}

// Visibility sweep (Slam.cpp:1089-1108): for every valid map point, Optimizer::project_point
// (Optimizer.cpp:26-48) with the camera->world pose; bit 0 = inside the image (increase_visible),
// bit 1 = some keypoint within TRACK_VISIBILITY_RADIUS (increase_found).  Every workgroup first
// bins the frame's keypoints into an LDS grid of 16-pixel cells (counting sort: counts, a block
// scan, a scatter), so a projected point tests only the keypoints of the 3 x 3 cells around it —
// any keypoint closer than the 8-pixel radius lies there — with the same double expression as a
// scan of all keypoints (the result is an "any" and does not depend on the order).  Round 3: the
// linear scan over up to 400 keypoints per point took 47-63 us per keyframe on the tracking CUs.
constexpr int kVisCell = 16, kVisMaxCells = 4096;
static_assert(kVisCell >= vs_trk::cfg::TRACK_VISIBILITY_RADIUS + 1, "a keypoint within the radius lies in the 3 x 3 cells");
__global__ __launch_bounds__(256) void k_visibility(const double* __restrict__ pos, const uint8_t* __restrict__ valid,
                                                    int n_mp, const vs_keypoint* __restrict__ kps, int nkp,
                                                    double r0, double r1, double r2, double r3, double r4, double r5,
                                                    double r6, double r7, double r8, double t0, double t1, double t2,
                                                    double fx, double fy, double cx, double cy, int img_w, int img_h,
                                                    uint8_t* __restrict__ flags) {
    __shared__ float s_x[kCap], s_y[kCap];
    __shared__ int s_start[kVisMaxCells + 1], s_cur[kVisMaxCells];
    __shared__ int s_part[256];
    const int tid = threadIdx.x;
    const int gw = (img_w + kVisCell - 1) / kVisCell, gh = (img_h + kVisCell - 1) / kVisCell, ncell = gw * gh;
    auto cell_of = [&](float x, float y) {
        const int ix = min(max((int)(x * (1.0f / kVisCell)), 0), gw - 1);
        const int iy = min(max((int)(y * (1.0f / kVisCell)), 0), gh - 1);
        return iy * gw + ix;
    };
    for (int c = tid; c <= ncell; c += 256) s_start[c] = 0;
    __syncthreads();
    for (int i = tid; i < nkp; i += 256) atomicAdd(&s_start[cell_of(kps[i].x, kps[i].y) + 1], 1);
    __syncthreads();
    // inclusive scan of s_start[1 .. ncell]: each thread a contiguous range, then the range totals
    const int per = (ncell + 255) / 256, c0 = 1 + tid * per, c1 = min(c0 + per, ncell + 1);
    int run = 0;
    for (int c = c0; c < c1; c++) run += s_start[c];
    s_part[tid] = run;
    __syncthreads();
    if (tid < 64) {  // one wave scans the 256 totals (4 per lane)
        int v[4], t = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) t += (v[j] = s_part[4 * tid + j]);
        int incl = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(incl, o);
            if (tid >= o) incl += u;
        }
        int base = incl - t;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            s_part[4 * tid + j] = base;  // exclusive prefix of thread 4 tid + j's range
            base += v[j];
        }
    }
    __syncthreads();
    run = s_part[tid];
    for (int c = c0; c < c1; c++) {
        run += s_start[c];
        s_start[c] = run;
    }
    __syncthreads();
    for (int c = tid; c < ncell; c += 256) s_cur[c] = s_start[c];
    __syncthreads();
    for (int i = tid; i < nkp; i += 256) {
        const float x = kps[i].x, y = kps[i].y;
        const int slot = atomicAdd(&s_cur[cell_of(x, y)], 1);
        s_x[slot] = x;
        s_y[slot] = y;
    }
    __syncthreads();
    const int m = blockIdx.x * blockDim.x + tid;
    if (m >= n_mp) return;
    uint8_t f = 0;
    if (valid[m]) {
        // R_cam = R^T, t_cam = -R_cam t, pc = R_cam Pw + t_cam
        const double tc0 = -(r0 * t0 + r3 * t1 + r6 * t2), tc1 = -(r1 * t0 + r4 * t1 + r7 * t2),
                     tc2 = -(r2 * t0 + r5 * t1 + r8 * t2);
        const double X = pos[3 * m], Y = pos[3 * m + 1], Z = pos[3 * m + 2];
        const double z = (r2 * X + r5 * Y + r8 * Z) + tc2;
        double u = -1, v = -1;
        if (!(z < 1e-6)) {
            u = fx * ((r0 * X + r3 * Y + r6 * Z) + tc0) / z + cx;
            v = fy * ((r1 * X + r4 * Y + r7 * Z) + tc1) / z + cy;
        }
        if (u >= 0 && u < img_w && v >= 0 && v < img_h) {
            f = 1;
            const double rr = vs_trk::cfg::TRACK_VISIBILITY_RADIUS * vs_trk::cfg::TRACK_VISIBILITY_RADIUS;
            const int ux = min((int)(u / kVisCell), gw - 1), uy = min((int)(v / kVisCell), gh - 1);
            for (int gy = max(uy - 1, 0); gy <= min(uy + 1, gh - 1) && f != 3; gy++)
                for (int k = s_start[gy * gw + max(ux - 1, 0)]; k < s_start[gy * gw + min(ux + 1, gw - 1) + 1]; k++) {
                    const double dx = u - s_x[k], dy = v - s_y[k];
                    if (dx * dx + dy * dy < rr) {
                        f = 3;
                        break;
                    }
                }
        }
    }
    flags[m] = f;
}

// Pinned bump allocator for small host<->device transfers; reset after every synchronisation.
struct Pinned {
    char* base = nullptr;
    size_t cap = 0, used = 0;
    unsigned flags = hipHostMallocDefault;
    explicit Pinned(unsigned f = hipHostMallocDefault) : flags(f) {}
    ~Pinned() {
        if (base) (void)hipHostFree(base);
    }
    int reserve(size_t n) {
        if (n <= cap) return VS_OK;
        if (base) (void)hipHostFree(base);
        base = nullptr;
        cap = 0;
        used = 0;
        size_t c = std::max(n, (size_t)1 << 20);
        if (hipHostMalloc(&base, c, flags) != hipSuccess) {
            set_error("hipHostMalloc failed");
            return VS_ERR_NOMEM;
        }
        cap = c;
        dev = base;
        if ((flags & hipHostMallocMapped) && hipHostGetDevicePointer(&dev, base, 0) != hipSuccess) {
            set_error("hipHostGetDevicePointer failed");
            return VS_ERR_HIP;
        }
        return VS_OK;
    }
    void* dev = nullptr;  // the device's address of base (mapped allocations)
    // the device's address of [p, p + bytes) when it lies in this coherent mapped block, else nullptr
    char* dev_of(const void* p, size_t bytes) const {
        const char* c = static_cast<const char*>(p);
        if (!(flags & hipHostMallocCoherent) || !(flags & hipHostMallocMapped) || c < base || c + bytes > base + cap)
            return nullptr;
        return static_cast<char*>(dev) + (c - base);
    }
    static int copy_kernel(const void* src, void* dst, size_t bytes, hipStream_t st) {
        const int blocks = (int)std::min<size_t>((bytes / 16 + 256) / 256, 64);
        hipLaunchKernelGGL(k_copy_bytes, dim3(blocks), dim3(256), 0, st, static_cast<const char*>(src),
                           static_cast<char*>(dst), bytes);
        VS_HIP(hipGetLastError());
        return VS_OK;
    }
    // dst (in this block) <- src (device memory), enqueued on st
    int to_host(void* dst, const void* src, size_t bytes, hipStream_t st) const {
        if (bytes == 0) return VS_OK;
        if (char* d = dev_of(dst, bytes)) return copy_kernel(src, d, bytes, st);
        VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
        return VS_OK;
    }
    // dst (device memory) <- src (in this block), enqueued on st
    int to_device(void* dst, const void* src, size_t bytes, hipStream_t st) const {
        if (bytes == 0) return VS_OK;
        if (char* d = dev_of(src, bytes)) return copy_kernel(d, dst, bytes, st);
        VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
        return VS_OK;
    }
    char* take(size_t n) {
        size_t o = (used + 15) & ~(size_t)15;
        if (o + n > cap) return nullptr;
        used = o + n;
        return base + o;
    }
};

// Chain result block layout (device and pinned host copy):
//   ints[32]: 0-1 pair slots, 2 seed, 3 nraw, 4 ngood, 5 nkept, 6 ok3d, 7 okE, 8-15 F diag,
//             16-19 3D-3D diag, 20-27 E diag
//   doubles[36]: 0-8 F, 9-10 epipolar errors, 11-19 R3, 20-22 t3, 23-31 RE, 32-34 tE, 35 scale
//   good[cap], kept[cap], then raw[cap] (never copied back)
constexpr size_t kChainInts = 0, kChainDbl = 128, kChainGood = 128 + 36 * 8;
constexpr size_t kChainKept = kChainGood + (size_t)kCap * sizeof(vs_match);
constexpr size_t kChainRaw = kChainKept + (size_t)kCap * sizeof(vs_match);
constexpr size_t kChainSync = kChainRaw + (size_t)kCap * sizeof(vs_match);  // k_ransac3d's arrival counter + results
constexpr int kChainSplit3d = 4;  // k_ransac3d workgroups per chain (its 200 hypotheses on 4 CUs)
constexpr size_t kChainEmSync = kChainSync + 256;  // k_emat's split-workgroup meeting area (one problem)
constexpr int kChainSplitEm = 8;  // k_emat workgroups per chain (its first 64 iterations on the chain's 8 CUs)
constexpr size_t kChainFmSync = kChainEmSync + kEmSyncBytes;  // k_fmat's (one pair)
constexpr size_t kChainBytes = kChainFmSync + kFmSyncBytes;
// chain header: pair slots, the 3D-3D seed, 0, then its MT19937 init_genrand state
constexpr int kHdrWords = 4 + 624;
constexpr size_t kHdrBytes = kHdrWords * sizeof(uint32_t);
constexpr size_t kSpecBlock = (kHdrBytes + kChainRaw + 64 + 255) & ~(size_t)255;  // a speculation's pinned [header | result]

// Extraction chunks: the batch's network + post-processing runs chunk by chunk on the extraction
// streams while the tracker consumes the chunks already done (process_batch_dev).  The batch is
// split evenly into ceil(nb / chunk) chunks (8, 8, 8, 8 at B = 32; 8, 8, 7, 7 at 30: never a
// short tail chunk that runs the whole network for one frame).  Round 1 (tracking-bound, no
// prefetch) wanted a small first chunk; with the next batch prefetched behind the current one and
// the tracker faster than the network, larger chunks win because the network's small layers
// (60 x 80 conv4 / heads) fill the chip better (same-box A/B, 4 rounds: 3, 4, 5, 7, 8, 5 -> 1624;
// 8, 8, 8, 8 -> 1688 frames/s).  VS_SLAM_CHUNK (1..kXChunk) sets the target chunk size.
constexpr int kXChunk = 16;
constexpr int kXFirst = 8;

// Host-side wall time per back-end operation (VS_SLAM_HOST_PROFILE=1: printed to stderr when the
// vs_slam is destroyed); the rest of process_frame is the tracker's own host logic.
enum HostOp { kHChain, kHMatch, kHFmat, kHMotion, kHTlm, kHPnp, kHMatchMap, kHAppend, kHVis, kHFrame, kHWait, kHSpec, kHLoop,
              kHTlmSync, kHSpecNext, kHOps };
static const char* const kHostOpNames[kHOps] = {"chain", "match", "find_fundamental", "motion_points",
                                                "track_local_map", "solve_pnp", "match_map", "map_append",
                                                "visibility", "process_frame (total)", "extract wait",
                                                "chain: speculation wait", "loop_eval", "track_local_map: sync",
                                                "next chain read-ahead wait"};
struct HostProf {
    bool on = false;
    long skip = 64;  // frames before counting starts (first launches load code objects)
    double ms[kHOps] = {};
    long n[kHOps] = {};
};
struct HostTimer {
    HostProf& p;
    int k;
    std::chrono::steady_clock::time_point t0;
    HostTimer(HostProf& pp, int kk) : p(pp), k(kk) {
        if (p.on) t0 = std::chrono::steady_clock::now();
    }
    ~HostTimer() {
        if (!p.on) return;
        p.ms[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        p.n[k]++;
    }
};

// One helper thread that enqueues the NEXT batch's extraction (≈ 200 HIP calls: per chunk the
// network layers, post-processing, copies and events) while the caller's thread goes on tracking
// the current batch.  One task at a time; join() waits for it and hands its error over.
struct AsyncEnqueue {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<int()> task;
    bool has_task = false, busy = false, quit = false;
    int rc = VS_OK;
    std::string err;
    const char* what = "next-batch extraction";
    void start(int device) {
        th = std::thread([this, device] {
            (void)hipSetDevice(device);
            for (;;) {
                std::function<int()> t;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return has_task || quit; });
                    if (!has_task) return;
                    t = std::move(task);
                    has_task = false;
                    busy = true;
                }
                const int r = t();
                const std::string e = r != VS_OK ? std::string(vs_last_error()) : std::string();
                {
                    std::lock_guard<std::mutex> lk(mu);
                    if (r != VS_OK && rc == VS_OK) {
                        rc = r;
                        err = e;
                    }
                    busy = false;
                }
                cv.notify_all();
            }
        });
    }
    void submit(std::function<int()> f) {
        {
            std::lock_guard<std::mutex> lk(mu);
            task = std::move(f);
            has_task = true;
        }
        cv.notify_all();
    }
    int join() {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !has_task && !busy; });
        const int r = rc;
        rc = VS_OK;
        if (r != VS_OK) set_error(std::string("vs_slam: ") + what + ": " + err);
        return r;
    }
    void stop() {
        if (!th.joinable()) return;
        (void)join();
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv.notify_all();
        th.join();
    }
};

struct GpuOps {
    vs_ctx* ctx = nullptr;
    AsyncEnqueue aq;
    bool async_enqueue = true;  // VS_SLAM_ASYNC_ENQUEUE=0: enqueue the next batch on the caller's thread
    // A second helper launches the next frame's speculative chain (≈ 40 us of HIP calls) as soon as
    // chain() has decided it, beside this thread's local-map tracking launches
    // (VS_SLAM_SPEC_ASYNC=0: launched on this thread once the tracking kernels are enqueued).
    AsyncEnqueue sq;
    bool spec_async = true, spec_inflight = false;
    HostProf hprof;
    bool hprof_armed = false;
    // speculative PnP of the tracked points, run right behind local-map tracking (see solve_pnp)
    bool spec_valid = false;
    vs_trk::PnPResult spec;
    std::vector<float> spec_obj, spec_img;
    hipStream_t s = nullptr;   // tracking stream (the context's stream is swapped to it during vs_slam calls)
    hipStream_t xs = nullptr;  // extraction stream (the network)
    // post-processing stream on the extraction CU set: a chunk's decode / NMS / sampling / copies run
    // here while the network of the next chunk already runs on xs
    hipStream_t xp = nullptr;
    hipEvent_t region_done[2] = {nullptr, nullptr};  // last post-processing that read a region's network output
    hipEvent_t xdone = nullptr;  // the last extraction enqueued (ctx->scratch_busy while this vs_slam lives)
    // Speculative front chain of the batch's next frame (see chain()): its own stream on the tracking
    // CU set, result block, header, matcher key state and pinned host block [header | result].
    hipStream_t s2 = nullptr;
    DevBuf mstate2;
    Pinned cpin{hipHostMallocCoherent | hipHostMallocMapped};
    // Up to two speculative chains in flight on s2 (VS_SLAM_SPEC_DEPTH=2, the default): the next frame's
    // and the one after it, whose reference frame is picked on the device (k_pick_ref) from the ratio-test
    // count of the chain before it, by the keyframe rule chain() predicts with.  Each has its own result
    // block, header, event and pinned [header | result] block.
    struct ChainSpec {
        bool valid = false;
        const vs_trk::Frame* cur = nullptr;
        int ref_slot = -1, cur_slot = -1;  // ref_slot < 0: picked on the device, read back with the result
        uint32_t seed = 0;
        int kf_slot = -1, base_slot = -1, gap = 0;  // the device pick's inputs
        long seq = 0, prev_seq = 0;                 // launch order; the chain whose count the pick read
        hipEvent_t ev = nullptr;
        DevBuf buf, hdr;
        char* hbase = nullptr;
    } cspec[2];
    long cspec_seq = 0;
    int spec_depth = 2;  // VS_SLAM_SPEC_DEPTH=1: one chain ahead only
    int find_spec(const vs_trk::Frame* f) const {
        for (int k = 0; k < 2; k++)
            if (cspec[k].valid && cspec[k].cur == f) return k;
        return -1;
    }
    // the reference slot a speculation ran with (a device pick: from its result block, once its event passed)
    int spec_ref_slot(const ChainSpec& E) const {
        return E.ref_slot >= 0 ? E.ref_slot : reinterpret_cast<const int*>(E.hbase + kHdrBytes + kChainInts)[28];
    }
    // E is the chain of the frame in slot cur_slot with seed, against reference rs as the rule decides it
    // for the frame before it (kf_slot / base_slot / gap) on the count of the chain prev_seq: host-chosen
    // with rs, or device-picked from that same chain and candidates
    static bool spec_matches(const ChainSpec& E, int rs, int kf_slot, int base_slot, int gap, uint32_t seed,
                             long prev_seq, int cur_slot) {
        if (!E.valid || E.cur_slot != cur_slot || E.seed != seed) return false;
        if (E.ref_slot >= 0) return E.ref_slot == rs;
        return prev_seq != 0 && E.prev_seq == prev_seq && E.kf_slot == kf_slot && E.base_slot == base_slot &&
               E.gap == gap;
    }
    bool cspec_on = true;                       // VS_SLAM_SPEC_CHAIN=0 disables
    const vs_trk::Frame* next_frame = nullptr;  // the batch's next frame (process_batch_dev)
    hipEvent_t next_ready = nullptr;            // its extraction chunk's event
    long cspec_hits = 0, cspec_launched = 0;
    struct SpecReq {  // the speculation chain() decided on, launched by flush_spec()
        bool pending = false;
        int ref_slot = -1, nxt_slot = -1;
        const vs_trk::Frame* nxt = nullptr;
        uint32_t seed = 0;
        hipEvent_t ready = nullptr;
    } spec_req;
    bool own_streams = false;
    // One extraction in flight or in use: chunk boundaries (frame index of each chunk's first frame,
    // then nb), one event per chunk, the pinned keypoints / counts, the batch region it writes and
    // the caller's frame buffers.  Two sets: the batch being tracked and the next one, prefetched
    // (vs_slam_prefetch_batch_dev) into the other region while this one is tracked.
    struct XBatch {
        std::vector<int> ch;
        std::vector<hipEvent_t> ev;   // chunk c post-processed (xp)
        std::vector<hipEvent_t> net;  // chunk c's network done (xs)
        Pinned pin;
        int region = 0, nb = 0;
        const uint8_t* bgr = nullptr;
        const float* depth = nullptr;
        bool pending = false;  // prefetched, not yet claimed by a process_batch_dev call
    } xb[2];
    int xcur = 0;                      // the set of the batch being tracked
    struct {
        int nb = 0;
        const uint8_t* bgr = nullptr;
        const float* depth = nullptr;
    } hint;                            // the next batch, to prefetch behind the current one

    int chunk = kXFirst;          // target frames per extraction chunk (VS_SLAM_CHUNK overrides)
    int B = 0, h = 0, w = 0, S = 0, batch_region = 0;
    double K[4] = {vs_trk::cfg::FX, vs_trk::cfg::FY, vs_trk::cfg::CX, vs_trk::cfg::CY};
    DevBuf pool_kps, pool_desc, pool_n, pool_depth, pool_norms, semi, dgrid;
    DevBuf pool_grid;  // per slot: the keypoint grid of local-map tracking (vs::kTlmGridInts ints, round 6)
    bool pre_grid = true;  // VS_SLAM_PRE_GRID=0: the grid kernel in the tracking chain instead (A/B)
    DevBuf chain_buf, work, rows_buf, map_pos, map_desc, map_valid, map_tmp, pnp_io, hdr_buf;
    int map_cap = 0, map_n = 0;
    bool valid_dirty = false;
    Pinned pin{hipHostMallocCoherent | hipHostMallocMapped};  // results come back by k_copy_bytes (d2h)
    std::vector<vs_trk::Frame*> owner;  // persistent slot owners (slots 2B .. 2B + kPersist)
    // Keyframe feature archive (loop closure reads keyframes long after their slots are gone):
    // [arch_cap][kCap] keypoints, [arch_cap][kCap][256] descriptors, [arch_cap] counts.
    DevBuf arch_kps, arch_desc, arch_n;
    int arch_cap = 0, arch_used = 0;
    std::vector<CopyJob> cjobs;  // pending copies, one k_copy_jobs launch per flush_copies()
    DevBuf cjob_buf;
    DevBuf lc_buf;  // loop-closure candidate pool and outputs
    DevBuf dlt_buf;  // [kCap] DLT solutions of a keyframe match (match_dlt)
    int err = VS_OK;                     // first error inside an Ops call (the tracker has no error channel)

    vs_keypoint* kps_of(int slot) const { return pool_kps.as<vs_keypoint>() + (size_t)slot * kCap; }
    float* desc_of(int slot) const { return pool_desc.as<float>() + (size_t)slot * kCap * 256; }
    float* depth_of(int slot) const { return pool_depth.as<float>() + (size_t)slot * h * w; }
    float* norms_of(int slot) const { return pool_norms.as<float>() + (size_t)slot * kCap; }
    int* grid_of(int slot) const { return pool_grid.as<int>() + (size_t)slot * kTlmGridInts; }

    // Two streams on disjoint CU sets: the latency-bound tracking kernels keep VS_SLAM_TRACK_CUS
    // (default 32) CUs to themselves, so they never queue behind the network's long-running
    // workgroups, and the next chunks' network runs on the rest meanwhile.  Plain streams when
    // the CU-mask extension is unavailable.
    int make_streams() {
        int ncu = 0;
        VS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        const char* env = std::getenv("VS_SLAM_TRACK_CUS");
        const int tcu = env ? std::atoi(env) : 32;
        // VS_SLAM_SPEC_CUS > 0: the speculative chain gets CUs of its own, carved from the
        // extraction set.  Default 32 (round 3): with the chain launched at chain() time it overlaps
        // the local-map / PnP kernels, whose 100 one-wave EPnP hypotheses then share SIMDs with the
        // chain's 1024-wave RANSAC grids (k_pnp_hyp median 190 -> 139 us with a CU set of its own);
        // the Winograd network keeps up on the remaining 192 CUs.  Same-box host profile
        // (profiles/r03t_*): process_frame 496 / 466 / 457 us and 1,943 / 2,029 / 2,061 frames/s at
        // 0 / 16 / 32 chain CUs.  0: the chain shares the tracking CUs.  Round 4 default 8: with the
        // tracker at ~0.40 ms per frame the chain (one F-RANSAC workgroup, a 3D-3D grid) still ends
        // before its frame is tracked on 8 CUs, and the network gains 24: same box, three rounds,
        // 2,305 -> 2,339 frames/s (profiles/r04z_cu_partition.txt; 4 CUs: 2,252).
        const char* senv = std::getenv("VS_SLAM_SPEC_CUS");
        const int scu = senv ? std::max(0, std::atoi(senv)) : 8;
        // VS_SLAM_POST_CUS > 0: the extraction post-processing (xp) gets CUs of its own, taken from
        // the network's set (default 0: it shares the network's CUs)
        const char* penv = std::getenv("VS_SLAM_POST_CUS");
        const int pcu = penv ? std::max(0, std::atoi(penv)) : 0;
        bool masked = false;
        if (tcu > 0 && ncu >= 2 * (tcu + scu + pcu)) {
            const int words = (ncu + 31) / 32;
            std::vector<uint32_t> tm(words, 0u), xm(words, 0u), sm(words, 0u), pm(words, 0u);
            // VS_SLAM_CU_SPREAD=1 (experiments): each set takes the same share of every 1/8 of the CU
            // ids (one XCD each when the ids run XCD by XCD) instead of one contiguous range
            const char* spr = std::getenv("VS_SLAM_CU_SPREAD");
            const bool spread = spr && spr[0] == '1' && ncu % 8 == 0;
            for (int cu = 0; cu < ncu; cu++) {
                const int j = spread ? cu % (ncu / 8) : cu;
                const int t = spread ? tcu / 8 : tcu, sp = spread ? scu / 8 : scu, pp = spread ? pcu / 8 : pcu;
                (j < t ? tm : j < t + sp ? sm : j < t + sp + pp ? pm : xm)[cu / 32] |= 1u << (cu % 32);
            }
            if (scu == 0) sm = tm;
            if (pcu == 0) pm = xm;
            // VS_SLAM_SPEC_SET=net with VS_SLAM_SPEC_CUS=0 (experiments): the speculative chain on the
            // network's CUs instead of the tracking CUs
            if (const char* ss = std::getenv("VS_SLAM_SPEC_SET"))
                if (scu == 0 && std::strcmp(ss, "net") == 0) sm = xm;
            // VS_SLAM_POST_SET = track / spec / all: the post-processing stream on the tracking CUs, the chain's, or on
            // every CU (experiments: the tracking CUs idle between latency-bound kernels)
            if (const char* ps = std::getenv("VS_SLAM_POST_SET")) {
                if (std::strcmp(ps, "track") == 0) pm = tm;
                if (std::strcmp(ps, "spec") == 0 && scu > 0) pm = sm;
                if (std::strcmp(ps, "all") == 0)
                    for (int k = 0; k < words; k++) pm[k] = tm[k] | xm[k] | sm[k];
            }
            // VS_SLAM_NET_SET = spec (default) / none / track / all: the network stream also on the
            // speculative chains' CUs (with two chains in flight they wait for the network's frames
            // anyway; the headline is extraction-bound: +3.5 %, profiles/r06s_net_on_spec_cus_ab.txt), on
            // the tracking CUs (-9 %: the tracking chain is latency-bound) or both
            {
                const char* ns = std::getenv("VS_SLAM_NET_SET");
                if (!ns) ns = "spec";
                const bool wspec = std::strcmp(ns, "spec") == 0 || std::strcmp(ns, "all") == 0;
                const bool wtrack = std::strcmp(ns, "track") == 0 || std::strcmp(ns, "all") == 0;
                for (int k = 0; k < words; k++) xm[k] |= (wspec ? sm[k] : 0u) | (wtrack ? tm[k] : 0u);
            }
            masked = hipExtStreamCreateWithCUMask(&s, words, tm.data()) == hipSuccess;
            if (masked && hipExtStreamCreateWithCUMask(&xs, words, xm.data()) != hipSuccess) {
                (void)hipStreamDestroy(s);
                s = nullptr;
                masked = false;
            }
            if (masked && hipExtStreamCreateWithCUMask(&s2, words, sm.data()) != hipSuccess) {
                (void)hipStreamDestroy(s);
                (void)hipStreamDestroy(xs);
                s = xs = nullptr;
                masked = false;
            }
            if (masked && hipExtStreamCreateWithCUMask(&xp, words, pm.data()) != hipSuccess) {
                (void)hipStreamDestroy(s);
                (void)hipStreamDestroy(xs);
                (void)hipStreamDestroy(s2);
                s = xs = s2 = nullptr;
                masked = false;
            }
        }
        if (!masked) {
            VS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            VS_HIP(hipStreamCreateWithFlags(&xs, hipStreamNonBlocking));
            VS_HIP(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
            VS_HIP(hipStreamCreateWithFlags(&xp, hipStreamNonBlocking));
        }
        for (auto& e : region_done) VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        for (auto& E : cspec) VS_HIP(hipEventCreateWithFlags(&E.ev, hipEventDisableTiming));
        VS_HIP(hipEventCreateWithFlags(&tlm_ev, hipEventDisableTiming));
        VS_HIP(hipEventCreateWithFlags(&tspec.ev, hipEventDisableTiming));
        VS_HIP(hipEventCreateWithFlags(&xdone, hipEventDisableTiming));
        // the extraction streams share the context's network / NMS scratch: any other stream that
        // uses it waits for the last extraction enqueued here (vs::scratch_order)
        ctx->scratch_busy = xdone;
        ctx->scratch_owner[0] = xs;
        ctx->scratch_owner[1] = xp;
        own_streams = true;
        return VS_OK;
    }
    void destroy_streams() {
        aq.stop();  // no enqueue may still be running when the streams go
        sq.stop();
        if (!own_streams) return;
        (void)hipStreamSynchronize(xs);
        (void)hipStreamSynchronize(xp);
        (void)hipStreamSynchronize(s);
        (void)hipStreamSynchronize(s2);
        if (ctx->scratch_busy == xdone) {
            ctx->scratch_busy = nullptr;
            ctx->scratch_owner[0] = ctx->scratch_owner[1] = nullptr;
        }
        (void)hipEventDestroy(xdone);
        for (auto& e : region_done) (void)hipEventDestroy(e);
        for (auto& X : xb) {
            for (hipEvent_t e : X.ev) (void)hipEventDestroy(e);
            for (hipEvent_t e : X.net) (void)hipEventDestroy(e);
            X.ev.clear();
            X.net.clear();
        }
        for (auto& E : cspec) (void)hipEventDestroy(E.ev);
        (void)hipEventDestroy(tlm_ev);
        (void)hipEventDestroy(tspec.ev);
        (void)hipStreamDestroy(xs);
        (void)hipStreamDestroy(xp);
        (void)hipStreamDestroy(s);
        (void)hipStreamDestroy(s2);
        own_streams = false;
    }

    int init(vs_ctx* c, int max_batch, int hh, int ww) {
        ctx = c;
        VS_CHECK(make_streams());
        if (const char* e = std::getenv("VS_SLAM_ASYNC_ENQUEUE")) async_enqueue = e[0] != '0';
        if (async_enqueue) aq.start(ctx->device);
        if (const char* e = std::getenv("VS_SLAM_SPEC_ASYNC")) spec_async = e[0] != '0';
        sq.what = "speculative chain launch";
        if (spec_async) sq.start(ctx->device);
        if (const char* fc = std::getenv("VS_SLAM_CHUNK")) chunk = std::max(1, std::min(kXChunk, std::atoi(fc)));
        const char* hp = std::getenv("VS_SLAM_HOST_PROFILE");
        hprof.on = hp && hp[0] == '1';
        if (hprof.on) hprof.on = false, hprof.skip = 64, hprof_armed = true;
        B = max_batch;
        h = hh;
        w = ww;
        S = 2 * B + kPersist;
        VS_CHECK(pool_kps.ensure((size_t)S * kCap * sizeof(vs_keypoint)));
        VS_CHECK(pool_desc.ensure((size_t)S * kCap * 256 * sizeof(float)));
        VS_CHECK(pool_n.ensure((size_t)S * sizeof(int)));
        VS_CHECK(pool_depth.ensure((size_t)S * h * w * sizeof(float)));
        VS_CHECK(pool_norms.ensure((size_t)S * kCap * sizeof(float)));
        VS_CHECK(pool_grid.ensure((size_t)S * kTlmGridInts * sizeof(int)));
        if (const char* e = std::getenv("VS_SLAM_PRE_GRID")) pre_grid = e[0] != '0';
        VS_HIP(hipMemsetAsync(pool_n.p, 0, (size_t)S * sizeof(int), s));
        const int hc = (h + 7) / 8, wc = (w + 7) / 8;
        // network outputs per batch region (2 B frames): a chunk's post-processing reads its own
        // frames' rows while later chunks (and the prefetched batch) write theirs
        VS_CHECK(semi.ensure((size_t)2 * B * hc * wc * VS_SEMI_CH * sizeof(float)));
        VS_CHECK(dgrid.ensure((size_t)2 * B * hc * wc * VS_DESC_DIM * sizeof(float)));
        VS_CHECK(chain_buf.ensure(kChainBytes));
        VS_HIP(hipMemsetAsync(chain_buf.as<char>() + kChainSync, 0, kChainBytes - kChainSync, s));
        if (const char* e = std::getenv("VS_SLAM_R3_SPLIT")) r3_split = std::max(1, std::min(kMaxSplit3d, std::atoi(e)));
        VS_CHECK(hdr_buf.ensure(kHdrBytes));
        VS_CHECK(mstate2.ensure(2 * kCap * sizeof(unsigned long long) + 256));
        VS_HIP(hipMemsetAsync(mstate2.p, 0xFF, 2 * kCap * sizeof(unsigned long long), s));
        VS_HIP(hipMemsetAsync(mstate2.as<char>() + 2 * kCap * sizeof(unsigned long long), 0, 256, s));
        for (auto& E : cspec) {
            VS_CHECK(E.buf.ensure(kChainBytes));
            VS_HIP(hipMemsetAsync(E.buf.as<char>() + kChainSync, 0, kChainBytes - kChainSync, s));
            VS_CHECK(E.hdr.ensure(kHdrBytes));
        }
        VS_CHECK(cpin.reserve(2 * kSpecBlock));
        for (int k = 0; k < 2; k++) cspec[k].hbase = cpin.base + k * kSpecBlock;
        if (const char* e = std::getenv("VS_SLAM_SPEC_DEPTH")) spec_depth = std::max(1, std::min(2, std::atoi(e)));
        if (const char* e = std::getenv("VS_SLAM_SPEC_CHAIN")) cspec_on = e[0] != '0';
        VS_CHECK(pin.reserve((size_t)4 << 20));
        VS_CHECK(spin.reserve((size_t)1 << 20));  // one speculation: <= 8 KB table + ~60 KB results at 1024 keypoints
        if (const char* e = std::getenv("VS_SLAM_SPEC_TLM")) tlm_spec_on = e[0] != '0';
        owner.assign(kPersist, nullptr);
        VS_CHECK(grow_map(1 << 16));
        // map-sized scratch up front (a later growth would wait for the extraction stream too):
        // map_tmp holds the gathered descriptors of PnP-recovery / loop-closure map matching (1 KB per
        // candidate map point; 64 MB = 65k points, the size grow_map starts with)
        VS_CHECK(map_tmp.ensure((size_t)64 << 20));
        VS_CHECK(work.ensure((size_t)1 << 20));
        VS_CHECK(pnp_io.ensure((size_t)1 << 20));
        VS_CHECK(dlt_buf.ensure((size_t)kCap * sizeof(float4)));
        VS_CHECK(rows_buf.ensure((size_t)64 << 10));
        // the context's per-stage scratch at its largest in-loop size: local-map tracking for 200k
        // map points, PnP hypothesis tables for the largest RANSAC budget (loop closure: 300)
        VS_CHECK(ctx->tlm.ensure((size_t)64 << 20));
        VS_HIP(hipMemsetAsync(ctx->tlm.p, 0, 16, s));  // the work list's length (k_tlm_best re-zeroes it)
        VS_CHECK(ctx->pnp.ensure((size_t)4 * VS_PNP_MAX_ITERS * (6 * sizeof(int) + 6 * sizeof(double))));
        VS_CHECK(pnp_reserve(ctx, s));  // the PnP subset table (built once here, not in the loop)
        VS_CHECK(emat_reserve(ctx, s));  // and findEssentialMat's
        // Loop closure (every 200 keyframes, candidates every 5th keyframe >= 200 ids back,
        // LoopCloser.cpp:44-49): the keyframe archive for kArchInit keyframes (215 MB of HBM), the
        // candidate pool and the matcher key state for kLoopPairs candidates, reserved here because
        // every hipFree inside the loop waits for the extraction stream as well.
        VS_CHECK(grow_archive(kArchInit));
        VS_CHECK(lc_buf.ensure(LcLayout(kLoopPairs).total));
        VS_CHECK(match_reserve(ctx, kLoopPairs, kCap, s));
        VS_HIP(hipStreamSynchronize(s));
        return VS_OK;
    }

    int sync() {
        VS_HIP(hipStreamSynchronize(s));
        pin.used = 0;
        return VS_OK;
    }
    // pinned staging space; synchronises (and grows) when the area is exhausted
    char* take(size_t n) {
        char* p = pin.take(n);
        if (p) return p;
        if (failed(sync()) || failed(pin.reserve(n + 64))) return nullptr;
        return pin.take(n);
    }
    int d2h(void* dst, const void* src, size_t bytes) { return pin.to_host(dst, src, bytes, s); }
    // H2D of a host array through the pinned staging area
    int upload(void* dst, const void* src, size_t bytes) {
        if (bytes == 0) return VS_OK;
        char* p = pin.take(bytes);
        if (!p) {
            VS_CHECK(sync());
            VS_CHECK(pin.reserve(bytes + 64));
            p = pin.take(bytes);
        }
        std::memcpy(p, src, bytes);
        return pin.to_device(dst, p, bytes, s);
    }

    int grow_map(int need) {
        if (need <= map_cap) return VS_OK;
        map_ver++;
        int cap = std::max(need, map_cap * 2);
        DevBuf np, nd, nv;
        VS_CHECK(np.ensure((size_t)cap * 3 * sizeof(double)));
        VS_CHECK(nd.ensure((size_t)cap * 256 * sizeof(float)));
        VS_CHECK(nv.ensure((size_t)cap));
        if (map_n > 0) {
            VS_HIP(hipMemcpyAsync(np.p, map_pos.p, (size_t)map_n * 3 * sizeof(double), hipMemcpyDeviceToDevice, s));
            VS_HIP(hipMemcpyAsync(nd.p, map_desc.p, (size_t)map_n * 256 * sizeof(float), hipMemcpyDeviceToDevice, s));
            VS_HIP(hipMemcpyAsync(nv.p, map_valid.p, (size_t)map_n, hipMemcpyDeviceToDevice, s));
        }
        VS_HIP(hipStreamSynchronize(s));
        map_pos.release();
        map_desc.release();
        map_valid.release();
        map_pos = np;
        map_desc = nd;
        map_valid = nv;
        np.p = nd.p = nv.p = nullptr;  // ownership moved
        map_cap = cap;
        return VS_OK;
    }

    int sync_valid(const vs_trk::Map& m) {
        if (!valid_dirty) return VS_OK;
        VS_CHECK(upload(map_valid.p, m.valid.data(), m.valid.size()));
        valid_dirty = false;
        return VS_OK;
    }

    // ---- frame slots -----------------------------------------------------------------------
    int persistent_slot(vs_trk::Frame* f) {
        for (int i = 0; i < kPersist; i++)
            if (!owner[i]) {
                owner[i] = f;
                return 2 * B + i;
            }
        set_error("vs_slam: out of persistent frame slots");
        return -1;
    }
    void release_slot(vs_trk::Frame* f) {
        if (f->slot >= 2 * B) owner[f->slot - 2 * B] = nullptr;
        f->slot = -1;
    }
    // queued: the caller flushes (flush_copies) before anything reads slot `to`
    int copy_slot(int from, int to) {
        cjobs.push_back({kps_of(from), kps_of(to), kCap * sizeof(vs_keypoint)});
        cjobs.push_back({desc_of(from), desc_of(to), (size_t)kCap * 256 * sizeof(float)});
        cjobs.push_back({pool_n.as<int>() + from, pool_n.as<int>() + to, sizeof(int)});
        cjobs.push_back({depth_of(from), depth_of(to), (size_t)h * w * sizeof(float)});
        cjobs.push_back({norms_of(from), norms_of(to), kCap * sizeof(float)});
        cjobs.push_back({grid_of(from), grid_of(to), (size_t)kTlmGridInts * sizeof(int)});
        return VS_OK;
    }
    int flush_copies() {
        if (cjobs.empty()) return VS_OK;
        const int nj = (int)cjobs.size();
        size_t mx = 0;
        for (const CopyJob& j : cjobs) mx = std::max(mx, (size_t)j.bytes);
        VS_CHECK(cjob_buf.ensure((size_t)nj * sizeof(CopyJob)));
        VS_CHECK(upload(cjob_buf.p, cjobs.data(), (size_t)nj * sizeof(CopyJob)));
        const unsigned bx = (unsigned)std::min<size_t>(64, std::max<size_t>(1, (mx / 16 + 255) / 256));
        hipLaunchKernelGGL(k_copy_jobs, dim3(bx, nj), dim3(256), 0, s, cjob_buf.as<CopyJob>());
        cjobs.clear();
        VS_HIP(hipGetLastError());
        return VS_OK;
    }
    // Host features (SPCF cache / caller-extracted) into a persistent slot.
    int upload_frame(vs_trk::Frame& f, const float* desc) {
        const int slot = persistent_slot(&f);
        if (slot < 0) return VS_ERR_CAPACITY;
        f.slot = slot;
        const int n = (int)f.kps.size();
        VS_CHECK(upload(kps_of(slot), f.kps.data(), (size_t)n * sizeof(vs_keypoint)));
        VS_CHECK(upload(desc_of(slot), desc, (size_t)n * 256 * sizeof(float)));
        VS_CHECK(upload(pool_n.as<int>() + slot, &n, sizeof(int)));
        VS_CHECK(desc_norms(ctx, 1, desc_of(slot), pool_n.as<int>() + slot, kCap, norms_of(slot), s));
        VS_CHECK(tlm_grid_slots(kps_of(slot), pool_n.as<int>() + slot, 1, kCap, vs_trk::cfg::IMAGE_WIDTH,
                                vs_trk::cfg::IMAGE_HEIGHT, grid_of(slot), s));
        if (f.depth)
            VS_CHECK(upload(depth_of(slot), f.depth, (size_t)h * w * sizeof(float)));
        else
            VS_HIP(hipMemsetAsync(depth_of(slot), 0, (size_t)h * w * sizeof(float), s));
        return VS_OK;
    }
    // B frames already in HBM -> network + post-processing straight into batch region slots,
    // depth copied beside them, keypoints back to pinned host memory, one chunk (<= kXChunk frames) at a time on
    // the extraction stream; chunk c's event marks its slots and host keypoints ready.  Enqueue
    // only: wait_chunk() hands a chunk to the tracker.
    int enqueue_extraction(XBatch& X, int nb, const uint8_t* d_bgr, const float* d_depth) {
        X.region = batch_region;
        batch_region ^= 1;
        X.nb = nb;
        X.bgr = d_bgr;
        X.depth = d_depth;
        const int s0 = X.region * B;
        X.ch.assign(1, 0);
        const int nch_even = (nb + chunk - 1) / chunk;  // even split, no short tail chunk
        for (int c = 0; c < nch_even; c++) X.ch.push_back(X.ch.back() + nb / nch_even + (c < nb % nch_even ? 1 : 0));
        const int nch = (int)X.ch.size() - 1;
        while ((int)X.ev.size() < nch) {
            hipEvent_t e, en;
            VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            VS_HIP(hipEventCreateWithFlags(&en, hipEventDisableTiming));
            X.ev.push_back(e);
            X.net.push_back(en);
        }
        VS_CHECK(X.pin.reserve((size_t)nb * kCap * sizeof(vs_keypoint) + (size_t)nb * sizeof(int) + 64));
        char* hk = X.pin.base;
        int* hn = reinterpret_cast<int*>(hk + (size_t)nb * kCap * sizeof(vs_keypoint));
        const int hc = (h + 7) / 8, wc = (w + 7) / 8;
        // the region's previous batch has finished reading its network outputs, and work the caller
        // enqueued on other streams over the context's shared scratch has finished with it
        VS_HIP(hipStreamWaitEvent(xs, region_done[X.region], 0));
        VS_CHECK(scratch_acquire_owner(ctx, xs));
        const size_t semi_f = (size_t)hc * wc * VS_SEMI_CH, dgrid_f = (size_t)hc * wc * VS_DESC_DIM;
        for (int c = 0; c < nch; c++) {
            const int f0 = X.ch[c], m = X.ch[c + 1] - X.ch[c];
            float* sm = semi.as<float>() + (size_t)(s0 + f0) * semi_f;
            float* dg = dgrid.as<float>() + (size_t)(s0 + f0) * dgrid_f;
            VS_CHECK(sp_forward(ctx, m, d_bgr + (size_t)f0 * h * w * 3, 3, h, w, xs, sm, dg, true));
            VS_HIP(hipEventRecord(X.net[c], xs));
            VS_HIP(hipStreamWaitEvent(xp, X.net[c], 0));
            VS_CHECK(sp_postprocess(ctx, m, hc, wc, h, w, kps_of(s0 + f0), desc_of(s0 + f0), pool_n.as<int>() + s0 + f0,
                                    kCap, xp, sm, dg, true));
            // descriptor row norms once per frame (matching reuses them for every pair)
            VS_CHECK(desc_norms(ctx, m, desc_of(s0 + f0), pool_n.as<int>() + s0 + f0, kCap, norms_of(s0 + f0), xp));
            // the keypoint grid of local-map tracking, per frame, while the keypoints are fresh (round 6:
            // one kernel off the tracking chain)
            VS_CHECK(tlm_grid_slots(kps_of(s0 + f0), pool_n.as<int>() + s0 + f0, m, kCap, vs_trk::cfg::IMAGE_WIDTH,
                                    vs_trk::cfg::IMAGE_HEIGHT, grid_of(s0 + f0), xp));
            if (d_depth)
                VS_HIP(hipMemcpyAsync(depth_of(s0 + f0), d_depth + (size_t)f0 * h * w, (size_t)m * h * w * sizeof(float),
                                      hipMemcpyDeviceToDevice, xp));
            else
                VS_HIP(hipMemsetAsync(depth_of(s0 + f0), 0, (size_t)m * h * w * sizeof(float), xp));
            VS_HIP(hipMemcpyAsync(hk + (size_t)f0 * kCap * sizeof(vs_keypoint), kps_of(s0 + f0),
                                  (size_t)m * kCap * sizeof(vs_keypoint), hipMemcpyDeviceToHost, xp));
            VS_HIP(hipMemcpyAsync(hn + f0, pool_n.as<int>() + s0 + f0, (size_t)m * sizeof(int), hipMemcpyDeviceToHost, xp));
            VS_HIP(hipEventRecord(X.ev[c], xp));
        }
        VS_HIP(hipEventRecord(region_done[X.region], xp));
        VS_HIP(hipEventRecord(xdone, xp));  // covers xs too (xp waited for every chunk's network)
        return VS_OK;
    }
    // The batch's extraction: the one prefetched for exactly these buffers, or enqueued now; then the
    // hinted next batch is prefetched behind it into the other region (free: the previous batch's
    // live frames moved to persistent slots when it settled).
    int extract_batch(std::vector<vs_trk::FramePtr>& frames, const uint8_t* d_bgr, const float* d_depth) {
        VS_CHECK(aq.join());  // the previous call's prefetch enqueue has finished touching xs / xp / xb
        const int nb = (int)frames.size();
        XBatch& P = xb[xcur ^ 1];
        if (P.pending && !(P.bgr == d_bgr && P.depth == d_depth && P.nb == nb)) {
            VS_HIP(hipStreamSynchronize(xs));  // a stale prefetch: let it land, its region is free again
            VS_HIP(hipStreamSynchronize(xp));
            P.pending = false;
            batch_region = P.region;
        }
        xcur ^= 1;
        XBatch& X = xb[xcur];
        if (X.pending) {
            X.pending = false;
        } else {
            VS_CHECK(enqueue_extraction(X, nb, d_bgr, d_depth));
        }
        for (int b = 0; b < nb; b++) frames[b]->slot = X.region * B + b;
        if (hint.nb > 0) {
            XBatch& N = xb[xcur ^ 1];
            const int hnb = hint.nb;
            const uint8_t* hb = hint.bgr;
            const float* hd = hint.depth;
            hint.nb = 0;
            // pending only once the whole enqueue succeeded: a half-built prefetch is never claimed
            auto task = [this, &N, hnb, hb, hd] {
                const int r = enqueue_extraction(N, hnb, hb, hd);
                N.pending = r == VS_OK;
                return r;
            };
            if (async_enqueue)
                aq.submit(task);
            else
                VS_CHECK(task());
        }
        return VS_OK;
    }
    // Chunk c of the batch is extracted: its keypoints to the frames, and the tracking stream
    // ordered after it.
    int wait_chunk(std::vector<vs_trk::FramePtr>& frames, int c) {
        HostTimer ht(hprof, kHWait);
        const int nb = (int)frames.size();
        const XBatch& X = xb[xcur];
        const int f0 = X.ch[c], m = X.ch[c + 1] - X.ch[c];
        VS_HIP(hipEventSynchronize(X.ev[c]));
        VS_HIP(hipStreamWaitEvent(s, X.ev[c], 0));
        const char* hk = X.pin.base;
        const int* hn = reinterpret_cast<const int*>(hk + (size_t)nb * kCap * sizeof(vs_keypoint));
        for (int b = f0; b < f0 + m; b++) {
            const int n = hn[b];
            if (n == VS_ERR_NOTCONV) {
                set_error("vs_slam: NMS could not be completed for a frame");
                return VS_ERR_NOTCONV;
            }
            if (n < 0 || n > kCap) {
                set_error("vs_slam: keypoint count out of range");
                return VS_ERR_CAPACITY;
            }
            const auto* kp = reinterpret_cast<const vs_trk::Keypoint*>(hk + (size_t)b * kCap * sizeof(vs_keypoint));
            frames[b]->kps.assign(kp, kp + n);
            frames[b]->mp_idx.assign(n, -1);
        }
        return VS_OK;
    }

    // ---- Ops interface (host/tracker.hpp) ----------------------------------------------------
    // Errors cannot propagate through the tracker (the reference has no error channel there):
    // the first one is latched in `err`, results are emptied, and the C ABI reports it.
    bool failed(int rc) {
        if (rc != VS_OK && err == VS_OK) err = rc;
        return rc != VS_OK;
    }

    int enqueue_match(int qslot, int tslot, float ratio, int* meta) {
        const int pr[2] = {qslot, tslot};
        VS_CHECK(upload(meta, pr, sizeof(pr)));
        char* c = chain_buf.as<char>();
        return match_pairs(ctx, 1, meta, S, pool_desc.as<float>(), pool_n.as<int>(), kCap, ratio,
                           reinterpret_cast<vs_match*>(c + kChainRaw), meta + 3, reinterpret_cast<vs_match*>(c + kChainGood),
                           meta + 4, s, pool_norms.as<float>());
    }

    // one header: pair slots, the 3D-3D seed and its MT19937 init_genrand state (624 serial steps,
    // cheaper on the host than on one GPU lane)
    static void fill_hdr(uint32_t* hdr, int ref_slot, int cur_slot, uint32_t seed) {
        hdr[0] = (uint32_t)ref_slot;
        hdr[1] = (uint32_t)cur_slot;
        hdr[2] = seed;
        hdr[3] = 0;
        hdr[4] = seed;
        for (int i = 1; i < 624; i++) hdr[4 + i] = 1812433253u * (hdr[3 + i] ^ (hdr[3 + i] >> 30)) + (uint32_t)i;
    }
    // match -> F verification -> 3D-3D -> E fallback for the pair in the header, on stream st, into
    // the result block cbuf, copied back to hout (pinned); keys / cnt: the matcher's key state
    // (nullptr: the context's)
    struct PickArgs {  // a device-picked reference (k_pick_ref)
        const int* prev;
        int kf_slot, base_slot, gap;
    };
    int enqueue_chain(hipStream_t st, char* cbuf, int* dh, const uint32_t* hhdr, char* hout, unsigned long long* keys,
                      unsigned* cnt, const PickArgs* pick = nullptr) {
        int* di = reinterpret_cast<int*>(cbuf + kChainInts);
        double* dd = reinterpret_cast<double*>(cbuf + kChainDbl);
        vs_match* good = reinterpret_cast<vs_match*>(cbuf + kChainGood);
        vs_match* kept = reinterpret_cast<vs_match*>(cbuf + kChainKept);
        const Pinned& P = (hout >= cpin.base && hout < cpin.base + cpin.cap) ? cpin : pin;  // the speculative or the direct chain
        VS_CHECK(P.to_device(dh, hhdr, kHdrBytes, st));
        if (pick) {
            hipLaunchKernelGGL(k_pick_ref, dim3(1), dim3(64), 0, st, pick->prev, pick->kf_slot, pick->base_slot,
                               pick->gap, dh, di);
            VS_HIP(hipGetLastError());
        }
        VS_CHECK(match_pairs(ctx, 1, dh, S, pool_desc.as<float>(), pool_n.as<int>(), kCap, vs_trk::cfg::L2_RATIO_THRESHOLD,
                             reinterpret_cast<vs_match*>(cbuf + kChainRaw), di + 3, good, di + 4, st,
                             pool_norms.as<float>(), keys, cnt));
        VS_CHECK(fmat_pairs(ctx, 1, dh, pool_kps.as<vs_keypoint>(), kCap, good, di + 4, dd, kept, di + 5, dd + 9, di + 8,
                            st, 0, cbuf + kChainFmSync));
        VS_CHECK(ransac3d_pairs(ctx, 1, dh, pool_kps.as<vs_keypoint>(), kCap, kept, di + 5, pool_depth.as<float>(), h, w,
                                K, reinterpret_cast<const uint32_t*>(dh + 2), 200, 0.05, dd + 11, dd + 20, di + 6, di + 16,
                                st, reinterpret_cast<const uint32_t*>(dh + 4), r3_split,
                                reinterpret_cast<int*>(cbuf + kChainSync)));
        VS_CHECK(emat_pairs(ctx, 1, dh, pool_kps.as<vs_keypoint>(), kCap, kept, di + 5, di + 6, pool_depth.as<float>(), h,
                            w, K, dd + 23, dd + 32, dd + 35, di + 7, di + 20, st, kChainSplitEm, cbuf + kChainEmSync));
        return P.to_host(hout, cbuf, kChainRaw, st);
    }
    static vs_trk::ChainResult parse_chain(const char* hc) {
        vs_trk::ChainResult R;
        const int* hi = reinterpret_cast<const int*>(hc + kChainInts);
        const double* hd = reinterpret_cast<const double*>(hc + kChainDbl);
        const auto* hg = reinterpret_cast<const vs_trk::Match*>(hc + kChainGood);
        const auto* hk = reinterpret_cast<const vs_trk::Match*>(hc + kChainKept);
        R.n_raw = hi[3];
        R.good.assign(hg, hg + hi[4]);
        R.kept.assign(hk, hk + hi[5]);
        R.f_ok = hi[12] != 0;  // F diag[4] = F ok
        R.f_iters = hi[9];     // F diag[1] = iterations run
        R.epi_before = hd[9];
        R.epi_after = hd[10];
        R.ok3d = hi[6] != 0;
        std::memcpy(R.R3.data(), hd + 11, 9 * sizeof(double));
        std::memcpy(R.t3.data(), hd + 20, 3 * sizeof(double));
        R.okE = !R.ok3d && hi[7] != 0;
        std::memcpy(R.RE.data(), hd + 23, 9 * sizeof(double));
        std::memcpy(R.tE.data(), hd + 32, 3 * sizeof(double));
        R.scale = hd[35];
        return R;
    }
    vs_trk::ChainResult chain_impl(const vs_trk::Frame& ref, const vs_trk::Frame& cur, uint32_t seed) {
        uint32_t* hh = reinterpret_cast<uint32_t*>(take(kHdrBytes));
        if (!hh) return vs_trk::ChainResult();
        fill_hdr(hh, ref.slot, cur.slot, seed);
        char* hc = take(kChainRaw);
        if (!hc || failed(enqueue_chain(s, chain_buf.as<char>(), hdr_buf.as<int>(), hh, hc, nullptr, nullptr)) ||
            failed(sync()))
            return vs_trk::ChainResult();
        return parse_chain(hc);
    }
    // The chain of the batch's next frame against this call's reference frame with the next seed,
    // on s2 beside this frame's local-map tracking and PnP: it is the next frame's chain whenever
    // this frame neither becomes a keyframe nor is rejected (the reference frame and the processed
    // count then carry over, Slam.cpp:838, 276).  chain() uses it only when slots and seed match.
    // pick_prev >= 0: the reference is picked on the device from that entry's chain (launched before this
    // one on s2): kf_slot if its frame becomes a keyframe by the rule, else base_slot (gap: that frame's
    // id gap to base_slot's frame).
    int launch_spec_chain(int ref_slot, const vs_trk::Frame& nxt, uint32_t seed, hipEvent_t ready, int pick_prev = -1,
                          int kf_slot = -1, int base_slot = -1, int gap = 0) {
        // the entry: a free one, else the older (never the one the pick reads)
        int k = !cspec[0].valid ? 0 : !cspec[1].valid ? 1 : (cspec[0].seq < cspec[1].seq ? 0 : 1);
        if (k == pick_prev) k ^= 1;
        ChainSpec& E = cspec[k];
        VS_HIP(hipEventSynchronize(E.ev));  // its previous chain released the buffers
        uint32_t* hh = reinterpret_cast<uint32_t*>(E.hbase);
        fill_hdr(hh, pick_prev >= 0 ? base_slot : ref_slot, nxt.slot, seed);
        if (ready) VS_HIP(hipStreamWaitEvent(s2, ready, 0));  // its extraction chunk
        unsigned long long* keys = mstate2.as<unsigned long long>();
        unsigned* cnt = reinterpret_cast<unsigned*>(mstate2.as<char>() + 2 * kCap * sizeof(unsigned long long));
        PickArgs pk{};
        if (pick_prev >= 0) pk = PickArgs{cspec[pick_prev].buf.as<int>(), kf_slot, base_slot, gap};
        VS_CHECK(enqueue_chain(s2, E.buf.as<char>(), E.hdr.as<int>(), hh, E.hbase + kHdrBytes, keys, cnt,
                               pick_prev >= 0 ? &pk : nullptr));
        VS_HIP(hipEventRecord(E.ev, s2));
        E.valid = true;
        E.cur = &nxt;
        E.ref_slot = pick_prev >= 0 ? -1 : ref_slot;
        E.cur_slot = nxt.slot;
        E.seed = seed;
        E.kf_slot = kf_slot;
        E.base_slot = base_slot;
        E.gap = gap;
        E.prev_seq = pick_prev >= 0 ? cspec[pick_prev].seq : 0;
        E.seq = ++cspec_seq;
        cspec_launched++;
        return VS_OK;
    }
    // Waits until the helper has enqueued the speculations it was given (cspec[] and their events are then
    // this thread's again); its error, if any, is latched.
    void spec_sync() {
        if (!spec_inflight) return;
        spec_inflight = false;
        failed(sq.join());
    }
    vs_trk::ChainResult chain(const vs_trk::Frame& ref, const vs_trk::Frame& cur, uint32_t seed) {
        HostTimer ht(hprof, kHChain);
        vs_trk::ChainResult R;
        {
            HostTimer hw(hprof, kHSpec);
            spec_sync();
        }
        // the next frame's chain read back ahead of this call (speculate_next), the frame after it then
        // already launched
        const bool nhit = cnext.valid && cnext.cur == &cur && cnext.ref_slot == ref.slot && cnext.cur_slot == cur.slot &&
                          cnext.seed == seed;
        const bool launched = nhit && cnext.launched_next;
        if (nhit) R = cnext.R;
        cnext.valid = false;
        bool hit = false;
        long r_seq = nhit ? cnext.seq : 0;  // the speculation R came from
        const int e = nhit ? -1 : find_spec(&cur);
        if (e >= 0) {
            ChainSpec& E = cspec[e];
            if (E.cur_slot == cur.slot && E.seed == seed && (E.ref_slot < 0 || E.ref_slot == ref.slot)) {
                HostTimer hw(hprof, kHSpec);
                if (failed(hipEventSynchronize(E.ev) == hipSuccess ? VS_OK : VS_ERR_HIP)) return R;
                hit = spec_ref_slot(E) == ref.slot;
                if (hit) {
                    R = parse_chain(E.hbase + kHdrBytes);
                    r_seq = E.seq;
                }
            }
            E.valid = false;  // this frame's: used or not, it is done
        }
        if (!launched)  // speculations for later frames stay unless this frame's own chain was not launched ahead
            for (auto& E : cspec)
                if (E.valid && E.cur != next_frame && E.cur != next2_frame) E.valid = false;
        if (nhit) {
        } else if (hit) {
            cspec_hits++;
        } else {
            R = chain_impl(ref, cur, seed);
        }
        // The next frame's reference is this one's unless this frame becomes a keyframe, which the
        // rules of Slam.cpp:1061-1072 / is_keyframe (:1360) predict from the frame-id gap and this
        // chain's match count; a wrong guess only costs the speculation.
        // The launch itself (~40 us of HIP calls) is deferred until this frame's local-map tracking
        // and PnP are enqueued (flush_spec), so it overlaps them instead of delaying them.
        spec_req.pending = false;
        if (!launched && cspec_on && err == VS_OK && next_frame && next_frame != &cur && next_frame->slot >= 0 &&
            ref.slot >= 0) {
            const int ng = (int)R.good.size(), gap = cur.id - ref.id;
            const bool kf = (gap >= vs_trk::cfg::KF_MIN_FRAME_GAP && ng >= vs_trk::cfg::KF_MIN_MATCHES) ||
                            (ng < 2 * vs_trk::cfg::MIN_MATCHES && gap >= 5);
            const int rs = kf && cur.slot >= 0 ? cur.slot : ref.slot;
            const int e1 = find_spec(next_frame);
            if (e1 >= 0 && spec_matches(cspec[e1], rs, cur.slot, ref.slot, gap, seed + 1u, r_seq, next_frame->slot))
                return R;  // already in flight (a device pick on this very chain's count)
            if (e1 >= 0) cspec[e1].valid = false;
            spec_req.pending = true;
            spec_req.ref_slot = rs;
            spec_req.nxt = next_frame;
            spec_req.nxt_slot = next_frame->slot;
            spec_req.seed = seed + 1u;
            spec_req.ready = next_ready;
            if (spec_async) {  // launched now by the helper, beside this frame's tracking launches
                const SpecReq q = spec_req;
                spec_req.pending = false;
                if (q.nxt->slot == q.nxt_slot) {
                    spec_inflight = true;
                    sq.submit([this, q] { return launch_spec_chain(q.ref_slot, *q.nxt, q.seed, q.ready); });
                }
            }
        }
        return R;
    }
    // Launches the speculative chain chain() asked for, if its frames still sit in the same slots;
    // called once the frame's tracking kernels are enqueued, and at the end of every frame.
    void flush_spec() {
        if (!spec_req.pending) return;
        spec_req.pending = false;
        if (err != VS_OK || spec_req.nxt->slot != spec_req.nxt_slot) return;
        failed(launch_spec_chain(spec_req.ref_slot, *spec_req.nxt, spec_req.seed, spec_req.ready));
    }

    std::vector<vs_trk::Match> match(const vs_trk::Frame& a, const vs_trk::Frame& b, float ratio) {
        HostTimer ht(hprof, kHMatch);
        std::vector<vs_trk::Match> out;
        char* c = chain_buf.as<char>();
        int* di = reinterpret_cast<int*>(c + kChainInts);
        if (failed(enqueue_match(a.slot, b.slot, ratio, di))) return out;
        char* hc = take(kChainKept);
        if (!hc || failed(d2h(hc, c, kChainKept)))
            return out;
        if (failed(sync())) return out;
        const int ng = reinterpret_cast<const int*>(hc)[4];
        const auto* hg = reinterpret_cast<const vs_trk::Match*>(hc + kChainGood);
        out.assign(hg, hg + ng);
        return out;
    }

    // match() plus the DLT of every good match (triangulation input) in the same round trip
    std::vector<vs_trk::Match> match_dlt(const vs_trk::Frame& a, const vs_trk::Frame& b, float ratio, const double P1[12],
                                         const double P2[12], std::vector<std::array<float, 4>>& X4) {
        HostTimer ht(hprof, kHMatch);
        std::vector<vs_trk::Match> out;
        X4.clear();
        char* c = chain_buf.as<char>();
        int* di = reinterpret_cast<int*>(c + kChainInts);
        if (failed(enqueue_match(a.slot, b.slot, ratio, di))) return out;
        DltProj P;
        std::memcpy(P.P1, P1, sizeof(P.P1));
        std::memcpy(P.P2, P2, sizeof(P.P2));
        float4* dX = dlt_buf.as<float4>();
        hipLaunchKernelGGL(k_dlt, dim3((kCap + 63) / 64), dim3(64), 0, s, reinterpret_cast<const vs_match*>(c + kChainGood),
                           di + 4, kps_of(a.slot), kps_of(b.slot), P, dX);
        char* hc = take(kChainKept + (size_t)kCap * sizeof(float4));
        if (!hc || failed(d2h(hc, c, kChainKept)) || failed(d2h(hc + kChainKept, dX, (size_t)kCap * sizeof(float4))))
            return out;
        if (failed(sync())) return out;
        const int ng = reinterpret_cast<const int*>(hc)[4];
        const auto* hg = reinterpret_cast<const vs_trk::Match*>(hc + kChainGood);
        out.assign(hg, hg + ng);
        X4.resize(ng);
        std::memcpy(X4.data(), hc + kChainKept, (size_t)ng * sizeof(float4));
        return out;
    }

    bool find_fundamental(const std::vector<float>& p1, const std::vector<float>& p2, std::vector<uint8_t>& mask) {
        HostTimer ht(hprof, kHFmat);
        const int n = (int)(p1.size() / 2);
        mask.assign(std::max(n, 1), 0);
        double F[9];
        int ok = 0;
        if (failed(vs_find_fundamental(ctx, p1.data(), p2.data(), n, 3.0, 0.999, 1000, F, mask.data(), &ok, nullptr,
                                       nullptr)))
            return false;
        return ok != 0;
    }

    vs_trk::ChainResult motion_points(const vs_trk::Frame& ref, const vs_trk::Frame& cur, const std::vector<float>& p1,
                                      const std::vector<float>& p2, uint32_t seed) {
        HostTimer ht(hprof, kHMotion);
        vs_trk::ChainResult R;
        const int n = (int)(p1.size() / 2);
        if (!ref.depth || !cur.depth) {  // the RGB-D tracker path; monocular callers use vs_estimate_motion
            failed(VS_ERR_ARG);
            set_error("vs_slam: post-stationary motion needs both depth maps on the host");
            return R;
        }
        int ok = 0;
        if (failed(vs_ransac_3d3d(ctx, p1.data(), p2.data(), n, ref.depth, cur.depth, h, w, K, seed, 200, 0.05,
                                  R.R3.data(), R.t3.data(), &ok, nullptr)))
            return R;
        R.ok3d = ok != 0;
        if (!R.ok3d) {
            int eok = 0;
            if (failed(vs_estimate_motion(ctx, p1.data(), p2.data(), n, K, ref.depth, cur.depth, h, w, R.RE.data(),
                                          R.tE.data(), &R.scale, &eok, nullptr)))
                return R;
            R.okE = eok != 0;
        }
        return R;
    }

    // One local-map tracking launch into a work area (device) and a pinned block: one device block
    // read back with ONE copy, [tracking words | speculative PnP io + result], the refinement's PnP on
    // the tracked points right behind the tracking kernels (the tracker calls solve_pnp on exactly these
    // next, Slam.cpp:1057-1059; solve_pnp checks), its input gathered by k_tlm_resolve, the keypoint
    // grid built at extraction.  Observations can outnumber keypoints (a later map point may take a
    // keypoint over with a smaller distance, Slam.cpp:460-465, each takeover adding an observation):
    // obs_cap = 4 per keypoint first, the exact count on a rerun.
    struct TlmLaunch {
        int nkp = 0, obs_cap = 0, cap = 0;
        size_t wbytes = 0, io_pad = 0;
        bool spec_run = false;
        char* hall = nullptr;  // the pinned result block
    };
    int enqueue_tlm(const vs_trk::Map& m, const vs_trk::Frame& f, const double* R, const double* t, int obs_cap,
                    DevBuf& wk, char* h_kpmp, char* hall_area, size_t hall_cap, TlmLaunch& L) {
        const int nkp = (int)f.kps.size();
        L.nkp = nkp;
        L.obs_cap = obs_cap;
        const int words = 2 + nkp + 2 * obs_cap;
        L.wbytes = ((size_t)words * sizeof(int) + 255) & ~(size_t)255;
        L.cap = std::max(nkp, 1);
        const size_t io_bytes = 16 + (size_t)L.cap * 5 * sizeof(float);
        L.io_pad = (io_bytes + 15) & ~(size_t)15;
        const size_t spec_bytes = L.io_pad + 12 * sizeof(double) + 8 * sizeof(int);
        const bool spec_on = nkp > 0 && nkp <= 1024;
        VS_CHECK(wk.ensure(L.wbytes + (spec_on ? spec_bytes + (size_t)L.cap : 0)));
        int* d = wk.as<int>();
        int* d_kpmp = d + 2;
        int* d_obs = d + 2 + nkp;
        std::memcpy(h_kpmp, f.mp_idx.data(), (size_t)nkp * sizeof(int));  // read by k_tlm_resolve itself
        char* io = wk.as<char>() + L.wbytes;
        vs::TlmExtra ex;
        ex.grid = pre_grid && nkp <= 1024 ? grid_of(f.slot) : nullptr;
        if (spec_on) {
            ex.gather_io = reinterpret_cast<float*>(io);
            ex.gather_cap = L.cap;
        }
        VS_CHECK(vs::track_local_map(ctx, map_pos.as<double>(), map_desc.as<float>(), map_valid.as<uint8_t>(), m.size(),
                                     kps_of(f.slot), desc_of(f.slot), nkp, R, t, K, vs_trk::cfg::IMAGE_WIDTH,
                                     vs_trk::cfg::IMAGE_HEIGHT, d_kpmp, d_obs, d_obs + obs_cap, obs_cap, d, s,
                                     reinterpret_cast<const int*>(h_kpmp), &ex));
        L.spec_run = false;
        if (spec_on) {
            double* dRt = reinterpret_cast<double*>(io + L.io_pad);
            int* dstat = reinterpret_cast<int*>(dRt + 12);
            L.spec_run = vs::solve_pnp(ctx, 1, reinterpret_cast<const float*>(io + 16),
                                       reinterpret_cast<const float*>(io + 16 + (size_t)L.cap * 3 * sizeof(float)),
                                       reinterpret_cast<const int*>(io), K, 100, 10, dRt, dRt + 9, dstat,
                                       reinterpret_cast<uint8_t*>(dstat + 8), s, L.cap) == VS_OK;
        }
        const size_t rb = L.wbytes + (L.spec_run ? spec_bytes : 0);
        if (rb > hall_cap) return VS_ERR_CAPACITY;
        L.hall = hall_area;
        const Pinned& P = (hall_area >= spin.base && hall_area < spin.base + spin.cap) ? spin : pin;
        return P.to_host(L.hall, wk.p, rb, s);
    }
    // The launch's results (its copy has landed): kp -> map-point table, observations, the speculative
    // PnP; returns tracked, or -1 when the observations overflowed obs_cap (rerun with L.obs_cap set to
    // their count).
    int read_tlm(vs_trk::Frame& f, TlmLaunch& L, std::vector<std::pair<int, int>>& obs) {
        const int* hb = reinterpret_cast<const int*>(L.hall);
        const int nkp = L.nkp, cap = L.cap;
        spec_valid = false;
        if (L.spec_run) {
            const char* hs = L.hall + L.wbytes;
            const int n = reinterpret_cast<const int*>(hs)[1];
            const float* so = reinterpret_cast<const float*>(hs + 16);
            spec_obj.assign(so, so + (size_t)3 * n);
            spec_img.assign(so + (size_t)3 * cap, so + (size_t)3 * cap + (size_t)2 * n);
            const double* Rt = reinterpret_cast<const double*>(hs + L.io_pad);
            const int* st = reinterpret_cast<const int*>(Rt + 12);
            spec = vs_trk::PnPResult();
            spec.success = n > 0 && st[0] != 0;
            spec.inlier_count = spec.success ? st[1] : 0;
            if (spec.success) {
                std::memcpy(spec.R_world.data(), Rt, 9 * sizeof(double));
                std::memcpy(spec.t_world.data(), Rt + 9, 3 * sizeof(double));
            }
            spec_valid = true;
        }
        const int n_obs = hb[1];
        if (n_obs > L.obs_cap) {
            spec_valid = false;
            L.obs_cap = n_obs;
            return -1;
        }
        std::memcpy(f.mp_idx.data(), hb + 2, (size_t)nkp * sizeof(int));
        obs.clear();
        for (int i = 0; i < n_obs; i++) obs.emplace_back(hb[2 + nkp + i], hb[2 + nkp + L.obs_cap + i]);
        return hb[0];
    }

    // ---- round 6: speculative local-map tracking of the batch's next frame ----------------------
    // While frame i's tracking kernels run, the next frame's front chain (the speculative chain on s2)
    // is read back as soon as it lands, the next-but-one frame's chain is launched, and — when the
    // tracker's rules make frame i a non-keyframe and the next frame's path plain
    // (Tracker::predict_next_pose) — the next frame's local-map tracking + PnP is enqueued behind frame
    // i's at the predicted pose, into its own work area and pinned block.  Frame i + 1's
    // track_local_map uses it only when its frame, slot, keypoints, pose (bit for bit), map size and
    // map version equal the speculation's: the results are then the ones the call would compute.
    std::function<bool(const vs_trk::Frame&, const vs_trk::Frame&, const vs_trk::ChainResult&, const vs_trk::Frame**,
                       vs_trk::M3&, vs_trk::V3&, bool)>
        predict;                  // Tracker::predict_next_pose (set by vs_slam_create)
    bool tlm_spec_on = true;      // VS_SLAM_SPEC_TLM=0 disables
    int r3_split = kChainSplit3d;  // VS_SLAM_R3_SPLIT: k_ransac3d workgroups per chain (1 = one CU)
    bool next_kps_ready = false;  // the next frame's keypoints are on the host (its chunk was waited)
    // the batch being tracked and its next chunk to wait (process_batch_dev's loop): speculate_next waits
    // for the chunk of a next frame that starts one, instead of skipping the speculation
    std::vector<vs_trk::FramePtr>* bframes = nullptr;
    int* bchunk = nullptr;
    int next_index = -1;
    const vs_trk::Frame* next2_frame = nullptr;  // the frame after it, and its chunk's event
    hipEvent_t next2_ready = nullptr;
    const vs_trk::Frame* next3_frame = nullptr;  // and the one after that (VS_SLAM_SPEC_DEPTH=2)
    hipEvent_t next3_ready = nullptr;
    struct NextChain {  // the next frame's chain, read back ahead of its chain() call
        bool valid = false, launched_next = false;
        const vs_trk::Frame* cur = nullptr;
        int ref_slot = -1, cur_slot = -1;
        uint32_t seed = 0;
        long seq = 0;  // the speculation it came from
        vs_trk::ChainResult R;
    } cnext;
    struct TlmSpec {
        bool valid = false;
        const vs_trk::Frame* f = nullptr;
        int slot = -1, map_n = 0;
        long map_ver = 0;
        vs_trk::M3 R;
        vs_trk::V3 t;
        TlmLaunch L;
        hipEvent_t ev = nullptr;
    } tspec;
    DevBuf work2;
    Pinned spin{hipHostMallocCoherent | hipHostMallocMapped};  // the speculation's pinned block (never reset)
    hipEvent_t tlm_ev = nullptr;  // the direct launch's copy has landed
    long map_ver = 0;             // bumped by every map append and valid-flag change
    long tspec_launched = 0, tspec_hits = 0;

    // Reads the next frame's speculative chain back (waiting for it) into cnext.
    bool take_next_chain(const vs_trk::Frame* nxt) {
        spec_sync();
        const int e = find_spec(nxt);
        if (e < 0) return false;
        ChainSpec& E = cspec[e];
        HostTimer hw(hprof, kHSpecNext);
        if (failed(hipEventSynchronize(E.ev) == hipSuccess ? VS_OK : VS_ERR_HIP)) return false;
        cnext.R = parse_chain(E.hbase + kHdrBytes);
        cnext.valid = true;
        cnext.launched_next = false;
        cnext.cur = E.cur;
        cnext.ref_slot = spec_ref_slot(E);
        cnext.cur_slot = E.cur_slot;
        cnext.seed = E.seed;
        cnext.seq = E.seq;
        E.valid = false;
        cspec_hits++;
        return true;
    }
    void speculate_next(const vs_trk::Map& m, const vs_trk::Frame& f) {
        const vs_trk::Frame* nxt = next_frame;
        if (!tlm_spec_on || !predict || err != VS_OK || !nxt || nxt->slot < 0 || valid_dirty) return;
        if (!cnext.valid && !take_next_chain(nxt)) return;
        if (!(cnext.valid && cnext.cur == nxt)) return;
        const vs_trk::Frame* ref = nullptr;
        vs_trk::M3 R;
        vs_trk::V3 t;
        if (!next_kps_ready && bframes && bchunk) {  // the next frame opens a chunk: wait for it now (once
            const XBatch& X = xb[xcur];             // this frame is known to stay a non-keyframe, whose
            const int c = *bchunk;                   // remaining work then needs nothing on this stream)
            if (c + 1 < (int)X.ch.size() && next_index == X.ch[c] && predict(f, *nxt, cnext.R, &ref, R, t, true)) {
                if (failed(wait_chunk(*bframes, c))) return;
                ++*bchunk;
                next_kps_ready = true;
            }
        }
        if (!next_kps_ready || nxt->kps.empty() || nxt->kps.size() > 1024) return;
        if (!std::all_of(nxt->mp_idx.begin(), nxt->mp_idx.end(), [](int v) { return v < 0; })) return;
        if (!predict(f, *nxt, cnext.R, &ref, R, t, false) || !ref || ref->slot != cnext.ref_slot ||
            nxt->slot != cnext.cur_slot)
            return;
        // the frame after it: its chain against the reference chain() would predict (the rule of
        // chain(): the next frame becomes a keyframe by the id gap and its match count)
        if (!cnext.launched_next && cspec_on && next2_frame && next2_frame->slot >= 0) {
            const int ng = (int)cnext.R.good.size(), gap = nxt->id - ref->id;
            const bool kf = (gap >= vs_trk::cfg::KF_MIN_FRAME_GAP && ng >= vs_trk::cfg::KF_MIN_MATCHES) ||
                            (ng < 2 * vs_trk::cfg::MIN_MATCHES && gap >= 5);
            const int rs = kf ? nxt->slot : ref->slot;
            const vs_trk::Frame* n2 = next2_frame;
            const uint32_t sd = cnext.seed + 1u;
            hipEvent_t rdy = next2_ready;
            // launched one frame earlier with its reference picked on the device from the next frame's count?
            const int e2 = find_spec(n2);
            const bool have = e2 >= 0 && spec_matches(cspec[e2], rs, nxt->slot, ref->slot, gap, sd, cnext.seq, n2->slot);
            if (e2 >= 0 && !have) cspec[e2].valid = false;
            // depth 2: the chain after it too, its reference picked on the device from n2's count
            const vs_trk::Frame* n3 = spec_depth >= 2 ? next3_frame : nullptr;
            const bool go3 = n3 && n3->slot >= 0 && find_spec(n3) < 0;
            const int kf3 = n2->slot, base3 = rs, gap3 = n2->id - (kf ? nxt->id : ref->id);
            hipEvent_t rdy3 = next3_ready;
            auto job = [this, have, rs, n2, sd, rdy, go3, n3, kf3, base3, gap3, rdy3]() -> int {
                if (!have) VS_CHECK(launch_spec_chain(rs, *n2, sd, rdy));
                const int p = go3 ? find_spec(n2) : -1;
                if (p >= 0) VS_CHECK(launch_spec_chain(-1, *n3, sd + 1u, rdy3, p, kf3, base3, gap3));
                return VS_OK;
            };
            if (spec_async) {  // ~40 us of HIP calls per chain, on the helper beside this thread's tracking launch
                spec_inflight = true;
                sq.submit(job);
            } else if (failed(job())) {
                return;
            }
            cnext.launched_next = true;
        }
        const int nkp = (int)nxt->kps.size();
        TlmSpec& T = tspec;
        T.valid = false;
        char* hk = spin.base;
        char* ha = spin.base + 8192;
        if (failed(enqueue_tlm(m, *nxt, R.data(), t.data(), std::max(4 * nkp, 64), work2, hk, ha, spin.cap - 8192, T.L)))
            return;
        if (failed(hipEventRecord(T.ev, s) == hipSuccess ? VS_OK : VS_ERR_HIP)) return;
        T.valid = true;
        T.f = nxt;
        T.slot = nxt->slot;
        T.map_n = m.size();
        T.map_ver = map_ver;
        T.R = R;
        T.t = t;
        tspec_launched++;
    }

    int track_local_map(vs_trk::Map& m, vs_trk::Frame& f, std::vector<std::pair<int, int>>& obs) {
        HostTimer ht(hprof, kHTlm);
        obs.clear();
        const int nkp = (int)f.kps.size();
        if (failed(sync_valid(m))) return 0;
        TlmSpec& T = tspec;
        const bool hit = T.valid && T.f == &f && T.slot == f.slot && T.L.nkp == nkp && T.map_n == m.size() &&
                         T.map_ver == map_ver && std::memcmp(T.R.data(), f.R.data(), sizeof(T.R)) == 0 &&
                         std::memcmp(T.t.data(), f.t.data(), sizeof(T.t)) == 0 &&
                         std::all_of(f.mp_idx.begin(), f.mp_idx.end(), [](int v) { return v < 0; });
        T.valid = false;
        if (hit) {
            tspec_hits++;
            TlmLaunch L = T.L;
            hipEvent_t ev = T.ev;
            // the speculation's copy block stays untouched until the next speculation is enqueued,
            // which waits for nothing of ours: read it first
            {
                HostTimer hs(hprof, kHTlmSync);
                if (failed(hipEventSynchronize(ev) == hipSuccess ? VS_OK : VS_ERR_HIP)) return 0;
            }
            std::vector<std::pair<int, int>> o2;
            std::vector<int> kpmp_save = f.mp_idx;
            const int tracked = read_tlm(f, L, o2);
            const bool spec_ok = spec_valid;
            const vs_trk::PnPResult sp = spec;
            const std::vector<float> so = spec_obj, si = spec_img;
            if (tracked >= 0) {
                obs.swap(o2);
                flush_spec();
                speculate_next(m, f);  // the frame after this one, behind nothing of ours
                spec_valid = spec_ok;  // (speculate_next does not touch the PnP speculation, but be explicit)
                spec = sp;
                spec_obj = so;
                spec_img = si;
                return tracked;
            }
            f.mp_idx = kpmp_save;  // overflowed: the direct path below with the exact capacity
        }
        int obs_cap = std::max(4 * nkp, 64);
        for (int attempt = 0; attempt < 2; attempt++) {
            char* hk = take((size_t)std::max(nkp, 1) * sizeof(int));
            const int words = 2 + nkp + 2 * obs_cap;
            const int cap = std::max(nkp, 1);
            const size_t rb = (((size_t)words * sizeof(int) + 255) & ~(size_t)255) + ((16 + (size_t)cap * 20 + 15) & ~(size_t)15) +
                              12 * sizeof(double) + 8 * sizeof(int);
            char* ha = hk ? take(rb) : nullptr;
            if (!hk || !ha) return 0;
            TlmLaunch L;
            if (failed(enqueue_tlm(m, f, f.R.data(), f.t.data(), obs_cap, work, hk, ha, rb, L))) return 0;
            if (failed(hipEventRecord(tlm_ev, s) == hipSuccess ? VS_OK : VS_ERR_HIP)) return 0;
            flush_spec();  // the next frame's chain, launched while these kernels run
            if (attempt == 0) speculate_next(m, f);
            {
                HostTimer hs(hprof, kHTlmSync);
                if (failed(hipEventSynchronize(tlm_ev) == hipSuccess ? VS_OK : VS_ERR_HIP)) return 0;
            }
            pin.used = 0;  // every pinned transfer of ours is before tlm_ev (the speculation uses spin)
            const int tracked = read_tlm(f, L, obs);
            if (tracked >= 0) return tracked;
            obs_cap = L.obs_cap;  // rerun from the same inputs with room for every observation
        }
        failed(VS_ERR_CAPACITY);
        return 0;
    }

    // Slam::solve_pnp on the device: one packed pinned upload (offsets, object and image points),
    // the PnP kernels, one packed download of (R, t, status).
    vs_trk::PnPResult solve_pnp(const std::vector<float>& obj, const std::vector<float>& img, int iters, int min_inliers) {
        HostTimer ht(hprof, kHPnp);
        if (spec_valid) {  // the speculative run had exactly these inputs: its result is this call's
            spec_valid = false;
            const auto same = [](const std::vector<float>& a, const std::vector<float>& b) {  // bit-exact
                return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(float)) == 0;
            };
            if (iters == 100 && min_inliers == 10 && same(obj, spec_obj) && same(img, spec_img)) return spec;
        }
        vs_trk::PnPResult r;
        const int n = (int)(obj.size() / 3);
        if (n == 0) return r;
        if (iters > VS_PNP_MAX_ITERS) {
            failed(VS_ERR_ARG);
            return r;
        }
        const size_t in_bytes = 16 + (size_t)n * 5 * sizeof(float);
        const size_t in_pad = (in_bytes + 15) & ~(size_t)15;
        const size_t out_bytes = 12 * sizeof(double) + 8 * sizeof(int);
        if (failed(pnp_io.ensure(in_pad + out_bytes + (size_t)n))) return r;
        char* d = pnp_io.as<char>();
        char* hb = take(in_bytes);
        if (!hb) return r;
        const int off[4] = {0, n, 0, 0};
        std::memcpy(hb, off, 16);
        std::memcpy(hb + 16, obj.data(), (size_t)n * 3 * sizeof(float));
        std::memcpy(hb + 16 + (size_t)n * 3 * sizeof(float), img.data(), (size_t)n * 2 * sizeof(float));
        if (failed(pin.to_device(d, hb, in_bytes, s)))
            return r;
        double* dRt = reinterpret_cast<double*>(d + in_pad);
        int* dstat = reinterpret_cast<int*>(dRt + 12);
        if (failed(vs::solve_pnp(ctx, 1, reinterpret_cast<const float*>(d + 16),
                                 reinterpret_cast<const float*>(d + 16 + (size_t)n * 3 * sizeof(float)),
                                 reinterpret_cast<const int*>(d), K, iters, min_inliers, dRt, dRt + 9, dstat,
                                 reinterpret_cast<uint8_t*>(dstat + 8), s, n)))
            return r;
        char* ho = take(out_bytes);
        if (!ho || failed(d2h(ho, dRt, out_bytes)) || failed(sync())) return r;
        const int* st = reinterpret_cast<const int*>(ho + 12 * sizeof(double));
        r.success = st[0] != 0;
        r.inlier_count = st[0] ? st[1] : 0;  // PnPResult.inlier_count stays 0 on failure (Slam.cpp:510)
        if (r.success) {
            std::memcpy(r.R_world.data(), ho, 9 * sizeof(double));
            std::memcpy(r.t_world.data(), ho + 9 * sizeof(double), 3 * sizeof(double));
        }
        return r;
    }

    int grow_archive(int need) {
        if (need <= arch_cap) return VS_OK;
        VS_CHECK(flush_copies());  // pending archive copies target the old buffers
        const int cap = std::max(need, std::max(16, 2 * arch_cap));
        DevBuf nk, nd, nn;
        VS_CHECK(nk.ensure((size_t)cap * kCap * sizeof(vs_keypoint)));
        VS_CHECK(nd.ensure((size_t)cap * kCap * 256 * sizeof(float)));
        VS_CHECK(nn.ensure((size_t)cap * sizeof(int)));
        if (arch_used > 0) {
            VS_HIP(hipMemcpyAsync(nk.p, arch_kps.p, (size_t)arch_used * kCap * sizeof(vs_keypoint), hipMemcpyDeviceToDevice, s));
            VS_HIP(hipMemcpyAsync(nd.p, arch_desc.p, (size_t)arch_used * kCap * 256 * sizeof(float), hipMemcpyDeviceToDevice, s));
            VS_HIP(hipMemcpyAsync(nn.p, arch_n.p, (size_t)arch_used * sizeof(int), hipMemcpyDeviceToDevice, s));
        }
        VS_HIP(hipStreamSynchronize(s));
        arch_kps.release();
        arch_desc.release();
        arch_n.release();
        arch_kps = nk;
        arch_desc = nd;
        arch_n = nn;
        nk.p = nd.p = nn.p = nullptr;  // ownership moved
        arch_cap = cap;
        return VS_OK;
    }
    // loop_eval's candidate pool for P candidates: [P + 1] frames (keypoints, descriptors, counts),
    // pairs, raw / good lists, counts, E-RANSAC outputs
    struct LcLayout {
        size_t kb, db, nb, pb, mb, cb, rb, gb, sb, total;
        explicit LcLayout(int P) {
            auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
            const size_t F = (size_t)P + 1;
            kb = al(F * kCap * sizeof(vs_keypoint));
            db = al(F * kCap * 256 * sizeof(float));
            nb = al(F * sizeof(int));
            pb = al((size_t)2 * P * sizeof(int));
            mb = al((size_t)P * kCap * sizeof(vs_match));
            cb = al((size_t)P * sizeof(int));
            rb = al((size_t)P * 16 * sizeof(double));
            gb = al((size_t)P * 8 * sizeof(int));
            sb = al(F * sizeof(FrameSrc));
            total = kb + db + nb + pb + 2 * mb + 3 * cb + rb + gb + sb;
        }
    };
    // A keyframe's features into the archive (at settle, while its pool slot is still intact; queued,
    // flushed by the caller)
    int archive(vs_trk::Frame* f) {
        if (f->kf_slot >= 0 || f->slot < 0) return VS_OK;
        VS_CHECK(grow_archive(arch_used + 1));
        const int a = arch_used++;
        cjobs.push_back({kps_of(f->slot), arch_kps.as<vs_keypoint>() + (size_t)a * kCap, kCap * sizeof(vs_keypoint)});
        cjobs.push_back({desc_of(f->slot), arch_desc.as<float>() + (size_t)a * kCap * 256, (size_t)kCap * 256 * sizeof(float)});
        cjobs.push_back({pool_n.as<int>() + f->slot, arch_n.as<int>() + a, sizeof(int)});
        f->kf_slot = a;
        return VS_OK;
    }

    // LoopCloser::detect's candidate evaluation (LoopCloser.cpp:50-76) for all candidates at once:
    // the current frame and the candidates gathered into one pool (keyframes from the archive, or
    // from their pool slot within the batch that made them), one match_pairs launch over the P
    // (current, keyframe) pairs, one E-RANSAC launch over their good lists, one read-back.
    std::vector<vs_trk::LoopEval> loop_eval(const vs_trk::Frame& cur, const std::vector<const vs_trk::Frame*>& kfs) {
        HostTimer ht(hprof, kHLoop);
        const int P = (int)kfs.size(), F = P + 1;
        std::vector<vs_trk::LoopEval> out(P);
        if (P == 0 || cur.slot < 0) return out;
        const LcLayout Lb(P);
        const size_t kb = Lb.kb, db = Lb.db, nb = Lb.nb, pb = Lb.pb, mb = Lb.mb, cb = Lb.cb, rb = Lb.rb;
        if (failed(lc_buf.ensure(Lb.total)) || failed(match_reserve(ctx, P, kCap, s))) return out;
        char* base = lc_buf.as<char>();
        auto* d_kps = reinterpret_cast<vs_keypoint*>(base);
        auto* d_desc = reinterpret_cast<float*>(base + kb);
        auto* d_n = reinterpret_cast<int*>(base + kb + db);
        auto* d_pairs = reinterpret_cast<int*>(base + kb + db + nb);
        auto* d_raw = reinterpret_cast<vs_match*>(base + kb + db + nb + pb);
        auto* d_good = reinterpret_cast<vs_match*>(base + kb + db + nb + pb + mb);
        char* tail = base + kb + db + nb + pb + 2 * mb;
        auto* d_nraw = reinterpret_cast<int*>(tail);
        auto* d_ngood = reinterpret_cast<int*>(tail + cb);
        auto* d_ok = reinterpret_cast<int*>(tail + 2 * cb);
        auto* d_Rt = reinterpret_cast<double*>(tail + 3 * cb);  // R [P][9] | t [P][3] | scale [P]
        auto* d_diag = reinterpret_cast<int*>(tail + 3 * cb + rb);
        // the pool: one gather launch from a table of source rows (archive or pool slot)
        std::vector<FrameSrc> src(F);
        src[0] = {kps_of(cur.slot), desc_of(cur.slot), pool_n.as<int>() + cur.slot};
        std::vector<int> pairs(2 * P);
        for (int i = 0; i < P; i++) {
            const vs_trk::Frame* k = kfs[i];
            if (k->kf_slot >= 0)
                src[i + 1] = {arch_kps.as<vs_keypoint>() + (size_t)k->kf_slot * kCap,
                              arch_desc.as<float>() + (size_t)k->kf_slot * kCap * 256, arch_n.as<int>() + k->kf_slot};
            else if (k->slot >= 0)
                src[i + 1] = {kps_of(k->slot), desc_of(k->slot), pool_n.as<int>() + k->slot};
            else {
                set_error("vs_slam: a loop-closure keyframe has no device features");
                failed(VS_ERR_CAPACITY);
                return out;
            }
            pairs[2 * i] = 0;
            pairs[2 * i + 1] = i + 1;
        }
        auto* d_src = reinterpret_cast<FrameSrc*>(tail + 3 * cb + rb + Lb.gb);
        if (failed(upload(d_src, src.data(), src.size() * sizeof(FrameSrc)))) return out;
        hipLaunchKernelGGL(k_gather_frames, dim3(F, 8), dim3(256), 0, s, d_src, d_kps, d_desc, d_n);
        if (failed(upload(d_pairs, pairs.data(), pairs.size() * sizeof(int)))) return out;
        if (failed(match_pairs(ctx, P, d_pairs, F, d_desc, d_n, kCap, vs_trk::cfg::L2_RATIO_THRESHOLD, d_raw, d_nraw,
                               d_good, d_ngood, s)))
            return out;
        if (failed(emat_pairs(ctx, P, d_pairs, d_kps, kCap, d_good, d_ngood, nullptr, nullptr, h, w, K, d_Rt,
                              d_Rt + 9 * P, d_Rt + 12 * P, d_ok, d_diag, s)))
            return out;
        char* hb = take((size_t)P * 9 * sizeof(int));
        if (!hb) return out;
        if (failed(d2h(hb, d_ngood, (size_t)P * sizeof(int))) ||
            failed(d2h(hb + (size_t)P * sizeof(int), d_diag, (size_t)P * 8 * sizeof(int))) || failed(sync()))
            return out;
        const int* ng = reinterpret_cast<const int*>(hb);
        const int* dg = ng + P;
        for (int i = 0; i < P; i++) {
            out[i].n_good = ng[i];
            out[i].inliers = dg[8 * i + 3];
        }
        return out;
    }

    // Optimizer::pose_graph_optimize's solve (Optimizer.cpp:677-778) on the GPU (csrc/pgo.hip)
    void pose_graph(std::vector<vs_trk::M3>& R, std::vector<vs_trk::V3>& t, const std::vector<vs_trk::PgoLoop>& loops,
                    const vs_trk::V3* gravity, double height, int iters) {
        const int N = (int)R.size(), L = (int)loops.size();
        std::vector<double> Rf((size_t)N * 9), tf((size_t)N * 3), lR((size_t)L * 9 + 1), lt((size_t)L * 3 + 1),
            ls((size_t)L * 2 + 1);
        std::vector<int> lf(L + 1), lto(L + 1);
        for (int i = 0; i < N; i++) {
            std::memcpy(&Rf[9 * i], R[i].data(), 72);
            std::memcpy(&tf[3 * i], t[i].data(), 24);
        }
        for (int l = 0; l < L; l++) {
            lf[l] = loops[l].from;
            lto[l] = loops[l].to;
            std::memcpy(&lR[9 * l], loops[l].R.data(), 72);
            std::memcpy(&lt[3 * l], loops[l].t.data(), 24);
            ls[2 * l] = loops[l].trans_sigma;
            ls[2 * l + 1] = loops[l].rot_sigma;
        }
        if (failed(vs_pose_graph_optimize(ctx, N, Rf.data(), tf.data(), L, lf.data(), lto.data(), lR.data(), lt.data(),
                                          ls.data(), gravity ? gravity->data() : nullptr, height, iters, nullptr,
                                          nullptr)))
            return;
        for (int i = 0; i < N; i++) {
            std::memcpy(R[i].data(), &Rf[9 * i], 72);
            std::memcpy(t[i].data(), &tf[3 * i], 24);
        }
    }
    void pgo_points(const std::vector<vs_trk::M3>& Ro, const std::vector<vs_trk::V3>& to, const std::vector<vs_trk::M3>& Rn,
                    const std::vector<vs_trk::V3>& tn, const std::vector<int>& kf, vs_trk::Map& m) {
        const int N = (int)Ro.size(), M = m.size();
        if (M == 0) return;
        std::vector<double> a((size_t)N * 9), b((size_t)N * 3), c((size_t)N * 9), d((size_t)N * 3);
        for (int i = 0; i < N; i++) {
            std::memcpy(&a[9 * i], Ro[i].data(), 72);
            std::memcpy(&b[3 * i], to[i].data(), 24);
            std::memcpy(&c[9 * i], Rn[i].data(), 72);
            std::memcpy(&d[3 * i], tn[i].data(), 24);
        }
        if (failed(vs_pgo_transform_points(ctx, N, a.data(), b.data(), c.data(), d.data(), M, kf.data(), m.pos.data())))
            return;
        // the device copy of the map follows (tracking after a PGO sees the corrected points)
        if (failed(upload(map_pos.as<double>(), m.pos.data(), (size_t)M * 3 * sizeof(double)))) return;
        failed(sync());
    }

    std::vector<std::pair<int, int>> match_map(const vs_trk::Map& m, const vs_trk::Frame& f, const std::vector<int>& ids,
                                               float ratio) {
        HostTimer ht(hprof, kHMatchMap);
        std::vector<std::pair<int, int>> out;
        const int n1 = (int)f.kps.size(), n2 = (int)ids.size();
        if (n1 == 0 || n2 < 2) return out;
        const size_t tbytes = (size_t)n2 * 256 * sizeof(float), ibytes = (size_t)n2 * sizeof(int);
        const size_t obytes = (size_t)2 * n1 * sizeof(vs_match) + 2 * sizeof(int);
        if (failed(map_tmp.ensure(tbytes + ibytes + obytes))) return out;
        float* d_t = map_tmp.as<float>();
        int* d_ids = reinterpret_cast<int*>(map_tmp.as<char>() + tbytes);
        vs_match* d_raw = reinterpret_cast<vs_match*>(map_tmp.as<char>() + tbytes + ibytes);
        vs_match* d_good = d_raw + n1;
        int* d_cnt = reinterpret_cast<int*>(d_good + n1);
        if (failed(upload(d_ids, ids.data(), ibytes))) return out;
        hipLaunchKernelGGL(k_gather_rows, dim3((n2 + 3) / 4), dim3(256), 0, s, map_desc.as<float>(), d_ids, n2, d_t);
        if (failed(match_sets(ctx, desc_of(f.slot), n1, d_t, n2, ratio, d_raw, d_good, d_cnt, s))) return out;
        char* hb = take((size_t)n1 * sizeof(vs_match) + 2 * sizeof(int));
        if (!hb) return out;
        if (failed(d2h(hb, d_cnt, 2 * sizeof(int))))
            return out;
        if (failed(d2h(hb + 2 * sizeof(int), d_good, (size_t)n1 * sizeof(vs_match))))
            return out;
        if (failed(sync())) return out;
        const int ng = reinterpret_cast<const int*>(hb)[1];
        const auto* g = reinterpret_cast<const vs_match*>(hb + 2 * sizeof(int));
        for (int i = 0; i < ng; i++) out.emplace_back(g[i].query_idx, g[i].train_idx);
        return out;
    }

    void map_append(const vs_trk::Map& m, int first, const vs_trk::Frame& src, const std::vector<int>& rows) {
        HostTimer ht(hprof, kHAppend);
        const int k = (int)rows.size();
        map_ver++;
        if (failed(grow_map(first + k))) return;
        if (k == 0) {
            map_n = first;
            return;
        }
        // one staging upload (positions, then the source rows) and one kernel (positions, descriptor
        // rows, valid flags)
        const size_t pbytes = (size_t)3 * k * sizeof(double), rbytes = (size_t)k * sizeof(int);
        if (failed(rows_buf.ensure(pbytes + rbytes))) return;
        char* hb = take(pbytes + rbytes);
        if (!hb) return;
        std::memcpy(hb, m.pos.data() + (size_t)3 * first, pbytes);
        std::memcpy(hb + pbytes, rows.data(), rbytes);
        if (failed(pin.to_device(rows_buf.p, hb, pbytes + rbytes, s))) return;
        const double* d_pos = rows_buf.as<double>();
        const int* d_rows = reinterpret_cast<const int*>(rows_buf.as<char>() + pbytes);
        hipLaunchKernelGGL(k_map_append, dim3((k + 3) / 4), dim3(256), 0, s, d_pos, d_rows, k, desc_of(src.slot),
                           map_pos.as<double>() + (size_t)3 * first, map_desc.as<float>() + (size_t)first * 256,
                           map_valid.as<uint8_t>() + first);
        map_n = first + k;
        // no synchronisation: the next append's upload into rows_buf is ordered behind this gather on
        // the same stream, and the pinned staging it came from is recycled only at a sync()
    }

    void map_valid_changed() {
        valid_dirty = true;
        map_ver++;
    }

    void visibility(const vs_trk::Map& m, const vs_trk::Frame& f, const vs_trk::M3& R, const vs_trk::V3& t,
                    std::vector<uint8_t>& flags) {
        HostTimer ht(hprof, kHVis);
        const int n = m.size();
        flags.assign(n, 0);
        if (n == 0) return;
        if (failed(sync_valid(m)) || failed(map_tmp.ensure((size_t)n))) return;
        const int ncell = ((vs_trk::cfg::IMAGE_WIDTH + kVisCell - 1) / kVisCell) *
                          ((vs_trk::cfg::IMAGE_HEIGHT + kVisCell - 1) / kVisCell);
        if (ncell > kVisMaxCells || (int)f.kps.size() > kCap) {
            vs::set_error("vs_slam: visibility: keypoint count or grid size out of range");
            failed(VS_ERR_ARG);
            return;
        }
        uint8_t* d_flags = map_tmp.as<uint8_t>();
        hipLaunchKernelGGL(k_visibility, dim3((n + 255) / 256), dim3(256), 0, s, map_pos.as<double>(),
                           map_valid.as<uint8_t>(), n, kps_of(f.slot), (int)f.kps.size(), R[0], R[1], R[2], R[3], R[4],
                           R[5], R[6], R[7], R[8], t[0], t[1], t[2], K[0], K[1], K[2], K[3], vs_trk::cfg::IMAGE_WIDTH,
                           vs_trk::cfg::IMAGE_HEIGHT, d_flags);
        char* hb = take((size_t)n);
        if (!hb) return;
        if (failed(d2h(hb, d_flags, (size_t)n)))
            return;
        if (failed(sync())) return;
        std::memcpy(flags.data(), hb, (size_t)n);
    }
};

}  // namespace vs

struct vs_slam {
    vs::GpuOps ops;
    std::unique_ptr<vs_trk::Tracker<vs::GpuOps>> trk;
    std::vector<vs_trk::FramePtr> batch;  // frames of the batch being processed
    FILE* trace = nullptr;                // VS_TRACE_GPU=path: stage trace (debugging aid)
    // dense fusion (main.cpp:1116-1139): processed frames with depth, pose right after process_frame
    vs_dense* dense = nullptr;
    std::vector<const float*> dense_depth;
    std::vector<double> dense_R, dense_t;
};

using namespace vs;

namespace {

// The context's stream is the tracking stream for the duration of a vs_slam call, so the vs_*
// entry points the back end calls enqueue behind the tracker's own kernels.
struct CtxStream {
    vs_ctx* c;
    hipStream_t old;
    CtxStream(vs_ctx* cc, hipStream_t st) : c(cc), old(cc->stream) { c->stream = st; }
    ~CtxStream() { c->stream = old; }
};

// main.cpp:1116-1118: a processed frame with real depth joins the dense cloud with its pose now
void dense_record(vs_slam* sl, const vs_trk::Frame& f) {
    if (!sl->dense || !f.depth || f.slot < 0) return;
    sl->dense_depth.push_back(sl->ops.depth_of(f.slot));
    sl->dense_R.insert(sl->dense_R.end(), f.R.begin(), f.R.end());
    sl->dense_t.insert(sl->dense_t.end(), f.t.begin(), f.t.end());
}

// After a batch (or a single frame): the recorded frames are fused into the dense cloud (before
// any slot moves), live frames still sitting in a batch-region slot move to persistent slots; dead
// frames drop their device slot and host working data (the map keeps only their pose for the
// trajectory).
int settle(vs_slam* sl) {
    GpuOps& o = sl->ops;
    auto& T = *sl->trk;
    o.spec_sync();
    if (o.err != VS_OK) {
        const int r = o.err;
        o.err = VS_OK;
        return r;
    }
    for (auto& E : o.cspec) VS_HIP(hipStreamWaitEvent(o.s, E.ev, 0));  // a discarded speculation still reads the pool
    for (const auto& f : T.map().frames)  // new keyframes' features into the archive (loop closure)
        if (f->keyframe && f->kf_slot < 0 && f->slot >= 0) VS_CHECK(o.archive(f.get()));
    VS_CHECK(o.flush_copies());  // before any slot below is released and reused
    if (sl->dense && !sl->dense_depth.empty()) {
        VS_CHECK(vs_dense_integrate_dev(sl->dense, (int)sl->dense_depth.size(), sl->dense_depth.data(), o.h, o.w,
                                        sl->dense_R.data(), sl->dense_t.data(), o.s));
        sl->dense_depth.clear();
        sl->dense_R.clear();
        sl->dense_t.clear();
    }
    for (int i = 0; i < kPersist; i++) {
        vs_trk::Frame* f = o.owner[i];
        if (f && !T.is_live(f)) {
            o.release_slot(f);
            if (!f->keyframe) {  // keyframes keep their host keypoints (LoopCloser.cpp:48 checks them)
                f->kps.clear();
                f->kps.shrink_to_fit();
            }
            f->mp_idx.clear();
            f->mp_idx.shrink_to_fit();
            f->depth_store = std::vector<float>();
            f->depth = nullptr;
        }
    }
    for (auto& f : sl->batch) {
        if (T.is_live(f.get())) {
            if (f->slot >= 0 && f->slot < 2 * o.B) {
                const int to = o.persistent_slot(f.get());
                if (to < 0) {
                    // the moves queued so far are complete (their frames already point at the new slots):
                    // run them before reporting, so that no later flush copies a reused batch slot
                    // 
                    const int rc = o.flush_copies();
                    return rc != VS_OK ? rc : VS_ERR_CAPACITY;
                }
                VS_CHECK(o.copy_slot(f->slot, to));
                f->slot = to;
            }
        } else if (f->slot >= 0 && f->slot < 2 * o.B) {
            f->slot = -1;
            if (!f->keyframe) {
                f->kps.clear();
                f->kps.shrink_to_fit();
            }
            f->mp_idx.clear();
            f->mp_idx.shrink_to_fit();
            f->depth = nullptr;
        }
    }
    VS_CHECK(o.flush_copies());  // the slot moves
    T.retain_live_frames();  // live frames keep a host copy of their depth beyond the caller's buffer
    sl->batch.clear();
    return o.sync();
}

}  // namespace

extern "C" {

int vs_slam_create(vs_ctx* ctx, int max_batch, int h, int w, vs_slam** out) {
    VS_ARG(ctx && out, "vs_slam_create: null argument");
    VS_ARG(max_batch >= 1 && max_batch <= 256, "vs_slam_create: max_batch must be in [1, 256]");
    VS_ARG(h == vs_trk::cfg::IMAGE_HEIGHT && w == vs_trk::cfg::IMAGE_WIDTH,
           "vs_slam_create: the reference tracker is fixed to 640x480 (Config.h:10-11)");
    *out = nullptr;
    VS_HIP(hipSetDevice(ctx->device));
    vs_slam* sl = new (std::nothrow) vs_slam();
    if (!sl) return VS_ERR_NOMEM;
    int rc = sl->ops.init(ctx, max_batch, h, w);
    if (rc != VS_OK) {
        delete sl;
        return rc;
    }
    sl->trk = std::make_unique<vs_trk::Tracker<GpuOps>>(sl->ops);
    vs_trk::Tracker<GpuOps>* trk = sl->trk.get();
    sl->ops.predict = [trk](const vs_trk::Frame& cur, const vs_trk::Frame& nxt, const vs_trk::ChainResult& C,
                            const vs_trk::Frame** ref, vs_trk::M3& R, vs_trk::V3& t, bool cur_only) {
        return trk->predict_next_pose(cur, nxt, C, ref, R, t, cur_only);
    };
    if (const char* p = std::getenv("VS_TRACE_GPU")) sl->trace = std::fopen(p, "w");
    sl->trk->set_trace(sl->trace);
    *out = sl;
    return VS_OK;
}

void vs_slam_destroy(vs_slam* sl) {
    if (!sl) return;
    GpuOps& o = sl->ops;
    if (o.hprof.on)
        for (int k = 0; k < kHOps; k++)
            if (o.hprof.n[k])
                std::fprintf(stderr, "vs_slam host %-22s %8ld calls %10.3f ms  %8.1f us/call\n", kHostOpNames[k],
                             o.hprof.n[k], o.hprof.ms[k], 1e3 * o.hprof.ms[k] / o.hprof.n[k]);
    if (o.hprof.on) {
        std::fprintf(stderr, "vs_slam speculative chains: %ld launched, %ld used\n", o.cspec_launched, o.cspec_hits);
        std::fprintf(stderr, "vs_slam speculative next-frame local-map tracking: %ld launched, %ld used\n",
                     o.tspec_launched, o.tspec_hits);
        const vs_trk::PhaseProf& ph = sl->trk->phase_prof();
        for (int k = 0; k < vs_trk::PH_N; k++)
            if (ph.n[k])
                std::fprintf(stderr, "vs_slam phase %-27s %8ld calls %10.3f ms  %8.1f us/call\n", vs_trk::phase_name(k),
                             ph.n[k], ph.ms[k], 1e3 * ph.ms[k] / ph.n[k]);
    }
    o.destroy_streams();
    DevBuf* bufs[] = {&o.pool_kps, &o.pool_desc, &o.pool_n, &o.pool_depth, &o.pool_norms, &o.pool_grid, &o.semi, &o.dgrid,
                      &o.chain_buf,    &o.work, &o.rows_buf,      &o.map_pos, &o.map_desc,  &o.map_valid, &o.map_tmp,
                      &o.pnp_io,       &o.hdr_buf, &o.cspec[0].buf, &o.cspec[0].hdr, &o.cspec[1].buf, &o.cspec[1].hdr, &o.mstate2,
                      &o.arch_kps,     &o.arch_desc, &o.arch_n,   &o.lc_buf,    &o.dlt_buf, &o.cjob_buf};
    for (DevBuf* b : bufs) b->release();
    if (sl->trace) std::fclose(sl->trace);
    delete sl;
}

int vs_slam_set_initial_pose(vs_slam* sl, const double R[9], const double t[3]) {
    VS_ARG(sl && R && t, "vs_slam_set_initial_pose: null argument");
    vs_trk::M3 Rm;
    vs_trk::V3 tv;
    std::memcpy(Rm.data(), R, sizeof(Rm));
    std::memcpy(tv.data(), t, sizeof(tv));
    sl->trk->set_initial_pose(Rm, tv);
    return VS_OK;
}

int vs_slam_set_accelerometer(vs_slam* sl, const double* samples, int n) {
    VS_ARG(sl && n >= 0 && (n == 0 || samples), "vs_slam_set_accelerometer: bad arguments");
    std::vector<vs_trk::AccelSample> a(n);
    for (int i = 0; i < n; i++) a[i] = {samples[4 * i], samples[4 * i + 1], samples[4 * i + 2], samples[4 * i + 3]};
    sl->trk->set_accelerometer_data(std::move(a));
    sl->trk->compute_gravity_direction();
    return VS_OK;
}

int vs_slam_prefetch_batch_dev(vs_slam* sl, int B, const uint8_t* d_bgr, const float* d_depth) {
    VS_ARG(sl && d_bgr, "vs_slam_prefetch_batch_dev: null argument");
    VS_ARG(B >= 1 && B <= sl->ops.B, "vs_slam_prefetch_batch_dev: B out of range");
    sl->ops.hint.nb = B;
    sl->ops.hint.bgr = d_bgr;
    sl->ops.hint.depth = d_depth;
    return VS_OK;
}

int vs_slam_process_batch_dev(vs_slam* sl, int B, const uint8_t* d_bgr, const float* d_depth,
                              const float* const* h_depth, const double* timestamps, const int* ids, int* processed) {
    VS_ARG(sl && d_bgr && timestamps && ids && processed, "vs_slam_process_batch_dev: null argument");
    VS_ARG(B >= 1 && B <= sl->ops.B, "vs_slam_process_batch_dev: B out of range");
    VS_ARG(!d_depth == !h_depth, "vs_slam_process_batch_dev: depth must be given on both sides or neither");
    GpuOps& o = sl->ops;
    VS_HIP(hipSetDevice(o.ctx->device));
    CtxStream use(o.ctx, o.s);
    sl->batch.clear();
    for (int b = 0; b < B; b++) {
        auto f = std::make_shared<vs_trk::Frame>();
        f->id = ids[b];
        f->timestamp = timestamps[b];
        f->dh = o.h;
        f->dw = o.w;
        f->depth = h_depth ? h_depth[b] : nullptr;
        sl->batch.push_back(f);
    }
    int rc = o.extract_batch(sl->batch, d_bgr, d_depth);
    for (int b = 0, c = 0; b < B && rc == VS_OK; b++) {
        const auto& X = o.xb[o.xcur];
        if (b == X.ch[c]) rc = o.wait_chunk(sl->batch, c++);
        if (rc != VS_OK) break;
        // the next frame and its chunk's event, for the speculative chain (chain()); the frame after
        // it, for the read-ahead of speculate_next
        o.next_frame = b + 1 < B ? sl->batch[b + 1].get() : nullptr;
        o.next_ready = b + 1 < B ? X.ev[b + 1 == X.ch[c] ? c : c - 1] : nullptr;
        o.next_kps_ready = b + 1 < X.ch[c];  // the next frame's chunk was waited (host keypoints)
        o.bframes = &sl->batch;
        o.bchunk = &c;
        o.next_index = b + 1;
        o.next2_frame = b + 2 < B ? sl->batch[b + 2].get() : nullptr;
        o.next3_frame = b + 3 < B ? sl->batch[b + 3].get() : nullptr;
        o.next2_ready = o.next3_ready = nullptr;
        for (int d = 2; d <= 3; d++)
            if (b + d < B) {
                int c2 = c;
                while (b + d >= X.ch[c2]) c2++;
                (d == 2 ? o.next2_ready : o.next3_ready) = X.ev[c2 - 1];
            }
        if (o.hprof_armed && --o.hprof.skip < 0) o.hprof.on = sl->trk->phase_prof().on = true, o.hprof_armed = false;
        {
            HostTimer ht(o.hprof, kHFrame);
            processed[b] = sl->trk->process_frame(sl->batch[b]) ? 1 : 0;
        }
        o.flush_spec();  // a frame that tracked no local map still launches its speculation
        if (processed[b]) dense_record(sl, *sl->batch[b]);
        if (o.err != VS_OK) {
            rc = o.err;
            o.err = VS_OK;
        }
    }
    o.next_frame = nullptr;
    o.next_ready = nullptr;
    o.next2_frame = nullptr;
    o.next2_ready = nullptr;
    o.next3_frame = nullptr;
    o.next3_ready = nullptr;
    o.next_kps_ready = false;
    o.bframes = nullptr;
    o.bchunk = nullptr;
    o.next_index = -1;
    o.spec_sync();
    o.cnext.valid = false;  // (no speculation outlives the call: its frames may go)
    o.tspec.valid = false;
    if (rc == VS_OK && o.err != VS_OK) rc = o.err;
    o.err = VS_OK;
    for (auto& E : o.cspec) E.valid = false;
    o.spec_req.pending = false;
    // The helper's next-batch enqueue has finished before the call returns, so no thread of this
    // vs_slam touches the context's scratch once the caller has it back; the prefetched batch's
    // device work is ordered before the caller's own use of that scratch by vs::scratch_order.
    const int rj = o.aq.join();
    if (rc == VS_OK) rc = rj;
    if (rc != VS_OK) {
        (void)hipStreamSynchronize(o.xs);  // nothing may still write the pool after an error
        (void)hipStreamSynchronize(o.xp);
        (void)hipStreamSynchronize(o.s2);
        o.xb[o.xcur ^ 1].pending = false;  // a prefetch that failed (or raced an error) is dropped
        o.batch_region = o.xb[o.xcur].region ^ 1;
        sl->dense_depth.clear();
        sl->dense_R.clear();
        sl->dense_t.clear();
        return rc;
    }
    return settle(sl);
}

int vs_slam_process_features(vs_slam* sl, int n_kp, const vs_keypoint* kps, const float* desc, const float* depth,
                             double timestamp, int id, int* processed) {
    VS_ARG(sl && processed && n_kp >= 0 && n_kp <= kCap, "vs_slam_process_features: bad arguments");
    VS_ARG(n_kp == 0 || (kps && desc), "vs_slam_process_features: null features");
    GpuOps& o = sl->ops;
    VS_HIP(hipSetDevice(o.ctx->device));
    CtxStream use(o.ctx, o.s);
    auto f = std::make_shared<vs_trk::Frame>();
    f->id = id;
    f->timestamp = timestamp;
    f->dh = o.h;
    f->dw = o.w;
    f->depth = depth;
    const auto* kp = reinterpret_cast<const vs_trk::Keypoint*>(kps);
    f->kps.assign(kp, kp + n_kp);
    f->mp_idx.assign(n_kp, -1);
    VS_CHECK(o.upload_frame(*f, desc));
    *processed = sl->trk->process_frame(f) ? 1 : 0;
    if (o.err != VS_OK) {
        int rc = o.err;
        o.err = VS_OK;
        return rc;
    }
    if (*processed) dense_record(sl, *f);
    sl->batch.assign(1, f);
    return settle(sl);
}

int vs_slam_attach_dense(vs_slam* sl, vs_dense* d) {
    VS_ARG(sl, "vs_slam_attach_dense: null argument");
    sl->dense = d;
    sl->dense_depth.clear();
    sl->dense_R.clear();
    sl->dense_t.clear();
    return VS_OK;
}

int vs_slam_run_posthoc_pgo(vs_slam* sl, int* loop_edges) {
    VS_ARG(sl, "vs_slam_run_posthoc_pgo: null argument");
    GpuOps& o = sl->ops;
    VS_HIP(hipSetDevice(o.ctx->device));
    CtxStream use(o.ctx, o.s);
    const int n = sl->trk->run_posthoc_pgo();
    if (loop_edges) *loop_edges = n;
    if (o.err != VS_OK) {
        const int rc = o.err;
        o.err = VS_OK;
        return rc;
    }
    return VS_OK;
}

int vs_slam_finish(vs_slam* sl) {
    VS_ARG(sl, "vs_slam_finish: null argument");
    sl->trk->run_rts_smoother();
    return VS_OK;
}

int vs_slam_trajectory(vs_slam* sl, int cap, int* ids, double* timestamps, double* R, double* t, int* n) {
    VS_ARG(sl && n, "vs_slam_trajectory: null argument");
    const auto& fr = sl->trk->map().frames;
    *n = (int)fr.size();
    for (int i = 0; i < (int)fr.size() && i < cap; i++) {
        if (ids) ids[i] = fr[i]->id;
        if (timestamps) timestamps[i] = fr[i]->timestamp;
        if (R) std::memcpy(R + 9 * i, fr[i]->R.data(), 9 * sizeof(double));
        if (t) std::memcpy(t + 3 * i, fr[i]->t.data(), 3 * sizeof(double));
    }
    return VS_OK;
}

int vs_slam_stats(vs_slam* sl, int* out, int cap) {
    VS_ARG(sl && out, "vs_slam_stats: null argument");
    const auto& S = sl->trk->stats();
    const auto& m = sl->trk->map();
    int valid = 0;
    for (uint8_t v : m.valid) valid += v;
    const int v[VS_SLAM_NSTATS] = {S.processed,      S.rejected,       S.via_3d3d,       S.via_emat,
                                   S.emat_failed,    S.bridges,        S.recoveries,     S.recovery_failed,
                                   S.stationary,     S.keyframes,      S.pnp_refined,    S.periodic_pnp,
                                   S.tracked_total,  S.triangulated,   S.depth_points,   S.culled,
                                   S.chains_discarded, m.size(),       valid,            sl->trk->frame_count(),
                                   sl->trk->keyframe_count(), sl->trk->last_match_count(), S.f_iters,
                                   sl->trk->loop_count()};
    for (int i = 0; i < cap && i < VS_SLAM_NSTATS; i++) out[i] = v[i];
    return VS_OK;
}

int vs_slam_loops(vs_slam* sl, int cap, int* edges, double* constraints, int* n_edges, int* n_constraints) {
    VS_ARG(sl && n_edges && n_constraints, "vs_slam_loops: null argument");
    const auto& E = sl->trk->loop_edges();
    const auto& C = sl->trk->loop_constraints();
    *n_edges = (int)E.size();
    *n_constraints = (int)C.size();
    for (int i = 0; i < (int)E.size() && i < cap && edges; i++) {
        edges[2 * i] = E[i].first;
        edges[2 * i + 1] = E[i].second;
    }
    for (int i = 0; i < (int)C.size() && i < cap && constraints; i++) {
        double* c = constraints + 16 * i;
        c[0] = C[i].from_id;
        c[1] = C[i].to_id;
        std::memcpy(c + 2, C[i].R_rel.data(), 9 * sizeof(double));
        std::memcpy(c + 11, C[i].t_rel.data(), 3 * sizeof(double));
        c[14] = C[i].trans_sigma;
        c[15] = C[i].rot_sigma;
    }
    return VS_OK;
}

int vs_slam_map(vs_slam* sl, int cap, double* pos, uint8_t* valid, int* n) {
    VS_ARG(sl && n, "vs_slam_map: null argument");
    const auto& m = sl->trk->map();
    *n = m.size();
    for (int i = 0; i < m.size() && i < cap; i++) {
        if (pos) std::memcpy(pos + 3 * i, &m.pos[3 * i], 3 * sizeof(double));
        if (valid) valid[i] = m.valid[i];
    }
    return VS_OK;
}

}  // extern "C"
