// dense.hip — F4 dense voxel fusion (reference src/main.cpp:1081-1146, written out by :1463-1474):
// every processed frame with real depth back-projects its depth map on a DENSE_PIXEL_STEP grid
// with the frame's pose at processing time, and a point is appended to the dense cloud the first
// time its DENSE_VOXEL_SIZE voxel is seen (std::unordered_set<tuple<int,int,int>>::insert(..).second,
// :1133-1139).  The cloud is the ordered list of those first points.
//
// Device layout (HBM):
//   keys   [T] u64   packed voxel (x, y, z as 21-bit two's complement), ~0 = empty; open addressing,
//                    linear probing, T a power of two (default 2^24 slots, 256 MB with stamps);
//   stamps [T] u64   smallest insertion stamp seen for the slot: stamp = the sample's position in
//                    the reference's insertion order (frame order, then row-major grid order);
//   cloud  [cap][3]  f64 points in insertion order; count / error flags beside.
// One integrate call (<= kDF frames per launch group) runs four kernels: insert (one thread per
// grid sample: key, atomicCAS into the table, atomicMin of its stamp), count (per 256 samples:
// winners = samples whose stamp is the slot's minimum and newer than every earlier call), a
// one-workgroup exclusive scan of the block counts, and an ordered write (ballot compaction).  The
// result equals the sequential std::unordered_set loop point for point and in order.
// Arithmetic as the reference writes it, compiled with -ffp-contract=off: x = (u - cx) * z / fx,
// p = R x + t - origin left to right, voxel = (int)floor(p * (1 / voxel_size)).
// HBM-bound byte work: per sample one 4 B depth read (a 32 B sector), 16 B of table traffic and
// 24 B per new point; a frame of 640 x 480 at step 8 is 4800 samples.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "vs_internal.h"

namespace vs {

constexpr int kDF = 32;                           // frames per launch group (kernel-argument block)
constexpr unsigned long long kEmpty = ~0ull;
constexpr int kPackBits = 21;
constexpr int kPackLim = 1 << (kPackBits - 1);    // voxel coordinates in [-2^20, 2^20)
constexpr unsigned kErrTable = 1u, kErrCapacity = 2u;

struct DenseFrames {
    const float* depth[kDF];
    double R[kDF][9];
    double t[kDF][3];
};

struct DenseArgs {
    int nf, h, w, step, nu, spf;
    double max_depth, fx, fy, cx, cy, inv_voxel, ox, oy, oz;
    unsigned long long* keys;
    unsigned long long* stamps;
    unsigned long long mask;
    unsigned long long seq0;  // stamp of this group's first sample
    int* slot;                // per sample: table slot, -1 = no point
    int* bcnt;                // per 256-sample block: new points
    long long* boff;          // per block: first cloud index
    long long* count;         // points in the cloud
    double* cloud;
    long long cap;
    unsigned* err;
};

// (int)std::floor(d) as x86-64 evaluates it: cvttsd2si gives INT_MIN for NaN and out-of-range
__device__ __forceinline__ int x86_floor_i32(double d) {
    const double f = floor(d);
    return (f >= -2147483648.0 && f < 2147483648.0) ? (int)f : INT_MIN;
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// main.cpp:1121-1136 for grid sample i of frame f: false if the depth is rejected
__device__ __forceinline__ bool dense_point(const DenseArgs& a, const DenseFrames& F, int f, int i, double p[3],
                                            int vox[3]) {
    const int gv = i / a.nu, gu = i - gv * a.nu;
    const int v = gv * a.step, u = gu * a.step;
    const float z = F.depth[f][(size_t)v * a.w + u];
    if (z <= 0 || (double)z >= a.max_depth) return false;
    const double zd = (double)z;
    const double x_cam = ((double)u - a.cx) * zd / a.fx;
    const double y_cam = ((double)v - a.cy) * zd / a.fy;
    const double* R = F.R[f];
    const double* t = F.t[f];
    p[0] = R[0] * x_cam + R[1] * y_cam + R[2] * zd + t[0] - a.ox;
    p[1] = R[3] * x_cam + R[4] * y_cam + R[5] * zd + t[1] - a.oy;
    p[2] = R[6] * x_cam + R[7] * y_cam + R[8] * zd + t[2] - a.oz;
    for (int k = 0; k < 3; k++) vox[k] = x86_floor_i32(p[k] * a.inv_voxel);
    return true;
}

__global__ __launch_bounds__(256) void k_dense_insert(DenseArgs a, DenseFrames F) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= a.nf * a.spf) return;
    const int f = g / a.spf, i = g - f * a.spf;
    double p[3];
    int vox[3];
    int slot = -1;
    if (dense_point(a, F, f, i, p, vox)) {
        bool packable = true;
        unsigned long long key = 0;
        for (int k = 0; k < 3; k++) {
            packable = packable && vox[k] >= -kPackLim && vox[k] < kPackLim;
            key = (key << kPackBits) | ((unsigned long long)(unsigned)vox[k] & ((1ull << kPackBits) - 1));
        }
        if (!packable) {
            // Outside +-2^20 voxels (a diverged pose; INT_MIN from NaN / overflow): the reference
            // still inserts the (int, int, int) tuple.  Such voxels get a 63-bit hash of all 96 bits
            // with the top bit set — disjoint from the packed keys (top bit 0), unique unless two
            // out-of-range voxels collide in 63 bits (documented).
            unsigned long long hv = mix64(((unsigned long long)(unsigned)vox[0] << 32) | (unsigned)vox[1]);
            hv = mix64(hv ^ (unsigned long long)(unsigned)vox[2] ^ 0x9E3779B97F4A7C15ull);
            key = (hv & 0x7FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;
            if (key == kEmpty) key ^= 1ull;
        }
        {
            const unsigned long long stamp = a.seq0 + (unsigned long long)g;
            unsigned long long h = mix64(key) & a.mask;
            for (unsigned long long probe = 0; probe <= a.mask; probe++) {
                const unsigned long long prev = atomicCAS(a.keys + h, kEmpty, key);
                if (prev == kEmpty || prev == key) {
                    atomicMin(a.stamps + h, stamp);
                    slot = (int)h;
                    break;
                }
                h = (h + 1) & a.mask;
            }
            if (slot < 0) atomicOr(a.err, kErrTable);
        }
    }
    a.slot[g] = slot;
}

__device__ __forceinline__ bool dense_winner(const DenseArgs& a, int g) {
    if (g >= a.nf * a.spf) return false;
    const int s = a.slot[g];
    // the slot's minimum stamp is this sample's, and no earlier call saw the voxel (stamps of
    // earlier calls are all below seq0)
    return s >= 0 && a.stamps[s] == a.seq0 + (unsigned long long)g;
}

__global__ __launch_bounds__(256) void k_dense_count(DenseArgs a) {
    __shared__ int s_w[4];
    const int g = blockIdx.x * 256 + threadIdx.x;
    const unsigned long long bal = __ballot(dense_winner(a, g));
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = __popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) a.bcnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// one workgroup: boff[b] = count + sum(bcnt[0..b)), then count += total
__global__ __launch_bounds__(1024) void k_dense_scan(DenseArgs a, int nblk) {
    __shared__ long long s_part[1024];
    __shared__ long long s_base;
    const int tid = threadIdx.x;
    if (tid == 0) s_base = *a.count;
    __syncthreads();
    for (int c0 = 0; c0 < nblk; c0 += 1024) {
        const int b = c0 + tid;
        const long long v = b < nblk ? a.bcnt[b] : 0;
        s_part[tid] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
            const long long add = tid >= o ? s_part[tid - o] : 0;
            __syncthreads();
            s_part[tid] += add;
            __syncthreads();
        }
        if (b < nblk) a.boff[b] = s_base + s_part[tid] - v;
        __syncthreads();
        if (tid == 0) s_base += s_part[1023];
        __syncthreads();
    }
    if (tid == 0) *a.count = s_base;
}

__global__ __launch_bounds__(256) void k_dense_write(DenseArgs a, DenseFrames F) {
    __shared__ int s_w[4];
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool win = dense_winner(a, g);
    const unsigned long long bal = __ballot(win);
    if (lane == 0) s_w[wv] = __popcll(bal);
    __syncthreads();
    if (!win) return;
    long long idx = a.boff[blockIdx.x] + __popcll(bal & ((1ull << lane) - 1ull));
    for (int k = 0; k < wv; k++) idx += s_w[k];
    if (idx >= a.cap) {
        atomicOr(a.err, kErrCapacity);
        return;
    }
    const int f = g / a.spf, i = g - f * a.spf;
    double p[3];
    int vox[3];
    dense_point(a, F, f, i, p, vox);
    a.cloud[3 * idx] = p[0];
    a.cloud[3 * idx + 1] = p[1];
    a.cloud[3 * idx + 2] = p[2];
}

}  // namespace vs

struct vs_dense {
    vs_ctx* ctx = nullptr;
    vs_dense_config cfg{};
    unsigned long long mask = 0;
    unsigned long long seq = 0;  // samples integrated so far (the next stamp)
    vs::DevBuf keys, stamps, cloud, state, scratch;  // state: {count (i64), err (u32)}
    hipStream_t last = nullptr;
};

using namespace vs;

namespace {

hipStream_t pick(vs_dense* d, void* stream) { return stream ? (hipStream_t)stream : d->ctx->stream; }

int dense_reset(vs_dense* d, hipStream_t s) {
    VS_HIP(hipMemsetAsync(d->keys.p, 0xFF, (size_t)(d->mask + 1) * 8, s));
    VS_HIP(hipMemsetAsync(d->stamps.p, 0xFF, (size_t)(d->mask + 1) * 8, s));
    VS_HIP(hipMemsetAsync(d->state.p, 0, 16, s));
    d->seq = 0;
    d->last = s;
    return VS_OK;
}

}  // namespace

extern "C" {

void vs_dense_default_config(vs_dense_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->pixel_step = 8;      // Config::DENSE_PIXEL_STEP (Config.h:118)
    c->max_depth = 5.0;     // Config::DENSE_MAX_DEPTH (:119)
    c->voxel_size = 0.02;   // Config::DENSE_VOXEL_SIZE (:120)
    c->fx = 525.0;          // Config::FX / FY / CX / CY (:14-17)
    c->fy = 525.0;
    c->cx = 319.5;
    c->cy = 239.5;
    c->table_log2 = 24;
    c->max_points = 8 << 20;
}

int vs_dense_create(vs_ctx* ctx, const vs_dense_config* cfg, vs_dense** out) {
    VS_ARG(ctx && out, "vs_dense_create: null argument");
    *out = nullptr;
    vs_dense_config c;
    if (cfg)
        c = *cfg;
    else
        vs_dense_default_config(&c);
    VS_ARG(c.pixel_step >= 1 && c.voxel_size > 0 && c.fx != 0 && c.fy != 0, "vs_dense_create: bad configuration");
    VS_ARG(c.table_log2 >= 10 && c.table_log2 <= 30, "vs_dense_create: table_log2 must be in [10, 30]");
    VS_ARG(c.max_points >= 1 && c.max_points <= (1ll << c.table_log2), "vs_dense_create: max_points out of range");
    VS_HIP(hipSetDevice(ctx->device));
    vs_dense* d = new (std::nothrow) vs_dense();
    if (!d) return VS_ERR_NOMEM;
    d->ctx = ctx;
    d->cfg = c;
    d->mask = (1ull << c.table_log2) - 1;
    const size_t T = (size_t)d->mask + 1;
    int rc = VS_OK;
    if (rc == VS_OK) rc = d->keys.ensure(T * 8);
    if (rc == VS_OK) rc = d->stamps.ensure(T * 8);
    if (rc == VS_OK) rc = d->cloud.ensure((size_t)c.max_points * 3 * sizeof(double));
    if (rc == VS_OK) rc = d->state.ensure(16);
    if (rc == VS_OK) rc = dense_reset(d, ctx->stream);
    if (rc != VS_OK) {
        vs_dense_destroy(d);
        return rc;
    }
    *out = d;
    return VS_OK;
}

void vs_dense_destroy(vs_dense* d) {
    if (!d) return;
    if (d->last) (void)hipStreamSynchronize(d->last);
    d->keys.release();
    d->stamps.release();
    d->cloud.release();
    d->state.release();
    d->scratch.release();
    delete d;
}

int vs_dense_reset(vs_dense* d, void* stream) {
    VS_ARG(d, "vs_dense_reset: null argument");
    VS_HIP(hipSetDevice(d->ctx->device));
    return dense_reset(d, pick(d, stream));
}

int vs_dense_integrate_dev(vs_dense* d, int nf, const float* const* d_depth, int h, int w, const double* R,
                           const double* t, void* stream) {
    VS_ARG(d && nf >= 0 && h > 0 && w > 0, "vs_dense_integrate_dev: bad arguments");
    if (nf == 0) return VS_OK;
    VS_ARG(d_depth && R && t, "vs_dense_integrate_dev: null argument");
    for (int f = 0; f < nf; f++) VS_ARG(d_depth[f], "vs_dense_integrate_dev: null depth map");
    VS_HIP(hipSetDevice(d->ctx->device));
    const hipStream_t s = pick(d, stream);
    const vs_dense_config& c = d->cfg;
    DenseArgs a{};
    a.h = h;
    a.w = w;
    a.step = c.pixel_step;
    a.nu = (w + c.pixel_step - 1) / c.pixel_step;
    a.spf = a.nu * ((h + c.pixel_step - 1) / c.pixel_step);
    a.max_depth = c.max_depth;
    a.fx = c.fx;
    a.fy = c.fy;
    a.cx = c.cx;
    a.cy = c.cy;
    a.inv_voxel = 1.0 / c.voxel_size;  // main.cpp:1086 (DENSE_VOXEL_INV)
    a.ox = c.origin[0];
    a.oy = c.origin[1];
    a.oz = c.origin[2];
    a.keys = d->keys.as<unsigned long long>();
    a.stamps = d->stamps.as<unsigned long long>();
    a.mask = d->mask;
    a.cloud = d->cloud.as<double>();
    a.cap = c.max_points;
    a.count = d->state.as<long long>();
    a.err = reinterpret_cast<unsigned*>(d->state.as<char>() + 8);
    const int max_samples = kDF * a.spf, max_blk = (max_samples + 255) / 256;
    const size_t slot_b = ((size_t)max_samples * sizeof(int) + 255) & ~(size_t)255;
    const size_t cnt_b = ((size_t)max_blk * sizeof(int) + 255) & ~(size_t)255;
    VS_CHECK(d->scratch.ensure(slot_b + cnt_b + (size_t)max_blk * sizeof(long long)));
    a.slot = d->scratch.as<int>();
    a.bcnt = reinterpret_cast<int*>(d->scratch.as<char>() + slot_b);
    a.boff = reinterpret_cast<long long*>(d->scratch.as<char>() + slot_b + cnt_b);
    ProfScope ps(d->ctx, "dense_fusion", s);
    for (int f0 = 0; f0 < nf; f0 += kDF) {
        DenseFrames F{};
        a.nf = std::min(kDF, nf - f0);
        for (int f = 0; f < a.nf; f++) {
            F.depth[f] = d_depth[f0 + f];
            std::memcpy(F.R[f], R + 9 * (size_t)(f0 + f), 9 * sizeof(double));
            std::memcpy(F.t[f], t + 3 * (size_t)(f0 + f), 3 * sizeof(double));
        }
        a.seq0 = d->seq;
        const int n = a.nf * a.spf, nblk = (n + 255) / 256;
        hipLaunchKernelGGL(k_dense_insert, dim3(nblk), dim3(256), 0, s, a, F);
        hipLaunchKernelGGL(k_dense_count, dim3(nblk), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_dense_scan, dim3(1), dim3(1024), 0, s, a, nblk);
        hipLaunchKernelGGL(k_dense_write, dim3(nblk), dim3(256), 0, s, a, F);
        VS_HIP(hipGetLastError());
        d->seq += (unsigned long long)n;
    }
    d->last = s;
    return VS_OK;
}

int vs_dense_size(vs_dense* d, long long* n) {
    VS_ARG(d && n, "vs_dense_size: null argument");
    VS_HIP(hipSetDevice(d->ctx->device));
    if (d->last) VS_HIP(hipStreamSynchronize(d->last));
    struct {
        long long count;
        unsigned err, pad;
    } st;
    VS_HIP(hipMemcpy(&st, d->state.p, sizeof(st), hipMemcpyDeviceToHost));
    *n = std::min<long long>(st.count, d->cfg.max_points);
    if (st.err & kErrTable) {
        set_error("vs_dense: voxel table full (raise table_log2)");
        return VS_ERR_CAPACITY;
    }
    if (st.err & kErrCapacity) {
        set_error("vs_dense: more points than max_points");
        return VS_ERR_CAPACITY;
    }
    return VS_OK;
}

int vs_dense_points(vs_dense* d, long long cap, double* xyz, long long* n) {
    VS_ARG(d && n && cap >= 0 && (cap == 0 || xyz), "vs_dense_points: bad arguments");
    VS_CHECK(vs_dense_size(d, n));
    const long long m = std::min(cap, *n);
    if (m > 0) VS_HIP(hipMemcpy(xyz, d->cloud.p, (size_t)m * 3 * sizeof(double), hipMemcpyDeviceToHost));
    return VS_OK;
}

const double* vs_dense_points_dev(vs_dense* d) { return d ? d->cloud.as<double>() : nullptr; }

// main.cpp:1463-1474: ascii PLY, std::fixed with 6 decimals
int vs_dense_write_ply(vs_dense* d, const char* path) {
    VS_ARG(d && path, "vs_dense_write_ply: null argument");
    long long n = 0;
    VS_CHECK(vs_dense_size(d, &n));
    if (n == 0) return VS_OK;  // main.cpp:1462: no file for an empty cloud
    std::vector<double> p((size_t)n * 3);
    if (n > 0) VS_HIP(hipMemcpy(p.data(), d->cloud.p, p.size() * sizeof(double), hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path, "w");
    if (!f) {
        set_error("vs_dense_write_ply: cannot create file");
        return VS_ERR_IO;
    }
    std::fprintf(f, "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
                    "property float z\nend_header\n", n);
    for (long long i = 0; i < n; i++) std::fprintf(f, "%.6f %.6f %.6f\n", p[3 * i], p[3 * i + 1], p[3 * i + 2]);
    const bool ok = std::fclose(f) == 0;
    if (!ok) {
        set_error("vs_dense_write_ply: write failed");
        return VS_ERR_IO;
    }
    return VS_OK;
}

}  // extern "C"
