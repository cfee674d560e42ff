// track.hip — Slam::track_local_map on gfx950 (reference src/Slam.cpp:380-469).
//
// The reference walks every map point in order and, for the keypoints within 12 px of its
// projection (30-px grid, :388-455), keeps the first strictly smaller L2 descriptor distance
// below 0.5; the keypoint then takes the map point if that distance beats the keypoint's best so
// far (:460-465).  Phases (one stream, no host round trip):
//   k_tlm_grid     the 30-px keypoint grid in keypoint order, built in LDS by one workgroup;
//   k_tlm_cand     one lane per map point: projection, image / depth gates, the keypoints within
//                  12 px in the reference's visiting order (the point's candidate list);
//   k_tlm_dist     one lane per (map point, candidate): the fp64 L2 distance in cv::norm's order
//                  (float differences, squares summed in groups of four) — the HBM-bound part;
//   k_tlm_resolve  per map point the first strictly smaller distance below 0.5, then the
//                  order-dependent assignment decided in parallel (a candidate wins iff its
//                  distance is below every earlier candidate's for the same keypoint), giving
//                  exactly the reference's kp->map-point table, tracked count and observation
//                  list in map-point order.
// Compiled with -ffp-contract=off: distances and projections equal the CPU restatement bit for bit.
#include <hip/hip_runtime.h>

#include "vs_internal.h"

namespace vs {

constexpr int kTlmCell = 30;       // TRACK_GRID_CELL_SIZE (Config.h:108)
constexpr double kTlmRadius = 12;  // TRACK_SEARCH_RADIUS (Config.h:109)
constexpr double kTlmDesc = 0.5;   // TRACK_DESC_THRESHOLD (Config.h:110)
constexpr int kTlmMaxKp = 1024;

// Keypoint grid (Slam.cpp:389-401): per-cell keypoint lists in keypoint order, built in LDS by one
// workgroup: a keypoint's slot is its cell's prefix count plus the number of earlier keypoints in
// the same cell (the order the reference's push_back produces).
constexpr int kTlmMaxCells = 4096;
// The grid of one frame's keypoints into start[GW * GH + 1] / items[nkp + 1] (-1 in the item slots past
// the grid's last, nit .. nkp); one 1024-thread workgroup.
__device__ void tlm_build_grid(const vs_keypoint* __restrict__ kps, int nkp, int GW, int GH, int* __restrict__ start,
                               int* __restrict__ items) {
    __shared__ int s_cell[kTlmMaxKp];
    __shared__ int s_start[kTlmMaxCells + 1];
    const int tid = threadIdx.x, nc = GW * GH;
    for (int c = tid; c <= nc; c += blockDim.x) s_start[c] = 0;
    __syncthreads();
    for (int ki = tid; ki < nkp; ki += blockDim.x) {
        const int gx = min((int)(kps[ki].x / kTlmCell), GW - 1);
        const int gy = min((int)(kps[ki].y / kTlmCell), GH - 1);
        const int c = (gx >= 0 && gy >= 0) ? gy * GW + gx : -1;
        s_cell[ki] = c;
        if (c >= 0) atomicAdd(&s_start[c + 1], 1);
    }
    __syncthreads();
    // s_start[c + 1] += s_start[c] over the cells: every thread takes 4 consecutive cells, the
    // threads' totals are scanned across the workgroup (integer sums: any order is exact)
    __shared__ int s_wsum[16];
    {
        const int c0 = 4 * tid;
        int v[4], run = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = c0 + k < nc ? s_start[c0 + k + 1] : 0;
            run += v[k];
            v[k] = run;  // inclusive within the thread
        }
        const int lane = tid & 63, wv = tid >> 6;
        int incl = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[wv] = incl;
        __syncthreads();
        int before = incl - run;  // exclusive within the wave
        for (int w = 0; w < wv; w++) before += s_wsum[w];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (c0 + k < nc) s_start[c0 + k + 1] = before + v[k];
    }
    __syncthreads();
    for (int ki = tid; ki < nkp; ki += blockDim.x) {
        const int c = s_cell[ki];
        if (c < 0) continue;
        int rank = 0;
        for (int kj = 0; kj < ki; kj++) rank += s_cell[kj] == c;
        items[s_start[c] + rank] = ki;
    }
    for (int c = tid; c <= nc; c += blockDim.x) start[c] = s_start[c];
    for (int i = s_start[nc] + tid; i <= nkp; i += blockDim.x) items[i] = -1;
}

// Also: the kp -> map-point table from pinned host memory when given (src), so the call needs no
// upload or memset of its own.
__global__ __launch_bounds__(1024) void k_tlm_grid(const vs_keypoint* __restrict__ kps, int nkp, int GW, int GH,
                                                   int* __restrict__ start, int* __restrict__ items,
                                                   int* __restrict__ work_n, const int* __restrict__ src,
                                                   int* __restrict__ kp_to_mp) {
    crit_prio();
    if (threadIdx.x == 0) *work_n = 0;  // the candidate work list of this call (k_tlm_cand appends)
    if (src)
        for (int i = threadIdx.x; i < nkp; i += blockDim.x) kp_to_mp[i] = src[i];
    tlm_build_grid(kps, nkp, GW, GH, start, items);
}

// Round 6: the grids of a batch of frame slots, built when their keypoints exist (the tracker's
// extraction chunk, off the tracking chain); one workgroup per frame: grid[f] = start | items of frame
// slot0 + f (kTlmGridInts ints per slot), counts from n[f].
__global__ __launch_bounds__(1024) void k_tlm_grid_slots(const vs_keypoint* __restrict__ kps, const int* __restrict__ n,
                                                         int kp_stride, int GW, int GH, int* __restrict__ grid) {
    const int f = blockIdx.x;
    const int nkp = min(max(n[f], 0), kTlmMaxKp);
    int* start = grid + (size_t)f * kTlmGridInts;
    tlm_build_grid(kps + (size_t)f * kp_stride, nkp, GW, GH, start, start + GW * GH + 1);
}

__device__ double desc_l2_dev(const float* __restrict__ a, const float* __restrict__ b) {
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const float4* b4 = reinterpret_cast<const float4*>(b);
    double s = 0;
    for (int q = 0; q < 64; q++) {
        const float4 x = a4[q], y = b4[q];
        const double v0 = (double)(x.x - y.x), v1 = (double)(x.y - y.y);
        const double v2 = (double)(x.z - y.z), v3 = (double)(x.w - y.w);
        s += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
    }
    return sqrt(s);
}

struct TlmPose {
    double Rc[9], tc[3], fx, fy, cx, cy;
};

// Phase 1, one lane per map point: projection (:421-431) and the keypoints within the search
// radius in the reference's visiting order (cells row by row, keypoints in insertion order,
// :434-450), stored as the map point's candidate list.  A point with more candidates than slots
// (not reachable with NMS-spaced keypoints, kept for safety) evaluates them itself and stores its
// winner as its single candidate, whose distance phase 2 recomputes identically.
constexpr int kTlmMaxCand = 40;
__global__ __launch_bounds__(256) void k_tlm_cand(const double* __restrict__ mp_pos, const float* __restrict__ mp_desc,
                                                  const uint8_t* __restrict__ mp_valid, int n_mp,
                                                  const vs_keypoint* __restrict__ kps, const float* __restrict__ desc,
                                                  const int* __restrict__ start, const int* __restrict__ items, int GW,
                                                  int GH, int img_w, int img_h, TlmPose T, int* __restrict__ cnt,
                                                  int* __restrict__ cand, int* __restrict__ work,
                                                  int* __restrict__ work_n) {
    crit_prio();
    // the keypoint grid and the keypoint coordinates in LDS (one coalesced pass; every lookup of
    // the candidate scan then stays on chip)
    __shared__ int s_start[kTlmMaxCells + 1];
    __shared__ int s_items[kTlmMaxKp];
    __shared__ float2 s_xy[kTlmMaxKp];
    const int nc = GW * GH;
    for (int i = threadIdx.x; i <= nc; i += 256) s_start[i] = start[i];
    __syncthreads();
    const int nit = s_start[nc];
    for (int i = threadIdx.x; i < nit; i += 256) {
        const int ki = items[i];
        s_items[i] = ki;
        s_xy[ki] = make_float2(kps[ki].x, kps[ki].y);
    }
    __syncthreads();
    const int mp = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    int c = 0;
    int* my = cand + (size_t)min(mp, n_mp - 1) * kTlmMaxCand;
    if (mp < n_mp && mp_valid[mp]) {
        const double x = mp_pos[3 * mp], y = mp_pos[3 * mp + 1], z = mp_pos[3 * mp + 2];
        const double* Rc = T.Rc;
        const double px = Rc[0] * x + Rc[1] * y + Rc[2] * z + T.tc[0];
        const double py = Rc[3] * x + Rc[4] * y + Rc[5] * z + T.tc[1];
        const double pz = Rc[6] * x + Rc[7] * y + Rc[8] * z + T.tc[2];
        if (!(pz < (double)0.1f || pz > 50.0)) {
            const double u = T.fx * px / pz + T.cx;
            const double v = T.fy * py / pz + T.cy;
            if (!(u < 0 || u >= img_w || v < 0 || v >= img_h)) {
                const int gx0 = max(0, (int)((u - kTlmRadius) / kTlmCell));
                const int gy0 = max(0, (int)((v - kTlmRadius) / kTlmCell));
                const int gx1 = min(GW - 1, (int)((u + kTlmRadius) / kTlmCell));
                const int gy1 = min(GH - 1, (int)((v + kTlmRadius) / kTlmCell));
                for (int gy = gy0; gy <= gy1; gy++)
                    for (int gx = gx0; gx <= gx1; gx++) {
                        const int cc = gy * GW + gx;
                        for (int it = s_start[cc]; it < s_start[cc + 1]; it++) {
                            const int ki = s_items[it];
                            const double dx = u - (double)s_xy[ki].x, dy = v - (double)s_xy[ki].y;
                            if (dx * dx + dy * dy > kTlmRadius * kTlmRadius) continue;
                            if (c < kTlmMaxCand) my[c] = ki;
                            c++;
                        }
                    }
                if (c > kTlmMaxCand) {  // overflow: the sequential scan, winner only
                    int bk = -1;
                    double bd = kTlmDesc;
                    const float* md = mp_desc + (size_t)mp * 256;
                    for (int gy = gy0; gy <= gy1; gy++)
                        for (int gx = gx0; gx <= gx1; gx++) {
                            const int cc = gy * GW + gx;
                            for (int it = s_start[cc]; it < s_start[cc + 1]; it++) {
                                const int ki = s_items[it];
                                const double dx = u - (double)s_xy[ki].x, dy = v - (double)s_xy[ki].y;
                                if (dx * dx + dy * dy > kTlmRadius * kTlmRadius) continue;
                                const double d = desc_l2_dev(md, desc + (size_t)ki * 256);
                                if (d < bd) {
                                    bd = d;
                                    bk = ki;
                                }
                            }
                        }
                    c = 0;
                    if (bk >= 0) my[c++] = bk;
                }
            }
        }
    }
    if (mp < n_mp) cnt[mp] = c;
    // append this map point's (map point, slot) pairs to the distance work list: one atomic per
    // wave (the list order is irrelevant: every distance lands at its own slot)
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int total = __shfl(incl, 63);
    int base = 0;
    if (lane == 63 && total > 0) base = atomicAdd(work_n, total);
    base = __shfl(base, 63);
    for (int j = 0; j < c; j++) work[base + incl - c + j] = mp * kTlmMaxCand + j;
}

// Phase 2: the cv::norm distance (:451) of every (map point, candidate) pair on the work list
// (a few per visible map point), one wave per pair, grid-stride: lane q loads float4 q of both
// descriptors (one coalesced 1 KB row each) and forms the group term ((v0^2 + v1^2) + v2^2) + v3^2
// in double; the 64 terms are then added in order q = 0..63 by lane 0 from LDS — the same terms and
// the same sequential sum as desc_l2_dev (cv::norm's groups of four), so bit-identical, with the
// loads in parallel instead of a 64-step strided walk per lane.
__global__ __launch_bounds__(256) void k_tlm_dist(const float* __restrict__ mp_desc, const float* __restrict__ desc,
                                                  const int* __restrict__ cand, const int* __restrict__ work,
                                                  const int* __restrict__ work_n, double* __restrict__ dist) {
    crit_prio();
    __shared__ double s_t[4][64];
    const int n = *work_n;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = blockIdx.x * 4 + wv; i < n; i += gridDim.x * 4) {  // wave-uniform
        const int r = work[i];
        const float4 x = reinterpret_cast<const float4*>(mp_desc + (size_t)(r / kTlmMaxCand) * 256)[lane];
        const float4 y = reinterpret_cast<const float4*>(desc + (size_t)cand[r] * 256)[lane];
        const double v0 = (double)(x.x - y.x), v1 = (double)(x.y - y.y);
        const double v2 = (double)(x.z - y.z), v3 = (double)(x.w - y.w);
        s_t[wv][lane] = v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            double s = 0;
#pragma unroll
            for (int q = 0; q < 64; q++) s += s_t[wv][q];
            dist[r] = sqrt(s);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Assignment in map-point order (Slam.cpp:460-465), decided in parallel: keypoint ki's best
// distance is a running minimum over the map points that chose it, so a candidate (map point m
// with best keypoint ki, distance d) is applied — kp_to_mp[ki] = m, one tracked++ and one
// add_observation — iff d is strictly below every earlier candidate's distance for ki.
// result[0] = tracked, result[1] = observations produced (all of them, even beyond obs_cap).
//
// Phase 3a, one lane per map point: its first strictly smaller distance below the threshold in
// visiting order (:439-456) -> (keypoint or -1, distance).
// Also the map point's rank among its block's candidates and the block's candidate count, so the
// resolve kernel places every candidate in map-point order without a serial scan.
__global__ __launch_bounds__(256) void k_tlm_best(const int* __restrict__ cnt, const int* __restrict__ cand,
                                                  const double* __restrict__ dist, int n_mp, int* __restrict__ best_ki,
                                                  double* __restrict__ best_d, int* __restrict__ rank,
                                                  int* __restrict__ blkcnt, int* __restrict__ work_n) {
    crit_prio();
    // k_tlm_dist (the last reader of the work list's length) has finished: zero it for the next call,
    // whose k_tlm_cand appends without a grid kernel to reset it (round 6)
    if (blockIdx.x == 0 && threadIdx.x == 0) *work_n = 0;
    __shared__ int s_w[4];
    const int mp = blockIdx.x * 256 + threadIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int ki0 = -1;
    double bd = kTlmDesc;
    if (mp < n_mp) {
        const int c = cnt[mp];
        for (int j = 0; j < c; j++) {
            const double d = dist[(size_t)mp * kTlmMaxCand + j];
            if (d < bd) {
                bd = d;
                ki0 = cand[(size_t)mp * kTlmMaxCand + j];
            }
        }
    }
    const unsigned long long bal = __ballot(ki0 >= 0);
    if (lane == 0) s_w[wv] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < wv; k++) off += s_w[k];
    if (mp < n_mp) {
        best_ki[mp] = ki0;
        best_d[mp] = bd;
        rank[mp] = off + __popcll(bal & ((1ull << lane) - 1ull));
    }
    if (threadIdx.x == 0) blkcnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

constexpr int kTlmCandBuf = 4096;  // candidates buffered in LDS between resolve passes
constexpr int kTlmMaxBlk = 4096;  // map points / 256 handled by the direct placement

struct TlmResolveShared {
    unsigned long long best[kTlmMaxKp];  // bits of the running minimum (d >= 0: order-preserving)
    int kpmp[kTlmMaxKp];
    int bcnt[kTlmMaxKp];  // candidates of a keypoint in the current pass
    int seg[kTlmMaxKp];   // their segment in order[]
    int order[kTlmCandBuf];  // the pass's candidates grouped by keypoint (any order within a group)
    int cmp[kTlmCandBuf], cki[kTlmCandBuf];
    unsigned long long cd[kTlmCandBuf];
    int pre[kTlmMaxBlk];
    int wcnt[16];
    int nobs, nc, total;
};
// ~120 KB: one workgroup per CU within gfx950's 160 KB of LDS (this kernel is written for gfx950 only)
static_assert(sizeof(TlmResolveShared) <= 160 * 1024, "k_tlm_resolve's shared state exceeds gfx950's 160 KB LDS");

// One pass over the nc buffered candidates (map-point order): winners are strictly below the
// carried minimum and below every earlier buffered candidate of the keypoint; the last winner of a
// keypoint has its smallest distance (winners strictly decrease); observations are compacted in
// candidate order.  The earlier candidates of a keypoint are found through a counting sort by
// keypoint (counts, a scan over the nkp keypoints, the scatter), so a candidate compares with its own
// keypoint's group only, however many candidates a keypoint draws.
__device__ void tlm_resolve_pass(TlmResolveShared& S, int nc, int nkp, int* __restrict__ obs_mp,
                                 int* __restrict__ obs_kp, int obs_cap) {
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    int slot[kTlmCandBuf / 1024];
#pragma unroll
    for (int r = 0; r < kTlmCandBuf / 1024; r++) {
        const int t = r * 1024 + tid;
        slot[r] = t < nc ? atomicAdd(&S.bcnt[S.cki[t]], 1) : 0;
    }
    __syncthreads();
    {  // exclusive scan of the counts, one keypoint per thread (nkp <= 1024)
        const int c = tid < nkp ? S.bcnt[tid] : 0;
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) S.wcnt[wv] = incl;
        __syncthreads();
        int base = incl - c;
        for (int w = 0; w < wv; w++) base += S.wcnt[w];
        if (tid < nkp) S.seg[tid] = base;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kTlmCandBuf / 1024; r++) {
        const int t = r * 1024 + tid;
        if (t < nc) S.order[S.seg[S.cki[t]] + slot[r]] = t;
    }
    __syncthreads();
    bool win[kTlmCandBuf / 1024];
#pragma unroll
    for (int r = 0; r < kTlmCandBuf / 1024; r++) {
        const int t = r * 1024 + tid;
        win[r] = false;
        if (t < nc) {
            const int ki = S.cki[t];
            const unsigned long long d = S.cd[t];
            bool w = d < S.best[ki];
            const int s0 = S.seg[ki], nb = S.bcnt[ki];
            for (int k = 0; k < nb && w; k++) {  // the keypoint's other candidates: earlier and not larger -> loses
                const int j = S.order[s0 + k];
                if (j < t && S.cd[j] <= d) w = false;
            }
            win[r] = w;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kTlmCandBuf / 1024; r++) {
        const int t = r * 1024 + tid;
        if (t < nc) {
            S.bcnt[S.cki[t]] = 0;  // every reader is past the barrier above
            if (win[r]) atomicMin(&S.best[S.cki[t]], S.cd[t]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kTlmCandBuf / 1024; r++) {
        if (r * 1024 >= nc) break;  // uniform
        const int t = r * 1024 + tid;
        const bool w = win[r];
        if (w && S.best[S.cki[t]] == S.cd[t]) S.kpmp[S.cki[t]] = S.cmp[t];
        const unsigned long long wb = __ballot(w);
        if (lane == 0) S.wcnt[wv] = __popcll(wb);
        __syncthreads();
        int o = S.nobs, nw = 0;
        for (int k = 0; k < 16; k++) {
            if (k < wv) o += S.wcnt[k];
            nw += S.wcnt[k];
        }
        if (w) {
            o += __popcll(wb & ((1ull << lane) - 1ull));
            if (o < obs_cap) {
                obs_mp[o] = S.cmp[t];
                obs_kp[o] = S.cki[t];
            }
        }
        __syncthreads();
        if (tid == 0) S.nobs += nw;
        __syncthreads();
    }
}

// Phase 3b: the assignment in map-point order (Slam.cpp:460-465).  The candidates (k_tlm_best)
// go to an LDS buffer in map-point order at block prefix + rank, kTlmCandBuf of them per pass.
// The PnP input the tracker's refinement takes next (Slam::refine_pose_via_local_pnp's tracked_points,
// Slam.cpp:1408-1420): keypoints in order whose (final) map point is valid, as float object points and
// image points; io = [off {0, n, 0, 0} | obj cap x 3 | img cap x 2].
struct TlmGatherArgs {
    const double* pos = nullptr;
    const uint8_t* valid = nullptr;
    const vs_keypoint* kps = nullptr;
    float* io = nullptr;
    int cap = 0;
};

__global__ __launch_bounds__(1024) void k_tlm_resolve(const int* __restrict__ best_ki, const double* __restrict__ best_d,
                                                      const int* __restrict__ rank, const int* __restrict__ blkcnt,
                                                      int n_mp, int nkp, int* __restrict__ kp_to_mp,
                                                      int* __restrict__ obs_mp, int* __restrict__ obs_kp, int obs_cap,
                                                      int* __restrict__ result, const int* __restrict__ src,
                                                      TlmGatherArgs G) {
    crit_prio();
    __shared__ TlmResolveShared S;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int nblk = (n_mp + 255) / 256;
    for (int k = tid; k < nkp; k += 1024) {
        S.best[k] = (unsigned long long)__double_as_longlong(1e9);
        S.kpmp[k] = src ? src[k] : kp_to_mp[k];  // src: the host's table in pinned memory (no upload)
        S.bcnt[k] = 0;
    }
    if (tid == 0) {
        S.nobs = S.nc = 0;
        S.total = INT_MAX;
    }
    if (nblk <= kTlmMaxBlk) {
        // exclusive prefix over the block counts: 4 consecutive blocks per thread, a wave scan of the
        // thread totals, the waves' totals across the workgroup (integer sums: exact in any order)
        int v[4], run = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int b = 4 * tid + k;
            v[k] = b < nblk ? blkcnt[b] : 0;
            run += v[k];
        }
        int incl = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (lane == 63) S.wcnt[wv] = incl;
        __syncthreads();
        int before = incl - run, all = 0;
        for (int w = 0; w < 16; w++) {
            if (w < wv) before += S.wcnt[w];
            all += S.wcnt[w];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int b = 4 * tid + k;
            if (b < nblk) S.pre[b] = before;
            before += v[k];
        }
        if (tid == 0) S.total = all;
    }
    __syncthreads();
    if (nblk <= kTlmMaxBlk) {
        // Passes over windows of kTlmCandBuf candidates in map-point order: candidate j (block prefix +
        // rank) goes to slot j - p0 of the pass whose window holds it.  Each pass reads every map point's
        // (ki, rank, d) with all loads of a round in flight (L2 latency, not a chain of 1024-point
        // chunks); a pass's outcome does not depend on where a window ends (a candidate wins iff it is
        // below every earlier candidate of its keypoint, carried across passes in S.best).
        const int total = S.total;
        for (int p0 = 0; p0 < total; p0 += kTlmCandBuf) {
            const int pend = min(total, p0 + kTlmCandBuf);
            for (int m0 = 0; m0 < n_mp; m0 += 16 * 1024) {
                // all loads of the round issued before any is used: the rank and distance are read
                // unconditionally (in bounds), so they do not wait for best_ki
                int kis[16], rks[16];
                double bds[16];
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int mp = min(m0 + u * 1024 + tid, n_mp - 1);
                    kis[u] = best_ki[mp];
                    rks[u] = rank[mp];
                    bds[u] = best_d[mp];
                }
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const int mp = m0 + u * 1024 + tid;
                    if (mp >= n_mp || kis[u] < 0) continue;
                    const int j = S.pre[mp >> 8] + rks[u];
                    if (j < p0 || j >= pend) continue;
                    S.cmp[j - p0] = mp;
                    S.cki[j - p0] = kis[u];
                    S.cd[j - p0] = (unsigned long long)__double_as_longlong(bds[u]);
                }
            }
            __syncthreads();
            tlm_resolve_pass(S, pend - p0, nkp, obs_mp, obs_kp, obs_cap);
        }
    } else {  // more than kTlmMaxBlk * 256 map points: 1024 at a time, a pass whenever the buffer could overflow
        for (int c0 = 0; c0 < n_mp; c0 += 1024) {
            const int mp = c0 + tid;
            const int ki0 = mp < n_mp ? best_ki[mp] : -1;
            const bool cand_ok = ki0 >= 0;
            const unsigned long long bal = __ballot(cand_ok);
            if (lane == 0) S.wcnt[wv] = __popcll(bal);
            __syncthreads();
            int off = S.nc, add = 0;
            for (int k = 0; k < 16; k++) {
                if (k < wv) off += S.wcnt[k];
                add += S.wcnt[k];
            }
            if (cand_ok) {
                const int j = off + __popcll(bal & ((1ull << lane) - 1ull));
                S.cmp[j] = mp;
                S.cki[j] = ki0;
                S.cd[j] = (unsigned long long)__double_as_longlong(best_d[mp]);
            }
            __syncthreads();
            const int nc = S.nc + add;
            if (tid == 0) S.nc = nc;
            __syncthreads();
            if (nc + 1024 <= kTlmCandBuf && c0 + 1024 < n_mp) continue;  // uniform
            tlm_resolve_pass(S, nc, nkp, obs_mp, obs_kp, obs_cap);
            if (tid == 0) S.nc = 0;
            __syncthreads();
        }
    }
    __syncthreads();
    for (int k = tid; k < nkp; k += 1024) kp_to_mp[k] = S.kpmp[k];
    if (tid == 0) {
        result[0] = S.nobs;  // each record is one tracked++ and one add_observation
        result[1] = S.nobs;
    }
    if (G.io) {  // nkp <= 1024: one keypoint per thread, in order (a block prefix of the ballots)
        const int id = tid < nkp ? S.kpmp[tid] : -1;
        const bool use = id >= 0 && id < n_mp && G.valid[id];
        const unsigned long long bal = __ballot(use);
        __syncthreads();  // every reader of S.wcnt above is done
        if (lane == 0) S.wcnt[wv] = __popcll(bal);
        __syncthreads();
        int o = 0, n = 0;
        for (int k = 0; k < 16; k++) {
            if (k < wv) o += S.wcnt[k];
            n += S.wcnt[k];
        }
        float* obj = G.io + 4;
        float* img = obj + 3 * G.cap;
        if (use) {
            o += __popcll(bal & ((1ull << lane) - 1ull));
            obj[3 * o] = (float)G.pos[3 * id];
            obj[3 * o + 1] = (float)G.pos[3 * id + 1];
            obj[3 * o + 2] = (float)G.pos[3 * id + 2];
            img[2 * o] = G.kps[tid].x;
            img[2 * o + 1] = G.kps[tid].y;
        }
        if (tid == 0) {
            int* off = reinterpret_cast<int*>(G.io);
            off[0] = 0;
            off[1] = n;
            off[2] = off[3] = 0;
        }
    }
}


int tlm_grid_slots(const vs_keypoint* d_kps, const int* d_n, int nframes, int kp_stride, int img_w, int img_h,
                   int* d_grid, hipStream_t s) {
    if (nframes <= 0) return VS_OK;
    VS_ARG(img_w > 0 && img_h > 0 && ((img_w + kTlmCell - 1) / kTlmCell) * ((img_h + kTlmCell - 1) / kTlmCell) <= kTlmMaxCells,
           "tlm_grid_slots: image too large for the keypoint grid");
    static_assert(kTlmGridInts >= kTlmMaxCells + 1 + kTlmMaxKp + 1, "grid slot too small");
    const int GW = (img_w + kTlmCell - 1) / kTlmCell, GH = (img_h + kTlmCell - 1) / kTlmCell;
    hipLaunchKernelGGL(k_tlm_grid_slots, dim3(nframes), dim3(1024), 0, s, d_kps, d_n, kp_stride, GW, GH, d_grid);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int track_local_map(vs_ctx* ctx, const double* d_mp_pos, const float* d_mp_desc, const uint8_t* d_mp_valid, int n_mp,
                    const vs_keypoint* d_kps, const float* d_desc, int nkp, const double R[9], const double t[3],
                    const double K[4], int img_w, int img_h, int* d_kp_to_mp, int* d_obs_mp, int* d_obs_kp,
                    int obs_cap, int* d_result, hipStream_t s, const int* h_kp_to_mp_src, const TlmExtra* ex) {
    VS_ARG(nkp >= 0 && nkp <= kTlmMaxKp, "track_local_map: at most 1024 keypoints");
    VS_ARG(img_w > 0 && img_h > 0, "track_local_map: bad image size");
    VS_ARG(((img_w + kTlmCell - 1) / kTlmCell) * ((img_h + kTlmCell - 1) / kTlmCell) <= kTlmMaxCells,
           "track_local_map: image too large for the keypoint grid");
    VS_ARG(!ex || !ex->gather_io || ex->gather_cap >= nkp, "track_local_map: gather capacity below the keypoints");
    const int GW = (img_w + kTlmCell - 1) / kTlmCell, GH = (img_h + kTlmCell - 1) / kTlmCell;
    // layout: the work list's length first (a fixed place: k_tlm_best leaves it zero for the next
    // call), then the grid, the per-map-point arrays
    const size_t grid_bytes = 16 + (size_t)(GW * GH + 1) * sizeof(int) + (size_t)(nkp + 1) * sizeof(int);
    const size_t per_mp = 3 * sizeof(int) + sizeof(double) + (size_t)kTlmMaxCand * (2 * sizeof(int) + sizeof(double));
    const int nblk = (n_mp + 255) / 256;
    void* before = ctx->tlm.p;
    VS_CHECK(ctx->tlm.ensure(grid_bytes + 64 + (size_t)(n_mp + 1) * per_mp + (size_t)(nblk + 2) * sizeof(int)));
    char* base = static_cast<char*>(ctx->tlm.p);
    int* work_n = reinterpret_cast<int*>(base);
    const bool pre_grid = ex && ex->grid && nkp > 0;
    if (pre_grid && ctx->tlm.p != before) VS_HIP(hipMemsetAsync(work_n, 0, sizeof(int), s));  // a new buffer
    int* start = pre_grid ? const_cast<int*>(ex->grid) : reinterpret_cast<int*>(base + 16);
    int* items = start + GW * GH + 1;
    double* dist = reinterpret_cast<double*>(base + ((grid_bytes + 15) / 16) * 16);
    int* cand = reinterpret_cast<int*>(dist + (size_t)(n_mp + 1) * kTlmMaxCand);
    int* cnt = cand + (size_t)(n_mp + 1) * kTlmMaxCand;
    int* best_ki = cnt + (n_mp + 1);
    int* rank = best_ki + (n_mp + 1);
    int* blkcnt = rank + (n_mp + 1) + 1;
    int* work = blkcnt + nblk + 1;
    double* best_d =
        reinterpret_cast<double*>(base + (((size_t)(reinterpret_cast<char*>(work + (size_t)(n_mp + 1) * kTlmMaxCand) - base) + 15) / 16) * 16);
    TlmPose T;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T.Rc[i * 3 + j] = R[j * 3 + i];
    for (int i = 0; i < 3; i++) T.tc[i] = -(T.Rc[i * 3 + 0] * t[0] + T.Rc[i * 3 + 1] * t[1] + T.Rc[i * 3 + 2] * t[2]);
    T.fx = K[0];
    T.fy = K[1];
    T.cx = K[2];
    T.cy = K[3];
    ProfScope ps(ctx, "track_local_map", s);
    if (pre_grid) {
        // the grid was built with the frame's keypoints; k_tlm_resolve reads the host's table itself
    } else if (nkp > 0) {
        hipLaunchKernelGGL(k_tlm_grid, dim3(1), dim3(1024), 0, s, d_kps, nkp, GW, GH, start, items, work_n,
                           h_kp_to_mp_src, d_kp_to_mp);
    } else {
        VS_HIP(hipMemsetAsync(items, 0xff, sizeof(int), s));
        VS_HIP(hipMemsetAsync(start, 0, (size_t)(GW * GH + 1) * sizeof(int), s));
        VS_HIP(hipMemsetAsync(work_n, 0, sizeof(int), s));
    }
    if (n_mp > 0) {
        hipLaunchKernelGGL(k_tlm_cand, dim3((n_mp + 255) / 256), dim3(256), 0, s, d_mp_pos, d_mp_desc, d_mp_valid, n_mp,
                           d_kps, d_desc, start, items, GW, GH, img_w, img_h, T, cnt, cand, work, work_n);
        hipLaunchKernelGGL(k_tlm_dist, dim3(512), dim3(256), 0, s, d_mp_desc, d_desc, cand, work, work_n, dist);
    }
    if (n_mp > 0)
        hipLaunchKernelGGL(k_tlm_best, dim3(nblk), dim3(256), 0, s, cnt, cand, dist, n_mp, best_ki, best_d, rank,
                           blkcnt, work_n);
    TlmGatherArgs G;
    if (ex && ex->gather_io) {
        G.pos = d_mp_pos;
        G.valid = d_mp_valid;
        G.kps = d_kps;
        G.io = ex->gather_io;
        G.cap = ex->gather_cap;
    }
    hipLaunchKernelGGL(k_tlm_resolve, dim3(1), dim3(1024), 0, s, best_ki, best_d, rank, blkcnt, n_mp, nkp, d_kp_to_mp,
                       d_obs_mp, d_obs_kp, obs_cap, d_result, pre_grid ? h_kp_to_mp_src : nullptr, G);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
