// track.hip — Slam::track_local_map on gfx950 (reference src/Slam.cpp:380-469).
//
// The reference walks every map point in order and, for the keypoints within 12 px of its
// projection (30-px grid, :388-455), keeps the first strictly smaller L2 descriptor distance
// below 0.5; the keypoint then takes the map point if that distance beats the keypoint's best so
// far (:460-465).  Two phases:
//   k_tlm_match    one lane per map point: projection, grid cells, candidate distances (fp64,
//                  cv::norm's order: float differences, squares summed in groups of four), best
//                  keypoint + distance — independent across map points, the HBM-bound part;
//   k_tlm_resolve  the order-dependent assignment: candidates (map points with a best keypoint)
//                  compacted in map-point order 1024 at a time and applied sequentially, which
//                  yields exactly the reference's final kp->map-point table, tracked count and
//                  (map point, keypoint) observation list in map-point order.
// Compiled with -ffp-contract=off: distances and projections equal the CPU restatement bit for bit.
#include <hip/hip_runtime.h>

#include "vs_internal.h"

namespace vs {

constexpr int kTlmCell = 30;       // TRACK_GRID_CELL_SIZE (Config.h:108)
constexpr double kTlmRadius = 12;  // TRACK_SEARCH_RADIUS (Config.h:109)
constexpr double kTlmDesc = 0.5;   // TRACK_DESC_THRESHOLD (Config.h:110)
constexpr int kTlmMaxKp = 1024;

// Keypoint grid: cells in keypoint order (counting sort on one lane; <= 1024 keypoints).
__global__ void k_tlm_grid(const vs_keypoint* __restrict__ kps, int nkp, int GW, int GH, int* __restrict__ start,
                           int* __restrict__ items) {
    if (threadIdx.x != 0) return;
    const int nc = GW * GH;
    for (int c = 0; c <= nc; c++) start[c] = 0;
    for (int ki = 0; ki < nkp; ki++) {
        int gx = min((int)(kps[ki].x / kTlmCell), GW - 1);
        int gy = min((int)(kps[ki].y / kTlmCell), GH - 1);
        if (gx >= 0 && gy >= 0) start[gy * GW + gx + 1]++;
    }
    for (int c = 0; c < nc; c++) start[c + 1] += start[c];
    // second pass places keypoints in order; reuse items[] write cursors from start[]
    for (int ki = 0, filled = 0; ki < nkp; ki++) {
        (void)filled;
        int gx = min((int)(kps[ki].x / kTlmCell), GW - 1);
        int gy = min((int)(kps[ki].y / kTlmCell), GH - 1);
        if (gx >= 0 && gy >= 0) {
            const int c = gy * GW + gx;
            int pos = start[c];
            while (items[pos] != -1) pos++;  // items pre-filled with -1
            items[pos] = ki;
        }
    }
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

__global__ __launch_bounds__(256) void k_tlm_match(const double* __restrict__ mp_pos, const float* __restrict__ mp_desc,
                                                   const uint8_t* __restrict__ mp_valid, int n_mp,
                                                   const vs_keypoint* __restrict__ kps, const float* __restrict__ desc,
                                                   const int* __restrict__ start, const int* __restrict__ items, int GW,
                                                   int GH, int img_w, int img_h, TlmPose T, int* __restrict__ best_ki,
                                                   double* __restrict__ best_d) {
    const int mp = blockIdx.x * 256 + threadIdx.x;
    if (mp >= n_mp) return;
    int bk = -1;
    double bd = kTlmDesc;
    if (mp_valid[mp]) {
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
                const float* md = mp_desc + (size_t)mp * 256;
                for (int gy = gy0; gy <= gy1; gy++)
                    for (int gx = gx0; gx <= gx1; gx++) {
                        const int c = gy * GW + gx;
                        for (int it = start[c]; it < start[c + 1]; it++) {
                            const int ki = items[it];
                            const double dx = u - (double)kps[ki].x, dy = v - (double)kps[ki].y;
                            if (dx * dx + dy * dy > kTlmRadius * kTlmRadius) continue;
                            const double d = desc_l2_dev(md, desc + (size_t)ki * 256);
                            if (d < bd) {
                                bd = d;
                                bk = ki;
                            }
                        }
                    }
            }
        }
    }
    best_ki[mp] = bk;
    best_d[mp] = bd;
}

// Sequential assignment in map-point order (Slam.cpp:460-465).  One 1024-lane workgroup.
// result[0] = tracked, result[1] = observations produced (all of them, even beyond obs_cap).
__global__ __launch_bounds__(1024) void k_tlm_resolve(const int* __restrict__ best_ki, const double* __restrict__ best_d,
                                                      int n_mp, int nkp, int* __restrict__ kp_to_mp,
                                                      int* __restrict__ obs_mp, int* __restrict__ obs_kp, int obs_cap,
                                                      int* __restrict__ result) {
    __shared__ double s_best[kTlmMaxKp];
    __shared__ int s_kpmp[kTlmMaxKp];
    __shared__ int s_cmp[1024];
    __shared__ int s_wcnt[16];
    __shared__ int s_nobs;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    for (int k = tid; k < nkp; k += 1024) {
        s_best[k] = 1e9;
        s_kpmp[k] = kp_to_mp[k];
    }
    if (tid == 0) s_nobs = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n_mp; c0 += 1024) {
        const int mp = c0 + tid;
        const bool cand = mp < n_mp && best_ki[mp] >= 0;
        const unsigned long long bal = __ballot(cand);
        if (lane == 0) s_wcnt[wv] = __popcll(bal);
        __syncthreads();
        int off = 0;
        for (int k = 0; k < wv; k++) off += s_wcnt[k];
        if (cand) s_cmp[off + __popcll(bal & ((1ull << lane) - 1ull))] = mp;
        __syncthreads();
        if (tid == 0) {
            int nc = 0;
            for (int k = 0; k < 16; k++) nc += s_wcnt[k];
            int nobs = s_nobs;
            for (int j = 0; j < nc; j++) {
                const int m = s_cmp[j];
                const int ki = best_ki[m];
                const double d = best_d[m];
                if (d < s_best[ki]) {
                    s_kpmp[ki] = m;
                    s_best[ki] = d;
                    if (nobs < obs_cap) {
                        obs_mp[nobs] = m;
                        obs_kp[nobs] = ki;
                    }
                    nobs++;
                }
            }
            s_nobs = nobs;
        }
        __syncthreads();
    }
    for (int k = tid; k < nkp; k += 1024) kp_to_mp[k] = s_kpmp[k];
    if (tid == 0) {
        result[0] = s_nobs;  // each record is one tracked++ and one add_observation
        result[1] = s_nobs;
    }
}

int track_local_map(vs_ctx* ctx, const double* d_mp_pos, const float* d_mp_desc, const uint8_t* d_mp_valid, int n_mp,
                    const vs_keypoint* d_kps, const float* d_desc, int nkp, const double R[9], const double t[3],
                    const double K[4], int img_w, int img_h, int* d_kp_to_mp, int* d_obs_mp, int* d_obs_kp,
                    int obs_cap, int* d_result, hipStream_t s) {
    VS_ARG(nkp >= 0 && nkp <= kTlmMaxKp, "track_local_map: at most 1024 keypoints");
    VS_ARG(img_w > 0 && img_h > 0, "track_local_map: bad image size");
    const int GW = (img_w + kTlmCell - 1) / kTlmCell, GH = (img_h + kTlmCell - 1) / kTlmCell;
    const size_t grid_bytes = (size_t)(GW * GH + 1) * sizeof(int) + (size_t)(nkp + 1) * sizeof(int);
    const size_t per_mp = sizeof(int) + sizeof(double);
    VS_CHECK(ctx->tlm.ensure(grid_bytes + 16 + (size_t)(n_mp + 1) * per_mp));
    char* base = static_cast<char*>(ctx->tlm.p);
    int* start = reinterpret_cast<int*>(base);
    int* items = start + GW * GH + 1;
    double* best_d = reinterpret_cast<double*>(base + ((grid_bytes + 15) / 16) * 16);
    int* best_ki = reinterpret_cast<int*>(best_d + n_mp + 1);
    TlmPose T;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T.Rc[i * 3 + j] = R[j * 3 + i];
    for (int i = 0; i < 3; i++) T.tc[i] = -(T.Rc[i * 3 + 0] * t[0] + T.Rc[i * 3 + 1] * t[1] + T.Rc[i * 3 + 2] * t[2]);
    T.fx = K[0];
    T.fy = K[1];
    T.cx = K[2];
    T.cy = K[3];
    ProfScope ps(ctx, "track_local_map", s);
    VS_HIP(hipMemsetAsync(items, 0xff, (size_t)(nkp + 1) * sizeof(int), s));
    if (nkp > 0) hipLaunchKernelGGL(k_tlm_grid, dim3(1), dim3(64), 0, s, d_kps, nkp, GW, GH, start, items);
    else VS_HIP(hipMemsetAsync(start, 0, (size_t)(GW * GH + 1) * sizeof(int), s));
    if (n_mp > 0)
        hipLaunchKernelGGL(k_tlm_match, dim3((n_mp + 255) / 256), dim3(256), 0, s, d_mp_pos, d_mp_desc, d_mp_valid, n_mp,
                           d_kps, d_desc, start, items, GW, GH, img_w, img_h, T, best_ki, best_d);
    hipLaunchKernelGGL(k_tlm_resolve, dim3(1), dim3(1024), 0, s, best_ki, best_d, n_mp, nkp, d_kp_to_mp, d_obs_mp,
                       d_obs_kp, obs_cap, d_result);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
