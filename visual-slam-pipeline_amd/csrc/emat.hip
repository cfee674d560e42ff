// emat.hip — Slam::estimate_motion (reference src/Slam.cpp:1193-1213: cv::findEssentialMat(K,
// RANSAC, 0.999, 1.0 px) + cv::recoverPose + the inlier and determinant checks) and the depth scale
// (Slam::estimate_scale_from_depth / _single_depth, :73-207) on gfx950.
//
// One workgroup (4 wave64s) per problem.  The reference runs this path when the 3D-3D estimate
// fails (Slam.cpp:965-984), so in the pipeline a problem whose 3D-3D result is ok exits at once.
// RANSAC: chunks of 32 subsets drawn by lane 0 with the cv::RNG stream (5 distinct indices, no
// subset check), one 5-point solve per lane, 8 lanes of each wave (up to 10 models, LDS), rounds of 4 hypotheses scored
// by the waves (Sampson error, ballot counts, early exit below the current best) and replayed in
// order by lane 0.  recoverPose: the cheirality test of every point under the four decompositions
// in parallel.  Scale: per-point candidates sorted in LDS (bitonic), IQR filter, median.  Numerical
// kernels shared with the CPU restatement (emat_solvers.h, -ffp-contract=off).
#include <hip/hip_runtime.h>

#include "emat_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_em;

constexpr int kEmMaxPts = VS_EM_MAX_POINTS;
constexpr int kEmChunk = 32;  // 5-point solves per round, 8 per wave; workspace in LDS
constexpr int kEmThreads = 256;
constexpr int kEmWaves = kEmThreads / 64;

__device__ inline int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

struct EmShared {
    float px1[2 * kEmMaxPts], px2[2 * kEmMaxPts];  // pixels (the scale estimators use them)
    double q1[2 * kEmMaxPts], q2[2 * kEmMaxPts];   // normalised
    int subset[kEmChunk * 5];
    double Em[kEmChunk * kMaxModels * 9];
    double ws[kWsSize * kEmChunk];  // per-lane solver workspace, lane-interleaved
    int nmod[kEmChunk];
    int score[kEmChunk * kMaxModels];
    double sv[2 * kEmMaxPts];  // scale candidates (sorted)
    double E[9], R1[9], R2[9], t[3];
    uint64_t rng;
    int niters, best, best_iter, iter, done, ok, chunk, cnt[4], nsv;
    unsigned char mask[kEmMaxPts];
};

// ascending bitonic sort of S.sv[0..n) padded with +inf to a power of two (<= 2 * kEmMaxPts)
__device__ void sort_sv(EmShared& S, int n) {
    int m = 1;
    while (m < n) m <<= 1;
    for (int i = n + threadIdx.x; i < m; i += blockDim.x) S.sv[i] = __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= m; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const double a = S.sv[i], b = S.sv[l];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        S.sv[i] = b;
                        S.sv[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// Problem source: FROM_PAIRS = frame pairs (pipeline: kept matches, keypoints, depth slots), else
// point arrays with offsets (ABI single problem, depth1/depth2 host-uploaded or null).
// out: R [p][9], t [p][3], scale [p], ok [p], diag [p][8] = {E found, iterations, winning iteration,
// E inliers, recoverPose good, n, ran, 0}
template <bool FROM_PAIRS>
__global__ __launch_bounds__(kEmThreads) void k_emat(const int* __restrict__ pairs, const vs_keypoint* __restrict__ kps,
                                                     int cap, const vs_match* __restrict__ kept,
                                                     const int* __restrict__ nkept, const int* __restrict__ skip,
                                                     const float* __restrict__ pts1, const float* __restrict__ pts2,
                                                     const int* __restrict__ off, const float* __restrict__ depth,
                                                     const float* __restrict__ depth1, const float* __restrict__ depth2,
                                                     int h, int w, double fx, double fy, double cx, double cy,
                                                     double* __restrict__ R_out, double* __restrict__ t_out,
                                                     double* __restrict__ scale_out, int* __restrict__ ok_out,
                                                     int* __restrict__ diag) {
    __shared__ EmShared S;
    __shared__ int red_cnt[4 * kEmWaves];
    const int pb = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int* dg = diag + 8 * pb;
    if (tid == 0) {
        for (int k = 0; k < 8; k++) dg[k] = 0;
        dg[2] = -1;
        ok_out[pb] = 0;
        scale_out[pb] = -1.0;
    }
    if (skip && skip[pb]) return;  // 3D-3D succeeded: the reference never reaches estimate_motion
    int n;
    const float *d1 = nullptr, *d2 = nullptr;
    if (FROM_PAIRS) {
        n = min(nkept[pb], cap);
        const vs_match* gm = kept + (size_t)pb * cap;
        const vs_keypoint* kr = kps + (size_t)pairs[2 * pb] * cap;
        const vs_keypoint* kc = kps + (size_t)pairs[2 * pb + 1] * cap;
        for (int i = tid; i < n; i += blockDim.x) {
            const vs_match m = gm[i];
            S.px1[2 * i] = kr[m.query_idx].x;
            S.px1[2 * i + 1] = kr[m.query_idx].y;
            S.px2[2 * i] = kc[m.train_idx].x;
            S.px2[2 * i + 1] = kc[m.train_idx].y;
        }
        d1 = depth ? depth + (size_t)pairs[2 * pb] * h * w : nullptr;  // null: monocular, no scale
        d2 = depth ? depth + (size_t)pairs[2 * pb + 1] * h * w : nullptr;
    } else {
        const int o0 = off[pb];
        n = off[pb + 1] - o0;
        for (int i = tid; i < 2 * n; i += blockDim.x) {
            S.px1[i] = pts1[2 * (size_t)o0 + i];
            S.px2[i] = pts2[2 * (size_t)o0 + i];
        }
        d1 = depth1;
        d2 = depth2;
    }
    if (tid == 0) dg[5] = n;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        S.q1[2 * i] = ((double)S.px1[2 * i] - cx) / fx;
        S.q1[2 * i + 1] = ((double)S.px1[2 * i + 1] - cy) / fy;
        S.q2[2 * i] = ((double)S.px2[2 * i] - cx) / fx;
        S.q2[2 * i + 1] = ((double)S.px2[2 * i + 1] - cy) / fy;
    }
    if (n < 5) return;  // Slam.cpp:1195
    const double thr = 1.0 / ((fx + fy) / 2);
    const float thr2 = (float)(thr * thr);
    if (tid == 0) {
        S.rng = (uint64_t)-1;
        S.best = 0;
        S.best_iter = -1;
        S.iter = 0;
        S.done = n == 5;
        S.ok = 0;
        S.niters = 1000;
        if (n == 5) {  // count == modelPoints: a single kernel run, first model
            if (five_point(S.q1, S.q2, S.Em, S.ws, kEmChunk) > 0) {
                for (int k = 0; k < 9; k++) S.E[k] = S.Em[k];
                S.ok = 1;
            }
        }
    }
    __syncthreads();
    // ---- RANSAC (RANSACPointSetRegistrator, 5 model points) ----
    while (!S.done) {
        const int base = S.iter;
        if (tid == 0) {
            const int chunk = min(kEmChunk, S.niters - base);
            vs_pnp::CvRng rng(S.rng);
            for (int c = 0; c < chunk; c++)
                for (int i = 0; i < 5; i++)
                    for (;;) {
                        const int v = rng.uniform(0, n);
                        int j = 0;
                        while (j < i && S.subset[5 * c + j] != v) j++;
                        if (j == i) {
                            S.subset[5 * c + i] = v;
                            break;
                        }
                    }
            S.rng = rng.state;
            S.chunk = chunk;
        }
        __syncthreads();
        const int chunk = S.chunk;
        // the chunk's solves spread over the four waves (lanes 0..7 of each): one SIMD per wave, and
        // each wave waits only for the slowest of its 8 root searches, not of 32
        const int js = wv * (kEmChunk / kEmWaves) + lane;
        if (lane < kEmChunk / kEmWaves && js < chunk) {
            double s1[10], s2[10];
            for (int i = 0; i < 5; i++) {
                const int k = S.subset[5 * js + i];
                s1[2 * i] = S.q1[2 * k];
                s1[2 * i + 1] = S.q1[2 * k + 1];
                s2[2 * i] = S.q2[2 * k];
                s2[2 * i + 1] = S.q2[2 * k + 1];
            }
            S.nmod[js] = five_point(s1, s2, &S.Em[js * kMaxModels * 9], &S.ws[js], kEmChunk);
        }
        __syncthreads();
        for (int r0 = 0; r0 < chunk; r0 += kEmWaves) {
            const int hh = r0 + wv;
            if (hh < chunk && base + hh < S.niters) {
                const int bar = S.best > 4 ? S.best : 4;
                for (int k = 0; k < S.nmod[hh]; k++) {
                    const double* E = &S.Em[(hh * kMaxModels + k) * 9];
                    int cnt = 0;
                    for (int i0 = 0; i0 < n; i0 += 64) {
                        const int i = i0 + lane;
                        const bool in = i < n && sampson_err(E, S.q1[2 * i], S.q1[2 * i + 1], S.q2[2 * i],
                                                             S.q2[2 * i + 1]) <= thr2;
                        cnt += __popcll(__ballot(in));
                        if (cnt + max(0, n - i0 - 64) <= bar) {
                            cnt = -1;
                            break;
                        }
                    }
                    if (lane == 0) S.score[hh * kMaxModels + k] = cnt;
                }
            }
            __syncthreads();
            if (tid == 0) {
                int it = S.iter;
                for (int q = r0; q < min(r0 + kEmWaves, chunk) && it < S.niters; q++, it++)
                    for (int k = 0; k < S.nmod[q]; k++) {
                        const int cnt = S.score[q * kMaxModels + k];
                        if (cnt > (S.best > 4 ? S.best : 4)) {
                            S.best = cnt;
                            S.best_iter = it;
                            for (int e = 0; e < 9; e++) S.E[e] = S.Em[(q * kMaxModels + k) * 9 + e];
                            S.niters = vs_pnp::ransac_update_num_iters(0.999, (double)(n - cnt) / n, 5, S.niters);
                        }
                    }
                S.iter = it;
            }
            __syncthreads();
            if (S.iter >= S.niters) break;
        }
        if (tid == 0) {
            if (S.iter >= S.niters) S.done = 1;
            if (S.done) S.ok = S.best > 0;
        }
        __syncthreads();
    }
    if (tid == 0) {
        dg[0] = S.ok;
        dg[1] = S.iter;
        dg[2] = S.best_iter;
    }
    if (!S.ok) return;  // E.empty() (:1200)
    // ---- inliers of E (countNonZero(mask), :1202-1203) ----
    double E[9];
    for (int k = 0; k < 9; k++) E[k] = S.E[k];
    int local = 0;
    for (int i = tid; i < n; i += blockDim.x) {
        const bool in = n == 5 || sampson_err(E, S.q1[2 * i], S.q1[2 * i + 1], S.q2[2 * i], S.q2[2 * i + 1]) <= thr2;
        S.mask[i] = in;
        local += in;
    }
    local = wave_sum(local);
    if (lane == 0) red_cnt[wv] = local;
    __syncthreads();
    int inl = 0;
    for (int q = 0; q < kEmWaves; q++) inl += red_cnt[q];
    if (tid == 0) dg[3] = inl;
    __syncthreads();
    if (inl < 15) return;  // MIN_INLIERS
    // ---- recoverPose (distance 50) ----
    if (tid == 0) decompose_essential(E, S.R1, S.R2, S.t);
    __syncthreads();
    const double tn[3] = {-S.t[0], -S.t[1], -S.t[2]};
    int good[4] = {0, 0, 0, 0};
    for (int i = tid; i < n; i += blockDim.x) {
        if (!S.mask[i]) continue;
        const double x1 = S.q1[2 * i], y1 = S.q1[2 * i + 1], x2 = S.q2[2 * i], y2 = S.q2[2 * i + 1];
        good[0] += cheiral_ok(S.R1, S.t, x1, y1, x2, y2, 50.0);
        good[1] += cheiral_ok(S.R2, S.t, x1, y1, x2, y2, 50.0);
        good[2] += cheiral_ok(S.R1, tn, x1, y1, x2, y2, 50.0);
        good[3] += cheiral_ok(S.R2, tn, x1, y1, x2, y2, 50.0);
    }
    for (int c = 0; c < 4; c++) {
        good[c] = wave_sum(good[c]);
        if (lane == 0) red_cnt[4 * wv + c] = good[c];
    }
    __syncthreads();
    int g[4] = {0, 0, 0, 0};
    for (int q = 0; q < kEmWaves; q++)
        for (int c = 0; c < 4; c++) g[c] += red_cnt[4 * q + c];
    int pick;
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3])
        pick = 0;
    else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3])
        pick = 1;
    else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3])
        pick = 2;
    else
        pick = 3;
    const double* Rp = (pick & 1) ? S.R2 : S.R1;
    double tp[3];
    for (int k = 0; k < 3; k++) tp[k] = pick >= 2 ? tn[k] : S.t[k];
    if (tid == 0) dg[4] = g[pick];
    if (g[pick] < 15) return;                               // :1206
    if (fabs(vs_pnp::det3(Rp) - 1.0) > 0.01) return;       // :1208-1209
    // ---- scale (Slam.cpp:73-156, 162-207) ----
    double sc = -1.0;
    if (d1) {
        bool single = d2 == nullptr;
        if (!single) {
            if (tid == 0) S.nsv = 0;
            __syncthreads();
            for (int i = tid; i < n; i += blockDim.x) {
                const float u1 = S.px1[2 * i], v1 = S.px1[2 * i + 1], u2 = S.px2[2 * i], v2 = S.px2[2 * i + 1];
                const int px1 = (int)roundf(u1), py1 = (int)roundf(v1), px2 = (int)roundf(u2), py2 = (int)roundf(v2);
                if (px1 < 0 || px1 >= w || py1 < 0 || py1 >= h) continue;
                if (px2 < 0 || px2 >= w || py2 < 0 || py2 >= h) continue;
                const float z1 = d1[(size_t)py1 * w + px1], z2 = d2[(size_t)py2 * w + px2];
                if (z1 <= 0.1f || z1 > 10.0f || z2 <= 0.1f || z2 > 10.0f) continue;
                const double P1[3] = {(u1 - cx) * z1 / fx, (v1 - cy) * z1 / fy, (double)z1};
                const double P2[3] = {(u2 - cx) * z2 / fx, (v2 - cy) * z2 / fy, (double)z2};
                double dff[3];
                for (int r = 0; r < 3; r++)
                    dff[r] = P2[r] - (Rp[r * 3] * P1[0] + Rp[r * 3 + 1] * P1[1] + Rp[r * 3 + 2] * P1[2]);
                const double s = dff[0] * tp[0] + dff[1] * tp[1] + dff[2] * tp[2];
                if (s > 0.001 && s < 50.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
            }
            __syncthreads();
            const int c = S.nsv;
            if (c < 10) {
                single = true;
            } else {
                sort_sv(S, c);
                const double q1 = S.sv[c / 4], q3 = S.sv[3 * c / 4];
                const double lo = q1 - 1.5 * (q3 - q1), hi = q3 + 1.5 * (q3 - q1);
                int i1 = 0, i2 = 0;  // the filtered values are the contiguous run [i1, i2)
                while (i1 < c && !(S.sv[i1] >= lo)) i1++;
                i2 = i1;
                while (i2 < c && S.sv[i2] <= hi) i2++;
                sc = i2 > i1 ? S.sv[i1 + (i2 - i1) / 2] : S.sv[c / 2];
            }
        }
        if (single) {
            __syncthreads();
            if (tid == 0) S.nsv = 0;
            __syncthreads();
            for (int i = tid; i < n; i += blockDim.x) {
                const float u1 = S.px1[2 * i], v1 = S.px1[2 * i + 1];
                const int px1 = (int)roundf(u1), py1 = (int)roundf(v1);
                if (px1 < 0 || px1 >= w || py1 < 0 || py1 >= h) continue;
                const float z1 = d1[(size_t)py1 * w + px1];
                if (z1 <= 0.1f || z1 > 10.0f) continue;
                const double X1 = (u1 - cx) * z1 / fx, Y1 = (v1 - cy) * z1 / fy, Z1 = z1;
                const double Rx = Rp[0] * X1 + Rp[1] * Y1 + Rp[2] * Z1, Ry = Rp[3] * X1 + Rp[4] * Y1 + Rp[5] * Z1,
                             Rz = Rp[6] * X1 + Rp[7] * Y1 + Rp[8] * Z1;
                const double a = (S.px2[2 * i] - cx) / fx, den_x = tp[0] - a * tp[2];
                if (fabs(den_x) > 1e-4) {
                    const double s = (a * Rz - Rx) / den_x;
                    if (s > 0.001 && s < 100.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
                }
                const double b = (S.px2[2 * i + 1] - cy) / fy, den_y = tp[1] - b * tp[2];
                if (fabs(den_y) > 1e-4) {
                    const double s = (b * Rz - Ry) / den_y;
                    if (s > 0.001 && s < 100.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
                }
            }
            __syncthreads();
            const int c = S.nsv;
            if (c >= 10) {
                sort_sv(S, c);
                sc = S.sv[c / 2];
            } else {
                sc = -1.0;
            }
        }
    }
    if (tid == 0) {
        for (int k = 0; k < 9; k++) R_out[9 * pb + k] = Rp[k];
        for (int k = 0; k < 3; k++) t_out[3 * pb + k] = tp[k];
        scale_out[pb] = sc;
        ok_out[pb] = 1;
        dg[6] = 1;
    }
}

int emat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_kept,
               const int* d_nkept, const int* d_skip, const float* d_depth, int h, int w, const double K[4],
               double* d_R, double* d_t, double* d_scale, int* d_ok, int* d_diag, hipStream_t s) {
    if (P <= 0) return VS_OK;
    VS_ARG(cap <= kEmMaxPts, "emat_pairs: cap above VS_EM_MAX_POINTS");
    ProfScope ps(ctx, "emat_motion", s);
    hipLaunchKernelGGL(k_emat<true>, dim3(P), dim3(kEmThreads), 0, s, d_pairs, d_kps, cap, d_kept, d_nkept, d_skip,
                       nullptr, nullptr, nullptr, d_depth, nullptr, nullptr, h, w, K[0], K[1], K[2], K[3], d_R, d_t,
                       d_scale, d_ok, d_diag);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int emat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, const float* d_depth1,
                const float* d_depth2, int h, int w, const double K[4], double* d_R, double* d_t, double* d_scale,
                int* d_ok, int* d_diag, hipStream_t s) {
    if (P <= 0) return VS_OK;
    ProfScope ps(ctx, "emat_motion", s);
    hipLaunchKernelGGL(k_emat<false>, dim3(P), dim3(kEmThreads), 0, s, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                       d_p1, d_p2, d_off, nullptr, d_depth1, d_depth2, h, w, K[0], K[1], K[2], K[3], d_R, d_t,
                       d_scale, d_ok, d_diag);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
