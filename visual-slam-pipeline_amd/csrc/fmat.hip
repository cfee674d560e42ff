// fmat.hip — F-matrix verification of Slam::process_frame on gfx950 (reference
// src/Slam.cpp:880-910: extract_matched_points :1174-1187, cv::findFundamentalMat(FM_RANSAC,
// 3.0, RANSAC_PROB = 0.999), mask filtering of good_matches in order, compute_epipolar_error
// before and after :1217-1240).
//
// One workgroup (4 wave64s) per frame pair.  The registrators are sequential only through the
// cv::RNG stream and the shrinking iteration budget, so iterations run in chunks of 256:
// lane 0 draws the chunk's subsets (with the collinearity rejection, which depends on the data
// only), every lane solves one 7-point subset and scores its up to three models (inlier count
// for RANSAC, median error for LMedS), and lane 0 replays the acceptance rule over the chunk in
// iteration order.  A chunk past the final budget is never drawn.  The winning subset is
// re-solved for the final model (identical arithmetic), inliers are marked, the match list is
// compacted in order, and both epipolar errors are reduced over the workgroup.  Numerical
// kernels are shared with the CPU restatement (fmat_solvers.h, built with -ffp-contract=off).
#include <hip/hip_runtime.h>

#include "block_reduce.h"
#include "fmat_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_fm;

constexpr int kFmMaxPts = VS_FM_MAX_POINTS;
constexpr int kChunk = 256;

struct FmShared {
    float p1[2 * kFmMaxPts], p2[2 * kFmMaxPts];
    int subset[kChunk * 7];
    int nmod[kChunk];
    float score[kChunk * 3];  // RANSAC: inlier count; LMedS: median error
    int scan[256];
    double F[9];
    uint64_t rng;
    int best_subset[7];
    int niters, best, best_k, best_iter, iter, fail_at, done, aborted, ok, chunk, inliers;
    double min_median;
};

__device__ inline int solve_idx(const FmShared& S, const int* idx, double (*F)[9]) {
    float x1[7], y1[7], x2[7], y2[7];
    for (int i = 0; i < 7; i++) {
        x1[i] = S.p1[2 * idx[i]];
        y1[i] = S.p1[2 * idx[i] + 1];
        x2[i] = S.p2[2 * idx[i]];
        y2[i] = S.p2[2 * idx[i] + 1];
    }
    return run_7point(x1, y1, x2, y2, F);
}

// Problem source: FROM_MATCHES = pairs of frames + keypoints + good matches (pipeline), else
// point arrays with offsets (ABI single-problem path).
// diag[p][8] = {method, iterations run, winning iteration, inliers, F ok, n, kept, 0}
template <bool FROM_MATCHES>
__global__ __launch_bounds__(256) void k_fmat(const int* __restrict__ pairs, const vs_keypoint* __restrict__ kps,
                                              int cap, const vs_match* __restrict__ good,
                                              const int* __restrict__ ngood, const float* __restrict__ pts1,
                                              const float* __restrict__ pts2, const int* __restrict__ off,
                                              double thr, double conf, int max_iters, double* __restrict__ Fout,
                                              uint8_t* __restrict__ mask_out, vs_match* __restrict__ kept,
                                              int* __restrict__ nkept, double* __restrict__ err,
                                              int* __restrict__ diag) {
    __shared__ FmShared S;
    const int pb = blockIdx.x, tid = threadIdx.x;
    int n;
    const vs_match* gm = nullptr;
    if (FROM_MATCHES) {
        n = min(ngood[pb], cap);
        gm = good + (size_t)pb * cap;
        const vs_keypoint* kr = kps + (size_t)pairs[2 * pb] * cap;
        const vs_keypoint* kc = kps + (size_t)pairs[2 * pb + 1] * cap;
        for (int i = tid; i < n; i += blockDim.x) {  // extract_matched_points (:1184-1187)
            const vs_match m = gm[i];
            S.p1[2 * i] = kr[m.query_idx].x;
            S.p1[2 * i + 1] = kr[m.query_idx].y;
            S.p2[2 * i] = kc[m.train_idx].x;
            S.p2[2 * i + 1] = kc[m.train_idx].y;
        }
    } else {
        const int o0 = off[pb];
        n = off[pb + 1] - o0;
        for (int i = tid; i < 2 * n; i += blockDim.x) {
            S.p1[i] = pts1[2 * (size_t)o0 + i];
            S.p2[i] = pts2[2 * (size_t)o0 + i];
        }
    }
    int* dg = diag + 8 * pb;
    const int method = n < 7 ? 0 : n == 7 ? 1 : n >= 15 ? 2 : 3;
    if (tid == 0) {
        S.rng = (uint64_t)-1;
        S.best = 0;
        S.best_k = 0;
        S.best_iter = -1;
        S.iter = 0;
        S.fail_at = -1;
        S.done = method < 2;
        S.aborted = 0;
        S.ok = 0;
        S.min_median = DBL_MAX;
        S.niters = method == 2 ? (max_iters > 1 ? max_iters : 1) : 0;
        if (method == 3) {
            const int ni = vs_pnp::ransac_update_num_iters(conf, 0.45, 7, max_iters);
            S.niters = ni > 3 ? ni : 3;
        }
        if (method == 1) {
            const int all[7] = {0, 1, 2, 3, 4, 5, 6};
            double Fs[3][9];
            if (solve_idx(S, all, Fs) > 0) {
                for (int k = 0; k < 9; k++) S.F[k] = Fs[0][k];
                S.ok = 1;
            }
        }
    }
    __syncthreads();
    const float thr2 = (float)(thr * thr);
    // ---- registrator loop, one chunk of iterations at a time ----
    for (int base = 0; !S.done; base += kChunk) {
        if (tid == 0) {
            const int chunk = min(kChunk, S.niters - base);
            CvRng rng(S.rng);
            const int attempts = method == 2 ? 10000 : 1000;
            int j = 0;
            for (; j < chunk; j++)
                if (!get_subset(rng, S.p1, S.p2, n, attempts, S.subset + 7 * j)) {
                    S.fail_at = base + j;
                    break;
                }
            S.rng = rng.state;
            S.chunk = j;
        }
        __syncthreads();
        const int chunk = S.chunk;
        if (tid < chunk) {
            double Fs[3][9];
            const int nm = solve_idx(S, S.subset + 7 * tid, Fs);
            S.nmod[tid] = nm;
            for (int k = 0; k < nm; k++) {
                if (method == 2) {
                    int cnt = 0;
                    for (int i = 0; i < n; i++)
                        cnt += fm_error(Fs[k], S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1]) <= thr2;
                    S.score[3 * tid + k] = (float)cnt;
                } else {  // LMedS: n <= 14, median = element n/2 of the sorted errors
                    float e[14];
                    for (int i = 0; i < n; i++) {
                        const float v = fm_error(Fs[k], S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1]);
                        int q = i;
                        while (q > 0 && e[q - 1] > v) {
                            e[q] = e[q - 1];
                            q--;
                        }
                        e[q] = v;
                    }
                    S.score[3 * tid + k] = e[n / 2];
                }
            }
        }
        __syncthreads();
        if (tid == 0) {  // sequential replay of this chunk
            int it = base;
            for (; it < base + chunk && it < S.niters; it++) {
                const int h = it - base;
                for (int k = 0; k < S.nmod[h]; k++) {
                    if (method == 2) {
                        const int cnt = (int)S.score[3 * h + k];
                        if (cnt > (S.best > 6 ? S.best : 6)) {
                            S.best = cnt;
                            S.best_iter = it;
                            S.best_k = k;
                            for (int q = 0; q < 7; q++) S.best_subset[q] = S.subset[7 * h + q];
                            S.niters = vs_pnp::ransac_update_num_iters(conf, (double)(n - cnt) / n, 7, S.niters);
                        }
                    } else {
                        const double med = S.score[3 * h + k];
                        if (med < S.min_median) {
                            S.min_median = med;
                            S.best_iter = it;
                            S.best_k = k;
                            for (int q = 0; q < 7; q++) S.best_subset[q] = S.subset[7 * h + q];
                        }
                    }
                }
            }
            if (S.fail_at >= 0 && it == S.fail_at) {  // getSubset failed at this iteration
                if (it == 0) S.aborted = 1;
                S.done = 1;
            }
            if (it >= S.niters) S.done = 1;
            S.iter = it;
            if (S.done && !S.aborted) {
                const bool have = method == 2 ? S.best > 0 : S.min_median < DBL_MAX;
                if (have) {
                    double Fs[3][9];
                    solve_idx(S, S.best_subset, Fs);
                    for (int k = 0; k < 9; k++) S.F[k] = Fs[S.best_k][k];
                    S.ok = 1;
                }
            }
        }
        __syncthreads();
    }
    // ---- inliers of the final model ----
    float gate = thr2;
    if (method == 3 && S.ok) {
        double sigma = 2.5 * 1.4826 * (1 + 5. / (n - 7)) * sqrt(S.min_median);
        sigma = sigma > 0.001 ? sigma : 0.001;
        gate = (float)(sigma * sigma);
    }
    const bool have_f = S.ok;
    double F[9];
    for (int k = 0; k < 9; k++) F[k] = S.F[k];
    // contiguous segment per lane so the compaction keeps the reference's order
    const int per = (n + 255) / 256, lo = min(n, tid * per), hi = min(n, lo + per);
    int local = 0;
    uint32_t bits = 0;  // per <= 8 since n <= 2048
    for (int i = lo; i < hi; i++) {
        bool in = true;
        if (have_f && method != 1)
            in = fm_error(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1]) <= gate;
        bits |= (uint32_t)in << (i - lo);
        local += in;
    }
    S.scan[tid] = local;
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int q = 0; q < 256; q++) {
            const int c = S.scan[q];
            S.scan[q] = acc;
            acc += c;
        }
        S.inliers = acc;
    }
    __syncthreads();
    bool ok = have_f;
    if (method == 3 && have_f && S.inliers < 7) ok = false;  // LMeDS: result = count >= modelPoints
    // keep everything when F is empty (Slam.cpp:887, 892)
    {
        int w = ok ? S.scan[tid] : lo;
        for (int i = lo; i < hi; i++) {
            const bool in = ok ? ((bits >> (i - lo)) & 1u) : true;
            if (mask_out) mask_out[(FROM_MATCHES ? (size_t)pb * cap : (size_t)off[pb]) + i] = ok ? in : 0;
            if (FROM_MATCHES && in) kept[(size_t)pb * cap + w++] = gm[i];
        }
    }
    // ---- epipolar errors (Slam.cpp:888-890, 903-905) ----
    double part[4] = {0, 0, 0, 0}, tot[4];
    if (ok) {
        for (int i = lo; i < hi; i++) {
            double term;
            if (epipolar_term(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1], term)) {
                part[0] += term;
                part[1] += 1.0;
                if ((bits >> (i - lo)) & 1u) {
                    part[2] += term;
                    part[3] += 1.0;
                }
            }
        }
    }
    __shared__ double red4[4 * 4];
    block_sum<4>(part, red4, tot);
    if (tid == 0) {
        const int kept_n = ok ? S.inliers : n;
        if (FROM_MATCHES) nkept[pb] = kept_n;
        err[2 * pb] = (ok && tot[1] > 0) ? tot[0] / tot[1] : 0.0;
        err[2 * pb + 1] = (ok && S.inliers > 0 && tot[3] > 0) ? tot[2] / tot[3] : 0.0;
        for (int k = 0; k < 9; k++) Fout[9 * pb + k] = ok ? F[k] : 0.0;
        dg[0] = method;
        dg[1] = S.iter;
        dg[2] = S.best_iter;
        dg[3] = (method == 1 && ok) ? n : (have_f ? S.inliers : 0);
        dg[4] = ok;
        dg[5] = n;
        dg[6] = kept_n;
        dg[7] = 0;
    }
}

int fmat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_good,
               const int* d_ngood, double* d_F, vs_match* d_kept, int* d_nkept, double* d_err, int* d_diag,
               hipStream_t s) {
    if (P <= 0) return VS_OK;
    VS_ARG(cap <= kFmMaxPts, "fmat_pairs: cap above VS_FM_MAX_POINTS");
    ProfScope ps(ctx, "fmat_ransac", s);
    hipLaunchKernelGGL(k_fmat<true>, dim3(P), dim3(256), 0, s, d_pairs, d_kps, cap, d_good, d_ngood, nullptr, nullptr,
                       nullptr, 3.0, 0.999, 1000, d_F, nullptr, d_kept, d_nkept, d_err, d_diag);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int fmat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, double thr, double conf,
                int max_iters, double* d_F, uint8_t* d_mask, double* d_err, int* d_diag, hipStream_t s) {
    if (P <= 0) return VS_OK;
    ProfScope ps(ctx, "fmat_ransac", s);
    hipLaunchKernelGGL(k_fmat<false>, dim3(P), dim3(256), 0, s, nullptr, nullptr, 0, nullptr, nullptr, d_p1, d_p2,
                       d_off, thr, conf, max_iters, d_F, d_mask, nullptr, nullptr, d_err, d_diag);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
