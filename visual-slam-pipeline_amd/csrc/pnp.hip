// pnp.hip — Slam::solve_pnp (reference src/Slam.cpp:505-529: cv::solvePnPRansac, 8 px,
// confidence 0.99, then R_world = R_cam^T, t_world = -R_cam^T tvec) on gfx950.
//
// One workgroup (4 wave64s) per PnP problem; a batch of problems (frames, or the periodic /
// recovery / loop callers) is one grid.  The OpenCV RANSAC loop is sequential only through its
// adaptive iteration budget, and that budget only shrinks, so the workgroup
//   1. draws every subset of the initial budget with the cv::RNG stream (lane 0; the stream does
//      not depend on the models because checkSubset is trivially true for PnP),
//   2. solves the EPnP hypotheses and counts their inliers in parallel, one hypothesis per lane,
//   3. replays the accept / RANSACUpdateNumIters sequence on lane 0 over the counts — exactly
//      the hypotheses the sequential loop would have evaluated, in its order,
//   4. re-solves the winning subset, marks the inliers, and refines (rvec, tvec) with the LM of
//      pnp_solvers.h, the 28 normal-equation sums reduced deterministically over the lanes.
// Numerical kernels are shared with the CPU restatement (pnp_solvers.h; this file is built
// with -ffp-contract=off like the oracle).
#include <hip/hip_runtime.h>

#include "block_reduce.h"
#include "pnp_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_pnp;

constexpr int kPnpMaxIters = VS_PNP_MAX_ITERS;

struct PnpShared {
    int subset[kPnpMaxIters * 5];
    int count[kPnpMaxIters];  // -1: EPnP failed on the subset
    double red[4 * kLmTerms];
    LmState lm;
    double rv[3], tv[3];
    int best, best_iter, niters_run, go;
};

__device__ inline bool epnp_subset(const float* obj, const float* img, const int* idx, int m, const Cam& K, double* rv,
                                   double* tv) {
    double X[15], uv[10];
    for (int j = 0; j < m; j++) {
        const int i = idx[j];
        X[3 * j] = obj[3 * i];
        X[3 * j + 1] = obj[3 * i + 1];
        X[3 * j + 2] = obj[3 * i + 2];
        uv[2 * j] = img[2 * i];
        uv[2 * j + 1] = img[2 * i + 1];
    }
    double R[9], t[3];
    if (!epnp<5>(X, uv, m, K, R, t)) return false;
    rod_m2v(R, rv);
    for (int k = 0; k < 3; k++) tv[k] = t[k];
    return true;
}

// stat[p][8] = {success, inliers, ransac iterations, best iteration, lm iterations, lm accepted, n, 0}
__global__ __launch_bounds__(256) void k_pnp_ransac(const float* __restrict__ obj_all, const float* __restrict__ img_all,
                                                    const int* __restrict__ off, double fx, double fy, double cx,
                                                    double cy, int max_iters, float thr2, double conf,
                                                    int min_inliers, double* __restrict__ Rw, double* __restrict__ tw,
                                                    int* __restrict__ stat, uint8_t* __restrict__ mask_all) {
    __shared__ PnpShared S;
    const int pb = blockIdx.x, tid = threadIdx.x;
    const int o0 = off[pb], n = off[pb + 1] - o0;
    const float* obj = obj_all + 3 * (size_t)o0;
    const float* img = img_all + 2 * (size_t)o0;
    uint8_t* mask = mask_all + o0;
    const Cam K{fx, fy, cx, cy};
    int* st = stat + 8 * pb;
    for (int i = tid; i < n; i += blockDim.x) mask[i] = 0;
    if (tid == 0)
        for (int k = 0; k < 8; k++) st[k] = 0;
    if (tid == 0) st[6] = n;
    if (n < min_inliers || n < 4) return;  // Slam.cpp:512; OpenCV needs >= 4 points
    const int model_points = n == 4 ? 4 : 5;
    const int niters0 = max_iters > 1 ? max_iters : 1;

    if (n == model_points) {  // OpenCV: a single EPnP on all points, every point an inlier
        if (tid == 0) {
            int idx[5] = {0, 1, 2, 3, 4};
            const bool ok = epnp_subset(obj, img, idx, n, K, S.rv, S.tv);
            S.best = ok ? n : 0;
            S.best_iter = -1;
            S.niters_run = 0;
        }
        __syncthreads();
        if (S.best == 0) return;
        for (int i = tid; i < n; i += blockDim.x) mask[i] = 1;
        if (tid == 0) {  // no refinement on this path
            for (int k = 0; k < 3; k++) {
                S.lm.p[k] = S.rv[k];
                S.lm.p[3 + k] = S.tv[k];
            }
            S.lm.iters = S.lm.accepted = 0;
        }
    } else {
        // 1. subsets (cv::RNG, getSubset)
        if (tid == 0) {
            CvRng rng((uint64_t)-1);
            for (int it = 0; it < niters0; it++) {
                int* idx = S.subset + 5 * it;
                for (int i = 0; i < model_points; i++)
                    for (;;) {
                        idx[i] = rng.uniform(0, n);
                        int j = 0;
                        while (j < i && idx[j] != idx[i]) j++;
                        if (j == i) break;
                    }
            }
        }
        __syncthreads();
        // 2. hypotheses in parallel
        for (int h = tid; h < niters0; h += blockDim.x) {
            double rv[3], tv[3];
            int cnt = -1;
            if (epnp_subset(obj, img, S.subset + 5 * h, model_points, K, rv, tv)) {
                double R[9];
                rod_v2m(rv, R);
                cnt = 0;
                for (int i = 0; i < n; i++)
                    cnt += reproj_err2(R, tv, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i],
                                       img[2 * i + 1]) <= thr2;
            }
            S.count[h] = cnt;
        }
        __syncthreads();
        // 3. sequential replay of the accept / update rule
        if (tid == 0) {
            int niters = niters0, best = 0, best_iter = -1, it = 0;
            for (; it < niters; it++) {
                const int c = S.count[it];
                if (c < 0) continue;
                if (c > (best > model_points - 1 ? best : model_points - 1)) {
                    best = c;
                    best_iter = it;
                    niters = ransac_update_num_iters(conf, (double)(n - c) / n, model_points, niters);
                }
            }
            S.best = best;
            S.best_iter = best_iter;
            S.niters_run = it;
            if (best > 0) epnp_subset(obj, img, S.subset + 5 * best_iter, model_points, K, S.rv, S.tv);
        }
        __syncthreads();
        if (tid == 0) {
            st[2] = S.niters_run;
            st[3] = S.best_iter;
        }
        if (S.best <= 0) return;
        // 4. inliers of the winning model, then LM on them
        double R[9];
        const double rv0[3] = {S.rv[0], S.rv[1], S.rv[2]}, tv0[3] = {S.tv[0], S.tv[1], S.tv[2]};
        rod_v2m(rv0, R);
        for (int i = tid; i < n; i += blockDim.x)
            mask[i] = reproj_err2(R, tv0, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1]) <=
                      thr2;
        // (each lane re-reads only the mask entries it wrote itself)
        // Thread 0 owns S.lm; block_sum's barriers order its updates after every lane has read
        // the previous candidate.
        double p[6] = {rv0[0], rv0[1], rv0[2], tv0[0], tv0[1], tv0[2]};
        for (bool first = true;; first = false) {
            LmRots L;
            lm_rotations(p, L);
            double acc[kLmTerms], tot[kLmTerms];
            for (int k = 0; k < kLmTerms; k++) acc[k] = 0;
            for (int i = tid; i < n; i += blockDim.x)
                if (mask[i])
                    lm_point(L, p + 3, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1], acc);
            block_sum<kLmTerms>(acc, S.red, tot);
            if (tid == 0) {
                if (first)
                    S.lm.init(p, tot);
                else
                    S.lm.accept_or_reject(tot);
                S.go = S.lm.step();
            }
            __syncthreads();
            if (!S.go) break;
            for (int k = 0; k < 6; k++) p[k] = S.lm.cand[k];
        }
    }
    // outputs: Slam.cpp:519-526
    if (tid == 0) {
        const int inl = S.best;
        st[1] = inl;
        st[4] = S.lm.iters;
        st[5] = S.lm.accepted;
        const int success = inl >= min_inliers;
        st[0] = success;
        if (success) {
            const double rv[3] = {S.lm.p[0], S.lm.p[1], S.lm.p[2]};
            double Rc[9];
            rod_v2m(rv, Rc);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) Rw[9 * pb + i * 3 + j] = Rc[j * 3 + i];
            for (int i = 0; i < 3; i++)
                tw[3 * pb + i] =
                    -(Rc[0 * 3 + i] * S.lm.p[3] + Rc[1 * 3 + i] * S.lm.p[4] + Rc[2 * 3 + i] * S.lm.p[5]);
        }
    }
}

int solve_pnp(vs_ctx* ctx, int nprob, const float* d_obj, const float* d_img, const int* d_off, const double K[4],
              int ransac_iters, int min_inliers, double* d_R, double* d_t, int* d_stat, uint8_t* d_mask,
              hipStream_t s) {
    if (nprob <= 0) return VS_OK;
    VS_ARG(ransac_iters <= kPnpMaxIters, "solve_pnp: ransac_iters above kPnpMaxIters");
    ProfScope ps(ctx, "solve_pnp", s);
    const float thr = (float)8.0;  // Config::PNP_RANSAC_THRESHOLD passed as float (Slam.cpp:517)
    const float thr2 = (float)((double)thr * (double)thr);
    hipLaunchKernelGGL(k_pnp_ransac, dim3(nprob), dim3(256), 0, s, d_obj, d_img, d_off, K[0], K[1], K[2], K[3],
                       ransac_iters, thr2, 0.99, min_inliers, d_R, d_t, d_stat, d_mask);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
