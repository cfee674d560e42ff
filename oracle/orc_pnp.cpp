// orc_pnp.cpp — CPU restatement of Slam::solve_pnp (reference src/Slam.cpp:505-529), i.e.
// cv::solvePnPRansac(obj, img, K, no distortion, useExtrinsicGuess = false, iters,
// (float)PNP_RANSAC_THRESHOLD = 8 px (include/Config.h:78), confidence 0.99) followed by the
// camera -> world conversion.  TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// OpenCV 4.x (external, unpinned) is restated from its published algorithm:
//   * n == model points (5, or 4 for n == 4): one EPnP solve on all points, all inliers;
//   * otherwise RANSACPointSetRegistrator::run — cv::RNG((uint64)-1), getSubset drawing
//     rng.uniform(0, n) with repeats rejected, EPnP on the subset (model stored as
//     Rodrigues(R), tvec), PnPRansacCallback::computeError (float squared reprojection error
//     against projectPoints' float output), inlier iff err <= (float)(thr * thr), the model wins
//     when its count exceeds max(best, modelPoints - 1), then
//     niters = RANSACUpdateNumIters(conf, (n - count) / n, modelPoints, niters);
//   * refinement: solvePnP(SOLVEPNP_ITERATIVE, useExtrinsicGuess = true) on the RANSAC inliers,
//     restated as the LM of pnp_solvers.h;  inliers reported are the RANSAC inliers.
// The numerical kernels (EPnP, LM terms, Rodrigues, RNG) come from the product's host/device
// header so that the oracle checks the device RANSAC driver, scoring and reductions; EPnP/LM
// themselves are pinned by known-answer tests (tests/test_oracle_pnp.py).
#include <cstring>
#include <vector>

#include "../visual-slam-pipeline_amd/csrc/pnp_solvers.h"
#include "oracle.h"

using namespace vs_pnp;

namespace {

void model_rt(const double* rv, const double* tv, double* R, double* t) {
    rod_v2m(rv, R);
    for (int k = 0; k < 3; k++) t[k] = tv[k];
}

// The LM sums in the device's order (pnp.hip k_pnp_ransac: lane t of 256 accumulates the inliers
// i = t mod 256 in index order; block_sum: xor butterfly inside each wave64, then waves 0..3 in
// order), so the accept / stop decisions, which compare costs at rounding level near convergence,
// are bit-identical.  OpenCV's own summation order (cvCalcMatMulDeriv + gemm) is unpinned either way.
void lm_eval(const float* obj, const float* img, const std::vector<int>& idx, const Cam& K, const double* p,
             double* acc) {
    constexpr int kLanes = 256;
    LmRots L;
    lm_rotations(p, L);
    std::vector<double> part((size_t)kLanes * kLmTerms, 0.0);
    for (int i : idx)
        lm_point(L, p + 3, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1],
                 &part[(size_t)(i % kLanes) * kLmTerms]);
    for (int k = 0; k < kLmTerms; k++) {
        double wsum[kLanes / 64];
        for (int w = 0; w < kLanes / 64; w++) {
            double v[64], nv[64];
            for (int l = 0; l < 64; l++) v[l] = part[(size_t)(64 * w + l) * kLmTerms + k];
            for (int o = 32; o > 0; o >>= 1) {
                for (int l = 0; l < 64; l++) nv[l] = v[l] + v[l ^ o];
                for (int l = 0; l < 64; l++) v[l] = nv[l];
            }
            wsum[w] = v[0];
        }
        double sacc = wsum[0];
        for (int w = 1; w < kLanes / 64; w++) sacc += wsum[w];
        acc[k] = sacc;
    }
}

bool epnp_on(const float* obj, const float* img, const int* idx, int m, const Cam& K, double* rv, double* tv) {
    std::vector<double> X(3 * m), uv(2 * m);
    for (int j = 0; j < m; j++) {
        const int i = idx ? idx[j] : j;
        for (int c = 0; c < 3; c++) X[3 * j + c] = obj[3 * i + c];
        uv[2 * j] = img[2 * i];
        uv[2 * j + 1] = img[2 * i + 1];
    }
    double R[9], t[3];
    if (!epnp<8>(X.data(), uv.data(), m, K, R, t)) return false;
    rod_m2v(R, rv);
    for (int k = 0; k < 3; k++) tv[k] = t[k];
    return true;
}

}  // namespace

extern "C" int orc_epnp(const double* X, const double* uv, int n, const double K[4], double R[9], double t[3]) {
    const Cam cam{K[0], K[1], K[2], K[3]};
    if (n > 4096) return 0;
    return epnp<4096>(X, uv, n, cam, R, t) ? 1 : 0;
}

// the stage results of epnp_small_eig (216 doubles per problem, pnp_solvers.h dbg layout), as the
// device's vs_debug_epnp_mode(3) dumps them
extern "C" int orc_epnp_eig_stages(const double* X, const double* uv, const int* m, int count, const double K[4],
                                   double* out) {
    const Cam cam{K[0], K[1], K[2], K[3]};
    for (int p = 0; p < count; p++) {
        double* o = out + (size_t)p * 216;
        for (int k = 0; k < 216; k++) o[k] = 0.0;
        double cw[4][3], al[5][4], v[4][12];
        if (m[p] >= 4 && m[p] <= 5 && epnp_control<5>(X + 15 * p, m[p], cw, al)) epnp_small_eig(al, uv + 10 * p, m[p], cam, v, o);
    }
    return 0;
}

// test hook mirroring the device's vs_debug_epnp (pnp.hip): per problem (v[4][12] of
// epnp_small_eig, R[9], t[3], ok, rod_m2v(R)[3], rod_v2m of it[9]) for m = 4 / 5 points
extern "C" int orc_epnp_debug(const double* X, const double* uv, const int* m, int count, const double K[4],
                              double* out) {
    const Cam cam{K[0], K[1], K[2], K[3]};
    for (int p = 0; p < count; p++) {
        double* o = out + (size_t)p * 73;
        double cw[4][3], al[5][4], v[4][12], R[9] = {}, t[3] = {};
        bool ok = m[p] >= 4 && m[p] <= 5 && epnp_control<5>(X + 15 * p, m[p], cw, al);
        if (ok) epnp_small_eig(al, uv + 10 * p, m[p], cam, v);
        for (int k = 0; k < 48; k++) o[k] = ok ? v[k / 12][k % 12] : 0.0;
        ok = ok && epnp<5>(X + 15 * p, uv + 10 * p, m[p], cam, R, t);
        for (int k = 0; k < 9; k++) o[48 + k] = R[k];
        for (int k = 0; k < 3; k++) o[57 + k] = t[k];
        o[60] = ok ? 1.0 : 0.0;
        double rv[3], R2[9];
        rod_m2v(R, rv);
        rod_v2m(rv, R2);
        for (int k = 0; k < 3; k++) o[61 + k] = rv[k];
        for (int k = 0; k < 9; k++) o[64 + k] = R2[k];
    }
    return 0;
}

extern "C" int orc_pnp_ransac(const float* obj, const float* img, int n, const double K[4], int max_iters,
                              double thr, double conf, double rvec[3], double tvec[3], uint8_t* mask,
                              int* n_inliers, int diag[4]) {
    const Cam cam{K[0], K[1], K[2], K[3]};
    if (diag) diag[0] = diag[1] = diag[2] = diag[3] = 0;
    *n_inliers = 0;
    if (n < 4) return 0;
    const int model_points = n == 4 ? 4 : 5;
    if (n == model_points) {
        if (!epnp_on(obj, img, nullptr, n, cam, rvec, tvec)) return 0;
        if (mask) memset(mask, 1, n);
        *n_inliers = n;
        return 1;
    }
    CvRng rng((uint64_t)-1);
    int niters = max_iters > 1 ? max_iters : 1, best = 0, best_iter = -1;
    double best_rv[3] = {0, 0, 0}, best_tv[3] = {0, 0, 0};
    const float thr2 = (float)(thr * thr);
    int iter = 0;
    for (; iter < niters; iter++) {
        int idx[5];
        for (int i = 0; i < model_points; i++) {  // getSubset (checkSubset is always true for PnP)
            for (;;) {
                idx[i] = rng.uniform(0, n);
                int j = 0;
                while (j < i && idx[j] != idx[i]) j++;
                if (j == i) break;
            }
        }
        double rv[3], tv[3];
        if (!epnp_on(obj, img, idx, model_points, cam, rv, tv)) continue;
        double R[9], t[3];
        model_rt(rv, tv, R, t);
        int cnt = 0;
        for (int i = 0; i < n; i++)
            cnt += reproj_err2(R, t, cam, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1]) <=
                   thr2;
        if (cnt > (best > model_points - 1 ? best : model_points - 1)) {
            best = cnt;
            best_iter = iter;
            for (int k = 0; k < 3; k++) {
                best_rv[k] = rv[k];
                best_tv[k] = tv[k];
            }
            niters = ransac_update_num_iters(conf, (double)(n - cnt) / n, model_points, niters);
        }
    }
    if (diag) {
        diag[0] = iter;
        diag[1] = best_iter;
    }
    if (best <= 0) return 0;
    double R[9], t[3];
    model_rt(best_rv, best_tv, R, t);
    std::vector<int> inl;
    for (int i = 0; i < n; i++) {
        const bool in =
            reproj_err2(R, t, cam, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1]) <= thr2;
        if (mask) mask[i] = in;
        if (in) inl.push_back(i);
    }
    // refinement on the inliers from the RANSAC model
    double p0[6] = {best_rv[0], best_rv[1], best_rv[2], best_tv[0], best_tv[1], best_tv[2]};
    double acc[kLmTerms];
    lm_eval(obj, img, inl, cam, p0, acc);
    LmState S;
    S.init(p0, acc);
    while (S.step()) {
        lm_eval(obj, img, inl, cam, S.cand, acc);
        S.accept_or_reject(acc);
    }
    for (int k = 0; k < 3; k++) {
        rvec[k] = S.p[k];
        tvec[k] = S.p[3 + k];
    }
    if (diag) {
        diag[2] = S.iters;
        diag[3] = S.accepted;
    }
    *n_inliers = best;
    return 1;
}

// Slam::solve_pnp (Slam.cpp:505-529)
extern "C" int orc_solve_pnp(const float* obj, const float* img, int n, const double K[4], int ransac_iters,
                             int min_inliers, double R_world[9], double t_world[3], int* inlier_count) {
    *inlier_count = 0;
    if (n < min_inliers) return 0;  // :512
    double rv[3], tv[3];
    int inl = 0;
    const int ok = orc_pnp_ransac(obj, img, n, K, ransac_iters, (double)(float)8.0, 0.99, rv, tv, nullptr, &inl,
                                  nullptr);
    if (!ok || inl < min_inliers) return 0;  // :519
    double Rc[9];
    rod_v2m(rv, Rc);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R_world[i * 3 + j] = Rc[j * 3 + i];  // R_cam^T (:524)
    for (int i = 0; i < 3; i++)
        t_world[i] = -(Rc[0 * 3 + i] * tv[0] + Rc[1 * 3 + i] * tv[1] + Rc[2 * 3 + i] * tv[2]);  // :525
    *inlier_count = inl;
    return 1;
}
