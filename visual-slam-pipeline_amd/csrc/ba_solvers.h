// ba_solvers.h — host/device arithmetic of Optimizer::local_bundle_adjustment (reference
// src/Optimizer.cpp:187-599), shared by the CPU restatement (oracle/orc_ba.cpp) and the kernels
// (ba.hip) so both evaluate every element with the same operations in the same order:
//   * ba_obs_terms      one observation's Huber-weighted Jacobians and residual (:331-405):
//                       analytic point / translation blocks, forward-difference rotation block
//                       (eps 1e-6 on the Rodrigues vector), weight w = min(1, 5 / |r|), sqrt(w)
//                       scaling;
//   * ba_add_pose/point/cross   the Hpp, bp, Hmm, bm and Hpm accumulations (:407-451);
//   * ba_point_inverse  Hmm * diag(1 + lambda), |det| < 1e-20 -> skipped, else the Cholesky
//                       inverse (cv::invert DECOMP_CHOLESKY) (:478-493);
//   * ba_schur_*        U = Hpm Hinv, S -= U Hpm^T, b -= U bm, dm = Hinv (-bm - Hpm^T dp)
//                       (:495-539), products summed over k in ascending order.
#pragma once

#include "pnp_solvers.h"  // VS_HD, Rodrigues

namespace vs_ba {

constexpr double kHuber = 5.0;       // HUBER_DELTA (:192)
constexpr double kRotEps = 1e-6;     // numeric rotation Jacobian step (:382)
constexpr double kPoseDamp = 1e10;   // Hpp += 1e10 I (:454-458)
constexpr int kMaxIter = 15;         // MAX_ITER (:294)
constexpr int kCostChunk = 256;      // fixed chunking of the global cost sums (see orc_ba.cpp)

struct Cam {
    double fx, fy, cx, cy;
};

// pose cache: R = Rodrigues(rvec) (camera -> world), t, and the three rotation-perturbed R's
struct PoseC {
    double R[9], t[3], Rp[3][9];
};

VS_HD inline void pose_cache(const double* rvec, const double* tvec, PoseC& p) {
    vs_pnp::rod_v2m(rvec, p.R);
    for (int k = 0; k < 3; k++) p.t[k] = tvec[k];
    for (int d = 0; d < 3; d++) {
        double rp[3] = {rvec[0], rvec[1], rvec[2]};
        rp[d] += kRotEps;
        vs_pnp::rod_v2m(rp, p.Rp[d]);
    }
}

struct ObsTerms {
    int valid;
    double Jp[2][6], Jm[2][3];
    double ru_w, rv_w, cost;
};

// :331-405 (the per-observation body of the accumulation loop)
VS_HD inline void ba_obs_terms(const PoseC& pc, const double* P, double obs_u, double obs_v, const Cam& K,
                               ObsTerms& o) {
    const double* Rd = pc.R;
    const double* td = pc.t;
    const double dx_ = P[0] - td[0], dy_ = P[1] - td[1], dz_ = P[2] - td[2];
    const double X = Rd[0] * dx_ + Rd[3] * dy_ + Rd[6] * dz_;
    const double Y = Rd[1] * dx_ + Rd[4] * dy_ + Rd[7] * dz_;
    const double Z = Rd[2] * dx_ + Rd[5] * dy_ + Rd[8] * dz_;
    if (Z < 1e-6) {
        o.valid = 0;
        return;
    }
    o.valid = 1;
    const double inv_z = 1.0 / Z;
    const double inv_z2 = inv_z * inv_z;
    const double u_proj = K.fx * X * inv_z + K.cx;
    const double v_proj = K.fy * Y * inv_z + K.cy;
    const double ru = u_proj - obs_u, rv = v_proj - obs_v;
    const double r_norm = sqrt(ru * ru + rv * rv);
    double w = 1.0;
    if (r_norm > kHuber) w = kHuber / r_norm;
    const double sw = sqrt(w);
    o.cost = w * (ru * ru + rv * rv);
    o.ru_w = ru * sw;
    o.rv_w = rv * sw;
    const double dp00 = K.fx * inv_z, dp02 = -K.fx * X * inv_z2;
    const double dp11 = K.fy * inv_z, dp12 = -K.fy * Y * inv_z2;
    for (int c = 0; c < 3; c++) {
        const double rc0 = Rd[c * 3 + 0], rc1 = Rd[c * 3 + 1], rc2 = Rd[c * 3 + 2];
        o.Jm[0][c] = (dp00 * rc0 + dp02 * rc2) * sw;
        o.Jm[1][c] = (dp11 * rc1 + dp12 * rc2) * sw;
    }
    for (int d = 0; d < 3; d++) {
        const double* Rp = pc.Rp[d];
        const double Xp = Rp[0] * dx_ + Rp[3] * dy_ + Rp[6] * dz_;
        const double Yp = Rp[1] * dx_ + Rp[4] * dy_ + Rp[7] * dz_;
        const double Zp = Rp[2] * dx_ + Rp[5] * dy_ + Rp[8] * dz_;
        if (Zp < 1e-6) {
            o.Jp[0][d] = 0;
            o.Jp[1][d] = 0;
            continue;
        }
        const double up = K.fx * Xp / Zp + K.cx;
        const double vp = K.fy * Yp / Zp + K.cy;
        o.Jp[0][d] = (up - u_proj) / kRotEps * sw;
        o.Jp[1][d] = (vp - v_proj) / kRotEps * sw;
    }
    for (int c = 0; c < 3; c++) {
        o.Jp[0][c + 3] = -o.Jm[0][c];
        o.Jp[1][c + 3] = -o.Jm[1][c];
    }
}

// Hpp (6x6, both triangles as the reference writes them) and bp
VS_HD inline void ba_add_pose(const ObsTerms& o, double* H, double* b) {
    for (int r = 0; r < 6; r++)
        for (int c = r; c < 6; c++) {
            const double val = o.Jp[0][r] * o.Jp[0][c] + o.Jp[1][r] * o.Jp[1][c];
            H[r * 6 + c] += val;
            if (r != c) H[c * 6 + r] += val;
        }
    for (int r = 0; r < 6; r++) b[r] += o.Jp[0][r] * o.ru_w + o.Jp[1][r] * o.rv_w;
}

// Hmm (3x3) and bm
VS_HD inline void ba_add_point(const ObsTerms& o, double* H, double* b) {
    for (int r = 0; r < 3; r++)
        for (int c = r; c < 3; c++) {
            const double val = o.Jm[0][r] * o.Jm[0][c] + o.Jm[1][r] * o.Jm[1][c];
            H[r * 3 + c] += val;
            if (r != c) H[c * 3 + r] += val;
        }
    for (int r = 0; r < 3; r++) b[r] += o.Jm[0][r] * o.ru_w + o.Jm[1][r] * o.rv_w;
}

// Hpm (6x3) for the (keyframe, point) pair
VS_HD inline void ba_add_cross(const ObsTerms& o, double* Hpm) {
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 3; c++) Hpm[r * 3 + c] += o.Jp[0][r] * o.Jm[0][c] + o.Jp[1][r] * o.Jm[1][c];
}

// Hmm_d = Hmm * diag(1 + lambda); returns false (Hinv = 0) when |det| < 1e-20 or not SPD.
VS_HD inline bool ba_point_inverse(const double* Hmm, double lambda, double* Hinv) {
    double A[9];
    for (int i = 0; i < 9; i++) A[i] = Hmm[i];
    for (int d = 0; d < 3; d++) A[d * 3 + d] *= (1.0 + lambda);
    const double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                       A[2] * (A[3] * A[7] - A[4] * A[6]);
    for (int i = 0; i < 9; i++) Hinv[i] = 0;
    if (fabs(det) < 1e-20) return false;
    double L[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < 3; j++) {
        double s = A[j * 3 + j];
        for (int k = 0; k < j; k++) s -= L[j * 3 + k] * L[j * 3 + k];
        if (!(s > 0)) return false;
        L[j * 3 + j] = sqrt(s);
        for (int i = j + 1; i < 3; i++) {
            double v = A[i * 3 + j];
            for (int k = 0; k < j; k++) v -= L[i * 3 + k] * L[j * 3 + k];
            L[i * 3 + j] = v / L[j * 3 + j];
        }
    }
    for (int c = 0; c < 3; c++) {  // solve L L^T x = e_c
        double y[3];
        for (int i = 0; i < 3; i++) {
            double v = (i == c) ? 1.0 : 0.0;
            for (int k = 0; k < i; k++) v -= L[i * 3 + k] * y[k];
            y[i] = v / L[i * 3 + i];
        }
        for (int i = 2; i >= 0; i--) {
            double v = y[i];
            for (int k = i + 1; k < 3; k++) v -= L[k * 3 + i] * Hinv[k * 3 + c];
            Hinv[i * 3 + c] = v / L[i * 3 + i];
        }
    }
    return true;
}

// U = Hpm (6x3) * Hinv (3x3)
VS_HD inline void ba_schur_u(const double* Hpm, const double* Hinv, double* U) {
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 3; c++)
            U[r * 3 + c] = Hpm[r * 3 + 0] * Hinv[0 * 3 + c] + Hpm[r * 3 + 1] * Hinv[1 * 3 + c] +
                           Hpm[r * 3 + 2] * Hinv[2 * 3 + c];
}

// one element of S_contrib = U_a (6x3) * Hpm_b^T (3x6)
VS_HD inline double ba_schur_s(const double* Ua, const double* Hpm_b, int r, int c) {
    return Ua[r * 3 + 0] * Hpm_b[c * 3 + 0] + Ua[r * 3 + 1] * Hpm_b[c * 3 + 1] + Ua[r * 3 + 2] * Hpm_b[c * 3 + 2];
}

// one element of bp_contrib = U_a (6x3) * bm (3)
VS_HD inline double ba_schur_b(const double* Ua, const double* bm, int r) {
    return Ua[r * 3 + 0] * bm[0] + Ua[r * 3 + 1] * bm[1] + Ua[r * 3 + 2] * bm[2];
}

// rhs -= Hpm^T (3x6) dp_k (6)
VS_HD inline void ba_backsub_add(const double* Hpm, const double* dpk, double* rhs) {
    for (int c = 0; c < 3; c++) {
        double s = 0;
        for (int r = 0; r < 6; r++) s += Hpm[r * 3 + c] * dpk[r];
        rhs[c] -= s;
    }
}

// project_fn (:276-290): (-1, -1) when behind the camera
VS_HD inline bool ba_project(const PoseC& pc, const double* P, const Cam& K, double& u, double& v) {
    const double* Rd = pc.R;
    const double px = P[0] - pc.t[0], py = P[1] - pc.t[1], pz = P[2] - pc.t[2];
    const double X = Rd[0] * px + Rd[3] * py + Rd[6] * pz;
    const double Y = Rd[1] * px + Rd[4] * py + Rd[7] * pz;
    const double Z = Rd[2] * px + Rd[5] * py + Rd[8] * pz;
    if (Z < 1e-6) {
        u = v = -1;
        return false;
    }
    u = K.fx * X / Z + K.cx;
    v = K.fy * Y / Z + K.cy;
    return true;
}

// new_cost term (:547-556): +100 behind the camera, Huber-weighted squared residual otherwise
VS_HD inline double ba_new_cost_term(const PoseC& pc, const double* P, double obs_u, double obs_v, const Cam& K) {
    double u, v;
    ba_project(pc, P, K, u, v);
    if (u < 0) return 100.0;
    const double du = u - obs_u, dv = v - obs_v;
    const double rn = sqrt(du * du + dv * dv);
    const double w = (rn > kHuber) ? kHuber / rn : 1.0;
    return w * (du * du + dv * dv);
}

// error_before / error_after term (:263-268, 571-576): skipped when the projection has u < 0
VS_HD inline double ba_sq_err_term(const PoseC& pc, const double* P, double obs_u, double obs_v, const Cam& K) {
    double u, v;
    ba_project(pc, P, K, u, v);
    if (u < 0) return 0.0;
    const double dx = u - obs_u, dy = v - obs_v;
    return dx * dx + dy * dy;
}

}  // namespace vs_ba
