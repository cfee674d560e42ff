// orc_ransac3d.cpp — CPU restatement of Slam::estimate_motion_3d3d (reference src/Slam.cpp:214-375).
// TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Literal at the algorithm level: round()-ed depth lookups and (0.1, 10] depth gate (:236-262),
// N >= 10 (:265), std::mt19937(seed) sampling with rejection (:276-283), centroid + 3x3
// cross-covariance + SVD + reflection fix + t = c2 - R c1 (:285-303), inlier count with
// ||P2 - (R P1 + t)|| < thr (:305-311), first strictly-better iteration wins (:313-317),
// >= 10 inliers (:320), refit over all inliers (:324-358), sanity gates (:361-372).
// cv::SVD::compute (external) is restated as a one-sided (Hestenes) Jacobi SVD in fp64 with
// singular values sorted descending and a null left vector completed by a cross product; R is
// unique for rank >= 2 cross-covariances, so any accurate SVD yields the same R up to rounding.
// cv::Mat expression rounding (MatExpr AddEx scaling) is unpinned; sums here run left to right.
#include "oracle.h"

#include <cmath>
#include <random>
#include <vector>

namespace {

struct V3 {
    double x, y, z;
};

// One-sided Jacobi SVD of a 3x3 matrix A (row-major): A = U diag(s) V^T, s descending.
void svd3(const double A[9], double U[9], double s[3], double V[9]) {
    double a[3][3];  // columns of A being orthogonalised: a[col][row]
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) a[c][r] = A[r * 3 + c];
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};  // v[col][row]
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int r = 0; r < 3; r++) {
                    alpha += a[p][r] * a[p][r];
                    beta += a[q][r] * a[q][r];
                    gamma += a[p][r] * a[q][r];
                }
                if (gamma == 0.0) continue;
                double conv = std::fabs(gamma) / std::sqrt(alpha * beta);
                if (!(conv > 1e-15)) continue;
                off = std::fmax(off, conv);
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
                for (int r = 0; r < 3; r++) {
                    double ap = a[p][r], aq = a[q][r];
                    a[p][r] = c * ap - sn * aq;
                    a[q][r] = sn * ap + c * aq;
                    double vp = v[p][r], vq = v[q][r];
                    v[p][r] = c * vp - sn * vq;
                    v[q][r] = sn * vp + c * vq;
                }
            }
        if (off <= 1e-15) break;
    }
    double sv[3];
    for (int c = 0; c < 3; c++) sv[c] = std::sqrt(a[c][0] * a[c][0] + a[c][1] * a[c][1] + a[c][2] * a[c][2]);
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
            if (sv[ord[j]] > sv[ord[i]]) { int tmp = ord[i]; ord[i] = ord[j]; ord[j] = tmp; }
    double u[3][3];
    for (int k = 0; k < 3; k++) {
        int c = ord[k];
        s[k] = sv[c];
        for (int r = 0; r < 3; r++) V[r * 3 + k] = v[c][r];
        if (sv[c] > 1e-300)
            for (int r = 0; r < 3; r++) u[k][r] = a[c][r] / sv[c];
        else
            for (int r = 0; r < 3; r++) u[k][r] = 0;
    }
    // Complete U when the smallest singular value vanishes (rank-2 H from 3 points).
    if (!(s[2] > 1e-12 * (s[0] > 0 ? s[0] : 1.0))) {
        u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
        u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
        u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
        double nn = std::sqrt(u[2][0] * u[2][0] + u[2][1] * u[2][1] + u[2][2] * u[2][2]);
        if (nn > 0) for (int r = 0; r < 3; r++) u[2][r] /= nn;
    }
    for (int k = 0; k < 3; k++)
        for (int r = 0; r < 3; r++) U[r * 3 + k] = u[k][r];
}

double det3(const double M[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// Kabsch from cross-covariance H = sum (P1-c1)(P2-c2)^T: R = V U^T with reflection fix.
void kabsch(const double H[9], double R[9]) {
    double U[9], s[3], V[9];
    svd3(H, U, s, V);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[i * 3 + j] = V[i * 3 + 0] * U[j * 3 + 0] + V[i * 3 + 1] * U[j * 3 + 1] + V[i * 3 + 2] * U[j * 3 + 2];
    if (det3(R) < 0) {
        for (int i = 0; i < 3; i++) V[i * 3 + 2] = -V[i * 3 + 2];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                R[i * 3 + j] = V[i * 3 + 0] * U[j * 3 + 0] + V[i * 3 + 1] * U[j * 3 + 1] + V[i * 3 + 2] * U[j * 3 + 2];
    }
}

bool is_inlier(const double R[9], const double t[3], const V3& p1, const V3& p2, double thr) {
    double qx = R[0] * p1.x + R[1] * p1.y + R[2] * p1.z + t[0];
    double qy = R[3] * p1.x + R[4] * p1.y + R[5] * p1.z + t[1];
    double qz = R[6] * p1.x + R[7] * p1.y + R[8] * p1.z + t[2];
    double dx = p2.x - qx, dy = p2.y - qy, dz = p2.z - qz;
    double ss = dx * dx;
    ss += dy * dy;
    ss += dz * dz;
    return std::sqrt(ss) < thr;
}

}  // namespace

extern "C" {

void orc_mt19937(uint32_t seed, int count, uint32_t* out) {
    std::mt19937 rng(seed);
    for (int i = 0; i < count; i++) out[i] = (uint32_t)rng();
}

int orc_ransac_3d3d(const float* pts1, const float* pts2, int n, const float* depth1,
                    const float* depth2, int h, int w, const double K[4], uint32_t seed, int iters,
                    double thr, double R_out[9], double t_out[3], int diag[4]) {
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    diag[0] = diag[1] = diag[2] = diag[3] = 0;
    diag[2] = -1;
    std::vector<V3> P1, P2;
    for (int i = 0; i < n; i++) {
        float x1 = pts1[2 * i], y1 = pts1[2 * i + 1], x2 = pts2[2 * i], y2 = pts2[2 * i + 1];
        int px1 = (int)std::round(x1), py1 = (int)std::round(y1);
        int px2 = (int)std::round(x2), py2 = (int)std::round(y2);
        if (px1 < 0 || px1 >= w || py1 < 0 || py1 >= h) continue;
        if (px2 < 0 || px2 >= w || py2 < 0 || py2 >= h) continue;
        float d1 = depth1[(size_t)py1 * w + px1], d2 = depth2[(size_t)py2 * w + px2];
        if (d1 <= 0.1f || d1 > 10.0f) continue;  // Config::DEPTH_MIN / DEPTH_MAX
        if (d2 <= 0.1f || d2 > 10.0f) continue;
        P1.push_back({(x1 - cx) * d1 / fx, (y1 - cy) * d1 / fy, (double)d1});
        P2.push_back({(x2 - cx) * d2 / fx, (y2 - cy) * d2 / fy, (double)d2});
    }
    const int N = (int)P1.size();
    diag[0] = N;
    if (N < 10) return 0;

    std::mt19937 rng(seed);
    int best_inliers = 0;
    double best_R[9] = {0}, best_t[3] = {0};
    for (int iter = 0; iter < iters; iter++) {
        int i0 = rng() % N;
        int i1, i2;
        do { i1 = rng() % N; } while (i1 == i0);
        do { i2 = rng() % N; } while (i2 == i0 || i2 == i1);
        const int id[3] = {i0, i1, i2};
        V3 c1 = {(P1[i0].x + P1[i1].x + P1[i2].x) / 3.0, (P1[i0].y + P1[i1].y + P1[i2].y) / 3.0,
                 (P1[i0].z + P1[i1].z + P1[i2].z) / 3.0};
        V3 c2 = {(P2[i0].x + P2[i1].x + P2[i2].x) / 3.0, (P2[i0].y + P2[i1].y + P2[i2].y) / 3.0,
                 (P2[i0].z + P2[i1].z + P2[i2].z) / 3.0};
        double H[9] = {0};
        for (int k = 0; k < 3; k++) {
            double a[3] = {P1[id[k]].x - c1.x, P1[id[k]].y - c1.y, P1[id[k]].z - c1.z};
            double b[3] = {P2[id[k]].x - c2.x, P2[id[k]].y - c2.y, P2[id[k]].z - c2.z};
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) H[r * 3 + c] += a[r] * b[c];
        }
        double R[9];
        kabsch(H, R);
        double t[3] = {c2.x - (R[0] * c1.x + R[1] * c1.y + R[2] * c1.z),
                       c2.y - (R[3] * c1.x + R[4] * c1.y + R[5] * c1.z),
                       c2.z - (R[6] * c1.x + R[7] * c1.y + R[8] * c1.z)};
        int inl = 0;
        for (int j = 0; j < N; j++) inl += is_inlier(R, t, P1[j], P2[j], thr);
        if (inl > best_inliers) {
            best_inliers = inl;
            for (int k = 0; k < 9; k++) best_R[k] = R[k];
            for (int k = 0; k < 3; k++) best_t[k] = t[k];
            diag[2] = iter;
        }
    }
    diag[1] = best_inliers;
    if (best_inliers < 10) return 0;

    V3 c1 = {0, 0, 0}, c2 = {0, 0, 0};
    std::vector<int> idx;
    for (int j = 0; j < N; j++)
        if (is_inlier(best_R, best_t, P1[j], P2[j], thr)) {
            c1.x += P1[j].x; c1.y += P1[j].y; c1.z += P1[j].z;
            c2.x += P2[j].x; c2.y += P2[j].y; c2.z += P2[j].z;
            idx.push_back(j);
        }
    const int cnt = (int)idx.size();
    diag[3] = cnt;
    c1.x /= cnt; c1.y /= cnt; c1.z /= cnt;
    c2.x /= cnt; c2.y /= cnt; c2.z /= cnt;
    double H[9] = {0};
    for (int j : idx) {
        double a[3] = {P1[j].x - c1.x, P1[j].y - c1.y, P1[j].z - c1.z};
        double b[3] = {P2[j].x - c2.x, P2[j].y - c2.y, P2[j].z - c2.z};
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) H[r * 3 + c] += a[r] * b[c];
    }
    kabsch(H, R_out);
    t_out[0] = c2.x - (R_out[0] * c1.x + R_out[1] * c1.y + R_out[2] * c1.z);
    t_out[1] = c2.y - (R_out[3] * c1.x + R_out[4] * c1.y + R_out[5] * c1.z);
    t_out[2] = c2.z - (R_out[6] * c1.x + R_out[7] * c1.y + R_out[8] * c1.z);
    double tn = std::sqrt(t_out[0] * t_out[0] + t_out[1] * t_out[1] + t_out[2] * t_out[2]);
    if (tn > 0.2) return 0;      // RANSAC_3D3D_MAX_TRANSLATION (Config.h:67)
    if (tn < 0.0001) return 0;
    if (std::fabs(det3(R_out) - 1.0) > 0.01) return 0;
    return 1;
}

}  // extern "C"
