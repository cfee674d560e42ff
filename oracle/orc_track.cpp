// orc_track.cpp — CPU restatement of Slam::track_local_map (reference src/Slam.cpp:380-469).
// TEST INFRASTRUCTURE ONLY (see oracle.h).
//
// Literal: 30-px keypoint grid of 22 x 16 cells filled in keypoint order (:388-401); world->camera
// transform R_cam = R^T, t_cam = -R_cam t (:403-406); every valid map point with a descriptor
// (:416-418) projected with the Config intrinsics, rejected outside z in [0.1f, 50] or the image
// (:420-431); cells within +-12 px (:434-438), keypoints within 12 px (:445-447), the first
// strictly smaller L2 descriptor distance below 0.5 wins (:449-455); the keypoint takes the map
// point if that distance beats its best so far (:460-465).
// cv::norm(a, b, NORM_L2) on float rows (external, OpenCV 4.x normL2Sqr<float, double>): per
// element (double)(a - b) with the difference in float, squares summed in double in groups of
// four ((v0^2 + v1^2) + v2^2) + v3^2 added to the running sum, then sqrt.
#include <cmath>
#include <vector>

#include "oracle.h"

namespace {

double desc_l2(const float* a, const float* b) {
    double s = 0;
    for (int k = 0; k < 256; k += 4) {
        double v0 = (double)(a[k] - b[k]), v1 = (double)(a[k + 1] - b[k + 1]);
        double v2 = (double)(a[k + 2] - b[k + 2]), v3 = (double)(a[k + 3] - b[k + 3]);
        s += v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
    }
    return std::sqrt(s);
}

}  // namespace

extern "C" {

int orc_track_local_map(const double* mp_pos, const float* mp_desc, const uint8_t* mp_valid, int n_mp,
                        const orc_keypoint* kps, const float* descs, int nkp, const double R[9],
                        const double t[3], const double K[4], int img_w, int img_h, int* kp_to_mp,
                        int* obs_mp, int* obs_kp, int obs_cap, int* n_obs) {
    *n_obs = 0;
    if (nkp <= 0) return 0;
    const int CELL = 30;  // TRACK_GRID_CELL_SIZE (Config.h:108)
    const int GW = (img_w + CELL - 1) / CELL, GH = (img_h + CELL - 1) / CELL;
    std::vector<std::vector<int>> grid(GW * GH);
    for (int ki = 0; ki < nkp; ki++) {
        int gx = std::min((int)(kps[ki].x / CELL), GW - 1);
        int gy = std::min((int)(kps[ki].y / CELL), GH - 1);
        if (gx >= 0 && gy >= 0) grid[gy * GW + gx].push_back(ki);
    }
    std::vector<double> best_desc_dist(nkp, 1e9);
    double Rc[9], tc[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Rc[i * 3 + j] = R[j * 3 + i];
    for (int i = 0; i < 3; i++) tc[i] = -(Rc[i * 3 + 0] * t[0] + Rc[i * 3 + 1] * t[1] + Rc[i * 3 + 2] * t[2]);
    const double SR = 12.0, SR2 = SR * SR, THR = 0.5;  // TRACK_SEARCH_RADIUS, TRACK_DESC_THRESHOLD
    int tracked = 0;
    for (int mp = 0; mp < n_mp; mp++) {
        if (!mp_valid[mp]) continue;
        const double x = mp_pos[3 * mp], y = mp_pos[3 * mp + 1], z = mp_pos[3 * mp + 2];
        double px = Rc[0] * x + Rc[1] * y + Rc[2] * z + tc[0];
        double py = Rc[3] * x + Rc[4] * y + Rc[5] * z + tc[1];
        double pz = Rc[6] * x + Rc[7] * y + Rc[8] * z + tc[2];
        if (pz < 0.1f || pz > 50.0) continue;  // DEPTH_MIN (float), TRIANG_MAX_DEPTH
        double u = K[0] * px / pz + K[2];
        double v = K[1] * py / pz + K[3];
        if (u < 0 || u >= img_w || v < 0 || v >= img_h) continue;
        int gx0 = std::max(0, (int)((u - SR) / CELL));
        int gy0 = std::max(0, (int)((v - SR) / CELL));
        int gx1 = std::min(GW - 1, (int)((u + SR) / CELL));
        int gy1 = std::min(GH - 1, (int)((v + SR) / CELL));
        int best_ki = -1;
        double best_dist = THR;
        const float* md = mp_desc + (size_t)mp * 256;
        for (int gy = gy0; gy <= gy1; gy++)
            for (int gx = gx0; gx <= gx1; gx++)
                for (int ki : grid[gy * GW + gx]) {
                    double dx = u - kps[ki].x, dy = v - kps[ki].y;
                    if (dx * dx + dy * dy > SR2) continue;
                    double d = desc_l2(md, descs + (size_t)ki * 256);
                    if (d < best_dist) {
                        best_dist = d;
                        best_ki = ki;
                    }
                }
        if (best_ki >= 0 && best_dist < best_desc_dist[best_ki]) {
            kp_to_mp[best_ki] = mp;
            best_desc_dist[best_ki] = best_dist;
            if (*n_obs < obs_cap) {
                obs_mp[*n_obs] = mp;
                obs_kp[*n_obs] = best_ki;
            }
            (*n_obs)++;
            tracked++;
        }
    }
    return tracked;
}

}  // extern "C"
