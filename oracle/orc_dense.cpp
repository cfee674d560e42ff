// orc_dense.cpp — TEST INFRASTRUCTURE: the reference's dense voxel fusion loop restated
// sequentially (main.cpp:1081-1139): per processed frame with real depth, a DENSE_PIXEL_STEP grid
// is back-projected with the frame's pose and a point is appended the first time its voxel is
// inserted into the set.  Same expressions and evaluation order as the reference (built with
// -ffp-contract=off like an x86-64 -O3 build without FMA).
#include <cmath>
#include <set>
#include <tuple>
#include <vector>

#include "oracle.h"

struct orc_dense {
    int step;
    double max_depth, inv, fx, fy, cx, cy, ox, oy, oz;
    std::set<std::tuple<int, int, int>> voxels;  // membership only: the hash of :1087-1093 is irrelevant
    std::vector<double> cloud;
};

extern "C" {

orc_dense* orc_dense_create(int pixel_step, double max_depth, double voxel_size, double fx, double fy, double cx,
                            double cy, double ox, double oy, double oz) {
    orc_dense* d = new orc_dense();
    d->step = pixel_step;
    d->max_depth = max_depth;
    d->inv = 1.0 / voxel_size;  // :1086
    d->fx = fx;
    d->fy = fy;
    d->cx = cx;
    d->cy = cy;
    d->ox = ox;
    d->oy = oy;
    d->oz = oz;
    return d;
}

void orc_dense_destroy(orc_dense* d) { delete d; }

// :1121-1139 for one frame (depth rows x cols, R row-major camera -> world)
void orc_dense_integrate(orc_dense* d, const float* depth, int rows, int cols, const double* R, const double* t) {
    for (int v = 0; v < rows; v += d->step) {
        for (int u = 0; u < cols; u += d->step) {
            float z = depth[(size_t)v * cols + u];
            if (z <= 0 || z >= d->max_depth) continue;
            double x_cam = (u - d->cx) * z / d->fx;
            double y_cam = (v - d->cy) * z / d->fy;
            double px = R[0] * x_cam + R[1] * y_cam + R[2] * z + t[0] - d->ox;
            double py = R[3] * x_cam + R[4] * y_cam + R[5] * z + t[1] - d->oy;
            double pz = R[6] * x_cam + R[7] * y_cam + R[8] * z + t[2] - d->oz;
            auto vk = std::make_tuple((int)std::floor(px * d->inv), (int)std::floor(py * d->inv),
                                      (int)std::floor(pz * d->inv));
            if (d->voxels.insert(vk).second) {
                d->cloud.push_back(px);
                d->cloud.push_back(py);
                d->cloud.push_back(pz);
            }
        }
    }
}

long long orc_dense_points(const orc_dense* d, double* xyz, long long cap) {
    const long long n = (long long)(d->cloud.size() / 3);
    for (long long i = 0; i < n && i < cap; i++)
        for (int k = 0; k < 3; k++) xyz[3 * i + k] = d->cloud[3 * i + k];
    return n;
}

}  // extern "C"
