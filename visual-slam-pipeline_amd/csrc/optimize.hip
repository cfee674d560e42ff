// optimize.hip — Optimizer::project_point / Optimizer::optimize_pose on gfx950
// (reference src/Optimizer.cpp:26-48, 54-180).
//
// One workgroup per pose problem (a batch of frames runs as a grid).  Each LM iteration follows
// the reference: Rodrigues(rvec), forward-difference Jacobian with eps = 1e-6 on all six
// parameters (the three rotation-perturbed matrices are shared by every point), J^T J + lambda I,
// Cholesky solve, accept when the RMS reprojection error drops (lambda / 2) else lambda * 10, stop
// when the error change is below 1e-6 or after 10 iterations.  Points are spread over the lanes;
// the 27 normal-equation sums and the error sums are reduced in a fixed order (per-lane partials,
// then a shuffle tree, then the four waves), so results are deterministic.  The sums differ from
// the oracle's sequential order by rounding only (tests bound the pose and RMS differences).
#include <hip/hip_runtime.h>

#include <cfloat>

#include "block_reduce.h"
#include "cr_math.h"
#include "vs_internal.h"

namespace vs {

__device__ void rodrigues_v2m(const double r[3], double R[9]) {
    const double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < DBL_EPSILON) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    const double c = vs_cr::cos(theta), s = vs_cr::sin(theta), c1 = 1.0 - c;
    const double itheta = theta ? 1.0 / theta : 0.0;
    const double rx = r[0] * itheta, ry = r[1] * itheta, rz = r[2] * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int i = 0; i < 9; i++) R[i] = c * ((i % 4 == 0) ? 1.0 : 0.0) + c1 * rrt[i] + s * rx_[i];
}

__device__ void rodrigues_m2v(const double R[9], double r[3]) {
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = vs_cr::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            r[0] = r[1] = r[2] = 0;
            return;
        }
        double t = (R[0] + 1) * 0.5;
        rx = sqrt(fmax(t, 0.));
        t = (R[4] + 1) * 0.5;
        ry = sqrt(fmax(t, 0.)) * (R[1] < 0 ? -1. : 1.);
        t = (R[8] + 1) * 0.5;
        rz = sqrt(fmax(t, 0.)) * (R[2] < 0 ? -1. : 1.);
        if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
        theta /= sqrt(rx * rx + ry * ry + rz * rz);
        r[0] = rx * theta;
        r[1] = ry * theta;
        r[2] = rz * theta;
        return;
    }
    double vth = 1 / (2 * s);
    vth *= theta;
    r[0] = rx * vth;
    r[1] = ry * vth;
    r[2] = rz * vth;
}

// Optimizer::project_point with the camera->world pose given as R_cam = R^T and t_cam.
struct CamPose {
    double Rc[9], tc[3];
};

__device__ CamPose cam_pose(const double R[9], const double t[3]) {
    CamPose p;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) p.Rc[i * 3 + j] = R[j * 3 + i];
    for (int i = 0; i < 3; i++) p.tc[i] = -(p.Rc[i * 3 + 0] * t[0] + p.Rc[i * 3 + 1] * t[1] + p.Rc[i * 3 + 2] * t[2]);
    return p;
}

__device__ void project_dev(const CamPose& p, const double* pw, const double K[4], double& u, double& v) {
    double pc[3];
    for (int i = 0; i < 3; i++) pc[i] = p.Rc[i * 3 + 0] * pw[0] + p.Rc[i * 3 + 1] * pw[1] + p.Rc[i * 3 + 2] * pw[2] + p.tc[i];
    const double z = pc[2];
    if (z < 1e-6) {
        u = -1;
        v = -1;
        return;
    }
    u = K[0] * pc[0] / z + K[2];
    v = K[1] * pc[1] / z + K[3];
}

__device__ int cholesky6(double* A, double* b) {
    const int n = 6;
    for (int j = 0; j < n; j++) {
        double s = A[j * n + j];
        for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
        if (s < DBL_EPSILON) return 0;
        const double d = sqrt(s);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double v = A[i * n + j];
            for (int k = 0; k < j; k++) v -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = v / d;
        }
    }
    for (int i = 0; i < n; i++) {
        double v = b[i];
        for (int k = 0; k < i; k++) v -= A[i * n + k] * b[k];
        b[i] = v / A[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double v = b[i];
        for (int k = i + 1; k < n; k++) v -= A[k * n + i] * b[k];
        b[i] = v / A[i * n + i];
    }
    return 1;
}

struct OptShared {
    double red[4 * 28];
    double rvec[3], tvec[3], lambda;
    double rv_new[3], tv_new[3];
    int solved, stop, accepted, iters;
};

// sum of squared reprojection residuals of all points under (R, t)
__device__ double sq_err(const double* P, const float* p2, int n, const double R[9], const double t[3],
                         const double K[4], double* s_red) {
    const CamPose cp = cam_pose(R, t);
    double part[1] = {0.0};
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        double u, v;
        project_dev(cp, P + 3 * i, K, u, v);
        const double dx = u - (double)p2[2 * i], dy = v - (double)p2[2 * i + 1];
        part[0] += dx * dx + dy * dy;
    }
    double out[1];
    block_sum<1>(part, s_red, out);
    return out[0];
}

// problems p: P[off[p]..off[p+1]) points; R/t in/out [p][9]/[p][3]; res[p] = {rms_before,
// rms_after, iterations, accepted}
__global__ __launch_bounds__(256) void k_optimize_pose(const double* __restrict__ P, const float* __restrict__ p2,
                                                       const int* __restrict__ off, double fx, double fy, double cx,
                                                       double cy, double* __restrict__ Rio, double* __restrict__ tio,
                                                       double* __restrict__ res, int* __restrict__ ok) {
    __shared__ OptShared S;
    const int pb = blockIdx.x;
    const int o0 = off[pb], n = off[pb + 1] - o0;
    const double K[4] = {fx, fy, cx, cy};
    const double* Pp = P + 3 * (size_t)o0;
    const float* pp = p2 + 2 * (size_t)o0;
    if (n < 3) {  // Optimizer.cpp:60-62: {0, 0}, pose untouched
        if (threadIdx.x == 0) {
            res[4 * pb] = res[4 * pb + 1] = res[4 * pb + 2] = res[4 * pb + 3] = 0;
            ok[pb] = 0;
        }
        return;
    }
    double R0[9], t0[3];
    for (int k = 0; k < 9; k++) R0[k] = Rio[9 * pb + k];
    for (int k = 0; k < 3; k++) t0[k] = tio[3 * pb + k];
    if (threadIdx.x == 0) {
        rodrigues_m2v(R0, S.rvec);
        for (int k = 0; k < 3; k++) S.tvec[k] = t0[k];
        S.lambda = 1e-3;  // OPT_LM_LAMBDA
        S.accepted = 0;
        S.iters = 0;
    }
    const double err_before = sqrt(sq_err(Pp, pp, n, R0, t0, K, S.red) / n);
    const double eps = 1e-6;
    for (int iter = 0; iter < 10; iter++) {  // OPT_MAX_ITERATIONS
        double rvec[3], tvec[3];
        for (int k = 0; k < 3; k++) {
            rvec[k] = S.rvec[k];
            tvec[k] = S.tvec[k];
        }
        double Rcur[9];
        rodrigues_v2m(rvec, Rcur);
        CamPose cp = cam_pose(Rcur, tvec), cpr[3], cpt[3];
        for (int j = 0; j < 3; j++) {
            double rp[3] = {rvec[0], rvec[1], rvec[2]};
            rp[j] += eps;
            double Rp[9];
            rodrigues_v2m(rp, Rp);
            cpr[j] = cam_pose(Rp, tvec);
            double tp[3] = {tvec[0], tvec[1], tvec[2]};
            tp[j] += eps;
            cpt[j] = cam_pose(Rcur, tp);
        }
        // normal equations: 21 upper-triangle JtJ entries, 6 Jtr, 1 current squared error
        double acc[28];
        for (int k = 0; k < 28; k++) acc[k] = 0;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            double u, v;
            project_dev(cp, Pp + 3 * i, K, u, v);
            const double ru = u - (double)pp[2 * i], rv = v - (double)pp[2 * i + 1];
            double ju[6], jv[6];
            for (int j = 0; j < 6; j++) {
                double up, vp;
                project_dev(j < 3 ? cpr[j] : cpt[j - 3], Pp + 3 * i, K, up, vp);
                ju[j] = (up - u) / eps;
                jv[j] = (vp - v) / eps;
            }
            int k = 0;
            for (int a = 0; a < 6; a++)
                for (int c = a; c < 6; c++) acc[k++] += ju[a] * ju[c] + jv[a] * jv[c];
            for (int a = 0; a < 6; a++) acc[21 + a] += ju[a] * ru + jv[a] * rv;
            acc[27] += ru * ru + rv * rv;
        }
        double tot[28];
        block_sum<28>(acc, S.red, tot);
        if (threadIdx.x == 0) {
            double A[36], b[6];
            int k = 0;
            for (int a = 0; a < 6; a++)
                for (int c = a; c < 6; c++) {
                    A[a * 6 + c] = tot[k];
                    A[c * 6 + a] = tot[k];
                    k++;
                }
            for (int a = 0; a < 6; a++) A[a * 6 + a] += S.lambda;
            for (int a = 0; a < 6; a++) b[a] = -tot[21 + a];
            S.solved = cholesky6(A, b);
            if (S.solved) {
                for (int a = 0; a < 3; a++) {
                    S.rv_new[a] = rvec[a] + b[a];
                    S.tv_new[a] = tvec[a] + b[3 + a];
                }
            } else {
                S.lambda *= 10;
            }
            S.iters++;
        }
        __syncthreads();
        if (!S.solved) continue;
        double rv_new[3], tv_new[3], Rnew[9];
        for (int a = 0; a < 3; a++) {
            rv_new[a] = S.rv_new[a];
            tv_new[a] = S.tv_new[a];
        }
        rodrigues_v2m(rv_new, Rnew);
        const double error_new = sqrt(sq_err(Pp, pp, n, Rnew, tv_new, K, S.red) / n);
        const double current_error = sqrt(tot[27] / n);
        if (threadIdx.x == 0) {
            if (error_new < current_error) {
                for (int a = 0; a < 3; a++) {
                    S.rvec[a] = rv_new[a];
                    S.tvec[a] = tv_new[a];
                }
                S.lambda /= 2;
                S.accepted++;
            } else {
                S.lambda *= 10;
            }
            S.stop = fabs(current_error - error_new) < 1e-6;  // OPT_CONVERGENCE
        }
        __syncthreads();
        if (S.stop) break;
    }
    double Ropt[9], topt[3];
    for (int k = 0; k < 3; k++) topt[k] = S.tvec[k];
    {
        double rv[3] = {S.rvec[0], S.rvec[1], S.rvec[2]};
        rodrigues_v2m(rv, Ropt);
    }
    const double err_after = sqrt(sq_err(Pp, pp, n, Ropt, topt, K, S.red) / n);
    if (threadIdx.x == 0) {
        for (int k = 0; k < 9; k++) Rio[9 * pb + k] = Ropt[k];
        for (int k = 0; k < 3; k++) tio[3 * pb + k] = topt[k];
        res[4 * pb] = err_before;
        res[4 * pb + 1] = err_after;
        res[4 * pb + 2] = S.iters;
        res[4 * pb + 3] = S.accepted;
        ok[pb] = 1;
    }
}

int optimize_pose(vs_ctx* ctx, int nprob, const double* d_P, const float* d_p2, const int* d_off, const double K[4],
                  double* d_R, double* d_t, double* d_res, int* d_ok, hipStream_t s) {
    if (nprob <= 0) return VS_OK;
    ProfScope ps(ctx, "optimize_pose", s);
    hipLaunchKernelGGL(k_optimize_pose, dim3(nprob), dim3(256), 0, s, d_P, d_p2, d_off, K[0], K[1], K[2], K[3], d_R,
                       d_t, d_res, d_ok);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs
