// pnp.hip — Slam::solve_pnp (reference src/Slam.cpp:505-529: cv::solvePnPRansac, 8 px,
// confidence 0.99, then R_world = R_cam^T, t_world = -R_cam^T tvec) on gfx950.
//
// A batch of problems (frames, or the periodic / recovery / loop callers) is one grid per stage.
// The OpenCV RANSAC loop is sequential only through its adaptive iteration budget, and that
// budget only shrinks, so
//   1. k_pnp_subsets draws every subset of the initial budget from the cv::RNG stream (one
//      workgroup per problem; jump-ahead + pointer doubling, the stream does not depend on the
//      models because checkSubset is trivially true for PnP),
//   2. k_pnp_hyp solves the EPnP hypotheses and counts their inliers, one wave64 per hypothesis
//      (solving only a first wave of 16 and the rest on demand was tried: with this data the
//      budget rarely ends inside 16 iterations, and the two serialized waves cost 50 % more),
//   3. k_pnp_ransac replays the accept / RANSACUpdateNumIters sequence over the counts — exactly
//      the hypotheses the sequential loop would have evaluated, in its order — marks the winner's
//      inliers and refines (rvec, tvec) with the LM of pnp_solvers.h, the 28 normal-equation sums
//      reduced in a fixed lane / butterfly order that the oracle restates.
// Numerical kernels are shared with the CPU restatement (pnp_solvers.h; this file is built
// with -ffp-contract=off like the oracle).
#include <hip/hip_runtime.h>

#include <climits>

#include "block_reduce.h"
#include "pnp_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_pnp;

constexpr int kPnpMaxIters = VS_PNP_MAX_ITERS;

#ifdef VS_PNP_PROFILE
// k_pnp_hyp phase cycle counters (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_pnp_cycles[32];  // k_pnp_hyp 0-5, 13-21 (1-3, 13-14 eigen stages, 15-19 the variants' stages, 20-21 loads / Rodrigues, 22-25 control points), 6-7 k_pnp_ransac, 8-12 its LM split
#define PNP_T0() long long _pn_t = clock64()
#define PNP_T(k)                                                             \
    do {                                                                     \
        if (threadIdx.x == 0) atomicAdd(&g_pnp_cycles[k], clock64() - _pn_t); \
        _pn_t = clock64();                                                   \
    } while (0)
#else
#define PNP_T0()
#define PNP_T(k)
#endif

struct PnpShared {
    LmRots rots;
    double red[4 * kLmTerms];
    LmState lm;
    double rv[3], tv[3];
    int best, best_iter, niters_run, go;
};

// Per-problem hypothesis table in global memory: subsets [iters][5], counts [iters] (-1 = EPnP
// failed), models [iters][6] = (rvec, tvec).
struct PnpHyp {
    int* subset;
    int* count;
    double* model;
    int stride;  // hypotheses per problem
    int tab_n0;  // >= 0: subset is the context's table by point count (row n - tab_n0); -1: per problem
};

// Subsets depend on (n, iteration budget) only, so the usual budget's are drawn once per context
// for every n in [kPnpTabMinN, kPnpTabMaxN] (2 MB) and k_pnp_hyp indexes that table by n: no
// subset launch on the tracker's per-frame path.
constexpr int kPnpTabIters = 100, kPnpTabMinN = 6, kPnpTabMaxN = 1024;
constexpr int kPnpLdsPts = 512;  // points k_pnp_hyp stages in LDS (the tracker's problems have <= 400)

__device__ __forceinline__ const int* pnp_subset(const PnpHyp& H, int pb, int n, int h) {
    return H.tab_n0 >= 0 ? H.subset + ((size_t)(n - H.tab_n0) * H.stride + h) * 5
                         : H.subset + ((size_t)pb * H.stride + h) * 5;
}

__device__ inline bool pnp_problem_runs(int n, int min_inliers, int model_points) {
    return !(n < min_inliers || n < 4) && n != model_points;
}

// a lane's double, read by the whole wave (static lane index: two v_readlane into SGPRs)
__device__ __forceinline__ double lane_bcast(double x, int src) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

struct EpShared {
    double R[10][10];  // R of M^T = Q R (upper triangle)
    double B[10][10];  // R R^T
    double U[8][10];   // tridiagonal reflectors (indices k+1..9), tt their taus
    double tt[8];
    double v[4][12];   // the four eigenvectors (pnp_solvers.h epnp_small_eig's v)
};

// pnp_solvers.h epnp_small_eig spread over one wave, bit-identical to it: lane j < 2m keeps column j
// of M^T in registers through the QR (each reflector read by the wave with v_readlane), lanes a <= b
// form B = R R^T from LDS, lane i < 10 keeps row i of B through the tridiagonalisation (B stays
// exactly symmetric, so a lane's own reflector entry is its column k), lanes 0-31 / 32-63 run the
// multisection for the smallest / second smallest eigenvalue (one Sturm count per lane, a ballot
// picks the subinterval), lanes 0 / 1 the inverse iterations, lanes 0-3 the back-transformations.
#ifdef VS_PNP_PROFILE
#define EP_T(k)                                                                   \
    do {                                                                          \
        if (lane == 0) atomicAdd(&g_pnp_cycles[k], (unsigned long long)(clock64() - tprof)); \
        tprof = clock64();                                                        \
    } while (0)
#else
#define EP_T(k)
#endif
__device__ __forceinline__ void epnp_small_eig_wave(const double (*al)[4], const double* uv, int m, const Cam& K,
                                                    int lane, EpShared& S, [[maybe_unused]] long long& tprof) {
    const int nc = 2 * m;
    double c[12], t[12];
#pragma unroll
    for (int r = 0; r < 12; r++) c[r] = lane < nc ? ep_mt(al, uv, K, lane, r) : 0.0;
    double my_alpha = 0, my_tau = 0;
    // 1. QR of M^T
#pragma unroll
    for (int k = 0; k < 10; k++) {
        if (k >= nc) continue;  // (m = 4: 8 columns; not break: the loop must unroll for static k)
#pragma unroll
        for (int r = 0; r < 12; r++) t[r] = r >= k ? c[r] * c[r] : -0.0;
        double alpha, u0, tau;
        ep_householder(tsum<12>(t), c[k], alpha, u0, tau);
        if (lane == k) {
            c[k] = u0;
            my_alpha = alpha;
            my_tau = tau;
        }
        double u[12];
#pragma unroll
        for (int r = k; r < 12; r++) u[r] = lane_bcast(c[r], k);
        const double tk = lane_bcast(tau, k);
        if (lane > k && lane < nc) {
#pragma unroll
            for (int r = 0; r < 12; r++) t[r] = r >= k ? u[r] * c[r] : -0.0;
            const double f = tk * tsum<12>(t);
#pragma unroll
            for (int r = k; r < 12; r++) c[r] = c[r] - f * u[r];
        }
    }
    double x[12];  // lanes 0..3: the vectors mapped back through Q
    const int nz = nc == 10 ? 2 : 4;
#pragma unroll
    for (int r = 0; r < 12; r++) x[r] = (lane < nz && r == nc + lane) ? 1.0 : 0.0;
    if (nc == 10) {
        // 2. B = R R^T
        if (lane < 10) {
#pragma unroll
            for (int a = 0; a < 10; a++) S.R[a][lane] = a < lane ? c[a] : a == lane ? my_alpha : 0.0;
        }
        __syncthreads();
        if (lane < 55) {  // upper-triangle element (a, b), a <= b
            int a = 0, rem = lane;
            while (rem >= 10 - a) {
                rem -= 10 - a;
                a++;
            }
            const int b = a + rem;
#pragma unroll
            for (int k = 0; k < 10; k++) t[k] = k >= b ? S.R[a][k] * S.R[b][k] : -0.0;
            const double s = tsum<10>(t);
            S.B[a][b] = s;
            S.B[b][a] = s;
        }
        __syncthreads();
        EP_T(1);
        // tridiagonalisation
        double br[10];
#pragma unroll
        for (int j = 0; j < 10; j++) br[j] = lane < 10 ? S.B[lane][j] : 0.0;
        double d[10], e[9];
#pragma unroll
        for (int k = 0; k < 8; k++) {
#pragma unroll
            for (int j = 0; j < 10; j++) t[j] = j > k ? br[j] * br[j] : -0.0;
            double alpha, u0, tk0;
            ep_householder(tsum<10>(t), br[k + 1], alpha, u0, tk0);
            e[k] = lane_bcast(alpha, k);
            d[k] = lane_bcast(br[k], k);
            const double tk = lane_bcast(tk0, k);
            double U[10];
            U[k + 1] = lane_bcast(u0, k);
#pragma unroll
            for (int j = k + 2; j < 10; j++) U[j] = lane_bcast(br[j], k);
            if (lane == k) {
#pragma unroll
                for (int j = k + 1; j < 10; j++) S.U[k][j] = U[j];
                S.tt[k] = tk;
            }
            const bool act = lane > k && lane < 10;
            const double uo = lane == k + 1 ? U[k + 1] : br[k];  // this row's reflector entry (B symmetric)
#pragma unroll
            for (int j = 0; j < 10; j++) t[j] = j > k ? br[j] * U[j] : -0.0;
            const double p = act ? tk * tsum<10>(t) : 0.0;
#pragma unroll
            for (int i = 0; i < 10; i++) t[i] = i > k ? lane_bcast(p, i) * U[i] : -0.0;
            const double Kc = (0.5 * tk) * tsum<10>(t);
            const double w = p - Kc * uo;
            double wj[10];
#pragma unroll
            for (int j = k + 1; j < 10; j++) wj[j] = lane_bcast(w, j);
            if (act) {
#pragma unroll
                for (int j = k + 1; j < 10; j++) br[j] = br[j] - (uo * wj[j] + w * U[j]);
            }
        }
        d[8] = lane_bcast(br[8], 8);
        d[9] = lane_bcast(br[9], 9);
        e[8] = lane_bcast(br[9], 8);
        EP_T(2);
        // 3. scaled to ||T|| in [1, 2); multisection: lanes 0-31 the smallest eigenvalue, 32-63 the
        //    second smallest
        double lo = 0, hi = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const double rad = (i > 0 ? fabs(e[i - 1]) : 0.0) + (i < 9 ? fabs(e[i]) : 0.0);
            const double l = d[i] - rad, h = d[i] + rad;
            lo = (i == 0 || l < lo) ? l : lo;
            hi = (i == 0 || h > hi) ? h : hi;
        }
        const double sc = ep_scale(fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi));
        double e2[9];
#pragma unroll
        for (int i = 0; i < 10; i++) d[i] *= sc;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            e[i] *= sc;
            e2[i] = e[i] * e[i];
        }
        lo *= sc;
        hi *= sc;
        const int tsel = lane >> 5;
        const double fj = ep_frac(lane & 31);
        double a0 = lo, b0 = hi, a1 = lo, b1 = hi;
        for (int st = 0; st < kEpMsSteps; st++) {
            const double a = tsel ? a1 : a0, wd = tsel ? b1 - a1 : b0 - a0;
            const bool above = ep_sturm(d, e2, a + wd * fj) > tsel;
            const unsigned long long bal = __ballot(above);
            const unsigned m0 = (unsigned)bal, m1 = (unsigned)(bal >> 32);
            const int j0 = m0 ? __builtin_ctz(m0) : kEpMsPts, j1 = m1 ? __builtin_ctz(m1) : kEpMsPts;
            const double w0 = b0 - a0, w1 = b1 - a1;
            const double na0 = j0 > 0 ? a0 + w0 * ep_frac(j0 - 1) : a0;
            const double nb0 = j0 < kEpMsPts ? a0 + w0 * ep_frac(j0) : b0;
            const double na1 = j1 > 0 ? a1 + w1 * ep_frac(j1 - 1) : a1;
            const double nb1 = j1 < kEpMsPts ? a1 + w1 * ep_frac(j1) : b1;
            a0 = na0;
            b0 = nb0;
            a1 = na1;
            b1 = nb1;
        }
        EP_T(3);
        // 4. inverse iteration, lane q for eigenvalue q
        const double tnorm = fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi);
        const double tiny = tnorm > 0 ? DBL_EPSILON * tnorm : DBL_MIN;
        const double lam0 = 0.5 * (a0 + b0), lam1 = 0.5 * (a1 + b1);
        const bool cluster = lam1 - lam0 <= 1e-3 * tnorm;
        double y[10];
        if (lane < 2) {
            EpLu f;
            ep_lu(d, e, lane ? lam1 : lam0, tiny, f);
#pragma unroll
            for (int i = 0; i < 10; i++) y[i] = ep_start(i);
            for (int it = 0; it < kEpInvIters; it++) {
                ep_lu_solve(f, y);
                if (cluster) {
                    double y0[10];
#pragma unroll
                    for (int i = 0; i < 10; i++) y0[i] = lane_bcast(y[i], 0);
                    if (lane == 1) ep_orth10(y0, y);
                }
            }
            ep_normalize10(y);
            // back through the tridiagonal reflectors
#pragma unroll
            for (int k = 7; k >= 0; k--) {
#pragma unroll
                for (int i = 0; i < 10; i++) t[i] = i > k ? S.U[k][i] * y[i] : -0.0;
                const double fk = S.tt[k] * tsum<10>(t);
#pragma unroll
                for (int i = k + 1; i < 10; i++) y[i] = y[i] - fk * S.U[k][i];
            }
        }
        double yt[10];
#pragma unroll
        for (int i = 0; i < 10; i++) {
            const double y0 = lane_bcast(y[i], 0), y1 = lane_bcast(y[i], 1);
            yt[i] = lane == 2 ? y0 : y1;
        }
        if (lane == 2 || lane == 3) {
#pragma unroll
            for (int r = 0; r < 10; r++) x[r] = yt[r];
        }
    }
    EP_T(13);
    // 5. v = Q x, lanes 0..3
#pragma unroll
    for (int k = 9; k >= 0; k--) {
        if (k >= nc) continue;
        double u[12];
#pragma unroll
        for (int r = k; r < 12; r++) u[r] = lane_bcast(c[r], k);
        const double tk = lane_bcast(my_tau, k);
#pragma unroll
        for (int r = 0; r < 12; r++) t[r] = r >= k ? u[r] * x[r] : -0.0;
        const double fk = tk * tsum<12>(t);
#pragma unroll
        for (int r = k; r < 12; r++) x[r] = x[r] - fk * u[r];
    }
    if (lane < 4) {
#pragma unroll
        for (int r = 0; r < 12; r++) S.v[lane][r] = x[r];
    }
    EP_T(14);
}

// 1. subsets of the initial budget from the cv::RNG stream (getSubset: repeats rejected); the
//    stream does not depend on the models because checkSubset is trivially true for PnP.  One
//    workgroup per problem, up to 256 iterations per round: raw draws out of order with the
//    cv::RNG jump-ahead (pnp_solvers.h), J0[p] = one past the 5th distinct draw from p for every
//    p, pointer doubling for each iteration's first draw, subsets assembled in parallel.
constexpr int kPnpRaw = 2048;
constexpr int kPnpLevels = 8;  // 2^8 >= 256 iterations per round
struct PnpMwcPow {
    uint64_t v[kPnpRaw];
};
constexpr PnpMwcPow make_pnp_mwc_pow() {
    PnpMwcPow t{};
    uint64_t s = kMwcR1;
    for (int i = 0; i < kPnpRaw; i++) {
        t.v[i] = s;
        s = mwc_step(s);
    }
    return t;
}
__constant__ PnpMwcPow g_pnp_mwc_pow = make_pnp_mwc_pow();

// n_base >= 0: problem pb has n = n_base + pb points (the table build; off unused, rows pb).
__global__ __launch_bounds__(256) void k_pnp_subsets(const int* __restrict__ off, int n_base, int niters0,
                                                     int min_inliers, PnpHyp H) {
    __shared__ int s_draw[kPnpRaw];
    __shared__ uint16_t s_J[kPnpLevels][kPnpRaw + 2];
    __shared__ int s_start[256];
    __shared__ int s_navail;
    __shared__ uint64_t s_rng;
    const int pb = blockIdx.x, tid = threadIdx.x;
    const int n = n_base >= 0 ? n_base + pb : off[pb + 1] - off[pb];
    const int model_points = n == 4 ? 4 : 5;
    if (!pnp_problem_runs(n, min_inliers, model_points)) return;  // running problems have n > 5
    float per = 0.f;
    for (int k = 0; k < 5; k++) per += (float)n / (float)(n - k);
    if (tid == 0) s_rng = (uint64_t)-1;
    int base = 0;
    while (base < niters0) {
        const int want = min(256, niters0 - base);
        const int R = min(kPnpRaw, (int)(want * per * 1.15f) + 64);
        __syncthreads();
        const uint64_t s1 = mwc_step(s_rng);
        for (int r = tid; r < R; r += 256) s_draw[r] = (int)((unsigned)mwc_jump(s1, r, g_pnp_mwc_pow.v[r]) % (unsigned)n);
        if (tid == 0) s_navail = want;
        __syncthreads();
        for (int p = tid; p <= R + 1; p += 256) {
            int e = R + 1;
            if (p < R) {
                int cur[5] = {-1, -1, -1, -1, -1};
                int i = 0, q = p;
                while (i < 5 && q < R) {
                    const int v = s_draw[q++];
                    bool dup = false;
#pragma unroll
                    for (int k = 0; k < 5; k++) dup |= (k < i) & (cur[k] == v);
                    if (!dup) {
#pragma unroll
                        for (int k = 0; k < 5; k++) cur[k] = (k == i) ? v : cur[k];
                        i++;
                    }
                }
                if (i == 5) e = q;
            }
            s_J[0][p] = (uint16_t)e;
        }
        __syncthreads();
        int L = 0;
        while ((1 << L) < want) L++;
        for (int k = 1; k < L; k++) {
            for (int p = tid; p <= R + 1; p += 256) s_J[k][p] = s_J[k - 1][s_J[k - 1][p]];
            __syncthreads();
        }
        for (int t = tid; t < want; t += 256) {
            int p = 0;
            for (int k = 0; k < L; k++)
                if ((t >> k) & 1) p = s_J[k][p];
            const bool avail = p < R && s_J[0][p] <= R;
            s_start[t] = avail ? p : -1;
            if (!avail) atomicMin(&s_navail, t);
        }
        __syncthreads();
        const int T = s_navail;
        for (int t = tid; t < T; t += 256) {
            int cur[5] = {-1, -1, -1, -1, -1};
            int i = 0, q = s_start[t];
            while (i < 5) {
                const int v = s_draw[q++];
                bool dup = false;
#pragma unroll
                for (int k = 0; k < 5; k++) dup |= (k < i) & (cur[k] == v);
                if (!dup) {
#pragma unroll
                    for (int k = 0; k < 5; k++) cur[k] = (k == i) ? v : cur[k];
                    i++;
                }
            }
            int* dst = H.subset + ((size_t)pb * H.stride + base + t) * 5;
#pragma unroll
            for (int k = 0; k < 5; k++) dst[k] = cur[k];
        }
        if (tid == 0) {
            if (T > 0) {
                const int P = s_J[0][s_start[T - 1]];  // raw draws consumed
                s_rng = mwc_jump(s1, P - 1, g_pnp_mwc_pow.v[P - 1]);
            } else {  // the window held no complete subset (not reachable for n > 5): one serially
                CvRng rng(s_rng);
                int cur[5] = {-1, -1, -1, -1, -1};
                for (int i = 0; i < 5; i++)
                    for (;;) {
                        const int v = rng.uniform(0, n);
                        bool dup = false;
                        for (int k = 0; k < i; k++) dup |= cur[k] == v;
                        if (!dup) {
                            cur[i] = v;
                            break;
                        }
                    }
                int* dst = H.subset + ((size_t)pb * H.stride + base) * 5;
                for (int k = 0; k < 5; k++) dst[k] = cur[k];
                s_rng = rng.state;
            }
        }
        base += T > 0 ? T : 1;
    }
}

// 2. one hypothesis per wave64 workgroup: EPnP on its subset with the four smallest eigenvectors
//    of M^T M spread over the wave (epnp_small_eig_wave: QR null space + tridiagonal multisection and
//    inverse iteration, bit-identical to the host's epnp_small_eig; round 5, replacing the 12 x 12
//    round-robin Jacobi), the three beta approximations on lanes 0-2, then the inlier count over all
//    points by the whole wave.
__global__ __launch_bounds__(64) void k_pnp_hyp(const float* __restrict__ obj_all, const float* __restrict__ img_all,
                                                const int* __restrict__ off, double fx, double fy, double cx, double cy,
                                                int niters0, float thr2, int min_inliers, PnpHyp H) {
    crit_prio();
    __shared__ EpShared sE;
    __shared__ float sObj[3 * kPnpLdsPts], sImg[2 * kPnpLdsPts];  // the problem's first points, for the count
    __shared__ double sX[15], sUV[10], sAl[5][4], sCw[4][3];
    __shared__ double sErr[3], sRt[3][12], sL[6][10], sRho[6];
    __shared__ int sOk;
    const int pb = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
    const int o0 = off[pb], n = off[pb + 1] - o0;
    const int model_points = n == 4 ? 4 : 5;
    // n == model points: OpenCV's single EPnP on all points, hypothesis 0 here (k_pnp_ransac reads it)
    const bool single = n == model_points && !(n < min_inliers || n < 4);
    if (h >= niters0 || (single ? h > 0 : !pnp_problem_runs(n, min_inliers, model_points))) return;
    const float* obj = obj_all + 3 * (size_t)o0;
    const float* img = img_all + 2 * (size_t)o0;
    const Cam K{fx, fy, cx, cy};
    const int* idx = single ? nullptr : pnp_subset(H, pb, n, h);
    const int m = model_points;
    PNP_T0();
    // the problem's points (up to kPnpLdsPts) into LDS, loaded beside the subset indices: the
    // subset gather and the inlier count then read LDS instead of two dependent global loads
    const int nl = n < kPnpLdsPts ? n : kPnpLdsPts;
    const int si = lane < m ? (single ? lane : idx[lane]) : 0;
    {
        float ob[3 * kPnpLdsPts / 64], im[2 * kPnpLdsPts / 64];
#pragma unroll
        for (int j = 0; j < 3 * kPnpLdsPts / 64; j++) ob[j] = lane + 64 * j < 3 * nl ? obj[lane + 64 * j] : 0.f;
#pragma unroll
        for (int j = 0; j < 2 * kPnpLdsPts / 64; j++) im[j] = lane + 64 * j < 2 * nl ? img[lane + 64 * j] : 0.f;
#pragma unroll
        for (int j = 0; j < 3 * kPnpLdsPts / 64; j++) sObj[lane + 64 * j] = ob[j];
#pragma unroll
        for (int j = 0; j < 2 * kPnpLdsPts / 64; j++) sImg[lane + 64 * j] = im[j];
    }
    __syncthreads();
    if (lane < m) {
        const float* o = si < nl ? sObj + 3 * si : obj + 3 * si;
        const float* q = si < nl ? sImg + 2 * si : img + 2 * si;
        sX[3 * lane] = o[0];
        sX[3 * lane + 1] = o[1];
        sX[3 * lane + 2] = o[2];
        sUV[2 * lane] = q[0];
        sUV[2 * lane + 1] = q[1];
    }
    __syncthreads();
    PNP_T(21);
    if (lane == 0) {
        double cw[4][3], al[5][4], Xr[15];
#pragma unroll
        for (int i = 0; i < 15; i++) Xr[i] = i < 3 * m ? sX[i] : 0.0;  // registers, not LDS, in the sums
#ifdef VS_PNP_PROFILE
        const int cslot[4] = {22, 23, 24, 25};
        auto cmark = [&](int k) {
            atomicAdd(&g_pnp_cycles[cslot[k]], (unsigned long long)(clock64() - _pn_t));
            _pn_t = clock64();
        };
        sOk = epnp_control<5>(Xr, m, cw, al, cmark);
#else
        sOk = epnp_control<5>(Xr, m, cw, al);
#endif
        for (int i = 0; i < 4; i++)
            for (int c = 0; c < 3; c++) sCw[i][c] = cw[i][c];
        for (int i = 0; i < m; i++)
            for (int j = 0; j < 4; j++) sAl[i][j] = al[i][j];
    }
    __syncthreads();
    PNP_T(0);
    bool ok = sOk != 0;
    if (ok) {
        // the four smallest eigenvectors of M^T M (pnp_solvers.h epnp_small_eig, spread over the wave)
#ifdef VS_PNP_PROFILE
        epnp_small_eig_wave(sAl, sUV, m, K, lane, sE, _pn_t);
#else
        long long tp = 0;
        epnp_small_eig_wave(sAl, sUV, m, K, lane, sE, tp);
#endif
        __syncthreads();
        // L_6x10 and rho once for the three approximations, one entry per lane, kept in LDS with
        // the eigenvectors, alphas and points: the variants read them there instead of holding
        // ~190 VGPRs of copies through the Gauss-Newton loop
        if (lane < 60) sL[lane / 10][lane % 10] = epnp_L_entry(sE.v, lane / 10, lane % 10);
        if (lane < 6) sRho[lane] = epnp_rho_entry(sCw, lane);
        __syncthreads();
        if (lane < 3) {  // one beta approximation per lane
            double R[9], t[3];
            // the three approximations as one code path on lanes 0..2 (pnp_solvers.h
            // epnp_betas_init_uniform: bit-identical to epnp_variant's divergent solves)
            double be[4];
            epnp_betas_init_uniform(lane, sL, sRho, be);
#ifdef VS_PNP_PROFILE
            PNP_T(15);  // L, rho, initial betas
            const int slot[4] = {16, 17, 18, 19};
            auto mark = [&](int k) {
                if (lane == 0) atomicAdd(&g_pnp_cycles[slot[k]], (unsigned long long)(clock64() - _pn_t));
                _pn_t = clock64();
            };
            sErr[lane] = epnp_refine<5>(be, sL, sRho, sE.v, sAl, sX, sUV, m, K, R, t, mark);
#else
            sErr[lane] = epnp_refine<5>(be, sL, sRho, sE.v, sAl, sX, sUV, m, K, R, t);
#endif
            for (int k = 0; k < 9; k++) sRt[lane][k] = R[k];
            for (int k = 0; k < 3; k++) sRt[lane][9 + k] = t[k];
        }
        __syncthreads();
        PNP_T(4);
    }
    // model = the first lowest-error approximation (epnp()), as (rvec, tvec)
    double rv[3] = {0, 0, 0}, tv[3] = {0, 0, 0};
    if (ok) {
        int best = 0;
        for (int v = 1; v < 3; v++)
            if (sErr[v] < sErr[best]) best = v;
        rod_m2v(sRt[best], rv);
        for (int k = 0; k < 3; k++) tv[k] = sRt[best][9 + k];
    }
    int cnt = -1;
    if (ok) {
        double R[9];
        rod_v2m(rv, R);
        PNP_T(20);
        int c = 0;
        for (int i = lane; i < nl; i += 64)
            c += reproj_err2(R, tv, K, sObj[3 * i], sObj[3 * i + 1], sObj[3 * i + 2], sImg[2 * i], sImg[2 * i + 1]) <= thr2;
        for (int i = nl + lane; i < n; i += 64)
            c += reproj_err2(R, tv, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1]) <= thr2;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
        cnt = c;
    }
    PNP_T(5);
    if (lane == 0) {
        H.count[(size_t)pb * H.stride + h] = cnt;
        double* mo = H.model + ((size_t)pb * H.stride + h) * 6;
        for (int k = 0; k < 3; k++) {
            mo[k] = rv[k];
            mo[3 + k] = tv[k];
        }
    }
}

// 3-4. per problem: the sequential accept / RANSACUpdateNumIters replay over the counts (exactly
// the hypotheses the OpenCV loop evaluates, in its order), the winner's inlier mask, and the LM
// refinement with the 28 normal-equation sums reduced deterministically over the lanes.
// stat[p][8] = {success, inliers, ransac iterations, best iteration, lm iterations, lm accepted, n, 0}
__global__ __launch_bounds__(256) void k_pnp_ransac(const float* __restrict__ obj_all, const float* __restrict__ img_all,
                                                    const int* __restrict__ off, double fx, double fy, double cx,
                                                    double cy, int max_iters, float thr2, double conf,
                                                    int min_inliers, PnpHyp H, double* __restrict__ Rw,
                                                    double* __restrict__ tw, int* __restrict__ stat,
                                                    uint8_t* __restrict__ mask_all) {
    crit_prio();
    __shared__ PnpShared S;
    __shared__ double s_lden[kPnpMaxIters];
    __shared__ int s_cnt[kPnpMaxIters];  // the counts, staged for the serial replay (LDS, not L2, latency)
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

    if (n == model_points) {  // OpenCV: a single EPnP on all points (k_pnp_hyp's hypothesis 0), every point an inlier
        if (tid == 0) {
            const size_t h0 = (size_t)pb * H.stride;
            const bool ok = H.count[h0] >= 0;
            for (int k = 0; k < 3; k++) {
                S.rv[k] = H.model[h0 * 6 + k];
                S.tv[k] = H.model[h0 * 6 + 3 + k];
            }
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
        const int* count = H.count + (size_t)pb * H.stride;
        PNP_T0();
        // every hypothesis' outlier-ratio term at once (it depends on its count only), then the
        // sequential accept / budget replay reads them
        for (int it = tid; it < niters0; it += blockDim.x) {
            const int c = count[it];
            s_cnt[it] = c;
            s_lden[it] = c >= 0 ? ransac_log_denom((double)(n - c) / n, model_points) : 0.0;
        }
        __syncthreads();
        // The sequential loop `for (it = 0; it < niters; it++) if (count > max(best, mp - 1)) { best,
        // niters = update(niters) }` on wave 0: a hypothesis is accepted iff its count exceeds every
        // earlier count and the floor mp - 1 (the running best is the prefix maximum), so the accepted
        // positions of 64 hypotheses at a time come from one wave scan; only they are walked in order,
        // each applying the same budget update to the running niters and stopping at the first
        // position >= niters.  The loop's exit value is max(final niters, last accepted + 1).
        if (tid < 64) {
            const double log_num = ransac_log_num(conf);
            int niters = niters0, best = 0, best_iter = -1, floor_max = model_points - 1;
            bool stop = false;
            for (int base = 0; base < niters && !stop; base += 64) {
                const int i = base + tid;
                const int c = i < niters0 ? s_cnt[i] : -1;
                int m = c;  // inclusive prefix maximum over the chunk
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(m, o);
                    if (tid >= o) m = m > t ? m : t;
                }
                int ex = __shfl_up(m, 1);
                if (tid == 0) ex = INT_MIN;
                const int prev = ex > floor_max ? ex : floor_max;
                unsigned long long acc = __ballot(c > prev);
                while (acc) {
                    const int l = __ffsll((long long)acc) - 1;
                    acc &= acc - 1;
                    const int j = base + l;
                    if (j >= niters) {
                        stop = true;
                        break;
                    }
                    best = __shfl(c, l);
                    best_iter = j;
                    niters = ransac_update_from_denom(log_num, s_lden[j], niters);
                }
                const int cm = __shfl(m, 63);
                floor_max = cm > floor_max ? cm : floor_max;
            }
            if (tid == 0) {
                S.best = best;
                S.best_iter = best_iter;
                S.niters_run = niters > best_iter + 1 ? niters : best_iter + 1;
            }
        }
        if (tid == 0) {
            const int best = S.best, best_iter = S.best_iter;
            if (best > 0) {
                const double* mo = H.model + ((size_t)pb * H.stride + best_iter) * 6;
                for (int k = 0; k < 3; k++) {
                    S.rv[k] = mo[k];
                    S.tv[k] = mo[3 + k];
                }
            }
        }
        __syncthreads();
        PNP_T(6);
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
        // Thread 0 owns S.lm; the barrier after its update orders it after every lane's read of the
        // previous candidate, and the next reduction's writes to S.red after its reads.
        double p[6] = {rv0[0], rv0[1], rv0[2], tv0[0], tv0[1], tv0[2]};
        for (bool first = true;; first = false) {
            // the 7 rotations of lm_rotations (R(r), R(r +- h e_k)), one per lane, shared via LDS
            if (tid < 7) {
                double r[3] = {p[0], p[1], p[2]};
                if (tid > 0) r[(tid - 1) / 2] += ((tid - 1) % 2 == 0) ? kLmStep : -kLmStep;
                rod_v2m(r, S.rots.R[tid]);
            }
            __syncthreads();
            PNP_T(8);  // rotations
            const LmRots& L = S.rots;
            double acc[kLmTerms], tot[kLmTerms];
            for (int k = 0; k < kLmTerms; k++) acc[k] = 0;
            for (int i = tid; i < n; i += blockDim.x)
                if (mask[i])
                    lm_point(L, p + 3, K, obj[3 * i], obj[3 * i + 1], obj[3 * i + 2], img[2 * i], img[2 * i + 1], acc);
            PNP_T(9);  // point terms (thread 0's share)
            block_sum_to0<kLmTerms>(acc, S.red, tot);  // tot valid on thread 0 (its only reader)
            PNP_T(10);  // reduction
            if (tid == 0) {
                if (first)
                    S.lm.init(p, tot);
                else
                    S.lm.accept_or_reject(tot);
                S.go = S.lm.step();
            }
            __syncthreads();
            PNP_T(11);  // LM control + solve
#ifdef VS_PNP_PROFILE
            if (tid == 0) atomicAdd(&g_pnp_cycles[12], 1ull);  // LM evaluations
#endif
            if (!S.go) break;
            for (int k = 0; k < 6; k++) p[k] = S.lm.cand[k];
        }
        PNP_T(7);  // (after the LM loop: its last iteration's exit)
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

// The context's subset table for kPnpTabIters (built on first use; the build is synchronised
// once so that any stream may read the table afterwards).
static int pnp_table(vs_ctx* ctx, hipStream_t s, int** tab) {
    constexpr int rows = kPnpTabMaxN - kPnpTabMinN + 1;
    if (!ctx->pnp_tab_ready) {
        VS_CHECK(ctx->pnp_tab.ensure((size_t)rows * kPnpTabIters * 5 * sizeof(int)));
        PnpHyp T{};
        T.subset = ctx->pnp_tab.as<int>();
        T.stride = kPnpTabIters;
        T.tab_n0 = -1;
        hipLaunchKernelGGL(k_pnp_subsets, dim3(rows), dim3(256), 0, s, nullptr, kPnpTabMinN, kPnpTabIters, 0, T);
        VS_HIP(hipGetLastError());
        VS_HIP(hipStreamSynchronize(s));
        ctx->pnp_tab_ready = true;
    }
    *tab = ctx->pnp_tab.as<int>();
    return VS_OK;
}

int subset_table(int rows, int n_base, int iters, int* out, hipStream_t s) {
    VS_ARG(rows > 0 && n_base > 5 && iters > 0 && out, "subset_table: bad arguments");
    PnpHyp T{};
    T.subset = out;
    T.stride = iters;
    T.tab_n0 = -1;
    hipLaunchKernelGGL(k_pnp_subsets, dim3(rows), dim3(256), 0, s, nullptr, n_base, iters, 0, T);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int pnp_reserve(vs_ctx* ctx, hipStream_t s) {
    int* tab;
    return pnp_table(ctx, s, &tab);
}

int solve_pnp(vs_ctx* ctx, int nprob, const float* d_obj, const float* d_img, const int* d_off, const double K[4],
              int ransac_iters, int min_inliers, double* d_R, double* d_t, int* d_stat, uint8_t* d_mask,
              hipStream_t s, int max_n) {
    if (nprob <= 0) return VS_OK;
    VS_ARG(ransac_iters <= kPnpMaxIters, "solve_pnp: ransac_iters above kPnpMaxIters");
    ProfScope ps(ctx, "solve_pnp", s);
    const float thr = (float)8.0;  // Config::PNP_RANSAC_THRESHOLD passed as float (Slam.cpp:517)
    const float thr2 = (float)((double)thr * (double)thr);
    const int niters0 = ransac_iters > 1 ? ransac_iters : 1;
    const size_t per = (size_t)nprob * niters0;
    VS_CHECK(ctx->pnp.ensure(per * (6 * sizeof(int) + 6 * sizeof(double))));
    PnpHyp H;
    H.model = ctx->pnp.as<double>();
    H.subset = reinterpret_cast<int*>(H.model + per * 6);
    H.count = H.subset + per * 5;
    H.stride = niters0;
    H.tab_n0 = -1;
    if (niters0 == kPnpTabIters && max_n >= 0 && max_n <= kPnpTabMaxN) {
        VS_CHECK(pnp_table(ctx, s, &H.subset));
        H.tab_n0 = kPnpTabMinN;
    } else {
        hipLaunchKernelGGL(k_pnp_subsets, dim3(nprob), dim3(256), 0, s, d_off, -1, niters0, min_inliers, H);
    }
    hipLaunchKernelGGL(k_pnp_hyp, dim3(nprob, niters0), dim3(64), 0, s, d_obj, d_img, d_off, K[0], K[1], K[2], K[3],
                       niters0, thr2, min_inliers, H);
    hipLaunchKernelGGL(k_pnp_ransac, dim3(nprob), dim3(256), 0, s, d_obj, d_img, d_off, K[0], K[1], K[2], K[3],
                       ransac_iters, thr2, 0.99, min_inliers, H, d_R, d_t, d_stat, d_mask);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

// test hook: the sequential EPnP (the n == model-points path of k_pnp_ransac) on count problems of
// m = 4 / 5 points, one thread each: out[p] = (v[4][12] of epnp_small_eig, R[9], t[3], ok, rod_m2v(R), rod_v2m of it)
__global__ void k_debug_epnp(const double* X, const double* uv, const int* m, int count, double fx, double fy,
                             double cx, double cy, double* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= count) return;
    const Cam K{fx, fy, cx, cy};
    double* o = out + (size_t)p * 73;
    double cw[4][3], al[5][4], v[4][12], R[9] = {}, t[3] = {};
    bool ok = epnp_control<5>(X + 15 * p, m[p], cw, al);
    if (ok) epnp_small_eig(al, uv + 10 * p, m[p], K, v);
    for (int k = 0; k < 48; k++) o[k] = ok ? v[k / 12][k % 12] : 0.0;
    ok = ok && epnp<5>(X + 15 * p, uv + 10 * p, m[p], K, R, t);
    for (int k = 0; k < 9; k++) o[48 + k] = R[k];
    for (int k = 0; k < 3; k++) o[57 + k] = t[k];
    o[60] = ok ? 1.0 : 0.0;
    double rv[3], R2[9];  // the model's Rodrigues round trip (k_pnp_ransac: rod_m2v, then rod_v2m)
    rod_m2v(R, rv);
    rod_v2m(rv, R2);
    for (int k = 0; k < 3; k++) o[61 + k] = rv[k];
    for (int k = 0; k < 9; k++) o[64 + k] = R2[k];
}

// The same sequential EPnP behind a call boundary the compiler may not remove (the
// product once called it out of line from k_pnp_ransac and got eigenvectors different from the host's).
// mode 1: one problem per lane; mode 2: one problem per wave, called by lane 0 alone (the divergent call
// k_pnp_ransac made).
__device__ __attribute__((noinline)) bool epnp_out_of_line(const double* X, const double* uv, int m, const Cam& K,
                                                          double* R, double* t) {
    return epnp<5>(X, uv, m, K, R, t);
}

__device__ __attribute__((noinline)) void eig_out_of_line(const double (*al)[4], const double* uv, int m, const Cam& K,
                                                          double v[4][12], double* dbg) {
    epnp_small_eig(al, uv, m, K, v, dbg);
}

// mode 3: the control points inline, epnp_small_eig out of line, its stage results (216 doubles) in out
__global__ void k_debug_eig_ool(const double* X, const double* uv, const int* m, int count, double fx, double fy,
                                double cx, double cy, double* out) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= count) return;
    const Cam K{fx, fy, cx, cy};
    double cw[4][3], al[5][4], v[4][12];
    double* o = out + (size_t)p * 216;
    for (int k = 0; k < 216; k++) o[k] = 0.0;
    if (epnp_control<5>(X + 15 * p, m[p], cw, al)) eig_out_of_line(al, uv + 10 * p, m[p], K, v, o);
}

__global__ void k_debug_epnp_ool(const double* X, const double* uv, const int* m, int count, double fx, double fy,
                                 double cx, double cy, double* out, int mode) {
    const int p = mode == 2 ? blockIdx.x : blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= count || (mode == 2 && threadIdx.x != 0)) return;
    const Cam K{fx, fy, cx, cy};
    double* o = out + (size_t)p * 73;
    double R[9] = {}, t[3] = {};
    const bool ok = epnp_out_of_line(X + 15 * p, uv + 10 * p, m[p], K, R, t);
    for (int k = 0; k < 48; k++) o[k] = 0.0;
    for (int k = 0; k < 9; k++) o[48 + k] = R[k];
    for (int k = 0; k < 3; k++) o[57 + k] = t[k];
    o[60] = ok ? 1.0 : 0.0;
    double rv[3], R2[9];
    rod_m2v(R, rv);
    rod_v2m(rv, R2);
    for (int k = 0; k < 3; k++) o[61 + k] = rv[k];
    for (int k = 0; k < 9; k++) o[64 + k] = R2[k];
}

}  // namespace vs

extern "C" int vs_debug_epnp(const double* X, const double* uv, const int* m, int count, const double* K, double* out);

// mode 0: vs_debug_epnp; 1, 2: the out-of-line call (k_debug_epnp_ool)
extern "C" int vs_debug_epnp_mode(const double* X, const double* uv, const int* m, int count, const double* K,
                                  double* out, int mode) {
    if (count <= 0) return 0;
    if (mode == 0) return vs_debug_epnp(X, uv, m, count, K, out);
    double *dX, *duv, *dout;
    int* dm;
    if (hipMalloc(&dX, sizeof(double) * 15 * count) != hipSuccess) return -1;
    (void)hipMalloc(&duv, sizeof(double) * 10 * count);
    (void)hipMalloc(&dout, sizeof(double) * 73 * count);
    (void)hipMalloc(&dm, sizeof(int) * count);
    (void)hipMemcpy(dX, X, sizeof(double) * 15 * count, hipMemcpyHostToDevice);
    (void)hipMemcpy(duv, uv, sizeof(double) * 10 * count, hipMemcpyHostToDevice);
    (void)hipMemcpy(dm, m, sizeof(int) * count, hipMemcpyHostToDevice);
    const dim3 grid(mode == 2 ? count : (count + 63) / 64);
    size_t per = 73;
    if (mode == 3) {  // out: [count][216] stage results
        per = 216;
        (void)hipFree(dout);
        (void)hipMalloc(&dout, sizeof(double) * per * count);
        hipLaunchKernelGGL(vs::k_debug_eig_ool, grid, dim3(64), 0, 0, dX, duv, dm, count, K[0], K[1], K[2], K[3], dout);
    } else {
        hipLaunchKernelGGL(vs::k_debug_epnp_ool, grid, dim3(64), 0, 0, dX, duv, dm, count, K[0], K[1], K[2], K[3], dout,
                           mode);
    }
    const hipError_t e = hipMemcpy(out, dout, sizeof(double) * per * count, hipMemcpyDeviceToHost);
    (void)hipFree(dX);
    (void)hipFree(duv);
    (void)hipFree(dout);
    (void)hipFree(dm);
    return e == hipSuccess ? 0 : -1;
}

extern "C" int vs_debug_epnp(const double* X, const double* uv, const int* m, int count, const double* K,
                             double* out) {
    if (count <= 0) return 0;
    double *dX, *duv, *dout;
    int* dm;
    if (hipMalloc(&dX, sizeof(double) * 15 * count) != hipSuccess) return -1;
    (void)hipMalloc(&duv, sizeof(double) * 10 * count);
    (void)hipMalloc(&dout, sizeof(double) * 73 * count);
    (void)hipMalloc(&dm, sizeof(int) * count);
    (void)hipMemcpy(dX, X, sizeof(double) * 15 * count, hipMemcpyHostToDevice);
    (void)hipMemcpy(duv, uv, sizeof(double) * 10 * count, hipMemcpyHostToDevice);
    (void)hipMemcpy(dm, m, sizeof(int) * count, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(vs::k_debug_epnp, dim3((count + 63) / 64), dim3(64), 0, 0, dX, duv, dm, count, K[0], K[1], K[2],
                       K[3], dout);
    const hipError_t e = hipMemcpy(out, dout, sizeof(double) * 73 * count, hipMemcpyDeviceToHost);
    (void)hipFree(dX);
    (void)hipFree(duv);
    (void)hipFree(dout);
    (void)hipFree(dm);
    return e == hipSuccess ? 0 : -1;
}

#ifdef VS_PNP_PROFILE
extern "C" int vs_debug_pnp_cycles(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_pnp_cycles), sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_pnp_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
