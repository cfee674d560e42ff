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

#ifndef VS_PNP_JACOBI
#define VS_PNP_JACOBI 2  // 0: the round-2 single-copy Jacobi (shuffled angles, two barriers per round); 1: every lane its two angles;
                         // 2: ping-pong, each angle computed once (lanes 36..41) and read from LDS (1 -> 2: Jacobi -7 %)
#endif

#ifdef VS_PNP_PROFILE
// k_pnp_hyp phase cycle counters (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_pnp_cycles[16];  // 0-5 k_pnp_hyp, 6-7 k_pnp_ransac, 8-12 its LM split
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

__device__ __forceinline__ const int* pnp_subset(const PnpHyp& H, int pb, int n, int h) {
    return H.tab_n0 >= 0 ? H.subset + ((size_t)(n - H.tab_n0) * H.stride + h) * 5
                         : H.subset + ((size_t)pb * H.stride + h) * 5;
}

__device__ __attribute__((noinline)) bool epnp_subset(const float* obj, const float* img, const int* idx, int m, const Cam& K, double* rv,
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

__device__ inline bool pnp_problem_runs(int n, int min_inliers, int model_points) {
    return !(n < min_inliers || n < 4) && n != model_points;
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

// 2. one hypothesis per wave64 workgroup: EPnP on its subset with the 12 x 12 eigen-decomposition
//    spread over the wave (LDS-resident round-robin Jacobi: a round's 6 disjoint rotations run in
//    parallel with the per-element arithmetic of the sequential sym_eig_rr<12>, so the model is
//    bit-identical to the host's), the three beta
//    approximations on lanes 0-2, then the inlier count over all points by the whole wave.
__global__ __launch_bounds__(64) void k_pnp_hyp(const float* __restrict__ obj_all, const float* __restrict__ img_all,
                                                const int* __restrict__ off, double fx, double fy, double cx, double cy,
                                                int niters0, float thr2, int min_inliers, PnpHyp H) {
    crit_prio();
#if VS_PNP_JACOBI >= 1
    __shared__ double sAb[2][144], sVb[2][144];  // ping-pong matrices: one barrier per Jacobi round
    [[maybe_unused]] __shared__ double sC[6], sS[6];  // VS_PNP_JACOBI 2: the round's angles
    [[maybe_unused]] __shared__ int sAct[6];
    double* sA = sAb[0];
    double* sV = sVb[0];
#else
    __shared__ double sA[144], sV[144];
#endif
    __shared__ double sX[15], sUV[10], sAl[5][4], sCw[4][3];
    __shared__ double sTot, sOff, sErr[3], sRt[3][12];
    __shared__ int sOk, sPerm[12];
    const int pb = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
    const int o0 = off[pb], n = off[pb + 1] - o0;
    const int model_points = n == 4 ? 4 : 5;
    if (h >= niters0 || !pnp_problem_runs(n, min_inliers, model_points)) return;
    const float* obj = obj_all + 3 * (size_t)o0;
    const float* img = img_all + 2 * (size_t)o0;
    const Cam K{fx, fy, cx, cy};
    const int* idx = pnp_subset(H, pb, n, h);
    const int m = model_points;
    PNP_T0();
    if (lane < m) {
        const int i = idx[lane];
        sX[3 * lane] = obj[3 * i];
        sX[3 * lane + 1] = obj[3 * i + 1];
        sX[3 * lane + 2] = obj[3 * i + 2];
        sUV[2 * lane] = img[2 * i];
        sUV[2 * lane + 1] = img[2 * i + 1];
    }
    __syncthreads();
    if (lane == 0) {
        double cw[4][3], al[5][4];
        sOk = epnp_control(sX, m, cw, al);
        for (int i = 0; i < 4; i++)
            for (int c = 0; c < 3; c++) sCw[i][c] = cw[i][c];
        for (int i = 0; i < m; i++)
            for (int j = 0; j < 4; j++) sAl[i][j] = al[i][j];
    }
    __syncthreads();
    PNP_T(0);
    bool ok = sOk != 0;
    if (ok) {
        for (int e = lane; e < 144; e += 64) {
            sA[e] = epnp_mtm<5>(sAl, sUV, m, K, e / 12, e % 12);
            sV[e] = (e / 12 == e % 12) ? 1.0 : 0.0;
        }
        __syncthreads();
        // sym_eig_rr<12> (pnp_solvers.h): the 6 disjoint rotations of each round in parallel
        if (lane == 0) {
            double total = 0;
            for (int i = 0; i < 144; i++) total += sA[i] * sA[i];
            sTot = total;
        }
        __syncthreads();
        PNP_T(1);
        const double total = sTot;
#if VS_PNP_JACOBI >= 1
        // Round-robin Jacobi with the matrices ping-ponged between two LDS copies: every lane of
        // 0..35 reads its 2 x 2 block (pair a rows i0 < i1, pair b columns j0 < j1), its V entries
        // (rows 2a, 2a + 1 at the block's columns) and the two diagonal blocks of its pairs from the
        // round's copy, computes both angles itself (no shuffles; the same inputs as the diagonal
        // lane's, so the same angles), rotates (column b, then row a, as the sequential statement)
        // and writes every value to the other copy; one barrier per round.  VS_PNP_JACOBI 2 (the
        // default): lanes 36..41 compute the round's six angles once (same inputs, same angles) and the
        // block lanes read theirs from LDS.  Bit-identical to sym_eig_rr<12>.
        {
            const int ba = lane / 6, bb = lane % 6;
            const bool blk = lane < 36;
            int pk[11];  // the lane's round pairs, packed 4 bits each (rounds unrolled: static indices)
#pragma unroll
            for (int r = 0; r < 11; r++) {
                int a0, a1, b0, b1;
                rr_pair(12, r, ba, a0, a1);
                rr_pair(12, r, bb, b0, b1);
                pk[r] = a0 | a1 << 4 | b0 << 8 | b1 << 12;
            }
            int cur = 0;
            for (int sweep = 0; sweep < 30; sweep++) {
                if (lane == 0) {
                    const double* A = sAb[cur];
                    double o = 0;
                    for (int p = 0; p < 12; p++)
                        for (int q = p + 1; q < 12; q++) o += A[p * 12 + q] * A[p * 12 + q];
                    sOff = o;
                }
                __syncthreads();
                if (!(sOff > 1e-32 * total)) break;
#pragma unroll
                for (int r = 0; r < 11; r++) {
                    const double* A = sAb[cur];
                    const double* V = sVb[cur];
                    double* An = sAb[cur ^ 1];
                    double* Vn = sVb[cur ^ 1];
#if VS_PNP_JACOBI == 2
                    if (lane >= 36 && lane < 42) {  // pair k's angle once (the same inputs as every user's)
                        int p0, q0;
                        rr_pair(12, r, lane - 36, p0, q0);
                        double c, sn;
                        const bool act = jacobi_angle_nb(A[p0 * 12 + p0], A[q0 * 12 + q0], A[p0 * 12 + q0], c, sn);
                        sC[lane - 36] = c;
                        sS[lane - 36] = sn;
                        sAct[lane - 36] = act;
                    }
                    __syncthreads();
#endif
                    if (blk) {
                        const int i0 = pk[r] & 15, i1 = (pk[r] >> 4) & 15, j0 = (pk[r] >> 8) & 15, j1 = pk[r] >> 12;
                        double x00 = A[i0 * 12 + j0], x01 = A[i0 * 12 + j1], x10 = A[i1 * 12 + j0], x11 = A[i1 * 12 + j1];
                        const double p0 = V[(2 * ba) * 12 + j0], q0 = V[(2 * ba) * 12 + j1];
                        const double p1 = V[(2 * ba + 1) * 12 + j0], q1 = V[(2 * ba + 1) * 12 + j1];
#if VS_PNP_JACOBI == 2
                        const double ca = sC[ba], sa = sS[ba], cb = sC[bb], sb = sS[bb];
                        const bool acta = sAct[ba] != 0, actb = sAct[bb] != 0;
#else
                        // both angles branch-free (jacobi_angle_nb) and the skipped rotations as
                        // selects: one straight-line block per round, the two angle chains interleaved
                        double ca, sa, cb, sb;
                        const bool acta = jacobi_angle_nb(A[i0 * 12 + i0], A[i1 * 12 + i1], A[i0 * 12 + i1], ca, sa);
                        const bool actb = jacobi_angle_nb(A[j0 * 12 + j0], A[j1 * 12 + j1], A[j0 * 12 + j1], cb, sb);
#endif
                        {
                            const double y00 = cb * x00 - sb * x01, y01 = sb * x00 + cb * x01;
                            const double y10 = cb * x10 - sb * x11, y11 = sb * x10 + cb * x11;
                            x00 = actb ? y00 : x00;
                            x01 = actb ? y01 : x01;
                            x10 = actb ? y10 : x10;
                            x11 = actb ? y11 : x11;
                        }
                        {
                            const double y00 = ca * x00 - sa * x10, y10 = sa * x00 + ca * x10;
                            const double y01 = ca * x01 - sa * x11, y11 = sa * x01 + ca * x11;
                            x00 = acta ? y00 : x00;
                            x01 = acta ? y01 : x01;
                            x10 = acta ? y10 : x10;
                            x11 = acta ? y11 : x11;
                        }
                        An[i0 * 12 + j0] = x00;
                        An[i0 * 12 + j1] = x01;
                        An[i1 * 12 + j0] = x10;
                        An[i1 * 12 + j1] = x11;
                        const double v0 = cb * p0 - sb * q0, w0 = sb * p0 + cb * q0;
                        const double v1 = cb * p1 - sb * q1, w1 = sb * p1 + cb * q1;
                        Vn[(2 * ba) * 12 + j0] = actb ? v0 : p0;
                        Vn[(2 * ba) * 12 + j1] = actb ? w0 : q0;
                        Vn[(2 * ba + 1) * 12 + j0] = actb ? v1 : p1;
                        Vn[(2 * ba + 1) * 12 + j1] = actb ? w1 : q1;
                    }
                    cur ^= 1;
                    __syncthreads();
                }
            }
            sA = sAb[cur];
            sV = sVb[cur];
        }
#else
        for (int sweep = 0; sweep < 30; sweep++) {
            if (lane == 0) {
                double o = 0;
                for (int p = 0; p < 12; p++)
                    for (int q = p + 1; q < 12; q++) o += sA[p * 12 + q] * sA[p * 12 + q];
                sOff = o;
            }
            __syncthreads();
            if (!(sOff > 1e-32 * total)) break;
            // Each lane of 0..35 keeps one 2 x 2 block of A in registers for the round: (pair a rows
            // i0 < i1, pair b columns j0 < j1), a = lane / 6, b = lane % 6.  The diagonal-block lanes
            // (a == b) compute the round's angles from their registers and shuffle them out; every
            // block takes its column rotation (b) and then its row rotation (a) -- per element exactly
            // the sequential statement's column-then-row order; V's rows 2a, 2a + 1 take the column
            // rotation of pair b in the same lane; the blocks go back to the LDS matrix and the next
            // round's blocks are read.
            const int ba = lane / 6, bb = lane % 6;
            const bool blk = lane < 36;
            int i0, i1, j0, j1;
            double x00 = 0, x01 = 0, x10 = 0, x11 = 0, p0 = 0, q0 = 0, p1 = 0, q1 = 0;
            // the round's A block and the V entries (rows 2a, 2a + 1 at the block's columns)
            int pk[11];  // the lane's round pairs, packed 4 bits each (rounds unrolled: static indices)
#pragma unroll
            for (int r = 0; r < 11; r++) {
                int a0, a1, b0, b1;
                rr_pair(12, r, ba, a0, a1);
                rr_pair(12, r, bb, b0, b1);
                pk[r] = a0 | a1 << 4 | b0 << 8 | b1 << 12;
            }
            auto load_blk = [&](int r) {
                i0 = pk[r] & 15;
                i1 = (pk[r] >> 4) & 15;
                j0 = (pk[r] >> 8) & 15;
                j1 = pk[r] >> 12;
                x00 = sA[i0 * 12 + j0];
                x01 = sA[i0 * 12 + j1];
                x10 = sA[i1 * 12 + j0];
                x11 = sA[i1 * 12 + j1];
                p0 = sV[(2 * ba) * 12 + j0];
                q0 = sV[(2 * ba) * 12 + j1];
                p1 = sV[(2 * ba + 1) * 12 + j0];
                q1 = sV[(2 * ba + 1) * 12 + j1];
            };
            if (blk) load_blk(0);
#pragma unroll
            for (int r = 0; r < 11; r++) {
                double c = 1.0, sn = 0.0;
                int act = 0;
                if (blk && ba == bb) act = jacobi_angle(x00, x11, x01, c, sn);  // (A[p][p], A[q][q], A[p][q])
                const double ca = __shfl(c, 7 * ba), sa = __shfl(sn, 7 * ba);
                const double cb = __shfl(c, 7 * bb), sb = __shfl(sn, 7 * bb);
                const int acta = __shfl(act, 7 * ba), actb = __shfl(act, 7 * bb);
                if (blk) {
                    if (actb) {
                        const double y00 = cb * x00 - sb * x01, y01 = sb * x00 + cb * x01;
                        const double y10 = cb * x10 - sb * x11, y11 = sb * x10 + cb * x11;
                        x00 = y00;
                        x01 = y01;
                        x10 = y10;
                        x11 = y11;
                    }
                    if (acta) {
                        const double y00 = ca * x00 - sa * x10, y10 = sa * x00 + ca * x10;
                        const double y01 = ca * x01 - sa * x11, y11 = sa * x01 + ca * x11;
                        x00 = y00;
                        x01 = y01;
                        x10 = y10;
                        x11 = y11;
                    }
                    sA[i0 * 12 + j0] = x00;
                    sA[i0 * 12 + j1] = x01;
                    sA[i1 * 12 + j0] = x10;
                    sA[i1 * 12 + j1] = x11;
                }
                // V's rows 2a, 2a + 1 at this block's column pair b take the column rotation the
                // lane already holds for A (each V entry once per round, no shuffles)
                if (blk && actb) {
                    sV[(2 * ba) * 12 + j0] = cb * p0 - sb * q0;
                    sV[(2 * ba) * 12 + j1] = sb * p0 + cb * q0;
                    sV[(2 * ba + 1) * 12 + j0] = cb * p1 - sb * q1;
                    sV[(2 * ba + 1) * 12 + j1] = sb * p1 + cb * q1;
                }
                __syncthreads();
                if (blk && r + 1 < 11) load_blk(r + 1);  // the next round's block
                __syncthreads();
            }
        }
#endif
        PNP_T(2);
        // eigenvalues in descending order, columns of V swapped along (sym_eig_rr's selection
        // sort): lane 0 runs the sort on the eigenvalues and a column index, the wave moves the
        // columns once (the same moves as swapping them step by step)
        if (lane == 0) {
            double w[12];
            int pm[12];
#pragma unroll
            for (int i = 0; i < 12; i++) {
                w[i] = sA[i * 12 + i];
                pm[i] = i;
            }
#pragma unroll
            for (int i = 0; i < 11; i++) {
                int mx = i;
                double wm = w[i];
#pragma unroll
                for (int j = i + 1; j < 12; j++)
                    if (w[j] > wm) {
                        mx = j;
                        wm = w[j];
                    }
                // swap entries i and mx with compile-time indices only (the arrays stay in registers)
                int pmx = pm[i];
#pragma unroll
                for (int j = i + 1; j < 12; j++) pmx = j == mx ? pm[j] : pmx;
#pragma unroll
                for (int j = i + 1; j < 12; j++)
                    if (j == mx) {
                        w[j] = w[i];
                        pm[j] = pm[i];
                    }
                w[i] = wm;
                pm[i] = pmx;
            }
#pragma unroll
            for (int i = 0; i < 12; i++) sPerm[i] = pm[i];
        }
        __syncthreads();
        {
            double tv[3];
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int e = lane + 64 * u;
                if (e < 144) tv[u] = sV[(e / 12) * 12 + sPerm[e % 12]];
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int e = lane + 64 * u;
                if (e < 144) sV[e] = tv[u];
            }
        }
        __syncthreads();
        PNP_T(3);
        if (lane < 3) {  // one beta approximation per lane
            double cw[4][3], v[4][12], L[6][10], rho[6], al[5][4], X[15], uv[10];
            for (int i = 0; i < 4; i++)
                for (int c = 0; c < 3; c++) cw[i][c] = sCw[i][c];
            // constant bounds (m <= 5): the copies unroll and the arrays stay in registers
#pragma unroll
            for (int i = 0; i < 5; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) al[i][j] = i < m ? sAl[i][j] : 0.0;
#pragma unroll
            for (int i = 0; i < 15; i++) X[i] = i < 3 * m ? sX[i] : 0.0;
#pragma unroll
            for (int i = 0; i < 10; i++) uv[i] = i < 2 * m ? sUV[i] : 0.0;
            epnp_L_rho(sV, cw, v, L, rho);
            double R[9], t[3];
            // the three approximations as one code path on lanes 0..2 (pnp_solvers.h
            // epnp_betas_init_uniform: bit-identical to epnp_variant's divergent solves)
            double be[4];
            epnp_betas_init_uniform(lane, L, rho, be);
            sErr[lane] = epnp_refine<5>(be, L, rho, v, al, X, uv, m, K, R, t);
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
        int c = 0;
        for (int i = lane; i < n; i += 64)
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

}  // namespace vs

#ifdef VS_PNP_PROFILE
extern "C" int vs_debug_pnp_cycles(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_pnp_cycles), sizeof(unsigned long long) * 16) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_pnp_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
