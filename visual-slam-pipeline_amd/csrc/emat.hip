// emat.hip — Slam::estimate_motion (reference src/Slam.cpp:1193-1213: cv::findEssentialMat(K,
// RANSAC, 0.999, 1.0 px) + cv::recoverPose + the inlier and determinant checks) and the depth scale
// (Slam::estimate_scale_from_depth / _single_depth, :73-207) on gfx950.
//
// The reference runs this path when the 3D-3D estimate fails (Slam.cpp:965-984), so in the pipeline
// a problem whose 3D-3D result is ok exits at once.  RANSAC (round 6): one 5-point solve per wave64,
// spread over the wave's lanes (five_point_wave: the host's stage arithmetic, bit-identical models);
// subsets from the context's table (the cv::RNG stream depends on the point count only); a problem's
// first 8 G iterations on G workgroups of 8 waves at once, every model's inlier count (Sampson
// error, ballot counts), then the problem's last workgroup to arrive replays the accept / budget
// sequence in order and, while the budget asks for more, continues alone in rounds of 8 (early exit
// below the current best).  recoverPose: the cheirality test of every point under the four
// decompositions in parallel.  Scale: per-point candidates sorted in LDS (bitonic), IQR filter,
// median.  Numerical kernels shared with the CPU restatement (emat_solvers.h, -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "emat_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_em;

constexpr int kEmMaxPts = VS_EM_MAX_POINTS;
constexpr int kEmWaves = 8;  // one RANSAC iteration per wave; 8 wave64s (2 per SIMD, <= 256 VGPRs)
constexpr int kEmThreads = 64 * kEmWaves;
constexpr int kEmIters = 1000;  // findEssentialMat's maxIters

__device__ inline int wave_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// a lane's double, read by the whole wave (uniform lane index: two v_readlane into SGPRs)
__device__ __forceinline__ double em_bcast(double x, int src) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// LDS written by some lanes of a wave, then read by others of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one wave's 5-point workspace (LDS)
struct EmWave {
    double B[36];       // the rotated null-space basis E0..E3, row-major
    double AA[200];     // the 10 x 20 coefficient matrix (stage 2), then the reduced columns 10..19
    double bx[3][4], by[3][4], b1[3][5];
    double C[12], R[12];  // a level's cuts; the previous level's roots
    double E[kMaxModels * 9];
    int nc;
};

// The 5-point solver (emat_solvers.h five_point) on one wave: every lane holds the same 5
// correspondences; the stages run the host's arithmetic, spread where they are independent —
// the 20 coefficient columns one per lane, Gauss-Jordan with column c in lane c (pivot and row
// multipliers broadcast from lane k), every monotone interval of a derivative level on its own lane
// (the roots then gathered in interval order with the host's rule), one root's model per lane —
// so the models are bit-identical to the host's, in the same order.  Writes W.E, returns the count.
__device__ __forceinline__ int five_point_wave(const double* q1, const double* q2, EmWave& W, int lane,
                                               long long* ck = nullptr) {
#define EM_CK(i)                                  \
    do {                                          \
        if (ck && lane == 0) ck[i] = wall_clock64(); \
    } while (0)
    EM_CK(0);
    {
        double B[4][9];
        if (!fp_basis(q1, q2, B)) return 0;  // uniform
        if (lane == 0) {
#pragma unroll
            for (int e = 0; e < 36; e++) W.B[e] = B[e / 9][e % 9];
        }
    }
    wave_lds_sync();
    EM_CK(1);
    if (lane < 20) {  // stage 2: the monomial columns
        int i = 0, j = 0, k = 0, t = 0;
        for (int a = 0; a < 4; a++)
            for (int b = a; b < 4; b++)
                for (int c = b; c < 4; c++, t++)
                    if (t == lane) i = a, j = b, k = c;
        double acc[10];
        const int col = fp_column(W.B, i, j, k, acc);
#pragma unroll
        for (int r = 0; r < 10; r++) W.AA[r * 20 + col] = acc[r];
    }
    wave_lds_sync();
    EM_CK(2);
    // stage 3: Gauss-Jordan, lane c holding column c (the host updates columns >= k only)
    double a[10];
#pragma unroll
    for (int r = 0; r < 10; r++) a[r] = lane < 20 ? W.AA[r * 20 + lane] : 0.0;
#pragma unroll
    for (int k = 0; k < 10; k++) {
        int p = k;
        double big = fabs(a[k]);
#pragma unroll
        for (int r = k + 1; r < 10; r++) {
            const double v = fabs(a[r]);
            if (v > big) {
                big = v;
                p = r;
            }
        }
        p = __builtin_amdgcn_readlane(p, k);
        big = em_bcast(big, k);
        if (!(big > 1e-300)) return 0;
        const bool act = lane >= k;
        double pkc = a[k];
#pragma unroll
        for (int r = k + 1; r < 10; r++) pkc = r == p ? a[r] : pkc;
#pragma unroll
        for (int r = k + 1; r < 10; r++)
            if (r == p && act) a[r] = a[k];  // the pivot row moves to row p
        const double inv = 1.0 / em_bcast(pkc, k);
        if (act) {
            pkc *= inv;
            a[k] = pkc;
        }
#pragma unroll
        for (int r = 0; r < 10; r++) {
            if (r == k) continue;
            const double f = em_bcast(a[r], k);
            if (f == 0) continue;
            if (act) a[r] = a[r] - f * pkc;
        }
    }
    if (lane >= 10 && lane < 20) {
#pragma unroll
        for (int r = 0; r < 10; r++) W.AA[r * 20 + lane] = a[r];
    }
    wave_lds_sync();
    EM_CK(3);
    // stage 4 (uniform): B(z) and its determinant
    double cp[11];
    {
        double bx[3][4], by[3][4], b1[3][5];
        fp_bpoly(W.AA, 1, bx, by, b1, cp);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 3; i++) {
#pragma unroll
                for (int q = 0; q < 4; q++) W.bx[i][q] = bx[i][q], W.by[i][q] = by[i][q];
#pragma unroll
                for (int q = 0; q < 5; q++) W.b1[i][q] = b1[i][q];
            }
        }
    }
    EM_CK(4);
    // stage 5: the real roots, one monotone interval per lane at every derivative level
    double bound;
    const int n = roots_degree_bound(cp, bound);
    int nr = 0;
    if (n > 0) {
#pragma unroll
        for (int m = 9; m >= 0; m--) {
            if (m > n - 1) continue;
            double D[11];
            roots_deriv(cp, n, m, D);
            if (lane == 0) {
                int q = 0;
                W.C[q++] = -bound;
                for (int i = 0; i < nr; i++) {
                    const double ri = W.R[i];
                    if (ri > -bound && ri < bound) W.C[q++] = ri;
                }
                W.C[q++] = bound;
                W.nc = q;
            }
            wave_lds_sync();
            const int nc = W.nc;
            int kind = 0;
            double r = 0;
            if (lane + 1 < nc) kind = roots_interval(D, m, lane, W.C[lane], W.C[lane + 1], r);
            // in interval order: an at-root cut repeating the last root found is the same root
            unsigned long long msk = __ballot(kind != 0);
            int cnt = 0;
            double last = 0;
            while (msk) {
                const int l = __ffsll((long long)msk) - 1;
                msk &= msk - 1;
                const int kl = __builtin_amdgcn_readlane(kind, l);
                const double vl = em_bcast(r, l);
                if (kl == 1 && !(cnt == 0 || last != vl)) continue;
                if (lane == 0) W.R[cnt] = vl;
                last = vl;
                cnt++;
            }
            nr = cnt;
            wave_lds_sync();
        }
    }
    EM_CK(5);
    // stage 6: one root's model per lane, kept in root order
    bool ok = false;
    double e[9];
    if (lane < nr) ok = fp_model(W.R[lane], W.bx, W.by, W.b1, W.B, e);
    const unsigned long long msk = __ballot(ok);
    const int slot = __popcll(msk & ((1ull << lane) - 1));
    if (ok && slot < kMaxModels) {
#pragma unroll
        for (int q = 0; q < 9; q++) W.E[slot * 9 + q] = e[q];
    }
    wave_lds_sync();
    EM_CK(6);
#undef EM_CK
    const int cntm = __popcll(msk);
    return cntm < kMaxModels ? cntm : kMaxModels;
}

// The first rounds of a problem are split over G workgroups; their models and counts meet here
// (per problem, kEmSyncBytes): arrival counter, iteration bound, then per iteration of the budget.
struct EmSync {
    int arrived;
    int bound_enc;  // 0: no bound yet; else kEmBoundBase - (the smallest published iteration bound)
    int pad[14];
    int nmod[kEmIters];
    int count[kEmIters * kMaxModels];
    double model[kEmIters * kMaxModels * 9];
};
constexpr int kEmBoundBase = 1 << 20;
static_assert(sizeof(EmSync) <= kEmSyncBytes, "EmSync");

struct EmShared {
    float px1[2 * kEmMaxPts], px2[2 * kEmMaxPts];  // pixels (the scale estimators use them)
    double q1[2 * kEmMaxPts], q2[2 * kEmMaxPts];   // normalised
    union {
        EmWave wv[kEmWaves];
        double sv[2 * kEmMaxPts];  // scale candidates (sorted), after RANSAC
    };
    int nmod[kEmWaves];
    int score[kEmWaves * kMaxModels];
    int rcnt[64][kMaxModels];  // the replay's counts of 64 iterations
    double E[9], R1[9], R2[9], t[3], tn[3];
    int niters, best, best_iter, iter, done, ok, chunk, cnt[4], nsv, last;
    unsigned char mask[kEmMaxPts];
};

// ascending bitonic sort of S.sv[0..n) padded with +inf to a power of two (<= 2 * kEmMaxPts)
__device__ void sort_sv(EmShared& S, int n) {
    int m = 1;
    while (m < n) m <<= 1;
    for (int i = n + threadIdx.x; i < m; i += blockDim.x) S.sv[i] = __builtin_inf();
    __syncthreads();
    for (int k = 2; k <= m; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < m; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const double a = S.sv[i], b = S.sv[l];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        S.sv[i] = b;
                        S.sv[l] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// the inlier count of model E over the problem's points by one wave; -1 as soon as it cannot exceed
// bar (a count <= bar is never accepted, so the early exit changes no decision)
__device__ inline int em_count(const EmShared& S, const double* E, int n, float thr2, int bar, int lane) {
    int cnt = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const bool in = i < n && sampson_err(E, S.q1[2 * i], S.q1[2 * i + 1], S.q2[2 * i], S.q2[2 * i + 1]) <= thr2;
        cnt += __popcll(__ballot(in));
        if (cnt + max(0, n - i0 - 64) <= bar) return -1;
    }
    return cnt;
}

// this wave's iteration: subset from the context's table (row n - kEmTabMinN; n == 5: the points
// themselves, findEssentialMat's single kernel run), the wave's models into its EmWave
__device__ __forceinline__ int em_solve(const EmShared& S, EmWave& W, const int* __restrict__ tab, int n, int it, int lane) {
    int idx[5];
    if (n == 5) {
#pragma unroll
        for (int i = 0; i < 5; i++) idx[i] = i;
    } else {
        const int* sub = tab + ((size_t)(n - kEmTabMinN) * kEmIters + it) * 5;
#pragma unroll
        for (int i = 0; i < 5; i++) idx[i] = sub[i];
    }
    double s1[10], s2[10];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        s1[2 * i] = S.q1[2 * idx[i]];
        s1[2 * i + 1] = S.q1[2 * idx[i] + 1];
        s2[2 * i] = S.q2[2 * idx[i]];
        s2[2 * i + 1] = S.q2[2 * idx[i] + 1];
    }
    return five_point_wave(s1, s2, W, lane);
}

// Problem source: FROM_PAIRS = frame pairs (pipeline: kept matches, keypoints, depth slots), else
// point arrays with offsets (ABI single problem, depth1/depth2 host-uploaded or null).
// out: R [p][9], t [p][3], scale [p], ok [p], diag [p][8] = {E found, iterations, winning iteration,
// E inliers, recoverPose good, n, ran, 0}
// Grid: P x G workgroups (G = split).  Workgroup g solves iterations 8 g .. 8 g + 7 (one per wave) and
// counts every model's inliers; the problem's last workgroup to arrive (agent-scope acq_rel counter in
// sync, re-armed by itself) replays the accept / budget sequence over the 8 G iterations in order,
// continues alone in rounds of 8 while the budget asks for more, then runs recoverPose and the scale.
template <bool FROM_PAIRS>
__global__ __launch_bounds__(kEmThreads) void k_emat(const int* __restrict__ pairs, const vs_keypoint* __restrict__ kps,
                                                     int cap, const vs_match* __restrict__ kept,
                                                     const int* __restrict__ nkept, const int* __restrict__ skip,
                                                     const float* __restrict__ pts1, const float* __restrict__ pts2,
                                                     const int* __restrict__ off, const float* __restrict__ depth,
                                                     const float* __restrict__ depth1, const float* __restrict__ depth2,
                                                     int h, int w, double fx, double fy, double cx, double cy,
                                                     double* __restrict__ R_out, double* __restrict__ t_out,
                                                     double* __restrict__ scale_out, int* __restrict__ ok_out,
                                                     int* __restrict__ diag, const int* __restrict__ tab, int G,
                                                     char* __restrict__ sync) {
    __shared__ EmShared S;
    __shared__ int red_cnt[4 * kEmWaves];
    const int P = gridDim.x / G, gw = blockIdx.x / P, pb = blockIdx.x - gw * P, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int* dg = diag + 8 * pb;
    if (gw == 0 && tid == 0) {
        for (int k = 0; k < 8; k++) dg[k] = 0;
        dg[2] = -1;
        ok_out[pb] = 0;
        scale_out[pb] = -1.0;
    }
    if (skip && skip[pb]) return;  // 3D-3D succeeded: the reference never reaches estimate_motion
    int n;
    const float *d1 = nullptr, *d2 = nullptr;
    if (FROM_PAIRS) {
        n = min(nkept[pb], cap);
        const vs_match* gm = kept + (size_t)pb * cap;
        const vs_keypoint* kr = kps + (size_t)pairs[2 * pb] * cap;
        const vs_keypoint* kc = kps + (size_t)pairs[2 * pb + 1] * cap;
        for (int i = tid; i < n; i += blockDim.x) {
            const vs_match m = gm[i];
            S.px1[2 * i] = kr[m.query_idx].x;
            S.px1[2 * i + 1] = kr[m.query_idx].y;
            S.px2[2 * i] = kc[m.train_idx].x;
            S.px2[2 * i + 1] = kc[m.train_idx].y;
        }
        d1 = depth ? depth + (size_t)pairs[2 * pb] * h * w : nullptr;  // null: monocular, no scale
        d2 = depth ? depth + (size_t)pairs[2 * pb + 1] * h * w : nullptr;
    } else {
        const int o0 = off[pb];
        n = off[pb + 1] - o0;
        for (int i = tid; i < 2 * n; i += blockDim.x) {
            S.px1[i] = pts1[2 * (size_t)o0 + i];
            S.px2[i] = pts2[2 * (size_t)o0 + i];
        }
        d1 = depth1;
        d2 = depth2;
    }
    if (gw == 0 && tid == 0) dg[5] = n;
    if (n < 5 || (n == 5 && gw > 0)) return;  // Slam.cpp:1195; n == 5: workgroup 0 alone
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        S.q1[2 * i] = ((double)S.px1[2 * i] - cx) / fx;
        S.q1[2 * i + 1] = ((double)S.px1[2 * i + 1] - cy) / fy;
        S.q2[2 * i] = ((double)S.px2[2 * i] - cx) / fx;
        S.q2[2 * i + 1] = ((double)S.px2[2 * i + 1] - cy) / fy;
    }
    __syncthreads();
    const double thr = 1.0 / ((fx + fy) / 2);
    const float thr2 = (float)(thr * thr);
    EmWave& W = S.wv[wv];
    // ---- RANSAC (RANSACPointSetRegistrator, 5 model points); n == 5: one kernel run, first model ----
    // Round 0: iterations 8 gw .. 8 gw + 7 on workgroup gw (ga = 8 G of them), every model's full inlier
    // count into sync.  A workgroup publishes, for each of its iterations j with a count c > 4, the bound
    // max(j + 1, RANSACUpdateNumIters(c, 1000)) on the iterations the sequential loop can run: if j is
    // reached, the running budget is at most that update from then on (the update is monotone in the
    // count and in the budget it starts from); if it is not, the loop ended before j.  Iterations at or
    // beyond the smallest published bound are never read by the replay, so a workgroup skips them.
    // Later rounds (the last workgroup alone, when the budget exceeds ga): 8 iterations from S.iter,
    // counts with the early exit below the round's starting best.  One solve site (em_solve inlined once).
    const int ga = min(kEmWaves * G, kEmIters);
    EmSync* sy = reinterpret_cast<EmSync*>(sync + (size_t)pb * kEmSyncBytes);
    for (int round = 0;; round++) {
        int it, bar = -1;
        bool run;
        if (n == 5) {
            it = 0;
            run = wv == 0;
        } else if (round == 0) {
            it = kEmWaves * gw + wv;
            const int enc = __hip_atomic_load(&sy->bound_enc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            run = it < ga && (enc == 0 || it < kEmBoundBase - enc);
        } else {
            it = S.iter + wv;
            run = it < S.niters;
            bar = S.best > 4 ? S.best : 4;
        }
        if (run) {
            const int nm = em_solve(S, W, tab, n, it, lane);
            if (n == 5) {
                if (lane == 0) {
                    S.ok = nm > 0;
                    for (int k = 0; k < 9; k++) S.E[k] = W.E[k];
                }
            } else if (round == 0) {
                int cmax = -1;
                for (int k = 0; k < nm; k++) {
                    const int c = em_count(S, &W.E[9 * k], n, thr2, -1, lane);
                    cmax = c > cmax ? c : cmax;
                    if (lane == 0) sy->count[it * kMaxModels + k] = c;
                }
                for (int q = lane; q < 9 * nm; q += 64) sy->model[it * kMaxModels * 9 + q] = W.E[q];
                if (lane == 0) {
                    sy->nmod[it] = nm;
                    if (cmax > 4) {
                        const int u = vs_pnp::ransac_update_num_iters(0.999, (double)(n - cmax) / n, 5, kEmIters);
                        const int bnd = u > it + 1 ? u : it + 1;
                        __hip_atomic_fetch_max(&sy->bound_enc, kEmBoundBase - bnd, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            } else {
                for (int k = 0; k < nm; k++) {
                    const int c = em_count(S, &W.E[9 * k], n, thr2, bar, lane);
                    if (lane == 0) S.score[wv * kMaxModels + k] = c;
                }
                if (lane == 0) S.nmod[wv] = nm;
            }
        }
        if (n == 5) {
            if (tid == 0) {
                S.iter = 0;
                S.best_iter = -1;
            }
            __syncthreads();
            break;
        }
        if (round == 0) {
            if (G > 1) {
                __threadfence();
                __syncthreads();
                if (tid == 0) {
                    const int old = __hip_atomic_fetch_add(&sy->arrived, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                    S.last = old == G - 1;
                    if (S.last) {  // re-armed for the next launch
                        __hip_atomic_store(&sy->arrived, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&sy->bound_enc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                __syncthreads();
                if (!S.last) return;
                __threadfence();
            } else if (tid == 0) {
                __hip_atomic_store(&sy->bound_enc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            // The accept / budget replay over the first ga iterations on wave 0: a model is accepted iff its
            // count exceeds the running best (every earlier count, floor 4), so 64 iterations at a time give
            // their accepted models from one wave scan; only those are walked in order, each applying the
            // budget update, stopping at the first iteration at or beyond the running budget.
            if (wv == 0) {
                int niters = kEmIters, best = 0, best_iter = -1, best_k = 0, floor_max = 4;
                bool stop = false;
                for (int base = 0; base < ga && base < niters && !stop; base += 64) {
                    const int i = base + lane;
                    int nm = i < ga ? sy->nmod[i] : 0;  // (iterations never solved lie beyond the stop)
                    nm = nm < 0 ? 0 : nm > kMaxModels ? kMaxModels : nm;
                    int mi = -1;
                    for (int k = 0; k < nm; k++) {
                        const int c = sy->count[i * kMaxModels + k];
                        S.rcnt[lane][k] = c;
                        mi = c > mi ? c : mi;
                    }
                    int m = mi;  // inclusive prefix maximum over the chunk
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int t = __shfl_up(m, o);
                        if (lane >= o) m = m > t ? m : t;
                    }
                    int ex = __shfl_up(m, 1);
                    if (lane == 0) ex = -1;
                    int run_best = ex > floor_max ? ex : floor_max;
                    unsigned bits = 0;
                    for (int k = 0; k < nm; k++) {
                        const int c = S.rcnt[lane][k];
                        if (c > run_best) {
                            bits |= 1u << k;
                            run_best = c;
                        }
                    }
                    wave_lds_sync();
                    unsigned long long acc = __ballot(bits != 0);
                    while (acc) {
                        const int l = __ffsll((long long)acc) - 1;
                        acc &= acc - 1;
                        const int j = base + l;
                        if (j >= niters) {
                            stop = true;
                            break;
                        }
                        unsigned bl = (unsigned)__builtin_amdgcn_readlane((int)bits, l);
                        while (bl) {
                            const int k = __ffs(bl) - 1;
                            bl &= bl - 1;
                            const int cnt = S.rcnt[l][k];
                            best = cnt;
                            best_iter = j;
                            best_k = k;
                            niters = vs_pnp::ransac_update_num_iters(0.999, (double)(n - cnt) / n, 5, niters);
                        }
                    }
                    const int cm = __shfl(m, 63);
                    floor_max = cm > floor_max ? cm : floor_max;
                    wave_lds_sync();
                }
                const int ran = niters > best_iter + 1 ? niters : best_iter + 1;
                if (lane == 0) {
                    S.niters = niters;
                    S.best = best;
                    S.best_iter = best_iter;
                    S.iter = ran < ga ? ran : ga;
                    S.done = S.iter >= niters;
                }
                if (best > 0 && lane < 9) S.E[lane] = sy->model[(best_iter * kMaxModels + best_k) * 9 + lane];
            }
        } else {
            __syncthreads();
            if (tid == 0) {
                const int chunk = min(kEmWaves, S.niters - S.iter);
                int i = S.iter;
                for (int q = 0; q < chunk && i < S.niters; q++, i++)
                    for (int k = 0; k < S.nmod[q]; k++) {
                        const int cnt = S.score[q * kMaxModels + k];
                        if (cnt > (S.best > 4 ? S.best : 4)) {
                            S.best = cnt;
                            S.best_iter = i;
                            for (int e = 0; e < 9; e++) S.E[e] = S.wv[q].E[9 * k + e];
                            S.niters = vs_pnp::ransac_update_num_iters(0.999, (double)(n - cnt) / n, 5, S.niters);
                        }
                    }
                S.iter = i;
                S.done = i >= S.niters;
            }
        }
        __syncthreads();
        if (S.done) {
            if (tid == 0) S.ok = S.best > 0;
            __syncthreads();
            break;
        }
    }
    if (tid == 0) {
        dg[0] = S.ok;
        dg[1] = S.iter;
        dg[2] = S.best_iter;
    }
    if (!S.ok) return;  // E.empty() (:1200)
    // ---- inliers of E (countNonZero(mask), :1202-1203) ----
    double E[9];
    for (int k = 0; k < 9; k++) E[k] = S.E[k];
    int local = 0;
    for (int i = tid; i < n; i += blockDim.x) {
        const bool in = n == 5 || sampson_err(E, S.q1[2 * i], S.q1[2 * i + 1], S.q2[2 * i], S.q2[2 * i + 1]) <= thr2;
        S.mask[i] = in;
        local += in;
    }
    local = wave_sum(local);
    if (lane == 0) red_cnt[wv] = local;
    __syncthreads();
    int inl = 0;
    for (int q = 0; q < kEmWaves; q++) inl += red_cnt[q];
    if (tid == 0) dg[3] = inl;
    __syncthreads();
    if (inl < 15) return;  // MIN_INLIERS
    // ---- recoverPose (distance 50) ----
    if (tid == 0) {
        decompose_essential(E, S.R1, S.R2, S.t);
        for (int k = 0; k < 3; k++) S.tn[k] = -S.t[k];
    }
    __syncthreads();
    const double* tn = S.tn;
    // one (point, decomposition) per work item: a single cheiral_ok site, inlined once
    int good[4] = {0, 0, 0, 0};
    for (int wi = tid; wi < 4 * n; wi += blockDim.x) {
        const int i = wi >> 2, c = wi & 3;
        if (!S.mask[i]) continue;
        const double x1 = S.q1[2 * i], y1 = S.q1[2 * i + 1], x2 = S.q2[2 * i], y2 = S.q2[2 * i + 1];
        const int ok = cheiral_ok((c & 1) ? S.R2 : S.R1, (c & 2) ? S.tn : S.t, x1, y1, x2, y2, 50.0);
        good[0] += c == 0 ? ok : 0;
        good[1] += c == 1 ? ok : 0;
        good[2] += c == 2 ? ok : 0;
        good[3] += c == 3 ? ok : 0;
    }
    for (int c = 0; c < 4; c++) {
        good[c] = wave_sum(good[c]);
        if (lane == 0) red_cnt[4 * wv + c] = good[c];
    }
    __syncthreads();
    int g[4] = {0, 0, 0, 0};
    for (int q = 0; q < kEmWaves; q++)
        for (int c = 0; c < 4; c++) g[c] += red_cnt[4 * q + c];
    int pick;
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3])
        pick = 0;
    else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3])
        pick = 1;
    else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3])
        pick = 2;
    else
        pick = 3;
    const double* Rp = (pick & 1) ? S.R2 : S.R1;
    double tp[3];
    for (int k = 0; k < 3; k++) tp[k] = pick >= 2 ? tn[k] : S.t[k];
    if (tid == 0) dg[4] = g[pick];
    if (g[pick] < 15) return;                               // :1206
    if (fabs(vs_pnp::det3(Rp) - 1.0) > 0.01) return;       // :1208-1209
    // ---- scale (Slam.cpp:73-156, 162-207) ----
    double sc = -1.0;
    if (d1) {
        bool single = d2 == nullptr;
        if (!single) {
            if (tid == 0) S.nsv = 0;
            __syncthreads();
            for (int i = tid; i < n; i += blockDim.x) {
                const float u1 = S.px1[2 * i], v1 = S.px1[2 * i + 1], u2 = S.px2[2 * i], v2 = S.px2[2 * i + 1];
                const int px1 = (int)roundf(u1), py1 = (int)roundf(v1), px2 = (int)roundf(u2), py2 = (int)roundf(v2);
                if (px1 < 0 || px1 >= w || py1 < 0 || py1 >= h) continue;
                if (px2 < 0 || px2 >= w || py2 < 0 || py2 >= h) continue;
                const float z1 = d1[(size_t)py1 * w + px1], z2 = d2[(size_t)py2 * w + px2];
                if (z1 <= 0.1f || z1 > 10.0f || z2 <= 0.1f || z2 > 10.0f) continue;
                const double P1[3] = {(u1 - cx) * z1 / fx, (v1 - cy) * z1 / fy, (double)z1};
                const double P2[3] = {(u2 - cx) * z2 / fx, (v2 - cy) * z2 / fy, (double)z2};
                double dff[3];
                for (int r = 0; r < 3; r++)
                    dff[r] = P2[r] - (Rp[r * 3] * P1[0] + Rp[r * 3 + 1] * P1[1] + Rp[r * 3 + 2] * P1[2]);
                const double s = dff[0] * tp[0] + dff[1] * tp[1] + dff[2] * tp[2];
                if (s > 0.001 && s < 50.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
            }
            __syncthreads();
            const int c = S.nsv;
            if (c < 10) {
                single = true;
            } else {
                sort_sv(S, c);
                const double q1 = S.sv[c / 4], q3 = S.sv[3 * c / 4];
                const double lo = q1 - 1.5 * (q3 - q1), hi = q3 + 1.5 * (q3 - q1);
                int i1 = 0, i2 = 0;  // the filtered values are the contiguous run [i1, i2)
                while (i1 < c && !(S.sv[i1] >= lo)) i1++;
                i2 = i1;
                while (i2 < c && S.sv[i2] <= hi) i2++;
                sc = i2 > i1 ? S.sv[i1 + (i2 - i1) / 2] : S.sv[c / 2];
            }
        }
        if (single) {
            __syncthreads();
            if (tid == 0) S.nsv = 0;
            __syncthreads();
            for (int i = tid; i < n; i += blockDim.x) {
                const float u1 = S.px1[2 * i], v1 = S.px1[2 * i + 1];
                const int px1 = (int)roundf(u1), py1 = (int)roundf(v1);
                if (px1 < 0 || px1 >= w || py1 < 0 || py1 >= h) continue;
                const float z1 = d1[(size_t)py1 * w + px1];
                if (z1 <= 0.1f || z1 > 10.0f) continue;
                const double X1 = (u1 - cx) * z1 / fx, Y1 = (v1 - cy) * z1 / fy, Z1 = z1;
                const double Rx = Rp[0] * X1 + Rp[1] * Y1 + Rp[2] * Z1, Ry = Rp[3] * X1 + Rp[4] * Y1 + Rp[5] * Z1,
                             Rz = Rp[6] * X1 + Rp[7] * Y1 + Rp[8] * Z1;
                const double a = (S.px2[2 * i] - cx) / fx, den_x = tp[0] - a * tp[2];
                if (fabs(den_x) > 1e-4) {
                    const double s = (a * Rz - Rx) / den_x;
                    if (s > 0.001 && s < 100.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
                }
                const double b = (S.px2[2 * i + 1] - cy) / fy, den_y = tp[1] - b * tp[2];
                if (fabs(den_y) > 1e-4) {
                    const double s = (b * Rz - Ry) / den_y;
                    if (s > 0.001 && s < 100.0) S.sv[atomicAdd(&S.nsv, 1)] = s;
                }
            }
            __syncthreads();
            const int c = S.nsv;
            if (c >= 10) {
                sort_sv(S, c);
                sc = S.sv[c / 2];
            } else {
                sc = -1.0;
            }
        }
    }
    if (tid == 0) {
        for (int k = 0; k < 9; k++) R_out[9 * pb + k] = Rp[k];
        for (int k = 0; k < 3; k++) t_out[3 * pb + k] = tp[k];
        scale_out[pb] = sc;
        ok_out[pb] = 1;
        dg[6] = 1;
    }
}

// The context's subset table: findEssentialMat's subsets depend on the point count only (the
// generator starts at cv::RNG((uint64)-1) on every call), so the full budget's are drawn once per
// context for every n in [kEmTabMinN, VS_EM_MAX_POINTS] (10 MB) by the PnP sampler (pnp.hip); built
// on first use and synchronised once, so that any stream may read it afterwards.
int emat_reserve(vs_ctx* ctx, hipStream_t s) {
    if (!ctx->em_tab_ready) {
        constexpr int rows = kEmMaxPts - kEmTabMinN + 1;
        VS_CHECK(ctx->em_tab.ensure((size_t)rows * kEmIters * 5 * sizeof(int)));
        VS_CHECK(subset_table(rows, kEmTabMinN, kEmIters, ctx->em_tab.as<int>(), s));
        VS_HIP(hipStreamSynchronize(s));
        ctx->em_tab_ready = true;
    }
    return VS_OK;
}

// the workgroup split and its meeting area.  Default: one problem (the ABI's single motion, latency-bound)
// the whole budget, kEmSplitMax workgroups; a batch of problems beside other streams (config[4]: the 32 pairs
// of a step beside the network) 8 — the solves' CU time, not their latency, is what such a step pays
// (profiles/r06em3_mono_split_ab.txt).  VS_EMAT_SPLIT=1..125 overrides both.
static int g_em_split_test = 0;  // vs_debug_emat_split (tests): forces every launch's split
static int em_launch_setup(vs_ctx* ctx, int P, int split, char** sync, hipStream_t s) {
    if (g_em_split_test > 0) split = g_em_split_test;
    static const int env_split = [] {
        const char* e = std::getenv("VS_EMAT_SPLIT");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 && v <= kEmSplitMax ? v : 0;
    }();
    if (split <= 0) split = env_split ? env_split : P == 1 ? kEmSplitMax : 8;
    VS_ARG(split <= kEmSplitMax, "emat: split above kEmSplitMax");
    VS_CHECK(emat_reserve(ctx, s));
    if (!*sync) {  // round 0 writes its models and counts there at every split, 1 included
        const size_t need = (size_t)P * kEmSyncBytes;
        if (ctx->em_sync.bytes < need) {
            VS_CHECK(ctx->em_sync.ensure(need));
            VS_HIP(hipMemsetAsync(ctx->em_sync.p, 0, ctx->em_sync.bytes, s));
        }
        *sync = ctx->em_sync.as<char>();
    }
    return split;
}

int emat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_kept,
               const int* d_nkept, const int* d_skip, const float* d_depth, int h, int w, const double K[4],
               double* d_R, double* d_t, double* d_scale, int* d_ok, int* d_diag, hipStream_t s, int split,
               char* d_sync) {
    if (P <= 0) return VS_OK;
    VS_ARG(!d_sync || P == 1, "emat_pairs: a caller's meeting area holds one problem");
    VS_ARG(cap <= kEmMaxPts, "emat_pairs: cap above VS_EM_MAX_POINTS");
    const int G = em_launch_setup(ctx, P, split, &d_sync, s);
    if (G < 0) return G;
    ProfScope ps(ctx, "emat_motion", s);
    hipLaunchKernelGGL(k_emat<true>, dim3(P * G), dim3(kEmThreads), 0, s, d_pairs, d_kps, cap, d_kept, d_nkept, d_skip,
                       nullptr, nullptr, nullptr, d_depth, nullptr, nullptr, h, w, K[0], K[1], K[2], K[3], d_R, d_t,
                       d_scale, d_ok, d_diag, ctx->em_tab.as<int>(), G, d_sync);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int emat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, const float* d_depth1,
                const float* d_depth2, int h, int w, const double K[4], double* d_R, double* d_t, double* d_scale,
                int* d_ok, int* d_diag, hipStream_t s) {
    if (P <= 0) return VS_OK;
    char* d_sync = nullptr;
    const int G = em_launch_setup(ctx, P, 0, &d_sync, s);
    if (G < 0) return G;
    ProfScope ps(ctx, "emat_motion", s);
    hipLaunchKernelGGL(k_emat<false>, dim3(P * G), dim3(kEmThreads), 0, s, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                       d_p1, d_p2, d_off, nullptr, d_depth1, d_depth2, h, w, K[0], K[1], K[2], K[3], d_R, d_t,
                       d_scale, d_ok, d_diag, ctx->em_tab.as<int>(), G, d_sync);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs

namespace vs {
// test hook: five_point_wave on count problems (one wave each): E_out [count][kMaxModels][9], nmod [count]
__global__ __launch_bounds__(64) void k_debug_five_point(const double* __restrict__ q1, const double* __restrict__ q2,
                                                         double* __restrict__ E_out, int* __restrict__ nmod,
                                                         long long* __restrict__ ck) {
    __shared__ EmWave W;
    const int p = blockIdx.x, lane = threadIdx.x;
    double s1[10], s2[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        s1[i] = q1[10 * (size_t)p + i];
        s2[i] = q2[10 * (size_t)p + i];
    }
    const int nm = five_point_wave(s1, s2, W, lane, ck ? ck + 8 * (size_t)p : nullptr);
    for (int q = lane; q < 9 * nm; q += 64) E_out[(size_t)p * kMaxModels * 9 + q] = W.E[q];
    if (lane == 0) nmod[p] = nm;
}
}  // namespace vs

// clocks (optional, [count][8]): wall_clock64 stamps after each stage of five_point_wave
extern "C" int vs_debug_five_point_ck(const double* q1, const double* q2, int count, double* E_out, int* nmod,
                                      long long* clocks);
// test hook: every later k_emat launch of the process uses `split` workgroups per problem (1..125; 0 restores
// the defaults), so the continuation rounds behind a small split are checked against the oracle
extern "C" int vs_debug_emat_split(int split) {
    if (split < 0 || split > vs::kEmSplitMax) return -1;
    vs::g_em_split_test = split;
    return 0;
}

extern "C" int vs_debug_five_point(const double* q1, const double* q2, int count, double* E_out, int* nmod) {
    return vs_debug_five_point_ck(q1, q2, count, E_out, nmod, nullptr);
}
extern "C" int vs_debug_five_point_ck(const double* q1, const double* q2, int count, double* E_out, int* nmod,
                                      long long* clocks) {
    if (count <= 0) return 0;
    double *d1, *d2, *dE;
    int* dn;
    const size_t nq = (size_t)count * 10, nE = (size_t)count * vs_em::kMaxModels * 9;
    if (hipMalloc(&d1, sizeof(double) * nq) != hipSuccess) return -1;
    (void)hipMalloc(&d2, sizeof(double) * nq);
    (void)hipMalloc(&dE, sizeof(double) * nE);
    (void)hipMalloc(&dn, sizeof(int) * count);
    long long* dck = nullptr;
    if (clocks) (void)hipMalloc(&dck, sizeof(long long) * 8 * count);
    (void)hipMemcpy(d1, q1, sizeof(double) * nq, hipMemcpyHostToDevice);
    (void)hipMemcpy(d2, q2, sizeof(double) * nq, hipMemcpyHostToDevice);
    (void)hipMemset(dE, 0, sizeof(double) * nE);
    hipLaunchKernelGGL(vs::k_debug_five_point, dim3(count), dim3(64), 0, 0, d1, d2, dE, dn, dck);
    hipError_t e = hipMemcpy(E_out, dE, sizeof(double) * nE, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(nmod, dn, sizeof(int) * count, hipMemcpyDeviceToHost);
    if (e == hipSuccess && clocks) e = hipMemcpy(clocks, dck, sizeof(long long) * 8 * count, hipMemcpyDeviceToHost);
    if (dck) (void)hipFree(dck);
    (void)hipFree(d1);
    (void)hipFree(d2);
    (void)hipFree(dE);
    (void)hipFree(dn);
    return e == hipSuccess ? 0 : -1;
}
