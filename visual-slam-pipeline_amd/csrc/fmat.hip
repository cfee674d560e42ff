// fmat.hip — F-matrix verification of Slam::process_frame on gfx950 (reference
// src/Slam.cpp:880-910: extract_matched_points :1174-1187, cv::findFundamentalMat(FM_RANSAC,
// 3.0, RANSAC_PROB = 0.999), mask filtering of good_matches in order, compute_epipolar_error
// before and after :1217-1240).
//
// One workgroup (8 wave64s) per frame pair.  The registrators are sequential only through the
// cv::RNG stream and the shrinking iteration budget, so iterations run in chunks (64, 128, then
// 256 hypotheses):
//   * subsets: every lane computes raw draws out of order with the cv::RNG jump-ahead
//     (pnp_solvers.h: state r = s1 * A^r mod (A 2^32 - 1), Mont(A^r) from a constant table) and
//     reduces them modulo n; J0[p] = the end of the 7-distinct-draw attempt that would start at
//     draw p (repeat rejection) for every p in parallel; pointer doubling (J_{k+1} = J_k o J_k)
//     gives attempt t's start J0^t(0) in log2(chunk) lookups; attempts are assembled and tested
//     for collinearity in parallel, and collinear attempts are dropped in order (getSubset's
//     retry).  A chunk in which nothing is accepted falls back to the exact serial getSubset
//     (attempt limit included), so the subsets are exactly OpenCV's;
//   * hypotheses: one 7-point solve per lane, models in LDS;
//   * RANSAC scoring in rounds of 8 hypotheses: wave w scores hypothesis r0 + w with its 64
//     lanes sweeping the points (ballot + popcount, division-free exact gate of fm_inlier,
//     early exit once a model can no longer beat the current best), then lane 0 replays the
//     round in iteration order and the rounds stop at the shrinking budget; LMedS (n <= 14)
//     scores per lane and replays per chunk.
// Then inliers are marked, the match list is compacted in order and both epipolar errors are
// reduced.  Numerical kernels are shared with the CPU restatement (fmat_solvers.h;
// -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "block_reduce.h"
#include "fmat_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_fm;

constexpr int kFmMaxPts = VS_FM_MAX_POINTS;
constexpr int kMaxChunk = 256;
constexpr int kThreads = 512;  // 8 wave64s, two per SIMD: the 7-point solver needs > 128 VGPRs (<= 256 at two waves per SIMD)
constexpr int kWaves = kThreads / 64;
constexpr int kRawCap = 7 * kMaxChunk + 128;
constexpr int kLevels = 8;  // pointer-doubling levels: 2^8 >= kMaxChunk attempts

// Round 6: the first chunk (64 hypotheses) is scored by G = kFmSplit workgroups at once — workgroup g
// scores hypotheses 8 g + w, 8 g + w + 8 G, ... on wave w (every model's full count) after drawing and solving
// the whole chunk like the others (the same subsets and models: the computation is deterministic) —
// and the pair's last workgroup to arrive replays the chunk in iteration order and continues alone.
// The counts meet in FmSync (kFmSyncBytes per pair, zeroed once, the counter re-armed by the kernel).
struct FmSync {
    int arrived;
    int pad[15];
    int count[kFmFirstChunk * 3];
};
static_assert(sizeof(FmSync) <= kFmSyncBytes, "FmSync");

// Mont(A^k), k < kRawCap: the generator stepped k times from the Montgomery one (pnp_solvers.h)
struct MwcPow {
    uint64_t v[kRawCap];
};
constexpr MwcPow make_mwc_pow() {
    MwcPow t{};
    uint64_t s = vs_pnp::kMwcR1;
    for (int i = 0; i < kRawCap; i++) {
        t.v[i] = s;
        s = vs_pnp::mwc_step(s);
    }
    return t;
}
__constant__ MwcPow g_mwc_pow = make_mwc_pow();

#ifdef VS_FM_PROFILE
// phase cycle counters (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_fm_cycles[8];
#define FM_T0() long long _fm_t = clock64()
#define FM_T(k)                                                              \
    do {                                                                     \
        if (threadIdx.x == 0) atomicAdd(&g_fm_cycles[k], clock64() - _fm_t); \
        _fm_t = clock64();                                                   \
    } while (0)
#else
#define FM_T0()
#define FM_T(k)
#endif

struct FmShared {
    float p1[2 * kFmMaxPts], p2[2 * kFmMaxPts];
    int draw[kRawCap];  // (unsigned)state % n of raw draw r
    int subset[kMaxChunk * 7];
    int start[kMaxChunk];  // raw position of attempt t
    int coll[kMaxChunk];
    union {
        double Fm[kMaxChunk * 3 * 9];
        uint16_t J[kLevels][kRawCap + 2];  // attempt-end maps (subset drawing only)
    };
    int nmod[kMaxChunk];
    float score[kMaxChunk * 3];  // RANSAC: inlier count; LMedS: median error
    int scan[kWaves];
    double F[9];
    uint64_t rng;
    int niters, best, best_iter, iter, fail_at, done, aborted, ok, chunk, inliers, serial_next, nchunk, navail,
        anycoll;
    double min_median;
};

__device__ inline int solve_idx(const FmShared& S, const int* idx, double (*F)[9]) {
    float x1[7], y1[7], x2[7], y2[7];
    for (int i = 0; i < 7; i++) {
        x1[i] = S.p1[2 * idx[i]];
        y1[i] = S.p1[2 * idx[i] + 1];
        x2[i] = S.p2[2 * idx[i]];
        y2[i] = S.p2[2 * idx[i] + 1];
    }
    return run_7point(x1, y1, x2, y2, F);
}

__device__ inline bool subset_collinear(const FmShared& S, const int* idx) {
    float x1[7], y1[7], x2[7], y2[7];
    for (int i = 0; i < 7; i++) {
        x1[i] = S.p1[2 * idx[i]];
        y1[i] = S.p1[2 * idx[i] + 1];
        x2[i] = S.p2[2 * idx[i]];
        y2[i] = S.p2[2 * idx[i] + 1];
    }
    return have_collinear(x1, y1, 7) || have_collinear(x2, y2, 7);
}

// Draws the next chunk's subsets into S.subset and sets S.chunk (may be 0 when getSubset failed,
// with S.fail_at set).  Called by all lanes.
__device__ void draw_subsets(FmShared& S, int n, int base, int want, int attempts) {
    const int tid = threadIdx.x;
    if (S.serial_next) {  // exact serial getSubset (after a collinear rejection, or a stall)
        if (tid == 0) {
            CvRng rng(S.rng);
            const bool found = get_subset(rng, S.p1, S.p2, n, attempts, S.subset);
            S.rng = rng.state;
            S.chunk = found ? 1 : 0;
            if (!found) S.fail_at = base;
            S.serial_next = 0;
        }
        __syncthreads();
        return;
    }
    FM_T0();
    // raw draws: expected draws per attempt with repeat rejection = sum_{k<7} n / (n - k)
    float per = 0.f;
    for (int k = 0; k < 7; k++) per += (float)n / (float)(n - k);
    const int R = min(kRawCap, (int)(want * per * 1.15f) + 64);
    const uint64_t s1 = vs_pnp::mwc_step(S.rng);
    for (int r = tid; r < R; r += kThreads)
        S.draw[r] = (int)((unsigned)vs_pnp::mwc_jump(s1, r, g_mwc_pow.v[r]) % (unsigned)n);
    if (tid == 0) {
        S.navail = want;
        S.anycoll = 0;
    }
    __syncthreads();
    FM_T(5);
    // J0[p]: one past the 7th distinct draw from p (R + 1: the draws run out)
    for (int p = tid; p <= R + 1; p += kThreads) {
        int e = R + 1;
        if (p < R) {
            int cur[7] = {-1, -1, -1, -1, -1, -1, -1};
            int i = 0, q = p;
            while (i < 7 && q < R) {
                const int v = S.draw[q++];
                bool dup = false;
                VS_UNROLL
                for (int k = 0; k < 7; k++) dup |= (k < i) & (cur[k] == v);
                if (!dup) {
                    VS_UNROLL
                    for (int k = 0; k < 7; k++) cur[k] = (k == i) ? v : cur[k];
                    i++;
                }
            }
            if (i == 7) e = q;
        }
        S.J[0][p] = (uint16_t)e;
    }
    __syncthreads();
    int L = 0;
    while ((1 << L) < want) L++;
    for (int k = 1; k < L; k++) {
        for (int p = tid; p <= R + 1; p += kThreads) S.J[k][p] = S.J[k - 1][S.J[k - 1][p]];
        __syncthreads();
    }
    for (int t = tid; t < want; t += kThreads) {  // attempt t starts at J0^t(0)
        int p = 0;
        for (int k = 0; k < L; k++)
            if ((t >> k) & 1) p = S.J[k][p];
        const bool avail = p < R && S.J[0][p] <= R;
        S.start[t] = avail ? p : -1;
        if (!avail) atomicMin(&S.navail, t);
    }
    __syncthreads();
    FM_T(6);
    const int T = S.navail;
    for (int t = tid; t < T; t += kThreads) {  // assemble attempt t, collinearity (getSubset's retry test)
        int cur[7] = {-1, -1, -1, -1, -1, -1, -1};
        int i = 0, q = S.start[t];
        while (i < 7) {
            const int v = S.draw[q++];
            bool dup = false;
            VS_UNROLL
            for (int k = 0; k < 7; k++) dup |= (k < i) & (cur[k] == v);
            if (!dup) {
                VS_UNROLL
                for (int k = 0; k < 7; k++) cur[k] = (k == i) ? v : cur[k];
                i++;
            }
        }
        VS_UNROLL
        for (int k = 0; k < 7; k++) S.subset[7 * t + k] = cur[k];
        const int c = subset_collinear(S, S.subset + 7 * t);
        S.coll[t] = c;
        if (c) S.anycoll = 1;
    }
    __syncthreads();
    FM_T(7);
    if (tid == 0) {
        int j = T, last = T - 1;
        if (S.anycoll) {  // drop collinear attempts in order (rare)
            j = 0;
            last = -1;
            for (int t = 0; t < T; t++) {
                if (S.coll[t]) continue;
                if (j != t)
                    for (int k = 0; k < 7; k++) S.subset[7 * j + k] = S.subset[7 * t + k];
                last = t;
                j++;
            }
        }
        if (j == 0) {  // nothing accepted: the exact serial getSubset draws the next subset
            S.serial_next = 1;
            S.chunk = 0;
        } else {
            const int P = S.J[0][S.start[last]];  // raw draws consumed
            S.rng = vs_pnp::mwc_jump(s1, P - 1, g_mwc_pow.v[P - 1]);
            S.chunk = j;
        }
    }
    __syncthreads();
}

// Problem source: FROM_MATCHES = pairs of frames + keypoints + good matches (pipeline), else
// point arrays with offsets (ABI single-problem path).
// diag[p][8] = {method, iterations run, winning iteration, inliers, F ok, n, kept, chunks}
// Grid: G x P workgroups (G = split; blockIdx = g P + p).  sync: FmSync per pair (G > 1).
template <bool FROM_MATCHES>
__global__ __launch_bounds__(kThreads) void k_fmat(const int* __restrict__ pairs, const vs_keypoint* __restrict__ kps,
                                              int cap, const vs_match* __restrict__ good,
                                              const int* __restrict__ ngood, const float* __restrict__ pts1,
                                              const float* __restrict__ pts2, const int* __restrict__ off,
                                              double thr, double conf, int max_iters, double* __restrict__ Fout,
                                              uint8_t* __restrict__ mask_out, vs_match* __restrict__ kept,
                                              int* __restrict__ nkept, double* __restrict__ err,
                                              int* __restrict__ diag, int G, char* __restrict__ sync) {
    __shared__ FmShared S;
    __shared__ double red4[kWaves * 4];
    __shared__ int s_last;
    const int P = gridDim.x / G, gw = blockIdx.x / P, pb = blockIdx.x - gw * P;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int n;
    const vs_match* gm = nullptr;
    if (FROM_MATCHES) {
        n = min(ngood[pb], cap);
        gm = good + (size_t)pb * cap;
        const vs_keypoint* kr = kps + (size_t)pairs[2 * pb] * cap;
        const vs_keypoint* kc = kps + (size_t)pairs[2 * pb + 1] * cap;
        for (int i = tid; i < n; i += blockDim.x) {  // extract_matched_points (:1184-1187)
            const vs_match m = gm[i];
            S.p1[2 * i] = kr[m.query_idx].x;
            S.p1[2 * i + 1] = kr[m.query_idx].y;
            S.p2[2 * i] = kc[m.train_idx].x;
            S.p2[2 * i + 1] = kc[m.train_idx].y;
        }
    } else {
        const int o0 = off[pb];
        n = off[pb + 1] - o0;
        for (int i = tid; i < 2 * n; i += blockDim.x) {
            S.p1[i] = pts1[2 * (size_t)o0 + i];
            S.p2[i] = pts2[2 * (size_t)o0 + i];
        }
    }
    int* dg = diag + 8 * pb;
    const int method = n < 7 ? 0 : n == 7 ? 1 : n >= 15 ? 2 : 3;
    const bool split = G > 1 && method == 2;
    if (gw > 0 && !split) return;  // one workgroup per pair unless its RANSAC is split
    const float thr2 = (float)(thr * thr);
    if (tid == 0) {
        S.rng = (uint64_t)-1;
        S.best = 0;
        S.best_iter = -1;
        S.iter = 0;
        S.fail_at = -1;
        S.done = method < 2;
        S.aborted = 0;
        S.ok = 0;
        S.serial_next = 0;
        S.nchunk = 0;
        S.min_median = DBL_MAX;
        S.niters = method == 2 ? (max_iters > 1 ? max_iters : 1) : 0;
        if (method == 3) {
            const int ni = vs_pnp::ransac_update_num_iters(conf, 0.45, 7, max_iters);
            S.niters = ni > 3 ? ni : 3;
        }
    }
    __syncthreads();
    if (method == 1 && tid == 0) {
        const int all[7] = {0, 1, 2, 3, 4, 5, 6};
        if (solve_idx(S, all, reinterpret_cast<double(*)[9]>(S.Fm)) > 0) {
            for (int k = 0; k < 9; k++) S.F[k] = S.Fm[k];
            S.ok = 1;
        }
    }
    __syncthreads();
    // ---- registrator loop ----
    while (!S.done) {
        const int base = S.iter;
        const int want = min(min(kMaxChunk, 64 << min(S.nchunk, 2)), S.niters - base);
        draw_subsets(S, n, base, want, method == 2 ? 10000 : 1000);
        FM_T0();
        const int chunk = S.chunk;
        if (tid < chunk) {
            // the solver writes its models straight into LDS (no private array: dynamic model
            // indices would put one in scratch)
            double(*Fs)[9] = reinterpret_cast<double(*)[9]>(&S.Fm[tid * 27]);
            const int nm = solve_idx(S, S.subset + 7 * tid, Fs);
            S.nmod[tid] = nm;
            if (method == 3)  // LMedS: n <= 14, median = element n/2 of the sorted errors
                for (int k = 0; k < nm; k++) {
                    float e[14];
                    for (int i = 0; i < n; i++) {
                        const float v =
                            fm_error(Fs[k], S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1]);
                        int q = i;
                        while (q > 0 && e[q - 1] > v) {
                            e[q] = e[q - 1];
                            q--;
                        }
                        e[q] = v;
                    }
                    S.score[3 * tid + k] = e[n / 2];
                }
        }
        __syncthreads();
        FM_T(1);
        if (method == 2 && split && S.nchunk == 0) {
            // the first chunk split over the pair's workgroups: every model's full count (a count is
            // only ever compared with the running best, so the early exit changes no decision)
            FmSync* sy = reinterpret_cast<FmSync*>(sync + (size_t)pb * kFmSyncBytes);
            for (int h = kWaves * gw + wv; h < chunk; h += kWaves * G) {  // the whole chunk at any G
                for (int k = 0; k < S.nmod[h]; k++) {
                    const int m = 3 * h + k;
                    double F[9];
                    for (int q = 0; q < 9; q++) F[q] = S.Fm[m * 9 + q];
                    int cnt = 0;
                    for (int i0 = 0; i0 < n; i0 += 64) {
                        const int i = i0 + lane;
                        const bool in = i < n && fm_inlier(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i],
                                                           S.p2[2 * i + 1], thr2);
                        cnt += __popcll(__ballot(in));
                    }
                    if (lane == 0) sy->count[m] = cnt;
                }
            }
            __threadfence();
            __syncthreads();
            if (tid == 0) {
                const int old = __hip_atomic_fetch_add(&sy->arrived, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                s_last = old == G - 1;
                if (s_last) __hip_atomic_store(&sy->arrived, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            if (!s_last) return;
            __threadfence();
            for (int m = tid; m < 3 * chunk; m += kThreads) S.score[m] = (float)sy->count[m];
            __syncthreads();
            if (tid == 0) {  // the chunk in iteration order, stopping at the budget
                int it = S.iter;
                for (int hh = 0; hh < chunk && it < S.niters; hh++, it++)
                    for (int k = 0; k < S.nmod[hh]; k++) {
                        const int m = 3 * hh + k;
                        const int cnt = (int)S.score[m];
                        if (cnt > (S.best > 6 ? S.best : 6)) {
                            S.best = cnt;
                            S.niters = vs_pnp::ransac_update_num_iters(conf, (double)(n - cnt) / n, 7, S.niters);
                            S.best_iter = it;
                            for (int q = 0; q < 9; q++) S.F[q] = S.Fm[m * 9 + q];
                        }
                    }
                S.iter = it;
            }
            __syncthreads();
        } else if (method == 2) {
            // Rounds of kWaves hypotheses: wave w scores hypothesis r0 + w (its lanes sweep the
            // points), then lane 0 replays the round in iteration order.  A model whose count can
            // no longer exceed max(best, 6) at the round's start stops early (it cannot be taken:
            // the bar only rises during the replay); the round loop stops at the budget.
            for (int r0 = 0; r0 < chunk; r0 += kWaves) {
                const int h = r0 + wv;
                if (h < chunk && base + h < S.niters) {
                    const int bar = S.best > 6 ? S.best : 6;
                    for (int k = 0; k < S.nmod[h]; k++) {
                        const int m = 3 * h + k;
                        double F[9];
                        for (int q = 0; q < 9; q++) F[q] = S.Fm[m * 9 + q];
                        int cnt = 0;
                        for (int i0 = 0; i0 < n; i0 += 64) {
                            const int i = i0 + lane;
                            const bool in = i < n && fm_inlier(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i],
                                                               S.p2[2 * i + 1], thr2);
                            cnt += __popcll(__ballot(in));
                            if (cnt + max(0, n - i0 - 64) <= bar) {
                                cnt = -1;  // cannot be taken
                                break;
                            }
                        }
                        if (lane == 0) S.score[m] = (float)cnt;
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    int it = S.iter;
                    for (int hh = r0; hh < min(r0 + kWaves, chunk) && it < S.niters; hh++, it++)
                        for (int k = 0; k < S.nmod[hh]; k++) {
                            const int m = 3 * hh + k;
                            const int cnt = (int)S.score[m];
                            if (cnt > (S.best > 6 ? S.best : 6)) {
                                S.best = cnt;
                                S.niters = vs_pnp::ransac_update_num_iters(conf, (double)(n - cnt) / n, 7, S.niters);
                                S.best_iter = it;
                                for (int q = 0; q < 9; q++) S.F[q] = S.Fm[m * 9 + q];
                            }
                        }
                    S.iter = it;
                }
                __syncthreads();
                if (S.iter >= S.niters) break;
            }
        } else if (tid == 0) {  // LMedS: fixed budget, replay the chunk
            int it = base;
            for (; it < base + chunk && it < S.niters; it++) {
                const int h = it - base;
                for (int k = 0; k < S.nmod[h]; k++) {
                    const int m = 3 * h + k;
                    if (S.score[m] < S.min_median) {
                        S.min_median = S.score[m];
                        S.best_iter = it;
                        for (int q = 0; q < 9; q++) S.F[q] = S.Fm[m * 9 + q];
                    }
                }
            }
            S.iter = it;
        }
        FM_T(2);
        if (tid == 0) {
            const int it = S.iter;
            if (S.fail_at >= 0 && it == S.fail_at) {  // getSubset failed at this iteration
                if (it == 0) S.aborted = 1;
                S.done = 1;
            }
            if (it >= S.niters) S.done = 1;
            S.nchunk++;
            if (S.done && !S.aborted) S.ok = method == 2 ? S.best > 0 : S.min_median < DBL_MAX;
        }
        __syncthreads();
        FM_T(3);
    }
    FM_T0();
    // ---- inliers of the final model ----
    float gate = thr2;
    if (method == 3 && S.ok) {
        double sigma = 2.5 * 1.4826 * (1 + 5. / (n - 7)) * sqrt(S.min_median);
        sigma = sigma > 0.001 ? sigma : 0.001;
        gate = (float)(sigma * sigma);
    }
    const bool have_f = S.ok;
    double F[9];
    for (int k = 0; k < 9; k++) F[k] = S.F[k];
    // contiguous segment per lane so the compaction keeps the reference's order
    const int per = (n + kThreads - 1) / kThreads, lo = min(n, tid * per), hi = min(n, lo + per);
    int local = 0;
    uint32_t bits = 0;  // per <= 8 since n <= 2048
    for (int i = lo; i < hi; i++) {
        bool in = true;
        if (have_f && method != 1)
            in = fm_inlier(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1], gate);
        bits |= (uint32_t)in << (i - lo);
        local += in;
    }
    // exclusive scan of the per-thread counts: wave shuffles, then the kWaves wave totals
    int incl = local;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) S.scan[wv] = incl;
    __syncthreads();
    int wbase = 0, total = 0;
    for (int w = 0; w < kWaves; w++) {
        const int c = S.scan[w];
        wbase += w < wv ? c : 0;
        total += c;
    }
    const int excl = wbase + incl - local;
    if (tid == 0) S.inliers = total;
    __syncthreads();
    bool ok = have_f;
    if (method == 3 && have_f && S.inliers < 7) ok = false;  // LMeDS: result = count >= modelPoints
    // keep everything when F is empty (Slam.cpp:887, 892)
    {
        int w = ok ? excl : lo;
        for (int i = lo; i < hi; i++) {
            const bool in = ok ? ((bits >> (i - lo)) & 1u) : true;
            if (mask_out) mask_out[(FROM_MATCHES ? (size_t)pb * cap : (size_t)off[pb]) + i] = ok ? in : 0;
            if (FROM_MATCHES && in) kept[(size_t)pb * cap + w++] = gm[i];
        }
    }
    // ---- epipolar errors (Slam.cpp:888-890, 903-905) ----
    double part[4] = {0, 0, 0, 0}, tot[4];
    if (ok) {
        for (int i = lo; i < hi; i++) {
            double term;
            if (epipolar_term(F, S.p1[2 * i], S.p1[2 * i + 1], S.p2[2 * i], S.p2[2 * i + 1], term)) {
                part[0] += term;
                part[1] += 1.0;
                if ((bits >> (i - lo)) & 1u) {
                    part[2] += term;
                    part[3] += 1.0;
                }
            }
        }
    }
    block_sum<4, kWaves>(part, red4, tot);
    FM_T(4);
    if (tid == 0) {
        const int kept_n = ok ? S.inliers : n;
        if (FROM_MATCHES) nkept[pb] = kept_n;
        err[2 * pb] = (ok && tot[1] > 0) ? tot[0] / tot[1] : 0.0;
        err[2 * pb + 1] = (ok && S.inliers > 0 && tot[3] > 0) ? tot[2] / tot[3] : 0.0;
        for (int k = 0; k < 9; k++) Fout[9 * pb + k] = ok ? F[k] : 0.0;
        dg[0] = method;
        dg[1] = S.iter;
        dg[2] = S.best_iter;
        dg[3] = (method == 1 && ok) ? n : (have_f ? S.inliers : 0);
        dg[4] = ok;
        dg[5] = n;
        dg[6] = kept_n;
        dg[7] = S.nchunk;
    }
}

static int g_fm_split_test = -1;  // vs_debug_fmat_split (tests): forces every launch's split
// the pipeline's default: 1 unless VS_FMAT_SPLIT says otherwise
static int env_or_one() {
    static const int v = [] {
        const char* e = std::getenv("VS_FMAT_SPLIT");
        const int x = e ? std::atoi(e) : 0;
        return x >= 1 && x <= kFmSplit ? x : 1;
    }();
    return v;
}
// the split and its meeting area (the context's, zeroed, for callers without one).  Default: the ABI's point-set
// calls (latency-bound, alone on their CUs) kFmSplit; the pipeline's frame pairs 1 — beside the network on a
// shared CU set, eight workgroups waiting for free CUs cost more than the scoring rounds they save
// (profiles/r06fm_fmat_split_ab.txt).  VS_FMAT_SPLIT=1..8 overrides both.
static int fm_launch_setup(vs_ctx* ctx, int P, int split, char** sync, hipStream_t s) {
    static const int env_split = [] {
        const char* e = std::getenv("VS_FMAT_SPLIT");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 && v <= kFmSplit ? v : 0;
    }();
    if (split <= 0) split = env_split ? env_split : kFmSplit;
    if (g_fm_split_test > 0) split = g_fm_split_test;
    split = split < 1 ? 1 : split;
    VS_ARG(split <= kFmSplit, "fmat: split above kFmSplit");
    if (split > 1 && !*sync) {
        const size_t need = (size_t)P * kFmSyncBytes;
        if (ctx->fm_sync.bytes < need) {
            VS_CHECK(ctx->fm_sync.ensure(need));
            VS_HIP(hipMemsetAsync(ctx->fm_sync.p, 0, ctx->fm_sync.bytes, s));
        }
        *sync = ctx->fm_sync.as<char>();
    }
    return split;
}

int fmat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_good,
               const int* d_ngood, double* d_F, vs_match* d_kept, int* d_nkept, double* d_err, int* d_diag,
               hipStream_t s, int split, char* d_sync) {
    if (P <= 0) return VS_OK;
    VS_ARG(cap <= kFmMaxPts, "fmat_pairs: cap above VS_FM_MAX_POINTS");
    VS_ARG(!d_sync || P == 1, "fmat_pairs: a caller's meeting area holds one pair");
    const int G = fm_launch_setup(ctx, P, split > 0 ? split : env_or_one(), &d_sync, s);
    if (G < 0) return G;
    ProfScope ps(ctx, "fmat_ransac", s);
    hipLaunchKernelGGL(k_fmat<true>, dim3(P * G), dim3(kThreads), 0, s, d_pairs, d_kps, cap, d_good, d_ngood, nullptr,
                       nullptr, nullptr, 3.0, 0.999, 1000, d_F, nullptr, d_kept, d_nkept, d_err, d_diag, G, d_sync);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

int fmat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, double thr, double conf,
                int max_iters, double* d_F, uint8_t* d_mask, double* d_err, int* d_diag, hipStream_t s) {
    if (P <= 0) return VS_OK;
    char* d_sync = nullptr;
    const int G = fm_launch_setup(ctx, P, 0, &d_sync, s);
    if (G < 0) return G;
    ProfScope ps(ctx, "fmat_ransac", s);
    hipLaunchKernelGGL(k_fmat<false>, dim3(P * G), dim3(kThreads), 0, s, nullptr, nullptr, 0, nullptr, nullptr, d_p1,
                       d_p2, d_off, thr, conf, max_iters, d_F, d_mask, nullptr, nullptr, d_err, d_diag, G, d_sync);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs

// test hook: every later k_fmat launch of the process uses `split` workgroups per pair (1..8; 0 restores the defaults)
extern "C" int vs_debug_fmat_split(int split) {
    if (split < 0 || split > vs::kFmSplit) return -1;
    vs::g_fm_split_test = split > 0 ? split : -1;
    return 0;
}

#ifdef VS_FM_PROFILE
extern "C" int vs_debug_fm_cycles(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_fm_cycles), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_fm_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
