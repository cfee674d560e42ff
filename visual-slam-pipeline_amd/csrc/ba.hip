// ba.hip — Optimizer::local_bundle_adjustment (reference src/Optimizer.cpp:187-599) on gfx950,
// from the gathered window (:244): N keyframe poses, M points, observations in gather order.
//
// The sparsity structure is fixed across iterations and is prepared once on the host (the
// reference builds the same lists in its hash maps, :257-263, :443-451): observers per point in
// first-appearance order, the observations of every keyframe and of every point in gather order,
// and for every keyframe pair (a, b) the points both observe, ascending.  Each LM iteration is a
// fixed sequence of launches that return immediately once the device-side control block says done,
// so the host enqueues max_iter iterations without synchronising:
//   k_ba_pose_cache   R = Rodrigues(rvec) and the three rotation-perturbed R per keyframe
//   k_ba_obs          per-observation Jacobians, Huber weights, residuals (ba_obs_terms)
//   k_ba_kf_acc       per keyframe: Hpp, bp in gather order, + 1e10 I
//   k_ba_pt_acc       per point: Hmm, bm, Hpm in gather order, Cholesky inverse, U = Hpm Hinv
//   k_ba_schur        one workgroup per (a, b) block: S_ab = [a == b] Hpp_a (1 + lambda) on the
//                     diagonal - sum over common points (ascending) of U_a Hpm_b^T; b_a likewise
//   k_ba_chol         dense right-looking Cholesky + the two triangular solves (one workgroup), or
//   k_ba_chol_band    the same for a banded S (two waves: the pivot chain beside the column updates, the
//                     band in LDS; bit-identical results)
//   k_ba_update       back-substitution dm = Hinv (-bm - sum Hpm^T dp), new poses
//   k_ba_cost         new cost (fixed chunks) + accept / reject, lambda, convergence (last chunk)
// Every element is accumulated in the same order as the CPU restatement (oracle/orc_ba.cpp); the
// global cost sums use fixed chunks of 256 observations.  Arithmetic shared via ba_solvers.h.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ba_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_ba;

struct BaCtl {
    double lambda, total_cost, new_cost, err_before, err_after;
    int iter, accepted, done, solved, take, max_iter;
    unsigned arrive;  // k_ba_cost's arrival counter (left at 0)
};

struct BaDev {
    int N, M, n_obs, n_pairs, n_chunks, np;  // np: the Schur dimension 6N padded to 32
    int band;                                 // S_ij = 0 for i - j > band (k_ba_chol_band), from the observer pairs
    Cam K;
    const int *okf, *opt, *oslot, *kf_off, *kf_obs, *pt_off, *pt_obs, *pv_off, *pv_kf, *ab_off, *ab_u, *ab_h, *ab_j,
        *kb_off, *kb_u, *kb_j;
    const double* ouv;
    double *rv, *tv, *P, *rv_new, *tv_new, *P_new;
    PoseC *pc, *pc_new;
    ObsTerms* terms;
    double *Hpp, *bp, *Hmm, *bm, *Hpm, *Hinv, *U, *S, *bs, *dp, *chunk;
    int* pvalid;
    BaCtl* ctl;
    int* done_host;  // mapped pinned host memory: ctl->done after every accept / reject
};

#define BA_LIVE(d) \
    if (d.ctl->done) return

__global__ void k_ba_init(BaDev d, const double* R) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < d.N) vs_pnp::rod_m2v(R + 9 * i, d.rv + 3 * i);
}

__global__ void k_ba_pose_cache(BaDev d, int which, int check) {
    if (check) BA_LIVE(d);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= d.N) return;
    if (which == 0)
        pose_cache(d.rv + 3 * i, d.tv + 3 * i, d.pc[i]);
    else
        pose_cache(d.rv_new + 3 * i, d.tv_new + 3 * i, d.pc_new[i]);
}

__global__ void k_ba_obs(BaDev d) {
    BA_LIVE(d);
    const int o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= d.n_obs) return;
    ba_obs_terms(d.pc[d.okf[o]], d.P + 3 * (size_t)d.opt[o], d.ouv[2 * o], d.ouv[2 * o + 1], d.K, d.terms[o]);
}

// mode 0: total_cost; 1: new cost + accept/reject; 2: err_before; 3: err_after
// s: the cost summed over the chunks in order (k_ba_cost's last workgroup)
__device__ void ba_control(const BaDev& d, int mode, double s) {
    BaCtl& c = *d.ctl;
    if (mode <= 1 && c.done) return;
    if (mode == 0) {
        c.total_cost = s;
        return;
    }
    if (mode == 2) {
        c.err_before = sqrt(s / d.n_obs);
        return;
    }
    if (mode == 3) {
        c.err_after = sqrt(s / d.n_obs);
        return;
    }
    c.take = 0;
    if (!c.solved) {  // the oracle: lambda * 10 and the next iteration
        c.lambda *= 10;
    } else {
        c.new_cost = s;
        if (s < c.total_cost) {
            c.take = 1;
            c.lambda = c.lambda * 0.5 > 1e-7 ? c.lambda * 0.5 : 1e-7;
            c.accepted++;
            const double rel = (c.total_cost - s) / (c.total_cost + 1e-10);
            if (rel < 1e-4) c.done = 1;
        } else {
            c.lambda *= 5.0;
            if (c.lambda > 1e6) c.done = 1;
        }
    }
    c.iter++;
    if (c.iter >= c.max_iter) c.done = 1;
    __hip_atomic_store(d.done_host, c.done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The global cost and the LM control in one launch.  mode 0: total_cost from the terms; 1: new_cost
// (new params); 2: squared error (current params).  One 256-lane workgroup per fixed chunk of
// kCostChunk observations: the per-observation terms in parallel into LDS, then lane 0 sums them in
// observation order (the oracle's chunked order) and publishes the chunk with a device-scope atomic
// store; the last chunk to arrive (a device-scope counter, every earlier chunk's store performed
// before its arrival) sums the chunks in order and runs the control step cmode (ba_control).
__global__ __launch_bounds__(kCostChunk) void k_ba_cost(BaDev d, int mode, int check, int cmode) {
    if (check) BA_LIVE(d);
    __shared__ double s_v[kCostChunk];
    const int c = blockIdx.x, t = threadIdx.x;
    const int o0 = c * kCostChunk, o1 = min(d.n_obs, o0 + kCostChunk);
    const int o = o0 + t;
    double v = 0.0;
    if (o < o1) {
        const double* P = (mode == 1 ? d.P_new : d.P) + 3 * (size_t)d.opt[o];
        if (mode == 0)
            v = d.terms[o].valid ? d.terms[o].cost : 0.0;
        else if (mode == 1)
            v = ba_new_cost_term(d.pc_new[d.okf[o]], P, d.ouv[2 * o], d.ouv[2 * o + 1], d.K);
        else
            v = ba_sq_err_term(d.pc[d.okf[o]], P, d.ouv[2 * o], d.ouv[2 * o + 1], d.K);
    }
    s_v[t] = v;
    __syncthreads();
    if (t == 0) {
        double sum = 0;
        for (int k = 0; k < o1 - o0; k++) sum += s_v[k];
        __hip_atomic_store(d.chunk + c, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the chunk sum is ordered before the arrival by the HIP memory model (release RMW), and the
        // last arriver's loads after every other chunk's arrival (acquire RMW) — ADVICE r04: no
        // reliance on an inline s_waitcnt and the current ISA's ordering
        const unsigned prev = __hip_atomic_fetch_add(&d.ctl->arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)d.n_chunks - 1) {
            __hip_atomic_store(&d.ctl->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            double tot = 0;
            for (int k = 0; k < d.n_chunks; k++) tot += __hip_atomic_load(d.chunk + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ba_control(d, cmode, tot);
        }
    }
}

// Hpp, bp per keyframe in gather order (:407-451), one 64-lane workgroup per keyframe: lane
// l < 21 owns upper-triangular element l of Hpp (mirrored), lanes 21..26 own bp — each element is
// the same sequential sum over the keyframe's valid observations as in the oracle.  The observation
// terms are staged 64 at a time through two LDS buffers, the next stage's loads in flight while the
// current one is summed (one barrier per stage); an invalid observation adds +0.0, which leaves
// the sum unchanged (it starts at +0.0 and so is never -0.0).
__global__ __launch_bounds__(64) void k_ba_kf_acc(BaDev d) {
    BA_LIVE(d);
    __shared__ double s_t[2][64][16];  // per staged observation: Jp (12), ru_w, rv_w, valid (0 / 1)
    const int i = blockIdx.x, l = threadIdx.x;
    if (i >= d.N) return;
    int r = 0, c = 0;
    if (l < 21) {
        int k = l;
        while (k >= 6 - r) {
            k -= 6 - r;
            r++;
        }
        c = r + k;
    } else {
        r = l - 21;
    }
    // the two products of the lane's element: s[r] s[cb] + s[6 + r] s[cb2]
    const int cb = l < 21 ? c : 12, cb2 = l < 21 ? 6 + c : 13;
    const int q0 = d.kf_off[i], q1 = d.kf_off[i + 1];
    double v[15];
    auto fetch = [&](int qb) {
        if (qb + l < q1) {
            const ObsTerms& ot = d.terms[d.kf_obs[qb + l]];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                v[k] = ot.Jp[0][k];
                v[6 + k] = ot.Jp[1][k];
            }
            v[12] = ot.ru_w;
            v[13] = ot.rv_w;
            v[14] = ot.valid ? 1.0 : 0.0;
        }
    };
    fetch(q0);
    double acc = 0;
    int buf = 0;
    for (int qb = q0; qb < q1; qb += 64) {
        if (qb + l < q1)
#pragma unroll
            for (int k = 0; k < 15; k++) s_t[buf][l][k] = v[k];
        __syncthreads();
        if (qb + 64 < q1) fetch(qb + 64);
        const int m = min(64, q1 - qb);
        if (l < 27) {
            const double* T = &s_t[buf][0][0];
#pragma unroll 4
            for (int k = 0; k < m; k++) {
                const double* t = T + 16 * k;
                const double term = t[r] * t[cb] + t[6 + r] * t[cb2];
                acc += t[14] != 0.0 ? term : 0.0;
            }
        }
        buf ^= 1;
    }
    if (l < 21) {
        if (r == c) acc += kPoseDamp;
        d.Hpp[36 * i + r * 6 + c] = acc;
        d.Hpp[36 * i + c * 6 + r] = acc;
    } else if (l < 27) {
        d.bp[6 * i + r] = acc;
    }
}

// Hmm, bm and the Hpm blocks per point (one thread per point), in observation order.  Each Hpm
// slot (one per observing keyframe) is summed in registers over the observations of that slot and
// stored once (the oracle's += from zero, in the same order), instead of a read-modify-write of
// global memory per observation.
__global__ void k_ba_pt_acc(BaDev d) {
    BA_LIVE(d);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.M) return;
    double H[9], b[3];
    for (int k = 0; k < 9; k++) H[k] = 0;
    for (int k = 0; k < 3; k++) b[k] = 0;
    const int p0 = d.pv_off[j], np = d.pv_off[j + 1] - p0;
    const int qa = d.pt_off[j], qe = d.pt_off[j + 1];
    for (int q = qa; q < qe; q++) {
        const ObsTerms& ot = d.terms[d.pt_obs[q]];
        if (ot.valid) ba_add_point(ot, H, b);
    }
    for (int sl = 0; sl < np; sl++) {
        double X[18];
#pragma unroll
        for (int k = 0; k < 18; k++) X[k] = 0;
        for (int q = qa; q < qe; q++) {
            const int o = d.pt_obs[q];
            if (d.oslot[o] != sl) continue;
            const ObsTerms& ot = d.terms[o];
            if (ot.valid) ba_add_cross(ot, X);
        }
        double* dst = d.Hpm + 18 * (size_t)(p0 + sl);
#pragma unroll
        for (int k = 0; k < 18; k++) dst[k] = X[k];
    }
    for (int k = 0; k < 9; k++) d.Hmm[9 * (size_t)j + k] = H[k];
    for (int k = 0; k < 3; k++) d.bm[3 * (size_t)j + k] = b[k];
    double Hi[9];
    const bool ok = ba_point_inverse(H, d.ctl->lambda, Hi);
    d.pvalid[j] = ok;
    for (int k = 0; k < 9; k++) d.Hinv[9 * (size_t)j + k] = Hi[k];
    if (ok)
        for (int sl = 0; sl < np; sl++) ba_schur_u(d.Hpm + 18 * (size_t)(p0 + sl), Hi, d.U + 18 * (size_t)(p0 + sl));
}

// b_a = bp_a - sum over the points of keyframe a (ascending) of U_a bm, one 64-lane workgroup per
// keyframe (threads 0..5 own b_a(r)), staged like the S blocks
__device__ __forceinline__ void schur_b(const BaDev& d, int a, double (*s_U)[64][18], double (*s_H)[64][18],
                                        int (*s_ok)[64]) {
    const int t = threadIdx.x;
    double u[18];
    int ok = 0;
    double sb = t < 6 ? d.bp[6 * a + t] : 0.0;
    double bmv[3];
    const int k0 = d.kb_off[a], k1 = d.kb_off[a + 1];
    auto fetch_b = [&](int qb) {
        const int q = qb + t;
        if (q < k1) {
            const int j = d.kb_j[q];
            const double* U = d.U + 18 * (size_t)d.kb_u[q];
#pragma unroll
            for (int k = 0; k < 18; k++) u[k] = U[k];
#pragma unroll
            for (int k = 0; k < 3; k++) bmv[k] = d.bm[3 * (size_t)j + k];
            ok = d.pvalid[j];
        }
    };
    fetch_b(k0);
    int buf = 0;
    for (int qb = k0; qb < k1; qb += 64) {
        if (qb + t < k1) {
#pragma unroll
            for (int k = 0; k < 18; k++) s_U[buf][t][k] = u[k];
#pragma unroll
            for (int k = 0; k < 3; k++) s_H[buf][t][k] = bmv[k];
            s_ok[buf][t] = ok;
        }
        __syncthreads();
        if (qb + 64 < k1) fetch_b(qb + 64);
        const int m = min(64, k1 - qb);
        if (t < 6)
#pragma unroll 4
            for (int k = 0; k < m; k++) {
                const double v = ba_schur_b(s_U[buf][k], s_H[buf][k], t);
                sb -= s_ok[buf][k] ? v : 0.0;
            }
        buf ^= 1;
    }
    if (t < 6) d.bs[6 * a + t] = sb;
}

// grid: N*N workgroups of 64 threads, threads 0..35 owning S_ab(r, c), then N workgroups for b_a
// (schur_b).  The (U, Hpm) pairs of the common points are staged 64 at a time
// through two LDS buffers, the next stage's loads in flight while the current one is summed (one
// barrier per stage); sums run over the lists in order (the oracle's), a skipped point (no
// inverse) subtracting +0.0, which leaves every value unchanged.
__global__ __launch_bounds__(64) void k_ba_schur(BaDev d) {
    BA_LIVE(d);
    __shared__ double s_U[2][64][18], s_H[2][64][18];
    __shared__ int s_ok[2][64];
    const int t = threadIdx.x;
    if ((int)blockIdx.x >= d.N * d.N) {  // workgroups N*N ..: b_a, beside the S blocks
        schur_b(d, (int)blockIdx.x - d.N * d.N, s_U, s_H, s_ok);
        return;
    }
    const int a = blockIdx.x / d.N, b = blockIdx.x % d.N;
    const int np = d.np;
    const double lam = d.ctl->lambda;
    const int r = t / 6, c = t % 6;
    double s = 0.0;
    if (t < 36) {
        s = a == b ? d.Hpp[36 * a + r * 6 + c] : 0.0;
        if (a == b && r == c) s *= (1.0 + lam);
    }
    double u[18], h[18];
    int ok = 0;
    const int pair = a * d.N + b;
    const int q0 = d.ab_off[pair], q1 = d.ab_off[pair + 1];
    auto fetch = [&](int qb) {
        const int q = qb + t;
        if (q < q1) {
            const double* U = d.U + 18 * (size_t)d.ab_u[q];
            const double* Hh = d.Hpm + 18 * (size_t)d.ab_h[q];
#pragma unroll
            for (int k = 0; k < 18; k++) {
                u[k] = U[k];
                h[k] = Hh[k];
            }
            ok = d.pvalid[d.ab_j[q]];
        }
    };
    fetch(q0);
    int buf = 0;
    for (int qb = q0; qb < q1; qb += 64) {
        if (qb + t < q1) {
#pragma unroll
            for (int k = 0; k < 18; k++) {
                s_U[buf][t][k] = u[k];
                s_H[buf][t][k] = h[k];
            }
            s_ok[buf][t] = ok;
        }
        __syncthreads();
        if (qb + 64 < q1) fetch(qb + 64);
        const int m = min(64, q1 - qb);
        if (t < 36)
#pragma unroll 4
            for (int k = 0; k < m; k++) {
                const double v = ba_schur_s(s_U[buf][k], s_H[buf][k], r, c);
                s -= s_ok[buf][k] ? v : 0.0;
            }
        buf ^= 1;
    }
    if (t < 36) d.S[(size_t)(6 * a + r) * np + 6 * b + c] = s;
}


// S dp = -bs by Cholesky in the arithmetic of cv::solve(S, -bs, dp, DECOMP_CHOLESKY)
// (Optimizer.cpp:516; OpenCV's hal Cholesky): each L entry is (S_ij - sum_{k<j} L_ik L_jk) * R_j
// with the sum in ascending k and R_j = 1 / sqrt(S_jj - sum_{k<j} L_jk^2) kept as the diagonal;
// a pivot below DBL_EPSILON fails the solve; the substitutions multiply by R as well.
// S is held padded to np = 6N rounded up to 32 with an identity block (rows / columns n..np-1;
// k_ba_pad sets it once per call): every padded L entry and solution value is exactly 0 and the
// padded pivots are 1, and no real element ever takes a padded term, so the real part is
// bit-identical to the unpadded statement while every panel is a full 32 columns (straight-line
// code, no edge guards).  One workgroup, right-looking over 32-column panels — every element still
// takes its terms in ascending k, so the factor and the solution are bit-identical to the oracle's
// row-oriented statement (oracle/orc_ba.cpp chol_solve):
//   1. wave 0 factors the panel's 32 x 32 diagonal block in registers (lane = row, readlane
//      broadcasts): the 32-step sqrt -> reciprocal -> update chain runs without a workgroup
//      barrier, and one panel ahead, beside the other waves' trailing update (look-ahead);
//   2. every row below takes the diagonal block (a 32-step substitution per row, one thread per
//      row, the block's L and R broadcast out of LDS);
//   3. the trailing lower triangle takes the panel's 32 columns in 4 x 4 register tiles, the
//      panel held k-major in LDS (one 32-byte read per 4 rows);
//   4. both substitutions are blocked the same way: wave 0 solves the 32 x 32 diagonal block by
//      readlane broadcasts, the rows below (above) take the finished block in parallel.
constexpr int kCholNB = 32;
constexpr int kCholMaxN = 6 * VS_BA_MAX_KEYFRAMES;  // a multiple of kCholNB
static_assert(kCholMaxN % kCholNB == 0, "padded Schur dimension");
// k_ba_chol (512 lanes) maps one thread to one row below the panel (rb = tid - 64) and in both
// substitutions: every row beyond the first panel needs a thread of waves 1..7
static_assert(kCholMaxN - kCholNB <= 512 - 64, "k_ba_chol: one thread per row needs <= 448 rows below the panel");
constexpr int kCholLd = kCholMaxN;  // PnT row length

#ifdef VS_BA_PROFILE
// phase cycle counters of k_ba_chol (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_ba_cycles[16];
#define BA_T0() long long _ba_t = clock64()
#define BA_T(k)                                                               \
    do {                                                                      \
        if (threadIdx.x == 0) atomicAdd(&g_ba_cycles[k], clock64() - _ba_t);  \
        _ba_t = clock64();                                                    \
    } while (0)
#else
#define BA_T0()
#define BA_T(k)
#endif

// lane l's value of v, wave-uniform (two v_readlane_b32)
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// orders a wave's LDS accesses for the compiler (LDS itself is in order within a wave)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// S dp = -bs for a banded S (k_ba_chol's arithmetic, fewer terms).  When no point is seen by two
// keyframes more than Bb apart, S_ij = 0 for i - j > band = 6 Bb + 5, and a Cholesky factor keeps
// that band (no fill outside it).  Every term the dense statement adds outside the band is a
// product with an exact zero, so skipping them leaves every element's value unchanged (at most the
// sign of an exact-zero element can differ, which no later result sees) — the factor and the
// solution are the oracle's (oracle/orc_ba.cpp chol_solve), element for element in the same order.
// Right-looking with the matrix as its band in LDS (row i, offset d = i - j), two waves per column:
// wave 0 runs the pivot chain — R_{j+1} = 1 / sqrt(acc_{j+1,j+1} - (acc_{j+1,j} R_j)^2), then the
// next pivot's two inputs (the column-j updates of acc_{j+2,j+2} and acc_{j+2,j+1}, the same
// operations wave 1 would apply, stored by wave 0) — while wave 1 applies column j to the rest of the
// trailing band triangle (i, k), j < k <= i <= j + band, with L = acc * R taken on the fly (the stored
// value stays the accumulated one) and carries the forward substitution; one barrier per column.
// The waves touch disjoint cells within a column: wave 0 reads rows j + 1, j + 2 and writes two cells
// of row j + 2 that wave 1 does not read in that column; wave 1 writes rows >= j + 3.  The backward
// substitution keeps each open row's running value in a register of lane (row mod 64).  Chosen by
// the host when the band fits kBandMaxW columns; a pivot below DBL_EPSILON fails the solve as in
// k_ba_chol.
constexpr int kBandMaxW = 36;  // band + 1 <= kBandMaxW (band <= 35: Bb <= 5)
static_assert(((kCholMaxN + kBandMaxW) * kBandMaxW + 64 + kCholMaxN + 64 + kCholMaxN + 64) * sizeof(double) <= 160 * 1024,
              "k_ba_chol_band: the band, R and x must fit one CU's LDS (raise VS_BA_MAX_KEYFRAMES only with a "
              "narrower kBandMaxW)");
// 1.0 / sqrt(x), bit for bit, for 2^-700 <= x <= 2^700: the compiler's correctly rounded sqrt and
// division expansions without their range scaling (scale factor 1 in that range: v_rsq + the
// Goldschmidt steps, then v_rcp + two Newton steps + the final remainder step), 17 dependent
// operations instead of 31.  tools/r05/rsq_exact.hip compared it with 1.0 / sqrt(x) on 537 M inputs
// over the range: no difference.  Outside the range: the plain expression.
__device__ __forceinline__ double recip_sqrt_rn(double x) {
    if (!(x >= 0x1p-700 && x <= 0x1p700)) return 1.0 / sqrt(x);
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    const double s = fma(d, h, g);  // sqrt (x)
    double z = __builtin_amdgcn_rcp(s);
    double e = fma(-s, z, 1.0);
    z = fma(z, e, z);
    e = fma(-s, z, 1.0);
    z = fma(z, e, z);
    const double rr = fma(-s, z, 1.0);
    return fma(rr, z, z);
}
// trailing-triangle elements per lane for a band: ceil(band (band + 1) / 2 / 64)
constexpr int band_slots(int band) { return (band * (band + 1) / 2 + 63) / 64; }
constexpr int kBandThreads = 128;  // wave 0: the pivot chain, wave 1: the column updates (a third wave
                                   // sharing the updates measured no faster: both are latency-bound)
template <int NS>
__global__ __launch_bounds__(kBandThreads) void k_ba_chol_band(BaDev d) {
    BA_LIVE(d);
    BA_T0();
    const int n = 6 * d.N, np = d.np, B = d.band, W = B + 1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: scalar branches)
    // A[i * W + dd] = acc (i, i - dd), rows n .. n + B - 1 zero padding (elements past the last row
    // compute there, unread, instead of testing their row); the 64 cells past the padding rows are
    // each lane's dummy store target
    __shared__ double A[(kCholMaxN + kBandMaxW) * kBandMaxW + 64];
    __shared__ double Rd[kCholMaxN + 64], xs[kCholMaxN + 64];
    __shared__ int s_bad;
    // the band out of S (just written by k_ba_schur, in L2): eight loads in flight per thread, then
    // their LDS stores
    for (int e0 = tid; e0 < n * W; e0 += kBandThreads * 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = e0 + kBandThreads * u, i = e / W, dd = e - i * W;
            v[u] = (e < n * W && dd <= i) ? d.S[(size_t)i * np + (i - dd)] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (e0 + kBandThreads * u < n * W) A[e0 + kBandThreads * u] = v[u];
    }
    for (int i = tid; i < n; i += kBandThreads) xs[i] = -d.bs[i];
    for (int i = tid; i < B * W; i += kBandThreads) A[n * W + i] = 0.0;
    for (int i = n + tid; i < kCholMaxN + 64; i += kBandThreads) xs[i] = 0.0;
    if (tid == 0) s_bad = 0;
    const int dummyA = (kCholMaxN + kBandMaxW) * kBandMaxW + lane, dummyX = kCholMaxN + lane;
    // wave 1's trailing-triangle elements e = lane + 64 q -> (a, b), 0 <= b <= a < B, i = j + 1 + a,
    // k = j + 1 + b, as offsets from row j + 1: the element, L_ij's and L_kj's cells.  (0, 0) is the
    // pivot (wave 0 evaluates it), (1, 0) and (1, 1) are wave 0's; slots past the triangle read the
    // base cell and store to the dummy cell.
    const int nel = B * (B + 1) / 2;
    int oe[NS], oi[NS], ok[NS];
    bool dead[NS];
#pragma unroll
    for (int q = 0; q < NS; q++) {
        const int e = lane + 64 * q;
        int a = 0;
        while ((a + 1) * (a + 2) / 2 <= e) a++;
        const int b = e - a * (a + 1) / 2;
        dead[q] = e >= nel || e < 3;
        oe[q] = dead[q] ? 0 : a * W + (a - b);
        oi[q] = dead[q] ? 0 : a * W + a + 1;
        ok[q] = dead[q] ? 0 : b * W + b + 1;
    }
    __syncthreads();
    BA_T(5);  // the band, R and x into LDS
    if (A[0] < DBL_EPSILON) {
        if (tid == 0) d.ctl->solved = 0;
        return;
    }
    double Rj = recip_sqrt_rn(A[0]);  // R_0 (both waves)
    if (tid == 0) Rd[0] = Rj;
    // Each wave runs its own loop over the columns (wv is wave-uniform: scalar branches), one barrier
    // per column in each.  A bad pivot does not stop the loops (the rest computes on garbage and is
    // discarded): the verdict is shared once, after them.
    bool bad = false;
#ifdef VS_BA_PROFILE
    long long t_work = 0, t_wait = 0, t_a = clock64();
#define VS_BAND_T_BARRIER()          \
    do {                             \
        const long long t_b = clock64(); \
        t_work += t_b - t_a;         \
        __syncthreads();             \
        t_a = clock64();             \
        t_wait += t_a - t_b;         \
    } while (0)
#else
#define VS_BAND_T_BARRIER() __syncthreads()
#endif
    if (wv == 0) {
        double p1 = A[W + 1], p0 = A[W];  // acc (j+1, j), acc (j+1, j+1) before column j
        for (int j = 0; j < n; j++) {
            const int j1 = j + 1, base = j1 * W;
            // the next pivot's inputs, read before the chain so that their latency hides under it
            const double q22 = A[base + W], q21 = A[base + W + 1], q20 = A[base + W + 2], q10 = A[base + 1];
            const double l = p1 * Rj;
            const double accn = p0 - l * l;
            bad |= j1 < n && accn < DBL_EPSILON;
            const double Rn = recip_sqrt_rn(accn);
            // column j's updates of (j+2, j+2) and (j+2, j+1): wave 1's operations on those cells
            p0 = q22 - (q20 * Rj) * (q20 * Rj);
            p1 = q21 - (q20 * Rj) * (q10 * Rj);
            A[base + W] = p0;
            A[base + W + 1] = p1;
            Rd[j1 < n ? j1 : kCholMaxN + lane] = Rn;
            Rj = Rn;
            VS_BAND_T_BARRIER();
        }
    } else {
        double xj = xs[0];  // x_j with its forward terms so far
        for (int j = 0; j < n; j++) {
            const int j1 = j + 1, base = j1 * W;
            const double Rc = j == 0 ? Rj : Rd[j];
            double xi[NS], xl[NS], xk[NS];
#pragma unroll
            for (int q = 0; q < NS; q++) {
                xi[q] = A[base + oe[q]];
                xl[q] = A[base + oi[q]];
                xk[q] = A[base + ok[q]];
            }
            const bool fl = lane < B;  // the forward substitution's rows j + 1 .. j + B
            const double xf = xs[j1 + (fl ? lane : 0)], lf = A[base + (fl ? lane * W + lane + 1 : 0)];
            const double yj = xj * Rc;
#pragma unroll
            for (int q = 0; q < NS; q++) {
                const double v = xi[q] - (xl[q] * Rc) * (xk[q] * Rc);
                A[dead[q] ? dummyA : base + oe[q]] = v;
            }
            const double xn = xf - (lf * Rc) * yj;  // forward substitution: x_i -= L_ij y_j
            xs[fl ? j1 + lane : dummyX] = xn;
            xs[j] = yj;  // (every lane, the same value)
            xj = readlane_f64(xn, 0);
            VS_BAND_T_BARRIER();
        }
    }
#undef VS_BAND_T_BARRIER
#ifdef VS_BA_PROFILE
    if (lane == 0) {  // 8 + 2w / 9 + 2w: wave w's column work / barrier wait
        atomicAdd(&g_ba_cycles[8 + 2 * wv], (unsigned long long)t_work);
        atomicAdd(&g_ba_cycles[9 + 2 * wv], (unsigned long long)t_wait);
    }
#endif
    if (wv == 0 && bad) s_bad = 1;
    __syncthreads();
    BA_T(6);  // factorisation + forward substitution
    if (s_bad) {
        if (tid == 0) d.ctl->solved = 0;
        return;
    }
    if (wv != 0) return;
    // backward: x_k = y'_k R_k with y'_k = y_k - sum_{k' > k, descending} L_k'k x_k'.  Row i's running
    // value stays in lane (i mod 64)'s register — at most B < 64 rows are open at once — so the chain
    // from one step to the next is a readlane, two products and a difference: step k reads row k's
    // final value, every open row i in [k - B, k - 1] subtracts (L_ki R_i) x_k, and the lane that
    // finished row k takes up row k - 64 (the forward value, untouched until step k - 64 + B) with
    // its R.  A lane's row ib satisfies 0 <= k - ib <= 63, so its cell k W + k - ib is always inside
    // the band array (read unconditionally, used only while the row is open), one step ahead.
    int ib = (n - 1) - ((n - 1 - lane) & 63);  // this lane's open row (< 0: none)
    double acc = ib >= 0 ? xs[ib] : 0.0, ri = ib >= 0 ? Rd[ib] : 0.0;
    int aix = (n - 1) * (W + 1) - ib;
    double al = A[aix];
    for (int k0 = n - 1; k0 >= 0; k0 -= 64) {
        const double nxt = ib >= 64 ? xs[ib - 64] : 0.0, rnx = ib >= 64 ? Rd[ib - 64] : 0.0;
        const double rblk = Rd[k0 - lane >= 0 ? k0 - lane : 0];  // lane t: R_{k0 - t}
        const int kend = k0 - 63 > 0 ? k0 - 63 : 0;
        for (int k = k0; k >= kend; k--) {
            const int aixn = aix - (W + 1);
            const double aln = A[aixn > 0 ? aixn : 0];
            const double yk = readlane_f64(acc, k & 63);
            const double xkk = yk * readlane_f64(rblk, k0 - k);  // lane-uniform
            const double an = acc - (al * ri) * xkk;
            const bool open = (unsigned)(k - 1 - ib) < (unsigned)B, fin = k == ib;
            xs[fin ? k : dummyX] = xkk;
            acc = fin ? nxt : (open ? an : acc);
            ri = fin ? rnx : ri;
            ib = fin ? ib - 64 : ib;
            aix = fin ? aixn + 64 : aixn;
            al = aln;
        }
    }
    wave_lds_sync();
    for (int i = lane; i < n; i += 64) d.dp[i] = xs[i];
    if (lane == 0) d.ctl->solved = 1;
    BA_T(7);  // backward substitution + the solution out
}

// the padded rows n..np-1 of S: identity (their columns >= n above the diagonal are never read)
__global__ void k_ba_pad(BaDev d) {
    const int n = 6 * d.N, np = d.np;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (np - n) * np) return;
    const int i = n + g / np, j = g % np;
    d.S[(size_t)i * np + j] = i == j ? 1.0 : 0.0;
}

__global__ __launch_bounds__(512) void k_ba_chol(BaDev d) {
    BA_LIVE(d);
    const int n = 6 * d.N, np = d.np, tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    double* S = d.S;
    __shared__ __attribute__((aligned(16))) double PnT[kCholNB * kCholLd];  // the panel, k-major: PnT[k * kCholLd + row]
    __shared__ double Rd[kCholMaxN];                                         // reciprocal diagonal R
    __shared__ double xs[kCholMaxN];                                         // right-hand side / solution
    __shared__ double Dg[kCholNB * 33];                                      // wave 0's diagonal block
    __shared__ int bad;
    if (tid == 0) bad = 0;
    for (int i = tid; i < np; i += nt) xs[i] = i < n ? -d.bs[i] : 0.0;
    __syncthreads();
    BA_T0();
    // wave 0: the diagonal block at K0 factored in registers, lane i < 32 holding row K0 + i (lanes
    // 32.. duplicate row 31): the pivot and the column entries come by readlane (8 at a time: the
    // scheduler would otherwise hoist a whole column's into SGPRs), then the rows go to Dg (the
    // entries right of the diagonal are garbage, never read).  R into Rd; returns false if a pivot
    // is below DBL_EPSILON.
    auto diag_block = [&](int K0) {
        double g[kCholNB];
        const int lr = min(lane, kCholNB - 1);
#pragma unroll
        for (int c = 0; c < kCholNB; c++) g[c] = S[(size_t)(K0 + lr) * np + K0 + c];
        bool fail = false;
#pragma unroll
        for (int c = 0; c < kCholNB; c++) {
            const double s = readlane_f64(g[c], c);
            fail |= s < DBL_EPSILON;
            const double r = 1.0 / sqrt(s);
            if (lane == 0) Rd[K0 + c] = r;
            const double l = g[c] * r;
            g[c] = l;
#pragma unroll
            for (int j = c + 1; j < kCholNB; j++) {
                g[j] -= l * readlane_f64(l, j);
                if ((j - c) % 8 == 0) __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (lane < kCholNB)
#pragma unroll
            for (int c = 0; c < kCholNB; c++) Dg[lane * 33 + c] = g[c];
        return !fail;
    };
    // 4 x 4 tiles of the lower triangle: rows r0.., columns c0.. take the panel's 32 columns (PnT)
    auto tile_update = [&](int r0, int c0, bool diag) {
        double acc[4][4];
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[x][y] = S[(size_t)(r0 + x) * np + c0 + y];
#pragma unroll 8
        for (int k = 0; k < kCholNB; k++) {
            const double2* pr = reinterpret_cast<const double2*>(&PnT[k * kCholLd + r0]);
            const double2* pc = reinterpret_cast<const double2*>(&PnT[k * kCholLd + c0]);
            const double2 a01 = pr[0], a23 = pr[1], b01 = pc[0], b23 = pc[1];
            const double av[4] = {a01.x, a01.y, a23.x, a23.y}, bv[4] = {b01.x, b01.y, b23.x, b23.y};
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++) acc[x][y] -= av[x] * bv[y];
        }
        // (a diagonal tile's entries above the diagonal belong to S's upper triangle: not stored)
#pragma unroll
        for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
                if (!diag || y <= x) S[(size_t)(r0 + x) * np + c0 + y] = acc[x][y];
    };
    // forward substitution of the diagonal block at K0 (wave 0): y_i = (x_i - sum_{k<i} L_ik y_k) * R_i,
    // ascending k, the block's L from PnT (published in [A]).  Lane i keeps x_i and takes -0 * y_k for
    // k >= i (its row's upper part is zeroed), so the loop has no lane conditions; y_i = x_i R_i at
    // the end is the y_k the other lanes used.
    auto fwd_block = [&](int K0) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // per-block lane compares: not hoisted into live SGPR masks
        const int lr = min(ln, kCholNB - 1);
        double Lr[kCholNB];
#pragma unroll
        for (int c = 0; c < kCholNB; c++) {
            const double v = PnT[c * kCholLd + K0 + lr];
            Lr[c] = c < ln ? v : 0.0;
        }
        double x = xs[K0 + lr];
#pragma unroll
        for (int k = 0; k < kCholNB; k++) {
            const double y = readlane_f64(x, k) * Rd[K0 + k];
            x -= Lr[k] * y;
        }
        if (ln < kCholNB) xs[K0 + ln] = x * Rd[K0 + ln];
    };
    double a[kCholNB];
    // round K1: [D] wave 0 factors the diagonal block at K1 while waves 1.. finish the previous
    // panel's trailing update (rows / columns K1 + 32 ..); then panel K1: [A] publish the block,
    // [B] the rows below, [C] the next panel's columns
    for (int K1 = 0;; K1 += kCholNB) {
        if (tid < 64) {
            if (!diag_block(K1) && lane == 0) bad = 1;
        } else if (K1 > 0) {
            // forward substitution, rows below the previous block: x_i -= sum_c L_i,c y_c (ascending c;
            // the block's y from [C], the panel still in PnT)
            const int Kp = K1 - kCholNB, i = K1 + (tid - 64);
            if (i < np) {
                double sx = xs[i];
#pragma unroll
                for (int c = 0; c < kCholNB; c++) sx -= PnT[c * kCholLd + i] * xs[Kp + c];
                xs[i] = sx;
            }
            const int base = K1 + kCholNB, m2 = (np - base) / 4;
            const int tiles = m2 * (m2 + 1) / 2;
            for (int t = tid - 64; t < tiles; t += nt - 64) {
                int ti = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
                while (ti * (ti + 1) / 2 > t) ti--;
                while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
                const int tj = t - ti * (ti + 1) / 2;
                tile_update(base + 4 * ti, base + 4 * tj, ti == tj);
            }
        }
        __syncthreads();
        BA_T(0);
        if (bad) break;
        const int K0 = K1, below = np - K0 - kCholNB, rb = tid - 64;
        // [A] wave 0 publishes the factored diagonal block (PnT for the rows below, S for the
        // substitutions); waves 1.. load the panel rows below it
        if (tid < 64) {
            // lane (i, h): row i, columns 16 h .. 16 h + 15 (the entries right of the diagonal are
            // garbage: neither PnT's nor S's upper part is read, and S is rebuilt by every
            // iteration's k_ba_schur)
            const int i = lane & 31, h = lane >> 5;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int c = 16 * h + q;
                const double v = Dg[i * 33 + c];
                PnT[c * kCholLd + K0 + i] = v;
                S[(size_t)(K0 + i) * np + K0 + c] = v;
            }
        } else if (rb < below) {
#pragma unroll
            for (int c = 0; c < kCholNB; c++) a[c] = S[(size_t)(K0 + kCholNB + rb) * np + K0 + c];
        }
        __syncthreads();
        if (below == 0) break;
        // [B] rows below: L_ic = (S_ic - sum_{k<c} L_ik L_ck) * R_c, column by column
        if (tid >= 64 && rb < below) {
            const int i = K0 + kCholNB + rb;
            // column c + 1 of the block is read from LDS while column c is applied (two columns of
            // reads in flight, not the whole block's: the scheduler would hoist them all and spill)
            double col[2][kCholNB];
#pragma unroll
            for (int j = 1; j < kCholNB; j++) col[0][j] = PnT[K0 + j];
#pragma unroll
            for (int c = 0; c < kCholNB; c++) {
                if (c + 1 < kCholNB)
#pragma unroll
                    for (int j = c + 2; j < kCholNB; j++) col[(c + 1) & 1][j] = PnT[(c + 1) * kCholLd + K0 + j];
                const double l = a[c] * Rd[K0 + c];
                a[c] = l;
#pragma unroll
                for (int j = c + 1; j < kCholNB; j++) a[j] -= l * col[c & 1][j];
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int c = 0; c < kCholNB; c++) {
                PnT[c * kCholLd + i] = a[c];
                S[(size_t)i * np + K0 + c] = a[c];
            }
        }
        __syncthreads();
        BA_T(1);
        // [C] the next panel's columns (K0 + 32 .. K0 + 63, every row from K0 + 32) take this panel,
        // so that the next diagonal block and rows below are complete
        // (wave 0 meanwhile: the forward substitution of this block, fwd_block)
        const int Kn = K0 + kCholNB, mt = below / 4;
        const int tiles = 8 * mt - 28;  // the 8 x 8 lower-triangular head (36 tiles) + 8 per row block below
        if (tid < 64) fwd_block(K0);
        for (int t = tid - 64; tid >= 64 && t < tiles; t += nt - 64) {
            int ti, tj;
            if (t < 36) {
                ti = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
                while (ti * (ti + 1) / 2 > t) ti--;
                while ((ti + 1) * (ti + 2) / 2 <= t) ti++;
                tj = t - ti * (ti + 1) / 2;
            } else {
                ti = 8 + (t - 36) / 8;
                tj = (t - 36) % 8;
            }
            tile_update(Kn + 4 * ti, Kn + 4 * tj, ti == tj);
        }
        __syncthreads();
        BA_T(2);
    }
    if (bad) {
        if (tid == 0) d.ctl->solved = 0;
        return;
    }
    // the last block's forward substitution (the other blocks' ran inside the factorization)
    if (tid < 64) fwd_block(np - kCholNB);
    __syncthreads();
    BA_T(3);
    // 4b. L^T x = y: x_i = (y_i - sum_{k>i, descending} L_ki x_k) * R_i (the block's column entries
    // above the diagonal zeroed the same way)
    for (int K0 = np - kCholNB; K0 >= 0; K0 -= kCholNB) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        double Lc[kCholNB];
        if (tid < 64) {
            const int lc = min(ln, kCholNB - 1);
#pragma unroll
            for (int k = 0; k < kCholNB; k++) {
                const double v = S[(size_t)(K0 + k) * np + K0 + lc];
                Lc[k] = k > ln ? v : 0.0;
            }
            double x = xs[K0 + lc];
#pragma unroll
            for (int k = kCholNB - 1; k >= 0; k--) {
                const double v = readlane_f64(x, k) * Rd[K0 + k];
                x -= Lc[k] * v;
            }
            if (ln < kCholNB) xs[K0 + ln] = x * Rd[K0 + ln];
        } else {
            // the rows above: column i of the block's rows, loaded while wave 0 solves the block
            const int i = min(tid - 64, np - 1);
#pragma unroll
            for (int k = 0; k < kCholNB; k++) Lc[k] = S[(size_t)(K0 + k) * np + i];
        }
        __syncthreads();
        if (tid >= 64 && tid - 64 < K0) {
            const int i = tid - 64;
            double s = xs[i];
#pragma unroll
            for (int k = kCholNB - 1; k >= 0; k--) s -= Lc[k] * xs[K0 + k];
            xs[i] = s;
        }
        __syncthreads();
    }
    BA_T(4);
    for (int i = tid; i < n; i += nt) d.dp[i] = xs[i];
    if (tid == 0) d.ctl->solved = 1;
}

__global__ void k_ba_update(BaDev d) {
    BA_LIVE(d);
    if (!d.ctl->solved) return;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < d.M) {
        const int j = g;
        double rhs[3] = {-d.bm[3 * (size_t)j], -d.bm[3 * (size_t)j + 1], -d.bm[3 * (size_t)j + 2]};
        for (int p = d.pv_off[j]; p < d.pv_off[j + 1]; p++)
            ba_backsub_add(d.Hpm + 18 * (size_t)p, d.dp + 6 * d.pv_kf[p], rhs);
        const double* Hi = d.Hinv + 9 * (size_t)j;
        for (int c = 0; c < 3; c++)
            d.P_new[3 * (size_t)j + c] =
                d.P[3 * (size_t)j + c] + (Hi[c * 3 + 0] * rhs[0] + Hi[c * 3 + 1] * rhs[1] + Hi[c * 3 + 2] * rhs[2]);
    } else if (g < d.M + d.N) {
        const int i = g - d.M;
        for (int k = 0; k < 3; k++) {
            d.rv_new[3 * i + k] = d.rv[3 * i + k] + d.dp[6 * i + k];
            d.tv_new[3 * i + k] = d.tv[3 * i + k] + d.dp[6 * i + 3 + k];
        }
        pose_cache(d.rv_new + 3 * i, d.tv_new + 3 * i, d.pc_new[i]);  // for the new cost
    }
}

// an accepted step: the new parameters become current, and so does the pose cache (pc always
// belongs to rv / tv, so no pose-cache launch starts an iteration)
__global__ void k_ba_commit(BaDev d) {
    if (!d.ctl->take) return;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < 3 * d.M) {
        d.P[g] = d.P_new[g];
    } else if (g < 3 * d.M + d.N) {
        const int i = g - 3 * d.M;
        for (int k = 0; k < 3; k++) {
            d.rv[3 * i + k] = d.rv_new[3 * i + k];
            d.tv[3 * i + k] = d.tv_new[3 * i + k];
        }
        pose_cache(d.rv + 3 * i, d.tv + 3 * i, d.pc[i]);
    }
}

__global__ void k_ba_finish(BaDev d, double* R, double* t, double* P_out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < d.N) {
        if (g >= 1) {  // :584-588
            vs_pnp::rod_v2m(d.rv + 3 * g, R + 9 * g);
            for (int k = 0; k < 3; k++) t[3 * g + k] = d.tv[3 * g + k];
        }
    }
    if (g < 3 * d.M) P_out[g] = d.P[g];
}

static inline int cdiv(long a, int b) { return (int)((a + b - 1) / b); }

int local_ba(vs_ctx* ctx, int N, double* R, double* t, int M, double* P, int n_obs, const int* okf, const int* opt,
             const double* ouv, const double K4[4], int max_iter, double* err_before, double* err_after, int stats[3]) {
    *err_before = *err_after = 0;
    if (stats) stats[0] = stats[1] = stats[2] = 0;
    if (N < 2 || n_obs < 20 || M < 10) return VS_OK;  // :218, :250
    VS_ARG(N <= VS_BA_MAX_KEYFRAMES, "vs_local_ba: more keyframes than VS_BA_MAX_KEYFRAMES");
    for (int o = 0; o < n_obs; o++)
        VS_ARG(okf[o] >= 0 && okf[o] < N && opt[o] >= 0 && opt[o] < M, "vs_local_ba: observation index out of range");
    // host phase wall times (VS_BA_HOST_PROFILE=1: one stderr line per call)
    static const bool hprof = std::getenv("VS_BA_HOST_PROFILE") != nullptr;
    using hclock = std::chrono::steady_clock;
    const hclock::time_point h0 = hclock::now();
    hclock::time_point h1 = h0, h2 = h0, h3 = h0;
    // ---- structure (host, once; flat arrays) ----
    auto csr = [&](const int* key, int nk, std::vector<int>& off, std::vector<int>& lst) {
        off.assign(nk + 1, 0);
        for (int o = 0; o < n_obs; o++) off[key[o] + 1]++;
        for (int k = 0; k < nk; k++) off[k + 1] += off[k];
        lst.resize(n_obs);
        std::vector<int> fill(off.begin(), off.end() - 1);
        for (int o = 0; o < n_obs; o++) lst[fill[key[o]]++] = o;  // ascending observation index
    };
    std::vector<int> kf_off, kf_obs, pt_off, pt_obs;
    csr(okf, N, kf_off, kf_obs);
    csr(opt, M, pt_off, pt_obs);
    // the observers of every point: its distinct keyframes in order of first appearance among its
    // observations (point_observers, :257-263), and every observation's slot among them
    std::vector<int> oslot(n_obs), pv_off(M + 1), pv_kf(n_obs);
    int n_pairs = 0;
    for (int j = 0; j < M; j++) {
        const int b0 = n_pairs;
        pv_off[j] = b0;
        for (int q = pt_off[j]; q < pt_off[j + 1]; q++) {
            const int o = pt_obs[q], k = okf[o];
            int sl = 0;
            while (b0 + sl < n_pairs && pv_kf[b0 + sl] != k) sl++;
            if (b0 + sl == n_pairs) pv_kf[n_pairs++] = k;
            oslot[o] = sl;
        }
    }
    pv_off[M] = n_pairs;
    // common points per (a, b), ascending j, with the U (j, a) and Hpm (j, b) pair indices; and the
    // points of every keyframe, ascending, with U (j, a)
    std::vector<int> ab_cnt(N * N, 0), kb_cnt(N, 0);
    for (int j = 0; j < M; j++) {
        const int* ob = pv_kf.data() + pv_off[j];
        const int no = pv_off[j + 1] - pv_off[j];
        for (int x = 0; x < no; x++) {
            kb_cnt[ob[x]]++;
            for (int y = 0; y < no; y++) ab_cnt[ob[x] * N + ob[y]]++;
        }
    }
    // S's band: block (a, b) is nonzero only when a point is seen by both keyframes
    int band_blocks = 0;
    for (int a = 0; a < N; a++)
        for (int b = 0; b < a; b++)
            if (ab_cnt[a * N + b]) band_blocks = std::max(band_blocks, a - b);
    std::vector<int> ab_off(N * N + 1, 0), kb_off(N + 1, 0);
    for (int p = 0; p < N * N; p++) ab_off[p + 1] = ab_off[p] + ab_cnt[p];
    for (int a = 0; a < N; a++) kb_off[a + 1] = kb_off[a] + kb_cnt[a];
    std::vector<int> ab_u(ab_off.back()), ab_h(ab_off.back()), ab_j(ab_off.back()), kb_u(kb_off.back()),
        kb_j(kb_off.back());
    {
        std::vector<int> fa(ab_off.begin(), ab_off.end() - 1), fk(kb_off.begin(), kb_off.end() - 1);
        for (int j = 0; j < M; j++) {
            const int* ob = pv_kf.data() + pv_off[j];
            const int no = pv_off[j + 1] - pv_off[j];
            for (int x = 0; x < no; x++) {
                const int a = ob[x];
                kb_u[fk[a]] = pv_off[j] + x;
                kb_j[fk[a]++] = j;
                for (int y = 0; y < no; y++) {
                    const int p = a * N + ob[y];
                    ab_u[fa[p]] = pv_off[j] + x;
                    ab_h[fa[p]] = pv_off[j] + y;
                    ab_j[fa[p]++] = j;
                }
            }
        }
    }
    // ---- device buffers (one allocation) ----
    const int n_chunks = cdiv(n_obs, kCostChunk);
    const int n = 6 * N, np = (n + 31) / 32 * 32;
    size_t bytes = 0;
    auto take = [&](size_t b) {
        const size_t at = bytes;
        bytes += (b + 255) & ~(size_t)255;
        return at;
    };
    const size_t o_okf = take(4ull * n_obs), o_opt = take(4ull * n_obs), o_oslot = take(4ull * n_obs),
                 o_kfoff = take(4ull * (N + 1)), o_kfobs = take(4ull * n_obs), o_ptoff = take(4ull * (M + 1)),
                 o_ptobs = take(4ull * n_obs), o_pvoff = take(4ull * (M + 1)), o_pvkf = take(4ull * n_pairs),
                 o_aboff = take(4ull * (N * N + 1)), o_abu = take(4ull * ab_u.size()),
                 o_abh = take(4ull * ab_h.size()), o_abj = take(4ull * ab_j.size()), o_kboff = take(4ull * (N + 1)),
                 o_kbu = take(4ull * kb_u.size()), o_kbj = take(4ull * kb_j.size()), o_ouv = take(16ull * n_obs),
                 o_R = take(72ull * N), o_t = take(24ull * N), o_rv = take(24ull * N), o_tv = take(24ull * N),
                 o_P = take(24ull * M), o_rvn = take(24ull * N), o_tvn = take(24ull * N), o_Pn = take(24ull * M),
                 o_pc = take(sizeof(PoseC) * N), o_pcn = take(sizeof(PoseC) * N),
                 o_terms = take(sizeof(ObsTerms) * (size_t)n_obs), o_Hpp = take(288ull * N), o_bp = take(48ull * N),
                 o_Hmm = take(72ull * M), o_bm = take(24ull * M), o_Hpm = take(144ull * n_pairs),
                 o_Hinv = take(72ull * M), o_U = take(144ull * n_pairs), o_S = take(8ull * np * np),
                 o_bs = take(8ull * n), o_dp = take(8ull * n), o_chunk = take(8ull * n_chunks),
                 o_pvalid = take(4ull * M), o_ctl = take(sizeof(BaCtl));
    h1 = hclock::now();
    VS_CHECK(ctx->ba.ensure(bytes));
    char* base = ctx->ba.as<char>();
    if (!ctx->ba_done_h) {
        VS_HIP(hipHostMalloc((void**)&ctx->ba_done_h, 64, hipHostMallocMapped));
        VS_HIP(hipHostGetDevicePointer((void**)&ctx->ba_done_d, ctx->ba_done_h, 0));
        for (hipEvent_t& e : ctx->ba_ev) VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    volatile int* done_h = ctx->ba_done_h;
    *done_h = 0;
    hipStream_t s = ctx->stream;
    auto up = [&](size_t off, const void* src, size_t n_bytes) {
        return hipMemcpyAsync(base + off, src, n_bytes, hipMemcpyHostToDevice, s);
    };
    VS_HIP(up(o_okf, okf, 4ull * n_obs));
    VS_HIP(up(o_opt, opt, 4ull * n_obs));
    VS_HIP(up(o_oslot, oslot.data(), 4ull * n_obs));
    VS_HIP(up(o_kfoff, kf_off.data(), 4ull * (N + 1)));
    VS_HIP(up(o_kfobs, kf_obs.data(), 4ull * n_obs));
    VS_HIP(up(o_ptoff, pt_off.data(), 4ull * (M + 1)));
    VS_HIP(up(o_ptobs, pt_obs.data(), 4ull * n_obs));
    VS_HIP(up(o_pvoff, pv_off.data(), 4ull * (M + 1)));
    if (n_pairs) VS_HIP(up(o_pvkf, pv_kf.data(), 4ull * n_pairs));
    VS_HIP(up(o_aboff, ab_off.data(), 4ull * (N * N + 1)));
    if (!ab_u.empty()) {
        VS_HIP(up(o_abu, ab_u.data(), 4ull * ab_u.size()));
        VS_HIP(up(o_abh, ab_h.data(), 4ull * ab_h.size()));
        VS_HIP(up(o_abj, ab_j.data(), 4ull * ab_j.size()));
    }
    VS_HIP(up(o_kboff, kb_off.data(), 4ull * (N + 1)));
    if (!kb_u.empty()) {
        VS_HIP(up(o_kbu, kb_u.data(), 4ull * kb_u.size()));
        VS_HIP(up(o_kbj, kb_j.data(), 4ull * kb_j.size()));
    }
    VS_HIP(up(o_ouv, ouv, 16ull * n_obs));
    VS_HIP(up(o_R, R, 72ull * N));
    VS_HIP(up(o_t, t, 24ull * N));
    VS_HIP(up(o_tv, t, 24ull * N));
    VS_HIP(up(o_P, P, 24ull * M));
    BaCtl ctl0{};
    ctl0.lambda = 1e-4;
    ctl0.max_iter = max_iter;
    ctl0.done = max_iter <= 0;
    VS_HIP(up(o_ctl, &ctl0, sizeof(ctl0)));

    h2 = hclock::now();
    BaDev d;
    d.N = N;
    d.M = M;
    d.n_obs = n_obs;
    d.n_pairs = n_pairs;
    d.n_chunks = n_chunks;
    d.np = np;
    d.band = 6 * band_blocks + 5;
    d.K = Cam{K4[0], K4[1], K4[2], K4[3]};
    // the banded Cholesky when the band fits it (VS_BA_BAND=0: always the dense kernel, A/B)
    static const bool band_off = [] {
        const char* e = std::getenv("VS_BA_BAND");
        return e && e[0] == '0';
    }();
    bool use_band = !band_off && d.band + 1 <= kBandMaxW;
    void (*chol_band)(BaDev) = nullptr;  // the instantiation for the band's elements per lane
    switch (band_slots(d.band)) {
        case 1: chol_band = k_ba_chol_band<1>; break;
        case 2: chol_band = k_ba_chol_band<2>; break;
        case 3: chol_band = k_ba_chol_band<3>; break;
        case 5: chol_band = k_ba_chol_band<5>; break;
        case 7: chol_band = k_ba_chol_band<7>; break;
        case 10: chol_band = k_ba_chol_band<10>; break;
        default: use_band = false;  // (band = 6 Bb + 5 gives 1, 2, 3, 5, 7 or 10)
    }
#define BA_PTR(T, o) reinterpret_cast<T*>(base + (o))
    d.okf = BA_PTR(int, o_okf);
    d.opt = BA_PTR(int, o_opt);
    d.oslot = BA_PTR(int, o_oslot);
    d.kf_off = BA_PTR(int, o_kfoff);
    d.kf_obs = BA_PTR(int, o_kfobs);
    d.pt_off = BA_PTR(int, o_ptoff);
    d.pt_obs = BA_PTR(int, o_ptobs);
    d.pv_off = BA_PTR(int, o_pvoff);
    d.pv_kf = BA_PTR(int, o_pvkf);
    d.ab_off = BA_PTR(int, o_aboff);
    d.ab_u = BA_PTR(int, o_abu);
    d.ab_h = BA_PTR(int, o_abh);
    d.ab_j = BA_PTR(int, o_abj);
    d.kb_off = BA_PTR(int, o_kboff);
    d.kb_u = BA_PTR(int, o_kbu);
    d.kb_j = BA_PTR(int, o_kbj);
    d.ouv = BA_PTR(double, o_ouv);
    d.rv = BA_PTR(double, o_rv);
    d.tv = BA_PTR(double, o_tv);
    d.P = BA_PTR(double, o_P);
    d.rv_new = BA_PTR(double, o_rvn);
    d.tv_new = BA_PTR(double, o_tvn);
    d.P_new = BA_PTR(double, o_Pn);
    d.pc = BA_PTR(PoseC, o_pc);
    d.pc_new = BA_PTR(PoseC, o_pcn);
    d.terms = BA_PTR(ObsTerms, o_terms);
    d.Hpp = BA_PTR(double, o_Hpp);
    d.bp = BA_PTR(double, o_bp);
    d.Hmm = BA_PTR(double, o_Hmm);
    d.bm = BA_PTR(double, o_bm);
    d.Hpm = BA_PTR(double, o_Hpm);
    d.Hinv = BA_PTR(double, o_Hinv);
    d.U = BA_PTR(double, o_U);
    d.S = BA_PTR(double, o_S);
    d.bs = BA_PTR(double, o_bs);
    d.dp = BA_PTR(double, o_dp);
    d.chunk = BA_PTR(double, o_chunk);
    d.pvalid = BA_PTR(int, o_pvalid);
    d.ctl = BA_PTR(BaCtl, o_ctl);
    d.done_host = ctx->ba_done_d;
#undef BA_PTR
    {
        ProfScope ps(ctx, "local_ba", s);
        const int T = 256;
        hipLaunchKernelGGL(k_ba_init, dim3(cdiv(N, T)), dim3(T), 0, s, d, (const double*)(base + o_R));
        if (np > n) hipLaunchKernelGGL(k_ba_pad, dim3(cdiv((long)(np - n) * np, T)), dim3(T), 0, s, d);
        hipLaunchKernelGGL(k_ba_pose_cache, dim3(cdiv(N, T)), dim3(T), 0, s, d, 0, 0);
        hipLaunchKernelGGL(k_ba_cost, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 2, 0, 2);
        // Iteration it is enqueued once iteration it - 2 has finished and had not converged (the
        // flag ba_control mirrors to the host): the device always has the next iteration queued,
        // and at most one iteration past convergence is enqueued, where every launch returns at once.
        for (int it = 0; it < max_iter; it++) {
            if (it >= 2) {
                VS_HIP(hipEventSynchronize(ctx->ba_ev[it & 1]));
                if (*done_h) break;
            }
            hipLaunchKernelGGL(k_ba_obs, dim3(cdiv(n_obs, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_cost, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 0, 1, 0);
            hipLaunchKernelGGL(k_ba_kf_acc, dim3(N), dim3(64), 0, s, d);
            hipLaunchKernelGGL(k_ba_pt_acc, dim3(cdiv(M, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_schur, dim3(N * N + N), dim3(64), 0, s, d);
            if (use_band)
                hipLaunchKernelGGL(chol_band, dim3(1), dim3(kBandThreads), 0, s, d);
            else
                hipLaunchKernelGGL(k_ba_chol, dim3(1), dim3(512), 0, s, d);
            hipLaunchKernelGGL(k_ba_update, dim3(cdiv(M + N, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_cost, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 1, 1, 1);
            hipLaunchKernelGGL(k_ba_commit, dim3(cdiv(3 * M + N, T)), dim3(T), 0, s, d);
            VS_HIP(hipEventRecord(ctx->ba_ev[it & 1], s));
        }
        hipLaunchKernelGGL(k_ba_cost, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 2, 0, 3);
        hipLaunchKernelGGL(k_ba_finish, dim3(cdiv(3 * M + N, T)), dim3(T), 0, s, d, (double*)(base + o_R),
                           (double*)(base + o_t), (double*)(base + o_Pn));
        VS_HIP(hipGetLastError());
    }
    h3 = hclock::now();
    BaCtl out;
    VS_HIP(hipMemcpyAsync(&out, base + o_ctl, sizeof(out), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(R, base + o_R, 72ull * N, hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(t, base + o_t, 24ull * N, hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(P, base + o_Pn, 24ull * M, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    if (hprof) {
        auto ms = [](hclock::time_point a, hclock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        std::fprintf(stderr, "vs_local_ba host: structure %.3f ms, upload %.3f ms, enqueue %.3f ms, wait %.3f ms\n",
                     ms(h0, h1), ms(h1, h2), ms(h2, h3), ms(h3, hclock::now()));
    }
    *err_before = out.err_before;
    *err_after = out.err_after;
    if (stats) {
        stats[0] = out.iter;
        stats[1] = out.accepted;
        stats[2] = 1;
    }
    return VS_OK;
}

}  // namespace vs

#ifdef VS_BA_PROFILE
extern "C" int vs_debug_ba_cycles(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_ba_cycles), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_ba_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
