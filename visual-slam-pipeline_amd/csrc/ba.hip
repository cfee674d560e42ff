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
//   k_ba_chol         dense right-looking Cholesky + the two triangular solves (one workgroup)
//   k_ba_update       back-substitution dm = Hinv (-bm - sum Hpm^T dp), new poses
//   k_ba_chunk_sums / k_ba_control   new cost, accept / reject, lambda, convergence
// Every element is accumulated in the same order as the CPU restatement (oracle/orc_ba.cpp); the
// global cost sums use fixed chunks of 256 observations.  Arithmetic shared via ba_solvers.h.
#include <hip/hip_runtime.h>

#include <vector>

#include "ba_solvers.h"
#include "vs_internal.h"

namespace vs {

using namespace vs_ba;

struct BaCtl {
    double lambda, total_cost, new_cost, err_before, err_after;
    int iter, accepted, done, solved, take, max_iter;
};

struct BaDev {
    int N, M, n_obs, n_pairs, n_chunks;
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

// mode 0: total_cost from the terms; 1: new_cost (new params); 2: squared error (current params).
// One 256-lane workgroup per fixed chunk of kCostChunk observations: the per-observation terms in
// parallel into LDS, then lane 0 sums them in observation order (the oracle's chunked order).
__global__ __launch_bounds__(kCostChunk) void k_ba_chunk_sums(BaDev d, int mode, int check) {
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
        d.chunk[c] = sum;
    }
}

// Hpp, bp per keyframe in gather order (:407-451), one 64-lane workgroup per keyframe: lane
// l < 21 owns upper-triangular element l of Hpp (mirrored), lanes 21..26 own bp — each element is
// the same sequential sum over the keyframe's observations as in the oracle.  The observation
// indices are staged 64 at a time so the term loads do not wait on index loads.
__global__ __launch_bounds__(64) void k_ba_kf_acc(BaDev d) {
    BA_LIVE(d);
    __shared__ double s_t[64][15];  // per staged observation: Jp (12), ru_w, rv_w, valid
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
    double acc = 0;
    const int q0 = d.kf_off[i], q1 = d.kf_off[i + 1];
    for (int qb = q0; qb < q1; qb += 64) {
        if (qb + l < q1) {
            const ObsTerms& ot = d.terms[d.kf_obs[qb + l]];
            for (int k = 0; k < 6; k++) {
                s_t[l][k] = ot.Jp[0][k];
                s_t[l][6 + k] = ot.Jp[1][k];
            }
            s_t[l][12] = ot.ru_w;
            s_t[l][13] = ot.rv_w;
            s_t[l][14] = ot.valid ? 1.0 : 0.0;
        }
        __syncthreads();
        const int m = min(64, q1 - qb);
        if (l < 27)
            for (int k = 0; k < m; k++) {
                if (s_t[k][14] == 0.0) continue;
                if (l < 21)
                    acc += s_t[k][r] * s_t[k][c] + s_t[k][6 + r] * s_t[k][6 + c];
                else
                    acc += s_t[k][r] * s_t[k][12] + s_t[k][6 + r] * s_t[k][13];
            }
        __syncthreads();
    }
    if (l < 21) {
        if (r == c) acc += kPoseDamp;
        d.Hpp[36 * i + r * 6 + c] = acc;
        d.Hpp[36 * i + c * 6 + r] = acc;
    } else if (l < 27) {
        d.bp[6 * i + r] = acc;
    }
}

__global__ void k_ba_pt_acc(BaDev d) {
    BA_LIVE(d);
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d.M) return;
    double H[9], b[3];
    for (int k = 0; k < 9; k++) H[k] = 0;
    for (int k = 0; k < 3; k++) b[k] = 0;
    const int p0 = d.pv_off[j], np = d.pv_off[j + 1] - p0;
    for (int s = 0; s < np; s++)
        for (int k = 0; k < 18; k++) d.Hpm[18 * (size_t)(p0 + s) + k] = 0;
    for (int q = d.pt_off[j]; q < d.pt_off[j + 1]; q++) {
        const int o = d.pt_obs[q];
        const ObsTerms& ot = d.terms[o];
        if (!ot.valid) continue;
        ba_add_point(ot, H, b);
        ba_add_cross(ot, d.Hpm + 18 * (size_t)(p0 + d.oslot[o]));
    }
    for (int k = 0; k < 9; k++) d.Hmm[9 * (size_t)j + k] = H[k];
    for (int k = 0; k < 3; k++) d.bm[3 * (size_t)j + k] = b[k];
    double Hi[9];
    const bool ok = ba_point_inverse(H, d.ctl->lambda, Hi);
    d.pvalid[j] = ok;
    for (int k = 0; k < 9; k++) d.Hinv[9 * (size_t)j + k] = Hi[k];
    if (ok)
        for (int s = 0; s < np; s++) ba_schur_u(d.Hpm + 18 * (size_t)(p0 + s), Hi, d.U + 18 * (size_t)(p0 + s));
}

// grid: N*N workgroups of 64 threads; threads 0..35 own S_ab(r, c), threads 0..5 then own b_a(r)
// on the diagonal workgroups.  The (U, Hpm, point) index lists are staged 64 at a time in LDS so
// the products' loads do not wait on index loads; sums run over the lists in order (the oracle's).
__global__ __launch_bounds__(64) void k_ba_schur(BaDev d) {
    BA_LIVE(d);
    __shared__ double s_U[64][18], s_H[64][18];
    __shared__ int s_ok[64];
    const int a = blockIdx.x / d.N, b = blockIdx.x % d.N, t = threadIdx.x;
    const int n = 6 * d.N;
    const double lam = d.ctl->lambda;
    const int r = t / 6, c = t % 6;
    double s = 0.0;
    if (t < 36) {
        s = a == b ? d.Hpp[36 * a + r * 6 + c] : 0.0;
        if (a == b && r == c) s *= (1.0 + lam);
    }
    const int pair = a * d.N + b;
    const int q0 = d.ab_off[pair], q1 = d.ab_off[pair + 1];
    for (int qb = q0; qb < q1; qb += 64) {
        const int q = qb + t;
        if (q < q1) {
            const double* U = d.U + 18 * (size_t)d.ab_u[q];
            const double* Hh = d.Hpm + 18 * (size_t)d.ab_h[q];
            for (int k = 0; k < 18; k++) {
                s_U[t][k] = U[k];
                s_H[t][k] = Hh[k];
            }
            s_ok[t] = d.pvalid[d.ab_j[q]];
        }
        __syncthreads();
        const int m = min(64, q1 - qb);
        if (t < 36)
            for (int k = 0; k < m; k++)
                if (s_ok[k]) s -= ba_schur_s(s_U[k], s_H[k], r, c);
        __syncthreads();
    }
    if (t < 36) d.S[(size_t)(6 * a + r) * n + 6 * b + c] = s;
    if (a != b) return;
    double sb = t < 6 ? d.bp[6 * a + t] : 0.0;
    const int k0 = d.kb_off[a], k1 = d.kb_off[a + 1];
    for (int qb = k0; qb < k1; qb += 64) {
        const int q = qb + t;
        if (q < k1) {
            const int j = d.kb_j[q];
            const double* U = d.U + 18 * (size_t)d.kb_u[q];
            for (int k = 0; k < 18; k++) s_U[t][k] = U[k];
            for (int k = 0; k < 3; k++) s_H[t][k] = d.bm[3 * (size_t)j + k];
            s_ok[t] = d.pvalid[j];
        }
        __syncthreads();
        const int m = min(64, k1 - qb);
        if (t < 6)
            for (int k = 0; k < m; k++)
                if (s_ok[k]) sb -= ba_schur_b(s_U[k], s_H[k], t);
        __syncthreads();
    }
    if (t < 6) d.bs[6 * a + t] = sb;
}

// Right-looking Cholesky of S (lower triangle) and S dp = -bs, blocked, one workgroup:
//   * 32-column panels staged in LDS; one thread per panel row; per column every thread takes
//     the pivot sqrt itself and divides the column entries it needs on the fly, so one barrier
//     per column suffices (the divided column is stored one step later, when nothing reads it);
//   * the trailing lower triangle is updated by all waves in 4 x 4 register tiles;
//   * both triangular solves are blocked the same way: the rows below (above) a finished block
//     take that block's contributions in parallel, the 32 x 32 diagonal block is solved by one
//     wave out of LDS.
// Every element still receives its updates in the order of the oracle's sequential chol_solve
// (orc_ba.cpp: ascending k for the factor and the forward solve, descending k for the backward
// solve), so the factor and the solution are bit-identical.
constexpr int kCholNB = 32;
constexpr int kCholLd = kCholNB + 1;  // LDS row stride: rows one thread apart fall in different banks
constexpr int kCholMaxN = 6 * VS_BA_MAX_KEYFRAMES;

#ifdef VS_BA_PROFILE
// phase cycle counters of k_ba_chol (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_ba_cycles[8];
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

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(1024) void k_ba_chol(BaDev d) {
    BA_LIVE(d);
    const int n = 6 * d.N, tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    double* S = d.S;
    __shared__ double Pn[kCholMaxN * kCholLd];  // panel rows K0..n-1 x columns K0..K0+nb-1
    __shared__ double xs[kCholMaxN];
    __shared__ double Db[kCholNB * kCholLd];  // diagonal block for the solves
    __shared__ double Lc[kCholMaxN];           // the divided panel column of the current step
    __shared__ double s_piv;
    __shared__ int bad;
    if (tid == 0) bad = 0;
    __syncthreads();
    BA_T0();
    for (int K0 = 0; K0 < n; K0 += kCholNB) {
        const int nb = min(kCholNB, n - K0), rows = n - K0;
        for (int e = tid; e < rows * nb; e += nt) {
            const int r = e / nb, c = e % nb;
            Pn[r * kCholLd + c] = S[(size_t)(K0 + r) * n + K0 + c];
        }
        __syncthreads();
        BA_T(0);
        // panel: thread r owns row r, held in registers (columns unrolled).  Step kk: the owner of
        // row kk publishes the pivot sqrt; every row below divides its column-kk entry once and
        // publishes it in Lc; then each row applies column kk to its columns kk+1.. .
        double prow[kCholNB];
        const bool own = tid < rows;
#pragma unroll
        for (int c = 0; c < kCholNB; c++) prow[c] = (own && c < nb) ? Pn[tid * kCholLd + c] : 0.0;
        bool stop = false;
#pragma unroll
        for (int kk = 0; kk < kCholNB; kk++) {
            if (kk < nb && !stop) {
                if (tid == kk) {
                    const double v = prow[kk];
                    if (!(v > 0)) bad = 1;
                    s_piv = sqrt(v);
                    prow[kk] = s_piv;
                }
                __syncthreads();
                stop = bad != 0;
                if (!stop) {
                    const double piv = s_piv;
                    double lrk = 0.0;
                    if (own && tid > kk) {
                        lrk = prow[kk] / piv;
                        prow[kk] = lrk;
                        Lc[tid] = lrk;
                    }
                    __syncthreads();
                    if (own && tid > kk) {
#pragma unroll
                        for (int c = kk + 1; c < kCholNB; c++)
                            if (c < nb && c <= tid) prow[c] -= lrk * Lc[c];
                    }
                }
            }
        }
        __syncthreads();
        if (own && !bad)
#pragma unroll
            for (int c = 0; c < kCholNB; c++)
                if (c < nb && c <= tid) Pn[tid * kCholLd + c] = prow[c];
        __syncthreads();
        BA_T(1);
        if (bad) break;
        for (int e = tid; e < rows * nb; e += nt) {  // the factored L columns
            const int r = e / nb, c = e % nb;
            if (c <= r) S[(size_t)(K0 + r) * n + K0 + c] = Pn[r * kCholLd + c];
        }
        // trailing lower triangle (rows / columns K0 + nb ..), 4 x 4 tiles on or below the diagonal
        const int base = nb, m = rows - nb;
        const int mt = (m + 3) / 4;
        const long tiles = (long)mt * (mt + 1) / 2;
        for (long t = tid; t < tiles; t += nt) {
            int ti = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
            while ((long)ti * (ti + 1) / 2 > t) ti--;
            while ((long)(ti + 1) * (ti + 2) / 2 <= t) ti++;
            const int tj = (int)(t - (long)ti * (ti + 1) / 2);
            double acc[4][4];
            int ri[4], cj[4];
#pragma unroll
            for (int x = 0; x < 4; x++) {
                ri[x] = base + 4 * ti + x;
                cj[x] = base + 4 * tj + x;
            }
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++)
                    acc[x][y] = (ri[x] < rows && cj[y] <= ri[x]) ? S[(size_t)(K0 + ri[x]) * n + K0 + cj[y]] : 0.0;
            for (int kk = 0; kk < nb; kk++) {
                double a[4], b[4];
#pragma unroll
                for (int x = 0; x < 4; x++) {
                    a[x] = ri[x] < rows ? Pn[ri[x] * kCholLd + kk] : 0.0;
                    b[x] = cj[x] < rows ? Pn[cj[x] * kCholLd + kk] : 0.0;
                }
#pragma unroll
                for (int x = 0; x < 4; x++)
#pragma unroll
                    for (int y = 0; y < 4; y++) acc[x][y] -= a[x] * b[y];
            }
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++)
                    if (ri[x] < rows && cj[y] <= ri[x]) S[(size_t)(K0 + ri[x]) * n + K0 + cj[y]] = acc[x][y];
        }
        __syncthreads();
        BA_T(2);
    }
    if (bad) {
        if (tid == 0) d.ctl->solved = 0;
        return;
    }
    // L y = -bs: block by block; y[i] = (b[i] - sum_{k < i} L[i][k] y[k]) / L[i][i], the sum in
    // ascending k (the oracle's column sweep applies the same subtractions in the same order)
    for (int i = tid; i < n; i += nt) xs[i] = -d.bs[i];
    __syncthreads();
    for (int K0 = 0; K0 < n; K0 += kCholNB) {
        const int nb = min(kCholNB, n - K0);
        for (int e = tid; e < nb * nb; e += nt) Db[(e / nb) * kCholLd + e % nb] = S[(size_t)(K0 + e / nb) * n + K0 + e % nb];
        __syncthreads();
        if (tid < 64) {  // lane i holds x[K0 + i] and row i of the diagonal block
            double x = lane < nb ? xs[K0 + lane] : 0.0;
            double drow[kCholNB];
#pragma unroll
            for (int j = 0; j < kCholNB; j++) drow[j] = (lane < nb && j <= lane && j < nb) ? Db[lane * kCholLd + j] : 1.0;
#pragma unroll
            for (int k = 0; k < kCholNB; k++) {
                if (k < nb) {
                    const double q = x / drow[k];  // lane k: x[k] /= L[k][k]
                    if (lane == k) x = q;
                    const double xk = __shfl(q, k);
                    if (lane > k && lane < nb) x -= drow[k] * xk;
                }
            }
            if (lane < nb) xs[K0 + lane] = x;
        }
        __syncthreads();
        for (int i = K0 + nb + tid; i < n; i += nt) {  // rows below take this block, ascending k
            double s = xs[i];
            const double* Li = S + (size_t)i * n + K0;
            for (int k = 0; k < nb; k++) s -= Li[k] * xs[K0 + k];
            xs[i] = s;
        }
        __syncthreads();
    }
    BA_T(3);
    // L^T x = y: blocks from the last; rows above take a finished block in descending k
    const int nblk = (n + kCholNB - 1) / kCholNB;
    for (int bI = nblk - 1; bI >= 0; bI--) {
        const int K0 = bI * kCholNB, nb = min(kCholNB, n - K0);
        for (int e = tid; e < nb * nb; e += nt) Db[(e / nb) * kCholLd + e % nb] = S[(size_t)(K0 + e / nb) * n + K0 + e % nb];
        __syncthreads();
        if (tid < 64) {  // lane i holds x[K0 + i] and column i of the diagonal block
            double x = lane < nb ? xs[K0 + lane] : 0.0;
            double dcol[kCholNB];
#pragma unroll
            for (int j = 0; j < kCholNB; j++) dcol[j] = (lane < nb && j >= lane && j < nb) ? Db[j * kCholLd + lane] : 1.0;
#pragma unroll
            for (int kq = kCholNB - 1; kq >= 0; kq--) {
                if (kq < nb) {
                    const double q = x / dcol[kq];  // lane kq: x[kq] /= L[kq][kq]
                    if (lane == kq) x = q;
                    const double xk = __shfl(q, kq);
                    if (lane < kq) x -= dcol[kq] * xk;
                }
            }
            if (lane < nb) xs[K0 + lane] = x;
        }
        __syncthreads();
        for (int i = tid; i < K0; i += nt) {
            double s = xs[i];
            for (int k = nb - 1; k >= 0; k--) s -= S[(size_t)(K0 + k) * n + i] * xs[K0 + k];
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
    }
}

// mode 0: total_cost; 1: new cost + accept/reject; 2: err_before; 3: err_after
__global__ void k_ba_control(BaDev d, int mode) {
    BaCtl& c = *d.ctl;
    if (mode <= 1 && c.done) return;
    double s = 0;
    for (int k = 0; k < d.n_chunks; k++) s += d.chunk[k];
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
}

__global__ void k_ba_commit(BaDev d) {
    if (!d.ctl->take) return;
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < 3 * d.M)
        d.P[g] = d.P_new[g];
    else if (g < 3 * d.M + 3 * d.N) {
        const int k = g - 3 * d.M;
        d.rv[k] = d.rv_new[k];
        d.tv[k] = d.tv_new[k];
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
    // ---- structure (host, once) ----
    std::vector<std::vector<int>> observers(M);
    std::vector<int> oslot(n_obs);
    for (int o = 0; o < n_obs; o++) {
        auto& ob = observers[opt[o]];
        int s = 0;
        while (s < (int)ob.size() && ob[s] != okf[o]) s++;
        if (s == (int)ob.size()) ob.push_back(okf[o]);
        oslot[o] = s;
    }
    std::vector<int> pv_off(M + 1, 0), pv_kf;
    for (int j = 0; j < M; j++) {
        pv_off[j + 1] = pv_off[j] + (int)observers[j].size();
        pv_kf.insert(pv_kf.end(), observers[j].begin(), observers[j].end());
    }
    const int n_pairs = pv_off[M];
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
    // common points per (a, b), ascending j, with the U (j, a) and Hpm (j, b) pair indices; and the
    // points of every keyframe, ascending, with U (j, a)
    std::vector<int> ab_cnt(N * N, 0), kb_cnt(N, 0);
    for (int j = 0; j < M; j++) {
        const int no = (int)observers[j].size();
        for (int x = 0; x < no; x++) {
            kb_cnt[observers[j][x]]++;
            for (int y = 0; y < no; y++) ab_cnt[observers[j][x] * N + observers[j][y]]++;
        }
    }
    std::vector<int> ab_off(N * N + 1, 0), kb_off(N + 1, 0);
    for (int p = 0; p < N * N; p++) ab_off[p + 1] = ab_off[p] + ab_cnt[p];
    for (int a = 0; a < N; a++) kb_off[a + 1] = kb_off[a] + kb_cnt[a];
    std::vector<int> ab_u(ab_off.back()), ab_h(ab_off.back()), ab_j(ab_off.back()), kb_u(kb_off.back()),
        kb_j(kb_off.back());
    {
        std::vector<int> fa(ab_off.begin(), ab_off.end() - 1), fk(kb_off.begin(), kb_off.end() - 1);
        for (int j = 0; j < M; j++) {
            const int no = (int)observers[j].size();
            for (int x = 0; x < no; x++) {
                const int a = observers[j][x];
                kb_u[fk[a]] = pv_off[j] + x;
                kb_j[fk[a]++] = j;
                for (int y = 0; y < no; y++) {
                    const int p = a * N + observers[j][y];
                    ab_u[fa[p]] = pv_off[j] + x;
                    ab_h[fa[p]] = pv_off[j] + y;
                    ab_j[fa[p]++] = j;
                }
            }
        }
    }
    // ---- device buffers (one allocation) ----
    const int n_chunks = cdiv(n_obs, kCostChunk);
    const int n = 6 * N;
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
                 o_Hinv = take(72ull * M), o_U = take(144ull * n_pairs), o_S = take(8ull * n * n),
                 o_bs = take(8ull * n), o_dp = take(8ull * n), o_chunk = take(8ull * n_chunks),
                 o_pvalid = take(4ull * M), o_ctl = take(sizeof(BaCtl));
    VS_CHECK(ctx->ba.ensure(bytes));
    char* base = ctx->ba.as<char>();
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

    BaDev d;
    d.N = N;
    d.M = M;
    d.n_obs = n_obs;
    d.n_pairs = n_pairs;
    d.n_chunks = n_chunks;
    d.K = Cam{K4[0], K4[1], K4[2], K4[3]};
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
#undef BA_PTR
    {
        ProfScope ps(ctx, "local_ba", s);
        const int T = 256;
        hipLaunchKernelGGL(k_ba_init, dim3(cdiv(N, T)), dim3(T), 0, s, d, (const double*)(base + o_R));
        hipLaunchKernelGGL(k_ba_pose_cache, dim3(cdiv(N, T)), dim3(T), 0, s, d, 0, 0);
        hipLaunchKernelGGL(k_ba_chunk_sums, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 2, 0);
        hipLaunchKernelGGL(k_ba_control, dim3(1), dim3(1), 0, s, d, 2);
        for (int it = 0; it < max_iter; it++) {
            hipLaunchKernelGGL(k_ba_pose_cache, dim3(cdiv(N, T)), dim3(T), 0, s, d, 0, 1);
            hipLaunchKernelGGL(k_ba_obs, dim3(cdiv(n_obs, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_chunk_sums, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 0, 1);
            hipLaunchKernelGGL(k_ba_control, dim3(1), dim3(1), 0, s, d, 0);
            hipLaunchKernelGGL(k_ba_kf_acc, dim3(N), dim3(64), 0, s, d);
            hipLaunchKernelGGL(k_ba_pt_acc, dim3(cdiv(M, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_schur, dim3(N * N), dim3(64), 0, s, d);
            hipLaunchKernelGGL(k_ba_chol, dim3(1), dim3(1024), 0, s, d);
            hipLaunchKernelGGL(k_ba_update, dim3(cdiv(M + N, T)), dim3(T), 0, s, d);
            hipLaunchKernelGGL(k_ba_pose_cache, dim3(cdiv(N, T)), dim3(T), 0, s, d, 1, 1);
            hipLaunchKernelGGL(k_ba_chunk_sums, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 1, 1);
            hipLaunchKernelGGL(k_ba_control, dim3(1), dim3(1), 0, s, d, 1);
            hipLaunchKernelGGL(k_ba_commit, dim3(cdiv(3 * M + 3 * N, T)), dim3(T), 0, s, d);
        }
        hipLaunchKernelGGL(k_ba_pose_cache, dim3(cdiv(N, T)), dim3(T), 0, s, d, 0, 0);
        hipLaunchKernelGGL(k_ba_chunk_sums, dim3(n_chunks), dim3(kCostChunk), 0, s, d, 2, 0);
        hipLaunchKernelGGL(k_ba_control, dim3(1), dim3(1), 0, s, d, 3);
        hipLaunchKernelGGL(k_ba_finish, dim3(cdiv(3 * M + N, T)), dim3(T), 0, s, d, (double*)(base + o_R),
                           (double*)(base + o_t), (double*)(base + o_Pn));
        VS_HIP(hipGetLastError());
    }
    BaCtl out;
    VS_HIP(hipMemcpyAsync(&out, base + o_ctl, sizeof(out), hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(R, base + o_R, 72ull * N, hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(t, base + o_t, 24ull * N, hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(P, base + o_Pn, 24ull * M, hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
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
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_ba_cycles), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_ba_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
