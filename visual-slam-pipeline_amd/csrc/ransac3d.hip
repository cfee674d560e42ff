// ransac3d.hip — Slam::estimate_motion_3d3d on gfx950 (reference src/Slam.cpp:214-375).
//
// One workgroup per frame pair.  The reference's loop is restated step for step, in fp64:
//   back-projection of the matched keypoints with round()-ed depth lookups and the (0.1, 10]
//   depth gate, order preserved (:236-262); N >= 10 (:265);
//   std::mt19937(42 + frame_count) sampling with the same rejection loops (:276-283) — the
//   generator is a bit-exact MT19937 (parallel 3-phase twist into LDS); the triples of all
//   iterations are found at once (the draws an iteration starting at draw c consumes, for every
//   c, then pointer doubling gives each iteration's first draw);
//   every hypothesis (3-point Kabsch: centroids, cross-covariance, one-sided Jacobi SVD,
//   reflection fix, t = c2 - R c1) and its inlier count over all N points runs on its own lane;
//   the first strictly-best iteration wins (:313-317, an exact max/min reduction), >= 10 inliers
//   (:320), the refit over all inliers (:324-358) keeps each of its sums a sequential chain in
//   the reference's order (one chain per lane), then the sanity gates (:361-372).
// Compiled with -ffp-contract=off, so results equal the CPU restatement (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include "vs_internal.h"

namespace vs {

constexpr int kMaxPts3d = 512;
constexpr int kMaxIters3d = 1024;
constexpr int kMtN = 624;
constexpr int kDraws3d = 2 * kMtN;  // outputs of the two parallel twists
constexpr int kLevels3d = 10;       // 2^10 >= kMaxIters3d attempts

#ifdef VS_R3_PROFILE
// k_ransac3d phase cycle counters (profiling build only: make -C visual-slam-pipeline_amd prof)
__device__ unsigned long long g_r3_cycles[8];
#define R3_T0() long long _r3_t = clock64()
#define R3_T(k)                                                             \
    do {                                                                    \
        if (threadIdx.x == 0) atomicAdd(&g_r3_cycles[k], clock64() - _r3_t); \
        _r3_t = clock64();                                                  \
    } while (0)
#else
#define R3_T0()
#define R3_T(k)
#endif

struct D3 {
    double x, y, z;
};

__device__ void svd3_dev(const double A[9], double U[9], double s[3], double V[9]) {
    double a[3][3];
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) a[c][r] = A[r * 3 + c];
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
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
                double conv = fabs(gamma) / sqrt(alpha * beta);
                if (!(conv > 1e-15)) continue;
                off = fmax(off, conv);
                double zeta = (beta - alpha) / (2.0 * gamma);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
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
    for (int c = 0; c < 3; c++) sv[c] = sqrt(a[c][0] * a[c][0] + a[c][1] * a[c][1] + a[c][2] * a[c][2]);
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; i++)
        for (int j = i + 1; j < 3; j++)
            if (sv[ord[j]] > sv[ord[i]]) {
                int tmp = ord[i];
                ord[i] = ord[j];
                ord[j] = tmp;
            }
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
    if (!(s[2] > 1e-12 * (s[0] > 0 ? s[0] : 1.0))) {
        u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
        u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
        u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
        double nn = sqrt(u[2][0] * u[2][0] + u[2][1] * u[2][1] + u[2][2] * u[2][2]);
        if (nn > 0)
            for (int r = 0; r < 3; r++) u[2][r] /= nn;
    }
    for (int k = 0; k < 3; k++)
        for (int r = 0; r < 3; r++) U[r * 3 + k] = u[k][r];
}

__device__ double det3_dev(const double M[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

__device__ void kabsch_dev(const double H[9], double R[9]) {
    double U[9], s[3], V[9];
    svd3_dev(H, U, s, V);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            R[i * 3 + j] = V[i * 3 + 0] * U[j * 3 + 0] + V[i * 3 + 1] * U[j * 3 + 1] + V[i * 3 + 2] * U[j * 3 + 2];
    if (det3_dev(R) < 0) {
        for (int i = 0; i < 3; i++) V[i * 3 + 2] = -V[i * 3 + 2];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                R[i * 3 + j] = V[i * 3 + 0] * U[j * 3 + 0] + V[i * 3 + 1] * U[j * 3 + 1] + V[i * 3 + 2] * U[j * 3 + 2];
    }
}

__device__ bool inlier_dev(const double R[9], const double t[3], const D3& p1, const D3& p2, double thr) {
    double qx = R[0] * p1.x + R[1] * p1.y + R[2] * p1.z + t[0];
    double qy = R[3] * p1.x + R[4] * p1.y + R[5] * p1.z + t[1];
    double qz = R[6] * p1.x + R[7] * p1.y + R[8] * p1.z + t[2];
    double dx = p2.x - qx, dy = p2.y - qy, dz = p2.z - qz;
    double ss = dx * dx;
    ss += dy * dy;
    ss += dz * dz;
    return sqrt(ss) < thr;
}

__device__ void hypothesis_dev(const D3* P1, const D3* P2, int i0, int i1, int i2, double R[9], double t[3]) {
    const int id[3] = {i0, i1, i2};
    D3 c1 = {(P1[i0].x + P1[i1].x + P1[i2].x) / 3.0, (P1[i0].y + P1[i1].y + P1[i2].y) / 3.0,
             (P1[i0].z + P1[i1].z + P1[i2].z) / 3.0};
    D3 c2 = {(P2[i0].x + P2[i1].x + P2[i2].x) / 3.0, (P2[i0].y + P2[i1].y + P2[i2].y) / 3.0,
             (P2[i0].z + P2[i1].z + P2[i2].z) / 3.0};
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 3; k++) {
        double a[3] = {P1[id[k]].x - c1.x, P1[id[k]].y - c1.y, P1[id[k]].z - c1.z};
        double b[3] = {P2[id[k]].x - c2.x, P2[id[k]].y - c2.y, P2[id[k]].z - c2.z};
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) H[r * 3 + c] += a[r] * b[c];
    }
    kabsch_dev(H, R);
    t[0] = c2.x - (R[0] * c1.x + R[1] * c1.y + R[2] * c1.z);
    t[1] = c2.y - (R[3] * c1.x + R[4] * c1.y + R[5] * c1.z);
    t[2] = c2.z - (R[6] * c1.x + R[7] * c1.y + R[8] * c1.z);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
    uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
    return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// One MT19937 twist of `mt` (in LDS) in three dependency phases, then tempered outputs.
__device__ void mt_twist_block(uint32_t* mt, uint32_t* nw, uint32_t* out) {
    const int t = threadIdx.x;
    for (int i = t; i < 227; i += blockDim.x) nw[i] = mt_mix(mt[i], mt[i + 1], mt[i + 397]);
    __syncthreads();
    for (int i = 227 + t; i < 454; i += blockDim.x) nw[i] = mt_mix(mt[i], mt[i + 1], nw[i - 227]);
    __syncthreads();
    for (int i = 454 + t; i < kMtN; i += blockDim.x)
        nw[i] = mt_mix(mt[i], (i + 1 < kMtN) ? mt[i + 1] : nw[0], nw[i - 227]);
    __syncthreads();
    for (int i = t; i < kMtN; i += blockDim.x) {
        mt[i] = nw[i];
        out[i] = mt_temper(nw[i]);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_ransac3d(const int* __restrict__ pairs, const vs_keypoint* __restrict__ kps,
                                                  int cap, const vs_match* __restrict__ good,
                                                  const int* __restrict__ ngood, const float* __restrict__ depth,
                                                  int h, int w, double fx, double fy, double cx, double cy,
                                                  const uint32_t* __restrict__ seeds,
                                                  const uint32_t* __restrict__ mt_init, int iters, double thr,
                                                  double* __restrict__ R_out, double* __restrict__ t_out,
                                                  int* __restrict__ ok_out, int* __restrict__ diag_out, int G,
                                                  int* __restrict__ sync) {
    __shared__ D3 sP1[kMaxPts3d], sP2[kMaxPts3d];
    __shared__ uint32_t s_mt[kMtN], s_nw[kMtN], s_out[2 * kMtN];
    __shared__ int s_samp[kMaxIters3d * 3];
    __shared__ int s_wcnt[4], s_N;
    __shared__ int s_bc[4], s_bi[4];
    __shared__ uint16_t s_val[kDraws3d];                // draw c % N
    __shared__ uint16_t s_J[kLevels3d][kDraws3d + 2];  // attempt-end maps (pointer doubling)
    __shared__ int s_start[kMaxIters3d];
    __shared__ int s_navail;
    __shared__ double s_in[6][kMaxPts3d];  // inlier coordinates for the refit
    const int p = blockIdx.x / G, g = blockIdx.x % G;  // G workgroups per pair share its hypotheses
    const int rf = pairs[2 * p], cf = pairs[2 * p + 1];
    const int n = min(ngood[p], kMaxPts3d);
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const float* dep1 = depth + (size_t)rf * h * w;
    const float* dep2 = depth + (size_t)cf * h * w;

    R3_T0();
    // ---- back-projection + order-preserving compaction (two 256-row chunks) ----
    if (tid == 0) s_N = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += 256) {
        const int i = c0 + tid;
        bool valid = false;
        D3 a = {0, 0, 0}, b = {0, 0, 0};
        if (i < n) {
            const vs_match m = good[(size_t)p * cap + i];
            const vs_keypoint k1 = kps[(size_t)rf * cap + m.query_idx];
            const vs_keypoint k2 = kps[(size_t)cf * cap + m.train_idx];
            const int px1 = (int)roundf(k1.x), py1 = (int)roundf(k1.y);
            const int px2 = (int)roundf(k2.x), py2 = (int)roundf(k2.y);
            if (px1 >= 0 && px1 < w && py1 >= 0 && py1 < h && px2 >= 0 && px2 < w && py2 >= 0 && py2 < h) {
                const float d1 = dep1[(size_t)py1 * w + px1], d2 = dep2[(size_t)py2 * w + px2];
                if (!(d1 <= 0.1f || d1 > 10.0f) && !(d2 <= 0.1f || d2 > 10.0f)) {
                    valid = true;
                    a = {((double)k1.x - cx) * d1 / fx, ((double)k1.y - cy) * d1 / fy, (double)d1};
                    b = {((double)k2.x - cx) * d2 / fx, ((double)k2.y - cy) * d2 / fy, (double)d2};
                }
            }
        }
        const unsigned long long bal = __ballot(valid);
        if (lane == 0) s_wcnt[wv] = __popcll(bal);
        __syncthreads();
        int off = s_N;
        for (int k = 0; k < wv; k++) off += s_wcnt[k];
        if (valid) {
            const int pos = off + __popcll(bal & ((1ull << lane) - 1ull));
            sP1[pos] = a;
            sP2[pos] = b;
        }
        __syncthreads();
        if (tid == 0) s_N += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
        __syncthreads();
    }
    const int N = s_N;
    if (N < 10) {  // every workgroup of the pair sees the same N
        if (tid == 0 && g == 0) {
            ok_out[p] = 0;
            diag_out[4 * p + 0] = N;
            diag_out[4 * p + 1] = 0;
            diag_out[4 * p + 2] = -1;
            diag_out[4 * p + 3] = 0;
        }
        return;
    }

    R3_T(0);
    // ---- MT19937(seed): init_genrand (given by the caller, or on lane 0), two parallel twists =
    // 1248 outputs ----
    if (mt_init) {
        for (int i = tid; i < kMtN; i += blockDim.x) s_mt[i] = mt_init[(size_t)p * kMtN + i];
    } else if (tid == 0) {
        uint32_t x = seeds[p];
        s_mt[0] = x;
        for (int i = 1; i < kMtN; i++) {
            x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            s_mt[i] = x;
        }
    }
    __syncthreads();
    R3_T(1);
    mt_twist_block(s_mt, s_nw, s_out);
    mt_twist_block(s_mt, s_nw, s_out + kMtN);
    R3_T(2);
    // The reference's sampling loop (i0; i1 != i0; i2 != i0, i1 by redrawing) for every iteration
    // at once: J0[c] = one past the draws an iteration starting at draw c consumes, attempt it
    // starts at J0^it(0) (pointer doubling), then each iteration assembles its triple.  Beyond the
    // 1248 draws of the two twists (never for N >= 10 and 1024 iterations in practice) lane 0
    // continues the stream serially, twisting on its own.
    for (int c = tid; c < kDraws3d; c += blockDim.x) s_val[c] = (uint16_t)(s_out[c] % (uint32_t)N);
    if (tid == 0) s_navail = iters;
    __syncthreads();
    for (int c = tid; c < kDraws3d + 2; c += blockDim.x) {
        int e = kDraws3d + 1;
        if (c < kDraws3d) {
            const int a = s_val[c];
            int q = c + 1;
            while (q < kDraws3d && s_val[q] == a) q++;
            if (q < kDraws3d) {
                const int b = s_val[q++];
                while (q < kDraws3d && (s_val[q] == a || s_val[q] == b)) q++;
                if (q < kDraws3d) e = q + 1;
            }
        }
        s_J[0][c] = (uint16_t)e;
    }
    __syncthreads();
    int L = 0;
    while ((1 << L) < iters) L++;
    for (int k = 1; k < L; k++) {
        for (int c = tid; c < kDraws3d + 2; c += blockDim.x) s_J[k][c] = s_J[k - 1][s_J[k - 1][c]];
        __syncthreads();
    }
    for (int it = tid; it < iters; it += blockDim.x) {
        int c = 0;
        for (int k = 0; k < L; k++)
            if ((it >> k) & 1) c = s_J[k][c];
        const bool avail = c < kDraws3d && s_J[0][c] <= kDraws3d;
        s_start[it] = avail ? c : -1;
        if (!avail) atomicMin(&s_navail, it);
    }
    __syncthreads();
    const int navail = s_navail;
    for (int it = tid; it < navail; it += blockDim.x) {
        int c = s_start[it];
        const int i0 = s_val[c++];
        while (s_val[c] == i0) c++;
        const int i1 = s_val[c++];
        while (s_val[c] == i0 || s_val[c] == i1) c++;
        s_samp[3 * it + 0] = i0;
        s_samp[3 * it + 1] = i1;
        s_samp[3 * it + 2] = s_val[c];
    }
    if (tid == 0 && navail < iters) {
        int c = navail > 0 ? s_J[0][s_start[navail - 1]] : 0;
        auto draw = [&]() -> uint32_t {
            if (c < kDraws3d) return s_out[c++];
            int k = (c - kDraws3d) % kMtN;
            if (k == 0) {
                for (int i = 0; i < kMtN; i++)
                    s_nw[i] = mt_mix(s_mt[i], (i + 1 < kMtN) ? s_mt[i + 1] : s_nw[0],
                                     (i < 227) ? s_mt[i + 397] : s_nw[i - 227]);
                for (int i = 0; i < kMtN; i++) s_mt[i] = s_nw[i];
            }
            c++;
            return mt_temper(s_mt[k]);
        };
        for (int it = navail; it < iters; it++) {
            int i0 = (int)(draw() % (uint32_t)N);
            int i1, i2;
            do { i1 = (int)(draw() % (uint32_t)N); } while (i1 == i0);
            do { i2 = (int)(draw() % (uint32_t)N); } while (i2 == i0 || i2 == i1);
            s_samp[3 * it + 0] = i0;
            s_samp[3 * it + 1] = i1;
            s_samp[3 * it + 2] = i2;
        }
    }
    __syncthreads();
    R3_T(3);

    // ---- hypotheses: workgroup g takes iterations g, g + G, ...; Lh lanes per hypothesis split the
    // points (Lh = the largest power of two that keeps all of them on the 256 lanes at once) and sum
    // their counts; keep the first best per lane, then the first best overall ----
    const int hn = (iters - g + G - 1) / G;
    int Lh = 1;
    while (Lh < 64 && 2 * Lh * hn <= 256) Lh <<= 1;
    const int part = tid & (Lh - 1);
    int my_best = 0, my_it = INT_MAX;
    for (int k = tid / Lh; k < hn; k += 256 / Lh) {
        const int it = g + G * k;
        double R[9], t[3];
        hypothesis_dev(sP1, sP2, s_samp[3 * it], s_samp[3 * it + 1], s_samp[3 * it + 2], R, t);
        int inl = 0;
#pragma unroll 4
        for (int j = part; j < N; j += Lh) inl += inlier_dev(R, t, sP1[j], sP2[j], thr);  // unrolled: loads run ahead
        for (int o = 1; o < Lh; o <<= 1) inl += __shfl_xor(inl, o);  // the Lh lanes of this hypothesis (all active)
        if (inl > my_best) {
            my_best = inl;
            my_it = it;
        }
    }
    // first strictly-best iteration overall = max count, then min iteration (a total order, so the
    // butterfly / wave-order / workgroup-order reduction is exact)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int oc = __shfl_xor(my_best, o), oi = __shfl_xor(my_it, o);
        if (oc > my_best || (oc == my_best && oi < my_it)) {
            my_best = oc;
            my_it = oi;
        }
    }
    if (lane == 0) {
        s_bc[wv] = my_best;
        s_bi[wv] = my_it;
    }
    __syncthreads();
    R3_T(4);
    int bc = s_bc[0], bi = s_bi[0];
    for (int k = 1; k < 4; k++)
        if (s_bc[k] > bc || (s_bc[k] == bc && s_bi[k] < bi)) {
            bc = s_bc[k];
            bi = s_bi[k];
        }
    if (G > 1) {
        // the pair's last workgroup to finish takes the G results (agent-scope release/acquire on the
        // arrival counter) and continues with the winner; it re-arms the counter for the next launch
        int* sy = sync + (size_t)p * (1 + 2 * G);
        __shared__ int s_last;
        if (tid == 0) {
            __hip_atomic_store(&sy[1 + 2 * g], bc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&sy[2 + 2 * g], bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int old = __hip_atomic_fetch_add(&sy[0], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == G - 1;
            if (s_last) __hip_atomic_store(&sy[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!s_last) return;
        bc = 0;
        bi = INT_MAX;
        for (int q = 0; q < G; q++) {
            const int c = __hip_atomic_load(&sy[1 + 2 * q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int i = __hip_atomic_load(&sy[2 + 2 * q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c > bc || (c == bc && i < bi)) {
                bc = c;
                bi = i;
            }
        }
    }
    if (bc == 0) bi = -1;
    const int best_inliers = bc, best_it = bi;
    // inlier flags of the winning hypothesis, in parallel (every lane re-derives the model), then
    // the inlier list in index order
    if (best_inliers >= 10) {
        double bR[9], bt[3];
        hypothesis_dev(sP1, sP2, s_samp[3 * best_it], s_samp[3 * best_it + 1], s_samp[3 * best_it + 2], bR, bt);
        if (tid == 0) s_N = 0;
        __syncthreads();
        for (int c0 = 0; c0 < N; c0 += 256) {
            const int j = c0 + tid;
            const bool in = j < N && inlier_dev(bR, bt, sP1[j], sP2[j], thr);
            const unsigned long long bal = __ballot(in);
            if (lane == 0) s_wcnt[wv] = __popcll(bal);
            __syncthreads();
            int off = s_N;
            for (int k = 0; k < wv; k++) off += s_wcnt[k];
            if (in) {  // the inliers' coordinates, compacted in index order (coordinate-major)
                const int q = off + __popcll(bal & ((1ull << lane) - 1ull));
                s_in[0][q] = sP1[j].x;
                s_in[1][q] = sP1[j].y;
                s_in[2][q] = sP1[j].z;
                s_in[3][q] = sP2[j].x;
                s_in[4][q] = sP2[j].y;
                s_in[5][q] = sP2[j].z;
            }
            __syncthreads();
            if (tid == 0) s_N += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
            __syncthreads();
        }
    }
    R3_T(5);
    if (wv != 0) return;
    if (tid == 0) {
        diag_out[4 * p + 0] = N;
        diag_out[4 * p + 1] = best_inliers;
        diag_out[4 * p + 2] = best_inliers > 0 ? best_it : -1;
        diag_out[4 * p + 3] = 0;
        ok_out[p] = 0;
    }
    if (best_inliers < 10) return;
    // refit over all inliers (Slam.cpp:324-358): every sum is the reference's sequential chain over
    // the inliers in index order, one chain per lane (6 centroid coordinates, then 9 entries of H)
    const int cnt = s_N;
    double sum = 0;
    if (tid < 6) {  // c1.x, c1.y, c1.z, c2.x, c2.y, c2.z: each a sequential chain in index order
        const double* col = s_in[tid];
#pragma unroll 8
        for (int q = 0; q < cnt; q++) sum += col[q];
    }
    D3 c1, c2;
    c1.x = __shfl(sum, 0) / cnt; c1.y = __shfl(sum, 1) / cnt; c1.z = __shfl(sum, 2) / cnt;
    c2.x = __shfl(sum, 3) / cnt; c2.y = __shfl(sum, 4) / cnt; c2.z = __shfl(sum, 5) / cnt;
    double hs = 0;
    if (tid < 9) {  // H[r][c] = sum (p1_r - c1_r)(p2_c - c2_c), sequential in index order
        const int r = tid / 3, c = tid % 3;
        const double m1 = r == 0 ? c1.x : r == 1 ? c1.y : c1.z;
        const double m2 = c == 0 ? c2.x : c == 1 ? c2.y : c2.z;
        const double* ca = s_in[r];
        const double* cb = s_in[3 + c];
#pragma unroll 8
        for (int q = 0; q < cnt; q++) hs += (ca[q] - m1) * (cb[q] - m2);
    }
    double H[9];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = __shfl(hs, k);
    if (tid != 0) return;
    diag_out[4 * p + 3] = cnt;
    double R[9];
    kabsch_dev(H, R);
    double t[3];
    t[0] = c2.x - (R[0] * c1.x + R[1] * c1.y + R[2] * c1.z);
    t[1] = c2.y - (R[3] * c1.x + R[4] * c1.y + R[5] * c1.z);
    t[2] = c2.z - (R[6] * c1.x + R[7] * c1.y + R[8] * c1.z);
    for (int k = 0; k < 9; k++) R_out[9 * p + k] = R[k];
    for (int k = 0; k < 3; k++) t_out[3 * p + k] = t[k];
    double tn = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    int ok = 1;
    if (tn > 0.2) ok = 0;  // RANSAC_3D3D_MAX_TRANSLATION (Config.h:67)
    if (tn < 0.0001) ok = 0;
    if (fabs(det3_dev(R) - 1.0) > 0.01) ok = 0;
    ok_out[p] = ok;
    R3_T(6);
}

int ransac3d_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_good,
                   const int* d_ngood, const float* d_depth, int h, int w, const double K[4],
                   const uint32_t* d_seeds, int iters, double thr, double* d_R, double* d_t, int* d_ok, int* d_diag,
                   hipStream_t s, const uint32_t* d_mt_init, int split, int* d_sync) {
    if (P <= 0) return VS_OK;
    VS_ARG(iters > 0 && iters <= kMaxIters3d, "ransac_3d3d: iters must be in [1, 1024]");
    VS_ARG(split >= 1 && split <= kMaxSplit3d && (split == 1 || d_sync), "ransac_3d3d: bad workgroup split");
    ProfScope ps(ctx, "ransac3d", s);
    hipLaunchKernelGGL(k_ransac3d, dim3(P * split), dim3(256), 0, s, d_pairs, d_kps, cap, d_good, d_ngood, d_depth, h,
                       w, K[0], K[1], K[2], K[3], d_seeds, d_mt_init, iters, thr, d_R, d_t, d_ok, d_diag, split,
                       d_sync);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

}  // namespace vs

#ifdef VS_R3_PROFILE
extern "C" int vs_debug_r3_cycles(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vs::g_r3_cycles), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vs::g_r3_cycles), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
