// sp_post.hip — SuperPoint post-processing on gfx950: heatmap decode, greedy NMS, descriptor
// sampling (reference src/FeatureExtractor.cpp:126-206 and nms() :219-259).
//
// Compiled with -ffp-contract=off: every float expression keeps the reference's evaluation order
// and IEEE rounding (division and sqrt correctly rounded), so the keypoints (pixel indices and
// scores) and the sampled descriptors are bit-identical to the CPU restatement given the same
// semi / desc tensors.
//
// NMS.  The reference sorts the candidates (score > 0.005) by score and greedily keeps a
// candidate unless a kept one lies in its 9x9 window, stopping at 400.  Here the greedy set is
// computed as a priority maximal independent set in parallel rounds over the dense heatmap: an
// undecided pixel becomes kept when every higher-priority pixel of its window is already out,
// and out when a kept pixel lies in its window.  States only move forward, so stale halo reads
// are safe and the fixed point is exactly the sequential greedy set for the total order
// (score desc, raster index asc).  The 400-cap then takes the 400 highest-priority kept pixels:
// greedy decisions never depend on lower-priority candidates, so the capped greedy output is the
// top 400 of the uncapped set.
//
// Score floor (round 3).  A strict local maximum (every other candidate of its window scores
// lower) is kept by the greedy whatever else happens.  So when a frame has at least 400 of them,
// the 400th kept pixel scores at least the 400th-largest strict-local-maximum score F, and no
// pixel scoring below F can be output or influence a pixel that can: those pixels start out
// decided (out).  k_nms_lmax histograms the strict local maxima's scores (2^-7-octave bins) and
// k_nms_floor takes the lower edge of the bin holding the 400th largest — a lower bound of F, so
// the argument holds and at most one bin's width more pixels stay undecided.  On
// a camera frame (and on random-weight heatmaps, where nearly every pixel is a candidate) this
// leaves a few hundred to a few thousand undecided pixels per frame, so the rounds converge in one
// or two iterations and only tiles with undecided pixels run at all.
//
// Round budget: a fixed number of tile rounds (kNmsRounds launches; each iterates its tile to a
// local fixed point) settles typical heatmaps; whatever is still undecided afterwards (a dependency
// chain crossing many tile borders) is finished by k_nms_finish, one workgroup per frame running
// the same priority-MIS rule over a compact list of the remaining pixels until none is left.  The
// result is the greedy set for every input; a frame that reaches k_nms_finish's round cap (only an
// adversarial dependency chain thousands of pixels long can) is reported (count = VS_ERR_NOTCONV
// on the device paths, VS_ERR_NOTCONV from the host entry points), never a wrong keypoint list.
//
// Ties.  The reference sorts with std::sort (unstable); the order used here breaks exact score
// ties by raster index.  The keypoint SET can differ from the reference's only through an exact tie
// that the greedy actually resolves: two candidates of equal score within one 9x9 window of which
// one is kept, or equal scores on both sides of the 400 cut; the keypoint LIST order additionally
// through output keypoints that share a score.  k_nms_select counts all three per frame (an output
// keypoint with an equal-score candidate in its window; the 400th and 401st kept pixel scoring the
// same; output keypoints sharing their score) into the context's tie totals (vs_nms_tie_stats):
// when all are zero the output list equals the reference's for ANY order of equal scores,
// std::sort's included (tests/test_oracle.py pins the claim on the CPU restatement).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "glibc_expf.h"
#include "vs_internal.h"

namespace vs {

constexpr float kConfThresh = 0.005f;  // SP_CONFIDENCE_THRESHOLD (Config.h:40)
constexpr int kRadius = 4;             // SP_NMS_RADIUS (Config.h:41)
constexpr int kMaxKeypoints = 400;     // SP_MAX_KEYPOINTS (Config.h:42)
constexpr int kNmsTile = 32;
constexpr int kNmsReg = kNmsTile + 2 * kRadius;
constexpr int kNmsMaxRounds = 2;          // tile-round launches before k_nms_finish (4: 3 % slower, 1: 55 %)
constexpr int kFinishMaxRounds = 1 << 14; // k_nms_finish's round cap (VS_NMS_FINISH_ROUNDS overrides)

enum : uint8_t { ST_UNDECIDED = 0, ST_KEPT = 1, ST_OUT = 2 };

// ---------------------------------------------------------------------------------------------
// A4 decode (inside k_nms_lmax): softmax of each 8x8 cell over its 65 channels, dustbin dropped.
// std::exp(float) is glibc's expf, which is not correctly rounded; glibc_expf.h restates its
// algorithm instruction for instruction (checked exhaustively against libm on the host by
// tests/test_oracle.py, and on the device through the decode parity tests of
// tests/test_gpu_parity.py).  The maximum and the sum run over the channels in order, as the
// reference's loops do.

// Workgroup -> (frame, tile), XCD-aware: the hardware deals consecutive workgroups to the eight
// XCDs in turn, so workgroup L runs on XCD L % 8; the mapping hands each XCD a contiguous run of
// tiles (a frame per XCD at 8 frames of 300 tiles), so the 4-px halo rows a tile shares with its
// neighbours are fetched into one L2 instead of one per XCD.
__device__ __forceinline__ void tile_of_block(int ntiles, int B, int& b, int& tile) {
    const int N = ntiles * B, L = blockIdx.y * gridDim.x + blockIdx.x;
    const int per = N / 8, rem = N % 8, xcd = L % 8, k = L / 8;
    const int logical = (xcd < rem ? xcd * (per + 1) : rem * (per + 1) + (xcd - rem) * per) + k;
    b = logical / ntiles;
    tile = logical - b * ntiles;
}

// 9-wide windows over a (32 + 8)^2 LDS region of 32-bit score keys: row pass (40 region rows x 32
// interior columns), then the column pass per interior pixel.  u32 score bits order like the
// scores (all candidates are > 0).
constexpr int kNmsThreads = 256;

// Strict local maxima of the candidate heatmap -> a per-frame histogram of their scores: bin =
// (score bits >> 16) - kFloorBin0, i.e. 2^-7-octave bins over [2^-11, 2) (every candidate scores
// in (0.005, 1]).  One workgroup per 32x32 tile; an LDS histogram per workgroup, flushed with one
// global atomic per touched bin (same-address atomics per local maximum would serialise in L2).
constexpr int kFloorBins = 2048;
constexpr unsigned kFloorBin0 = 0x3A00u;  // bits >> 16 of 2^-11
__device__ __forceinline__ int floor_bin(unsigned key) {
    const int bin = (int)(key >> 16) - (int)kFloorBin0;
    return bin < 0 ? 0 : bin >= kFloorBins ? kFloorBins - 1 : bin;
}

// The decode is fused in: the workgroup decodes the 6 x 6 cells under its 40 x 40 region straight
// from semi into LDS (the heatmap is never re-read from HBM here) and writes its 32 x 32 interior
// to the heatmap once, for the NMS rounds and the selection.
constexpr int kNmsCells = kNmsTile / 8 + 2;  // cells per side under a tile's region (4-px halo < a cell)
__global__ __launch_bounds__(kNmsThreads) void k_nms_lmax(const float* __restrict__ semi, int hc, int wc,
                                                          float* __restrict__ heat, int B, int Hp, int Wp,
                                                          int tiles_x, int ntiles, int* __restrict__ hist) {
    post_prio();
    int b, tile;
    tile_of_block(ntiles, B, b, tile);
    constexpr int kPw = kNmsCells * 8, kNc = kNmsCells * kNmsCells;
    constexpr int kWaves = kNmsThreads / 64, kCpw = kNc / kWaves;  // cells per wave
    static_assert(kNc % kWaves == 0 && kCpw <= 64, "k_nms_lmax: the region's cells split evenly over the waves");
    __shared__ float s_prob[kPw * kPw];  // the cells' probabilities, 48 x 48 px
    // the decode's exps, then (dead after the decode) the window passes' keys and row maxima
    constexpr int kExpWords = kWaves * kCpw * kSemiCh, kKeyWords = kNmsReg * kNmsReg + kNmsReg * kNmsTile;
    __shared__ unsigned s_u[kExpWords > kKeyWords ? kExpWords : kKeyWords];
    __shared__ float s_csum[kNc];
    __shared__ int s_hist[kFloorBins];
    __shared__ int s_any;
    unsigned* s_key = s_u;                        // [kNmsReg * kNmsReg]
    unsigned* s_rmax = s_u + kNmsReg * kNmsReg;   // [kNmsReg * kNmsTile]
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int gx0 = tx * kNmsTile - kRadius, gy0 = ty * kNmsTile - kRadius;
    const int cx0 = tx * (kNmsTile / 8) - 1, cy0 = ty * (kNmsTile / 8) - 1;  // the region's first cell
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_any = 0;
    for (int i = threadIdx.x; i < kFloorBins; i += kNmsThreads) s_hist[i] = 0;
    {
        // decode, kCpw cells per wave: lane c holds channel c of each cell (the dustbin channel 64 read
        // by every lane), the maxima by butterfly (the maximum's value does not depend on the order;
        // only the sign of a zero maximum could, and x - 0 and x - (-0) are equal for every x that
        // reaches expf), the exps to LDS, lanes 0 .. kCpw - 1 sum one cell's 65 exps each in channel
        // order, every lane divides its channel
        float v[kCpw], dust[kCpw], mx[kCpw];
        bool ok[kCpw];
#pragma unroll
        for (int j = 0; j < kCpw; j++) {
            const int q = wv * kCpw + j, ci = q / kNmsCells, cj = q - ci * kNmsCells;
            const int cy = cy0 + ci, cx = cx0 + cj;
            ok[j] = cy >= 0 && cy < hc && cx >= 0 && cx < wc;
            const float* p = semi + (((size_t)b * hc + (ok[j] ? cy : 0)) * wc + (ok[j] ? cx : 0)) * kSemiCh;
            v[j] = p[lane];
            dust[j] = p[64];
        }
#pragma unroll
        for (int j = 0; j < kCpw; j++) {
            float m = v[j] > dust[j] ? v[j] : dust[j];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float t = __shfl_xor(m, o);
                m = t > m ? t : m;
            }
            mx[j] = m;
        }
        float* ex = reinterpret_cast<float*>(s_u) + wv * kCpw * kSemiCh;
        float xd = 0.0f;  // lane j < kCpw: cell j's dustbin term
#pragma unroll
        for (int j = 0; j < kCpw; j++) {
            v[j] = vs_expf::glibc_expf(v[j] - mx[j]);
            ex[j * kSemiCh + lane] = v[j];
            if (lane == j) xd = dust[j] - mx[j];
        }
        if (lane < kCpw) ex[lane * kSemiCh + 64] = vs_expf::glibc_expf(xd);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < kCpw) {
            const float* e = ex + lane * kSemiCh;
            float sum = 0.0f;
            for (int c = 0; c < kSemiCh; c++) sum += e[c];
            s_csum[wv * kCpw + lane] = sum;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < kCpw; j++) {
            const int q = wv * kCpw + j, ci = q / kNmsCells, cj = q - ci * kNmsCells;
            if (ok[j]) s_prob[(ci * 8 + lane / 8) * kPw + cj * 8 + (lane % 8)] = div_rn(v[j], s_csum[q]);
        }
    }
    __syncthreads();  // s_prob complete; the exps are dead (s_u becomes the keys)
    float* hb = heat + (size_t)b * Hp * Wp;
    for (int i = threadIdx.x; i < kNmsReg * kNmsReg; i += kNmsThreads) {
        const int ry = i / kNmsReg, rx = i - ry * kNmsReg;
        const int gy = gy0 + ry, gx = gx0 + rx;
        unsigned key = 0;
        if (gy >= 0 && gy < Hp && gx >= 0 && gx < Wp) {
            const float v = s_prob[(ry + 8 - kRadius) * kPw + rx + 8 - kRadius];
            key = v > kConfThresh ? __float_as_uint(v) : 0u;
        }
        s_key[i] = key;
    }
    // the interior to the heatmap (rows of 32 floats, 16-byte stores)
    for (int i = threadIdx.x; i < kNmsTile * kNmsTile / 4; i += kNmsThreads) {
        const int iy = i / (kNmsTile / 4), ix = 4 * (i - iy * (kNmsTile / 4));
        const int gy = gy0 + kRadius + iy, gx = gx0 + kRadius + ix;  // Wp is a multiple of 8
        if (gy < Hp && gx < Wp) {
            const float* q = &s_prob[(iy + 8) * kPw + ix + 8];
            *reinterpret_cast<float4*>(hb + (size_t)gy * Wp + gx) = make_float4(q[0], q[1], q[2], q[3]);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kNmsReg * kNmsTile; i += kNmsThreads) {
        const int ry = i / kNmsTile, ix = i - ry * kNmsTile;
        const unsigned* r = s_key + ry * kNmsReg + ix;
        unsigned m = r[0];
#pragma unroll
        for (int d = 1; d <= 2 * kRadius; d++) m = max(m, r[d]);
        s_rmax[i] = m;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kNmsTile * kNmsTile / kNmsThreads; j++) {
        const int kk = threadIdx.x + kNmsThreads * j;
        const int iy = kk / kNmsTile, ix = kk - iy * kNmsTile;
        const unsigned key = s_key[(iy + kRadius) * kNmsReg + ix + kRadius];
        if (key != 0 && gy0 + kRadius + iy < Hp && gx0 + kRadius + ix < Wp) {
            unsigned m = 0;
#pragma unroll
            for (int d = 0; d <= 2 * kRadius; d++) m = max(m, s_rmax[(iy + d) * kNmsTile + ix]);
            if (m == key) {  // the window maximum: strict unless another window pixel scores the same
                int eq = 0;
                for (int dy = 0; dy <= 2 * kRadius; dy++)
                    for (int dx = 0; dx <= 2 * kRadius; dx++) eq += s_key[(iy + dy) * kNmsReg + ix + dx] == key;
                if (eq == 1) {
                    atomicAdd(&s_hist[floor_bin(key)], 1);
                    s_any = 1;
                }
            }
        }
    }
    __syncthreads();
    if (!s_any) return;
    int* hg = hist + (size_t)b * kFloorBins;
    for (int i = threadIdx.x; i < kFloorBins; i += kNmsThreads)
        if (s_hist[i]) atomicAdd(&hg[i], s_hist[i]);
}

// Per frame: F = the lower edge of the histogram bin that holds the max_kp-th largest strict-local-
// maximum score (a lower bound of that score, so at least max_kp strict local maxima score >= F),
// or 0 (no floor) with fewer.  One workgroup per frame: a suffix scan over the bins from the top.
__global__ __launch_bounds__(kNmsThreads) void k_nms_floor(const int* __restrict__ hist, int max_kp,
                                                           unsigned* __restrict__ floor_bits) {
    post_prio();
    constexpr int PER = kFloorBins / kNmsThreads;  // bins per thread (thread 0 owns the top bins)
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int* h = hist + (size_t)b * kFloorBins;
    int v[PER], tot = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {  // thread t owns bins hi(t) down to hi(t) - PER + 1, top first
        v[k] = h[kFloorBins - 1 - (t * PER + k)];
        tot += v[k];
    }
    int incl = tot;  // inclusive scan over threads in descending-bin order
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    __shared__ int s_w[kNmsThreads / 64];
    __shared__ unsigned s_floor;
    if (lane == 63) s_w[wv] = incl;
    if (t == 0) s_floor = 0u;
    __syncthreads();
    int before = incl - tot;
    for (int w = 0; w < wv; w++) before += s_w[w];
    // the thread whose range crosses max_kp names the bin
    if (before < max_kp && before + tot >= max_kp) {
        int run = before;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            if (run < max_kp && run + v[k] >= max_kp)
                s_floor = (unsigned)(kFloorBins - 1 - (t * PER + k) + (int)kFloorBin0) << 16;
            run += v[k];
        }
    }
    __syncthreads();
    if (t == 0) floor_bits[b] = s_floor;
}

// One NMS round over a 32x32 tile (+4 halo).  The tile iterates to its local fixed point, writes
// its interior states back and flags itself (and its frame) if anything is still undecided.
// tflags[r][b][tile] != 0  <=>  the tile's interior still had undecided pixels after round r-1
// (round 0: every tile); flags[r*B + b] != 0  <=>  some tile of frame b did.  Round 0 derives the
// initial states from the heatmap and the frame's floor (undecided iff score > 0.005 and >= F).
// Each local iteration evaluates, for every interior pixel, M = the 9x9 window max of the
// undecided pixels' score bits (0 when not undecided) and K = the 9x9 window OR of the kept
// flags, both separable in LDS.  An undecided pixel with K set is out; one whose own score is
// below M is blocked; one whose score equals M is kept unless an equal-score undecided pixel
// precedes it in raster order inside its window (the total order's tie break).
__device__ __forceinline__ unsigned long long nms_key(float s, unsigned raster) {
    return ((unsigned long long)__float_as_uint(s) << 32) | (unsigned)(0xFFFFFFFFu - raster);
}

__global__ __launch_bounds__(kNmsThreads) void k_nms_round(const float* __restrict__ heat, uint8_t* __restrict__ state,
                                                           int* __restrict__ flags, uint8_t* __restrict__ tflags,
                                                           const unsigned* __restrict__ floor_bits, int r, int B,
                                                           int Hp, int Wp, int tiles_x, int ntiles) {
    post_prio();
    int b, tile;
    tile_of_block(ntiles, B, b, tile);
    if (flags[r * B + b] == 0) return;
    if (r > 0 && tflags[((size_t)r * B + b) * ntiles + tile] == 0) return;
    __shared__ unsigned s_key[kNmsReg * kNmsReg];
    __shared__ unsigned s_rmax[kNmsReg * kNmsTile];
    __shared__ uint8_t s_kept[kNmsReg * kNmsReg];
    __shared__ uint8_t s_rkept[kNmsReg * kNmsTile];
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int gx0 = tx * kNmsTile - kRadius, gy0 = ty * kNmsTile - kRadius;
    const float* hb = heat + (size_t)b * Hp * Wp;
    uint8_t* sb = state + (size_t)b * Hp * Wp;
    const unsigned fl = floor_bits[b];
    int any = 0;
    for (int i = threadIdx.x; i < kNmsReg * kNmsReg; i += kNmsThreads) {
        const int ry = i / kNmsReg, rx = i - ry * kNmsReg;
        const int gy = gy0 + ry, gx = gx0 + rx;
        unsigned key = 0;
        uint8_t kept = 0;
        if (gy >= 0 && gy < Hp && gx >= 0 && gx < Wp) {
            const float v = hb[(size_t)gy * Wp + gx];
            uint8_t st;
            if (r == 0)  // halo pixels of other tiles: their round-0 state, derived the same way
                st = (v > kConfThresh && __float_as_uint(v) >= fl) ? ST_UNDECIDED : ST_OUT;
            else
                st = sb[(size_t)gy * Wp + gx];
            if (st == ST_UNDECIDED) key = __float_as_uint(v);
            kept = (st == ST_KEPT);
        }
        s_key[i] = key;
        s_kept[i] = kept;
        any |= key != 0 && ry >= kRadius && ry < kRadius + kNmsTile && rx >= kRadius && rx < kRadius + kNmsTile;
    }
    if (__syncthreads_or(any)) {
        int changed;
        do {
            for (int i = threadIdx.x; i < kNmsReg * kNmsTile; i += kNmsThreads) {
                const int ry = i / kNmsTile, ix = i - ry * kNmsTile;
                const int base = ry * kNmsReg + ix;
                unsigned m = s_key[base];
                uint8_t k = s_kept[base];
#pragma unroll
                for (int d = 1; d <= 2 * kRadius; d++) {
                    m = max(m, s_key[base + d]);
                    k |= s_kept[base + d];
                }
                s_rmax[i] = m;
                s_rkept[i] = k;
            }
            __syncthreads();
            uint8_t dec[kNmsTile * kNmsTile / kNmsThreads];
            int ch = 0;
#pragma unroll
            for (int j = 0; j < kNmsTile * kNmsTile / kNmsThreads; j++) {
                const int kk = threadIdx.x + kNmsThreads * j;
                const int iy = kk / kNmsTile, ix = kk - iy * kNmsTile;
                const unsigned key = s_key[(iy + kRadius) * kNmsReg + ix + kRadius];
                dec[j] = 0;
                if (key == 0) continue;
                unsigned m = 0;
                uint8_t k = 0;
#pragma unroll
                for (int d = 0; d <= 2 * kRadius; d++) {
                    m = max(m, s_rmax[(iy + d) * kNmsTile + ix]);
                    k |= s_rkept[(iy + d) * kNmsTile + ix];
                }
                if (k) {
                    dec[j] = ST_OUT;
                } else if (m == key) {
                    // equal-score undecided pixels earlier in raster order (rows above, then left)
                    bool first = true;
                    for (int d = 0; d < kRadius * (2 * kRadius + 1) + kRadius && first; d++) {
                        const int dy = d / (2 * kRadius + 1), dx = d - dy * (2 * kRadius + 1);
                        first = s_key[(iy + dy) * kNmsReg + ix + dx] != key;
                    }
                    if (first) dec[j] = ST_KEPT;
                }
                ch |= dec[j] != 0;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kNmsTile * kNmsTile / kNmsThreads; j++) {
                if (!dec[j]) continue;
                const int kk = threadIdx.x + kNmsThreads * j;
                const int iy = kk / kNmsTile, ix = kk - iy * kNmsTile;
                const int p = (iy + kRadius) * kNmsReg + ix + kRadius;
                s_key[p] = 0;
                if (dec[j] == ST_KEPT) s_kept[p] = 1;
            }
            changed = __syncthreads_or(ch);
        } while (changed);
    } else if (r > 0) {
        return;  // nothing undecided inside any more: nothing to write
    }
    int und = 0;
#pragma unroll
    for (int j = 0; j < kNmsTile * kNmsTile / kNmsThreads; j++) {
        const int kk = threadIdx.x + kNmsThreads * j;
        const int iy = kk / kNmsTile, ix = kk - iy * kNmsTile;
        const int gy = gy0 + kRadius + iy, gx = gx0 + kRadius + ix;
        if (gy < Hp && gx < Wp) {
            const int p = (iy + kRadius) * kNmsReg + ix + kRadius;
            const uint8_t v = s_kept[p] ? ST_KEPT : (s_key[p] ? ST_UNDECIDED : ST_OUT);
            sb[(size_t)gy * Wp + gx] = v;
            und |= (v == ST_UNDECIDED);
        }
    }
    // only a tile with undecided interior pixels has anything to do next round (its neighbours'
    // decisions reach it through the halo it reloads)
    if (__syncthreads_or(und) && threadIdx.x == 0) {
        tflags[((size_t)(r + 1) * B + b) * ntiles + tile] = 1;
        flags[(r + 1) * B + b] = 1;
    }
}

// Finishes the NMS of frames the tile rounds left undecided (flags[R * B + b] != 0), one workgroup
// per frame: the frame's undecided pixels are listed once, then each round walks the list, decides
// what it can with the tile rounds' rule (out if a kept pixel is in the window, kept if no
// undecided window pixel outranks it), stores the decision at once and compacts the rest into the
// other list ([B][2][npx] scratch).  Deciding in place is safe for the same reason stale halo reads
// are: states only move forward and a decided state is final.  Every round decides at least the
// highest-priority undecided pixel, so the loop ends; max_rounds bounds adversarial dependency
// chains, ferr[b] = 1 reports hitting it.
__global__ __launch_bounds__(1024) void k_nms_finish(const float* __restrict__ heat, uint8_t* __restrict__ state,
                                                     const int* __restrict__ flags, int R, int B, int Hp, int Wp,
                                                     int* __restrict__ lists, int max_rounds, int* __restrict__ ferr) {
    post_prio();
    const int b = blockIdx.x;
    if (flags[R * B + b] == 0) return;
    __shared__ int s_n[2];
    const int npx = Hp * Wp;
    const float* hb = heat + (size_t)b * npx;
    uint8_t* sb = state + (size_t)b * npx;
    int* lst[2] = {lists + (size_t)b * 2 * npx, lists + (size_t)b * 2 * npx + npx};
    if (threadIdx.x == 0) s_n[0] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < npx; i += blockDim.x)
        if (sb[i] == ST_UNDECIDED) lst[0][atomicAdd(&s_n[0], 1)] = i;
    __syncthreads();
    int cur = 0;
    for (int round = 0; round < max_rounds; round++) {
        const int n = s_n[cur];
        if (n == 0) return;
        if (threadIdx.x == 0) s_n[cur ^ 1] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int p = lst[cur][i], py = p / Wp, px = p - py * Wp;
            const unsigned long long key = nms_key(hb[p], (unsigned)p);
            bool kept_near = false, blocked = false;
            for (int dy = -kRadius; dy <= kRadius && !kept_near; dy++) {
                const int y = py + dy;
                if (y < 0 || y >= Hp) continue;
                for (int dx = -kRadius; dx <= kRadius; dx++) {
                    const int x = px + dx;
                    if (x < 0 || x >= Wp || (dx == 0 && dy == 0)) continue;
                    const int q = y * Wp + x;
                    const uint8_t st = sb[q];
                    if (st == ST_KEPT) {
                        kept_near = true;
                        break;
                    }
                    if (st == ST_UNDECIDED && nms_key(hb[q], (unsigned)q) > key) blocked = true;
                }
            }
            if (kept_near) sb[p] = ST_OUT;
            else if (!blocked) sb[p] = ST_KEPT;
            else lst[cur ^ 1][atomicAdd(&s_n[cur ^ 1], 1)] = p;
        }
        __syncthreads();
        cur ^= 1;
    }
    if (threadIdx.x == 0 && s_n[cur] != 0) ferr[b] = 1;
}

// Kept pixels -> 64-bit priority keys (score bits << 32 | ~raster index), unordered.  Each thread
// reads four state bytes at once; one atomic per wave reserves the wave's slots.
__global__ __launch_bounds__(256) void k_nms_collect(const float* __restrict__ heat, const uint8_t* __restrict__ state,
                                                     int Hp, int Wp, unsigned long long* __restrict__ keys,
                                                     int* __restrict__ keycnt, int key_cap) {
    post_prio();
    const int b = blockIdx.y;
    const int npx = Hp * Wp, nq = npx / 4;  // Wp is a multiple of 8
    const int lane = threadIdx.x & 63;
    const uchar4* st = reinterpret_cast<const uchar4*>(state + (size_t)b * npx);
    for (int q0 = blockIdx.x * 256; q0 < nq; q0 += gridDim.x * 256) {  // (uniform trip count per wave)
        const int q = q0 + threadIdx.x;
        uchar4 v = make_uchar4(0, 0, 0, 0);
        if (q < nq) v = st[q];
        const int f[4] = {v.x == ST_KEPT, v.y == ST_KEPT, v.z == ST_KEPT, v.w == ST_KEPT};
        const int cnt = f[0] + f[1] + f[2] + f[3];
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const int tot = __shfl(incl, 63);
        if (tot == 0) continue;
        int base = 0;
        if (lane == 63) base = atomicAdd(&keycnt[b], tot);
        base = __shfl(base, 63) + incl - cnt;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (f[k]) {
                const int i = 4 * q + k;
                const unsigned long long key = ((unsigned long long)__float_as_uint(heat[(size_t)b * npx + i]) << 32) |
                                               (unsigned)(0xFFFFFFFFu - (unsigned)i);
                if (base < key_cap) keys[(size_t)b * key_cap + base] = key;
                base++;
            }
    }
}

// Top-K of the kept keys (exact MSB-first radix select over the 64-bit keys, which are unique),
// bitonic sort of the K winners in descending priority, keypoint records, border erase
// (FeatureExtractor.cpp:155-160), and the frame's tie accounting (see the header): window ties =
// selected pixels with an equal-score candidate in their 9x9 window, cut tie = the K-th and the
// (K+1)-th kept pixel score the same, order ties = selected keypoints sharing their score with
// another selected one.  ties[b] = {window, cut, order}; totals += {frames, frames with a tie,
// window ties, cut ties, order ties}.  One 1024-thread workgroup per frame.
constexpr int kSelSort = 512;
__global__ __launch_bounds__(1024) void k_nms_select(const unsigned long long* __restrict__ keys,
                                                     const int* __restrict__ keycnt, int key_cap, int max_kp,
                                                     int Wp, int Hp, int h, int w, vs_keypoint* __restrict__ kps,
                                                     int cap, int* __restrict__ nout, int* __restrict__ err,
                                                     const int* __restrict__ ferr, const float* __restrict__ heat,
                                                     int* __restrict__ ties, unsigned long long* __restrict__ totals) {
    post_prio();
    const int b = blockIdx.x;
    if (ferr[b]) {  // NMS not finished: no keypoints, a negative count that every consumer rejects
        if (threadIdx.x == 0) nout[b] = VS_ERR_NOTCONV;
        return;
    }
    __shared__ int hist[256];
    __shared__ unsigned long long s_sel[kSelSort];
    __shared__ int s_nsel;
    __shared__ int s_wk[16], s_ww[16], s_wo[16];
    __shared__ unsigned long long s_prefix, s_mask, s_next;
    __shared__ int s_krem;
    int nk = keycnt[b];
    if (nk > key_cap) {
        if (threadIdx.x == 0) atomicOr(err, 1);
        nk = key_cap;
    }
    const unsigned long long* kb = keys + (size_t)b * key_cap;
    const int K = nk < max_kp ? nk : max_kp;
    unsigned long long kth = 0;
    if (K > 0 && K < nk) {
        if (threadIdx.x == 0) {
            s_prefix = 0;
            s_mask = 0;
            s_krem = K;
        }
        for (int pass = 0; pass < 8; pass++) {
            const int shift = 56 - 8 * pass;
            if (threadIdx.x < 256) hist[threadIdx.x] = 0;
            __syncthreads();
            const unsigned long long pre = s_prefix, msk = s_mask;
            for (int i = threadIdx.x; i < nk; i += blockDim.x) {
                unsigned long long k = kb[i];
                if ((k & msk) == pre) atomicAdd(&hist[(k >> shift) & 255], 1);
            }
            __syncthreads();
            if (threadIdx.x < 64) {  // the digit holding the rem-th largest: a suffix scan on wave 0
                const int lane = threadIdx.x, rem = s_krem;
                int c[4], sum = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {  // lane l owns digits 255 - 4l .. 252 - 4l, top first
                    c[k] = hist[255 - 4 * lane - k];
                    sum += c[k];
                }
                int incl = sum;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int y = __shfl_up(incl, o);
                    if (lane >= o) incl += y;
                }
                int acc = incl - sum;
                if (acc < rem && acc + sum >= rem) {
                    int d = 255 - 4 * lane;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (acc + c[k] >= rem) break;
                        acc += c[k];
                        d--;
                    }
                    s_krem = rem - acc;
                    s_prefix = pre | ((unsigned long long)d << shift);
                    s_mask = msk | (255ull << shift);
                }
            }
            __syncthreads();
        }
        kth = s_prefix;  // the K-th largest key
    }
    if (threadIdx.x == 0) {
        s_nsel = 0;
        s_next = 0;
    }
    for (int i = threadIdx.x; i < kSelSort; i += blockDim.x) s_sel[i] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < nk; i += blockDim.x) {
        unsigned long long k = kb[i];
        if (K > 0 && k >= kth) {
            int slot = atomicAdd(&s_nsel, 1);
            if (slot < kSelSort) s_sel[slot] = k;
        } else if (K > 0) {
            atomicMax(&s_next, k);  // the (K+1)-th kept key
        }
    }
    __syncthreads();
    // bitonic sort, descending (zero keys pad the tail)
    for (int size = 2; size <= kSelSort; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = threadIdx.x; i < kSelSort; i += blockDim.x) {
                int j = i ^ stride;
                if (j > i) {
                    bool desc = ((i & size) == 0);
                    unsigned long long a = s_sel[i], c = s_sel[j];
                    if (desc ? (a < c) : (a > c)) {
                        s_sel[i] = c;
                        s_sel[j] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    // keypoint records in priority order with the border erase, one selected pixel per thread
    // (order-preserving ballot compaction), and the frame's window / order ties
    const int i = threadIdx.x, lane = i & 63, wv = i >> 6;
    bool keep = false, wtie = false, otie = false;
    vs_keypoint kp;
    if (i < K && i < kSelSort) {
        const unsigned long long k = s_sel[i];
        const unsigned idx = 0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull);
        const int px = (int)(idx % (unsigned)Wp), py = (int)(idx / (unsigned)Wp);
        const unsigned sc = (unsigned)(k >> 32);
        keep = !(px >= w || py >= h);
        kp.x = (float)px;
        kp.y = (float)py;
        kp.size = 8.0f;
        kp.angle = -1.0f;
        kp.response = __uint_as_float(sc);
        kp.octave = 0;
        kp.class_id = -1;
        otie = (i > 0 && (unsigned)(s_sel[i - 1] >> 32) == sc) || (i + 1 < K && (unsigned)(s_sel[i + 1] >> 32) == sc);
        const float* hb = heat + (size_t)b * Hp * Wp;
        for (int dy = -kRadius; dy <= kRadius; dy++) {
            const int y = py + dy;
            if (y < 0 || y >= Hp) continue;
            for (int dx = -kRadius; dx <= kRadius; dx++) {
                const int x = px + dx;
                if (x < 0 || x >= Wp || (dx == 0 && dy == 0)) continue;
                wtie |= __float_as_uint(hb[(size_t)y * Wp + x]) == sc;
            }
        }
    }
    const unsigned long long bk = __ballot(keep), bw = __ballot(wtie), bo = __ballot(otie);
    if (lane == 0) {
        s_wk[wv] = __popcll(bk);
        s_ww[wv] = __popcll(bw);
        s_wo[wv] = __popcll(bo);
    }
    __syncthreads();
    if (keep) {
        int off = __popcll(bk & ((1ull << lane) - 1ull));
        for (int k2 = 0; k2 < wv; k2++) off += s_wk[k2];
        kps[(size_t)b * cap + off] = kp;
    }
    if (threadIdx.x == 0) {
        int n = 0, wt = 0, ot = 0;
        for (int k2 = 0; k2 < 16; k2++) {
            n += s_wk[k2];
            wt += s_ww[k2];
            ot += s_wo[k2];
        }
        nout[b] = n;
        const int ct = (K > 0 && K < nk && (s_next >> 32) == (kth >> 32)) ? 1 : 0;
        ties[3 * b] = wt;
        ties[3 * b + 1] = ct;
        ties[3 * b + 2] = ot;
        atomicAdd(&totals[0], 1ull);
        atomicAdd(&totals[1], (wt || ct || ot) ? 1ull : 0ull);
        atomicAdd(&totals[2], (unsigned long long)wt);
        atomicAdd(&totals[3], (unsigned long long)ct);
        atomicAdd(&totals[4], (unsigned long long)ot);
    }
}

// The descriptor head's L2 normalisation of one grid cell (MagicLeap export convention, SURVEY.md
// 8(a) A3): the cell's 256 channels 4 per lane across a wave, sum of squares per lane then a
// butterfly (every lane ends with the same bits: each step adds the same two values), norm clamped
// at 1e-12, correctly rounded sqrt and division.  Shared by the grid pass and the sampler's
// per-corner form, so both give the same bits.
__device__ __forceinline__ float4 desc_cell_l2(float4 v) {
    float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    const float nrm = fmaxf(sqrt_rn(ss), 1e-12f);
    return make_float4(div_rn(v.x, nrm), div_rn(v.y, nrm), div_rn(v.z, nrm), div_rn(v.w, nrm));
}

// The whole grid normalised in place (the network's "desc" output for callers that take the grid:
// vs_network_batch_dev, vs_superpoint_forward).  One wave per cell, 16-byte accesses.
__global__ __launch_bounds__(256) void k_desc_l2norm(float* __restrict__ d, long npix) {
    const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= npix) return;
    float4* row = reinterpret_cast<float4*>(d + (size_t)p * kDescDim);
    row[lane] = desc_cell_l2(row[lane]);
}

int desc_grid_l2norm(vs_ctx* ctx, long npix, float* grid, hipStream_t s) {
    ProfScope ps(ctx, "desc_l2norm", s);
    hipLaunchKernelGGL(k_desc_l2norm, dim3((unsigned)((npix + 3) / 4)), dim3(256), 0, s, grid, npix);
    VS_HIP(hipGetLastError());
    return VS_OK;
}

// A6: bilinear sampling of the normalised coarse grid + per-keypoint L2 normalisation.  One wave
// per keypoint; each lane owns 4 channels; the sum of squares runs sequentially over c = 0..255
// on lane 0 (the reference's order) from LDS.  norm_corners: the grid is the head's raw output and
// each of the four corner cells is normalised here (desc_cell_l2, the same bits as the grid pass)
// — the pipeline's form: the network never writes and re-reads the normalised grid.
__global__ __launch_bounds__(256) void k_sample(const float* __restrict__ dgrid, int hc, int wc,
                                                const vs_keypoint* __restrict__ kps, const int* __restrict__ nkp,
                                                int cap, float* __restrict__ desc, int norm_corners) {
    post_prio();
    __shared__ float s_v[4][256];
    __shared__ float s_norm[4];
    const int b = blockIdx.y;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wv;
    const bool active = i < nkp[b];
    float val[4] = {0, 0, 0, 0};
    if (active) {
        const vs_keypoint kp = kps[(size_t)b * cap + i];
        float sx = kp.x / 8.0f;
        float sy = kp.y / 8.0f;
        int x0 = max(0, min((int)floorf(sx), wc - 1));
        int y0 = max(0, min((int)floorf(sy), hc - 1));
        int x1 = min(x0 + 1, wc - 1);
        int y1 = min(y0 + 1, hc - 1);
        float wx = sx - x0;
        float wy = sy - y0;
        const float* g = dgrid + (size_t)b * hc * wc * 256;
        float4 v00 = reinterpret_cast<const float4*>(g + ((size_t)y0 * wc + x0) * 256)[lane];
        float4 v01 = reinterpret_cast<const float4*>(g + ((size_t)y0 * wc + x1) * 256)[lane];
        float4 v10 = reinterpret_cast<const float4*>(g + ((size_t)y1 * wc + x0) * 256)[lane];
        float4 v11 = reinterpret_cast<const float4*>(g + ((size_t)y1 * wc + x1) * 256)[lane];
        if (norm_corners) {  // (wave-uniform)
            v00 = desc_cell_l2(v00);
            v01 = desc_cell_l2(v01);
            v10 = desc_cell_l2(v10);
            v11 = desc_cell_l2(v11);
        }
        const float a00[4] = {v00.x, v00.y, v00.z, v00.w}, a01[4] = {v01.x, v01.y, v01.z, v01.w};
        const float a10[4] = {v10.x, v10.y, v10.z, v10.w}, a11[4] = {v11.x, v11.y, v11.z, v11.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
            val[e] = (1 - wy) * ((1 - wx) * a00[e] + wx * a01[e]) + wy * ((1 - wx) * a10[e] + wx * a11[e]);
            s_v[wv][4 * lane + e] = val[e];
        }
    }
    __syncthreads();
    if (active && lane == 0) {
        float nrm = 0;
        for (int c = 0; c < 256; c++) {
            float v = s_v[wv][c];
            nrm += v * v;
        }
        s_norm[wv] = sqrt_rn(nrm);
    }
    __syncthreads();
    if (active) {
        const float nrm = s_norm[wv];
        if (nrm > 1e-8f) {
#pragma unroll
            for (int e = 0; e < 4; e++) val[e] = div_rn(val[e], nrm);
        }
        float4 o = {val[0], val[1], val[2], val[3]};
        reinterpret_cast<float4*>(desc + ((size_t)b * cap + i) * 256)[lane] = o;
    }
}

int sp_postprocess(vs_ctx* ctx, int B, int hc, int wc, int h, int w, vs_keypoint* d_kps, float* d_desc,
                   int* d_n, int cap, hipStream_t s, const float* semi, const float* dgrid, bool grid_raw) {
    VS_CHECK(scratch_order(ctx, s));
    ScratchUse scratch_use(ctx, s);
    if (!semi) semi = ctx->semi.as<float>();
    if (!dgrid) dgrid = ctx->dgrid.as<float>();
    const int Hp = hc * 8, Wp = wc * 8;
    const size_t npx = (size_t)B * Hp * Wp;
    // Kept pixels (and strict local maxima) are pairwise >= radius+1 apart (Chebyshev), so at most
    // ceil(H/5)*ceil(W/5).
    const int key_cap = ((Hp + kRadius) / (kRadius + 1)) * ((Wp + kRadius) / (kRadius + 1));
    const int max_kp = cap < kMaxKeypoints ? cap : kMaxKeypoints;
    const int tiles_x = (Wp + kNmsTile - 1) / kNmsTile, tiles_y = (Hp + kNmsTile - 1) / kNmsTile;
    const int ntiles = tiles_x * tiles_y;
    VS_CHECK(ctx->heat.ensure(npx * sizeof(float)));
    VS_CHECK(ctx->state.ensure(npx));
    // flags (ints): [rounds + 1][B] undecided-after-round, the capacity word, ferr [B], keycnt [B],
    // floor [B], ties [B][3], the floor histograms [B][kFloorBins]; then tile flags (bytes)
    // [rounds + 1][B][ntiles]
    const size_t nflag = (size_t)(kNmsMaxRounds + 1) * B + 1 + 6 * (size_t)B + (size_t)B * kFloorBins;
    VS_CHECK(ctx->flags.ensure(nflag * sizeof(int) + (size_t)(kNmsMaxRounds + 1) * B * ntiles));
    VS_CHECK(ctx->nms_list.ensure(npx * 2 * sizeof(int)));
    const char* fr_env = getenv("VS_NMS_FINISH_ROUNDS");  // test knob: forces the error path
    const int finish_rounds = fr_env && atoi(fr_env) > 0 ? atoi(fr_env) : kFinishMaxRounds;
    VS_CHECK(ctx->keys.ensure((size_t)B * key_cap * sizeof(unsigned long long)));
    if (!ctx->tie_totals.p) {
        VS_CHECK(ctx->tie_totals.ensure(5 * sizeof(unsigned long long)));
        VS_HIP(hipMemsetAsync(ctx->tie_totals.p, 0, 5 * sizeof(unsigned long long), s));
    }
    int* flags = ctx->flags.as<int>();
    int* err = flags + (size_t)(kNmsMaxRounds + 1) * B;
    int* ferr = err + 1;
    int* keycnt = ferr + B;
    unsigned* floor_bits = reinterpret_cast<unsigned*>(keycnt + B);
    int* ties = keycnt + 2 * B;
    int* fhist = ties + 3 * B;
    uint8_t* tflags = reinterpret_cast<uint8_t*>(flags + nflag);
    VS_HIP(hipMemsetAsync(flags, 0, nflag * sizeof(int) + (size_t)(kNmsMaxRounds + 1) * B * ntiles, s));
    VS_HIP(hipMemsetAsync(flags, 0x01, (size_t)B * sizeof(int), s));  // round 0 runs for every frame
    {
        ProfScope ps(ctx, "decode", s);  // decode + strict local maxima, one pass over semi
        hipLaunchKernelGGL(k_nms_lmax, dim3(ntiles, B), dim3(kNmsThreads), 0, s, semi, hc, wc, ctx->heat.as<float>(), B,
                           Hp, Wp, tiles_x, ntiles, fhist);
        VS_HIP(hipGetLastError());
    }
    {
        ProfScope ps(ctx, "nms_rounds", s);
        hipLaunchKernelGGL(k_nms_floor, dim3(B), dim3(kNmsThreads), 0, s, fhist, max_kp, floor_bits);
        for (int r = 0; r < kNmsMaxRounds; r++) {
            hipLaunchKernelGGL(k_nms_round, dim3(ntiles, B), dim3(kNmsThreads), 0, s, ctx->heat.as<float>(),
                               ctx->state.as<uint8_t>(), flags, tflags, floor_bits, r, B, Hp, Wp, tiles_x, ntiles);
        }
        hipLaunchKernelGGL(k_nms_finish, dim3(B), dim3(1024), 0, s, ctx->heat.as<float>(), ctx->state.as<uint8_t>(),
                           flags, kNmsMaxRounds, B, Hp, Wp, ctx->nms_list.as<int>(), finish_rounds, ferr);
        VS_HIP(hipGetLastError());
    }
    {
        ProfScope ps(ctx, "nms_select", s);
        hipLaunchKernelGGL(k_nms_collect, dim3(16, B), dim3(256), 0, s, ctx->heat.as<float>(), ctx->state.as<uint8_t>(),
                           Hp, Wp, ctx->keys.as<unsigned long long>(), keycnt, key_cap);
        hipLaunchKernelGGL(k_nms_select, dim3(B), dim3(1024), 0, s, ctx->keys.as<unsigned long long>(), keycnt, key_cap,
                           max_kp, Wp, Hp, h, w, d_kps, cap, d_n, err, ferr, ctx->heat.as<float>(), ties,
                           ctx->tie_totals.as<unsigned long long>());
        VS_HIP(hipGetLastError());
    }
    {
        ProfScope ps(ctx, "sample", s);
        hipLaunchKernelGGL(k_sample, dim3((max_kp + 3) / 4, B), dim3(256), 0, s, dgrid, hc, wc,
                           d_kps, d_n, cap, d_desc, (grid_raw && ctx->desc_l2) ? 1 : 0);
        VS_HIP(hipGetLastError());
    }
    return VS_OK;
}

// Completion check of the NMS (host-synchronous; used by the host entry points and the tests):
// VS_ERR_NOTCONV when k_nms_finish could not complete a frame (list or round cap), VS_ERR_CAPACITY
// when the packing bound was exceeded (internal error).
int sp_postprocess_check(vs_ctx* ctx, int B, hipStream_t s) {
    std::vector<int> f(B + 1);
    int* flags = ctx->flags.as<int>();
    VS_HIP(hipMemcpyAsync(f.data(), flags + (size_t)(kNmsMaxRounds + 1) * B, (B + 1) * sizeof(int),
                          hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    for (int b = 1; b <= B; b++)
        if (f[b]) {
            set_error("NMS: a frame reached the finishing pass's round cap");
            return VS_ERR_NOTCONV;
        }
    if (f[0]) {
        set_error("NMS kept more pixels than the packing bound (internal error)");
        return VS_ERR_CAPACITY;
    }
    return VS_OK;
}

}  // namespace vs
