// vs_internal.h — shared declarations of libvslam_hip.so's translation units (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/vslam_abi.h"

namespace vs {

// ---- IEEE-exact device math ---------------------------------------------------------------
// gfx950's v_sqrt_f32 is not correctly rounded and __fsqrt_rn lowers to it; the f64 sqrt is
// lowered with an fma refinement to the correctly rounded result, and rounding that to float is
// exact for sqrt (53 >= 2*24 + 2), so this equals the host's sqrtf bit for bit.
__device__ __forceinline__ float sqrt_rn(float x) { return (float)sqrt((double)x); }
// __fdiv_rn lowers to the v_div_scale / v_div_fmas / v_div_fixup correctly rounded sequence.
__device__ __forceinline__ float div_rn(float a, float b) { return __fdiv_rn(a, b); }

// ---- issue priority of the tracker's critical path ---------------------------------------
// The local-map tracking and PnP kernels of frame k share the tracking CUs with frame k + 1's
// speculative front chain (match, F-RANSAC, 3D-3D RANSAC: 1024-wave grids), which is not on the
// critical path.  Their waves raise their SIMD issue priority so the latency-bound chains of
// frame k issue first and the chain's waves fill the gaps.  (-DVS_NO_CRIT_PRIO: A/B builds.)
__device__ __forceinline__ void crit_prio() {
#ifndef VS_NO_CRIT_PRIO
    __builtin_amdgcn_s_setprio(3);
#endif
}

// The extraction post-processing (decode, NMS, sampling) shares the network's CUs with the next
// chunk's convolution waves, and the tracker waits for a chunk's features: its waves issue ahead of
// the convolutions'.  (-DVS_NO_POST_PRIO: A/B builds.)
__device__ __forceinline__ void post_prio() {
#ifndef VS_NO_POST_PRIO
    __builtin_amdgcn_s_setprio(2);
#endif
}

// ---- errors ------------------------------------------------------------------------------
void set_error(const std::string& msg);
#define VS_HIP(call)                                                                  \
    do {                                                                              \
        hipError_t e_ = (call);                                                       \
        if (e_ != hipSuccess) {                                                       \
            ::vs::set_error(std::string(#call) + ": " + hipGetErrorString(e_));       \
            return VS_ERR_HIP;                                                        \
        }                                                                             \
    } while (0)
#define VS_CHECK(rc)                   \
    do {                                \
        int rc_ = (rc);                 \
        if (rc_ != VS_OK) return rc_;   \
    } while (0)
#define VS_ARG(cond, msg)                         \
    do {                                          \
        if (!(cond)) {                            \
            ::vs::set_error(msg);                 \
            return VS_ERR_ARG;                    \
        }                                         \
    } while (0)

// ---- SuperPoint network description ----------------------------------------------------
// Canonical order (== the weight blob): conv1a conv1b conv2a conv2b conv3a conv3b conv4a conv4b
// convPa convPb convDa convDb.
struct LayerDef {
    const char* name;
    int cin, cout, k;
};
extern const LayerDef kLayers[12];
constexpr int kDescDim = 256;
constexpr int kSemiCh = 65;

// Device copy of one layer's parameters in the layout the conv kernels read:
// weight [k*k][cin][cout_pad] (cout fastest), bias [cout_pad]; padding columns are zero.
struct DevLayer {
    int cin, cout, cout_pad, k;
    float* w = nullptr;
    float* b = nullptr;
    // 3x3 layers with cin % 4 == 0: the Winograd F(2x2, 3x3) transformed weights U = G g G^T,
    // [16][cin][cout_pad] (transform element xi = 4 i + j), computed in fp64 and rounded once
    float* wu = nullptr;
    // the same layers' Winograd F(4x4, 3x3) weights U = G g G^T (round 5, wino4.hip; fp64, rounded once) in
    // the order the kernel's lanes load their B operands (winograd4_weights)
    float* wu4 = nullptr;
    // the same for k_wino4's 3-row-group variant (XG = 3, round 6: [nt][chunk][cg 4][row pair 3][lane][12])
    float* wu4x3 = nullptr;
    // conv1a (cin 1, 3x3): per output channel its 9 taps, bias, 0, 0 ([cout][12]) — read by the fused
    // conv1 kernel as wave-uniform (scalar) loads
    float* w1a_rows = nullptr;
};

// ---- growable device scratch -------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t n);  // grows (never shrinks); contents are not preserved
    void release();
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// ---- profiling ------------------------------------------------------------------------------
struct ProfStage {
    const char* name;
    double ms = 0;
    int launches = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
};

}  // namespace vs

struct vs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<float> h_weights;  // canonical blob
    // the model's "desc" output is L2-normalised over channels (true for the seeded / VSPW weights and
    // MagicLeap-style exports; an ONNX file whose "desc" is convDb's raw output sets it false, and the
    // descriptor grid is then sampled raw as FeatureExtractor.cpp:167-206 would)
    bool desc_l2 = true;
    vs::DevLayer layers[12];
    // convPa|convDa fused into one 128->512 conv (they share conv4b's output).
    vs::DevLayer head_a;

    // network activations (NHWC fp32) and post-processing scratch, sized per batch
    vs::DevBuf gray, act0, act1, semi, dgrid, heat, state, flags, keys, keycnt, nms_list;
    // host-API staging
    vs::DevBuf h_img, h_kps, h_desc, h_n, h_aux0, h_aux1, h_aux2, h_aux3, h_aux4, h_aux5;
    vs::DevBuf match_keys, match_cnt, norms_sets, tlm, ba, pnp;
    vs::DevBuf pnp_tab;  // PnP RANSAC subsets of the usual budget by point count (pnp.hip)
    bool pnp_tab_ready = false;
    vs::DevBuf em_tab;  // findEssentialMat subsets (1,000 iterations) by point count (emat.hip)
    bool em_tab_ready = false;
    vs::DevBuf em_sync;  // k_emat's split-workgroup meeting area for the context's own calls (zeroed)
    vs::DevBuf fm_sync;  // k_fmat's (zeroed)
    vs::DevBuf tie_totals;  // NMS tie accounting since the last reset: {frames, frames with a tie, window, cut, order}

    bool prof_on = false;
    int prof_mode = 0;  // 1: every stage, 2: extraction stages only (vs_profile_enable)
    std::vector<vs::ProfStage> prof;
    std::vector<hipEvent_t> event_pool;
    std::mutex prof_mu;  // a vs_slam enqueues its next batch's extraction from a helper thread
    // A vs_slam's extraction streams use the scratch above (gray .. nms_list) asynchronously, also
    // after its call returned (the prefetched next batch).  Work on any other stream that uses that
    // scratch first waits for scratch_busy (the last extraction it enqueued); null without a vs_slam.
    hipEvent_t scratch_busy = nullptr;
    hipStream_t scratch_owner[2] = {nullptr, nullptr};
    // ... and the other direction: such work records scratch_foreign when its launches are enqueued,
    // and the vs_slam's next extraction waits for it before it writes the scratch.
    hipEvent_t scratch_foreign = nullptr;
    bool scratch_foreign_pending = false;
    // local BA: the LM "done" flag mirrored into mapped pinned host memory by k_ba_control, and two
    // events, so that the host stops enqueueing iterations once the device has converged (ba.hip)
    int* ba_done_h = nullptr;
    int* ba_done_d = nullptr;
    hipEvent_t ba_ev[2] = {nullptr, nullptr};
};

namespace vs {

// profiling helpers (no-ops unless ctx->prof_on)
struct ProfScope {
    vs_ctx* ctx;
    int stage;
    hipStream_t s;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ProfScope(vs_ctx* c, const char* name, hipStream_t st);
    ~ProfScope();
};

// Orders work on stream s that uses the context's network / NMS scratch after a vs_slam's
// in-flight extraction (no-op on the vs_slam's own extraction streams and without one).
int scratch_order(vs_ctx* ctx, hipStream_t s);
// Marks the end of a non-owner stream's use of the shared scratch (see vs_ctx::scratch_foreign).
void scratch_release(vs_ctx* ctx, hipStream_t s);
// The owner side: the vs_slam's extraction stream `s` waits for the last foreign use, if any.
int scratch_acquire_owner(vs_ctx* ctx, hipStream_t s);
struct ScratchUse {  // scratch_order at construction, scratch_release at scope exit
    vs_ctx* ctx;
    hipStream_t s;
    ScratchUse(vs_ctx* c, hipStream_t st) : ctx(c), s(st) {}
    ~ScratchUse() { scratch_release(ctx, s); }
};

// ---- stage launchers (return VS_OK or an error code; enqueue on `s` only) ------------------
// Network: d_bgr is B x h x w x 3 u8 (or gray u8 when channels == 1, or nullptr when d_gray01
// already holds B x h x w fp32 in [0,1]).  Produces ctx->semi [B][hc][wc][65] and ctx->dgrid
// [B][hc][wc][256] (L2-normalised over channels; grid_raw: left as the head's raw output, for a
// post-processing call with grid_raw that normalises the four corners it samples instead).
// semi_out / dgrid_out (optional) replace ctx->semi / ctx->dgrid as the output tensors.
int sp_forward(vs_ctx* ctx, int B, const uint8_t* d_img, int channels, int h, int w,
               hipStream_t s, float* semi_out = nullptr, float* dgrid_out = nullptr, bool grid_raw = false);
// Post-processing: semi / dgrid (default ctx->semi / ctx->dgrid) -> keypoints, descriptors, counts.
int sp_postprocess(vs_ctx* ctx, int B, int hc, int wc, int h, int w, vs_keypoint* d_kps,
                   float* d_desc, int* d_n, int cap, hipStream_t s, const float* semi = nullptr,
                   const float* dgrid = nullptr, bool grid_raw = false);
// The grid's L2 normalisation in place (npix cells of 256 channels; sp_post.hip).
int desc_grid_l2norm(vs_ctx* ctx, long npix, float* grid, hipStream_t s);
// Winograd F(2x2, 3x3) stride-1 pad-1 convolution (sp_net.hip k_wino3), NHWC fp32: U = the
// transformed weights (winograd_weights), bias [cout_pad] (required), act 0 / 1 / 2 = none / ReLU /
// ReLU6 after the bias, then out = act(.) + res1, out = res2 + out (optional, [pixel][out_cstride]).
struct WinoArgs {
    const float* in;
    int in_cstride, in_coff;
    const float* wu;
    const float* wu3;  // wino4 only: the XG = 3 weight image (nullptr: XG = 2 only)
    const float* bias;
    int cin, cout, cout_pad;
    float* out;
    int out_cstride, out_coff;
    int B, H, W, nbx, nby;
    const float* w1a;
    const float* b1a;
    const float* res1;
    const float* res2;
    int act, pre_relu;
    // split-K over the input channels (blockIdx.y = split, splits <= 1: none): the output-transformed
    // partial sums (no bias, activation or residual) go to part [split][B*H*W][cout]; the caller
    // finishes them (midas.hip k_mid_splitk).  Non-pool, non-fused only.
    float* part;
    int splits;
};
int wino3_launch(WinoArgs a, bool pool, bool fuse1a, hipStream_t s);
// Winograd F(4x4, 3x3) (wino4.hip k_wino4): 16 x 16-pixel x 64-channel workgroups; bias + ReLU (+ 2 x 2 pool,
// + fused conv1a); wa.wu = winograd4_weights images.  VS_ERR_ARG for geometry it does not cover.
int wino4_launch(WinoArgs a, bool pool, bool fuse1a, hipStream_t s);
std::vector<float> winograd4_weights(const float* w, int cin, int cout_pad, int xg = 2);
// U[xi][ci][pos(co)] from direct-layout 3x3 weights w[(3a + b)][ci][co] (cout_pad columns; pos
// permutes each 32-column group for k_wino3's paired operand reads).  fp64, rounded once.
std::vector<float> winograd_weights(const float* w, int cin, int cout_pad);
// Matching
int match_pairs(vs_ctx* ctx, int P, const int* d_pairs, int F, const float* d_desc,
                const int* d_n, int cap, float ratio, vs_match* d_raw, int* d_nraw,
                vs_match* d_good, int* d_ngood, hipStream_t s,
                const float* d_norms = nullptr, unsigned long long* d_keys = nullptr,
                unsigned* d_cnt = nullptr);  // [F][cap] row norms when already known
// Sizes the context's matcher key state for P pairs of cap rows up front (no allocation inside
// a later match_pairs of at most that size).
int match_reserve(vs_ctx* ctx, int P, int cap, hipStream_t s);
// Sequential-fmaf squared norms of the descriptor rows of F frames ([F][cap], rows >= n[f] untouched).
int desc_norms(vs_ctx* ctx, int F, const float* d_desc, const int* d_n, int cap, float* d_norms, hipStream_t s);
// 3D-3D RANSAC
int ransac3d_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap,
                   const vs_match* d_good, const int* d_ngood, const float* d_depth, int h, int w,
                   const double K[4], const uint32_t* d_seeds, int iters, double thr,
                   double* d_R, double* d_t, int* d_ok, int* d_diag, hipStream_t s,
                   const uint32_t* d_mt_init = nullptr,  // [P][624] init_genrand states (optional)
                   int split = 1,            // workgroups per pair (1 .. kMaxSplit3d)
                   int* d_sync = nullptr);   // split > 1: [P][1 + 2 split] ints, zero before the first launch
constexpr int kMaxSplit3d = 8;
// Local-map tracking (d_result = {tracked, observations}).  h_kp_to_mp_src (optional): device-
// readable pinned host memory with the initial kp -> map-point table, copied into d_kp_to_mp by the
// first kernel (no separate upload); null = d_kp_to_mp already holds it.
// Round 6, the tracker's chain: a keypoint grid built ahead of time per frame slot (tlm_grid_slots:
// kTlmGridInts ints per slot, start | items), so the call skips its grid kernel, and the PnP input of
// the refinement gathered by the resolve kernel itself (io = [off {0, n, 0, 0} | obj cap x 3 | img cap x 2]).
constexpr int kTlmGridInts = 4096 + 1 + 1024 + 1;
struct TlmExtra {
    const int* grid = nullptr;  // this frame's slot in the grid pool, or null
    float* gather_io = nullptr;  // tracked_points (Slam.cpp:1408-1420) into this block, or null
    int gather_cap = 0;
};
int tlm_grid_slots(const vs_keypoint* d_kps, const int* d_n, int nframes, int kp_stride, int img_w, int img_h,
                   int* d_grid, hipStream_t s);
int track_local_map(vs_ctx* ctx, const double* d_mp_pos, const float* d_mp_desc, const uint8_t* d_mp_valid, int n_mp,
                    const vs_keypoint* d_kps, const float* d_desc, int nkp, const double R[9], const double t[3],
                    const double K[4], int img_w, int img_h, int* d_kp_to_mp, int* d_obs_mp, int* d_obs_kp,
                    int obs_cap, int* d_result, hipStream_t s, const int* h_kp_to_mp_src = nullptr,
                    const TlmExtra* ex = nullptr);
// Pose LM, nprob problems with point ranges d_off[p]..d_off[p+1]
int optimize_pose(vs_ctx* ctx, int nprob, const double* d_P, const float* d_p2, const int* d_off, const double K[4],
                  double* d_R, double* d_t, double* d_res, int* d_ok, hipStream_t s);
// PnP RANSAC + LM, nprob problems with point ranges d_off[p]..d_off[p+1]
// max_n: an upper bound of every problem's point count when the caller knows one (-1: unknown); with
// the usual budget (100) and max_n <= 1024 the subsets come from the context's table.
int solve_pnp(vs_ctx* ctx, int nprob, const float* d_obj, const float* d_img, const int* d_off, const double K[4],
              int ransac_iters, int min_inliers, double* d_R, double* d_t, int* d_stat, uint8_t* d_mask,
              hipStream_t s, int max_n = -1);
// Builds the context's PnP subset table now (synchronises s once); solve_pnp builds it on first use.
int pnp_reserve(vs_ctx* ctx, hipStream_t s);
// F-matrix verification: per frame pair (pipeline) or per point set (ABI single problem)
// F-RANSAC's first chunk (64 hypotheses) can be scored by split workgroups at once (fmat.hip; default 1 for
// frame pairs, kFmSplit for the ABI's point sets), meeting in d_sync (kFmSyncBytes per pair, zeroed once): a
// caller whose launches may overlap another's passes its own (P == 1), nullptr takes the context's.
constexpr int kFmSplit = 8, kFmFirstChunk = 64;
constexpr size_t kFmSyncBytes = 1024;
int fmat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_good,
               const int* d_ngood, double* d_F, vs_match* d_kept, int* d_nkept, double* d_err, int* d_diag,
               hipStream_t s, int split = 0, char* d_sync = nullptr);
int fmat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, double thr, double conf,
                int max_iters, double* d_F, uint8_t* d_mask, double* d_err, int* d_diag, hipStream_t s);
// Essential-matrix motion + depth scale (A12): per frame pair (pipeline) or per point set.
// The first 8 split RANSAC iterations of a problem run on split workgroups (emat.hip), which meet in
// d_sync (kEmSyncBytes per problem, zeroed once; re-armed by the kernel): a caller whose launches may
// overlap another's passes its own, nullptr takes the context's (split <= 0: the default — one problem
// the whole 1,000-iteration budget, kEmSplitMax; a batch 8; the tracker's chains pass 8).
constexpr int kEmSplitMax = 125;
constexpr size_t kEmSyncBytes = 786432;
constexpr int kEmTabMinN = 6;  // the subset table's first row: n = 6 (every n > 5 runs RANSAC)
int emat_pairs(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps, int cap, const vs_match* d_kept,
               const int* d_nkept, const int* d_skip, const float* d_depth, int h, int w, const double K[4],
               double* d_R, double* d_t, double* d_scale, int* d_ok, int* d_diag, hipStream_t s, int split = 0,
               char* d_sync = nullptr);
// Builds the context's findEssentialMat subset table now (synchronises s once); emat_* build it on first use.
int emat_reserve(vs_ctx* ctx, hipStream_t s);
// cv::RNG subsets (5 distinct indices, repeats redrawn) of rows problems with n = n_base + row points,
// iters per row, into out[row][iters][5] (pnp.hip: the PnP sampler, the same RANSACPointSetRegistrator)
int subset_table(int rows, int n_base, int iters, int* out, hipStream_t s);
int emat_points(vs_ctx* ctx, int P, const float* d_p1, const float* d_p2, const int* d_off, const float* d_depth1,
                const float* d_depth2, int h, int w, const double K[4], double* d_R, double* d_t, double* d_scale,
                int* d_ok, int* d_diag, hipStream_t s);
// Local bundle adjustment over a gathered window (host arrays in/out, see vs_local_ba)
int local_ba(vs_ctx* ctx, int N, double* R, double* t, int M, double* P, int n_obs, const int* okf, const int* opt,
             const double* ouv, const double K4[4], int max_iter, double* err_before, double* err_after, int stats[3]);

}  // namespace vs
