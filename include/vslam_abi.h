/*
 * vslam_abi.h — C ABI of libvslam_hip.so, the MI355X (gfx950) implementation of the
 * per-frame compute hot path of salah-dev-stu/visual-slam-pipeline.
 *
 * Drop-in boundary.  Each entry point replaces one reference interface (file:line under the
 * reference tree); the C++ facade in visual-slam-pipeline_amd/host/ keeps the reference class
 * surfaces (FeatureExtractor / Frame / Optimizer / match_features / estimate_motion_3d3d) on
 * top of these calls, and INTEGRATION.md shows the binding a maintainer adds to Slam.cpp.
 *
 * Conventions
 *   - No C++ types, exceptions or OpenCV types cross this ABI: plain pointers, sizes, ints.
 *   - Every call returns int status: VS_OK (0) or a negative VS_ERR_* code; vs_last_error()
 *     returns a thread-local human-readable message for the last failure.
 *   - "host" entry points take caller-owned HOST buffers and are synchronous (the reference
 *     semantics).  "_dev" entry points take DEVICE pointers (hipMalloc'd, e.g. torch tensors)
 *     and a hipStream_t passed as void* (NULL = the context's own stream); they only enqueue.
 *   - A vs_ctx owns device scratch, the SuperPoint weights and a stream.  One context per
 *     host thread x GPU; contexts are not thread-safe (neither is the reference's
 *     FeatureExtractor, FeatureExtractor.cpp:52,79).
 *   - Layouts match the reference's OpenCV types bit for bit: vs_keypoint == cv::KeyPoint,
 *     vs_match == cv::DMatch, descriptors are row-major N x 256 fp32 (CV_32F), depth maps are
 *     row-major H x W fp32 metres with 0 = invalid (Frame.cpp:47-54), poses are row-major
 *     3x3 / 3x1 fp64 (CV_64F), K = {fx, fy, cx, cy} (Config.h:14-17).
 */
#ifndef VSLAM_ABI_H
#define VSLAM_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VS_ABI_VERSION 1

enum {
    VS_OK = 0,
    VS_ERR_ARG = -1,      /* bad argument (null pointer, bad size)                    */
    VS_ERR_HIP = -2,      /* HIP runtime failure (message in vs_last_error)           */
    VS_ERR_NOMEM = -3,    /* device or host allocation failed                         */
    VS_ERR_IO = -4,       /* weight file missing or malformed                         */
    VS_ERR_CAPACITY = -5, /* an internal bound was exceeded (message says which)      */
    VS_ERR_NOTCONV = -6   /* an iterative device stage did not converge (NMS rounds)  */
};

/* == cv::KeyPoint (28 B) == one SPCF keypoint record (FeatureExtractor.cpp:294-304). */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} vs_keypoint;

/* == cv::DMatch (16 B). */
typedef struct {
    int32_t query_idx, train_idx, img_idx;
    float distance;
} vs_match;

typedef struct vs_ctx vs_ctx;

/* ---- library / context --------------------------------------------------------------- */
int         vs_abi_version(void);
const char* vs_last_error(void);

/* Replaces FeatureExtractor::init (FeatureExtractor.h:18, FeatureExtractor.cpp:22-44).
 * superpoint_weights: the reference's own model file (models/superpoint_v1.onnx, Slam.cpp:28-31:
 * an ONNX SuperPoint export, read by the library's protobuf reader and mapped through the graph's
 * Conv nodes), a VSPW weight file (see vs_superpoint_save_weights), or NULL for the seeded
 * synthetic He-normal weights (seed VS_SYNTH_WEIGHT_SEED).  Unlike the reference, a failure is
 * reported (VS_ERR_IO, vs_last_error) instead of silently switching to ORB. */
#define VS_SYNTH_WEIGHT_SEED 20261015ull
int  vs_create(int device, const char* superpoint_weights, vs_ctx** out);
void vs_destroy(vs_ctx* ctx);
void* vs_stream(vs_ctx* ctx); /* the context's hipStream_t */

/* SuperPoint parameter blob, canonical order (PyTorch/ONNX layout per layer:
 * weight [Cout][Cin][kh][kw] then bias [Cout]; layers conv1a conv1b conv2a conv2b conv3a conv3b
 * conv4a conv4b convPa convPb convDa convDb).  Used by tests to build the fp32 torch reference. */
size_t vs_superpoint_num_params(void);
int    vs_superpoint_get_weights(vs_ctx* ctx, float* out, size_t count);
/* Host only (no device needed): the canonical weights (count = vs_superpoint_num_params()) read
 * from an ONNX SuperPoint export — the file FeatureExtractor::init hands to ONNX Runtime
 * (FeatureExtractor.cpp:22-44) — mapped through the graph's Conv nodes; and the seeded synthetic
 * weights vs_create(…, NULL, …) uses. */
int    vs_superpoint_onnx_weights(const char* onnx_path, float* out, size_t count);
int    vs_superpoint_synth_weights(float* out, size_t count);
/* Host only: the ONNX export's "desc" output tail (FeatureExtractor.cpp:116-206 samples whatever the
 * graph returns): *normalized = 1 when "desc" is convDb's output L2-normalised over channels, 0 when
 * it is convDb's raw output.  Any other "desc" / "semi" tail (e.g. a softmax on "semi") is VS_ERR_IO,
 * as vs_create reports it.  vs_desc_normalized: the same flag of a context (1 for the seeded / VSPW
 * weights); with 0 the network's descriptor grid is not normalised before the keypoint sampling. */
int    vs_superpoint_onnx_desc_normalized(const char* onnx_path, int* normalized);
int    vs_desc_normalized(vs_ctx* ctx, int* normalized);
int    vs_superpoint_save_weights(vs_ctx* ctx, const char* path);

/* ---- A1-A6: FeatureExtractor::extract (FeatureExtractor.cpp:49-81, 87-207, 219-259) ---- */
/* One frame, host buffers.  img: H x W BGR (channels=3, cv::Mat 8UC3) or gray (channels=1),
 * row stride in bytes.  kps: cap records; desc: cap*256 floats; *n = keypoints written
 * (descending score order, reference NMS semantics).  cap must be >= 1; at most
 * min(cap, 400) keypoints are kept (SP_MAX_KEYPOINTS, Config.h:42). */
#define VS_SP_MAX_KEYPOINTS 400
int vs_extract(vs_ctx* ctx, const uint8_t* img, int h, int w, int channels, size_t stride,
               vs_keypoint* kps, float* desc, int cap, int* n);

/* B frames, host buffers: imgs[b] points at frame b; kps is B*cap, desc B*cap*256, n is B. */
int vs_extract_batch(vs_ctx* ctx, int B, const uint8_t* const* imgs, int h, int w, int channels,
                     size_t stride, vs_keypoint* kps, float* desc, int cap, int* n);

/* B frames, device buffers (offline batch mode): d_imgs is B contiguous H x W x 3 BGR u8
 * frames; outputs d_kps [B][cap], d_desc [B][cap][256], d_n [B].  Enqueue only (no host sync):
 * a frame whose NMS could not be completed on the device (its undecided pixels exceed the
 * finishing pass's list) gets d_n[b] = VS_ERR_NOTCONV and no keypoints; every consumer of d_n in
 * this library (matching, the tracker) treats a negative count as an error / empty frame. */
int vs_extract_batch_dev(vs_ctx* ctx, int B, const uint8_t* d_imgs, int h, int w,
                         vs_keypoint* d_kps, float* d_desc, int* d_n, int cap, void* stream);

/* The two halves of vs_extract_batch_dev, so a caller can overlap one batch's post-processing
 * with the next batch's network on another stream.  Network: d_imgs (B BGR u8 frames) ->
 * d_semi [B][H/8][W/8][VS_SEMI_CH] logits and d_dgrid [B][H/8][W/8][VS_DESC_DIM] L2-normalised
 * coarse descriptors (channel-last; H, W rounded up to multiples of 8).  Post-processing (A4-A6:
 * decode, NMS, top-k, border erase, descriptor sampling) reads them and writes d_kps / d_desc /
 * d_n as vs_extract_batch_dev does.  Network scratch and post-processing scratch are disjoint in
 * the context, so the two may run concurrently on different streams (one call of each at a time). */
#define VS_SEMI_CH 65
#define VS_DESC_DIM 256
int vs_network_batch_dev(vs_ctx* ctx, int B, const uint8_t* d_imgs, int h, int w, float* d_semi,
                         float* d_dgrid, void* stream);
int vs_postprocess_batch_dev(vs_ctx* ctx, int B, const float* d_semi, const float* d_dgrid, int h,
                             int w, vs_keypoint* d_kps, float* d_desc, int* d_n, int cap,
                             void* stream);

/* Stage isolation.  Network only: gray fp32 image (already /255 normalised, H x W) ->
 * semi [65][H/8][W/8] and desc [256][H/8][W/8], the ORT output layout
 * (FeatureExtractor.cpp:120-124,167-168).  H and W must be multiples of 8. */
int vs_superpoint_forward(vs_ctx* ctx, const float* gray01, int h, int w, float* semi,
                          float* desc_grid);
/* Post-network only (A4-A6): ORT-layout semi/desc -> keypoints + sampled descriptors, for a
 * padded image of Hp = 8*Hc rows, Wp = 8*Wc cols and original size h x w (border erase
 * FeatureExtractor.cpp:155-160). */
int vs_postprocess(vs_ctx* ctx, const float* semi, const float* desc_grid, int hc, int wc,
                   int h, int w, vs_keypoint* kps, float* desc, int cap, int* n);

/* ---- A7: Slam::match_features (Slam.cpp:1140-1172) -------------------------------------- */
/* desc1 = query (reference keyframe), desc2 = train (current frame), rows of 256 fp32.
 * Exact L2 2-NN (replaces FLANN's approximate search), raw = best neighbour of
 * every query row when n2 >= 2, good = rows with d0 < ratio * d1, both in query order.
 * raw/good need n1 records each. */
int vs_match_ratio(vs_ctx* ctx, const float* desc1, int n1, const float* desc2, int n2,
                   float ratio, vs_match* raw, int* n_raw, vs_match* good, int* n_good);

/* P frame pairs on device: d_pairs[2p] = query frame, d_pairs[2p+1] = train frame, indexing
 * the F frames of d_desc [F][cap][256] and d_n [F].  Outputs d_raw/d_good [P][cap],
 * d_nraw/d_ngood [P]. */
int vs_match_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, int F, const float* d_desc,
                       const int* d_n, int cap, float ratio, vs_match* d_raw, int* d_nraw,
                       vs_match* d_good, int* d_ngood, void* stream);

/* ---- A9: Slam::estimate_motion_3d3d (Slam.cpp:214-375) ---------------------------------- */
/* pts1/pts2: n (x,y) float pairs (matched keypoint positions), depth1/depth2: h x w fp32
 * metres.  seed = 42 + frame_count_ (Slam.cpp:276), iters = RANSAC_3D3D_ITERATIONS (200),
 * thr = RANSAC_3D3D_INLIER_THRESH (0.05).  R,t map ref-camera points to current-camera points.
 * *ok = the reference's boolean result; diag (may be NULL) receives
 * {N back-projected, best inliers, best iteration, refit inliers}. */
int vs_ransac_3d3d(vs_ctx* ctx, const float* pts1, const float* pts2, int n,
                   const float* depth1, const float* depth2, int h, int w, const double K[4],
                   uint32_t seed, int iters, double thr, double R[9], double t[3], int* ok,
                   int diag[4]);

/* P pairs on device, fed straight from vs_match_pairs_dev's good lists: pair p uses
 * d_good[p][0..d_ngood[p]) with keypoints d_kps[F][cap] and depth maps d_depth [F][h][w] of
 * its two frames.  Outputs d_R [P][9], d_t [P][3], d_ok [P], d_diag [P][4].
 * seeds[p] (device) = 42 + frame_count for that pair. */
int vs_ransac_3d3d_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps,
                             int cap, const vs_match* d_good, const int* d_ngood,
                             const float* d_depth, int h, int w, const double K[4],
                             const uint32_t* d_seeds, int iters, double thr, double* d_R,
                             double* d_t, int* d_ok, int* d_diag, void* stream);

/* ---- A11: Slam::track_local_map (Slam.cpp:380-469) -------------------------------------- */
/* Map points: mp_pos n_mp x 3 fp64 (world), mp_desc n_mp x 256 fp32, mp_valid[i] = valid AND
 * has a descriptor (Slam.cpp:417-418).  Keypoints/descriptors of the frame (n_kp <= 1024), its
 * camera->world pose, K (the reference uses Config FX/FY/CX/CY) and image size (640 x 480 in the
 * reference, Config.h:10-11).  kp_to_mp (n_kp) is updated in place (Frame::map_point_indices);
 * *tracked = the reference's return value; the (map point, keypoint) pairs the reference passes
 * to MapPoint::add_observation are returned in map-point order (first obs_cap of *n_obs). */
int vs_track_local_map(vs_ctx* ctx, const double* mp_pos, const float* mp_desc,
                       const uint8_t* mp_valid, int n_mp, const vs_keypoint* kps,
                       const float* desc, int n_kp, const double R_world[9],
                       const double t_world[3], const double K[4], int img_w, int img_h,
                       int* kp_to_mp, int* tracked, int* obs_mp, int* obs_kp, int obs_cap,
                       int* n_obs);
/* Device variant (map resident in HBM); d_result[0] = tracked, d_result[1] = n_obs. */
int vs_track_local_map_dev(vs_ctx* ctx, const double* d_mp_pos, const float* d_mp_desc,
                           const uint8_t* d_mp_valid, int n_mp, const vs_keypoint* d_kps,
                           const float* d_desc, int n_kp, const double R_world[9],
                           const double t_world[3], const double K[4], int img_w, int img_h,
                           int* d_kp_to_mp, int* d_obs_mp, int* d_obs_kp, int obs_cap,
                           int* d_result, void* stream);

/* ---- A13: Optimizer::optimize_pose (Optimizer.cpp:54-180) ------------------------------- */
/* p3d n x 3 fp64 world points, p2d n x 2 fp32 pixels; R, t = camera->world pose in/out (the
 * frame's pose is updated, Optimizer.cpp:166-168).  RMS reprojection error before/after; both 0
 * and the pose untouched when n < 3 (Optimizer.cpp:60-62). */
int vs_optimize_pose(vs_ctx* ctx, const double* p3d, const float* p2d, int n, const double K[4],
                     double R[9], double t[3], double* rms_before, double* rms_after);
/* nprob independent problems on device: points d_off[p] .. d_off[p+1]; d_R [p][9], d_t [p][3]
 * in/out; d_res [p][4] = {rms_before, rms_after, iterations, accepted steps}; d_ok [p]. */
int vs_optimize_pose_batch_dev(vs_ctx* ctx, int nprob, const double* d_p3d, const float* d_p2d,
                               const int* d_off, const double K[4], double* d_R, double* d_t,
                               double* d_res, int* d_ok, void* stream);

/* ---- A10: Slam::solve_pnp (Slam.cpp:505-529) --------------------------------------------- */
/* cv::solvePnPRansac(obj, img, K, no distortion, useExtrinsicGuess = false, ransac_iters,
 * 8 px (Config.h:78), confidence 0.99) + the camera -> world conversion (Slam.cpp:521-526).
 * obj_pts n x 3 fp32 (cv::Point3f), img_pts n x 2 fp32 (cv::Point2f); ransac_iters <=
 * VS_PNP_MAX_ITERS.  *success = PnPResult.success (n >= min_inliers, RANSAC found a model and
 * its inlier count >= min_inliers); R_world / t_world written on success; *inlier_count =
 * inliers.rows; inlier_mask (n, nullable) = the RANSAC inliers; diag (nullable) = {RANSAC
 * iterations run, winning iteration, LM iterations, LM accepted steps}. */
#define VS_PNP_MAX_ITERS 2048
int vs_solve_pnp(vs_ctx* ctx, const float* obj_pts, const float* img_pts, int n, const double K[4],
                 int ransac_iters, int min_inliers, double R_world[9], double t_world[3],
                 int* success, int* inlier_count, uint8_t* inlier_mask, int diag[4]);
/* nprob problems on device (one workgroup each): points d_off[p] .. d_off[p+1] of d_obj / d_img;
 * d_R [p][9], d_t [p][3] = world pose (written on success); d_stat [p][8] = {success, inliers,
 * RANSAC iterations, winning iteration, LM iterations, LM accepted, n, 0}; d_mask [total points]
 * = RANSAC inliers (required). */
int vs_solve_pnp_batch_dev(vs_ctx* ctx, int nprob, const float* d_obj, const float* d_img,
                           const int* d_off, const double K[4], int ransac_iters, int min_inliers,
                           double* d_R, double* d_t, int* d_stat, uint8_t* d_mask, void* stream);

/* ---- A8: F-matrix verification (Slam.cpp:880-910, 1174-1187, 1217-1240) -------------------- */
/* cv::findFundamentalMat(p1, p2, FM_RANSAC, thr, conf, max_iters) on one point set (n <=
 * VS_FM_MAX_POINTS, interleaved xy fp32).  *ok = F non-empty (F row-major, F(3,3) = 1);
 * mask (n, nullable) = inliers (all 0 when F is empty); diag (nullable) = {method 0 none /
 * 1 seven-point / 2 RANSAC (n >= 15) / 3 LMedS (8..14), iterations run, winning iteration,
 * inliers}; err (nullable) = Slam::compute_epipolar_error over all points and over the inliers
 * (0 when F is empty). */
#define VS_FM_MAX_POINTS 2048
int vs_find_fundamental(vs_ctx* ctx, const float* p1, const float* p2, int n, double thr,
                        double conf, int max_iters, double F[9], uint8_t* mask, int* ok,
                        int diag[4], double err[2]);
/* Slam.cpp:880-910 for P frame pairs on device: matches d_good [p][cap] (query -> keypoints of
 * slot d_pairs[2p], train -> slot d_pairs[2p+1], d_kps [slot][cap]) are verified with
 * findFundamentalMat(FM_RANSAC, 3.0, 0.999); d_kept [p][cap] / d_nkept [p] = the surviving
 * matches in order (all of them when F is empty); d_F [p][9] (zeros when empty); d_err [p][2] =
 * {epipolar_error_before_, epipolar_error_after_}; d_diag [p][8] = {method, iterations,
 * winning iteration, inliers, F ok, n, kept, 0}.  cap <= VS_FM_MAX_POINTS. */
int vs_fmat_verify_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps,
                             int cap, const vs_match* d_good, const int* d_ngood, double* d_F,
                             vs_match* d_kept, int* d_nkept, double* d_err, int* d_diag,
                             void* stream);

/* ---- A12: Slam::estimate_motion + depth scale (Slam.cpp:1193-1213, 73-207, used :965-984) ---- */
/* cv::findEssentialMat(K, RANSAC, 0.999, 1.0 px) + cv::recoverPose + the >= 15 inlier and
 * determinant checks on n <= VS_EM_MAX_POINTS pixel correspondences (interleaved xy fp32), then
 * Slam::estimate_scale_from_depth with the reference depth map depth1 and the current depth2
 * (h x w fp32 metres; depth2 NULL = single-depth variant, depth1 NULL = no scale).  *ok = the
 * reference's return value; R, t (unit) = relative motion x2 = R x1 + t (written when ok);
 * *scale = the estimate or -1 (the caller then falls back to its last good scale / MOTION_SCALE,
 * Slam.cpp:976-980); diag (nullable) = {E found, RANSAC iterations, winning iteration, E inliers,
 * recoverPose good, n, ran, 0}. */
#define VS_EM_MAX_POINTS 512
int vs_estimate_motion(vs_ctx* ctx, const float* p1, const float* p2, int n, const double K[4],
                       const float* depth1, const float* depth2, int h, int w, double R[9],
                       double t[3], double* scale, int* ok, int diag[8]);
/* Pipeline form on device: P frame pairs (d_pairs, keypoints d_kps [slot][cap], the F-verified
 * matches d_kept [p][cap] / d_nkept, depth slots d_depth [slot][h][w], or NULL for a monocular
 * stream: no scale, *d_scale = -1, BASELINE config[4]); pairs with d_skip[p] != 0
 * (e.g. the 3D-3D result was ok) are skipped.  d_R [p][9], d_t [p][3], d_scale [p], d_ok [p],
 * d_diag [p][8].  cap <= VS_EM_MAX_POINTS.  The RANSAC's workgroups meet in a per-context area
 * (round 6), so calls on one context must not overlap in time across different streams. */
int vs_emat_motion_pairs_dev(vs_ctx* ctx, int P, const int* d_pairs, const vs_keypoint* d_kps,
                             int cap, const vs_match* d_kept, const int* d_nkept, const int* d_skip,
                             const float* d_depth, int h, int w, const double K[4], double* d_R,
                             double* d_t, double* d_scale, int* d_ok, int* d_diag, void* stream);

/* ---- A14: Optimizer::local_bundle_adjustment (Optimizer.cpp:187-599) --------------------- */
/* The window as the reference gathers it (:205-244): N keyframe poses (camera -> world R_world
 * [N][9], t_world [N][3]; poses 1..N-1 are written back, :584-588), M map points [M][3]
 * (written back, :590-595) and n_obs observations (keyframe index, point index, u, v) in the
 * reference's gather order (keyframe-major, keypoint order).  max_iter = 15 reproduces the
 * reference (MAX_ITER, :294).  *err_before / *err_after = the returned RMS pair ({0, 0} and nothing
 * written when N < 2, n_obs < 20 or M < 10); stats (nullable) = {LM iterations, accepted steps,
 * ran}.  N <= VS_BA_MAX_KEYFRAMES. */
#define VS_BA_MAX_KEYFRAMES 64
int vs_local_ba(vs_ctx* ctx, int N, double* R_world, double* t_world, int M, double* points,
                int n_obs, const int* obs_kf, const int* obs_pt, const double* obs_uv,
                const double K[4], int max_iter, double* err_before, double* err_after,
                int stats[3]);

/* ---- F1: the tracking loop, Slam::process_frame (Slam.cpp:809-1135) ---------------------- */
/* A vs_slam is the reference's Slam object for the per-frame path: map, keyframes, EKF, RTS
 * smoother (host/tracker.hpp restates the control flow; every arithmetic stage runs on the GPU
 * through the context it was created on).  Images are 640 x 480 (Config.h:10-11), K is the
 * reference's (Config.h:14-17).  Loop closure runs as the reference's does (loop edges and PGO
 * constraints, vs_slam_loops); like the reference it never changes a pose (the pose graph is never
 * optimised: Slam.cpp:1748 has no caller). */
typedef struct vs_slam vs_slam;
#define VS_SLAM_NSTATS 24
/* max_batch: frames per vs_slam_process_batch_dev call (the device frame pool holds two batches). */
int  vs_slam_create(vs_ctx* ctx, int max_batch, int h, int w, vs_slam** out);
void vs_slam_destroy(vs_slam* slam);
/* Slam::set_initial_pose (Slam.cpp:35-38). */
int vs_slam_set_initial_pose(vs_slam* slam, const double R[9], const double t[3]);
/* Slam::set_accelerometer_data + compute_gravity_direction (Slam.cpp:1580-1616, called as in
 * main.cpp:1053-1066, i.e. after the initial pose): samples n x {timestamp, ax, ay, az}. */
int vs_slam_set_accelerometer(vs_slam* slam, const double* samples, int n);
/* B consecutive processed frames already in HBM (d_bgr B x h x w x 3 u8, d_depth B x h x w fp32
 * metres or NULL) plus the host copies of the depth maps (h_depth[b], read during the call;
 * NULL when d_depth is NULL), timestamps and frame ids (the image index, Frame::id).  Extracts all
 * B frames in one batched SuperPoint pass, then runs Slam::process_frame on each in order;
 * processed[b] = its return value. */
int vs_slam_process_batch_dev(vs_slam* slam, int B, const uint8_t* d_bgr, const float* d_depth,
                              const float* const* h_depth, const double* timestamps, const int* ids,
                              int* processed);
/* The frames of the NEXT vs_slam_process_batch_dev call (same B, d_bgr, d_depth), given before the
 * current one: the next call's extraction is enqueued right behind the current batch's, so it runs
 * while the current batch is tracked.  The buffers must stay unchanged until that call; a next
 * call with other buffers waits for the prefetch and extracts its own frames. */
int vs_slam_prefetch_batch_dev(vs_slam* slam, int B, const uint8_t* d_bgr, const float* d_depth);
/* One frame from host features (e.g. a FeatureExtractor SPCF cache hit, FeatureExtractor.cpp:54-61):
 * n_kp keypoints + n_kp x 256 descriptors, depth h x w fp32 metres (NULL = none). */
int vs_slam_process_features(vs_slam* slam, int n_kp, const vs_keypoint* kps, const float* desc,
                             const float* depth, double timestamp, int id, int* processed);
/* Slam::run_rts_smoother (Slam.cpp:1761-1810). */
int vs_slam_finish(vs_slam* slam);
/* Map frames in insertion order (Map::get_all_frames): *n = count; the first cap entries of ids,
 * timestamps, R (cap x 9, camera -> world) and t (cap x 3) are written (each nullable). */
int vs_slam_trajectory(vs_slam* slam, int cap, int* ids, double* timestamps, double* R, double* t,
                       int* n);
/* {processed, rejected (< 30 keypoints), via 3D-3D, via E-matrix, E failed, bridge keyframes,
 *  PnP recoveries, recoveries failed, stationary, keyframes, PnP refinements, periodic PnP,
 *  tracked map points (sum), triangulated points, depth points, culled points, chains recomputed,
 *  map points, valid map points, frame_count_, keyframe_count_, last match count,
 *  F-RANSAC iterations (sum over chains), 0} */
int vs_slam_stats(vs_slam* slam, int* out, int cap);
/* Loop closures (Slam::handle_loop_closure, Slam.cpp:730-798, every 200 keyframes): loop edges
 * (matched keyframe id, frame id; Slam::loop_edges_) and the PGO constraints of verified loops
 * (16 doubles each: from id, to id, R_rel[9], t_rel[3], trans_sigma, rot_sigma); the first cap of
 * each are written (buffers nullable).  stats[23] = LoopCloser::loop_count(). */
int vs_slam_loops(vs_slam* slam, int cap, int* edges, double* constraints, int* n_edges, int* n_constraints);
/* Map points (Map::map_points): *n = count; the first cap positions (world, x 3) and validity
 * bytes are written (each nullable). */
int vs_slam_map(vs_slam* slam, int cap, double* pos, uint8_t* valid, int* n);

/* ---- F3: DepthEstimator::estimate (DepthEstimator.cpp:39-112), MiDaS v2.1-small ---------------
 * The midas_v21_small_256 network (EfficientNet-Lite3 encoder, features 64, expand, non-negative)
 * with the reference's pre-processing (INTER_LINEAR resize to 256 x 256, 1/255, per-channel
 * mean / std on the BGR planes as :54-67 writes it) and post-processing (INTER_LINEAR resize back,
 * min-max normalisation when the range exceeds 1e-6, :96-109).  The reference never consumes the
 * result; BASELINE config[4] runs it per frame. */
typedef struct vs_midas vs_midas;
/* weights_path: the reference's own model file (models/midas_v21_small_256.onnx, Slam.cpp:30-31:
 * Conv nodes in graph order, BatchNormalization folded), a VSMW file (tools/midas_to_vsmw.py
 * converts a MiDaS state_dict, BatchNorm folded) or NULL for seeded He-normal weights. */
int vs_midas_create(vs_ctx* ctx, const char* weights_path, vs_midas** out);
void vs_midas_destroy(vs_midas* m);
size_t vs_midas_num_params(void);
double vs_midas_flops_per_frame(void);
int vs_midas_get_weights(vs_midas* m, float* out, size_t count);
/* Host only: canonical MiDaS weights from an ONNX export of midas_v21_small_256 (the file
 * DepthEstimator::init hands to ONNX Runtime, DepthEstimator.cpp:15-36; BatchNormalization folded)
 * and the seeded synthetic weights vs_midas_create(…, NULL, …) uses. */
int vs_midas_onnx_weights(const char* onnx_path, float* out, size_t count);
int vs_midas_synth_weights(float* out, size_t count);
/* B frames d_bgr [B][h][w][3] u8 -> d_depth [B][h][w] fp32 in [0, 1] (enqueue only). */
int vs_midas_estimate_dev(vs_midas* m, int B, const uint8_t* d_bgr, int h, int w, float* d_depth, void* stream);
/* The three stages separately (tests): d_input [B][256][256][3] fp32 (NHWC, normalised),
 * d_out [B][256][256] the network's output, d_depth as above. */
int vs_midas_preprocess_dev(vs_midas* m, int B, const uint8_t* d_bgr, int h, int w, float* d_input, void* stream);
int vs_midas_forward_dev(vs_midas* m, int B, const float* d_input, float* d_out, void* stream);
int vs_midas_postprocess_dev(vs_midas* m, int B, const float* d_small, int h, int w, float* d_depth, void* stream);

/* ---- (e) the offline frame-sharded front end (BASELINE config[3]) ---------------
 * One process per GPU; per step each rank extracts its B frames, the step's feature records are
 * all-gathered over RCCL (xGMI), and the B frame pairs ending in the rank's frames go through
 * match_features, F verification, 3D-3D RANSAC and the E fallback (Slam.cpp:838-984).  The C form
 * of python/vslam_pipeline.DevicePipeline, with bit-identical results.  RCCL is loaded at run time
 * (librccl.so.1); a one-rank batch does not need it. */
#define VS_BATCH_ID_BYTES 128 /* == NCCL_UNIQUE_ID_BYTES */
typedef struct vs_batch vs_batch;
typedef struct {
    int ok3d;                  /* estimate_motion_3d3d succeeded (R3, t3: pose of frame p+1 vs p) */
    double R3[9], t3[3];
    int okE;                   /* the essential-matrix fallback succeeded (only when ok3d == 0) */
    double RE[9], tE[3], scale; /* scale: estimate_scale_from_depth, -1 when unavailable */
    int n_good, n_kept;        /* ratio-test matches, F-verified matches */
} vs_pair_motion;
/* Rank 0 creates the communicator id and distributes the VS_BATCH_ID_BYTES bytes (MPI, a file...). */
int vs_batch_unique_id(void* id);
/* world == 1: id may be NULL (no communicator; with an id, one rank runs the exchange path). */
int vs_batch_create(vs_ctx* ctx, int B, int h, int w, int rank, int world, const void* id, vs_batch** out);
void vs_batch_destroy(vs_batch* b);
/* One step (synchronous): this rank's B frames d_bgr [B][h][w][3] u8 and depth [B][h][w] metres,
 * d_depth_prev the depth of frame rank * B - 1 (required with a communicator except on rank 0's
 * first step: VS_ERR_ARG otherwise), frame_count0 the processed-frame index of d_bgr[0] (RANSAC
 * seed 42 + index, Slam.cpp:276); out[p] = motion of pair (frame p - 1, frame p) of the block,
 * p = 0..B-1.  The neighbour frame's features arrive over a point-to-point ring (ncclSend /
 * ncclRecv: one record per rank per step), or from the all-gather in gather mode. */
int vs_batch_step_dev(vs_batch* b, const uint8_t* d_bgr, const float* d_depth, const float* d_depth_prev,
                      int frame_count0, vs_pair_motion* out, void* stream);
/* The same step split in two (round 5), so that consecutive steps overlap: submit enqueues the step
 * (network on the batch's network stream; post-processing, exchange and pair geometry on its geometry
 * stream; both first wait for the work already enqueued on `stream`) and returns without
 * synchronising; at most two steps are in flight, and the next step's network runs beside this
 * step's geometry.  The step's inputs (d_bgr, d_depth, d_depth_prev) must stay unchanged until its
 * collect returns.  collect waits for the oldest submitted step and writes its pair motions.
 * vs_batch_step_dev == submit + collect. */
int vs_batch_submit_dev(vs_batch* b, const uint8_t* d_bgr, const float* d_depth, const float* d_depth_prev,
                        int frame_count0, void* stream);
int vs_batch_collect(vs_batch* b, vs_pair_motion* out);
/* Gather mode (on != 0, with a communicator): every step all-gathers all ranks' records, so that
 * vs_batch_features_dev returns the whole step (rank 0 writing the SPCF cache).  Default: off. */
int vs_batch_set_gather(vs_batch* b, int on);
/* The last step's feature records on the device (gather mode: all ranks' frames in global order;
 * otherwise this rank's), e.g. for vs_spcf_write_dev. */
int vs_batch_features_dev(vs_batch* b, const vs_keypoint** d_kps, const float** d_desc, const int** d_n, int* frames);
/* Test support, host only (no device): vs_batch_step_dev's per-step record exchange
 * (csrc/batch_exchange.h — the ring halo, or the all-gather with gather != 0) run for `world` ranks in
 * one process over an in-memory transport, one thread per rank.  Inputs are [steps][world][B]
 * records (kps_in [..][cap], desc_in [..][cap][256], n_in); outputs slot 0 of every rank after
 * every step (slot0_kps [steps][world][cap], slot0_desc, slot0_n [steps][world]) and, with gather,
 * every rank's gathered tables (g_* [steps][world][world B] records).  world <= 64. */
int vs_batch_exchange_loopback(int world, int B, int cap, int steps, int gather, const vs_keypoint* kps_in,
                               const float* desc_in, const int* n_in, vs_keypoint* slot0_kps, float* slot0_desc,
                               int* slot0_n, vs_keypoint* g_kps, float* g_desc, int* g_n);

/* ---- F2: the SPCF feature cache as the batch interchange (FeatureExtractor.cpp:261-381) ---
 * Byte layout of the reference's save_cache / load_cache: u32 magic 0x53504346 ("SPCF"),
 * u32 version 1, u32 entry count, then per entry i32 frame_idx, i32 num_kp, num_kp x 28-B
 * keypoint records (x, y, size, angle, response f32, octave, class_id i32 == vs_keypoint),
 * i32 rows, cols, type (CV_32F = 5; 0, 0, 0 for an empty cv::Mat) and rows x cols fp32
 * descriptors.  The reference keys entries by the sequential extract-call index
 * (FeatureExtractor.cpp:52-61) and writes them sorted by it. */

/* Writes F frames (host buffers kps [F][cap], desc [F][cap][256], n [F]) as entries frame_idx[f].
 * append == 0 creates the file; append != 0 adds the entries to an existing file (header count
 * updated; a missing file is created).  A frame with n == 0 is written as the reference writes an
 * empty extraction (rows = cols = type = 0).  n[f] < 0 or > cap: VS_ERR_ARG. */
int vs_spcf_write(const char* path, int F, const int* frame_idx, const vs_keypoint* kps, const float* desc,
                  const int* n, int cap, int append);

/* The same from device buffers (vs_extract_batch_dev's outputs): copied on `stream`, then
 * written (synchronous). */
int vs_spcf_write_dev(vs_ctx* ctx, const char* path, int F, const int* frame_idx, const vs_keypoint* d_kps,
                      const float* d_desc, const int* d_n, int cap, int append, void* stream);

/* Reads an SPCF file.  *count = number of distinct frame indices (a repeated index keeps its last
 * entry, as the reference's map assignment does).  With non-null buffers (max_frames entries of
 * kps [cap], desc [cap][256]) the entries are returned sorted by frame index.  Bad magic / version,
 * a truncated file or a non-CV_32F / non-256-column descriptor matrix: VS_ERR_IO; more entries than
 * max_frames or keypoints than cap: VS_ERR_CAPACITY. */
int vs_spcf_read(const char* path, int max_frames, int cap, int* frame_idx, vs_keypoint* kps, float* desc, int* n,
                 int* count);

/* ---- F4: dense voxel fusion (main.cpp:1081-1146, dense_map.ply :1463-1474) -------------------
 * Every processed frame with real depth is back-projected on a pixel_step grid with its pose at
 * processing time; a point joins the cloud the first time its voxel (floor(p / voxel_size) per
 * axis) is seen, in the reference's insertion order (frame, then row-major grid).  The cloud lives
 * in HBM (a voxel hash table of 2^table_log2 slots plus max_points x 3 fp64).  Voxel coordinates
 * within [-2^20, 2^20) (+-20 km at 2 cm) are keyed exactly, farther ones (a diverged pose) by a
 * 63-bit hash of the three ints; a full table or more than max_points points: vs_dense_size
 * reports VS_ERR_CAPACITY.  vs_dense_write_ply writes no file for an empty cloud. */
typedef struct vs_dense vs_dense;
typedef struct vs_dense_config {
    int pixel_step;     /* Config::DENSE_PIXEL_STEP (8) */
    double max_depth;   /* Config::DENSE_MAX_DEPTH (5.0 m) */
    double voxel_size;  /* Config::DENSE_VOXEL_SIZE (0.02 m) */
    double fx, fy, cx, cy;
    double origin[3];   /* main.cpp's origin_offset (0, 0, 0) */
    int table_log2;     /* hash table slots (default 24) */
    long long max_points; /* cloud capacity (default 8 Mi points) */
} vs_dense_config;
void vs_dense_default_config(vs_dense_config* cfg);
/* cfg NULL = the reference's Config values. */
int vs_dense_create(vs_ctx* ctx, const vs_dense_config* cfg, vs_dense** out);
void vs_dense_destroy(vs_dense* d);
int vs_dense_reset(vs_dense* d, void* stream);
/* nf frames in insertion order: d_depth[f] a device h x w fp32 depth map (metres), R (nf x 9,
 * camera -> world, row-major) and t (nf x 3) on the host.  Enqueue only. */
int vs_dense_integrate_dev(vs_dense* d, int nf, const float* const* d_depth, int h, int w, const double* R,
                           const double* t, void* stream);
/* Synchronises with the last integrate; *n = points in the cloud. */
int vs_dense_size(vs_dense* d, long long* n);
/* The first min(cap, n) points (x, y, z fp64) to host memory; *n = points in the cloud. */
int vs_dense_points(vs_dense* d, long long cap, double* xyz, long long* n);
/* The cloud in HBM ([max_points][3] fp64; valid after vs_dense_size). */
const double* vs_dense_points_dev(vs_dense* d);
/* dense_map.ply as main.cpp:1463-1474 writes it (ascii, 6 decimals). */
int vs_dense_write_ply(vs_dense* d, const char* path);
/* Attach a dense cloud to a tracker: every frame vs_slam_process_batch_dev / _features reports as
 * processed and that has depth is integrated with its pose right after Slam::process_frame, as the
 * reference's main loop does (NULL detaches). */
int vs_slam_attach_dense(vs_slam* slam, vs_dense* d);

/* ---- F4: Optimizer::pose_graph_optimize (Optimizer.cpp:654-863), g2o LM restated -------------
 * N keyframe poses (camera -> world, R [N][9] row-major, t [N][3], keyframe order; the first is
 * fixed), odometry edges between consecutive keyframes from these poses, L loop constraints
 * (vertex indices lc_from / lc_to, measurement R_rel [L][9] / t_rel [L][3], sigmas [L][2] =
 * {trans, rot}), and, when gravity is non-NULL, a height prior g . t = height on every vertex.
 * Nothing happens for N < 3, or with no loops and no prior (as the reference returns 0).
 * R / t are overwritten with the optimised poses.  stats (nullable) = {iterations, accepted steps,
 * trials, loop edges}; chi2 (nullable) = {before, after, final lambda}.  Synchronous. */
int vs_pose_graph_optimize(vs_ctx* ctx, int N, double* R, double* t, int L, const int* lc_from, const int* lc_to,
                           const double* lc_R, const double* lc_t, const double* lc_sigma, const double* gravity,
                           double height, int iterations, int stats[4], double chi2[3]);
/* Optimizer.cpp:829-859: map point i moves with keyframe kf[i] (-1: unchanged) by
 * new_k * old_k^-1; pos [M][3] in place.  Synchronous. */
int vs_pgo_transform_points(vs_ctx* ctx, int N, const double* R_old, const double* t_old, const double* R_new,
                            const double* t_new, int M, const int* kf, double* pos);
/* Slam::run_posthoc_pgo (Slam.cpp:1748-1755): the pose graph over the tracker's keyframes with its
 * loop constraints and height prior, then the non-keyframe translations and map points corrected
 * as Optimizer.cpp:780-859 does.  *loop_edges = pose_graph_optimize's return value. */
int vs_slam_run_posthoc_pgo(vs_slam* slam, int* loop_edges);

/* ---- NMS tie accounting (FeatureExtractor.cpp:238-259: std::sort, unstable) ------------------
 * Every post-processed frame on this context (vs_extract*, vs_postprocess*, a vs_slam's batches)
 * adds to five totals: out = {frames, frames with a tie, window ties (output keypoints with an
 * equal-score candidate inside their 9x9 window), cut ties (the 400th and 401st kept pixel score
 * the same), order ties (output keypoints sharing their score with another output keypoint)}.
 * Without window and cut ties the keypoint set is the reference's for any order of equal scores,
 * std::sort's included; without order ties also their order in the list.  The build breaks ties
 * by raster index.  reset != 0 zeroes the totals.  Synchronises the device. */
int vs_nms_tie_stats(vs_ctx* ctx, long long out[5], int reset);

/* ---- profiling ----------------------------------------------------------------------- */
/* When enabled, every stage of the _dev pipelines brackets its launches with hipEvents on the
 * stream it runs on; vs_profile_read returns per-stage accumulated milliseconds and launch
 * counts since the last reset.  Stage names are static strings.  on: 0 off, 1 every stage,
 * 2 the extraction stages only (network, post-processing, MiDaS: a tracker's host loop then runs
 * without per-stage event records). */
int vs_profile_enable(vs_ctx* ctx, int on);
int vs_profile_reset(vs_ctx* ctx);
int vs_profile_read(vs_ctx* ctx, int max_stages, const char** names, double* ms, int* launches,
                    int* n_stages);

/* ---- test support -------------------------------------------------------------------- */
/* The device's correctly rounded fp64 functions (csrc/cr_math.h, used by Rodrigues, the 7-point
 * cubic and RANSACUpdateNumIters) on n host inputs: op 0 sin(a), 1 cos(a), 2 acos(a), 3 log(a),
 * 4 pow(a, b) (b may be NULL for ops 0-3).  Synchronous; out has n entries. */
int vs_selftest_crmath(vs_ctx* ctx, int op, int n, const double* a, const double* b, double* out);

#ifdef __cplusplus
}
#endif
#endif /* VSLAM_ABI_H */
