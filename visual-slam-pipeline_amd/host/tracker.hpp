// tracker.hpp — host restatement of the reference's per-frame tracking loop, Slam::process_frame
// (reference src/Slam.cpp:809-1135) and the Slam helpers it calls, written once as a template over
// a compute back end `Ops`:
//
//   vs_trk::Tracker<GpuOps>     libvslam_hip.so (csrc/tracker.hip): every arithmetic stage is a
//                               HIP kernel behind the C ABI; this file is only the control flow.
//   vs_trk::Tracker<OracleOps>  oracle/liboracle.so (orc_slam.cpp), TEST INFRASTRUCTURE: the same
//                               control flow over the CPU restatements, so a trajectory computed on
//                               the GPU can be compared with one computed on the CPU stage by stage.
//
// What stays on the host (sequential, tiny fp64 logic around the kernels):
// the EKF (Slam.cpp:986-1047, 1654-1744), the keyframe policy (:1062-1129, 1359-1368), DLT
// triangulation (:1246-1356), depth back-projection (:1526-1577), map point culling (:473-500,
// 1110-1126), stationary / gravity handling (:615-694, 1579-1651) and the RTS smoother
// (:1761-1810).  What the back end does: the fused match -> F verification -> 3D-3D -> E-matrix
// chain (:838-984), matching for bridge / keyframe setup (:847-872, 699-705), PnP recovery
// matching against the map (:546-575), local-map tracking (:380-469), PnP (:505-529) and the
// O(map points x keypoints) visibility sweep (:1089-1108).
//
// Loop closure (F4: Slam::handle_loop_closure :730-798 with LoopCloser::detect, LoopCloser.cpp:16-100,
// every LC_CHECK_INTERVAL keyframes, :1084-1086) records loop edges and PGO constraints; like the
// reference it never changes a pose (run_posthoc_pgo has no caller).  Its back-end op evaluates every
// candidate keyframe at once (one batched match + E-RANSAC).  Keyframes keep their features for it.
// Deliberate omissions: local BA is disabled in the reference (Config.h:99).  The
// ORB fallback is out of scope.
#pragma once

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>

#include "../csrc/pnp_solvers.h"  // rod_v2m / rod_m2v / sym_eig: the shared host/device numerics

namespace vs_trk {

// ---- Config.h ------------------------------------------------------------------------------
namespace cfg {
constexpr int IMAGE_WIDTH = 640, IMAGE_HEIGHT = 480;
constexpr double FX = 525.0, FY = 525.0, CX = 319.5, CY = 239.5;
constexpr float DEPTH_MIN = 0.1f, DEPTH_MAX = 10.0f;
constexpr float L2_RATIO_THRESHOLD = 0.75f, FLANN_RATIO_THRESHOLD = 0.7f;
constexpr int MIN_MATCHES = 30;
constexpr double TRIANG_MAX_REPROJ_ERROR = 3.0, TRIANG_MIN_DEPTH = 0.05, TRIANG_MAX_DEPTH = 50.0,
                 TRIANG_MAX_CAM_DIST = 5.0;
constexpr int PNP_INTERVAL = 5, PNP_MIN_POINTS = 10;
constexpr double PNP_RECOVERY_MAX_JUMP = 1.5, PNP_RECOVERY_BLEND_CLOSE = 0.8, PNP_RECOVERY_BLEND_FAR = 0.3,
                 PNP_REFINE_MAX_JUMP = 1.0, PNP_PERIODIC_MAX_JUMP = 1.5, PNP_PERIODIC_BLEND = 0.5;
constexpr int KF_MIN_FRAME_GAP = 10, KF_MIN_MATCHES = 50;
constexpr double TRACK_VISIBILITY_RADIUS = 8.0;
constexpr float CULL_FOUND_RATIO_YOUNG = 0.15f, CULL_FOUND_RATIO_OLD = 0.30f;
constexpr double MOTION_SCALE = 0.05;
constexpr int LC_MIN_FRAME_GAP = 200, LC_MIN_INLIERS = 30, LC_CHECK_INTERVAL = 200, LC_NEARBY_FRAME_RANGE = 30;
constexpr double LC_MAX_JUMP = 0.5, LC_MIN_JUMP = 0.01, PGO_LC_TRANS_SIGMA = 0.03, PGO_LC_ROT_SIGMA = 0.01;
constexpr double EKF_SIGMA_VIS_3D3D = 0.04, EKF_SIGMA_VIS_EMAT = 0.10, EKF_SIGMA_HEIGHT = 0.01,
                 EKF_PROCESS_ACCEL = 1.0, EKF_VEL_DECAY = 0.95, EKF_INNOV_GATE = 0.3, EKF_MAX_STEP = 0.10;
}  // namespace cfg

// ---- types -----------------------------------------------------------------------------------
struct Keypoint {  // == cv::KeyPoint == vs_keypoint
    float x, y, size, angle, response;
    int32_t octave, class_id;
};
struct Match {  // == cv::DMatch == vs_match
    int32_t query_idx, train_idx, img_idx;
    float distance;
};
using M3 = std::array<double, 9>;  // row-major CV_64F 3x3
using V3 = std::array<double, 3>;

inline M3 eye3() { return {1, 0, 0, 0, 1, 0, 0, 0, 1}; }
inline M3 mul(const M3& A, const M3& B) {
    M3 C{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
    return C;
}
inline M3 mul_bt(const M3& A, const M3& B) {  // A * B^T
    M3 C{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            C[i * 3 + j] = A[i * 3] * B[j * 3] + A[i * 3 + 1] * B[j * 3 + 1] + A[i * 3 + 2] * B[j * 3 + 2];
    return C;
}
inline M3 tr(const M3& A) { return {A[0], A[3], A[6], A[1], A[4], A[7], A[2], A[5], A[8]}; }
inline V3 mulv(const M3& A, const V3& v) {
    return {A[0] * v[0] + A[1] * v[1] + A[2] * v[2], A[3] * v[0] + A[4] * v[1] + A[5] * v[2],
            A[6] * v[0] + A[7] * v[1] + A[8] * v[2]};
}
inline double norm3(const V3& v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// Frame (Frame.h:12-72): features, depth, camera->world pose, keyframe flag, map point indices.
struct Frame {
    int id = -1;
    double timestamp = 0.0;
    std::vector<Keypoint> kps;
    std::vector<float> desc;           // n x 256 host copy (back ends that keep device copies may leave it empty)
    const float* depth = nullptr;      // h x w metres, 0 = invalid (Frame::load_depth_image); nullptr = none
    std::vector<float> depth_store;    // owned copy once the caller's buffer may go away
    int dh = 0, dw = 0;
    M3 R = eye3();
    V3 t{0, 0, 0};
    bool keyframe = false;
    std::vector<int> mp_idx;           // Frame::map_point_indices
    int slot = -1;                     // back-end handle (device feature / depth slot)
    int kf_slot = -1;                  // back-end handle of a keyframe's archived features (loop closure)
    bool has_depth() const { return depth != nullptr; }
    bool has_desc() const { return !kps.empty(); }  // descriptors are empty iff there are no keypoints
    float depth_at(int py, int px) const { return depth[(size_t)py * dw + px]; }
    void own_depth() {
        if (depth && depth != depth_store.data()) {
            depth_store.assign(depth, depth + (size_t)dh * dw);
            depth = depth_store.data();
        }
    }
};
using FramePtr = std::shared_ptr<Frame>;

// Map (Map.h:10-40) with its MapPoints (MapPoint.h:8-48) as structure-of-arrays; descriptors are
// owned by the back end (device rows for the GPU, host rows for the oracle).
struct Map {
    std::vector<FramePtr> frames;       // insertion order (Map::add_frame)
    std::vector<double> pos;            // 3 per point, world
    std::vector<uint8_t> valid;         // MapPoint::is_valid (all points have descriptors)
    std::vector<int> visible, found, first_kf;
    std::vector<std::vector<std::pair<int, int>>> obs;  // (frame id, keypoint index)
    int size() const { return (int)valid.size(); }
    int add(const double p[3], int first_kf_id) {
        pos.insert(pos.end(), p, p + 3);
        valid.push_back(1);
        visible.push_back(0);
        found.push_back(0);
        first_kf.push_back(first_kf_id);
        obs.emplace_back();
        return size() - 1;
    }
    float found_ratio(int i) const { return visible[i] > 0 ? (float)found[i] / visible[i] : 0.0f; }
};

// Result of the back end's fused front chain for one (reference, current) pair:
// match_features (:841) -> findFundamentalMat + ordered filtering (:880-910) ->
// estimate_motion_3d3d on the kept points (:955) -> estimate_motion + estimate_scale_from_depth
// when 3D-3D fails (:965-984).
struct ChainResult {
    std::vector<Match> good;  // ratio-test matches, query order
    int n_raw = 0;
    bool f_ok = false;
    std::vector<Match> kept;  // good filtered by the F inlier mask (== good when F is empty)
    double epi_before = 0, epi_after = 0;
    bool ok3d = false;
    M3 R3{};
    V3 t3{};
    bool okE = false;
    M3 RE{};
    V3 tE{};
    double scale = -1.0;
    int f_iters = 0;  // F-RANSAC iterations run (findFundamentalMat's registrator)
};

struct PnPResult {  // Slam::PnPResult
    bool success = false;
    M3 R_world{};
    V3 t_world{};
    int inlier_count = 0;
};

// Slam.h LoopConstraint (PGO edge from a verified loop, Slam.cpp:788-797)
struct LoopConstraint {
    int from_id = -1, to_id = -1;
    M3 R_rel{};
    V3 t_rel{};
    double trans_sigma = 0, rot_sigma = 0;
};

// A loop constraint as the pose graph takes it: keyframe indices instead of frame ids
struct PgoLoop {
    int from = -1, to = -1;
    M3 R{};
    V3 t{};
    double trans_sigma = 0, rot_sigma = 0;
};

// One loop-closure candidate as LoopCloser::detect sees it (LoopCloser.cpp:50-76): ratio-test
// matches of the current frame against the keyframe, and the inliers of findEssentialMat on them
// (0 when E is empty).
struct LoopEval {
    int n_good = 0, inliers = 0;
};

struct AccelSample {
    double timestamp, ax, ay, az;
};

struct Stats {
    int processed = 0, rejected = 0, via_3d3d = 0, via_emat = 0, emat_failed = 0, bridges = 0, recoveries = 0,
        recovery_failed = 0, stationary = 0, keyframes = 0, pnp_refined = 0, periodic_pnp = 0, tracked_total = 0,
        triangulated = 0, depth_points = 0, culled = 0, chains_discarded = 0, f_iters = 0;
};

// Optional host wall time per phase of process_frame (a profiling aid: off unless a back end
// turns it on; the phases include their back-end calls).
enum Phase { PH_CHAIN, PH_RECOVERY, PH_MOTION_EKF, PH_TLM, PH_REFINE, PH_KEYFRAME, PH_N };
inline const char* phase_name(int k) {
    static const char* const n[PH_N] = {"chain + bridge", "recovery check", "stationary + motion + EKF",
                                        "local-map tracking", "PnP refinement", "keyframe work"};
    return n[k];
}
struct PhaseProf {
    bool on = false;
    double ms[PH_N] = {};
    long n[PH_N] = {};
};
struct PhaseScope {
    PhaseProf& p;
    int k;
    std::chrono::steady_clock::time_point t0;
    PhaseScope(PhaseProf& pp, int kk) : p(pp), k(kk) {
        if (p.on) t0 = std::chrono::steady_clock::now();
    }
    void end() {
        if (k < 0) return;
        if (p.on) {
            p.ms[k] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            p.n[k]++;
        }
        k = -1;
    }
    ~PhaseScope() { end(); }
};

// ---- the tracker -----------------------------------------------------------------------------
template <class Ops>
class Tracker {
   public:
    explicit Tracker(Ops& ops) : ops_(ops) {}

    void set_initial_pose(const M3& R, const V3& t) {  // Slam.cpp:35-38
        R_world_ = R;
        t_world_ = t;
    }
    void set_accelerometer_data(std::vector<AccelSample> d) { accel_ = std::move(d); }  // :1580-1582
    // Debugging aid: one line per stage result (hex floats) so that two back ends' runs can be
    // diffed to the first differing stage (tools/debug_tracker_divergence.py --trace).
    void set_trace(FILE* f) { trace_ = f; }
    PhaseProf& phase_prof() { return phase_; }

    // Slam::compute_gravity_direction (Slam.cpp:1587-1616)
    void compute_gravity_direction() {
        if (accel_.empty()) return;
        double ax = 0, ay = 0, az = 0;
        for (const auto& s : accel_) ax += s.ax, ay += s.ay, az += s.az;
        const int n = (int)accel_.size();
        V3 g = mulv(R_world_, V3{ax / n, ay / n, az / n});
        const double nrm = norm3(g);
        if (nrm > 1e-6)
            for (double& v : g) v /= nrm;
        int max_axis = 0;
        double max_val = 0;
        for (int i = 0; i < 3; i++)
            if (std::abs(g[i]) > max_val) max_val = std::abs(g[i]), max_axis = i;
        const double sign = g[max_axis] > 0 ? 1.0 : -1.0;
        gravity_ = V3{0, 0, 0};
        gravity_[max_axis] = sign;
        has_gravity_ = true;
        initial_height_ = t_world_[0] * gravity_[0] + t_world_[1] * gravity_[1] + t_world_[2] * gravity_[2];
        has_initial_height_ = true;
    }

    // Slam::process_frame (Slam.cpp:809-1135), from the point where the frame's features exist
    // (Frame::detect_features has run: kps / descriptors / mp_idx = -1).
    bool process_frame(const FramePtr& frame) {
        if (!frame) return false;
        last_pnp_ = false;
        last_loop_ = false;  // :813
        if ((int)frame->kps.size() < cfg::MIN_MATCHES) {  // :820-823
            last_frame_ = frame;
            stats_.rejected++;
            return false;
        }
        if (!last_frame_) {  // :826-835 first frame
            frame->R = R_world_;
            frame->t = t_world_;
            frame->keyframe = true;
            map_.frames.push_back(frame);
            last_frame_ = frame;
            last_keyframe_ = frame;
            keyframe_count_++;
            frame_count_++;
            stats_.processed++;
            stats_.keyframes++;
            return true;
        }
        // :838 reference frame; the whole front chain runs speculatively on the back end — its
        // match list is what :841 computes, and the F / 3D-3D / E results are only used when the
        // control flow reaches :880 with these matches
        ref_frame_ = (last_keyframe_ && last_keyframe_->has_desc()) ? last_keyframe_ : last_frame_;
        PhaseScope ph_chain(phase_, PH_CHAIN);
        ChainResult C = ops_.chain(*ref_frame_, *frame, 42u + (uint32_t)frame_count_);
        stats_.f_iters += C.f_iters;
        last_match_count_ = (int)C.good.size();
        trace_chain(frame->id, C);

        // :847-872 bridge keyframe when keyframe matching is weak
        if (last_match_count_ < cfg::MIN_MATCHES && last_frame_ && last_frame_ != ref_frame_) {
            auto temp = ops_.match(*last_frame_, *frame, cfg::L2_RATIO_THRESHOLD);
            if ((int)temp.size() >= cfg::MIN_MATCHES) {
                if (!last_frame_->keyframe) {
                    last_frame_->keyframe = true;
                    keyframe_count_++;
                    stats_.keyframes++;
                    stats_.bridges++;
                    if (last_keyframe_) {
                        match_and_triangulate(last_keyframe_, last_frame_);
                    }
                    create_points_from_depth(last_frame_);
                    last_keyframe_ = last_frame_;
                }
                ref_frame_ = last_keyframe_;
                C = ops_.chain(*ref_frame_, *frame, 42u + (uint32_t)frame_count_);
                stats_.f_iters += C.f_iters;
                last_match_count_ = (int)C.good.size();
            }
        }

        ph_chain.end();
        // :875-877 PnP recovery when tracking is lost
        PhaseScope ph_rec(phase_, PH_RECOVERY);
        const int pnp_result = try_pnp_recovery(frame);
        ph_rec.end();
        if (pnp_result == 1) return true;
        if (pnp_result == -1) {
            stats_.recovery_failed++;
            return false;
        }

        // :880-910 geometric verification (the chain's F stage on exactly these matches)
        if (C.f_ok) {
            epipolar_error_before_ = C.epi_before;
            if (!C.kept.empty()) epipolar_error_after_ = C.epi_after;
        }
        std::vector<Match> good = C.kept;

        PhaseScope ph_mot(phase_, PH_MOTION_EKF);
        if (process_stationary_frame(frame, good)) return true;  // :913

        bool recompute_motion = false;
        std::vector<float> p1, p2;
        if (was_stationary_ && last_frame_) {  // :916-951 post-stationary transition
            was_stationary_ = false;
            if (!last_frame_->keyframe) {
                last_frame_->keyframe = true;
                keyframe_count_++;
                stats_.keyframes++;
                create_points_from_depth(last_frame_);
                last_keyframe_ = last_frame_;
            }
            ref_frame_ = last_keyframe_;
            good = ops_.match(*ref_frame_, *frame, cfg::L2_RATIO_THRESHOLD);
            last_match_count_ = (int)good.size();
            points_of(*ref_frame_, *frame, good, p1, p2);
            if (good.size() >= 8) {
                std::vector<uint8_t> mask;
                if (ops_.find_fundamental(p1, p2, mask)) {
                    std::vector<Match> kept;
                    std::vector<float> q1, q2;
                    for (size_t i = 0; i < good.size(); i++)
                        if (mask[i]) {
                            kept.push_back(good[i]);
                            q1.insert(q1.end(), {p1[2 * i], p1[2 * i + 1]});
                            q2.insert(q2.end(), {p2[2 * i], p2[2 * i + 1]});
                        }
                    good.swap(kept);
                    p1.swap(q1);
                    p2.swap(q2);
                }
            }
            recompute_motion = true;
        }

        // :953-984 motion: 3D-3D preferred, essential matrix + depth scale as fallback
        if (recompute_motion) {
            stats_.chains_discarded++;
            C = ops_.motion_points(*ref_frame_, *frame, p1, p2, 42u + (uint32_t)frame_count_);
        }
        if (recompute_motion) trace_chain(frame->id, C);
        const bool use_3d3d = C.ok3d;
        const M3 R_ref = ref_frame_->R;
        const V3 t_ref = ref_frame_->t;
        M3 R_new;
        V3 t_new;
        if (use_3d3d) {
            R_new = mul_bt(R_ref, C.R3);
            const V3 m = mulv(R_new, C.t3);
            t_new = {t_ref[0] - m[0], t_ref[1] - m[1], t_ref[2] - m[2]};
            stats_.via_3d3d++;
        } else {
            if (!C.okE) {
                last_frame_ = frame;
                stats_.emat_failed++;
                return false;
            }
            double scale = C.scale;
            if (scale <= 0) {
                scale = (last_good_scale_ > 0) ? last_good_scale_ : cfg::MOTION_SCALE;
            } else {
                last_good_scale_ = scale;
            }
            R_new = mul_bt(R_ref, C.RE);
            const V3 st{scale * C.tE[0], scale * C.tE[1], scale * C.tE[2]};
            const V3 m = mulv(R_new, st);
            t_new = {t_ref[0] - m[0], t_ref[1] - m[1], t_ref[2] - m[2]};
            stats_.via_emat++;
        }

        // :986-1047 EKF predict + update
        {
            Snapshot snap;
            const double ekf_dt = ekf_fuse(t_new, use_3d3d, frame->timestamp, &snap);
            V3 ekf_pos{x_[0], x_[1], x_[2]};
            V3 delta{ekf_pos[0] - t_world_[0], ekf_pos[1] - t_world_[1], ekf_pos[2] - t_world_[2]};
            const double step = norm3(delta);
            if (step > cfg::EKF_MAX_STEP && step > 1e-6) {  // :1026-1033 step clamp
                for (double& v : delta) v = v * (cfg::EKF_MAX_STEP / step);
                for (int i = 0; i < 3; i++) ekf_pos[i] = t_world_[i] + delta[i];
                for (int i = 0; i < 3; i++) x_[i] = ekf_pos[i];
                const double dt_frame = std::max(0.01, frame->timestamp - last_frame_time_);
                for (int i = 0; i < 3; i++) x_[i + 3] = delta[i] / dt_frame;
            }
            t_new = ekf_pos;
            std::memcpy(snap.x_filt, x_, sizeof(x_));
            snap.dt = ekf_dt;
            snap.frame_index = (int)map_.frames.size();
            snapshots_.push_back(snap);
        }
        last_frame_time_ = frame->timestamp;
        R_world_ = R_new;
        t_world_ = t_new;
        frame->R = R_world_;
        frame->t = t_world_;
        map_.frames.push_back(frame);
        trace_pose(frame->id, "motion+ekf", R_world_, t_world_);

        ph_mot.end();
        // :1057-1059 local map tracking + PnP refinement
        PhaseScope ph_tlm(phase_, PH_TLM);
        const int tracked = track_local_map(frame);
        ph_tlm.end();
        if (trace_)
            std::fprintf(trace_, "%d tlm %d %016llx\n", frame->id, tracked,
                         (unsigned long long)fnv(frame->mp_idx.data(), frame->mp_idx.size() * sizeof(int)));
        PhaseScope ph_ref(phase_, PH_REFINE);
        refine_pose_via_local_pnp(frame, tracked);
        ph_ref.end();
        trace_pose(frame->id, "refined", R_world_, t_world_);
        PhaseScope ph_kf(phase_, PH_KEYFRAME);

        // :1061-1070 proactive keyframe.  Deviation: the reference dereferences last_keyframe_
        // unconditionally here, which is null when the first frame was rejected (:820-823 keeps it
        // as last_frame_, so :826 never initialises a keyframe); with no keyframe the regular rule
        // below (:1360) makes this frame one, so skipping the check is the only defined reading.
        if (!frame->keyframe && last_keyframe_ && last_match_count_ < cfg::MIN_MATCHES * 2) {
            const int frames_since_kf = frame->id - last_keyframe_->id;
            if (frames_since_kf >= 5) {
                frame->keyframe = true;
                keyframe_count_++;
                stats_.keyframes++;
                setup_new_keyframe(frame);
                last_keyframe_ = frame;
            }
        }
        // :1072-1129 regular keyframe
        if (is_keyframe(frame, last_match_count_)) {
            frame->keyframe = true;
            keyframe_count_++;
            stats_.keyframes++;
            setup_new_keyframe(frame);
            if (keyframe_count_ % cfg::PNP_INTERVAL == 0) run_pnp(frame);
            if (keyframe_count_ % cfg::LC_CHECK_INTERVAL == 0) handle_loop_closure(frame);  // :1084-1086
            visibility_sweep(frame);  // :1088-1108
            if (keyframe_count_ % 3 == 0) cull_by_found_ratio();  // :1110-1126
            last_keyframe_ = frame;
        }
        last_frame_ = frame;
        frame_count_++;
        stats_.processed++;
        return true;
    }

    // Round 6 (back-end speculation, no state change): the pose the NEXT frame `nxt` will get at
    // Slam.cpp:953-1047 from its front-chain result C (match -> F -> 3D-3D / E against `ref`), computed
    // now, while `cur`'s local-map tracking runs.  Only where the plain path is certain: `cur` (the
    // frame being processed, past its motion and EKF step) does not become a keyframe (:1061-1072 decide
    // that from its match count and id gap, already known), `nxt` has enough keypoints and matches that
    // no bridge (:847), recovery (:875) or stationary branch (:913-951) can run, and the EKF runs.  The
    // pose is the EKF position before the step clamp (:1026-1033), which depends on `cur`'s refined
    // pose: the back end checks the prediction bit for bit against the pose process_frame then sets,
    // so a clamped (or otherwise different) step only costs the speculation.  ref_out: the frame the
    // next chain must have matched against.
    // cur_only: only the conditions on `cur` (nxt and C unused).
    bool predict_next_pose(const Frame& cur, const Frame& nxt, const ChainResult& C, const Frame** ref_out, M3& R,
                           V3& t, bool cur_only = false) {
        if (cur.keyframe || !last_keyframe_ || !ekf_init_) return false;
        if (!accel_.empty() || was_stationary_) return false;
        if (last_match_count_ < cfg::MIN_MATCHES * 2 && cur.id - last_keyframe_->id >= 5) return false;  // proactive kf
        if (cur.id - last_keyframe_->id >= cfg::KF_MIN_FRAME_GAP && last_match_count_ >= cfg::KF_MIN_MATCHES)
            return false;  // regular keyframe (is_keyframe with a last keyframe)
        if (cur_only) return true;
        if ((int)nxt.kps.size() < cfg::MIN_MATCHES || (int)C.good.size() < cfg::MIN_MATCHES) return false;
        if (!C.ok3d && !C.okE) return false;
        const Frame* ref = last_keyframe_->has_desc() ? last_keyframe_.get() : &cur;
        M3 R_new;
        V3 t_new;
        if (C.ok3d) {
            R_new = mul_bt(ref->R, C.R3);
            const V3 m = mulv(R_new, C.t3);
            t_new = {ref->t[0] - m[0], ref->t[1] - m[1], ref->t[2] - m[2]};
        } else {
            const double scale = C.scale > 0 ? C.scale : (last_good_scale_ > 0 ? last_good_scale_ : cfg::MOTION_SCALE);
            R_new = mul_bt(ref->R, C.RE);
            const V3 st{scale * C.tE[0], scale * C.tE[1], scale * C.tE[2]};
            const V3 m = mulv(R_new, st);
            t_new = {ref->t[0] - m[0], ref->t[1] - m[1], ref->t[2] - m[2]};
        }
        double x0[6], P0[36];
        std::memcpy(x0, x_, sizeof(x_));
        std::memcpy(P0, P_, sizeof(P_));
        const double lft = last_frame_time_;
        ekf_fuse(t_new, C.ok3d, nxt.timestamp, nullptr);
        t = V3{x_[0], x_[1], x_[2]};
        std::memcpy(x_, x0, sizeof(x_));
        std::memcpy(P_, P0, sizeof(P_));
        last_frame_time_ = lft;
        R = R_new;
        *ref_out = ref;
        return true;
    }

    // Slam::run_posthoc_pgo (Slam.cpp:1748-1755) -> Optimizer::pose_graph_optimize (Optimizer.cpp:654-863):
    // the back end optimises the keyframe graph (g2o LM, 20 iterations) and moves the map points;
    // the keyframe / non-keyframe pose bookkeeping (:789-827) is restated here.  Returns the number
    // of loop edges added.
    int run_posthoc_pgo() {
        if (!has_initial_height_ && loop_constraints_.empty()) return 0;  // :1749-1751
        const bool prior = has_initial_height_ && has_gravity_;          // has_height_prior && !gravity.empty()
        std::vector<Frame*> kfs;
        for (const FramePtr& f : map_.frames)
            if (f->keyframe) kfs.push_back(f.get());
        const int N = (int)kfs.size();
        if (N < 3) return 0;  // :670
        auto kf_index = [&](int id) {
            for (int i = 0; i < N; i++)
                if (kfs[i]->id == id) return i;
            return -1;
        };
        std::vector<PgoLoop> loops;
        for (const LoopConstraint& c : loop_constraints_) {  // :723-755
            const int a = kf_index(c.from_id), b = kf_index(c.to_id);
            if (a < 0 || b < 0) continue;
            loops.push_back({a, b, c.R_rel, c.t_rel, c.trans_sigma, c.rot_sigma});
        }
        if (loops.empty() && !prior) return 0;  // :775
        std::vector<M3> R_old(N), R_new(N);
        std::vector<V3> t_old(N), t_new(N);
        for (int i = 0; i < N; i++) {
            R_old[i] = R_new[i] = kfs[i]->R;
            t_old[i] = t_new[i] = kfs[i]->t;
        }
        ops_.pose_graph(R_new, t_new, loops, prior ? &gravity_ : nullptr, initial_height_, 20);  // :777-778
        for (int i = 0; i < N; i++) {  // :789-793
            kfs[i]->R = R_new[i];
            kfs[i]->t = t_new[i];
        }
        for (const FramePtr& f : map_.frames) {  // :795-827 non-keyframes: interpolated translation shift
            if (f->keyframe) continue;
            const int fid = f->id;
            int prev = -1, next = -1;
            for (int i = 0; i < N; i++) {
                if (kfs[i]->id <= fid) prev = i;
                if (kfs[i]->id > fid && next < 0) next = i;
            }
            if (prev < 0) continue;
            if (next < 0) next = prev;
            double alpha = 0.0;
            if (prev != next) alpha = (double)(fid - kfs[prev]->id) / (double)(kfs[next]->id - kfs[prev]->id);
            for (int k = 0; k < 3; k++) {
                const double dp = t_new[prev][k] - t_old[prev][k], dn = t_new[next][k] - t_old[next][k];
                f->t[k] += (1.0 - alpha) * dp + alpha * dn;
            }
        }
        std::vector<int> pkf(map_.size(), -1);  // :829-851 each valid point's keyframe
        for (int i = 0; i < map_.size(); i++) {
            if (!map_.valid[i] || map_.obs[i].empty()) continue;
            const int ofid = map_.obs[i][0].first;
            int k = kf_index(ofid);
            if (k < 0) {
                int best = 1 << 30;
                for (int q = 0; q < N; q++) {
                    const int d = std::abs(kfs[q]->id - ofid);
                    if (d < best) best = d, k = q;
                }
            }
            pkf[i] = k;
        }
        ops_.pgo_points(R_old, t_old, R_new, t_new, pkf, map_);  // :852-858
        return (int)loops.size();
    }

    // Slam::run_rts_smoother (Slam.cpp:1761-1810)
    void run_rts_smoother() {
        const int N = (int)snapshots_.size();
        if (N < 3) return;
        const double decay = cfg::EKF_VEL_DECAY;
        std::vector<std::array<double, 6>> xs(N);
        std::vector<std::array<double, 36>> Ps(N);
        std::memcpy(xs[N - 1].data(), snapshots_[N - 1].x_filt, sizeof(double) * 6);
        std::memcpy(Ps[N - 1].data(), snapshots_[N - 1].P_filt, sizeof(double) * 36);
        for (int k = N - 2; k >= 0; k--) {
            const double dt = snapshots_[k + 1].dt;
            double F[36];
            transition(dt, decay, F);
            double Pinv[36];
            pinv6(snapshots_[k + 1].P_pred, Pinv);
            double PFt[36], C[36];
            mm6(snapshots_[k].P_filt, F, PFt, false, true);
            mm6(PFt, Pinv, C, false, false);
            double dx[6];
            for (int i = 0; i < 6; i++) dx[i] = xs[k + 1][i] - snapshots_[k + 1].x_pred[i];
            for (int i = 0; i < 6; i++) {
                double s = 0;
                for (int j = 0; j < 6; j++) s += C[i * 6 + j] * dx[j];
                xs[k][i] = snapshots_[k].x_filt[i] + s;
            }
            double dP[36], CdP[36], CdPCt[36];
            for (int i = 0; i < 36; i++) dP[i] = Ps[k + 1][i] - snapshots_[k + 1].P_pred[i];
            mm6(C, dP, CdP, false, false);
            mm6(CdP, C, CdPCt, false, true);
            for (int i = 0; i < 36; i++) Ps[k][i] = snapshots_[k].P_filt[i] + CdPCt[i];
        }
        for (int k = 0; k < N; k++) {
            const int fid = snapshots_[k].frame_index;
            if (fid >= 0 && fid < (int)map_.frames.size()) map_.frames[fid]->t = {xs[k][0], xs[k][1], xs[k][2]};
        }
    }

    // Frames that outlive the current call (reference / last frames) must own their depth.
    void retain_live_frames() {
        for (const FramePtr& f : {last_frame_, last_keyframe_, ref_frame_})
            if (f) f->own_depth();
    }
    // Frames whose back-end resources may be released (no longer the last / reference frames).
    bool is_live(const Frame* f) const {
        return f == last_frame_.get() || f == last_keyframe_.get() || f == ref_frame_.get();
    }

    Map& map() { return map_; }
    const Map& map() const { return map_; }
    const Stats& stats() const { return stats_; }
    int frame_count() const { return frame_count_; }
    int keyframe_count() const { return keyframe_count_; }
    int last_match_count() const { return last_match_count_; }
    const M3& R_world() const { return R_world_; }
    const V3& t_world() const { return t_world_; }
    double epipolar_error_before() const { return epipolar_error_before_; }
    double epipolar_error_after() const { return epipolar_error_after_; }
    double reproj_error_before() const { return reproj_error_before_; }
    double reproj_error_after() const { return reproj_error_after_; }
    bool last_pnp() const { return last_pnp_; }
    bool last_was_loop() const { return last_loop_; }
    int loop_count() const { return loop_count_; }
    const std::vector<std::pair<int, int>>& loop_edges() const { return loop_edges_; }  // (matched id, frame id)
    const std::vector<LoopConstraint>& loop_constraints() const { return loop_constraints_; }

   private:
    FILE* trace_ = nullptr;
    PhaseProf phase_;
    static uint64_t fnv(const void* p, size_t n) {
        uint64_t h = 1469598103934665603ull;
        for (size_t i = 0; i < n; i++) h = (h ^ static_cast<const uint8_t*>(p)[i]) * 1099511628211ull;
        return h;
    }
    void trace_pose(int id, const char* tag, const M3& R, const V3& t) const {
        if (!trace_) return;
        if (id >= 0) std::fprintf(trace_, "%d %s", id, tag);
        for (double v : R) std::fprintf(trace_, " %a", v);
        for (double v : t) std::fprintf(trace_, " %a", v);
        std::fprintf(trace_, "\n");
    }
    void trace_chain(int id, const ChainResult& C) const {
        if (!trace_) return;
        std::fprintf(trace_, "%d chain ref=%d raw=%d good=%d/%016llx fok=%d fit=%d kept=%d epi=%a/%a ok3d=%d okE=%d sc=%a\n",
                     id, ref_frame_ ? ref_frame_->id : -1, C.n_raw, (int)C.good.size(),
                     (unsigned long long)fnv(C.good.data(), C.good.size() * sizeof(Match)), (int)C.f_ok, C.f_iters,
                     (int)C.kept.size(), C.epi_before, C.epi_after, (int)C.ok3d, (int)C.okE, C.scale);
        if (C.ok3d) trace_pose(id, "r3d", C.R3, C.t3);
        if (C.okE) trace_pose(id, "rE", C.RE, C.tE);
    }
    struct Snapshot {
        double x_pred[6], P_pred[36], x_filt[6], P_filt[36];
        double dt;
        int frame_index;
    };

    static void points_of(const Frame& a, const Frame& b, const std::vector<Match>& m, std::vector<float>& p1,
                          std::vector<float>& p2) {  // Slam::extract_matched_points (:1175-1188)
        p1.clear();
        p2.clear();
        for (const Match& x : m) {
            p1.insert(p1.end(), {a.kps[x.query_idx].x, a.kps[x.query_idx].y});
            p2.insert(p2.end(), {b.kps[x.train_idx].x, b.kps[x.train_idx].y});
        }
    }

    // Optimizer::project_point (Optimizer.cpp:26-48): pc = R^T Pw - R^T t
    static void project_point(const double* pw, const M3& R, const V3& t, double& u, double& v) {
        const M3 Rc = tr(R);
        const V3 tc = mulv(Rc, t);
        const V3 pc0 = mulv(Rc, V3{pw[0], pw[1], pw[2]});
        const V3 pc{pc0[0] - tc[0], pc0[1] - tc[1], pc0[2] - tc[2]};
        if (pc[2] < 1e-6) {
            u = v = -1;
            return;
        }
        u = cfg::FX * pc[0] / pc[2] + cfg::CX;
        v = cfg::FY * pc[1] / pc[2] + cfg::CY;
    }

    // Slam::track_local_map (:380-469): the back end returns the updated indices and the
    // observations in the order the reference adds them.
    int track_local_map(const FramePtr& frame) {
        if (frame->kps.empty()) return 0;
        std::vector<std::pair<int, int>> obs;
        const int tracked = ops_.track_local_map(map_, *frame, obs);
        for (const auto& o : obs) map_.obs[o.first].emplace_back(frame->id, o.second);
        stats_.tracked_total += tracked;
        return tracked;
    }

    // gather of tracked map points for PnP (:1408-1420, 1481-1494, 631-644)
    void tracked_points(const Frame& f, std::vector<float>& obj, std::vector<float>& img) const {
        obj.clear();
        img.clear();
        for (int i = 0; i < (int)f.mp_idx.size(); i++) {
            const int id = f.mp_idx[i];
            if (id >= 0 && id < map_.size() && map_.valid[id]) {
                obj.insert(obj.end(), {(float)map_.pos[3 * id], (float)map_.pos[3 * id + 1], (float)map_.pos[3 * id + 2]});
                img.insert(img.end(), {f.kps[i].x, f.kps[i].y});
            }
        }
    }

    // Slam::refine_pose_via_local_pnp (:1373-1473)
    void refine_pose_via_local_pnp(const FramePtr& frame, int tracked) {
        {
            const M3 Rc = tr(R_world_);
            const V3 tc0 = mulv(Rc, t_world_);
            double sum = 0;
            int cnt = 0;
            for (int i = 0; i < (int)frame->mp_idx.size(); i++) {
                const int id = frame->mp_idx[i];
                if (id < 0 || id >= map_.size() || !map_.valid[id]) continue;
                const V3 p0 = mulv(Rc, V3{map_.pos[3 * id], map_.pos[3 * id + 1], map_.pos[3 * id + 2]});
                const V3 pc{p0[0] - tc0[0], p0[1] - tc0[1], p0[2] - tc0[2]};
                if (pc[2] < 0.01) continue;
                const double u = cfg::FX * pc[0] / pc[2] + cfg::CX, v = cfg::FY * pc[1] / pc[2] + cfg::CY;
                const double dx = u - frame->kps[i].x, dy = v - frame->kps[i].y;
                sum += std::sqrt(dx * dx + dy * dy);
                cnt++;
            }
            reproj_error_before_ = cnt > 0 ? sum / cnt : 0.0;
            reproj_error_after_ = reproj_error_before_;
        }
        if (tracked < 10) return;
        std::vector<float> obj, img;
        tracked_points(*frame, obj, img);
        const M3 R_prev = R_world_;
        const V3 t_prev = t_world_;
        const PnPResult pnp = solve_pnp(obj, img, 100, 10);
        if (!pnp.success) return;
        const V3 d{pnp.t_world[0] - t_world_[0], pnp.t_world[1] - t_world_[1], pnp.t_world[2] - t_world_[2]};
        if (!(norm3(d) < cfg::PNP_REFINE_MAX_JUMP)) return;
        const double inlier_ratio = (double)pnp.inlier_count / (double)(obj.size() / 3);
        const double blend = std::min(0.5, 0.3 + 0.2 * std::max(0.0, std::min(1.0, (inlier_ratio - 0.5) / 0.5)));
        blend_pose(pnp, blend);
        frame->R = R_world_;
        frame->t = t_world_;
        stats_.pnp_refined++;
        auto reproj = [&](const M3& Rw, const V3& tw) {
            const M3 Rc = tr(Rw);
            const V3 tc0 = mulv(Rc, tw);
            double sum = 0;
            int cnt = 0;
            for (size_t pi = 0; pi < obj.size() / 3; pi++) {
                const V3 p0 = mulv(Rc, V3{obj[3 * pi], obj[3 * pi + 1], obj[3 * pi + 2]});
                const V3 pc{p0[0] - tc0[0], p0[1] - tc0[1], p0[2] - tc0[2]};
                if (pc[2] < 0.01) continue;
                const double u = cfg::FX * pc[0] / pc[2] + cfg::CX, v = cfg::FY * pc[1] / pc[2] + cfg::CY;
                const double dx = u - img[2 * pi], dy = v - img[2 * pi + 1];
                sum += std::sqrt(dx * dx + dy * dy);
                cnt++;
            }
            return cnt > 0 ? sum / cnt : 0.0;
        };
        reproj_error_before_ = reproj(R_prev, t_prev);
        reproj_error_after_ = reproj(R_world_, t_world_);
    }

    // t = (1-b) t + b t_pnp; R = Rodrigues((1-b) rvec(R) + b rvec(R_pnp))  (:1431-1443, 1504-1514)
    void blend_pose(const PnPResult& pnp, double blend) {
        V3 tb;
        for (int i = 0; i < 3; i++) tb[i] = (1.0 - blend) * t_world_[i] + blend * pnp.t_world[i];
        double rc[3], rp[3], rb[3];
        vs_pnp::rod_m2v(R_world_.data(), rc);
        vs_pnp::rod_m2v(pnp.R_world.data(), rp);
        for (int i = 0; i < 3; i++) rb[i] = (1.0 - blend) * rc[i] + blend * rp[i];
        M3 Rb;
        vs_pnp::rod_v2m(rb, Rb.data());
        R_world_ = Rb;
        t_world_ = tb;
    }

    PnPResult solve_pnp(const std::vector<float>& obj, const std::vector<float>& img, int iters, int min_inliers) {
        PnPResult r;
        if ((int)(obj.size() / 3) < min_inliers) return r;  // :512
        r = ops_.solve_pnp(obj, img, iters, min_inliers);
        if (trace_) {
            std::fprintf(trace_, "pnp n=%d in=%016llx/%016llx ok=%d inl=%d", (int)(obj.size() / 3),
                         (unsigned long long)fnv(obj.data(), obj.size() * 4), (unsigned long long)fnv(img.data(), img.size() * 4),
                         (int)r.success, r.inlier_count);
            trace_pose(-1, "", r.R_world, r.t_world);
        }
        return r;
    }

    // Slam::handle_loop_closure (:730-798) with LoopCloser::detect (LoopCloser.cpp:16-100)
    void handle_loop_closure(const FramePtr& frame) {
        // ---- LoopCloser::detect ----
        if (!frame->has_desc()) return;  // :23
        std::vector<const Frame*> kfs;   // Map::get_keyframes (Map.cpp:40-47)
        for (const FramePtr& f : map_.frames)
            if (f->keyframe) kfs.push_back(f.get());
        if (kfs.size() < 2) return;  // :26
        std::vector<const Frame*> cand;  // :44-49 every 5th keyframe at least LC_MIN_FRAME_GAP ids back
        int checked = 0;
        for (const Frame* kf : kfs) {
            if (frame->id - kf->id < cfg::LC_MIN_FRAME_GAP) continue;
            if (!kf->has_desc()) continue;
            checked++;
            if (checked % 5 != 0) continue;
            cand.push_back(kf);
        }
        if (cand.empty()) return;
        const std::vector<LoopEval> ev = ops_.loop_eval(*frame, cand);
        int best = -1, best_inliers = 0;
        for (size_t i = 0; i < cand.size(); i++) {  // :51-88
            if (ev[i].n_good < cfg::MIN_MATCHES) continue;
            if (ev[i].inliers < cfg::LC_MIN_INLIERS) continue;  // E.empty() gives 0 inliers
            if (ev[i].inliers > best_inliers) {
                best_inliers = ev[i].inliers;
                best = (int)i;
            }
        }
        if (best < 0 || best_inliers < cfg::LC_MIN_INLIERS) return;  // :91
        loop_count_++;
        const Frame* matched = cand[best];
        if (trace_) std::fprintf(trace_, "%d loop %d inliers %d\n", frame->id, matched->id, best_inliers);
        // ---- handle_loop_closure ----
        last_loop_ = true;
        loop_edges_.emplace_back(matched->id, frame->id);
        std::vector<int> ids;  // :743-761 valid map points observed within LC_NEARBY_FRAME_RANGE ids
        for (int i = 0; i < map_.size(); i++) {
            if (!map_.valid[i]) continue;
            for (const auto& ob : map_.obs[i])
                if (std::abs(ob.first - matched->id) < cfg::LC_NEARBY_FRAME_RANGE) {
                    ids.push_back(i);
                    break;
                }
        }
        std::vector<float> obj, img;
        if ((int)ids.size() >= 20 && frame->has_desc()) {  // :763-775 FLANN 2-NN (exact here) + ratio 0.7
            const auto pairs = ops_.match_map(map_, *frame, ids, cfg::FLANN_RATIO_THRESHOLD);
            for (const auto& q : pairs) {
                const int id = ids[q.second];
                obj.insert(obj.end(), {(float)map_.pos[3 * id], (float)map_.pos[3 * id + 1], (float)map_.pos[3 * id + 2]});
                img.insert(img.end(), {frame->kps[q.first].x, frame->kps[q.first].y});
            }
        }
        const PnPResult pnp = solve_pnp(obj, img, 300, 15);  // :779-780
        if (!pnp.success) return;
        const V3 d{pnp.t_world[0] - t_world_[0], pnp.t_world[1] - t_world_[1], pnp.t_world[2] - t_world_[2]};
        const double jump = norm3(d);
        if (jump >= cfg::LC_MAX_JUMP || jump <= cfg::LC_MIN_JUMP) return;  // :782-783
        LoopConstraint c;  // :788-797
        c.from_id = matched->id;
        c.to_id = frame->id;
        const M3 Rft = tr(matched->R);
        c.R_rel = mul(Rft, pnp.R_world);
        c.t_rel = mulv(Rft, V3{pnp.t_world[0] - matched->t[0], pnp.t_world[1] - matched->t[1],
                               pnp.t_world[2] - matched->t[2]});
        c.trans_sigma = cfg::PGO_LC_TRANS_SIGMA;
        c.rot_sigma = cfg::PGO_LC_ROT_SIGMA;
        loop_constraints_.push_back(c);
    }

    // Slam::run_pnp (:1477-1522)
    void run_pnp(const FramePtr& frame) {
        std::vector<float> obj, img;
        tracked_points(*frame, obj, img);
        const PnPResult pnp = solve_pnp(obj, img, 100, cfg::PNP_MIN_POINTS);
        if (!pnp.success) return;
        const V3 d{pnp.t_world[0] - frame->t[0], pnp.t_world[1] - frame->t[1], pnp.t_world[2] - frame->t[2]};
        if (norm3(d) > cfg::PNP_PERIODIC_MAX_JUMP) return;
        const double blend = cfg::PNP_PERIODIC_BLEND;
        V3 tb;
        for (int i = 0; i < 3; i++) tb[i] = (1.0 - blend) * frame->t[i] + blend * pnp.t_world[i];
        double rc[3], rp[3], rb[3];
        vs_pnp::rod_m2v(frame->R.data(), rc);
        vs_pnp::rod_m2v(pnp.R_world.data(), rp);
        for (int i = 0; i < 3; i++) rb[i] = (1.0 - blend) * rc[i] + blend * rp[i];
        M3 Rb;
        vs_pnp::rod_v2m(rb, Rb.data());
        R_world_ = Rb;
        t_world_ = tb;
        frame->R = R_world_;
        frame->t = t_world_;
        last_pnp_ = true;
        stats_.periodic_pnp++;
    }

    // Slam::try_pnp_recovery (:535-613): 1 recovered, 0 not needed, -1 failed
    int try_pnp_recovery(const FramePtr& frame) {
        if (pnp_recovery_cooldown_ > 0) pnp_recovery_cooldown_--;
        if (last_match_count_ >= cfg::MIN_MATCHES) return 0;
        if (pnp_recovery_cooldown_ > 0) {
            last_frame_ = frame;
            return -1;
        }
        std::vector<int> ids;
        for (int i = 0; i < map_.size(); i++)
            if (map_.valid[i]) ids.push_back(i);
        if ((int)ids.size() >= 50 && frame->has_desc()) {
            // FLANN knnMatch(frame descriptors, map descriptors, k = 2) + ratio 0.7 (exact 2-NN here)
            const auto pairs = ops_.match_map(map_, *frame, ids, cfg::FLANN_RATIO_THRESHOLD);
            std::vector<float> obj, img;
            for (const auto& q : pairs) {
                const int id = ids[q.second];
                obj.insert(obj.end(), {(float)map_.pos[3 * id], (float)map_.pos[3 * id + 1], (float)map_.pos[3 * id + 2]});
                img.insert(img.end(), {frame->kps[q.first].x, frame->kps[q.first].y});
            }
            if ((int)(obj.size() / 3) >= 20) {
                const PnPResult pnp = solve_pnp(obj, img, 300, 15);
                if (pnp.success) {
                    const V3 d{pnp.t_world[0] - t_world_[0], pnp.t_world[1] - t_world_[1], pnp.t_world[2] - t_world_[2]};
                    const double jump = norm3(d);
                    if (jump < cfg::PNP_RECOVERY_MAX_JUMP) {
                        const double blend = (jump < 0.1) ? cfg::PNP_RECOVERY_BLEND_CLOSE : cfg::PNP_RECOVERY_BLEND_FAR;
                        R_world_ = pnp.R_world;
                        for (int i = 0; i < 3; i++) t_world_[i] = (1.0 - blend) * t_world_[i] + blend * pnp.t_world[i];
                        frame->R = R_world_;
                        frame->t = t_world_;
                        map_.frames.push_back(frame);
                        frame->keyframe = true;
                        keyframe_count_++;
                        stats_.keyframes++;
                        create_points_from_depth(frame);
                        last_keyframe_ = frame;
                        last_frame_ = frame;
                        frame_count_++;
                        if (ekf_init_) {
                            for (int i = 0; i < 3; i++) x_[i] = t_world_[i];
                            for (int i = 3; i < 6; i++) x_[i] = 0;
                        }
                        last_frame_time_ = frame->timestamp;
                        pnp_recovery_cooldown_ = 10;
                        stats_.recoveries++;
                        stats_.processed++;
                        return 1;
                    }
                }
            }
        }
        last_frame_ = frame;
        return -1;
    }

    // Slam::is_frame_stationary (:1621-1651)
    bool is_frame_stationary(double ts) const {
        if (accel_.empty()) return false;
        const double window = 0.1, threshold = 0.15;
        int lo = 0, hi = (int)accel_.size() - 1;
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (accel_[mid].timestamp < ts - window)
                lo = mid + 1;
            else
                hi = mid;
        }
        std::vector<double> mags;
        for (int i = lo; i < (int)accel_.size() && accel_[i].timestamp <= ts + window; i++)
            mags.push_back(std::sqrt(accel_[i].ax * accel_[i].ax + accel_[i].ay * accel_[i].ay + accel_[i].az * accel_[i].az));
        if (mags.size() < 5) return false;
        double mean = 0;
        for (double m : mags) mean += m;
        mean /= mags.size();
        double var = 0;
        for (double m : mags) var += (m - mean) * (m - mean);
        var /= mags.size();
        return std::sqrt(var) < threshold;
    }

    // Slam::process_stationary_frame (:618-694)
    bool process_stationary_frame(const FramePtr& frame, const std::vector<Match>& good) {
        if (!is_frame_stationary(frame->timestamp) || frame_count_ <= 5) return false;
        frame->R = R_world_;
        frame->t = t_world_;
        map_.frames.push_back(frame);
        const int tracked = track_local_map(frame);
        if (tracked >= 10) {
            std::vector<float> obj, img;
            tracked_points(*frame, obj, img);
            const PnPResult pnp = solve_pnp(obj, img, 100, 10);
            if (pnp.success) {
                R_world_ = pnp.R_world;
                frame->R = R_world_;
                frame->t = t_world_;
            }
        }
        if (last_keyframe_) {
            const M3 Rd = mul(tr(R_world_), last_keyframe_->R);
            double rv[3];
            vs_pnp::rod_m2v(Rd.data(), rv);
            if (std::sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]) > 0.25) {
                frame->keyframe = true;
                keyframe_count_++;
                stats_.keyframes++;
                create_points_from_depth(frame);
                last_keyframe_ = frame;
            }
        }
        last_frame_ = frame;
        last_match_count_ = (int)good.size();
        frame_count_++;
        was_stationary_ = true;
        if (ekf_init_) {
            for (int i = 0; i < 3; i++) x_[i + 3] = 0, x_[i] = t_world_[i];
            for (int i = 3; i < 6; i++) {
                for (int j = 0; j < 6; j++) P_[i * 6 + j] = P_[j * 6 + i] = 0;
                P_[i * 6 + i] = 1e-4;
            }
        }
        last_frame_time_ = frame->timestamp;
        stats_.stationary++;
        stats_.processed++;
        return true;
    }

    // Slam::setup_new_keyframe (:699-725); local BA is disabled (Config.h:99)
    void setup_new_keyframe(const FramePtr& frame) {
        if (last_keyframe_) match_and_triangulate(last_keyframe_, frame);
        create_points_from_depth(frame);
        cull_map_points(frame);
    }

    // The projection matrices K [R | t] of two frames (Slam.cpp:1255-1262)
    static void proj_mats(const Frame& f1, const Frame& f2, double P1[12], double P2[12]) {
        const M3 R1c = tr(f1.R), R2c = tr(f2.R);
        const V3 m1 = mulv(R1c, f1.t), m2 = mulv(R2c, f2.t);
        const V3 t1c{-m1[0], -m1[1], -m1[2]}, t2c{-m2[0], -m2[1], -m2[2]};
        const double K[9] = {cfg::FX, 0, cfg::CX, 0, cfg::FY, cfg::CY, 0, 0, 1};
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 4; j++) {
                double s1 = 0, s2 = 0;
                for (int k = 0; k < 3; k++) {
                    s1 += K[i * 3 + k] * (j < 3 ? R1c[k * 3 + j] : t1c[k]);
                    s2 += K[i * 3 + k] * (j < 3 ? R2c[k * 3 + j] : t2c[k]);
                }
                P1[i * 4 + j] = s1;
                P2[i * 4 + j] = s2;
            }
    }

    // match(f1, f2) then triangulate_points on the good matches when there are enough
    // (Slam.cpp:713-716, :859-862).  The back end returns the DLT solution of every good match
    // with the matches (vs_trk::dlt_point; on the GPU one launch behind the matcher, one round trip).
    void match_and_triangulate(const FramePtr& f1, const FramePtr& f2) {
        double P1[12], P2[12];
        proj_mats(*f1, *f2, P1, P2);
        std::vector<std::array<float, 4>> X4;
        const auto m = ops_.match_dlt(*f1, *f2, cfg::L2_RATIO_THRESHOLD, P1, P2, X4);
        if ((int)m.size() >= cfg::MIN_MATCHES) triangulate_points(f1, f2, m, X4);
    }

    // Slam::triangulate_points (:1246-1356), with the DLT of match i in X4[i]
    void triangulate_points(const FramePtr& f1, const FramePtr& f2, const std::vector<Match>& matches,
                            const std::vector<std::array<float, 4>>& X4all) {
        const M3 R1c = tr(f1->R), R2c = tr(f2->R);
        const V3 m1 = mulv(R1c, f1->t), m2 = mulv(R2c, f2->t);
        const V3 t1c{-m1[0], -m1[1], -m1[2]}, t2c{-m2[0], -m2[1], -m2[2]};
        if (matches.size() < 5) return;
        const bool use_real_depth = f2->has_depth();
        std::vector<int> rows;
        std::vector<double> pts;
        for (size_t i = 0; i < matches.size(); i++) {
            const Keypoint& a = f1->kps[matches[i].query_idx];
            const Keypoint& b = f2->kps[matches[i].train_idx];
            const float* X4 = X4all[i].data();
            const float w = X4[3];
            if (std::abs(w) < 1e-6) continue;
            double pt[3] = {X4[0] / w, X4[1] / w, X4[2] / w};
            if (use_real_depth) {  // :1294-1310 Kinect depth overrides the triangulated depth
                const int px = (int)std::round(b.x), py = (int)std::round(b.y);
                if (px >= 0 && px < f2->dw && py >= 0 && py < f2->dh) {
                    const float z = f2->depth_at(py, px);
                    if (z > cfg::DEPTH_MIN && z < cfg::DEPTH_MAX) {
                        const double xc = (b.x - cfg::CX) * z / cfg::FX, yc = (b.y - cfg::CY) * z / cfg::FY;
                        const V3 pw0 = mulv(f2->R, V3{xc, yc, (double)z});
                        pt[0] = pw0[0] + f2->t[0];
                        pt[1] = pw0[1] + f2->t[1];
                        pt[2] = pw0[2] + f2->t[2];
                    }
                }
            }
            const V3 c1 = mulv(R1c, V3{pt[0], pt[1], pt[2]}), c2 = mulv(R2c, V3{pt[0], pt[1], pt[2]});
            const double z1 = c1[2] + t1c[2], z2 = c2[2] + t2c[2];
            if (z1 < cfg::TRIANG_MIN_DEPTH || z1 > cfg::TRIANG_MAX_DEPTH) continue;
            if (z2 < cfg::TRIANG_MIN_DEPTH || z2 > cfg::TRIANG_MAX_DEPTH) continue;
            double u, v;
            project_point(pt, f2->R, f2->t, u, v);
            double dx = u - b.x, dy = v - b.y;
            if (std::sqrt(dx * dx + dy * dy) > cfg::TRIANG_MAX_REPROJ_ERROR) continue;
            project_point(pt, f1->R, f1->t, u, v);
            dx = u - a.x;
            dy = v - a.y;
            if (std::sqrt(dx * dx + dy * dy) > cfg::TRIANG_MAX_REPROJ_ERROR) continue;
            const double ex = pt[0] - f2->t[0], ey = pt[1] - f2->t[1], ez = pt[2] - f2->t[2];
            if (std::sqrt(ex * ex + ey * ey + ez * ez) > cfg::TRIANG_MAX_CAM_DIST) continue;
            const int kp2 = matches[i].train_idx;
            const int id = map_.add(pt, keyframe_count_);
            map_.obs[id].emplace_back(f1->id, matches[i].query_idx);
            map_.obs[id].emplace_back(f2->id, kp2);
            f1->mp_idx[matches[i].query_idx] = id;
            f2->mp_idx[kp2] = id;
            rows.push_back(kp2);
            stats_.triangulated++;
        }
        if (!rows.empty()) ops_.map_append(map_, map_.size() - (int)rows.size(), *f2, rows);
    }

    // Slam::create_points_from_depth (:1526-1577)
    void create_points_from_depth(const FramePtr& frame) {
        if (!frame->has_depth()) return;
        std::vector<int> rows;
        for (int i = 0; i < (int)frame->kps.size(); i++) {
            if (frame->mp_idx[i] >= 0) continue;
            const float u = frame->kps[i].x, v = frame->kps[i].y;
            const int px = (int)std::round(u), py = (int)std::round(v);
            if (px < 0 || px >= frame->dw || py < 0 || py >= frame->dh) continue;
            const float z = frame->depth_at(py, px);
            if (z <= cfg::DEPTH_MIN || z > cfg::TRIANG_MAX_CAM_DIST) continue;
            const double xc = (u - cfg::CX) * z / cfg::FX, yc = (v - cfg::CY) * z / cfg::FY;
            const V3 pw0 = mulv(frame->R, V3{xc, yc, (double)z});
            const double pt[3] = {pw0[0] + frame->t[0], pw0[1] + frame->t[1], pw0[2] + frame->t[2]};
            const int id = map_.add(pt, keyframe_count_);
            map_.obs[id].emplace_back(frame->id, i);
            frame->mp_idx[i] = id;
            rows.push_back(i);
            stats_.depth_points++;
        }
        if (!rows.empty()) ops_.map_append(map_, map_.size() - (int)rows.size(), *frame, rows);
    }

    // Slam::cull_map_points (:473-500)
    void cull_map_points(const FramePtr& frame) {
        const M3 Rc = tr(frame->R);
        const V3 tc0 = mulv(Rc, frame->t);
        bool changed = false;
        for (int i = 0; i < (int)frame->mp_idx.size(); i++) {
            const int id = frame->mp_idx[i];
            if (id < 0 || id >= map_.size() || !map_.valid[id]) continue;
            const V3 p0 = mulv(Rc, V3{map_.pos[3 * id], map_.pos[3 * id + 1], map_.pos[3 * id + 2]});
            const V3 pc{p0[0] - tc0[0], p0[1] - tc0[1], p0[2] - tc0[2]};
            if (pc[2] < cfg::DEPTH_MIN) {
                map_.valid[id] = 0;
                changed = true;
                stats_.culled++;
                continue;
            }
            const double u = cfg::FX * pc[0] / pc[2] + cfg::CX, v = cfg::FY * pc[1] / pc[2] + cfg::CY;
            const double dx = u - frame->kps[i].x, dy = v - frame->kps[i].y;
            if (dx * dx + dy * dy > 400.0) {
                map_.valid[id] = 0;
                changed = true;
                stats_.culled++;
            }
        }
        if (changed) ops_.map_valid_changed();
    }

    // :1089-1108 visibility sweep (back end: one projection + keypoint radius test per point)
    void visibility_sweep(const FramePtr& frame) {
        std::vector<uint8_t> flags;
        ops_.visibility(map_, *frame, R_world_, t_world_, flags);
        for (int i = 0; i < map_.size(); i++) {
            if (flags[i] & 1) map_.visible[i]++;
            if (flags[i] & 2) map_.found[i]++;
        }
    }

    // :1110-1126 culling by found ratio
    void cull_by_found_ratio() {
        bool changed = false;
        for (int i = 0; i < map_.size(); i++) {
            if (!map_.valid[i]) continue;
            const int age = keyframe_count_ - map_.first_kf[i];
            if (age >= 3 && map_.visible[i] > 0 && map_.found_ratio(i) < cfg::CULL_FOUND_RATIO_YOUNG) {
                map_.valid[i] = 0;
                changed = true;
                stats_.culled++;
            }
            if (age >= 5 && (int)map_.obs[i].size() <= 2 && map_.found_ratio(i) < cfg::CULL_FOUND_RATIO_OLD) {
                if (map_.valid[i]) stats_.culled++;
                map_.valid[i] = 0;
                changed = true;
            }
        }
        if (changed) ops_.map_valid_changed();
    }

    // Slam::is_keyframe (:1359-1368)
    bool is_keyframe(const FramePtr& frame, int match_count) const {
        if (!last_keyframe_) return true;
        if (frame->id - last_keyframe_->id < cfg::KF_MIN_FRAME_GAP) return false;
        if (match_count < cfg::KF_MIN_MATCHES) return false;
        return true;
    }

    // ---- EKF (Slam.cpp:1654-1744), 6-state position + velocity ------------------------------
    static void transition(double dt, double decay, double F[36]) {
        for (int i = 0; i < 36; i++) F[i] = (i % 7 == 0) ? 1.0 : 0.0;
        for (int i = 0; i < 3; i++) {
            F[i * 6 + i + 3] = dt;
            F[(i + 3) * 6 + i + 3] = decay;
        }
    }
    // C = op(A) op(B) for 6x6
    static void mm6(const double* A, const double* B, double* C, bool ta, bool tb) {
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                double s = 0;
                for (int k = 0; k < 6; k++) s += (ta ? A[k * 6 + i] : A[i * 6 + k]) * (tb ? B[j * 6 + k] : B[k * 6 + j]);
                C[i * 6 + j] = s;
            }
    }
    // cv::Mat::inv(DECOMP_SVD) of a symmetric 6x6 (eigen-decomposition pseudo-inverse)
    static void pinv6(const double* P, double* out) {
        double A[36], w[6], V[36];
        std::memcpy(A, P, sizeof(A));
        vs_pnp::sym_eig<6>(A, w, V);
        const double tol = std::abs(w[0]) * 6 * 2.220446049250313e-16;
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                double s = 0;
                for (int k = 0; k < 6; k++)
                    if (std::abs(w[k]) > tol) s += V[i * 6 + k] * V[j * 6 + k] / w[k];
                out[i * 6 + j] = s;
            }
    }
    // :986-1016: EKF initialisation / prediction / visual update (innovation gate) / height update for
    // the motion estimate t_new of a frame at time ts; the snapshot's predicted and filtered parts when
    // given; returns the prediction interval.  x_ then holds the fused state (before the step clamp).
    double ekf_fuse(const V3& t_new, bool use_3d3d, double ts, Snapshot* snap) {
        if (!ekf_init_) ekf_initialize(t_world_, ts);
        const double dt = ts - last_frame_time_;
        if (dt > 0 && dt < 1.0) ekf_predict(dt);
        if (snap) {
            std::memcpy(snap->x_pred, x_, sizeof(x_));
            std::memcpy(snap->P_pred, P_, sizeof(P_));
        }
        const double sigma_vis = use_3d3d ? cfg::EKF_SIGMA_VIS_3D3D : cfg::EKF_SIGMA_VIS_EMAT;
        const V3 dinn{t_new[0] - x_[0], t_new[1] - x_[1], t_new[2] - x_[2]};
        const double innovation = norm3(dinn);
        if (innovation < cfg::EKF_INNOV_GATE)
            ekf_update_visual(t_new, sigma_vis);
        else
            ekf_update_visual(t_new, innovation * 0.5);
        if (has_gravity_ && has_initial_height_) ekf_update_height(initial_height_, cfg::EKF_SIGMA_HEIGHT);
        if (snap) std::memcpy(snap->P_filt, P_, sizeof(P_));
        return dt;
    }
    void ekf_initialize(const V3& pos, double ts) {
        for (int i = 0; i < 6; i++) x_[i] = i < 3 ? pos[i] : 0.0;
        for (int i = 0; i < 36; i++) P_[i] = 0;
        for (int i = 0; i < 3; i++) P_[i * 7] = 0.001;
        for (int i = 3; i < 6; i++) P_[i * 7] = 0.01;
        last_frame_time_ = ts;
        ekf_init_ = true;
    }
    void ekf_predict(double dt) {
        if (!ekf_init_ || dt <= 0) return;
        const double decay = cfg::EKF_VEL_DECAY;
        for (int i = 0; i < 3; i++) {
            x_[i] += x_[i + 3] * dt;
            x_[i + 3] *= decay;
        }
        double F[36], Q[36] = {0}, FP[36], FPFt[36];
        transition(dt, decay, F);
        const double sa = cfg::EKF_PROCESS_ACCEL;
        for (int i = 0; i < 3; i++) {
            Q[i * 7] = 0.25 * dt * dt * dt * dt * sa * sa;
            Q[(i + 3) * 7] = dt * dt * sa * sa;
            Q[i * 6 + i + 3] = 0.5 * dt * dt * dt * sa * sa;
            Q[(i + 3) * 6 + i] = Q[i * 6 + i + 3];
        }
        mm6(F, P_, FP, false, false);
        mm6(FP, F, FPFt, false, true);
        for (int i = 0; i < 36; i++) P_[i] = FPFt[i] + Q[i];
    }
    // Kalman update with H = rows of the identity / gravity (m rows); Joseph form (:1701-1744)
    void ekf_update(const double* H, int m, const double* z, double sigma) {
        double y[3], S[9], PHt[18], Kg[18];
        for (int r = 0; r < m; r++) {
            double hx = 0;
            for (int k = 0; k < 6; k++) hx += H[r * 6 + k] * x_[k];
            y[r] = z[r] - hx;
        }
        for (int i = 0; i < 6; i++)
            for (int r = 0; r < m; r++) {
                double s = 0;
                for (int k = 0; k < 6; k++) s += P_[i * 6 + k] * H[r * 6 + k];
                PHt[i * m + r] = s;
            }
        for (int a = 0; a < m; a++)
            for (int b = 0; b < m; b++) {
                double s = 0;
                for (int k = 0; k < 6; k++) s += H[a * 6 + k] * PHt[k * m + b];
                S[a * m + b] = s + (a == b ? sigma * sigma : 0.0);
            }
        double Si[9];
        inv_small(S, m, Si);
        for (int i = 0; i < 6; i++)
            for (int b = 0; b < m; b++) {
                double s = 0;
                for (int a = 0; a < m; a++) s += PHt[i * m + a] * Si[a * m + b];
                Kg[i * m + b] = s;
            }
        for (int i = 0; i < 6; i++) {
            double s = 0;
            for (int r = 0; r < m; r++) s += Kg[i * m + r] * y[r];
            x_[i] += s;
        }
        double IKH[36], T1[36], T2[36];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                double s = 0;
                for (int r = 0; r < m; r++) s += Kg[i * m + r] * H[r * 6 + j];
                IKH[i * 6 + j] = (i == j ? 1.0 : 0.0) - s;
            }
        mm6(IKH, P_, T1, false, false);
        mm6(T1, IKH, T2, false, true);
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++) {
                double s = 0;
                for (int r = 0; r < m; r++) s += Kg[i * m + r] * sigma * sigma * Kg[j * m + r];
                P_[i * 6 + j] = T2[i * 6 + j] + s;
            }
    }
    static void inv_small(const double* S, int m, double* out) {  // Gauss-Jordan, partial pivoting
        double a[3][6];
        for (int i = 0; i < m; i++)
            for (int j = 0; j < 2 * m; j++) a[i][j] = j < m ? S[i * m + j] : (j - m == i ? 1.0 : 0.0);
        for (int c = 0; c < m; c++) {
            int p = c;
            for (int r = c + 1; r < m; r++)
                if (std::abs(a[r][c]) > std::abs(a[p][c])) p = r;
            if (p != c)
                for (int j = 0; j < 2 * m; j++) std::swap(a[c][j], a[p][j]);
            const double d = a[c][c];
            if (d == 0) {
                for (int i = 0; i < m * m; i++) out[i] = 0;
                return;
            }
            for (int j = 0; j < 2 * m; j++) a[c][j] /= d;
            for (int r = 0; r < m; r++)
                if (r != c) {
                    const double f = a[r][c];
                    for (int j = 0; j < 2 * m; j++) a[r][j] -= f * a[c][j];
                }
        }
        for (int i = 0; i < m; i++)
            for (int j = 0; j < m; j++) out[i * m + j] = a[i][m + j];
    }
    void ekf_update_visual(const V3& z, double sigma) {
        if (!ekf_init_) return;
        double H[18] = {0};
        for (int i = 0; i < 3; i++) H[i * 6 + i] = 1.0;
        ekf_update(H, 3, z.data(), sigma);
    }
    void ekf_update_height(double h_target, double sigma) {
        if (!ekf_init_ || !has_gravity_) return;
        double H[6] = {gravity_[0], gravity_[1], gravity_[2], 0, 0, 0};
        ekf_update(H, 1, &h_target, sigma);
    }

    Ops& ops_;
    Map map_;
    M3 R_world_ = eye3();
    V3 t_world_{0, 0, 0};
    FramePtr last_frame_, last_keyframe_, ref_frame_;
    int frame_count_ = 0, keyframe_count_ = 0, last_match_count_ = 0;
    bool last_loop_ = false;
    int loop_count_ = 0;  // LoopCloser::loop_count_
    std::vector<std::pair<int, int>> loop_edges_;
    std::vector<LoopConstraint> loop_constraints_;
    double epipolar_error_before_ = 0, epipolar_error_after_ = 0, reproj_error_before_ = 0, reproj_error_after_ = 0;
    bool last_pnp_ = false;
    double last_good_scale_ = -1.0;
    std::vector<AccelSample> accel_;
    V3 gravity_{0, 0, 0};
    bool has_gravity_ = false;
    double initial_height_ = 0.0;
    bool has_initial_height_ = false, was_stationary_ = false;
    int pnp_recovery_cooldown_ = 0;
    double x_[6] = {0}, P_[36] = {0};
    bool ekf_init_ = false;
    double last_frame_time_ = 0;
    std::vector<Snapshot> snapshots_;
    Stats stats_;
};

}  // namespace vs_trk
