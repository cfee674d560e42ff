// vslam_amd.hpp — C++ host façade over the C ABI (include/vslam_abi.h), mirroring the reference's
// class surfaces for the per-frame hot path so that call sites read like the reference's:
//
//   FeatureExtractor      include/FeatureExtractor.h:13-66 (init, extract, SPCF feature cache)
//   match_features        Slam.h:69-70            (Slam.cpp:1140-1172)
//   extract_matched_points Slam.h:72-76           (Slam.cpp:1174-1187)
//   verify_fundamental    Slam.cpp:880-910        (findFundamentalMat FM_RANSAC 3.0 / 0.999 +
//                                                  compute_epipolar_error before/after + filtering)
//   estimate_motion_3d3d  Slam.h:133-137          (Slam.cpp:214-375)
//   solve_pnp / PnPResult Slam.h:120-131          (Slam.cpp:505-529)
//   track_local_map       Slam.h:96               (Slam.cpp:380-469)
//   Frame                 Frame.h:12-72           (Frame.cpp: detect_features :33-38, depth :47-54)
//   MapPoint / Map        MapPoint.h:8-48, Map.h:10-40 (the containers local BA gathers from)
//   Optimizer::project_point / optimize_pose / local_bundle_adjustment
//                         Optimizer.h:24-38       (Optimizer.cpp:26-48, 54-180, 187-599)
//
// OpenCV types are replaced by layout-compatible PODs (KeyPoint == cv::KeyPoint, DMatch ==
// cv::DMatch, Descriptors == an N x 256 CV_32F cv::Mat).  Every compute call goes to the GPU
// through libvslam_hip.so; there is no CPU fallback: failures throw vslam_amd::Error.
#pragma once

#include <array>
#include <cfloat>
#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

struct vs_ctx;

namespace vslam_amd {

struct Point2f {
    float x = 0, y = 0;
};
struct Point3f {
    float x = 0, y = 0, z = 0;
};
struct Point2d {
    double x = 0, y = 0;
};
struct Point3d {
    double x = 0, y = 0, z = 0;
};

// cv::KeyPoint (28 bytes: pt, size, angle, response, octave, class_id)
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
// cv::DMatch (16 bytes)
struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = FLT_MAX;
};

// N x 256 fp32 descriptor matrix (cv::Mat CV_32F, one row per keypoint)
struct Descriptors {
    static constexpr int kCols = 256;
    int rows = 0;
    std::vector<float> data;
    bool empty() const { return rows == 0; }
    const float* row(int i) const { return data.data() + (size_t)i * kCols; }
};

// 8-bit image view: BGR (channels = 3) or gray (channels = 1), row pitch `step` bytes (cv::Mat)
struct Image {
    const uint8_t* data = nullptr;
    int rows = 0, cols = 0, channels = 3;
    size_t step = 0;
};
// fp32 depth in metres (Frame::load_depth_image, Frame.cpp:46-53)
struct DepthImage {
    const float* data = nullptr;
    int rows = 0, cols = 0;
};

using Mat33 = std::array<double, 9>;  // row-major 3x3 (CV_64F)
using Vec3 = std::array<double, 3>;

struct Intrinsics {  // Config.h:14-17 (TUM fr1)
    double fx = 525.0, fy = 525.0, cx = 319.5, cy = 239.5;
};

class Error : public std::runtime_error {
   public:
    Error(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

   private:
    int code_;
};

// One GPU context (device, stream, weights, scratch).  Not thread-safe; one per thread.
class Context {
   public:
    explicit Context(int device = 0, const std::string& weights_path = "");
    ~Context();
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    vs_ctx* get() const { return h_; }
    const Intrinsics& K() const { return K_; }
    void set_intrinsics(const Intrinsics& K) { K_ = K; }

   private:
    vs_ctx* h_ = nullptr;
    Intrinsics K_;
};

// FeatureExtractor (FeatureExtractor.h): SuperPoint on the GPU plus the reference's SPCF binary
// feature cache keyed by the sequential extract index (FeatureExtractor.cpp:49-81, 261-360).
class FeatureExtractor {
   public:
    FeatureExtractor();
    ~FeatureExtractor();
    // Loads SuperPoint weights (VSPW file written by vs_superpoint_save_weights; "" = the seeded
    // synthetic weights) on device 0.  Returns false on failure (the reference then falls back
    // to ORB, which is out of scope here: extract() throws until init succeeds).
    bool init(const std::string& model_path, int device = 0);
    void extract(const Image& image, std::vector<KeyPoint>& keypoints, Descriptors& descriptors);
    bool using_superpoint() const { return ctx_ != nullptr; }
    Context* context() const { return ctx_.get(); }

    void set_cache_path(const std::string& path) { cache_path_ = path; }
    bool load_cache();
    bool save_cache();
    bool cache_active() const { return cache_loaded_; }
    int cache_size() const { return (int)cache_.size(); }

   private:
    struct CachedFeatures {
        std::vector<KeyPoint> keypoints;
        Descriptors descriptors;
    };
    std::unique_ptr<Context> ctx_;
    std::string cache_path_;
    bool cache_loaded_ = false;
    int extract_counter_ = 0;
    std::unordered_map<int, CachedFeatures> cache_;
};

// Slam::match_features: exact 2-NN + Lowe ratio 0.75
std::vector<DMatch> match_features(Context& ctx, const Descriptors& desc1, const Descriptors& desc2,
                                   std::vector<DMatch>* raw_matches_out = nullptr);

// Slam::extract_matched_points (host bookkeeping, as in the reference)
void extract_matched_points(const std::vector<KeyPoint>& kp1, const std::vector<KeyPoint>& kp2,
                            const std::vector<DMatch>& matches, std::vector<Point2f>& pts1,
                            std::vector<Point2f>& pts2);

// Slam.cpp:880-910: F = findFundamentalMat(FM_RANSAC, 3.0, 0.999); when F is non-empty the
// epipolar error is computed before and after and pts/matches keep only the inliers, in order.
struct FundamentalResult {
    bool has_F = false;
    Mat33 F{};
    std::vector<uint8_t> mask;
    double epipolar_error_before = 0, epipolar_error_after = 0;
};
FundamentalResult verify_fundamental(Context& ctx, std::vector<Point2f>& pts1, std::vector<Point2f>& pts2,
                                     std::vector<DMatch>& good_matches);

// Slam::estimate_motion_3d3d (the reference seeds std::mt19937 with 42 + frame_count_, :276)
bool estimate_motion_3d3d(Context& ctx, const std::vector<Point2f>& pts1, const std::vector<Point2f>& pts2,
                          const DepthImage& depth1, const DepthImage& depth2, uint32_t seed, Mat33& R_out,
                          Vec3& t_out);

// Slam::PnPResult / Slam::solve_pnp
struct PnPResult {
    bool success = false;
    Mat33 R_world{};
    Vec3 t_world{};
    int inlier_count = 0;
};
PnPResult solve_pnp(Context& ctx, const std::vector<Point3f>& obj_pts, const std::vector<Point2f>& img_pts,
                    int ransac_iters = 100, int min_inliers = 10);

// Slam::track_local_map over a map held as plain arrays (valid = MapPoint valid && has
// descriptor).  map_point_indices = Frame::map_point_indices (updated in place); observations
// (nullable) receives the (map point, keypoint) pairs MapPoint::add_observation is called with.
struct MapPointsView {
    const double* pos = nullptr;   // n x 3 world
    const float* desc = nullptr;   // n x 256
    const uint8_t* valid = nullptr;
    int n = 0;
};
int track_local_map(Context& ctx, const MapPointsView& map, const std::vector<KeyPoint>& keypoints,
                    const Descriptors& descriptors, const Mat33& R_world, const Vec3& t_world,
                    std::vector<int>& map_point_indices, std::vector<std::pair<int, int>>* observations = nullptr,
                    int img_w = 640, int img_h = 480);

// Frame (Frame.h:12-72): image, features, depth, camera->world pose, keyframe flag and
// map_point_indices.  The reference constructs from a file path (cv::imread + cvtColor,
// Frame.cpp:19-30); decoding is out of scope here, so the caller hands over the decoded 8-bit
// image (copied) — or none, which leaves the frame without features like a failed imread.
class FeatureExtractor;
class Frame {
   public:
    Frame() = default;
    Frame(int id, const Image& image, double timestamp = 0.0);
    // Frame::detect_features (Frame.cpp:33-38): extract, then map_point_indices = -1 per keypoint
    void detect_features(FeatureExtractor& extractor);
    // Frame::load_depth_image (Frame.cpp:47-54) from the decoded 16-bit TUM depth PNG:
    // depth = raw / 5000 m (Config.h:28), raw == 0 -> 0 (invalid)
    void load_depth_image(const uint16_t* raw, int rows, int cols, size_t step_bytes = 0);
    void set_depth_map(const DepthImage& depth);  // Frame::set_depth_map (copied)
    bool has_real_depth() const { return has_real_depth_; }
    DepthImage depth_map() const { return {depth_.data(), has_real_depth_ ? rows_ : 0, has_real_depth_ ? cols_ : 0}; }

    Mat33 get_rotation() const { return R_; }
    Vec3 get_translation() const { return t_; }
    std::array<double, 16> get_pose() const;  // Frame::get_pose (Frame.cpp:100-105): 4x4 [R t; 0 1]
    void set_rotation(const Mat33& R) { R_ = R; }
    void set_translation(const Vec3& t) { t_ = t; }
    void set_pose(const Mat33& R, const Vec3& t) {
        R_ = R;
        t_ = t;
    }
    int id() const { return id_; }
    double timestamp() const { return timestamp_; }
    Image image() const { return {pixels_.data(), rows_, cols_, channels_, (size_t)cols_ * channels_}; }
    const std::vector<KeyPoint>& keypoints() const { return keypoints_; }
    const Descriptors& descriptors() const { return descriptors_; }
    bool is_processed() const { return processed_; }
    bool is_keyframe() const { return is_keyframe_; }
    void set_keyframe(bool kf) { is_keyframe_ = kf; }
    std::vector<int>& map_point_indices() { return map_point_indices_; }
    const std::vector<int>& map_point_indices() const { return map_point_indices_; }

   private:
    int id_ = -1;
    double timestamp_ = 0.0;
    std::vector<uint8_t> pixels_;
    int rows_ = 0, cols_ = 0, channels_ = 3;
    std::vector<KeyPoint> keypoints_;
    Descriptors descriptors_;
    std::vector<float> depth_;
    Mat33 R_{1, 0, 0, 0, 1, 0, 0, 0, 1};
    Vec3 t_{0, 0, 0};
    bool processed_ = false, is_keyframe_ = false, has_real_depth_ = false;
    std::vector<int> map_point_indices_;
};

// MapPoint (MapPoint.h:8-48)
class MapPoint {
   public:
    MapPoint() = default;
    MapPoint(int id, const Point3d& position, const float* descriptor /* 256, nullable */);
    int id() const { return id_; }
    Point3d position() const { return position_; }
    void set_position(const Point3d& p) { position_ = p; }
    const std::vector<float>& descriptor() const { return descriptor_; }
    void add_observation(int frame_id, int keypoint_idx) { observations_.emplace_back(frame_id, keypoint_idx); }
    const std::vector<std::pair<int, int>>& observations() const { return observations_; }
    int observation_count() const { return (int)observations_.size(); }
    bool is_valid() const { return valid_; }
    void set_valid(bool v) { valid_ = v; }
    void increase_visible(int n = 1) { visible_count_ += n; }
    void increase_found(int n = 1) { found_count_ += n; }
    float get_found_ratio() const { return visible_count_ > 0 ? (float)found_count_ / visible_count_ : 0.0f; }
    int visible_count() const { return visible_count_; }
    int found_count() const { return found_count_; }
    void set_first_kf_id(int id) { first_kf_id_ = id; }
    int first_kf_id() const { return first_kf_id_; }

   private:
    int id_ = -1;
    Point3d position_;
    std::vector<std::pair<int, int>> observations_;
    std::vector<float> descriptor_;
    bool valid_ = true;
    int visible_count_ = 0, found_count_ = 0, first_kf_id_ = 0;
};

// Map (Map.h:10-40): frames in insertion order, map points, one mutex
class Map {
   public:
    void add_frame(std::shared_ptr<Frame> f) {
        std::lock_guard<std::mutex> lock(mutex_);
        frames_.push_back(std::move(f));
    }
    void add_map_point(const MapPoint& mp) {
        std::lock_guard<std::mutex> lock(mutex_);
        map_points_.push_back(mp);
    }
    std::shared_ptr<Frame> get_frame(int id) const;
    std::vector<std::shared_ptr<Frame>> get_all_frames() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return frames_;
    }
    int frame_count() const {
        std::lock_guard<std::mutex> lock(mutex_);
        return (int)frames_.size();
    }
    std::vector<std::shared_ptr<Frame>> get_keyframes() const;
    std::vector<MapPoint>& map_points() { return map_points_; }
    const std::vector<MapPoint>& map_points() const { return map_points_; }
    std::vector<std::shared_ptr<Frame>>& frames_direct() { return frames_; }
    std::mutex& mutex() { return mutex_; }

   private:
    std::vector<std::shared_ptr<Frame>> frames_;
    std::vector<MapPoint> map_points_;
    mutable std::mutex mutex_;
};

// Optimizer (Optimizer.h:22-48) over the GPU context.  Loop correction / pose graph optimisation
// (g2o) are out of scope.
class Optimizer {
   public:
    explicit Optimizer(Context& ctx) : ctx_(ctx) {}
    // Optimizer::project_point (Optimizer.cpp:26-48): world point -> pixel for a camera->world pose;
    // (-1, -1) behind the camera (z < 1e-6).  Host arithmetic, the reference's expression order.
    static Point2d project_point(const Point3d& pw, const Mat33& R_world, const Vec3& t_world, const Intrinsics& K);
    // the pose-only LM (Optimizer.cpp:54-180).  The pose is updated in place; returns {rms before,
    // rms after} ({0, 0} and untouched when fewer than 3 points).
    std::pair<double, double> optimize_pose(Mat33& R_world, Vec3& t_world, const std::vector<Point3d>& points_3d,
                                            const std::vector<Point2f>& points_2d);
    // the reference's signature: the frame's pose is read and written (Optimizer.cpp:166-168)
    std::pair<double, double> optimize_pose(const std::shared_ptr<Frame>& frame, const std::vector<Point3d>& points_3d,
                                            const std::vector<Point2f>& points_2d);
    // Optimizer::local_bundle_adjustment (Optimizer.cpp:187-599): the window gather under the map
    // mutex (:205-244: the last window_size keyframes, their valid map points in first-seen order,
    // observations keyframe-major in keypoint order), Schur-complement LM on the GPU (vs_local_ba),
    // write-back of poses 1..N-1 and of the points under the mutex (:580-596).  {0, 0} on bail-out.
    std::pair<double, double> local_bundle_adjustment(Map& map, int window_size = 10);

   private:
    Context& ctx_;
};

}  // namespace vslam_amd
