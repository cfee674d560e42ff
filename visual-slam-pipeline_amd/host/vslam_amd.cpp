// vslam_amd.cpp — C++ façade over the C ABI (see vslam_amd.hpp).  Only bookkeeping lives here
// (argument marshalling, the SPCF cache file, match filtering); all compute is in libvslam_hip.so.
#include "vslam_amd.hpp"

#include <algorithm>
#include <cstring>

#include "vslam_abi.h"

static_assert(sizeof(vslam_amd::KeyPoint) == sizeof(vs_keypoint), "KeyPoint must match vs_keypoint");
static_assert(sizeof(vslam_amd::DMatch) == sizeof(vs_match), "DMatch must match vs_match");

namespace vslam_amd {

namespace {

void check(int rc, const char* where) {
    if (rc != VS_OK) throw Error(rc, std::string(where) + ": " + vs_last_error());
}

std::array<double, 4> kvec(const Intrinsics& K) { return {K.fx, K.fy, K.cx, K.cy}; }

}  // namespace

// ---------------------------------------------------------------------------------- Context
Context::Context(int device, const std::string& weights_path) {
    check(vs_create(device, weights_path.empty() ? nullptr : weights_path.c_str(), &h_), "vs_create");
}

Context::~Context() {
    if (h_) vs_destroy(h_);
}

// ------------------------------------------------------------------------- FeatureExtractor
FeatureExtractor::FeatureExtractor() = default;
FeatureExtractor::~FeatureExtractor() = default;

bool FeatureExtractor::init(const std::string& model_path, int device) {
    try {
        ctx_ = std::make_unique<Context>(device, model_path);
        return true;
    } catch (const Error&) {
        ctx_.reset();
        return false;
    }
}

// FeatureExtractor::extract (FeatureExtractor.cpp:49-81): cache hit by sequential index, else
// extract on the GPU and remember the result when a cache path is set.
void FeatureExtractor::extract(const Image& image, std::vector<KeyPoint>& keypoints, Descriptors& descriptors) {
    const int idx = extract_counter_++;
    if (cache_loaded_) {
        auto it = cache_.find(idx);
        if (it != cache_.end()) {
            keypoints = it->second.keypoints;
            descriptors = it->second.descriptors;
            return;
        }
    }
    if (!ctx_) throw Error(VS_ERR_ARG, "FeatureExtractor::extract: not initialised (init() failed or not called)");
    const int cap = VS_SP_MAX_KEYPOINTS;
    keypoints.resize(cap);
    descriptors.data.resize((size_t)cap * Descriptors::kCols);
    int n = 0;
    check(vs_extract(ctx_->get(), image.data, image.rows, image.cols, image.channels,
                     image.step ? image.step : (size_t)image.cols * image.channels,
                     reinterpret_cast<vs_keypoint*>(keypoints.data()), descriptors.data.data(), cap, &n),
          "vs_extract");
    keypoints.resize(n);
    descriptors.rows = n;
    descriptors.data.resize((size_t)n * Descriptors::kCols);
    if (!cache_path_.empty()) cache_[idx] = CachedFeatures{keypoints, descriptors};
}

// SPCF cache file (FeatureExtractor.cpp:261-381) through the library's reader / writer
// (vs_spcf_read / vs_spcf_write: the reference's byte layout, entries sorted by index).
bool FeatureExtractor::load_cache() {
    if (cache_path_.empty()) return false;
    int count = 0;
    if (vs_spcf_read(cache_path_.c_str(), 0, 0, nullptr, nullptr, nullptr, nullptr, &count) != VS_OK) return false;
    const int cap = VS_SP_MAX_KEYPOINTS;
    std::vector<int> idx(count), n(count);
    std::vector<KeyPoint> kps((size_t)count * cap);
    std::vector<float> desc((size_t)count * cap * Descriptors::kCols);
    if (count > 0 && vs_spcf_read(cache_path_.c_str(), count, cap, idx.data(), reinterpret_cast<vs_keypoint*>(kps.data()),
                                  desc.data(), n.data(), &count) != VS_OK)
        return false;
    std::unordered_map<int, CachedFeatures> cache;
    for (int e = 0; e < count; e++) {
        CachedFeatures cf;
        cf.keypoints.assign(kps.begin() + (size_t)e * cap, kps.begin() + (size_t)e * cap + n[e]);
        cf.descriptors.rows = n[e];
        cf.descriptors.data.assign(desc.begin() + (size_t)e * cap * Descriptors::kCols,
                                   desc.begin() + ((size_t)e * cap + n[e]) * Descriptors::kCols);
        cache[idx[e]] = std::move(cf);
    }
    cache_ = std::move(cache);
    cache_loaded_ = true;
    return true;
}

bool FeatureExtractor::save_cache() {
    if (cache_path_.empty() || cache_.empty()) return false;
    std::vector<int> indices;
    indices.reserve(cache_.size());
    for (const auto& kv : cache_) indices.push_back(kv.first);
    std::sort(indices.begin(), indices.end());
    bool first = true;
    for (int idx : indices) {  // one entry at a time: no second copy of the whole cache
        const CachedFeatures& cf = cache_.at(idx);
        const int n = (int)cf.keypoints.size();
        if (cf.descriptors.rows != n) return false;
        if (vs_spcf_write(cache_path_.c_str(), 1, &idx, reinterpret_cast<const vs_keypoint*>(cf.keypoints.data()),
                          cf.descriptors.data.data(), &n, n, first ? 0 : 1) != VS_OK)
            return false;
        first = false;
    }
    return true;
}

// ------------------------------------------------------------------------------ Slam methods
std::vector<DMatch> match_features(Context& ctx, const Descriptors& desc1, const Descriptors& desc2,
                                   std::vector<DMatch>* raw_matches_out) {
    std::vector<DMatch> raw(std::max(desc1.rows, 1)), good(std::max(desc1.rows, 1));
    int n_raw = 0, n_good = 0;
    check(vs_match_ratio(ctx.get(), desc1.data.data(), desc1.rows, desc2.data.data(), desc2.rows, 0.75f,
                         reinterpret_cast<vs_match*>(raw.data()), &n_raw, reinterpret_cast<vs_match*>(good.data()),
                         &n_good),
          "vs_match_ratio");
    raw.resize(n_raw);
    good.resize(n_good);
    if (raw_matches_out) *raw_matches_out = std::move(raw);
    return good;
}

void extract_matched_points(const std::vector<KeyPoint>& kp1, const std::vector<KeyPoint>& kp2,
                            const std::vector<DMatch>& matches, std::vector<Point2f>& pts1,
                            std::vector<Point2f>& pts2) {
    pts1.clear();
    pts2.clear();
    pts1.reserve(matches.size());
    pts2.reserve(matches.size());
    for (const auto& m : matches) {
        pts1.push_back(kp1[m.queryIdx].pt);
        pts2.push_back(kp2[m.trainIdx].pt);
    }
}

FundamentalResult verify_fundamental(Context& ctx, std::vector<Point2f>& pts1, std::vector<Point2f>& pts2,
                                     std::vector<DMatch>& good_matches) {
    FundamentalResult r;
    const int n = (int)pts1.size();
    if (pts2.size() != pts1.size() || good_matches.size() != pts1.size())
        throw Error(VS_ERR_ARG, "verify_fundamental: pts1 / pts2 / good_matches sizes differ");
    r.mask.assign(std::max(n, 1), 0);
    int ok = 0, diag[4];
    double err[2];
    check(vs_find_fundamental(ctx.get(), reinterpret_cast<const float*>(pts1.data()),
                              reinterpret_cast<const float*>(pts2.data()), n, 3.0, 0.999, 1000, r.F.data(),
                              r.mask.data(), &ok, diag, err),
          "vs_find_fundamental");
    r.mask.resize(n);
    r.has_F = ok != 0;
    if (!r.has_F) return r;  // Slam.cpp:887, 892: nothing filtered without F
    r.epipolar_error_before = err[0];
    r.epipolar_error_after = err[1];
    size_t w = 0;
    for (int i = 0; i < n; i++)
        if (r.mask[i]) {
            pts1[w] = pts1[i];
            pts2[w] = pts2[i];
            good_matches[w] = good_matches[i];
            w++;
        }
    pts1.resize(w);
    pts2.resize(w);
    good_matches.resize(w);
    return r;
}

bool estimate_motion_3d3d(Context& ctx, const std::vector<Point2f>& pts1, const std::vector<Point2f>& pts2,
                          const DepthImage& depth1, const DepthImage& depth2, uint32_t seed, Mat33& R_out,
                          Vec3& t_out) {
    if (pts1.size() != pts2.size()) throw Error(VS_ERR_ARG, "estimate_motion_3d3d: point counts differ");
    if (depth1.rows != depth2.rows || depth1.cols != depth2.cols)
        throw Error(VS_ERR_ARG, "estimate_motion_3d3d: depth sizes differ");
    const auto K = kvec(ctx.K());
    int ok = 0, diag[4];
    check(vs_ransac_3d3d(ctx.get(), reinterpret_cast<const float*>(pts1.data()),
                         reinterpret_cast<const float*>(pts2.data()), (int)pts1.size(), depth1.data, depth2.data,
                         depth1.rows, depth1.cols, K.data(), seed, 200, 0.05, R_out.data(), t_out.data(), &ok,
                         diag),
          "vs_ransac_3d3d");
    return ok != 0;
}

PnPResult solve_pnp(Context& ctx, const std::vector<Point3f>& obj_pts, const std::vector<Point2f>& img_pts,
                    int ransac_iters, int min_inliers) {
    if (obj_pts.size() != img_pts.size()) throw Error(VS_ERR_ARG, "solve_pnp: point counts differ");
    PnPResult r;
    const auto K = kvec(ctx.K());
    int success = 0;
    check(vs_solve_pnp(ctx.get(), reinterpret_cast<const float*>(obj_pts.data()),
                       reinterpret_cast<const float*>(img_pts.data()), (int)obj_pts.size(), K.data(), ransac_iters,
                       min_inliers, r.R_world.data(), r.t_world.data(), &success, &r.inlier_count, nullptr,
                       nullptr),
          "vs_solve_pnp");
    r.success = success != 0;
    return r;
}

int track_local_map(Context& ctx, const MapPointsView& map, const std::vector<KeyPoint>& keypoints,
                    const Descriptors& descriptors, const Mat33& R_world, const Vec3& t_world,
                    std::vector<int>& map_point_indices, std::vector<std::pair<int, int>>* observations, int img_w,
                    int img_h) {
    const int n_kp = (int)keypoints.size();
    if (descriptors.rows != n_kp) throw Error(VS_ERR_ARG, "track_local_map: descriptor rows != keypoints");
    map_point_indices.resize(n_kp, -1);
    const auto K = kvec(ctx.K());
    int tracked = 0, n_obs = 0;
    const int obs_cap = n_kp;  // at most one observation per keypoint
    std::vector<int> obs_mp(std::max(obs_cap, 1)), obs_kp(std::max(obs_cap, 1));
    check(vs_track_local_map(ctx.get(), map.pos, map.desc, map.valid, map.n,
                             reinterpret_cast<const vs_keypoint*>(keypoints.data()), descriptors.data.data(), n_kp,
                             R_world.data(), t_world.data(), K.data(), img_w, img_h, map_point_indices.data(),
                             &tracked, obs_mp.data(), obs_kp.data(), obs_cap, &n_obs),
          "vs_track_local_map");
    if (observations) {
        observations->clear();
        for (int i = 0; i < std::min(n_obs, obs_cap); i++) observations->emplace_back(obs_mp[i], obs_kp[i]);
    }
    return tracked;
}

std::pair<double, double> Optimizer::optimize_pose(Mat33& R_world, Vec3& t_world,
                                                   const std::vector<Point3d>& points_3d,
                                                   const std::vector<Point2f>& points_2d) {
    if (points_3d.size() != points_2d.size()) throw Error(VS_ERR_ARG, "optimize_pose: point counts differ");
    const auto K = kvec(ctx_.K());
    double before = 0, after = 0;
    check(vs_optimize_pose(ctx_.get(), reinterpret_cast<const double*>(points_3d.data()),
                           reinterpret_cast<const float*>(points_2d.data()), (int)points_3d.size(), K.data(),
                           R_world.data(), t_world.data(), &before, &after),
          "vs_optimize_pose");
    return {before, after};
}

std::pair<double, double> Optimizer::optimize_pose(const std::shared_ptr<Frame>& frame,
                                                   const std::vector<Point3d>& points_3d,
                                                   const std::vector<Point2f>& points_2d) {
    if (!frame) throw Error(VS_ERR_ARG, "optimize_pose: null frame");
    Mat33 R = frame->get_rotation();
    Vec3 t = frame->get_translation();
    const auto r = optimize_pose(R, t, points_3d, points_2d);
    frame->set_pose(R, t);
    return r;
}

Point2d Optimizer::project_point(const Point3d& pw, const Mat33& R, const Vec3& t, const Intrinsics& K) {
    // R_cam = R^T, t_cam = -R_cam t, pc = R_cam Pw + t_cam (Optimizer.cpp:30-34)
    double tc[3], pc[3];
    for (int i = 0; i < 3; i++) tc[i] = -(R[0 * 3 + i] * t[0] + R[1 * 3 + i] * t[1] + R[2 * 3 + i] * t[2]);
    for (int i = 0; i < 3; i++) pc[i] = (R[0 * 3 + i] * pw.x + R[1 * 3 + i] * pw.y + R[2 * 3 + i] * pw.z) + tc[i];
    const double z = pc[2];
    if (z < 1e-6) return {-1, -1};
    return {K.fx * pc[0] / z + K.cx, K.fy * pc[1] / z + K.cy};
}

std::pair<double, double> Optimizer::local_bundle_adjustment(Map& map, int window_size) {
    std::vector<std::shared_ptr<Frame>> keyframes;
    std::vector<int> mp_global_ids;
    std::vector<double> points;
    std::vector<int> okf, opt;
    std::vector<double> ouv;
    {
        std::lock_guard<std::mutex> lock(map.mutex());
        const auto& mps = map.map_points();
        for (const auto& f : map.frames_direct())
            if (f->is_keyframe()) keyframes.push_back(f);
        const int start = std::max(0, (int)keyframes.size() - window_size);
        keyframes.erase(keyframes.begin(), keyframes.begin() + start);
        if ((int)keyframes.size() < 2) return {0, 0};
        std::unordered_map<int, int> local;
        for (int ki = 0; ki < (int)keyframes.size(); ki++) {
            const auto& idx = keyframes[ki]->map_point_indices();
            const auto& kps = keyframes[ki]->keypoints();
            for (int kpi = 0; kpi < (int)idx.size(); kpi++) {
                const int mp = idx[kpi];
                if (mp < 0 || mp >= (int)mps.size() || !mps[mp].is_valid()) continue;
                auto it = local.find(mp);
                int pt;
                if (it == local.end()) {
                    pt = (int)mp_global_ids.size();
                    local[mp] = pt;
                    mp_global_ids.push_back(mp);
                    const Point3d p = mps[mp].position();
                    points.insert(points.end(), {p.x, p.y, p.z});
                } else {
                    pt = it->second;
                }
                okf.push_back(ki);
                opt.push_back(pt);
                ouv.insert(ouv.end(), {(double)kps[kpi].pt.x, (double)kps[kpi].pt.y});
            }
        }
    }
    const int N = (int)keyframes.size(), M = (int)mp_global_ids.size(), n_obs = (int)okf.size();
    if (n_obs < 20 || M < 10) return {0, 0};  // Optimizer.cpp:250
    if (N > VS_BA_MAX_KEYFRAMES) throw Error(VS_ERR_ARG, "local_bundle_adjustment: window larger than VS_BA_MAX_KEYFRAMES");
    std::vector<double> R((size_t)N * 9), t((size_t)N * 3);
    for (int i = 0; i < N; i++) {
        const Mat33 Ri = keyframes[i]->get_rotation();
        const Vec3 ti = keyframes[i]->get_translation();
        std::copy(Ri.begin(), Ri.end(), R.begin() + 9 * i);
        std::copy(ti.begin(), ti.end(), t.begin() + 3 * i);
    }
    const auto K = kvec(ctx_.K());
    double before = 0, after = 0;
    int stats[3] = {0, 0, 0};
    check(vs_local_ba(ctx_.get(), N, R.data(), t.data(), M, points.data(), n_obs, okf.data(), opt.data(), ouv.data(),
                      K.data(), 15, &before, &after, stats),
          "vs_local_ba");
    {
        std::lock_guard<std::mutex> lock(map.mutex());  // :580-596
        auto& mps = map.map_points();
        for (int i = 1; i < N; i++) {
            Mat33 Ri;
            Vec3 ti;
            std::copy(R.begin() + 9 * i, R.begin() + 9 * i + 9, Ri.begin());
            std::copy(t.begin() + 3 * i, t.begin() + 3 * i + 3, ti.begin());
            keyframes[i]->set_pose(Ri, ti);
        }
        for (int j = 0; j < M; j++) {
            const int gid = mp_global_ids[j];
            if (gid >= 0 && gid < (int)mps.size() && mps[gid].is_valid())
                mps[gid].set_position({points[3 * j], points[3 * j + 1], points[3 * j + 2]});
        }
    }
    return {before, after};
}

// ----------------------------------------------------------------------- Frame / MapPoint / Map
Frame::Frame(int id, const Image& image, double timestamp) : id_(id), timestamp_(timestamp) {
    if (!image.data || image.rows <= 0 || image.cols <= 0) return;  // like a failed cv::imread
    if (image.channels != 3 && image.channels != 1) throw Error(VS_ERR_ARG, "Frame: 1 or 3 channels");
    rows_ = image.rows;
    cols_ = image.cols;
    channels_ = image.channels;
    const size_t row_bytes = (size_t)cols_ * channels_, step = image.step ? image.step : row_bytes;
    pixels_.resize(row_bytes * rows_);
    for (int r = 0; r < rows_; r++) std::memcpy(pixels_.data() + r * row_bytes, image.data + r * step, row_bytes);
}

void Frame::detect_features(FeatureExtractor& extractor) {
    if (pixels_.empty()) return;  // Frame.cpp:34 (gray_ empty)
    extractor.extract(image(), keypoints_, descriptors_);
    map_point_indices_.assign(keypoints_.size(), -1);
    processed_ = true;
}

void Frame::load_depth_image(const uint16_t* raw, int rows, int cols, size_t step_bytes) {
    if (!raw || rows <= 0 || cols <= 0) return;  // Frame.cpp:49 (empty image)
    const size_t step = step_bytes ? step_bytes : (size_t)cols * 2;
    depth_.assign((size_t)rows * cols, 0.0f);
    for (int r = 0; r < rows; r++) {
        const uint16_t* src = reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(raw) + r * step);
        for (int c = 0; c < cols; c++)  // convertTo(CV_32F, 1 / 5000) then setTo(0, raw == 0)
            depth_[(size_t)r * cols + c] = src[c] ? (float)src[c] * (float)(1.0 / 5000.0) : 0.0f;
    }
    rows_ = rows_ ? rows_ : rows;
    cols_ = cols_ ? cols_ : cols;
    has_real_depth_ = true;
}

void Frame::set_depth_map(const DepthImage& d) {
    depth_.assign(d.data, d.data + (size_t)d.rows * d.cols);
    rows_ = rows_ ? rows_ : d.rows;
    cols_ = cols_ ? cols_ : d.cols;
    has_real_depth_ = true;
}

std::array<double, 16> Frame::get_pose() const {
    return {R_[0], R_[1], R_[2], t_[0], R_[3], R_[4], R_[5], t_[1], R_[6], R_[7], R_[8], t_[2], 0, 0, 0, 1};
}

MapPoint::MapPoint(int id, const Point3d& position, const float* descriptor) : id_(id), position_(position) {
    if (descriptor) descriptor_.assign(descriptor, descriptor + Descriptors::kCols);
}

std::shared_ptr<Frame> Map::get_frame(int id) const {
    std::lock_guard<std::mutex> lock(mutex_);
    for (const auto& f : frames_)
        if (f->id() == id) return f;
    return nullptr;
}

std::vector<std::shared_ptr<Frame>> Map::get_keyframes() const {
    std::lock_guard<std::mutex> lock(mutex_);
    std::vector<std::shared_ptr<Frame>> out;
    for (const auto& f : frames_)
        if (f->is_keyframe()) out.push_back(f);
    return out;
}

}  // namespace vslam_amd
