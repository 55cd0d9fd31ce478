/* slamhot.hpp — C++ host layer over the slamhot C ABI (include/slamhot.h).
 *
 * The reference's host code is C++ (ORB_SLAM3::ORBextractor, ORB_SLAM3::ORBmatcher,
 * ORB_SLAM3::Optimizer).  These classes keep its names, argument meaning and error
 * behaviour, so a Tracking / LocalMapping port calls them the way it calls the originals;
 * only the OpenCV / map types are replaced by plain views (the shims in INTEGRATION.md do
 * the cv::Mat / KeyFrame conversion on top of this header).  Every method is a thin call
 * into libslamhot.so: all computation runs on the gfx950 device, and a missing device or
 * library surfaces as slamhot::Error (SLAM_ENODEV), never as a CPU fallback.
 *
 * Header-only; link with -lslamhot.  Thread-safety follows the reference: one extractor per
 * camera used by one thread at a time, matchers and solvers per calling thread.
 */
#ifndef SLAMHOT_HPP
#define SLAMHOT_HPP

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "slamhot.h"

namespace slamhot {

class Error : public std::runtime_error {
   public:
    Error(slam_status st, const std::string& what)
        : std::runtime_error(what + ": " + slamhot_status_string(st)), status(st) {}
    slam_status status;
};

inline void check(slam_status st, const char* what) {
    if (st != SLAM_OK) throw Error(st, what);
}

/* cv::KeyPoint memory layout (pt.x, pt.y, size, angle, response, octave, class_id). */
using KeyPoint = slam_keypoint;

/* A CV_8UC1 image as the reference passes it (cv::InputArray of a grayscale Mat). */
struct GrayImage {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;  // bytes per row
    bool empty() const { return data == nullptr || cols <= 0 || rows <= 0; }
};

/* Owning 8-bit matrix: descriptors (N x 32) and pyramid levels. */
struct Mat8U {
    int rows = 0, cols = 0;
    std::vector<uint8_t> data;
    const uint8_t* row(int r) const { return data.data() + (size_t)r * cols; }
};

/* ------------------------------------------------------------------------------------
 * ORBextractor (ORBextractor.h:45-111).  Construction mirrors
 * ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
 * (ORBextractor.cc:408-468); the device handle is sized for the frames it sees.
 * ---------------------------------------------------------------------------------- */
class ORBextractor {
   public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                 int device = 0)
        : device_(device) {
        prm_.nfeatures = nfeatures;
        prm_.scale_factor = scaleFactor;
        prm_.nlevels = nlevels;
        prm_.ini_th_fast = iniThFAST;
        prm_.min_th_fast = minThFAST;
        reserve(752, 480);  // EuRoC; grown on the first larger frame
        int nl = 0;
        check(slamhot_extractor_levels(ex_, &nl, nullptr, nullptr, nullptr, nullptr, nullptr), "levels");
        scale_.resize(nl);
        inv_scale_.resize(nl);
        sigma2_.resize(nl);
        inv_sigma2_.resize(nl);
        nfeat_.resize(nl);
        check(slamhot_extractor_levels(ex_, &nl, scale_.data(), inv_scale_.data(), sigma2_.data(),
                                       inv_sigma2_.data(), nfeat_.data()),
              "levels");
    }
    ~ORBextractor() { slamhot_extractor_destroy(ex_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    /* int operator()(InputArray image, InputArray mask, vector<KeyPoint>& keypoints,
     *                OutputArray descriptors, vector<int>& vLappingArea)
     * (ORBextractor.cc:1068-1150): returns monoIndex, or -1 for an empty image (:1072-1073,
     * outputs untouched).  The mask is ignored by the reference as well. */
    int operator()(const GrayImage& image, std::vector<KeyPoint>& keypoints, Mat8U& descriptors,
                   const std::vector<int>& vLappingArea) {
        if (image.empty()) return -1;
        reserve(image.cols, image.rows);
        const int lap0 = vLappingArea.size() > 0 ? vLappingArea[0] : 0;
        const int lap1 = vLappingArea.size() > 1 ? vLappingArea[1] : 0;
        int cap = 2 * prm_.nfeatures + 64, n = 0, mono = 0;
        for (int attempt = 0; attempt < 2; attempt++) {
            keypoints.resize(cap);
            descriptors.data.resize((size_t)cap * 32);
            const slam_status st = slamhot_extract(ex_, image.data, image.cols, image.rows,
                                                   image.step ? image.step : (size_t)image.cols, lap0, lap1,
                                                   keypoints.data(), descriptors.data.data(), cap, &n, &mono);
            if (st == SLAM_ECAP && attempt == 0) { cap = n; continue; }
            if (st == SLAM_EEMPTY) return -1;
            check(st, "ORBextractor::operator()");
            break;
        }
        keypoints.resize(n);
        descriptors.rows = n;
        descriptors.cols = 32;
        descriptors.data.resize((size_t)n * 32);
        last_frames_ = 1;
        return mono;
    }

    int inline GetLevels() const { return (int)scale_.size(); }
    float inline GetScaleFactor() const { return prm_.scale_factor; }
    std::vector<float> inline GetScaleFactors() const { return scale_; }
    std::vector<float> inline GetInverseScaleFactors() const { return inv_scale_; }
    std::vector<float> inline GetScaleSigmaSquares() const { return sigma2_; }
    std::vector<float> inline GetInverseScaleSigmaSquares() const { return inv_sigma2_; }
    /* mnFeaturesPerLevel (private in the reference, ORBextractor.h:99) */
    std::vector<int> GetFeaturesPerLevel() const { return nfeat_; }

    /* public std::vector<cv::Mat> mvImagePyramid (ORBextractor.h:83): host copies of the
     * last frame's levels (the device pyramid stays where k_stereo_* reads it). */
    std::vector<Mat8U> mvImagePyramid() const {
        std::vector<Mat8U> out;
        if (!last_frames_) return out;
        for (int l = 0; l < GetLevels(); l++) {
            Mat8U m;
            int w = 0, h = 0;
            check(slamhot_pyramid_level(ex_, 0, l, nullptr, 0, &w, &h), "pyramid_level size");
            m.cols = w;
            m.rows = h;
            m.data.resize((size_t)w * h);
            check(slamhot_pyramid_level(ex_, 0, l, m.data.data(), m.data.size(), &w, &h), "pyramid_level");
            out.push_back(std::move(m));
        }
        return out;
    }

    slam_extractor* handle() { return ex_; }

   private:
    void reserve(int w, int h) {
        if (ex_ && w <= max_w_ && h <= max_h_) return;
        if (ex_) slamhot_extractor_destroy(ex_);
        ex_ = nullptr;
        max_w_ = std::max(w, max_w_);
        max_h_ = std::max(h, max_h_);
        check(slamhot_extractor_create(&prm_, device_, max_w_, max_h_, 1, &ex_), "ORBextractor");
    }
    slam_orb_params prm_{};
    int device_ = 0, max_w_ = 0, max_h_ = 0, last_frames_ = 0;
    slam_extractor* ex_ = nullptr;
    std::vector<float> scale_, inv_scale_, sigma2_, inv_sigma2_;
    std::vector<int> nfeat_;
};

/* ------------------------------------------------------------------------------------
 * Frame construction after extraction (Frame.cc:730-792) for a Pinhole camera with OpenCV
 * distortion mDistCoef = (k1, k2, p1, p2[, k3]).
 * ---------------------------------------------------------------------------------- */
struct PinholeCalib {
    float K[4] = {0, 0, 0, 0};  // fx, fy, cx, cy (Pinhole::toK() and mK)
    std::vector<float> dist;    // mDistCoef
};

/* void Frame::UndistortKeyPoints() (Frame.cc:730-763) */
inline void UndistortKeyPoints(const PinholeCalib& c, const std::vector<KeyPoint>& mvKeys, std::vector<KeyPoint>& mvKeysUn,
                               int device = 0) {
    mvKeysUn.resize(mvKeys.size());
    check(slamhot_undistort_keypoints(device, c.K, c.dist.data(), (int)c.dist.size(), (int)mvKeys.size(),
                                      mvKeys.data(), mvKeysUn.data()),
          "UndistortKeyPoints");
}

/* void Frame::ComputeImageBounds(const cv::Mat&) (Frame.cc:765-792): {mnMinX, mnMaxX, mnMinY, mnMaxY} */
inline std::vector<float> ComputeImageBounds(const PinholeCalib& c, int cols, int rows) {
    std::vector<float> b(4);
    check(slamhot_image_bounds(c.K, c.dist.data(), (int)c.dist.size(), cols, rows, b.data()), "ComputeImageBounds");
    return b;
}

/* ------------------------------------------------------------------------------------
 * ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary.h:29-30),
 * resident on one device.  DBoW2::BowVector / FeatureVector come back as sorted pairs, the order
 * their std::maps iterate in.
 * ---------------------------------------------------------------------------------- */
using BowVector = std::vector<std::pair<uint32_t, double>>;                   // (WordId, WordValue)
using FeatureVector = std::vector<std::pair<uint32_t, std::vector<uint32_t>>>;  // (NodeId, features)

class Vocabulary {
   public:
    /* bool loadFromTextFile(const std::string&) (TemplatedVocabulary.h:1350-1436): ORBvoc.txt */
    explicit Vocabulary(const std::string& path, int device = 0) {
        check(slamhot_vocab_load_text(device, path.c_str(), &v_), "ORBVocabulary::loadFromTextFile");
    }
    /* a node table in DBoW2 order (slamhot_vocab_create) */
    Vocabulary(int device, int k, int L, int scoring, int weighting, int n_nodes, const int32_t* parent,
               const uint8_t* is_leaf, const uint8_t* desc, const double* weight) {
        check(slamhot_vocab_create(device, k, L, scoring, weighting, n_nodes, parent, is_leaf, desc, weight, &v_),
              "ORBVocabulary");
    }
    ~Vocabulary() { slamhot_vocab_destroy(v_); }
    Vocabulary(const Vocabulary&) = delete;
    Vocabulary& operator=(const Vocabulary&) = delete;

    /* void transform(const vector<TDescriptor>& features, BowVector& v, FeatureVector& fv,
     * int levelsup) (TemplatedVocabulary.h:1139-1206) over n descriptors of 32 bytes, row-contiguous */
    void transform(const uint8_t* desc, int n, BowVector& v, FeatureVector& fv, int levelsup) {
        std::vector<uint32_t> word(n), node(n), feat(n);
        std::vector<double> value(n);
        std::vector<int32_t> off(n + 1);
        int nw = 0, nn = 0;
        check(slamhot_compute_bow(v_, n, desc, levelsup, &nw, word.data(), value.data(), &nn, node.data(), off.data(),
                                  feat.data()),
              "ORBVocabulary::transform");
        v.resize(nw);
        for (int j = 0; j < nw; j++) v[j] = {word[j], value[j]};
        fv.resize(nn);
        for (int j = 0; j < nn; j++) fv[j] = {node[j], std::vector<uint32_t>(feat.begin() + off[j], feat.begin() + off[j + 1])};
    }

    slam_vocab* handle() { return v_; }

   private:
    slam_vocab* v_ = nullptr;
};

/* ------------------------------------------------------------------------------------
 * ORBmatcher (ORBmatcher.h:36-110).  The KeyFrame / Frame arguments arrive as their
 * matcher-relevant views; the MapPoint* outputs as indices into the other side (-1 = NULL).
 * ---------------------------------------------------------------------------------- */
struct KeyFrameBow : slam_bow_side {};  // pKF: descriptors, angles, MapPoint validity, mFeatVec
struct FrameBow : slam_bow_side {};     // F: descriptors, angles, mFeatVec (valid ignored)

/* The device half of a matcher: one slam_matcher handle (device scratch + a private stream).
 * The reference builds ORBmatcher(nnratio, checkOri) on the stack at every call site, with a
 * different ratio per site on the same thread (Tracking.cc:2566 0.7, :2700 0.9, :3475 0.75,
 * :3218 0.8), so the handle lives once per (thread, device) and every ORBmatcher is a light view
 * over it carrying its own nnratio / checkOri.  A slam_matcher is not shared between threads. */
class MatcherDevice {
   public:
    explicit MatcherDevice(int device) { check(slamhot_matcher_create(device, &m_), "ORBmatcher"); }
    ~MatcherDevice() { slamhot_matcher_destroy(m_); }
    MatcherDevice(const MatcherDevice&) = delete;
    MatcherDevice& operator=(const MatcherDevice&) = delete;
    slam_matcher* handle() const { return m_; }

    /* this thread's handle on `device`, created on first use, destroyed at thread exit */
    static slam_matcher* ForThisThread(int device) {
        static thread_local std::vector<std::pair<int, std::unique_ptr<MatcherDevice>>> per_device;
        for (auto& d : per_device)
            if (d.first == device) return d.second->handle();
        per_device.emplace_back(device, std::unique_ptr<MatcherDevice>(new MatcherDevice(device)));
        return per_device.back().second->handle();
    }

   private:
    slam_matcher* m_ = nullptr;
};

class ORBmatcher {
   public:
    static constexpr int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;  // ORBmatcher.h:90-92

    /* ORBmatcher(float nnratio, bool checkOri) (ORBmatcher.cc:36-39): cheap to construct per call,
     * as the reference does; the device handle is the calling thread's (MatcherDevice). */
    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
        : nnratio_(nnratio), check_ori_(checkOri), m_(MatcherDevice::ForThisThread(device)) {}
    ORBmatcher(const ORBmatcher&) = delete;
    ORBmatcher& operator=(const ORBmatcher&) = delete;
    float NNratio() const { return nnratio_; }
    bool CheckOrientation() const { return check_ori_; }

    /* static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) (ORBmatcher.cc:
     * 2561-2577): bit-set count of a XOR b over 8 x 32 bits.  A host utility in the
     * reference too (MapPoint::ComputeDistinctiveDescriptors etc. call it on the CPU). */
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) {
        int dist = 0;
        for (int i = 0; i < 8; i++) {
            uint32_t x, y;
            std::memcpy(&x, a + 4 * i, 4);
            std::memcpy(&y, b + 4 * i, 4);
            dist += __builtin_popcount(x ^ y);
        }
        return dist;
    }

    /* int SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
     * (ORBmatcher.cc:269-471): vpMapPointMatches[i] = KF feature whose MapPoint F's
     * feature i took, -1 = NULL.  Returns nmatches. */
    int SearchByBoW(const KeyFrameBow& KF, const FrameBow& F, std::vector<int>& vpMapPointMatches) {
        vpMapPointMatches.assign(F.n, -1);
        a2b_.assign(KF.n, -1);
        int n = 0;
        check(slamhot_search_by_bow(m_, &KF, &F, nnratio_, check_ori_, 0, a2b_.data(), vpMapPointMatches.data(), &n),
              "SearchByBoW(KF, F)");
        return n;
    }

    /* int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
     * (ORBmatcher.cc:823-963): vpMatches12[i] = KF2 feature matched by KF1 feature i. */
    int SearchByBoW(const KeyFrameBow& KF1, const KeyFrameBow& KF2, std::vector<int>& vpMatches12) {
        vpMatches12.assign(KF1.n, -1);
        b2a_.assign(KF2.n, -1);
        int n = 0;
        check(slamhot_search_by_bow(m_, &KF1, &KF2, nnratio_, check_ori_, 1, vpMatches12.data(), b2a_.data(), &n),
              "SearchByBoW(KF1, KF2)");
        return n;
    }

    /* int SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th,
     * const bool bFarPoints, const float thFarPoints) (ORBmatcher.cc:44-214): vpMapPoints as the
     * tracking records Frame::isInFrustum left (slam_mp_track) + their descriptors (32 B each);
     * f_match[i] = the MapPoint index F's feature i took (-1 = untouched).  Returns nmatches. */
    int SearchByProjection(const slam_frame_view& F, const std::vector<slam_mp_track>& vpMapPoints,
                           const uint8_t* mp_desc, float th, bool bFarPoints, float thFarPoints,
                           std::vector<int>& f_match) {
        f_match.assign(F.n, -1);
        int n = 0;
        check(slamhot_search_by_projection_local(m_, &F, (int)vpMapPoints.size(), vpMapPoints.data(), mp_desc,
                                                 nnratio_, th, bFarPoints, thFarPoints, f_match.data(), &n),
              "SearchByProjection(F, vpMapPoints)");
        return n;
    }

    /* int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th,
     * const bool bMono) (ORBmatcher.cc:2173-2389).  f_match[i]: the LastFrame feature whose MapPoint
     * CurrentFrame.mvpMapPoints[i] now holds, -1 untouched, -2 set to NULL by the rotation check
     * (the same convention for the KeyFrame variant below). */
    int SearchByProjection(const slam_frame_view& CurrentFrame, const slam_last_frame& LastFrame, float th, bool bMono,
                           std::vector<int>& f_match) {
        f_match.assign(CurrentFrame.n, -1);
        int n = 0;
        check(slamhot_search_by_projection_last(m_, &CurrentFrame, &LastFrame, nnratio_, check_ori_, th, bMono,
                                                f_match.data(), &n),
              "SearchByProjection(F, LastFrame)");
        return n;
    }

    /* int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
     * sAlreadyFound, const float th, const int ORBdist) (ORBmatcher.cc:2391-2513): the KeyFrame's
     * MapPoints with sAlreadyFound folded into slam_kf_points::use. */
    int SearchByProjection(const slam_frame_view& CurrentFrame, const slam_kf_points& KF, float th, int ORBdist,
                           std::vector<int>& f_match) {
        f_match.assign(CurrentFrame.n, -1);
        int n = 0;
        check(slamhot_search_by_projection_kf(m_, &CurrentFrame, &KF, nnratio_, check_ori_, th, ORBdist,
                                              f_match.data(), &n),
              "SearchByProjection(F, KF, sAlreadyFound)");
        return n;
    }

    /* Tracking::SearchLocalPoints' projection half (Tracking.cc:3213-3258): Frame::isInFrustum
     * for every local MapPoint and SearchByProjection on the ones in view, one device call.
     * track (n_mp) receives the isInFrustum records; returns nmatches, *nToMatch as the reference. */
    int SearchLocalPoints(const slam_frame_view& F, const std::vector<slam_mp_geom>& vpLocalMapPoints,
                          const uint8_t* mp_desc, float viewCosLimit, float th, bool bFarPoints, float thFarPoints,
                          std::vector<slam_mp_track>& track, int& nToMatch, std::vector<int>& f_match) {
        f_match.assign(F.n, -1);
        track.resize(vpLocalMapPoints.size());
        int n = 0;
        check(slamhot_search_local_points(m_, &F, (int)vpLocalMapPoints.size(), vpLocalMapPoints.data(), mp_desc,
                                          viewCosLimit, nnratio_, th, bFarPoints, thFarPoints, track.data(),
                                          &nToMatch, f_match.data(), &n),
              "SearchLocalPoints");
        return n;
    }

    slam_matcher* handle() { return m_; }

   private:
    float nnratio_;
    bool check_ori_;
    slam_matcher* m_ = nullptr;
    std::vector<int> a2b_, b2a_;  // the ABI's other-direction output (unused by the caller)
};

/* ------------------------------------------------------------------------------------
 * Optimizer::LocalBundleAdjustment (Optimizer.h:59, Optimizer.cc:1611-2078) over a window
 * the caller has built and flattened (Optimizer.cc:1613-1718; INTEGRATION.md shim).
 * ---------------------------------------------------------------------------------- */
struct LocalBAWindow {
    std::vector<float> kf_Tcw;        // n_kf x 16, KeyFrame::GetPose(), mnId order
    std::vector<uint8_t> kf_fixed;    // 0 free, 1 the map's init KF (setFixed, in lLocalKeyFrames), 2 lFixedCameras
    std::vector<float> pt_pos;        // n_pt x 3
    std::vector<int32_t> edge_pt, edge_kf;
    std::vector<float> edge_obs;      // n_edge x 3 (u, v, uRight < 0 -> mono)
    std::vector<float> edge_inv_sigma2;
    slam_camera cam{};
    // right-camera observations (EdgeSE3ProjectXYZToBody, Optimizer.cc:1883-1914): empty = none
    std::vector<uint8_t> edge_body;   // n_edge, 1 = body edge (edge_obs = right keypoint)
    std::vector<float> kf_Trl;        // n_kf x 16, KeyFrame::mTrl
    slam_camera cam2{};               // mpCamera2 parameters
    // a camera per KeyFrame (pKFi->fx..mbf / mpCamera2, Optimizer.cc:1840, 1869-1873, 1906):
    // empty = cam / cam2 for every KeyFrame
    std::vector<slam_camera> kf_cam, kf_cam2;
    bool inertial = false;            // pMap->IsInertial(): lambda0 = 100 (Optimizer.cc:1726)
    int n_kf() const { return (int)kf_fixed.size(); }
    int n_pt() const { return (int)pt_pos.size() / 3; }
    int n_edge() const { return (int)edge_pt.size(); }
};

struct LocalBAResult {
    std::vector<float> kf_Tcw, pt_pos;
    std::vector<uint8_t> edge_outlier;  // vToErase (Optimizer.cc:1995-2038)
    int iterations[2] = {0, 0}, trials = 0, n_outlier = 0;
    double chi2_initial = 0, chi2_final = 0;
    bool ran = false;  // false: *pbStopFlag was set on entry, nothing to write back (Optimizer.cc:1921-1923)
};

class LocalBundleAdjuster {
   public:
    /* warm: solve one synthetic window of warm_kf x warm_pt x warm_obs at construction
     * (slamhot_lba_warmup) so the first LocalBundleAdjustment is not the one that loads kernels and
     * allocates; the default is the config-4 window (50 KeyFrames, 2000 MapPoints, 8 observations).
     * That costs one solve (~3 ms) per construction and can throw a warm-up error: batched users
     * and short-lived handles pass warm = false ("LocalBundleAdjuster"). */
    explicit LocalBundleAdjuster(int device = 0, bool warm = true, int warm_kf = 50, int warm_pt = 2000,
                                 int warm_obs = 8) {
        check(slamhot_lba_create(device, &s_), "LocalBundleAdjuster");
        if (warm) {
            const slam_status st = slamhot_lba_warmup(s_, warm_kf, warm_pt, warm_obs);
            if (st != SLAM_OK) {
                slamhot_lba_destroy(s_);
                throw Error(st, "LocalBundleAdjuster warm-up");
            }
        }
    }
    ~LocalBundleAdjuster() { slamhot_lba_destroy(s_); }
    LocalBundleAdjuster(const LocalBundleAdjuster&) = delete;
    LocalBundleAdjuster& operator=(const LocalBundleAdjuster&) = delete;

    /* Many independent windows in one call (batched mode); pbStopFlag as the reference's. */
    void Solve(const std::vector<LocalBAWindow>& ws, const bool* pbStopFlag, std::vector<LocalBAResult>& out) {
        const int n = (int)ws.size();
        out.assign(n, LocalBAResult{});
        std::vector<const LocalBAWindow*> wp(n);
        for (int i = 0; i < n; i++) wp[i] = &ws[i];
        solve(wp.data(), out.data(), n, pbStopFlag);
    }
    /* One window (LocalMapping's call), without copying it.  `overlap` (optional) runs once on
     * this thread while the device works on the first LM steps (after the window has been
     * uploaded): host work of the caller that does not need the result, e.g. releasing scratch. */
    void Solve(const LocalBAWindow& w, const bool* pbStopFlag, LocalBAResult& out,
               const std::function<void()>& overlap = nullptr) {
        const LocalBAWindow* wp = &w;
        out = LocalBAResult{};
        solve(&wp, &out, 1, pbStopFlag, overlap);
    }

    slam_lba* handle() { return s_; }
   private:
    void solve(const LocalBAWindow* const* ws, LocalBAResult* out, int n, const bool* pbStopFlag,
               const std::function<void()>& overlap = nullptr) {
        std::vector<slam_lba_problem> probs(n);
        std::vector<slam_lba_result> res(n);
        for (int i = 0; i < n; i++) {
            const LocalBAWindow& w = *ws[i];
            slam_lba_problem& p = probs[i];
            p.n_kf = w.n_kf();
            p.kf_Tcw = w.kf_Tcw.data();
            p.kf_fixed = w.kf_fixed.data();
            p.n_pt = w.n_pt();
            p.pt_pos = w.pt_pos.data();
            p.n_edge = w.n_edge();
            p.edge_pt = w.edge_pt.data();
            p.edge_kf = w.edge_kf.data();
            p.edge_obs = w.edge_obs.data();
            p.edge_inv_sigma2 = w.edge_inv_sigma2.data();
            p.cam = w.cam;
            if (!w.edge_body.empty()) {
                p.edge_body = w.edge_body.data();
                p.kf_Trl = w.kf_Trl.data();
                p.cam2 = w.cam2;
            }
            if (!w.kf_cam.empty()) p.kf_cam = w.kf_cam.data();
            if (!w.kf_cam2.empty()) p.kf_cam2 = w.kf_cam2.data();
            p.user_lambda_init = w.inertial ? 100.0 : 0.0;  // this window's pMap->IsInertial() (:1726)
            out[i].kf_Tcw.resize(w.kf_Tcw.size());
            out[i].pt_pos.resize(w.pt_pos.size());
            out[i].edge_outlier.resize(w.edge_pt.size());
            res[i] = slam_lba_result{};
            res[i].kf_Tcw = out[i].kf_Tcw.data();
            res[i].pt_pos = out[i].pt_pos.data();
            res[i].edge_outlier = out[i].edge_outlier.data();
        }
        slam_lba_options opt{};
        opt.iters_first = 5;
        opt.iters_second = 10;
        opt.user_lambda_init = 0.0;  // per window below
        // the reference's `bool* pbStopFlag` itself: the solver reads it live (a C++ bool is one
        // byte), so LocalMapping setting mbAbortBA mid-solve stops the LM loop as in g2o
        static_assert(sizeof(bool) == 1, "slam_lba_options::stop_flag_bool expects a one-byte bool");
        opt.stop_flag_bool = reinterpret_cast<const volatile uint8_t*>(pbStopFlag);
        const volatile int32_t* sf = nullptr;
        // the step hook runs on this thread each time the host has a step's counters, with the
        // next steps already queued on the device: the first call runs `overlap`
        struct Hook {
            const std::function<void()>* fn;
            bool ran;
        } hk{&overlap, false};
        if (overlap) {
            opt.step_hook = [](void* ctx, int32_t) {
                Hook* h = static_cast<Hook*>(ctx);
                if (!h->ran) {
                    h->ran = true;
                    (*h->fn)();
                }
            };
            opt.step_hook_ctx = &hk;
        }
        check(slamhot_lba_solve(s_, n, probs.data(), &opt, sf, res.data()), "LocalBundleAdjustment");
        if (overlap && !hk.ran) overlap();  // nothing ran on the device (stop flag set on entry)
        for (int i = 0; i < n; i++) {
            out[i].iterations[0] = res[i].iterations[0];
            out[i].iterations[1] = res[i].iterations[1];
            out[i].trials = res[i].trials;
            out[i].n_outlier = res[i].n_outlier;
            out[i].chi2_initial = res[i].chi2_initial;
            out[i].chi2_final = res[i].chi2_final;
            out[i].ran = res[i].ran != 0;
        }
    }

    slam_lba* s_ = nullptr;
};

/* ------------------------------------------------------------------------------------
 * Motion-only BA: Optimizer::PoseOptimization (Optimizer.h:52, Optimizer.cc:824-1118).
 * ---------------------------------------------------------------------------------- */
class PoseOptimizer {
   public:
    explicit PoseOptimizer(int device = 0) { check(slamhot_pose_opt_create(device, &h_), "PoseOptimizer"); }
    ~PoseOptimizer() { slamhot_pose_opt_destroy(h_); }
    PoseOptimizer(const PoseOptimizer&) = delete;
    PoseOptimizer& operator=(const PoseOptimizer&) = delete;
    /* frames.size() Frames in one launch; results[i].outlier must point at frames[i].n bytes */
    void Solve(const std::vector<slam_pose_frame>& frames, std::vector<slam_pose_result>& results) {
        check(slamhot_pose_optimization(h_, (int)frames.size(), frames.data(), results.data()), "PoseOptimization");
    }
    slam_pose_opt* handle() { return h_; }

   private:
    slam_pose_opt* h_ = nullptr;
};

/* ------------------------------------------------------------------------------------
 * Frame::ComputeStereoMatches (Frame.h:112, Frame.cc:794-964) on the pyramids the two
 * extractors hold from their last call.
 * ---------------------------------------------------------------------------------- */
class StereoMatcher {
   public:
    explicit StereoMatcher(int device = 0) { check(slamhot_stereo_create(device, &h_), "StereoMatcher"); }
    ~StereoMatcher() { slamhot_stereo_destroy(h_); }
    StereoMatcher(const StereoMatcher&) = delete;
    StereoMatcher& operator=(const StereoMatcher&) = delete;
    void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, const std::vector<KeyPoint>& mvKeys,
                              const Mat8U& descLeft, const std::vector<KeyPoint>& mvKeysRight, const Mat8U& descRight,
                              float mbf, float mb, std::vector<float>& mvuRight, std::vector<float>& mvDepth) {
        mvuRight.assign(mvKeys.size(), -1.f);
        mvDepth.assign(mvKeys.size(), -1.f);
        check(slamhot_compute_stereo_matches(h_, left.handle(), right.handle(), (int)mvKeys.size(), mvKeys.data(),
                                             descLeft.data.data(), (int)mvKeysRight.size(), mvKeysRight.data(),
                                             descRight.data.data(), mbf, mb, mvuRight.data(), mvDepth.data()),
              "ComputeStereoMatches");
    }
    slam_stereo* handle() { return h_; }

   private:
    slam_stereo* h_ = nullptr;
};

/* ------------------------------------------------------------------------------------
 * LocalMapping's matchers: MapPoint::ComputeDistinctiveDescriptors,
 * ORBmatcher::SearchForTriangulation_, the search half of ORBmatcher::Fuse.
 * ---------------------------------------------------------------------------------- */
class LocalMapper {
   public:
    explicit LocalMapper(int device = 0) { check(slamhot_mapper_create(device, &h_), "LocalMapper"); }
    ~LocalMapper() { slamhot_mapper_destroy(h_); }
    LocalMapper(const LocalMapper&) = delete;
    LocalMapper& operator=(const LocalMapper&) = delete;

    /* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:349-423) for off.size()-1 MapPoints */
    void ComputeDistinctiveDescriptors(const std::vector<int32_t>& off, const uint8_t* desc, std::vector<int32_t>& best) {
        const int n = (int)off.size() - 1;
        best.assign(std::max(n, 0), -1);
        if (n > 0) check(slamhot_distinctive_descriptors(h_, n, off.data(), desc, best.data()), "ComputeDistinctiveDescriptors");
    }

    /* ORBmatcher::SearchForTriangulation_ (ORBmatcher.cc:1208-1433) for every pair at once;
     * vMatchedPairs[p] = (idx1, idx2) in idx1 order, returns the per-pair counts. */
    std::vector<int32_t> SearchForTriangulation(const std::vector<slam_tri_kf>& kfs, const std::vector<slam_tri_pair>& pairs,
                                                bool bCheckOri,
                                                std::vector<std::vector<std::pair<size_t, size_t>>>& vMatchedPairs) {
        int cap = 1;
        for (const slam_tri_kf& k : kfs) cap = std::max(cap, k.n);
        std::vector<int32_t> m12((size_t)pairs.size() * cap), nm(pairs.size(), 0);
        if (!pairs.empty())
            check(slamhot_search_for_triangulation(h_, (int)kfs.size(), kfs.data(), (int)pairs.size(), pairs.data(),
                                                   bCheckOri, cap, m12.data(), nm.data()),
                  "SearchForTriangulation_");
        vMatchedPairs.assign(pairs.size(), {});
        for (size_t p = 0; p < pairs.size(); p++)
            for (int i = 0; i < kfs[pairs[p].kf1].n; i++)
                if (m12[p * cap + i] >= 0) vMatchedPairs[p].emplace_back((size_t)i, (size_t)m12[p * cap + i]);
        return nm;
    }

    /* search half of int ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, th, bRight=false)
     * (ORBmatcher.cc:1629-1788); the caller applies the update half in list order */
    void FuseSearch(const slam_frame_view& KF, const float* mvInvLevelSigma2, const std::vector<slam_mp_geom>& mps,
                    const uint8_t* mp_desc, float th, std::vector<int32_t>& best_idx, std::vector<int32_t>& best_dist) {
        best_idx.assign(mps.size(), -1);
        best_dist.assign(mps.size(), 256);
        if (!mps.empty())
            check(slamhot_fuse_search(h_, &KF, mvInvLevelSigma2, (int)mps.size(), mps.data(), mp_desc, th,
                                      best_idx.data(), best_dist.data()),
                  "Fuse");
    }
    slam_mapper* handle() { return h_; }

   private:
    slam_mapper* h_ = nullptr;
};

namespace Optimizer {
/* int Optimizer::PoseOptimization(Frame* pFrame): returns nInitialCorrespondences - nBad
 * (0 below 3 correspondences); pose and mvbOutlier land in `out` (out.outlier -> n bytes). */
inline int PoseOptimization(PoseOptimizer& solver, const slam_pose_frame& F, slam_pose_result& out) {
    std::vector<slam_pose_frame> fs{F};
    std::vector<slam_pose_result> rs{out};
    solver.Solve(fs, rs);
    out = rs[0];
    return out.n_inliers;
}

/* static void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap,
 *     int& num_fixedKF, int& num_OptKF, int& num_MPs, int& num_edges)
 * on a flattened window: the four counters as the reference reports them (:1714-1718,
 * 1800-1921), the solved poses / points and vToErase in `out`. */
inline void LocalBundleAdjustment(LocalBundleAdjuster& solver, const LocalBAWindow& w, bool* pbStopFlag,
                                  LocalBAResult& out, int& num_fixedKF, int& num_OptKF, int& num_MPs,
                                  int& num_edges) {
    num_fixedKF = 0;
    num_OptKF = 0;
    for (uint8_t f : w.kf_fixed) {
        num_fixedKF += f ? 1 : 0;      // lFixedCameras.size() + the init KF (:1630-1675)
        num_OptKF += f == 2 ? 0 : 1;   // lLocalKeyFrames.size() (:1749)
    }
    num_MPs = w.n_pt();
    num_edges = w.n_edge();
    if (num_fixedKF == 0) return;  // Optimizer.cc:1714-1718
    solver.Solve(w, pbStopFlag, out);
}
}  // namespace Optimizer

}  // namespace slamhot

#endif  // SLAMHOT_HPP
