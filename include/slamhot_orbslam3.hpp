/* slamhot_orbslam3.hpp — the drop-in shim bodies, written against the reference's own types.
 *
 * Include AFTER OpenCV and the reference's headers (KeyFrame.h, MapPoint.h, Frame.h, Map.h):
 * every function here is a template over those classes, so the same text is the body of the
 * replaced reference function (the shims of INTEGRATION.md call these) and compiles in this
 * repo's tests against minimal stand-ins (tests/cpp/orbslam3_standins.hpp) that carry exactly
 * the members used here.  Each shim keeps the reference's control flow and map bookkeeping on
 * the host and hands the data-parallel work to libslamhot.so through include/slamhot.hpp.
 *
 *   ORBextractorCall          ORBextractor::operator()                 ORBextractor.cc:1068-1150
 *   SearchByBoW               ORBmatcher::SearchByBoW(KeyFrame*, Frame&) ORBmatcher.cc:269-471
 *   SearchByBoW               ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*) ORBmatcher.cc:823-963
 *   SearchByProjection        ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
 *                                                                        ORBmatcher.cc:2173-2389
 *   SearchByProjection        ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, th, ORBdist)
 *                                                                        ORBmatcher.cc:2391-2513
 *   ComputeBoW                Frame::ComputeBoW / KeyFrame::ComputeBoW   Frame.cc:721-728, KeyFrame.cc:105-114
 *   SearchLocalPoints         Tracking::SearchLocalPoints               Tracking.cc:3187-3258
 *   PoseOptimization          Optimizer::PoseOptimization(Frame*)      Optimizer.cc:824-1118
 *   ComputeStereoMatches      Frame::ComputeStereoMatches              Frame.cc:794-964
 *   BuildLocalWindow          Optimizer::LocalBundleAdjustment window  Optimizer.cc:1613-1718
 *   FlattenLocalWindow        its vertex / edge setup                  Optimizer.cc:1737-1918
 *   LocalBundleAdjustment     the whole function incl. write-back      Optimizer.cc:1611-2078
 *   Fuse                      ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>, th, false)  ORBmatcher.cc:1629-1818
 *
 * One header addition on the reference side: MapPoint gains the getters GetMinDistance() /
 * GetMaxDistance() (mfMinDistance / mfMaxDistance under mMutexPos).  The kernels need the raw
 * values (PredictScale divides mfMaxDistance, MapPoint.cc:551-566); the reference only exposes
 * them multiplied by 0.8f / 1.2f, which cannot be undone exactly in float.
 */
#ifndef SLAMHOT_ORBSLAM3_HPP
#define SLAMHOT_ORBSLAM3_HPP

#include <algorithm>
#include <cmath>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "slamhot.hpp"

namespace slamhot {
namespace orbslam3 {

static_assert(sizeof(cv::KeyPoint) == sizeof(slam_keypoint), "cv::KeyPoint is the 28-byte slam_keypoint");

inline const slam_keypoint* kp_ptr(const std::vector<cv::KeyPoint>& v) {
    return reinterpret_cast<const slam_keypoint*>(v.data());
}

inline void mat4(const cv::Mat& T, float* out) {  // a 4x4 CV_32F pose, row-major
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out[4 * r + c] = T.template at<float>(r, c);
}

inline cv::Mat mat_from(const float* p, int rows, int cols) {
    cv::Mat m(rows, cols, CV_32F);
    for (int r = 0; r < rows; r++)
        for (int c = 0; c < cols; c++) m.template at<float>(r, c) = p[r * cols + c];
    return m;
}

/* ------------------------------------------------------------------ ORBextractor::operator()
 * int operator()(InputArray image, InputArray mask, vector<KeyPoint>& keypoints,
 *                OutputArray descriptors, vector<int>& vLappingArea)   (ORBextractor.cc:1068-1150)
 * `hot` is the slamhot extractor the reference ORBextractor owns; mvImagePyramid is refreshed
 * when the caller reads it (stereo matching on the device does not need it). */
inline int ORBextractorCall(ORBextractor& hot, const cv::Mat& image, std::vector<cv::KeyPoint>& keypoints,
                            cv::Mat& descriptors, const std::vector<int>& vLappingArea,
                            std::vector<cv::Mat>* mvImagePyramid = nullptr) {
    if (image.empty()) return -1;  // ORBextractor.cc:1072-1073
    GrayImage g;
    g.data = image.data;
    g.cols = image.cols;
    g.rows = image.rows;
    g.step = image.step;
    std::vector<KeyPoint> kps;
    Mat8U desc;
    const int mono = hot(g, kps, desc, vLappingArea);
    keypoints.resize(kps.size());
    std::memcpy(static_cast<void*>(keypoints.data()), kps.data(), kps.size() * sizeof(slam_keypoint));
    descriptors.create((int)kps.size(), 32, CV_8U);
    if (!kps.empty()) std::memcpy(descriptors.data, desc.data.data(), desc.data.size());
    if (mvImagePyramid) {
        const std::vector<Mat8U> pyr = hot.mvImagePyramid();
        mvImagePyramid->resize(pyr.size());
        for (size_t l = 0; l < pyr.size(); l++) {
            (*mvImagePyramid)[l].create(pyr[l].rows, pyr[l].cols, CV_8U);
            std::memcpy((*mvImagePyramid)[l].data, pyr[l].data.data(), pyr[l].data.size());
        }
    }
    return mono;
}

/* DBoW2::FeatureVector (std::map<NodeId, vector<unsigned>>, ascending node id) as the CSR of
 * slam_bow_side; the arrays live in `store`. */
struct BowStore {
    std::vector<uint32_t> node_id, node_feat;
    std::vector<int32_t> node_off;
    std::vector<float> angle;
    std::vector<uint8_t> valid;
};

template <class FeatVec>
slam_bow_side bow_side(const FeatVec& fv, const cv::Mat& desc, const std::vector<cv::KeyPoint>& kps, BowStore& st) {
    st.node_id.clear();
    st.node_feat.clear();
    st.node_off.assign(1, 0);
    for (const auto& kv : fv) {
        st.node_id.push_back((uint32_t)kv.first);
        for (unsigned f : kv.second)  // features past mvKeysUn (a second camera's) are skipped, :858, :878
            if (f < kps.size()) st.node_feat.push_back(f);
        st.node_off.push_back((int32_t)st.node_feat.size());
    }
    st.angle.resize(kps.size());
    for (size_t i = 0; i < kps.size(); i++) st.angle[i] = kps[i].angle;
    slam_bow_side s{};
    s.n = (int32_t)kps.size();
    s.desc = desc.data;
    s.angle = st.angle.data();
    s.valid = nullptr;
    s.n_nodes = (int32_t)st.node_id.size();
    s.node_id = st.node_id.data();
    s.node_off = st.node_off.data();
    s.node_feat = st.node_feat.data();
    return s;
}

/* ------------------------------------------------------------------ ORBmatcher::SearchByBoW
 * int SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
 * (ORBmatcher.cc:269-471) */
template <class KeyFrame, class Frame, class MapPoint, class = typename std::enable_if<!std::is_pointer<Frame>::value>::type>
int SearchByBoW(slamhot::ORBmatcher& hot, KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    const std::vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    vpMapPointMatches = std::vector<MapPoint*>(F.N, static_cast<MapPoint*>(nullptr));
    BowStore sa, sb;
    KeyFrameBow A;
    FrameBow B;
    static_cast<slam_bow_side&>(A) = bow_side(pKF->mFeatVec, pKF->mDescriptors, pKF->mvKeysUn, sa);
    static_cast<slam_bow_side&>(B) = bow_side(F.mFeatVec, F.mDescriptors, F.mvKeysUn, sb);
    sa.valid.resize(vpMapPointsKF.size());
    for (size_t i = 0; i < vpMapPointsKF.size(); i++)  // pMP && !pMP->isBad() (:321-327)
        sa.valid[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad();
    A.valid = sa.valid.data();
    std::vector<int> idx;
    const int n = hot.SearchByBoW(A, B, idx);
    for (int j = 0; j < F.N; j++)
        if (idx[j] >= 0) vpMapPointMatches[j] = vpMapPointsKF[idx[j]];
    return n;
}

/* ------------------------------------------------------------------ ORBmatcher::SearchByBoW
 * int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
 * (ORBmatcher.cc:823-963): both sides need a MapPoint that is not bad (:862-866, :882-888);
 * vpMatches12[i] = the MapPoint of the KF2 feature KF1 feature i matched. */
template <class KeyFrame, class MapPoint>
int SearchByBoW(slamhot::ORBmatcher& hot, KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
    const std::vector<MapPoint*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MapPoint*> vpMapPoints2 = pKF2->GetMapPointMatches();
    vpMatches12 = std::vector<MapPoint*>(vpMapPoints1.size(), static_cast<MapPoint*>(nullptr));
    BowStore s1, s2;
    KeyFrameBow A, B;
    static_cast<slam_bow_side&>(A) = bow_side(pKF1->mFeatVec, pKF1->mDescriptors, pKF1->mvKeysUn, s1);
    static_cast<slam_bow_side&>(B) = bow_side(pKF2->mFeatVec, pKF2->mDescriptors, pKF2->mvKeysUn, s2);
    s1.valid.assign(A.n, 0);
    s2.valid.assign(B.n, 0);
    for (int i = 0; i < A.n && i < (int)vpMapPoints1.size(); i++)
        s1.valid[i] = vpMapPoints1[i] && !vpMapPoints1[i]->isBad();
    for (int i = 0; i < B.n && i < (int)vpMapPoints2.size(); i++)
        s2.valid[i] = vpMapPoints2[i] && !vpMapPoints2[i]->isBad();
    A.valid = s1.valid.data();
    B.valid = s2.valid.data();
    std::vector<int> idx;
    const int n = hot.SearchByBoW(A, B, idx);
    for (int i = 0; i < A.n; i++)
        if (idx[i] >= 0) vpMatches12[i] = vpMapPoints2[idx[i]];
    return n;
}

/* ------------------------------------------------------------------ Frame / KeyFrame::ComputeBoW
 * void Frame::ComputeBoW() (Frame.cc:721-728) and KeyFrame::ComputeBoW() (KeyFrame.cc:105-114):
 * mpORBvocabulary->transform(toDescriptorVector(mDescriptors), mBowVec, mFeatVec, 4) with the device
 * descent; mBowVec (DBoW2::BowVector) and mFeatVec (DBoW2::FeatureVector) are filled in key order.
 * `hot` is the process's device copy of mpORBvocabulary (one per vocabulary, shareable between
 * threads: the handle serialises its calls).  mDescriptors is N x 32 and row-contiguous, as
 * ORBextractor creates it. */
template <class Frame>
void ComputeBoW(Vocabulary& hot, Frame& F) {
    if (!F.mBowVec.empty()) return;  // :723
    BowVector v;
    FeatureVector fv;
    hot.transform(F.mDescriptors.data, F.mDescriptors.rows, v, fv, 4);
    F.mBowVec.clear();
    F.mFeatVec.clear();
    for (const auto& w : v) F.mBowVec.emplace_hint(F.mBowVec.end(), w.first, w.second);
    for (auto& nd : fv) F.mFeatVec.emplace_hint(F.mFeatVec.end(), nd.first, std::move(nd.second));
}
template <class KeyFrame>
void KeyFrameComputeBoW(Vocabulary& hot, KeyFrame* pKF) {
    if (!pKF->mBowVec.empty() && !pKF->mFeatVec.empty()) return;  // KeyFrame.cc:107
    pKF->mBowVec.clear();
    ComputeBoW(hot, *pKF);
}

/* The matcher-facing view of a Frame (grid bounds and scale tables are Frame statics / members). */
template <class Frame>
slam_frame_view frame_view(Frame& F, std::vector<int8_t>& mp_state, float* Tcw16) {
    slam_frame_view v{};
    v.n = F.N;
    v.kps_un = kp_ptr(F.mvKeysUn);
    v.uright = F.mvuRight.data();
    v.desc = F.mDescriptors.data;
    mp_state.assign(F.N, -1);
    for (int i = 0; i < F.N; i++)
        if (F.mvpMapPoints[i]) mp_state[i] = F.mvpMapPoints[i]->Observations() > 0 ? 1 : 0;
    v.mp_state = mp_state.data();
    v.min_x = Frame::mnMinX;
    v.min_y = Frame::mnMinY;
    v.max_x = Frame::mnMaxX;
    v.max_y = Frame::mnMaxY;
    v.grid_inv_w = Frame::mfGridElementWidthInv;
    v.grid_inv_h = Frame::mfGridElementHeightInv;
    v.nlevels = F.mnScaleLevels;
    v.scale = F.mvScaleFactors.data();
    v.log_scale = F.mfLogScaleFactor;
    v.fx = F.fx;
    v.fy = F.fy;
    v.cx = F.cx;
    v.cy = F.cy;
    v.bf = F.mbf;
    v.b = F.mb;
    mat4(F.mTcw, Tcw16);
    v.Tcw = Tcw16;
    return v;
}

/* ------------------------------------------------------------------ ORBmatcher::SearchByProjection
 * int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono)
 * (ORBmatcher.cc:2173-2389), Nleft == -1: TrackWithMotionModel's matcher (Tracking.cc:2683-2760).
 * Only the last frame's MapPoints that are set and not flagged mvbOutlier are read (:2196-2201); a
 * current feature is a candidate unless it holds a MapPoint with observations (:2248-2250).  The
 * matches land in CurrentFrame.mvpMapPoints, and so do the NULLs of the rotation check (:2366-2386). */
template <class Frame>
int SearchByProjection(slamhot::ORBmatcher& hot, Frame& CurrentFrame, const Frame& LastFrame, float th, bool bMono) {
    const int n = LastFrame.N;
    std::vector<uint8_t> has_mp(n, 0), outlier(n, 0), has_obs(n, 0), desc(32 * (size_t)n, 0);
    std::vector<float> pos(3 * (size_t)n, 0.f);
    for (int i = 0; i < n; i++) {
        auto* pMP = LastFrame.mvpMapPoints[i];
        if (!pMP) continue;
        has_mp[i] = 1;
        outlier[i] = LastFrame.mvbOutlier[i] ? 1 : 0;
        if (outlier[i]) continue;
        const cv::Mat X = pMP->GetWorldPos(), d = pMP->GetDescriptor();
        for (int k = 0; k < 3; k++) pos[3 * (size_t)i + k] = X.template at<float>(k);
        std::memcpy(&desc[32 * (size_t)i], d.data, 32);
        has_obs[i] = pMP->Observations() > 0;  // a match makes the candidate blocking (:2248-2250)
    }
    float Tl[16];
    mat4(LastFrame.mTcw, Tl);
    slam_last_frame L{};
    L.n = n;
    L.Tcw = Tl;
    L.kps = kp_ptr(LastFrame.mvKeys);      // octave (:2221)
    L.kps_un = kp_ptr(LastFrame.mvKeysUn); // angle (:2278)
    L.has_mp = has_mp.data();
    L.outlier = outlier.data();
    L.mp_pos = pos.data();
    L.mp_desc = desc.data();
    L.mp_has_obs = has_obs.data();
    std::vector<int8_t> st;
    float T[16];
    const slam_frame_view v = frame_view(CurrentFrame, st, T);
    std::vector<int> fm;
    const int nmatches = hot.SearchByProjection(v, L, th, bMono, fm);
    for (int i = 0; i < CurrentFrame.N; i++) {
        if (fm[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[fm[i]];
        else if (fm[i] == -2) CurrentFrame.mvpMapPoints[i] = nullptr;
    }
    return nmatches;
}

/* int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
 * const float th, const int ORBdist) (ORBmatcher.cc:2391-2513): Relocalization's matcher
 * (Tracking.cc:3455-3590).  The KeyFrame's MapPoints that are set, not bad and not in sAlreadyFound
 * (:2409-2413); a current feature holding any MapPoint is no candidate (:2455-2456). */
template <class Frame, class KeyFrame, class MapPoint>
int SearchByProjection(slamhot::ORBmatcher& hot, Frame& CurrentFrame, KeyFrame* pKF,
                       const std::set<MapPoint*>& sAlreadyFound, float th, int ORBdist) {
    const std::vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    const int n = (int)vpMPs.size();
    std::vector<uint8_t> use(n, 0), desc(32 * (size_t)n, 0);
    std::vector<float> pos(3 * (size_t)n, 0.f), max_d(n, 0.f), min_d(n, 0.f);
    for (int i = 0; i < n; i++) {
        MapPoint* pMP = vpMPs[i];
        if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
        use[i] = 1;
        const cv::Mat X = pMP->GetWorldPos(), d = pMP->GetDescriptor();
        for (int k = 0; k < 3; k++) pos[3 * (size_t)i + k] = X.template at<float>(k);
        std::memcpy(&desc[32 * (size_t)i], d.data, 32);
        max_d[i] = pMP->GetMaxDistance();  // raw: the kernel applies 1.2f / 0.8f and PredictScale (:2430-2437)
        min_d[i] = pMP->GetMinDistance();
    }
    slam_kf_points K{};
    K.n = n;
    K.kps_un = kp_ptr(pKF->mvKeysUn);  // angle (:2476)
    K.use = use.data();
    K.mp_pos = pos.data();
    K.max_dist = max_d.data();
    K.min_dist = min_d.data();
    K.mp_desc = desc.data();
    std::vector<int8_t> st;
    float T[16];
    const slam_frame_view v = frame_view(CurrentFrame, st, T);
    std::vector<int> fm;
    const int nmatches = hot.SearchByProjection(v, K, th, ORBdist, fm);
    for (int i = 0; i < CurrentFrame.N; i++) {
        if (fm[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[fm[i]];
        else if (fm[i] == -2) CurrentFrame.mvpMapPoints[i] = nullptr;
    }
    return nmatches;
}

/* ------------------------------------------------------------------ Tracking::SearchLocalPoints
 * void Tracking::SearchLocalPoints() (Tracking.cc:3187-3258) for a Frame with Nleft == -1: the
 * frame's own MapPoints are marked seen (bad ones dropped, :3190-3206); then Frame::isInFrustum of
 * every local MapPoint not seen / not bad and SearchByProjection(F, vpLocalMapPoints, th, bFarPoints,
 * thFarPoints) on the ones in view, one device call; the fields isInFrustum leaves (Frame.cc:497-554)
 * and IncreaseVisible are written back into the MapPoints, mmProjectPoints into the Frame
 * (:3227-3230), the matches into F.mvpMapPoints.  `th` is the caller's choice of :3234-3253
 * (sensor, IMU and relocalisation state of the Tracking thread).  Returns nToMatch. */
template <class Frame, class MapPoint>
int SearchLocalPoints(slamhot::ORBmatcher& hot, Frame& F, const std::vector<MapPoint*>& vpLocalMapPoints, float th,
                      bool bFarPoints, float thFarPoints, int* nmatches = nullptr) {
    for (auto& pMP : F.mvpMapPoints) {  // :3190-3206
        if (!pMP) continue;
        if (pMP->isBad()) {
            pMP = nullptr;
        } else {
            pMP->IncreaseVisible();
            pMP->mnLastFrameSeen = F.mnId;
            pMP->mbTrackInView = false;
            pMP->mbTrackInViewR = false;
        }
    }
    std::vector<slam_mp_geom> G(vpLocalMapPoints.size());
    std::vector<uint8_t> D(32 * G.size());
    for (size_t i = 0; i < G.size(); i++) {
        MapPoint* pMP = vpLocalMapPoints[i];
        slam_mp_geom& g = G[i];
        g.seen = pMP->mnLastFrameSeen == F.mnId;
        g.is_bad = pMP->isBad();
        g.has_obs = pMP->Observations() > 0;
        const cv::Mat P = pMP->GetWorldPos(), nrm = pMP->GetNormal(), d = pMP->GetDescriptor();
        for (int k = 0; k < 3; k++) {
            g.pos[k] = P.template at<float>(k);
            g.normal[k] = nrm.template at<float>(k);
        }
        g.min_dist = pMP->GetMinDistance();  // raw mfMinDistance / mfMaxDistance: the kernels apply the
        g.max_dist = pMP->GetMaxDistance();  // 0.8f / 1.2f invariance factors and PredictScale themselves
        std::memcpy(&D[32 * i], d.data, 32);
    }
    std::vector<int8_t> st;
    float T[16];
    slam_frame_view v = frame_view(F, st, T);
    std::vector<slam_mp_track> track;
    std::vector<int> f_match;
    int nToMatch = 0;
    const int n = hot.SearchLocalPoints(v, G, D.data(), 0.5f, th, bFarPoints, thFarPoints, track, nToMatch, f_match);
    for (size_t i = 0; i < G.size(); i++) {
        MapPoint* pMP = vpLocalMapPoints[i];
        if (G[i].seen || G[i].is_bad) continue;  // :3217-3220
        const slam_mp_track& t = track[i];
        pMP->mbTrackInView = t.in_view;          // isInFrustum, Frame.cc:497-554
        pMP->mTrackProjX = t.proj_x;             // -1, or the projection once it lies in the image
        pMP->mTrackProjY = t.proj_y;
        if (t.in_view) {
            pMP->IncreaseVisible();
            pMP->mTrackProjXR = t.proj_xr;
            pMP->mnTrackScaleLevel = t.scale_level;
            pMP->mTrackViewCos = t.view_cos;
            pMP->mTrackDepth = t.depth;
            F.mmProjectPoints[pMP->mnId] = cv::Point2f(pMP->mTrackProjX, pMP->mTrackProjY);  // :3227-3230
        }
    }
    for (int i = 0; i < F.N; i++)
        if (f_match[i] >= 0) F.mvpMapPoints[i] = vpLocalMapPoints[f_match[i]];
    if (nmatches) *nmatches = n;
    return nToMatch;
}

/* ------------------------------------------------------------------ Optimizer::PoseOptimization
 * int PoseOptimization(Frame* pFrame) (Optimizer.cc:824-1118), pinhole. */
template <class Frame>
int PoseOptimization(slamhot::PoseOptimizer& hot, Frame* pFrame) {
    const int N = pFrame->N;
    std::vector<uint8_t> has_mp(N), outl(N, 0);
    std::vector<float> mp_pos(3 * (size_t)N, 0.f);
    for (int i = 0; i < N; i++) {  // under MapPoint::mGlobalMutex in the reference (:861)
        auto* pMP = pFrame->mvpMapPoints[i];
        has_mp[i] = pMP != nullptr;
        if (pMP) {
            const cv::Mat X = pMP->GetWorldPos();
            for (int k = 0; k < 3; k++) mp_pos[3 * i + k] = X.template at<float>(k);
        }
    }
    slam_pose_frame F{};
    mat4(pFrame->mTcw, F.Tcw);
    F.n = N;
    F.kps_un = kp_ptr(pFrame->mvKeysUn);
    F.uright = pFrame->mvuRight.data();
    F.has_mp = has_mp.data();
    F.mp_pos = mp_pos.data();
    F.inv_sigma2 = pFrame->mvInvLevelSigma2.data();
    F.nlevels = (int)pFrame->mvInvLevelSigma2.size();
    F.cam = slam_camera{pFrame->fx, pFrame->fy, pFrame->cx, pFrame->cy, pFrame->mbf};
    slam_pose_result R{};
    R.outlier = outl.data();
    const int n = slamhot::Optimizer::PoseOptimization(hot, F, R);
    if (R.n_initial < 3) {  // Optimizer.cc:1012-1013: pose untouched, but the edge set-up loop
        for (int i = 0; i < N; i++)  // (:864-1005) has already cleared mvbOutlier of every MapPoint
            if (has_mp[i]) pFrame->mvbOutlier[i] = false;
        return 0;
    }
    for (int i = 0; i < N; i++)
        if (has_mp[i]) pFrame->mvbOutlier[i] = outl[i] != 0;
    pFrame->SetPose(mat_from(R.Tcw, 4, 4));
    return n;
}

/* ------------------------------------------------------------------ Frame::ComputeStereoMatches
 * (Frame.cc:794-964) right after the stereo Frame constructor's two extractions. */
template <class Frame>
void ComputeStereoMatches(slamhot::StereoMatcher& hot, ORBextractor& left, ORBextractor& right, Frame& F) {
    Mat8U dl, dr;
    dl.rows = F.mDescriptors.rows;
    dl.cols = 32;
    dl.data.assign(F.mDescriptors.data, F.mDescriptors.data + (size_t)dl.rows * 32);
    dr.rows = F.mDescriptorsRight.rows;
    dr.cols = 32;
    dr.data.assign(F.mDescriptorsRight.data, F.mDescriptorsRight.data + (size_t)dr.rows * 32);
    std::vector<KeyPoint> kl(F.mvKeys.size()), kr(F.mvKeysRight.size());
    std::memcpy(kl.data(), F.mvKeys.data(), kl.size() * sizeof(slam_keypoint));
    std::memcpy(kr.data(), F.mvKeysRight.data(), kr.size() * sizeof(slam_keypoint));
    hot.ComputeStereoMatches(left, right, kl, dl, kr, dr, F.mbf, F.mb, F.mvuRight, F.mvDepth);
}

/* ------------------------------------------------------------------ Optimizer::LocalBundleAdjustment */
template <class KeyFrame, class MapPoint>
struct LocalWindow {
    using Observations = decltype(std::declval<MapPoint&>().GetObservations());
    std::vector<KeyFrame*> lLocalKeyFrames, lFixedCameras;  // the reference's std::lists, same order
    std::vector<MapPoint*> lLocalMapPoints;
    // GetObservations() of every local MapPoint, in lLocalMapPoints order: read once for the fixed
    // cameras (Optimizer.cc:1655-1672) and reused by the edge setup (:1815), which the reference
    // fetches a second time from the unchanged map
    std::vector<Observations> observations;
    int num_fixedKF = 0;
};

/* Optimizer.cc:1613-1718.  Returns false where the reference returns (no fixed KeyFrame).  One
 * deviation: the "< 2 fixed" fallback pushes the reference's uninitialised pLowerKf /
 * pSecondLowerKF when no candidate exists (undefined behaviour); here they are skipped. */
template <class KeyFrame, class MapPoint, class Map>
bool BuildLocalWindow(KeyFrame* pKF, Map* pMap, LocalWindow<KeyFrame, MapPoint>& W) {
    W.lLocalKeyFrames.push_back(pKF);
    pKF->mnBALocalForKF = pKF->mnId;
    Map* pCurrentMap = pKF->GetMap();
    const std::vector<KeyFrame*> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
    for (KeyFrame* pKFi : vNeighKFs) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad() && pKFi->GetMap() == pCurrentMap) W.lLocalKeyFrames.push_back(pKFi);
    }
    W.num_fixedKF = 0;
    for (KeyFrame* pKFi : W.lLocalKeyFrames) {
        if (pKFi->mnId == pMap->GetInitKFid()) W.num_fixedKF = 1;
        for (MapPoint* pMP : pKFi->GetMapPointMatches())
            if (pMP && !pMP->isBad() && pMP->GetMap() == pCurrentMap && pMP->mnBALocalForKF != pKF->mnId) {
                W.lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
    }
    W.observations.clear();
    W.observations.reserve(W.lLocalMapPoints.size());
    for (MapPoint* pMP : W.lLocalMapPoints) {
        W.observations.push_back(pMP->GetObservations());
        for (const auto& ob : W.observations.back()) {
            KeyFrame* pKFi = ob.first;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad() && pKFi->GetMap() == pCurrentMap) W.lFixedCameras.push_back(pKFi);
            }
        }
    }
    W.num_fixedKF += (int)W.lFixedCameras.size();
    if (W.num_fixedKF < 2) {
        long lowerId = (long)pKF->mnId, secondLowerId = (long)pKF->mnId;
        KeyFrame *pLowerKf = nullptr, *pSecondLowerKF = nullptr;
        for (KeyFrame* pKFi : W.lLocalKeyFrames) {
            if (pKFi == pKF || pKFi->mnId == pMap->GetInitKFid()) continue;
            if ((long)pKFi->mnId < lowerId) {
                lowerId = (long)pKFi->mnId;
                pLowerKf = pKFi;
            } else if ((long)pKFi->mnId < secondLowerId) {
                secondLowerId = (long)pKFi->mnId;
                pSecondLowerKF = pKFi;
            }
        }
        auto remove = [&](KeyFrame* k) {  // std::list::remove
            W.lLocalKeyFrames.erase(std::remove(W.lLocalKeyFrames.begin(), W.lLocalKeyFrames.end(), k),
                                    W.lLocalKeyFrames.end());
        };
        if (pLowerKf) {
            W.lFixedCameras.push_back(pLowerKf);
            remove(pLowerKf);
            W.num_fixedKF++;
        }
        if (W.num_fixedKF < 2 && pSecondLowerKF) {
            W.lFixedCameras.push_back(pSecondLowerKF);
            remove(pSecondLowerKF);
            W.num_fixedKF++;
        }
    }
    return W.num_fixedKF != 0;
}

/* The vertex / edge setup (Optimizer.cc:1737-1918) as slam_lba_problem arrays: KeyFrames in
 * vertex-id (mnId) order, MapPoints in lLocalMapPoints order, per MapPoint its observations in
 * the observation map's order — the left (mono / stereo) edge, then the right-camera body edge
 * for KeyFrames with mpCamera2.  edge_refs[e] = the (KeyFrame, MapPoint) vToErase would name. */
template <class KeyFrame, class MapPoint, class Map>
void FlattenLocalWindow(const LocalWindow<KeyFrame, MapPoint>& W, Map* pMap, LocalBAWindow& out,
                        std::vector<KeyFrame*>& kfs, std::vector<std::pair<KeyFrame*, MapPoint*>>& edge_refs) {
    kfs.assign(W.lLocalKeyFrames.begin(), W.lLocalKeyFrames.end());
    kfs.insert(kfs.end(), W.lFixedCameras.begin(), W.lFixedCameras.end());
    std::stable_sort(kfs.begin(), kfs.end(), [](KeyFrame* a, KeyFrame* b) { return a->mnId < b->mnId; });
    // the vertex of an observing KeyFrame, or -1 when the edge is skipped (not a window KeyFrame, or
    // bad / another map: :1817, evaluated once per KeyFrame instead of once per edge): an
    // open-addressing table on the pointer (a few dozen entries, one probe per edge)
    Map* pCurrentMap = W.lLocalKeyFrames.empty() ? nullptr : W.lLocalKeyFrames.front()->GetMap();
    size_t tsize = 16;
    while (tsize < 4 * kfs.size()) tsize *= 2;
    std::vector<std::pair<KeyFrame*, int>> table(tsize, {nullptr, -1});
    auto slot_of = [&](KeyFrame* k) {
        return (size_t)(((uintptr_t)k >> 4) * 0x9E3779B97F4A7C15ull >> 40) & (tsize - 1);
    };
    for (size_t k = 0; k < kfs.size(); k++) {
        size_t h = slot_of(kfs[k]);
        while (table[h].first) h = (h + 1) & (tsize - 1);
        const bool usable = !kfs[k]->isBad() && kfs[k]->GetMap() == pCurrentMap;
        table[h] = {kfs[k], usable ? (int)k : -1};
    }
    auto vertex_of = [&](KeyFrame* k) -> int {
        for (size_t h = slot_of(k);; h = (h + 1) & (tsize - 1)) {
            if (table[h].first == k) return table[h].second;
            if (!table[h].first) return -1;
        }
    };
    std::vector<KeyFrame*> fixed(W.lFixedCameras.begin(), W.lFixedCameras.end());
    std::sort(fixed.begin(), fixed.end());
    out = LocalBAWindow{};
    // W.observations is BuildLocalWindow's copy of every MapPoint's observations; a window filled
    // otherwise (LocalWindow is a public struct), or whose copies were already released, reads
    // them from the MapPoints as the reference does (:1815)
    const bool have_obs = W.observations.size() == W.lLocalMapPoints.size();
    size_t nobs = 0;
    if (have_obs)
        for (const auto& o : W.observations) nobs += o.size();
    out.kf_Tcw.reserve(16 * kfs.size());
    out.pt_pos.reserve(3 * W.lLocalMapPoints.size());
    out.edge_pt.reserve(nobs);
    out.edge_kf.reserve(nobs);
    out.edge_obs.reserve(3 * nobs);
    out.edge_inv_sigma2.reserve(nobs);
    edge_refs.reserve(edge_refs.size() + nobs);
    bool rig = false;
    for (size_t k = 0; k < kfs.size(); k++) {
        KeyFrame* pKFi = kfs[k];
        float T[16];
        mat4(pKFi->GetPose(), T);
        out.kf_Tcw.insert(out.kf_Tcw.end(), T, T + 16);
        const bool is_fixed = std::binary_search(fixed.begin(), fixed.end(), pKFi);
        out.kf_fixed.push_back(is_fixed ? 2 : (pKFi->mnId == pMap->GetInitKFid() ? 1 : 0));  // :1741-1744
        rig = rig || pKFi->mpCamera2 != nullptr;
    }
    if (rig) {
        for (KeyFrame* pKFi : kfs) {
            float T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            if (pKFi->mpCamera2) mat4(pKFi->mTrl, T);
            out.kf_Trl.insert(out.kf_Trl.end(), T, T + 16);
        }
    }
    int pi = 0;
    typename LocalWindow<KeyFrame, MapPoint>::Observations fetched;
    for (MapPoint* pMP : W.lLocalMapPoints) {
        const cv::Mat P = pMP->GetWorldPos();
        for (int c = 0; c < 3; c++) out.pt_pos.push_back(P.template at<float>(c));
        if (!have_obs) fetched = pMP->GetObservations();
        for (const auto& ob : have_obs ? W.observations[pi] : fetched) {
            KeyFrame* pKFi = ob.first;
            const int vk = vertex_of(pKFi);
            if (vk < 0) continue;
            const int leftIndex = std::get<0>(ob.second);
            if (leftIndex != -1) {  // mono (:1819-1849) or stereo (:1850-1880)
                const cv::KeyPoint& kpUn = pKFi->mvKeysUn[leftIndex];
                const float ur = pKFi->mvuRight[leftIndex];
                out.edge_pt.push_back(pi);
                out.edge_kf.push_back(vk);
                out.edge_obs.push_back(kpUn.pt.x);
                out.edge_obs.push_back(kpUn.pt.y);
                out.edge_obs.push_back(ur < 0 ? -1.f : ur);
                out.edge_inv_sigma2.push_back(pKFi->mvInvLevelSigma2[kpUn.octave]);
                if (rig) out.edge_body.push_back(0);
                edge_refs.emplace_back(pKFi, pMP);
            }
            if (pKFi->mpCamera2) {  // EdgeSE3ProjectXYZToBody (:1883-1914)
                int rightIndex = std::get<1>(ob.second);
                if (rightIndex != -1) {
                    rightIndex -= pKFi->NLeft;
                    const cv::KeyPoint& kp = pKFi->mvKeysRight[rightIndex];
                    out.edge_pt.push_back(pi);
                    out.edge_kf.push_back(vk);
                    out.edge_obs.push_back(kp.pt.x);
                    out.edge_obs.push_back(kp.pt.y);
                    out.edge_obs.push_back(-1.f);
                    out.edge_inv_sigma2.push_back(pKFi->mvInvLevelSigma2[kp.octave]);
                    out.edge_body.push_back(1);
                    edge_refs.emplace_back(pKFi, pMP);
                }
            }
        }
        pi++;
    }
    // every edge uses its own KeyFrame's camera: mono e->pCamera = pKFi->mpCamera (:1840), stereo
    // e->fx..bf = pKFi->fx..mbf (:1869-1873), body e->pCamera = pKFi->mpCamera2 (:1906)
    auto cam2_of = [](KeyFrame* k) {  // GeometricCamera::getParameter (GeometricCamera.h:70)
        if (!k->mpCamera2) return slam_camera{};
        auto* c2 = k->mpCamera2;
        return slam_camera{c2->getParameter(0), c2->getParameter(1), c2->getParameter(2), c2->getParameter(3), 0.f};
    };
    KeyFrame* k0 = kfs.front();
    out.cam = slam_camera{k0->fx, k0->fy, k0->cx, k0->cy, k0->mbf};
    for (KeyFrame* pKFi : kfs)
        if (pKFi->mpCamera2) {
            out.cam2 = cam2_of(pKFi);
            break;
        }
    bool mixed = false;
    for (KeyFrame* pKFi : kfs) {
        const slam_camera c{pKFi->fx, pKFi->fy, pKFi->cx, pKFi->cy, pKFi->mbf}, c2 = cam2_of(pKFi);
        out.kf_cam.push_back(c);
        out.kf_cam2.push_back(c2);
        mixed = mixed || std::memcmp(&c, &out.cam, sizeof(c)) != 0 ||
                (pKFi->mpCamera2 && std::memcmp(&c2, &out.cam2, sizeof(c2)) != 0);
    }
    if (!mixed) {  // one calibration: cam / cam2 stand for every KeyFrame
        out.kf_cam.clear();
        out.kf_cam2.clear();
    }
    out.inertial = pMap->IsInertial();
}

/* static void Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag, Map* pMap,
 *     int& num_fixedKF, int& num_OptKF, int& num_MPs, int& num_edges)  (Optimizer.cc:1611-2078)
 * `hot`: slamhot::LocalBundleAdjuster (or anything with its Solve(window, stop, result, overlap)). */
template <class KeyFrame, class MapPoint, class Map, class Hot>
void LocalBundleAdjustment(Hot& hot, KeyFrame* pKF, bool* pbStopFlag, Map* pMap, int& num_fixedKF, int& num_OptKF,
                           int& num_MPs, int& num_edges) {
    LocalWindow<KeyFrame, MapPoint> W;
    const bool ok = BuildLocalWindow(pKF, pMap, W);
    num_fixedKF = W.num_fixedKF;
    num_MPs = (int)W.lLocalMapPoints.size();
    if (!ok) return;  // :1714-1718
    num_OptKF = (int)W.lLocalKeyFrames.size();
    LocalBAWindow flat;
    std::vector<KeyFrame*> kfs;
    std::vector<std::pair<KeyFrame*, MapPoint*>> edge_refs;
    FlattenLocalWindow(W, pMap, flat, kfs, edge_refs);
    num_edges = flat.n_edge();
    if (pbStopFlag && *pbStopFlag) return;  // :1921-1923
    LocalBAResult R;
    // optimize(5), stop check, optimize(10), outlier scan; the observation copies (no longer
    // needed) are released while the device runs the first LM steps
    hot.Solve(flat, pbStopFlag, R, [&W] { decltype(W.observations)().swap(W.observations); });
    if (!R.ran) return;  // the flag flipped between the check above and the solver's own: :1921-1923
    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);  // :2040
    for (size_t e = 0; e < edge_refs.size(); e++)           // vToErase (:2043-2052)
        if (R.edge_outlier[e] && !edge_refs[e].second->isBad()) {
            edge_refs[e].first->EraseMapPointMatch(edge_refs[e].second);
            edge_refs[e].second->EraseObservation(edge_refs[e].first);
        }
    cv::Mat Tcw(4, 4, CV_32F), Pos(3, 1, CV_32F);           // SetPose / SetWorldPos copy their argument
    for (size_t k = 0; k < kfs.size(); k++) {               // :2056-2063
        if (flat.kf_fixed[k] == 2) continue;                 // lFixedCameras are not written back
        std::memcpy(Tcw.data, &R.kf_Tcw[16 * k], 16 * sizeof(float));
        kfs[k]->SetPose(Tcw);
    }
    int i = 0;
    for (MapPoint* pMP : W.lLocalMapPoints) {               // :2066-2074
        std::memcpy(Pos.data, &R.pt_pos[3 * (size_t)i++], 3 * sizeof(float));
        pMP->SetWorldPos(Pos);
        pMP->UpdateNormalAndDepth();
    }
    pMap->IncreaseChangeIndex();
}

/* ------------------------------------------------------------------ ORBmatcher::Fuse
 * int Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th, const bool bRight)
 * for bRight == false (ORBmatcher.cc:1629-1818): the search half on the device, the update half
 * here in list order (its skip checks are re-evaluated: earlier updates can change them). */
template <class KeyFrame, class MapPoint>
int Fuse(LocalMapper& hot, KeyFrame* pKF, const std::vector<MapPoint*>& vpMapPoints, float th) {
    const int n = (int)vpMapPoints.size();
    std::vector<slam_mp_geom> G(n);
    std::vector<uint8_t> D(32 * (size_t)n, 0);
    for (int i = 0; i < n; i++) {
        MapPoint* pMP = vpMapPoints[i];
        slam_mp_geom& g = G[i];
        g.is_bad = !pMP || pMP->isBad();
        g.seen = pMP && pMP->IsInKeyFrame(pKF);
        if (!pMP) continue;
        const cv::Mat P = pMP->GetWorldPos(), nrm = pMP->GetNormal(), d = pMP->GetDescriptor();
        for (int k = 0; k < 3; k++) {
            g.pos[k] = P.template at<float>(k);
            g.normal[k] = nrm.template at<float>(k);
        }
        g.min_dist = pMP->GetMinDistance();  // raw mfMinDistance / mfMaxDistance: the kernels apply the
        g.max_dist = pMP->GetMaxDistance();  // 0.8f / 1.2f invariance factors and PredictScale themselves
        g.has_obs = pMP->Observations() > 0;
        std::memcpy(&D[32 * (size_t)i], d.data, 32);
    }
    slam_frame_view v{};
    v.n = pKF->N;
    v.kps_un = kp_ptr(pKF->mvKeysUn);
    v.uright = pKF->mvuRight.data();
    v.desc = pKF->mDescriptors.data;
    v.min_x = (float)pKF->mnMinX;
    v.min_y = (float)pKF->mnMinY;
    v.max_x = (float)pKF->mnMaxX;
    v.max_y = (float)pKF->mnMaxY;
    v.grid_inv_w = pKF->mfGridElementWidthInv;
    v.grid_inv_h = pKF->mfGridElementHeightInv;
    v.nlevels = pKF->mnScaleLevels;
    v.scale = pKF->mvScaleFactors.data();
    v.log_scale = pKF->mfLogScaleFactor;
    v.fx = pKF->fx;
    v.fy = pKF->fy;
    v.cx = pKF->cx;
    v.cy = pKF->cy;
    v.bf = pKF->mbf;
    v.b = pKF->mb;
    float T[16];
    mat4(pKF->GetPose(), T);
    v.Tcw = T;
    std::vector<int32_t> bi, bd;
    hot.FuseSearch(v, pKF->mvInvLevelSigma2.data(), G, D.data(), th, bi, bd);
    int nFused = 0;
    for (int i = 0; i < n; i++) {  // :1789-1816
        MapPoint* pMP = vpMapPoints[i];
        if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
        if (bd[i] > ORBmatcher::TH_LOW) continue;
        MapPoint* pMPinKF = pKF->GetMapPoint(bi[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, bi[i]);
            pKF->AddMapPoint(pMP, bi[i]);
        }
        nFused++;
    }
    return nFused;
}

}  // namespace orbslam3
}  // namespace slamhot

#endif  // SLAMHOT_ORBSLAM3_HPP
