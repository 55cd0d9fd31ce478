/* orbslam3_standins.hpp — TEST INFRASTRUCTURE: minimal stand-ins for the OpenCV and ORB-SLAM3
 * types that include/slamhot_orbslam3.hpp is written against, carrying exactly the members the
 * shims use, with the reference's names and types (KeyFrame.h, MapPoint.h, Frame.h, Map.h,
 * GeometricCamera.h; cv::Mat / cv::KeyPoint of OpenCV 4.x).  They let the drop-in shim bodies
 * compile and run here without OpenCV / g2o / the reference.  Not product code. */
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#define CV_8U 0
#define CV_32F 5

namespace cv {
struct Point2f {
    float x = 0, y = 0;
    Point2f() = default;
    Point2f(float x_, float y_) : x(x_), y(y_) {}
};
struct KeyPoint {  // OpenCV 4.x layout: pt, size, angle, response, octave, class_id
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
class Mat {
   public:
    int rows = 0, cols = 0, type_ = CV_8U;
    size_t step = 0;
    uint8_t* data = nullptr;
    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    void create(int r, int c, int t) {
        rows = r;
        cols = c;
        type_ = t;
        step = (size_t)c * elem();
        buf_ = std::make_shared<std::vector<uint8_t>>((size_t)r * step + 1);
        data = buf_->data();
    }
    size_t elem() const { return type_ == CV_32F ? 4 : 1; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    template <class T>
    T& at(int r, int c) {
        return reinterpret_cast<T*>(data + (size_t)r * step)[c];
    }
    template <class T>
    const T& at(int r, int c) const {
        return reinterpret_cast<const T*>(data + (size_t)r * step)[c];
    }
    template <class T>
    T& at(int i) {  // vector access of a column / row vector
        return cols == 1 ? at<T>(i, 0) : at<T>(0, i);
    }
    template <class T>
    const T& at(int i) const {
        return cols == 1 ? at<T>(i, 0) : at<T>(0, i);
    }
    Mat clone() const {
        Mat m(rows, cols, type_);
        if (rows && cols) std::memcpy(m.data, data, (size_t)rows * step);
        return m;
    }

   private:
    std::shared_ptr<std::vector<uint8_t>> buf_;
};
}  // namespace cv

namespace ORB_SLAM3 {

class KeyFrame;

class GeometricCamera {  // GeometricCamera.h:41-90 (parameters only)
   public:
    explicit GeometricCamera(std::vector<float> p) : mvParameters(std::move(p)) {}
    float getParameter(const int i) { return mvParameters[i]; }
    std::vector<float> mvParameters;
};

class Map {
   public:
    unsigned long mnInitKFid = 0;
    bool mbIsInertial = false;
    int mnChangeIdx = 0;
    std::mutex mMutexMapUpdate;
    unsigned long GetInitKFid() { return mnInitKFid; }
    bool IsInertial() { return mbIsInertial; }
    void IncreaseChangeIndex() { mnChangeIdx++; }
};

class MapPoint {
   public:
    long unsigned int mnId = 0;
    long unsigned int mnBALocalForKF = (unsigned long)-1;
    long unsigned int mnLastFrameSeen = (unsigned long)-1;
    bool mbTrackInView = false, mbTrackInViewR = false;
    float mTrackProjX = -1, mTrackProjY = -1, mTrackProjXR = -1, mTrackDepth = -1, mTrackViewCos = 0;
    int mnTrackScaleLevel = -1, mnVisible = 1, mnNormalUpdates = 0;
    cv::Mat mWorldPos{3, 1, CV_32F}, mNormalVector{3, 1, CV_32F}, mDescriptor{1, 32, CV_8U};
    float mfMinDistance = 0, mfMaxDistance = 0;
    bool mbBad = false;
    Map* mpMap = nullptr;
    std::map<KeyFrame*, std::tuple<int, int>> mObservations;  // ordered by pointer, as the reference

    bool isBad() { return mbBad; }
    Map* GetMap() { return mpMap; }
    cv::Mat GetWorldPos() { return mWorldPos.clone(); }
    void SetWorldPos(const cv::Mat& Pos) { mWorldPos = Pos.clone(); }
    cv::Mat GetNormal() { return mNormalVector.clone(); }
    cv::Mat GetDescriptor() { return mDescriptor.clone(); }
    float GetMinDistance() { return mfMinDistance; }
    float GetMaxDistance() { return mfMaxDistance; }
    float GetMinDistanceInvariance() { return 0.8f * mfMinDistance; }
    float GetMaxDistanceInvariance() { return 1.2f * mfMaxDistance; }
    std::map<KeyFrame*, std::tuple<int, int>> GetObservations() { return mObservations; }
    int Observations();  // nObs: 2 per stereo observation of a one-camera KeyFrame (MapPoint.cc:161-186)
    bool IsInKeyFrame(KeyFrame* pKF) { return mObservations.count(pKF) > 0; }
    void AddObservation(KeyFrame* pKF, int idx) { mObservations[pKF] = std::make_tuple(idx, -1); }
    void EraseObservation(KeyFrame* pKF) { mObservations.erase(pKF); }
    void IncreaseVisible(int n = 1) { mnVisible += n; }
    void UpdateNormalAndDepth() { mnNormalUpdates++; }
    void Replace(MapPoint* pMP);
};

class KeyFrame {
   public:
    long unsigned int mnId = 0;
    long unsigned int mnBALocalForKF = (unsigned long)-1, mnBAFixedForKF = (unsigned long)-1;
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0, mb = 0;
    int N = 0, NLeft = -1;
    std::vector<cv::KeyPoint> mvKeysUn, mvKeysRight;
    std::vector<float> mvuRight, mvInvLevelSigma2, mvScaleFactors;
    cv::Mat mDescriptors, mTcw{4, 4, CV_32F}, mTrl;
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;  // DBoW2::FeatureVector
    std::map<unsigned int, double> mBowVec;                       // DBoW2::BowVector
    int mnScaleLevels = 8, mnMinX = 0, mnMinY = 0, mnMaxX = 752, mnMaxY = 480;
    float mfLogScaleFactor = 0, mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    GeometricCamera* mpCamera2 = nullptr;
    bool mbBad = false;
    Map* mpMap = nullptr;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<KeyFrame*> mvpOrderedConnectedKeyFrames;

    bool isBad() { return mbBad; }
    Map* GetMap() { return mpMap; }
    cv::Mat GetPose() { return mTcw.clone(); }
    void SetPose(const cv::Mat& Tcw) { mTcw = Tcw.clone(); }
    std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() { return mvpOrderedConnectedKeyFrames; }
    std::vector<MapPoint*> GetMapPointMatches() { return mvpMapPoints; }
    MapPoint* GetMapPoint(const size_t& idx) { return mvpMapPoints[idx]; }
    void AddMapPoint(MapPoint* pMP, const size_t& idx) { mvpMapPoints[idx] = pMP; }
    void EraseMapPointMatch(MapPoint* pMP) {
        for (auto& m : mvpMapPoints)
            if (m == pMP) m = nullptr;
    }
};

inline int MapPoint::Observations() {
    int n = 0;
    for (const auto& o : mObservations) {
        const int li = std::get<0>(o.second), ri = std::get<1>(o.second);
        if (li != -1) n += (!o.first->mpCamera2 && o.first->mvuRight[li] >= 0) ? 2 : 1;
        if (ri != -1) n += 1;
    }
    return n;
}

inline void MapPoint::Replace(MapPoint* pMP) {  // MapPoint.cc:238-290 (observation transfer)
    if (pMP->mnId == mnId) return;
    auto obs = mObservations;
    mObservations.clear();
    mbBad = true;
    for (auto& o : obs) {
        KeyFrame* pKF = o.first;
        const int idx = std::get<0>(o.second);
        if (!pMP->IsInKeyFrame(pKF)) {
            if (idx != -1) {
                pKF->mvpMapPoints[idx] = pMP;
                pMP->AddObservation(pKF, idx);
            }
        } else if (idx != -1) {
            pKF->mvpMapPoints[idx] = nullptr;
        }
    }
}

class Frame {
   public:
    static float mnMinX, mnMinY, mnMaxX, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv;
    long unsigned int mnId = 0;
    int N = 0, mnScaleLevels = 8;
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0, mb = 0, mfLogScaleFactor = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
    std::vector<float> mvuRight, mvDepth, mvInvLevelSigma2, mvScaleFactors;
    cv::Mat mDescriptors, mDescriptorsRight, mTcw{4, 4, CV_32F};
    std::map<unsigned int, std::vector<unsigned int>> mFeatVec;
    std::map<unsigned int, double> mBowVec;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::map<long unsigned int, cv::Point2f> mmProjectPoints;
    void SetPose(cv::Mat Tcw) { mTcw = Tcw.clone(); }
};
inline float Frame::mnMinX = 0, Frame::mnMinY = 0, Frame::mnMaxX = 752, Frame::mnMaxY = 480,
             Frame::mfGridElementWidthInv = 64.f / 752.f, Frame::mfGridElementHeightInv = 48.f / 480.f;

}  // namespace ORB_SLAM3
