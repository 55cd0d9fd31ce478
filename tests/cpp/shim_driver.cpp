// shim_driver.cpp — TEST INFRASTRUCTURE: runs the drop-in shim bodies of
// include/slamhot_orbslam3.hpp on the ORB-SLAM3 stand-ins (orbslam3_standins.hpp).
//
//   shim_driver flatten MAP OUT   Optimizer::LocalBundleAdjustment's window + flattening only
//                                 (host logic: no device needed) -> counts + slam_lba_problem arrays
//   shim_driver lba MAP OUT       the whole LocalBundleAdjustment shim on the device -> counts,
//                                 KeyFrame poses, MapPoint positions, surviving observations
//   shim_driver pose FRAME OUT    the PoseOptimization shim on one Frame
//   shim_driver lbatime MAP OUT [N]  wall-clock per call of the LocalBundleAdjustment shim (N calls,
//                                 each on a freshly loaded map)
//   shim_driver bow PAIR OUT      ORB_SLAM3::ORBmatcher(nnratio, checkOri).SearchByBoW(pKF, F, ...)
//                                 through the reference-side binding of INTEGRATION.md, once per
//                                 (nnratio, checkOri) listed in PAIR, all on this one thread
//   shim_driver bowkk PAIR OUT    SearchByBoW(pKF1, pKF2, vpMatches12) per (nnratio, checkOri)
//   shim_driver projlast IN OUT   SearchByProjection(CurrentFrame, LastFrame, th, bMono) per call
//   shim_driver projkf IN OUT     SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
//   shim_driver computebow IN OUT Frame::ComputeBoW and KeyFrame::ComputeBoW per vocabulary
//   shim_driver extract IN OUT    ORBextractor::operator() incl. mvImagePyramid, per image
//   shim_driver stereo IN OUT     the stereo Frame's two extractions + ComputeStereoMatches
//   shim_driver localpoints IN OUT  Tracking::SearchLocalPoints (both halves)
//   shim_driver fuse IN OUT       ORBmatcher::Fuse(pKF, vpMapPoints, th) incl. its map updates
//
// MAP / FRAME are little-endian binaries written by tests/shim_io.py.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <set>
#include <string>

#include "orbslam3_standins.hpp"
// the shim bodies are written against these names (the reference's namespace)
using namespace ORB_SLAM3;
#include "slamhot_orbslam3.hpp"

namespace {

struct Reader {
    std::vector<char> buf;
    size_t pos = 0;
    explicit Reader(const char* path) {
        std::ifstream f(path, std::ios::binary);
        buf.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    template <class T>
    T get() {
        T v;
        std::memcpy(&v, buf.data() + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
    template <class T>
    void get(T* p, size_t n) {
        std::memcpy(p, buf.data() + pos, sizeof(T) * n);
        pos += sizeof(T) * n;
    }
};

struct Writer {
    FILE* f;
    explicit Writer(const char* path) : f(std::fopen(path, "wb")) {}
    ~Writer() { std::fclose(f); }
    template <class T>
    void put(const T& v) {
        std::fwrite(&v, sizeof(T), 1, f);
    }
    template <class T>
    void put(const std::vector<T>& v) {
        put<int32_t>((int32_t)v.size());
        if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f);
    }
};

struct World {
    Map map;
    std::vector<KeyFrame> kfs;  // contiguous: pointer order = index order (= mnId order here)
    std::vector<MapPoint> mps;
    std::unique_ptr<GeometricCamera> cam2;
    int cur = 0;
};

cv::Mat mat(const float* p, int r, int c) { return slamhot::orbslam3::mat_from(p, r, c); }

void load_map(const char* path, World& W) {
    Reader R(path);
    const int nkf = R.get<int32_t>(), nmp = R.get<int32_t>(), nobs = R.get<int32_t>();
    W.map.mnInitKFid = (unsigned long)R.get<int32_t>();
    W.cur = R.get<int32_t>();
    W.map.mbIsInertial = R.get<int32_t>() != 0;
    const bool rig = R.get<int32_t>() != 0;
    float cam[5], cam2[4], Trl[16], isig[8];
    R.get(cam, 5);
    R.get(cam2, 4);
    R.get(Trl, 16);
    R.get(isig, 8);
    if (rig) W.cam2.reset(new GeometricCamera({cam2[0], cam2[1], cam2[2], cam2[3]}));
    W.kfs.resize(nkf);
    W.mps.resize(nmp);
    for (int k = 0; k < nkf; k++) {
        KeyFrame& K = W.kfs[k];
        K.mnId = (unsigned long)R.get<int32_t>();
        const int nl = R.get<int32_t>(), nr = R.get<int32_t>();
        float T[16];
        R.get(T, 16);
        K.mTcw = mat(T, 4, 4);
        K.fx = cam[0];
        K.fy = cam[1];
        K.cx = cam[2];
        K.cy = cam[3];
        K.mbf = cam[4];
        K.mvInvLevelSigma2.assign(isig, isig + 8);
        K.N = nl;
        K.mvKeysUn.resize(nl);
        K.mvuRight.resize(nl);
        for (int i = 0; i < nl; i++) {
            K.mvKeysUn[i].pt.x = R.get<float>();
            K.mvKeysUn[i].pt.y = R.get<float>();
            K.mvKeysUn[i].octave = R.get<int32_t>();
            K.mvuRight[i] = R.get<float>();
        }
        K.mvKeysRight.resize(nr);
        for (int i = 0; i < nr; i++) {
            K.mvKeysRight[i].pt.x = R.get<float>();
            K.mvKeysRight[i].pt.y = R.get<float>();
            K.mvKeysRight[i].octave = R.get<int32_t>();
        }
        if (rig) {
            K.mpCamera2 = W.cam2.get();
            K.mTrl = mat(Trl, 4, 4);
            K.NLeft = nl;
            K.N = nl + nr;
        }
        K.mvpMapPoints.assign(K.N, nullptr);
        K.mpMap = &W.map;
    }
    for (int p = 0; p < nmp; p++) {
        MapPoint& M = W.mps[p];
        M.mnId = (unsigned long)R.get<int32_t>();
        float X[3];
        R.get(X, 3);
        M.mWorldPos = mat(X, 3, 1);
        M.mpMap = &W.map;
    }
    for (int o = 0; o < nobs; o++) {
        const int k = R.get<int32_t>(), p = R.get<int32_t>(), li = R.get<int32_t>(), ri = R.get<int32_t>();
        KeyFrame* K = &W.kfs[k];
        MapPoint* M = &W.mps[p];
        M->mObservations[K] = std::make_tuple(li, ri);
        if (li >= 0) K->mvpMapPoints[li] = M;
        if (ri >= 0) K->mvpMapPoints[ri] = M;
    }
    const int ncov = R.get<int32_t>();
    for (int i = 0; i < ncov; i++) W.kfs[W.cur].mvpOrderedConnectedKeyFrames.push_back(&W.kfs[R.get<int32_t>()]);
}

int run_flatten(const char* in, const char* out) {
    World W;
    load_map(in, W);
    slamhot::orbslam3::LocalWindow<KeyFrame, MapPoint> L;
    const bool ok = slamhot::orbslam3::BuildLocalWindow(&W.kfs[W.cur], &W.map, L);
    slamhot::LocalBAWindow F;
    std::vector<KeyFrame*> kfs;
    std::vector<std::pair<KeyFrame*, MapPoint*>> refs;
    if (ok) slamhot::orbslam3::FlattenLocalWindow(L, &W.map, F, kfs, refs);
    Writer O(out);
    O.put<int32_t>(ok);
    O.put<int32_t>(L.num_fixedKF);
    O.put<int32_t>((int32_t)L.lLocalKeyFrames.size());
    O.put<int32_t>((int32_t)L.lLocalMapPoints.size());
    std::vector<int32_t> kf_ids;
    for (KeyFrame* k : kfs) kf_ids.push_back((int32_t)k->mnId);
    std::vector<int32_t> mp_ids;
    for (MapPoint* m : L.lLocalMapPoints) mp_ids.push_back((int32_t)m->mnId);
    O.put(kf_ids);
    O.put(mp_ids);
    O.put(F.kf_Tcw);
    O.put(F.kf_fixed);
    O.put(F.pt_pos);
    O.put(F.edge_pt);
    O.put(F.edge_kf);
    O.put(F.edge_obs);
    O.put(F.edge_inv_sigma2);
    O.put(F.edge_body);
    O.put(F.kf_Trl);
    return 0;
}

int run_lba(const char* in, const char* out) {
    World W;
    load_map(in, W);
    slamhot::LocalBundleAdjuster solver(0);
    bool stop = false;
    int nf = 0, no = 0, nm = 0, ne = 0;
    slamhot::orbslam3::LocalBundleAdjustment<KeyFrame, MapPoint, Map>(solver, &W.kfs[W.cur], &stop, &W.map, nf, no,
                                                                       nm, ne);
    Writer O(out);
    O.put<int32_t>(nf);
    O.put<int32_t>(no);
    O.put<int32_t>(nm);
    O.put<int32_t>(ne);
    O.put<int32_t>(W.map.mnChangeIdx);
    std::vector<float> T, P;
    std::vector<int32_t> obs, upd;
    for (KeyFrame& k : W.kfs)
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) T.push_back(k.mTcw.at<float>(r, c));
    for (MapPoint& m : W.mps) {
        for (int c = 0; c < 3; c++) P.push_back(m.mWorldPos.at<float>(c));
        upd.push_back(m.mnNormalUpdates);
        for (auto& o : m.mObservations) {  // surviving (KeyFrame, MapPoint) observations
            obs.push_back((int32_t)(o.first - W.kfs.data()));
            obs.push_back((int32_t)(&m - W.mps.data()));
        }
    }
    O.put(T);
    O.put(P);
    O.put(obs);
    O.put(upd);
    return 0;
}

// wall-clock of the drop-in call: the LocalBundleAdjustment shim (window build, flatten, plan,
// upload, device solve, download, vToErase, write-back) on a freshly loaded map, `reps` times
int run_lba_time(const char* in, const char* out, int reps) {
    slamhot::LocalBundleAdjuster solver(0);
    std::vector<double> ms;
    int nf = 0, no = 0, nm = 0, ne = 0;
    for (int r = 0; r < reps; r++) {
        World W;
        load_map(in, W);
        bool stop = false;
        const auto t0 = std::chrono::steady_clock::now();
        slamhot::orbslam3::LocalBundleAdjustment<KeyFrame, MapPoint, Map>(solver, &W.kfs[W.cur], &stop, &W.map, nf, no,
                                                                           nm, ne);
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    double dev = 0, plan = 0;
    int syncs = 0;
    slamhot::check(slamhot_lba_last_stats(solver.handle(), &dev, &plan, &syncs), "lba_last_stats");
    // where the wall time goes: window build + flattening alone, the solve alone (host wall), on
    // fresh maps; the rest of a call is vToErase and the write-back
    std::vector<double> build_ms, solve_ms;
    for (int r = 0; r < reps; r++) {
        World W;
        load_map(in, W);
        const auto t0 = std::chrono::steady_clock::now();
        slamhot::orbslam3::LocalWindow<KeyFrame, MapPoint> L;
        slamhot::orbslam3::BuildLocalWindow(&W.kfs[W.cur], &W.map, L);
        slamhot::LocalBAWindow F;
        std::vector<KeyFrame*> kfs;
        std::vector<std::pair<KeyFrame*, MapPoint*>> refs;
        slamhot::orbslam3::FlattenLocalWindow(L, &W.map, F, kfs, refs);
        const auto t1 = std::chrono::steady_clock::now();
        slamhot::LocalBAResult res;
        bool stop = false;
        solver.Solve(F, &stop, res);
        const auto t2 = std::chrono::steady_clock::now();
        build_ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        solve_ms.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
    Writer O(out);
    O.put<int32_t>(nf);
    O.put<int32_t>(no);
    O.put<int32_t>(nm);
    O.put<int32_t>(ne);
    O.put(ms);
    O.put(std::vector<double>{dev, plan, (double)syncs});
    O.put(build_ms);
    O.put(solve_ms);
    return 0;
}

// host-only: the whole LocalBundleAdjustment shim with a stand-in for the device solve (results =
// inputs, every 50th edge an outlier), wall clock per call on fresh maps
struct HostOnlyLBA {
    void Solve(const slamhot::LocalBAWindow& f, const bool*, slamhot::LocalBAResult& r,
               const std::function<void()>& overlap = nullptr) {
        if (overlap) overlap();
        r = slamhot::LocalBAResult{};
        r.kf_Tcw = f.kf_Tcw;
        r.pt_pos = f.pt_pos;
        r.edge_outlier.assign(f.edge_pt.size(), 0);
        for (size_t e = 0; e < r.edge_outlier.size(); e += 50) r.edge_outlier[e] = 1;
        r.ran = true;
    }
};

int run_lba_host_time(const char* in, const char* out, int reps) {
    HostOnlyLBA hot;
    std::vector<double> ms;
    int nf = 0, no = 0, nm = 0, ne = 0;
    for (int r = 0; r < reps; r++) {
        World W;
        load_map(in, W);
        bool stop = false;
        const auto t0 = std::chrono::steady_clock::now();
        slamhot::orbslam3::LocalBundleAdjustment<KeyFrame, MapPoint, Map>(hot, &W.kfs[W.cur], &stop, &W.map, nf, no, nm,
                                                                           ne);
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    Writer O(out);
    O.put(ms);
    return 0;
}

// host-only: wall-clock of the window build + flattening on fresh maps (no device)
int run_flat_time(const char* in, const char* out, int reps) {
    std::vector<double> ms;
    for (int r = 0; r < reps; r++) {
        World W;
        load_map(in, W);
        const auto t0 = std::chrono::steady_clock::now();
        slamhot::orbslam3::LocalWindow<KeyFrame, MapPoint> L;
        slamhot::orbslam3::BuildLocalWindow(&W.kfs[W.cur], &W.map, L);
        slamhot::LocalBAWindow F;
        std::vector<KeyFrame*> kfs;
        std::vector<std::pair<KeyFrame*, MapPoint*>> refs;
        slamhot::orbslam3::FlattenLocalWindow(L, &W.map, F, kfs, refs);
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    Writer O(out);
    O.put(ms);
    return 0;
}

int run_pose(const char* in, const char* out) {
    Reader R(in);
    Frame F;
    F.N = R.get<int32_t>();
    float T[16], cam[5], isig[8];
    R.get(T, 16);
    R.get(cam, 5);
    R.get(isig, 8);
    F.mTcw = mat(T, 4, 4);
    F.fx = cam[0];
    F.fy = cam[1];
    F.cx = cam[2];
    F.cy = cam[3];
    F.mbf = cam[4];
    F.mvInvLevelSigma2.assign(isig, isig + 8);
    F.mvKeysUn.resize(F.N);
    F.mvuRight.resize(F.N);
    F.mvpMapPoints.assign(F.N, nullptr);
    F.mvbOutlier.assign(F.N, true);  // stale flags from an earlier optimisation of this Frame
    std::vector<MapPoint> mps(F.N);
    for (int i = 0; i < F.N; i++) {
        F.mvKeysUn[i].pt.x = R.get<float>();
        F.mvKeysUn[i].pt.y = R.get<float>();
        F.mvKeysUn[i].octave = R.get<int32_t>();
        F.mvuRight[i] = R.get<float>();
        const int has = R.get<int32_t>();
        float X[3];
        R.get(X, 3);
        if (has) {
            mps[i].mWorldPos = mat(X, 3, 1);
            F.mvpMapPoints[i] = &mps[i];
        }
    }
    slamhot::PoseOptimizer solver(0);
    const int n = slamhot::orbslam3::PoseOptimization(solver, &F);
    Writer O(out);
    O.put<int32_t>(n);
    std::vector<float> Tout;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) Tout.push_back(F.mTcw.at<float>(r, c));
    std::vector<uint8_t> outl;
    for (int i = 0; i < F.N; i++) outl.push_back(F.mvbOutlier[i] ? 1 : 0);
    O.put(Tout);
    O.put(outl);
    return 0;
}

}  // namespace

// The reference's ORBmatcher (ORBmatcher.h:36-110, stateful only in its two members), with the
// bodies exactly as INTEGRATION.md tells a maintainer to write them.
namespace ORB_SLAM3 {
class ORBmatcher {
   public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono);
    int SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                           const float th, const int ORBdist);

   protected:
    float mfNNratio;
    bool mbCheckOrientation;
};

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    slamhot::ORBmatcher hot(mfNNratio, mbCheckOrientation);  // this thread's device handle, this call's ratio
    return slamhot::orbslam3::SearchByBoW(hot, pKF, F, vpMapPointMatches);
}
int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
    slamhot::ORBmatcher hot(mfNNratio, mbCheckOrientation);
    return slamhot::orbslam3::SearchByBoW(hot, pKF1, pKF2, vpMatches12);
}
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
    slamhot::ORBmatcher hot(mfNNratio, mbCheckOrientation);
    return slamhot::orbslam3::SearchByProjection(hot, CurrentFrame, LastFrame, th, bMono);
}
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const std::set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
    slamhot::ORBmatcher hot(mfNNratio, mbCheckOrientation);
    return slamhot::orbslam3::SearchByProjection(hot, CurrentFrame, pKF, sAlreadyFound, th, ORBdist);
}
}  // namespace ORB_SLAM3

namespace {

// one side of SearchByBoW: N, descriptors, keypoint angles, [MapPoint validity], FeatureVector CSR
template <class Side>
void read_bow_side(Reader& R, Side& S, bool with_valid, std::vector<MapPoint>& mps) {
    const int n = R.get<int32_t>();
    S.N = n;
    S.mDescriptors.create(n, 32, CV_8U);
    if (n) R.get(S.mDescriptors.data, (size_t)n * 32);
    S.mvKeysUn.resize(n);
    for (int i = 0; i < n; i++) S.mvKeysUn[i].angle = R.get<float>();
    if (with_valid) {
        mps.resize(n);
        S.mvpMapPoints.assign(n, nullptr);
        for (int i = 0; i < n; i++) {
            mps[i].mnId = (unsigned long)i;
            if (R.get<uint8_t>()) S.mvpMapPoints[i] = &mps[i];
        }
    }
    const int nn = R.get<int32_t>();
    std::vector<uint32_t> id(nn);
    std::vector<int32_t> off(nn + 1);
    R.get(id.data(), nn);
    R.get(off.data(), nn + 1);
    std::vector<uint32_t> feat(off[nn]);
    R.get(feat.data(), feat.size());
    for (int k = 0; k < nn; k++) S.mFeatVec[id[k]].assign(feat.begin() + off[k], feat.begin() + off[k + 1]);
}

int run_bow(const char* in, const char* out) {
    Reader R(in);
    const int ncalls = R.get<int32_t>();
    std::vector<std::pair<float, bool>> calls;
    for (int c = 0; c < ncalls; c++) {
        const float r = R.get<float>();
        calls.emplace_back(r, R.get<int32_t>() != 0);
    }
    KeyFrame kf;
    Frame F;
    std::vector<MapPoint> mps, unused;
    read_bow_side(R, kf, true, mps);
    read_bow_side(R, F, false, unused);
    Writer O(out);
    for (const auto& c : calls) {  // Tracking.cc:2566 then :3475 on the Tracking thread
        ORB_SLAM3::ORBmatcher matcher(c.first, c.second);
        std::vector<MapPoint*> vpMapPointMatches;
        const int n = matcher.SearchByBoW(&kf, F, vpMapPointMatches);
        std::vector<int32_t> idx(F.N, -1);
        for (int i = 0; i < F.N; i++)
            if (vpMapPointMatches[i]) idx[i] = (int32_t)vpMapPointMatches[i]->mnId;
        O.put<int32_t>(n);
        O.put(idx);
    }
    return 0;
}


// ---------------------------------------------------------------- the remaining shims
// A Frame as the matchers see it (tests/shim_io.py write_frame): pose, camera, Frame statics,
// scale tables and per feature mvKeysUn, mvKeys, mvuRight, descriptor and the MapPoint it holds
// on entry (-1 none, 0 one without observations, 1 one with observations; bad flag).  The
// pre-existing MapPoints are `own` (mnId 1000000 + feature index).
struct FrameIn {
    Frame F;
    std::vector<MapPoint> own;
    std::vector<MapPoint*> initial;  // F.mvpMapPoints on entry
    KeyFrame obs_kf;                 // the one KeyFrame every "observed" MapPoint is seen in
};

void add_obs(MapPoint& m, KeyFrame& k, int idx) { m.mObservations[&k] = std::make_tuple(idx, -1); }

void read_frame(Reader& R, FrameIn& in) {
    Frame& F = in.F;
    F.N = R.get<int32_t>();
    F.mnId = (unsigned long)R.get<int32_t>();
    float T[16];
    R.get(T, 16);
    F.mTcw = mat(T, 4, 4);
    F.fx = R.get<float>();
    F.fy = R.get<float>();
    F.cx = R.get<float>();
    F.cy = R.get<float>();
    F.mbf = R.get<float>();
    F.mb = R.get<float>();
    Frame::mnMinX = R.get<float>();
    Frame::mnMinY = R.get<float>();
    Frame::mnMaxX = R.get<float>();
    Frame::mnMaxY = R.get<float>();
    Frame::mfGridElementWidthInv = R.get<float>();
    Frame::mfGridElementHeightInv = R.get<float>();
    F.mnScaleLevels = R.get<int32_t>();
    F.mvScaleFactors.resize(F.mnScaleLevels);
    R.get(F.mvScaleFactors.data(), F.mnScaleLevels);
    F.mfLogScaleFactor = R.get<float>();
    F.mvInvLevelSigma2.resize(F.mnScaleLevels);
    R.get(F.mvInvLevelSigma2.data(), F.mnScaleLevels);
    const int n = F.N;
    F.mvKeysUn.resize(n);
    F.mvKeys.resize(n);
    F.mvuRight.resize(n);
    F.mDescriptors.create(n, 32, CV_8U);
    F.mvpMapPoints.assign(n, nullptr);
    F.mvbOutlier.assign(n, false);
    in.own.resize(n);
    in.obs_kf.mvuRight.assign(1, -1.f);
    for (int i = 0; i < n; i++) {
        R.get(&F.mvKeysUn[i], 1);
        R.get(&F.mvKeys[i], 1);
        F.mvuRight[i] = R.get<float>();
        R.get(F.mDescriptors.data + 32 * (size_t)i, 32);
        const int st = R.get<int8_t>();
        const int bad = R.get<uint8_t>();
        MapPoint& m = in.own[i];
        m.mnId = 1000000ul + (unsigned long)i;
        m.mbBad = bad != 0;
        if (st >= 0) F.mvpMapPoints[i] = &m;
        if (st == 1) add_obs(m, in.obs_kf, 0);
    }
    in.initial = F.mvpMapPoints;
}

template <class V>
std::vector<int32_t> ids_of(const V& mps) {
    std::vector<int32_t> out;
    for (auto* m : mps) out.push_back(m ? (int32_t)m->mnId : -1);
    return out;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) through ORB_SLAM3::ORBmatcher
int run_projlast(const char* in, const char* out) {
    Reader R(in);
    FrameIn cur;
    read_frame(R, cur);
    Frame last;
    last.N = R.get<int32_t>();
    float T[16];
    R.get(T, 16);
    last.mTcw = mat(T, 4, 4);
    const int n = last.N;
    last.mvKeys.resize(n);
    last.mvKeysUn.resize(n);
    last.mvpMapPoints.assign(n, nullptr);
    last.mvbOutlier.assign(n, false);
    std::vector<MapPoint> mps(n);
    KeyFrame obs_kf;
    obs_kf.mvuRight.assign(1, -1.f);
    for (int i = 0; i < n; i++) {
        R.get(&last.mvKeys[i], 1);
        R.get(&last.mvKeysUn[i], 1);
        const int has = R.get<uint8_t>(), outl = R.get<uint8_t>(), obs = R.get<uint8_t>();
        float X[3];
        R.get(X, 3);
        MapPoint& m = mps[i];
        m.mnId = (unsigned long)i;
        m.mWorldPos = mat(X, 3, 1);
        R.get(m.mDescriptor.data, 32);
        if (obs) add_obs(m, obs_kf, 0);
        if (has) last.mvpMapPoints[i] = &m;
        last.mvbOutlier[i] = outl != 0;
    }
    const int ncalls = R.get<int32_t>();
    Writer O(out);
    for (int c = 0; c < ncalls; c++) {
        const float th = R.get<float>();
        const int mono = R.get<int32_t>();
        const float ratio = R.get<float>();
        const int ori = R.get<int32_t>();
        cur.F.mvpMapPoints = cur.initial;
        ORB_SLAM3::ORBmatcher matcher(ratio, ori != 0);
        const int nm = matcher.SearchByProjection(cur.F, last, th, mono != 0);
        O.put<int32_t>(nm);
        O.put(ids_of(cur.F.mvpMapPoints));
    }
    return 0;
}

// SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) through ORB_SLAM3::ORBmatcher
int run_projkf(const char* in, const char* out) {
    Reader R(in);
    FrameIn cur;
    read_frame(R, cur);
    KeyFrame kf;
    kf.N = R.get<int32_t>();
    const int n = kf.N;
    kf.mvKeysUn.resize(n);
    kf.mvpMapPoints.assign(n, nullptr);
    std::vector<MapPoint> mps(n);
    std::set<MapPoint*> found;
    for (int i = 0; i < n; i++) {
        R.get(&kf.mvKeysUn[i], 1);
        const int has = R.get<uint8_t>(), bad = R.get<uint8_t>(), fnd = R.get<uint8_t>();
        float X[3];
        R.get(X, 3);
        MapPoint& m = mps[i];
        m.mnId = 2000000ul + (unsigned long)i;
        m.mWorldPos = mat(X, 3, 1);
        m.mfMaxDistance = R.get<float>();
        m.mfMinDistance = R.get<float>();
        R.get(m.mDescriptor.data, 32);
        m.mbBad = bad != 0;
        if (has) kf.mvpMapPoints[i] = &m;
        if (has && fnd) found.insert(&m);
    }
    const int ncalls = R.get<int32_t>();
    Writer O(out);
    for (int c = 0; c < ncalls; c++) {
        const float th = R.get<float>();
        const int orb_dist = R.get<int32_t>();
        const float ratio = R.get<float>();
        const int ori = R.get<int32_t>();
        cur.F.mvpMapPoints = cur.initial;
        ORB_SLAM3::ORBmatcher matcher(ratio, ori != 0);
        const int nm = matcher.SearchByProjection(cur.F, &kf, found, th, orb_dist);
        O.put<int32_t>(nm);
        O.put(ids_of(cur.F.mvpMapPoints));
    }
    return 0;
}

// one KeyFrame side of SearchByBoW(KF1, KF2): MapPoints present (has) and bad flags, ids base + i
void read_kf_side(Reader& R, KeyFrame& K, std::vector<MapPoint>& mps, unsigned long base) {
    const int n = R.get<int32_t>();
    K.N = n;
    K.mDescriptors.create(n, 32, CV_8U);
    if (n) R.get(K.mDescriptors.data, (size_t)n * 32);
    K.mvKeysUn.resize(n);
    for (int i = 0; i < n; i++) K.mvKeysUn[i].angle = R.get<float>();
    mps.resize(n);
    K.mvpMapPoints.assign(n, nullptr);
    for (int i = 0; i < n; i++) {
        mps[i].mnId = base + (unsigned long)i;
        if (R.get<uint8_t>()) K.mvpMapPoints[i] = &mps[i];
    }
    for (int i = 0; i < n; i++) mps[i].mbBad = R.get<uint8_t>() != 0;
    const int nn = R.get<int32_t>();
    std::vector<uint32_t> id(nn);
    std::vector<int32_t> off(nn + 1);
    R.get(id.data(), nn);
    R.get(off.data(), nn + 1);
    std::vector<uint32_t> feat(off[nn]);
    R.get(feat.data(), feat.size());
    for (int k = 0; k < nn; k++) K.mFeatVec[id[k]].assign(feat.begin() + off[k], feat.begin() + off[k + 1]);
}

int run_bowkk(const char* in, const char* out) {
    Reader R(in);
    const int ncalls = R.get<int32_t>();
    std::vector<std::pair<float, bool>> calls;
    for (int c = 0; c < ncalls; c++) {
        const float r = R.get<float>();
        calls.emplace_back(r, R.get<int32_t>() != 0);
    }
    KeyFrame k1, k2;
    std::vector<MapPoint> m1, m2;
    read_kf_side(R, k1, m1, 3000000ul);
    read_kf_side(R, k2, m2, 0ul);
    Writer O(out);
    for (const auto& c : calls) {  // LoopClosing / LocalMapping build ORBmatcher(0.75, true) etc.
        ORB_SLAM3::ORBmatcher matcher(c.first, c.second);
        std::vector<MapPoint*> v12;
        const int n = matcher.SearchByBoW(&k1, &k2, v12);
        O.put<int32_t>(n);
        O.put(ids_of(v12));
    }
    return 0;
}

// Frame::ComputeBoW and KeyFrame::ComputeBoW over one vocabulary per case
int run_computebow(const char* in, const char* out) {
    Reader R(in);
    const int ncases = R.get<int32_t>();
    Writer O(out);
    for (int c = 0; c < ncases; c++) {
        const int k = R.get<int32_t>(), L = R.get<int32_t>(), scoring = R.get<int32_t>(),
                  weighting = R.get<int32_t>(), nn = R.get<int32_t>();
        std::vector<int32_t> parent(nn);
        std::vector<uint8_t> leaf(nn), ndesc(32 * (size_t)nn);
        std::vector<double> weight(nn);
        R.get(parent.data(), nn);
        R.get(leaf.data(), nn);
        R.get(ndesc.data(), ndesc.size());
        R.get(weight.data(), nn);
        const int nd = R.get<int32_t>();
        Frame F;
        F.mDescriptors.create(nd, 32, CV_8U);
        R.get(F.mDescriptors.data, 32 * (size_t)nd);
        KeyFrame K;
        K.mDescriptors = F.mDescriptors.clone();
        slamhot::Vocabulary voc(0, k, L, scoring, weighting, nn, parent.data(), leaf.data(), ndesc.data(), weight.data());
        slamhot::orbslam3::ComputeBoW(voc, F);
        std::memset(F.mDescriptors.data, 0, 32 * (size_t)nd);  // computed once: a second call keeps the vectors
        slamhot::orbslam3::ComputeBoW(voc, F);
        slamhot::orbslam3::KeyFrameComputeBoW(voc, &K);
        for (int side = 0; side < 2; side++) {
            const auto& bv = side ? K.mBowVec : F.mBowVec;
            const auto& fv = side ? K.mFeatVec : F.mFeatVec;
            std::vector<uint32_t> w, node, feat;
            std::vector<double> val;
            std::vector<int32_t> off{0};
            for (const auto& kv : bv) {
                w.push_back(kv.first);
                val.push_back(kv.second);
            }
            for (const auto& kv : fv) {
                node.push_back(kv.first);
                feat.insert(feat.end(), kv.second.begin(), kv.second.end());
                off.push_back((int32_t)feat.size());
            }
            O.put(w);
            O.put(val);
            O.put(node);
            O.put(off);
            O.put(feat);
        }
    }
    return 0;
}

// ORBextractor::operator() through the shim, incl. the mvImagePyramid refresh, one extractor
// (one camera) over several images
int run_extract(const char* in, const char* out) {
    Reader R(in);
    const int nfeat = R.get<int32_t>(), nlevels = R.get<int32_t>(), ini = R.get<int32_t>(), mn = R.get<int32_t>();
    const float scale = R.get<float>();
    slamhot::ORBextractor ex(nfeat, scale, nlevels, ini, mn);
    const int nimg = R.get<int32_t>();
    Writer O(out);
    std::vector<cv::Mat> mvImagePyramid;
    for (int i = 0; i < nimg; i++) {
        const int w = R.get<int32_t>(), h = R.get<int32_t>(), lap0 = R.get<int32_t>(), lap1 = R.get<int32_t>();
        cv::Mat img;
        if (w > 0 && h > 0) {
            img.create(h, w, CV_8U);
            R.get(img.data, (size_t)w * h);
        }
        std::vector<cv::KeyPoint> kps;
        cv::Mat desc;
        const std::vector<int> lap{lap0, lap1};
        const int mono = slamhot::orbslam3::ORBextractorCall(ex, img, kps, desc, lap, &mvImagePyramid);
        O.put<int32_t>(mono);
        O.put(kps);
        std::vector<uint8_t> d(desc.data, desc.data + (size_t)desc.rows * 32);
        O.put(d);
        O.put<int32_t>((int32_t)mvImagePyramid.size());
        for (const cv::Mat& m : mvImagePyramid) {
            O.put<int32_t>(m.rows);
            O.put<int32_t>(m.cols);
            O.put(std::vector<uint8_t>(m.data, m.data + (size_t)m.rows * m.cols));
        }
    }
    return 0;
}

// the stereo Frame constructor's host path (Frame.cc:98-152): two extractions, then
// ComputeStereoMatches
int run_stereo(const char* in, const char* out) {
    Reader R(in);
    const int nfeat = R.get<int32_t>(), nlevels = R.get<int32_t>(), ini = R.get<int32_t>(), mn = R.get<int32_t>();
    const float scale = R.get<float>();
    Frame F;
    F.mbf = R.get<float>();
    F.mb = R.get<float>();
    const int w = R.get<int32_t>(), h = R.get<int32_t>();
    cv::Mat l(h, w, CV_8U), r(h, w, CV_8U);
    R.get(l.data, (size_t)w * h);
    R.get(r.data, (size_t)w * h);
    slamhot::ORBextractor left(nfeat, scale, nlevels, ini, mn), right(nfeat, scale, nlevels, ini, mn);
    const std::vector<int> lap{0, 0};
    slamhot::orbslam3::ORBextractorCall(left, l, F.mvKeys, F.mDescriptors, lap);
    slamhot::orbslam3::ORBextractorCall(right, r, F.mvKeysRight, F.mDescriptorsRight, lap);
    slamhot::StereoMatcher sm(0);
    slamhot::orbslam3::ComputeStereoMatches(sm, left, right, F);
    Writer O(out);
    O.put(F.mvKeys);
    O.put(std::vector<uint8_t>(F.mDescriptors.data, F.mDescriptors.data + (size_t)F.mDescriptors.rows * 32));
    O.put(F.mvKeysRight);
    O.put(std::vector<uint8_t>(F.mDescriptorsRight.data, F.mDescriptorsRight.data + (size_t)F.mDescriptorsRight.rows * 32));
    O.put(F.mvuRight);
    O.put(F.mvDepth);
    return 0;
}

// Tracking::SearchLocalPoints: the frame's own MapPoints may also sit in the local map
// (frame_ref >= 0), the others are local-map objects (mnId 3000000 + j)
int run_localpoints(const char* in, const char* out) {
    Reader R(in);
    FrameIn cur;
    read_frame(R, cur);
    Frame& F = cur.F;
    const int nmp = R.get<int32_t>();
    std::vector<MapPoint> local(nmp);
    std::vector<MapPoint*> vpLocal(nmp);
    KeyFrame obs_kf;
    obs_kf.mvuRight.assign(1, -1.f);
    for (int j = 0; j < nmp; j++) {
        const int ref = R.get<int32_t>();
        MapPoint* m = ref >= 0 ? &cur.own[ref] : &local[j];
        if (ref < 0) m->mnId = 3000000ul + (unsigned long)j;
        float X[3], N[3];
        R.get(X, 3);
        R.get(N, 3);
        m->mWorldPos = mat(X, 3, 1);
        m->mNormalVector = mat(N, 3, 1);
        m->mfMinDistance = R.get<float>();
        m->mfMaxDistance = R.get<float>();
        const int seen = R.get<uint8_t>(), bad = R.get<uint8_t>(), obs = R.get<uint8_t>();
        R.get(m->mDescriptor.data, 32);
        if (ref < 0) {
            m->mbBad = bad != 0;
            if (seen) m->mnLastFrameSeen = F.mnId;
            if (obs) add_obs(*m, obs_kf, 0);
        }
        vpLocal[j] = m;
    }
    const float th = R.get<float>();
    const int far = R.get<int32_t>();
    const float th_far = R.get<float>();
    slamhot::ORBmatcher hot(0.8f);  // ORBmatcher matcher(0.8) (Tracking.cc:3234)
    int nmatches = 0;
    const int nToMatch = slamhot::orbslam3::SearchLocalPoints(hot, F, vpLocal, th, far != 0, th_far, &nmatches);
    Writer O(out);
    O.put<int32_t>(nToMatch);
    O.put<int32_t>(nmatches);
    O.put(ids_of(F.mvpMapPoints));
    std::vector<uint8_t> inview;
    std::vector<float> fl;
    std::vector<int32_t> iv;
    for (MapPoint* m : vpLocal) {
        inview.push_back(m->mbTrackInView);
        for (float v : {m->mTrackProjX, m->mTrackProjY, m->mTrackProjXR, m->mTrackDepth, m->mTrackViewCos}) fl.push_back(v);
        iv.push_back(m->mnTrackScaleLevel);
        iv.push_back(m->mnVisible);
        iv.push_back(m->mnLastFrameSeen == F.mnId);
    }
    O.put(inview);
    O.put(fl);
    O.put(iv);
    std::vector<int32_t> own_vis;
    for (const MapPoint& m : cur.own) own_vis.push_back(m.mnVisible);
    O.put(own_vis);
    std::vector<int32_t> pid;
    std::vector<float> pxy;
    for (const auto& kv : F.mmProjectPoints) {
        pid.push_back((int32_t)kv.first);
        pxy.push_back(kv.second.x);
        pxy.push_back(kv.second.y);
    }
    O.put(pid);
    O.put(pxy);
    return 0;
}

// ORBmatcher::Fuse(pKF, vpMapPoints, th) with the update half applied to the stand-in map:
// pKF is KeyFrame 0, the other observations sit in KeyFrames 1..D (slot = MapPoint index)
int run_fuse(const char* in, const char* out) {
    Reader R(in);
    KeyFrame kf;
    kf.mnId = 0;
    kf.N = R.get<int32_t>();
    float T[16];
    R.get(T, 16);
    kf.mTcw = mat(T, 4, 4);
    kf.fx = R.get<float>();
    kf.fy = R.get<float>();
    kf.cx = R.get<float>();
    kf.cy = R.get<float>();
    kf.mbf = R.get<float>();
    kf.mb = R.get<float>();
    kf.mnMinX = R.get<int32_t>();
    kf.mnMinY = R.get<int32_t>();
    kf.mnMaxX = R.get<int32_t>();
    kf.mnMaxY = R.get<int32_t>();
    kf.mfGridElementWidthInv = R.get<float>();
    kf.mfGridElementHeightInv = R.get<float>();
    kf.mnScaleLevels = R.get<int32_t>();
    kf.mvScaleFactors.resize(kf.mnScaleLevels);
    R.get(kf.mvScaleFactors.data(), kf.mnScaleLevels);
    kf.mfLogScaleFactor = R.get<float>();
    kf.mvInvLevelSigma2.resize(kf.mnScaleLevels);
    R.get(kf.mvInvLevelSigma2.data(), kf.mnScaleLevels);
    const int n = kf.N;
    kf.mvKeysUn.resize(n);
    kf.mvuRight.resize(n);
    kf.mDescriptors.create(n, 32, CV_8U);
    kf.mvpMapPoints.assign(n, nullptr);
    for (int i = 0; i < n; i++) {
        R.get(&kf.mvKeysUn[i], 1);
        kf.mvuRight[i] = R.get<float>();
        R.get(kf.mDescriptors.data + 32 * (size_t)i, 32);
    }
    const int nmp = R.get<int32_t>(), ndummy = R.get<int32_t>();
    std::vector<KeyFrame> others(ndummy);
    for (int d = 0; d < ndummy; d++) {
        others[d].mnId = (unsigned long)(1 + d);
        others[d].mvuRight.assign(nmp, -1.f);
        others[d].mvpMapPoints.assign(nmp, nullptr);
    }
    std::vector<MapPoint> mps(nmp);
    for (int j = 0; j < nmp; j++) {
        MapPoint& m = mps[j];
        m.mnId = (unsigned long)j;
        float X[3], N[3];
        R.get(X, 3);
        R.get(N, 3);
        m.mWorldPos = mat(X, 3, 1);
        m.mNormalVector = mat(N, 3, 1);
        m.mfMinDistance = R.get<float>();
        m.mfMaxDistance = R.get<float>();
        m.mbBad = R.get<uint8_t>() != 0;
        R.get(m.mDescriptor.data, 32);
        const int kf_idx = R.get<int32_t>(), nother = R.get<int32_t>();
        if (kf_idx >= 0) {
            m.mObservations[&kf] = std::make_tuple(kf_idx, -1);
            kf.mvpMapPoints[kf_idx] = &m;
        }
        for (int o = 0; o < nother; o++) {
            KeyFrame& K = others[R.get<int32_t>()];
            m.mObservations[&K] = std::make_tuple(j, -1);
            K.mvpMapPoints[j] = &m;
        }
    }
    const int nlist = R.get<int32_t>();
    std::vector<MapPoint*> list(nlist);
    for (int i = 0; i < nlist; i++) {
        const int j = R.get<int32_t>();
        list[i] = j >= 0 ? &mps[j] : nullptr;
    }
    const float th = R.get<float>();
    slamhot::LocalMapper hot(0);
    const int nfused = slamhot::orbslam3::Fuse(hot, &kf, list, th);
    Writer O(out);
    O.put<int32_t>(nfused);
    O.put(ids_of(kf.mvpMapPoints));
    std::vector<int32_t> st, obs;
    for (MapPoint& m : mps) {
        st.push_back(m.mbBad);
        st.push_back(m.Observations());
        std::vector<std::pair<int, int>> o;
        for (const auto& kv : m.mObservations) o.emplace_back((int)kv.first->mnId, std::get<0>(kv.second));
        std::sort(o.begin(), o.end());
        obs.push_back((int32_t)o.size());
        for (const auto& p : o) {
            obs.push_back(p.first);
            obs.push_back(p.second);
        }
    }
    O.put(st);
    O.put(obs);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: shim_driver MODE IN OUT (modes: see the header comment)\n");
        return 2;
    }
    const std::string mode = argv[1];
    try {
        if (mode == "flatten") return run_flatten(argv[2], argv[3]);
        if (mode == "lba") return run_lba(argv[2], argv[3]);
        if (mode == "pose") return run_pose(argv[2], argv[3]);
        if (mode == "bow") return run_bow(argv[2], argv[3]);
        if (mode == "lbatime") return run_lba_time(argv[2], argv[3], argc > 4 ? std::atoi(argv[4]) : 5);
        if (mode == "lbahost") return run_lba_host_time(argv[2], argv[3], argc > 4 ? std::atoi(argv[4]) : 20);
        if (mode == "flattime") return run_flat_time(argv[2], argv[3], argc > 4 ? std::atoi(argv[4]) : 20);
        if (mode == "bowkk") return run_bowkk(argv[2], argv[3]);
        if (mode == "projlast") return run_projlast(argv[2], argv[3]);
        if (mode == "projkf") return run_projkf(argv[2], argv[3]);
        if (mode == "computebow") return run_computebow(argv[2], argv[3]);
        if (mode == "extract") return run_extract(argv[2], argv[3]);
        if (mode == "stereo") return run_stereo(argv[2], argv[3]);
        if (mode == "localpoints") return run_localpoints(argv[2], argv[3]);
        if (mode == "fuse") return run_fuse(argv[2], argv[3]);
    } catch (const slamhot::Error& e) {
        std::fprintf(stderr, "slamhot error: %s\n", e.what());
        return 3;
    }
    return 2;
}
