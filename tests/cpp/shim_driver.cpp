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
//
// MAP / FRAME are little-endian binaries written by tests/shim_io.py.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
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
    Writer O(out);
    O.put<int32_t>(nf);
    O.put<int32_t>(no);
    O.put<int32_t>(nm);
    O.put<int32_t>(ne);
    O.put(ms);
    O.put(std::vector<double>{dev, plan, (double)syncs});
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
// SearchByBoW body exactly as INTEGRATION.md tells a maintainer to write it.
namespace ORB_SLAM3 {
class ORBmatcher {
   public:
    ORBmatcher(float nnratio = 0.6, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);

   protected:
    float mfNNratio;
    bool mbCheckOrientation;
};

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    slamhot::ORBmatcher hot(mfNNratio, mbCheckOrientation);  // this thread's device handle, this call's ratio
    return slamhot::orbslam3::SearchByBoW(hot, pKF, F, vpMapPointMatches);
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

// Instantiations of the shims this driver does not run (they must compile against the
// reference-shaped types; their device paths are exercised through include/slamhot.hpp).
[[maybe_unused]] void instantiate_all(slamhot::ORBmatcher& m, slamhot::LocalMapper& lm, slamhot::StereoMatcher& sm,
                                      slamhot::ORBextractor& exl, slamhot::ORBextractor& exr) {
    KeyFrame kf;
    Frame F;
    std::vector<MapPoint*> out, local;
    slamhot::orbslam3::SearchByBoW(m, &kf, F, out);
    slamhot::orbslam3::SearchLocalPoints(m, F, local, 1.f, false, 50.f);
    slamhot::orbslam3::Fuse(lm, &kf, local, 3.f);
    slamhot::orbslam3::ComputeStereoMatches(sm, exl, exr, F);
    std::vector<cv::KeyPoint> kps;
    cv::Mat img(480, 752, CV_8U), desc;
    std::vector<int> lap{0, 0};
    slamhot::orbslam3::ORBextractorCall(exl, img, kps, desc, lap);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: shim_driver flatten|lba|pose|bow IN OUT\n");
        return 2;
    }
    const std::string mode = argv[1];
    try {
        if (mode == "flatten") return run_flatten(argv[2], argv[3]);
        if (mode == "lba") return run_lba(argv[2], argv[3]);
        if (mode == "pose") return run_pose(argv[2], argv[3]);
        if (mode == "bow") return run_bow(argv[2], argv[3]);
        if (mode == "lbatime") return run_lba_time(argv[2], argv[3], argc > 4 ? std::atoi(argv[4]) : 5);
    } catch (const slamhot::Error& e) {
        std::fprintf(stderr, "slamhot error: %s\n", e.what());
        return 3;
    }
    return 2;
}
