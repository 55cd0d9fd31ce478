// host_driver.cpp — runs the C++ host layer (include/slamhot.hpp) the way a C++ caller of
// the reference does, on inputs written by tests/test_gpu_cpp_host.py, and writes the
// outputs back as raw binaries for the test to compare against the CPU oracle.
// TEST INFRASTRUCTURE: not part of the product; it only exercises slamhot.hpp.
//
//   host_driver extract <W> <H> <nfeatures> <lap0> <lap1> <image.u8> <out_prefix>
//       ORBextractor(nfeatures, 1.2, 8, 20, 7)(image, kps, desc, {lap0, lap1})
//       -> <out>.kp (N x 28 B), <out>.desc (N x 32 B), <out>.meta (text), <out>.pyr (levels)
//   host_driver bow <strict> <nnratio> <sideA.bin> <sideB.bin> <out.bin>
//       ORBmatcher(nnratio, true).SearchByBoW(A, B, matches) -> int32 n, int32 matches[]
//   host_driver lba <window.bin> <out.bin>
//       Optimizer::LocalBundleAdjustment(window) -> counters, poses, points, outliers, stats
//   host_driver mono <W> <H> <nframes> <n_init> <nfeatures> <images.u8> <calib.bin> <out.bin>
//       monocular Frame construction over a sequence: init / tracking extractors, lap (0, 1000),
//       UndistortKeyPoints, ComputeImageBounds
//
// Exit codes: 0 ok, 2 usage / file error, 3 slamhot::Error (message on stderr).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "slamhot.hpp"

namespace {

std::vector<uint8_t> read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

void write_file(const std::string& path, const void* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)n);
    if (!f) throw std::runtime_error("cannot write " + path);
}

struct Reader {
    const std::vector<uint8_t>& b;
    size_t o = 0;
    template <class T> T get() {
        T v;
        if (o + sizeof(T) > b.size()) throw std::runtime_error("truncated input");
        std::memcpy(&v, b.data() + o, sizeof(T));
        o += sizeof(T);
        return v;
    }
    template <class T> std::vector<T> vec(size_t n) {
        std::vector<T> v(n);
        if (o + n * sizeof(T) > b.size()) throw std::runtime_error("truncated input");
        if (n) std::memcpy(v.data(), b.data() + o, n * sizeof(T));
        o += n * sizeof(T);
        return v;
    }
};

struct Writer {
    std::vector<uint8_t> b;
    template <class T> void put(const T& v) {
        const auto* p = reinterpret_cast<const uint8_t*>(&v);
        b.insert(b.end(), p, p + sizeof(T));
    }
    template <class T> void vec(const std::vector<T>& v) {
        const auto* p = reinterpret_cast<const uint8_t*>(v.data());
        b.insert(b.end(), p, p + v.size() * sizeof(T));
    }
};

int run_extract(char** a) {
    const int W = std::atoi(a[0]), H = std::atoi(a[1]), nf = std::atoi(a[2]);
    const std::vector<int> lap = {std::atoi(a[3]), std::atoi(a[4])};
    const std::vector<uint8_t> img = read_file(a[5]);
    const std::string out = a[6];
    if (img.size() != (size_t)W * H) throw std::runtime_error("image size mismatch");
    slamhot::ORBextractor ex(nf, 1.2f, 8, 20, 7);
    std::vector<slamhot::KeyPoint> kps;
    slamhot::Mat8U desc;
    slamhot::GrayImage gi{img.data(), W, H, (size_t)W};
    const int mono = ex(gi, kps, desc, lap);
    // the empty-image contract: -1 and no exception (ORBextractor.cc:1072-1073)
    std::vector<slamhot::KeyPoint> k2;
    slamhot::Mat8U d2;
    const int empty_ret = ex(slamhot::GrayImage{}, k2, d2, lap);
    write_file(out + ".kp", kps.data(), kps.size() * sizeof(slamhot::KeyPoint));
    write_file(out + ".desc", desc.data.data(), desc.data.size());
    std::vector<uint8_t> pyr;
    for (const slamhot::Mat8U& m : ex.mvImagePyramid()) pyr.insert(pyr.end(), m.data.begin(), m.data.end());
    write_file(out + ".pyr", pyr.data(), pyr.size());
    std::ofstream meta(out + ".meta");
    meta << std::setprecision(9) << kps.size() << " " << mono << " " << empty_ret << " " << ex.GetLevels() << " " << ex.GetScaleFactor();
    for (float s : ex.GetScaleFactors()) meta << " " << s;
    for (int n : ex.GetFeaturesPerLevel()) meta << " " << n;
    meta << "\n";
    return 0;
}

// side file: int32 n | n x 32 desc | n f32 angle | int32 has_valid | [n u8 valid] |
//            int32 n_nodes | n_nodes u32 id | n_nodes+1 i32 off | off[n_nodes] u32 feat
struct Side {
    std::vector<uint8_t> desc, valid;
    std::vector<float> angle;
    std::vector<uint32_t> node_id, node_feat;
    std::vector<int32_t> node_off;
    slam_bow_side view() const {
        slam_bow_side s{};
        s.n = (int32_t)angle.size();
        s.desc = desc.data();
        s.angle = angle.data();
        s.valid = valid.empty() ? nullptr : valid.data();
        s.n_nodes = (int32_t)node_id.size();
        s.node_id = node_id.data();
        s.node_off = node_off.data();
        s.node_feat = node_feat.data();
        return s;
    }
};

Side read_side(const std::string& path) {
    const std::vector<uint8_t> b = read_file(path);
    Reader r{b};
    Side s;
    const int n = r.get<int32_t>();
    s.desc = r.vec<uint8_t>((size_t)n * 32);
    s.angle = r.vec<float>(n);
    if (r.get<int32_t>()) s.valid = r.vec<uint8_t>(n);
    const int nn = r.get<int32_t>();
    s.node_id = r.vec<uint32_t>(nn);
    s.node_off = r.vec<int32_t>(nn + 1);
    s.node_feat = r.vec<uint32_t>(s.node_off.back());
    return s;
}

int run_bow(char** a) {
    const int strict = std::atoi(a[0]);
    const float nnratio = (float)std::atof(a[1]);
    const Side A = read_side(a[2]), B = read_side(a[3]);
    slamhot::ORBmatcher m(nnratio, true);
    std::vector<int> matches;
    int n;
    if (strict) {
        slamhot::KeyFrameBow k1, k2;
        static_cast<slam_bow_side&>(k1) = A.view();
        static_cast<slam_bow_side&>(k2) = B.view();
        n = m.SearchByBoW(k1, k2, matches);
    } else {
        slamhot::KeyFrameBow kf;
        slamhot::FrameBow fr;
        static_cast<slam_bow_side&>(kf) = A.view();
        static_cast<slam_bow_side&>(fr) = B.view();
        n = m.SearchByBoW(kf, fr, matches);
    }
    Writer w;
    w.put<int32_t>(n);
    std::vector<int32_t> mm(matches.begin(), matches.end());
    w.vec(mm);
    // DescriptorDistance of the first descriptor pair, as a host-utility check
    w.put<int32_t>(A.angle.empty() || B.angle.empty() ? -1
                                                       : slamhot::ORBmatcher::DescriptorDistance(A.desc.data(), B.desc.data()));
    write_file(a[4], w.b.data(), w.b.size());
    return 0;
}

// window file: int32 n_kf n_pt n_edge inertial | 5 f32 cam | n_kf*16 f32 Tcw | n_kf u8 fixed |
//              n_pt*3 f32 | n_edge i32 pt | n_edge i32 kf | n_edge*3 f32 obs | n_edge f32 invs2
int run_lba(char** a) {
    const std::vector<uint8_t> b = read_file(a[0]);
    Reader r{b};
    slamhot::LocalBAWindow w;
    const int nkf = r.get<int32_t>(), npt = r.get<int32_t>(), ne = r.get<int32_t>();
    w.inertial = r.get<int32_t>() != 0;
    w.cam.fx = r.get<float>();
    w.cam.fy = r.get<float>();
    w.cam.cx = r.get<float>();
    w.cam.cy = r.get<float>();
    w.cam.bf = r.get<float>();
    w.kf_Tcw = r.vec<float>((size_t)nkf * 16);
    w.kf_fixed = r.vec<uint8_t>(nkf);
    w.pt_pos = r.vec<float>((size_t)npt * 3);
    w.edge_pt = r.vec<int32_t>(ne);
    w.edge_kf = r.vec<int32_t>(ne);
    w.edge_obs = r.vec<float>((size_t)ne * 3);
    w.edge_inv_sigma2 = r.vec<float>(ne);
    slamhot::LocalBundleAdjuster solver;
    slamhot::LocalBAResult res;
    bool stop = false;
    int num_fixedKF = 0, num_OptKF = 0, num_MPs = 0, num_edges = 0;
    slamhot::Optimizer::LocalBundleAdjustment(solver, w, &stop, res, num_fixedKF, num_OptKF, num_MPs, num_edges);
    Writer o;
    o.put<int32_t>(num_fixedKF);
    o.put<int32_t>(num_OptKF);
    o.put<int32_t>(num_MPs);
    o.put<int32_t>(num_edges);
    o.put<int32_t>(res.iterations[0]);
    o.put<int32_t>(res.iterations[1]);
    o.put<int32_t>(res.trials);
    o.put<int32_t>(res.n_outlier);
    o.put<double>(res.chi2_initial);
    o.put<double>(res.chi2_final);
    o.vec(res.kf_Tcw);
    o.vec(res.pt_pos);
    o.vec(res.edge_outlier);
    write_file(a[1], o.b.data(), o.b.size());
    return 0;
}

// Monocular Frame construction over a sequence (Tracking.cc:1335-1346, Frame.cc:262-330):
// frames < n_init go through the 5*nFeatures initialisation extractor (mpIniORBextractor),
// the rest through mpORBextractorLeft; ExtractORB(0, im, 0, 1000) (Frame.cc:306), then
// UndistortKeyPoints, plus ComputeImageBounds once.
// calib file: 4 f32 K | int32 nd | nd f32 dist.  Output: f32 bounds[4], then per frame
// int32 n, int32 mono, n x 28 B mvKeys, n x 28 B mvKeysUn, n x 32 B descriptors.
int run_mono(char** a) {
    const int W = std::atoi(a[0]), H = std::atoi(a[1]), nframes = std::atoi(a[2]), n_init = std::atoi(a[3]);
    const int nfeat = std::atoi(a[4]);
    const std::vector<uint8_t> imgs = read_file(a[5]);
    const std::vector<uint8_t> cb = read_file(a[6]);
    if (imgs.size() != (size_t)W * H * nframes) throw std::runtime_error("image size mismatch");
    Reader r{cb};
    slamhot::PinholeCalib calib;
    for (int i = 0; i < 4; i++) calib.K[i] = r.get<float>();
    calib.dist = r.vec<float>(r.get<int32_t>());
    slamhot::ORBextractor ini(5 * nfeat, 1.2f, 8, 20, 7), left(nfeat, 1.2f, 8, 20, 7);  // Tracking.cc: 5*nFeatures
    Writer o;
    for (float v : slamhot::ComputeImageBounds(calib, W, H)) o.put<float>(v);
    const std::vector<int> lap = {0, 1000};
    for (int f = 0; f < nframes; f++) {
        slamhot::ORBextractor& ex = f < n_init ? ini : left;
        std::vector<slamhot::KeyPoint> kps, kun;
        slamhot::Mat8U desc;
        slamhot::GrayImage gi{imgs.data() + (size_t)f * W * H, W, H, (size_t)W};
        const int mono = ex(gi, kps, desc, lap);
        slamhot::UndistortKeyPoints(calib, kps, kun);
        o.put<int32_t>((int32_t)kps.size());
        o.put<int32_t>(mono);
        o.vec(kps);
        o.vec(kun);
        o.vec(desc.data);
    }
    write_file(a[7], o.b.data(), o.b.size());
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: host_driver extract|bow|lba ...\n");
        return 2;
    }
    const std::string mode = argv[1];
    try {
        if (mode == "extract" && argc == 9) return run_extract(argv + 2);
        if (mode == "bow" && argc == 7) return run_bow(argv + 2);
        if (mode == "lba" && argc == 4) return run_lba(argv + 2);
        if (mode == "mono" && argc == 10) return run_mono(argv + 2);
        std::fprintf(stderr, "bad arguments for %s\n", mode.c_str());
        return 2;
    } catch (const slamhot::Error& e) {
        std::fprintf(stderr, "slamhot::Error %d: %s\n", (int)e.status, e.what());
        return 3;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
}
