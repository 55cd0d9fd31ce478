// Sanitizer driver (test infrastructure, CPU only, no HIP call): the LBA host planning path of
// six solver handles planning at once, each handle's pool growing between calls
// (slamhot_lba_plan_stress, built into a -DSLAMHOT_PLAN_BENCH library under TSan or ASan by
// `make sanitize-plan`).  Windows are synthetic config-4 shapes (50 KeyFrames, 2 fixed, 2000
// MapPoints x 8 observations, a third of them stereo), generated here.
//   plan_stress [threads] [rounds]    -> exit 0 and "plan_stress ok" when every plan agrees
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "slamhot.h"

extern "C" slam_status slamhot_lba_plan_stress(int nthreads, int rounds, const int* counts, int ncounts, int n_prob,
                                               const slam_lba_problem* probs, const slam_lba_options* opt);

namespace {

struct Window {
    std::vector<float> Tcw, pt, obs, isig;
    std::vector<uint8_t> fixed;
    std::vector<int32_t> ept, ekf;
};

struct Lcg {
    unsigned long long s;
    double next() {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return (double)(s >> 11) / 9007199254740992.0;
    }
};

Window make_window(int seed, int nkf, int npt, int obs) {
    Lcg r{(unsigned long long)seed * 7919ull + 17ull};
    Window w;
    w.Tcw.assign(16 * nkf, 0.f);
    w.fixed.assign(nkf, 0);
    for (int k = 0; k < nkf; k++) {
        float* T = &w.Tcw[16 * k];
        T[0] = T[5] = T[10] = T[15] = 1.f;
        T[3] = (float)(0.1 * k + 0.01 * r.next());
        T[7] = (float)(0.02 * r.next());
        T[11] = (float)(0.02 * r.next());
    }
    w.fixed[0] = 1;
    w.fixed[nkf - 1] = 2;
    for (int p = 0; p < npt; p++) {
        w.pt.push_back((float)(4.0 * r.next() - 2.0 + 0.1 * (p % nkf)));
        w.pt.push_back((float)(3.0 * r.next() - 1.5));
        w.pt.push_back((float)(3.0 + 4.0 * r.next()));
        const int k0 = (int)(r.next() * (nkf - obs));
        for (int o = 0; o < obs; o++) {
            w.ept.push_back(p);
            w.ekf.push_back(k0 + o);
            w.obs.push_back((float)(640.0 * r.next()));
            w.obs.push_back((float)(480.0 * r.next()));
            w.obs.push_back(r.next() < 0.33 ? (float)(300.0 * r.next()) : -1.f);
            w.isig.push_back(1.f / (float)(1 << (2 * (int)(r.next() * 3))));
        }
    }
    return w;
}

}  // namespace

int main(int argc, char** argv) {
    const int nthreads = argc > 1 ? std::atoi(argv[1]) : 6;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 3;
    const int nwin = 128;
    std::vector<Window> ws;
    for (int i = 0; i < 8; i++) ws.push_back(make_window(i, 50, 2000, 8));
    std::vector<slam_lba_problem> probs(nwin);
    for (int i = 0; i < nwin; i++) {
        const Window& w = ws[i % ws.size()];
        slam_lba_problem& P = probs[i];
        std::memset(&P, 0, sizeof(P));
        P.n_kf = (int32_t)w.fixed.size();
        P.kf_Tcw = w.Tcw.data();
        P.kf_fixed = w.fixed.data();
        P.n_pt = (int32_t)(w.pt.size() / 3);
        P.pt_pos = w.pt.data();
        P.n_edge = (int32_t)w.ept.size();
        P.edge_pt = w.ept.data();
        P.edge_kf = w.ekf.data();
        P.edge_obs = w.obs.data();
        P.edge_inv_sigma2 = w.isig.data();
        P.cam = slam_camera{458.654f, 457.296f, 367.215f, 248.375f, 47.9f};
    }
    slam_lba_options opt;
    std::memset(&opt, 0, sizeof(opt));
    opt.iters_first = 5;
    opt.iters_second = 10;
    const int counts[] = {4, 8, 128, 1, 16};
    const slam_status st = slamhot_lba_plan_stress(nthreads, rounds, counts, 5, nwin, probs.data(), &opt);
    if (st != SLAM_OK) {
        std::fprintf(stderr, "plan_stress: status %d\n", (int)st);
        return 1;
    }
    std::printf("plan_stress ok: %d threads x %d rounds x {4, 8, 128, 1, 16} windows\n", nthreads, rounds);
    return 0;
}
