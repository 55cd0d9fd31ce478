/*
 * pose_oracle.cpp — CPU restatement of Optimizer::PoseOptimization (Optimizer.cc:824-1118),
 * pinhole, with g2o's LM (optimization_algorithm_levenberg.cpp:61-194), unary edges
 * EdgeSE3ProjectXYZOnlyPose (OptimizableTypes.h:31-57, OptimizableTypes.cpp:49-63) and
 * EdgeStereoSE3ProjectXYZOnlyPose (types_six_dof_expmap.h:208-236, .cpp:339-404),
 * BaseUnaryEdge::constructQuadraticForm (base_unary_edge.hpp) and LinearSolverDense (Eigen
 * LDLT; restated as an unpivoted LDL^T that fails when a pivot is negative, like
 * LDLT::isPositive()).  TEST INFRASTRUCTURE ONLY (see oracle.h).  Parity unpinned (no Eigen /
 * g2o here, no reference fixtures).
 */
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/slamhot.h"
#include "g2o_math.hpp"
#include "g2o_sites.hpp"

namespace {

using namespace g2o_oracle;

struct PEdge {
    int idx;           // feature index
    bool stereo;
    double obs[3];
    double info;
    double Xw[3];
    double err[3];
    int level;         // 0 active, 1 outlier
    bool robust;
};

struct PoseSolver {
    double fx, fy, cx, cy, bf;
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;
    std::vector<PEdge> E;
    SE3 est;
    double H[36], b[6], x[6];
    double lambda = 0, ni = 2;
    int nBad = 0;

    // EdgeSE3ProjectXYZOnlyPose::computeError (OptimizableTypes.h:44-49 + Pinhole::project) and
    // EdgeStereoSE3ProjectXYZOnlyPose::computeError / cam_project (types_six_dof_expmap.cpp:
    // 377-386), chi2 and the Huber kernel as the reference's objects compute them (round 5,
    // g2o_sites.hpp, tests/test_fp64_sites.py)
    void compute_error(PEdge& e) const {
        double Xc[3];
        map_cc(est, e.Xw, Xc);
        if (!e.stereo) {
            const double K[4] = {fx, fy, cx, cy};
            double uv[2];
            project_cc(K, Xc, uv);
            e.err[0] = e.obs[0] - uv[0];
            e.err[1] = e.obs[1] - uv[1];
            e.err[2] = 0;
        } else {
            double p[3];
            cam_project_pose_stereo_cc(Xc, fx, fy, cx, cy, bf, p);
            e.err[0] = e.obs[0] - p[0];
            e.err[1] = e.obs[1] - p[1];
            e.err[2] = e.obs[2] - p[2];
        }
    }

    static double chi2(const PEdge& e) { return e.stereo ? chi2_3_cc(e.err, e.info) : chi2_2_cc(e.err, e.info); }

    void robustify(const PEdge& e, double c, double* rho) const {
        huber_cc(c, e.stereo ? delta_stereo : delta_mono, e.stereo ? dsqr_stereo : dsqr_mono, rho);
    }

    double active_errors() {
        for (PEdge& e : E)
            if (e.level == 0) compute_error(e);
        double chi = 0;
        for (const PEdge& e : E) {
            if (e.level != 0) continue;
            if (e.robust) {
                double rho[2];
                robustify(e, chi2(e), rho);
                chi += rho[0];
            } else {
                chi += chi2(e);
            }
        }
        return chi;
    }

    // OptimizableTypes.cpp.o @0x1630 (mono) and types_six_dof_expmap.cpp.o @0x1280 (stereo), as
    // compiled; A row-major 3x6 (row 2 zero for mono)
    void jacobian(const PEdge& e, double* A) const {
        if (!e.stereo) {
            const float Kf[2] = {(float)fx, (float)fy};
            lin_pose_mono_cc(est, e.Xw, Kf, A);
            for (int c = 0; c < 6; c++) A[12 + c] = 0;
        } else {
            lin_pose_stereo_cc(est, e.Xw, fx, fy, bf, A);
        }
    }

    // BlockSolver::buildSystem with BaseUnaryEdge::constructQuadraticForm
    void build_system() {
        std::memset(H, 0, sizeof(H));
        std::memset(b, 0, sizeof(b));
        for (const PEdge& e : E) {
            if (e.level != 0) continue;
            double A[18];
            jacobian(e, A);
            const int D = e.stereo ? 3 : 2;
            double rho1 = 1.0;
            if (e.robust) {
                double rho[2];
                robustify(e, chi2(e), rho);
                rho1 = rho[1];
            }
            const double w = rho1 * e.info;
            for (int c = 0; c < 6; c++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += A[6 * k + c] * (e.info * e.err[k]);
                b[c] -= rho1 * s;
            }
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 6; c++) {
                    double s = 0;
                    for (int k = 0; k < D; k++) s += (A[6 * k + r] * w) * A[6 * k + c];
                    H[6 * r + c] += s;
                }
        }
    }

    bool solve6(const double* M, const double* rhs, double* out) const {
        double L[36], d[6];
        for (int j = 0; j < 6; j++) {
            double dj = M[6 * j + j];
            for (int k = 0; k < j; k++) dj -= L[6 * j + k] * L[6 * j + k] * d[k];
            if (dj < 0.0) return false;  // LDLT::isPositive
            d[j] = dj;
            for (int i = j + 1; i < 6; i++) {
                double s = M[6 * i + j];
                for (int k = 0; k < j; k++) s -= L[6 * i + k] * L[6 * j + k] * d[k];
                L[6 * i + j] = s / dj;
            }
        }
        double y[6];
        for (int i = 0; i < 6; i++) {
            y[i] = rhs[i];
            for (int k = 0; k < i; k++) y[i] -= L[6 * i + k] * y[k];
        }
        for (int i = 0; i < 6; i++) y[i] /= d[i];
        for (int i = 5; i >= 0; i--)
            for (int k = i + 1; k < 6; k++) y[i] -= L[6 * k + i] * y[k];
        std::memcpy(out, y, sizeof(y));
        return true;
    }

    enum { OK, TERMINATE };

    int lm_solve(int iteration) {
        double currentChi = active_errors();
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) {
            double m = 0;
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(H[7 * j]), m);
            lambda = 1e-5 * m;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            const SE3 backup = est;
            double Hl[36];
            std::memcpy(Hl, H, sizeof(H));
            for (int j = 0; j < 6; j++) Hl[7 * j] += lambda;
            const bool ok2 = solve6(Hl, b, x);
            est = oplus_cc(x, est);  // VertexSE3Expmap::oplusImpl as compiled (g2o_sites.hpp, round 6)
            double tempChi = active_errors();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                est = backup;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) return TERMINATE;
        if ((iniChi - currentChi) * 1e3 < iniChi)
            nBad++;
        else
            nBad = 0;
        if (nBad >= 3) return TERMINATE;
        return OK;
    }

    void optimize(int iterations) {
        bool any = false;
        for (const PEdge& e : E) any |= e.level == 0;
        if (!any) return;  // initializeOptimization(0) finds no active vertex: optimize() fails
        bool ok = true;
        for (int i = 0; i < iterations && ok; i++) ok = lm_solve(i) == OK;
    }
};

}  // namespace

extern "C" int oracle_pose_optimization(const slam_pose_frame* F, slam_pose_result* R) {
    PoseSolver S;
    S.fx = F->cam.fx;
    S.fy = F->cam.fy;
    S.cx = F->cam.cx;
    S.cy = F->cam.cy;
    S.bf = F->cam.bf;
    const float deltaMono = std::sqrt(5.991), deltaStereo = std::sqrt(7.815);  // Optimizer.cc:852-853
    S.delta_mono = deltaMono;
    S.delta_stereo = deltaStereo;
    S.dsqr_mono = (float)(S.delta_mono * S.delta_mono);
    S.dsqr_stereo = (float)(S.delta_stereo * S.delta_stereo);
    for (int i = 0; i < F->n; i++) {
        if (!F->has_mp[i]) continue;
        PEdge e;
        e.idx = i;
        e.stereo = !(F->uright[i] < 0);
        e.obs[0] = F->kps_un[i].x;
        e.obs[1] = F->kps_un[i].y;
        e.obs[2] = e.stereo ? F->uright[i] : 0.0;
        e.info = F->inv_sigma2[F->kps_un[i].octave];
        for (int c = 0; c < 3; c++) e.Xw[c] = F->mp_pos[3 * i + c];
        e.err[0] = e.err[1] = e.err[2] = 0;
        e.level = 0;
        e.robust = true;
        S.E.push_back(e);
        R->outlier[i] = 0;  // pFrame->mvbOutlier[i] = false (:870, :905)
    }
    const int nInitial = (int)S.E.size();
    R->n_initial = nInitial;
    std::memcpy(R->Tcw, F->Tcw, sizeof(R->Tcw));
    if (nInitial < 3) {
        R->n_inliers = 0;
        return 0;
    }
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    int nBadObs = 0;
    for (int it = 0; it < 4; it++) {
        S.est = se3_from_cv(F->Tcw);  // vSE3->setEstimate(Converter::toSE3Quat(pFrame->mTcw))
        S.optimize(10);
        nBadObs = 0;
        for (PEdge& e : S.E) {
            if (R->outlier[e.idx]) S.compute_error(e);
            const float chi2 = (float)PoseSolver::chi2(e);
            if (chi2 > (e.stereo ? chi2Stereo : chi2Mono)) {
                R->outlier[e.idx] = 1;
                e.level = 1;
                nBadObs++;
            } else {
                R->outlier[e.idx] = 0;
                e.level = 0;
            }
            if (it == 2) e.robust = false;
        }
        if (nInitial < 10) break;  // optimizer.edges().size() < 10
    }
    se3_to_cv(S.est, R->Tcw);
    R->n_inliers = nInitial - nBadObs;
    return R->n_inliers;
}
