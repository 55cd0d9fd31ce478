/*
 * lba_oracle.cpp — CPU restatement of the g2o Levenberg-Marquardt / Schur solve that
 * Optimizer::LocalBundleAdjustment runs (Optimizer.cc:1611-2078).  TEST INFRASTRUCTURE ONLY
 * (see oracle.h): the checker for the device LBA and the CPU baseline of bench.py.
 *
 * Parity status: "parity unpinned" — g2o + Eigen cannot be built here (no Eigen, SURVEY.md
 * §8c) and the reference ships no BA fixtures.  Every step restates the g2o / Eigen code
 * cited next to it, in the reference's evaluation order, with the reference's float quirks
 * (float camera parameters, float Huber dsqr, float invz + float bf*invz in the stereo edge).
 * One documented deviation: LinearSolverEigen's SimplicialLDLT with AMD ordering
 * (linear_solver_eigen.h:60-237) is restated as a dense LDL^T in natural order; both factor
 * the same matrix exactly (no pivoting), so only rounding differs (<< the 1e-5 tolerance).
 */
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/slamhot.h"
#include "g2o_math.hpp"
#include "g2o_sites.hpp"

namespace {

using namespace g2o_oracle;

struct Edge {
    int pt, kf;
    bool stereo;
    bool body;              // EdgeSE3ProjectXYZToBody (right camera, mTrl)
    double obs[3];
    double info;            // invSigma2 (float) promoted: Information = I * invSigma2
    double err[3];          // _error of the last computeActiveErrors
    double A[9];            // _jacobianOplusXi (point), D x 3 row-major
    double B[18];           // _jacobianOplusXj (pose),  D x 6 row-major
    double Hpl[18];         // pose-landmark block B^T W A, 6 x 3 row-major
};

// One KeyFrame's pinhole parameters (float, promoted): the edge's camera.
struct KCam {
    double fx, fy, cx, cy, bf;
};

struct Solver {
    const slam_lba_problem* P;
    // per KeyFrame: its own camera (e->pCamera = pKFi->mpCamera, e->fx..bf = pKFi->fx..mbf,
    // Optimizer.cc:1840, 1869-1873) and its mpCamera2 (body edges, :1906)
    std::vector<KCam> kc, kc2;
    std::vector<SE3> trl;       // per KF: Converter::toSE3Quat(pKFi->mTrl)
    double delta_mono, delta_stereo;
    float dsqr_mono, dsqr_stereo;  // RobustKernelHuber::dsqr is float (robust_kernel_impl.h:84)
    std::vector<SE3> pose, pose_bak;
    std::vector<double> pt, pt_bak;
    std::vector<int> hidx;   // pose Hessian index (-1 fixed)
    int np = 0;              // free poses
    std::vector<Edge> E;
    std::vector<std::vector<int>> pt_edges;  // per point: edges with free pose, by pose index
    // system
    std::vector<double> Hpp;   // np x 36 diagonal blocks
    std::vector<double> Hll;   // npt x 9
    std::vector<double> b;     // 6 np + 3 npt
    std::vector<double> x;
    std::vector<double> Hs;    // dense (6 np)^2, row-major
    double lambda = -1, ni = 2;
    int nBad = 0;
    int stop = 0;
    int trials = 0;

    int npt() const { return P->n_pt; }

    // EdgeSE3ProjectXYZ::computeError (OptimizableTypes.h:97-102) + Pinhole::project
    // (Pinhole.cpp:42-48); EdgeStereoSE3ProjectXYZ::computeError / cam_project
    // (types_six_dof_expmap.h:157-162, types_six_dof_expmap.cpp:190-197).  Round 5: the mapping,
    // the stereo projection, chi2 and the Huber kernel as the reference's objects compute them
    // (g2o_sites.hpp, tests/test_fp64_sites.py).
    void compute_error(Edge& e) {
        double Xc[3];
        if (e.body) {
            // EdgeSE3ProjectXYZToBody::computeError (OptimizableTypes.h:127-132):
            // obs - pCamera->project((mTrl * T_lw).map(X_w)), as compiled (round 6: body_error_cc)
            const KCam& K2 = kc2[e.kf];
            const double Kd[4] = {K2.fx, K2.fy, K2.cx, K2.cy};
            body_error_cc(trl[e.kf], pose[e.kf], &pt[3 * e.pt], Kd, e.obs, e.err);
            return;
        }
        const KCam& K = kc[e.kf];
        map_cc(pose[e.kf], &pt[3 * e.pt], Xc);
        if (!e.stereo) {
            const double Kd[4] = {K.fx, K.fy, K.cx, K.cy};
            double uv[2];
            project_cc(Kd, Xc, uv);
            e.err[0] = e.obs[0] - uv[0];
            e.err[1] = e.obs[1] - uv[1];
        } else {
            double p[3];
            cam_project_stereo_cc(Xc, K.fx, K.fy, K.cx, K.cy, (float)K.bf, p);
            e.err[0] = e.obs[0] - p[0];
            e.err[1] = e.obs[1] - p[1];
            e.err[2] = e.obs[2] - p[2];
        }
    }

    // BaseEdge::chi2 (base_edge.h:58-61) with Information = invSigma2 * I, as compiled
    double chi2(const Edge& e) const { return e.stereo ? chi2_3_cc(e.err, e.info) : chi2_2_cc(e.err, e.info); }

    // RobustKernelHuber::robustify (robust_kernel_impl.cpp:79-91), as compiled
    void robustify(const Edge& e, double c, double* rho) const {
        huber_cc(c, e.stereo ? delta_stereo : delta_mono, e.stereo ? dsqr_stereo : dsqr_mono, rho);
    }

    bool depth_positive(const Edge& e) const {
        double Xc[3];
        if (e.body)  // OptimizableTypes.h:134-138, the product and mapping as computeError's
            map_cc(se3_mul_cc(trl[e.kf], pose[e.kf]), &pt[3 * e.pt], Xc);
        else  // isDepthPositive: _transformVector + t, z > 0 (Optimizer.cc.o final scan)
            map_cc(pose[e.kf], &pt[3 * e.pt], Xc);
        return Xc[2] > 0.0;
    }

    // SparseOptimizer::computeActiveErrors + activeRobustChi2 (sparse_optimizer.cpp:61-114)
    double active_errors() {
        for (Edge& e : E) compute_error(e);
        double chi = 0.0;
        for (const Edge& e : E) {
            double rho[2];
            robustify(e, chi2(e), rho);
            chi += rho[0];
        }
        return chi;
    }

    // EdgeSE3ProjectXYZ::linearizeOplus (OptimizableTypes.cpp:139-160) + Pinhole::projectJac
    // (Pinhole.cpp:88-97); EdgeStereoSE3ProjectXYZ::linearizeOplus (types_six_dof_expmap.cpp:228-275)
    void linearize(Edge& e) {
        if (e.body) {
            linearize_body(e);
            return;
        }
        const SE3& T = pose[e.kf];
        const double fx = kc[e.kf].fx, fy = kc[e.kf].fy, bf = kc[e.kf].bf;
        if (!e.stereo) {  // OptimizableTypes.cpp.o @0x1840, as compiled
            const float Kf[2] = {(float)fx, (float)fy};
            lin_mono_cc(T, &pt[3 * e.pt], Kf, e.A, e.B);
            return;
        }
        lin_stereo_cc(T, &pt[3 * e.pt], fx, fy, bf, e.A, e.B);  // types_six_dof_expmap.cpp.o @0xcf0
    }

    // EdgeSE3ProjectXYZToBody::linearizeOplus (OptimizableTypes.cpp:192-215) as compiled
    // (OptimizableTypes.cpp.o @0xf30, round 6: lin_body_cc): Xi = -projectJac(X_r) R(mTrl * T_lw),
    // Xj = (-projectJac(X_r) R(mTrl)) SE3deriv(X_l).
    void linearize_body(Edge& e) {
        const float Kf[2] = {(float)kc2[e.kf].fx, (float)kc2[e.kf].fy};
        lin_body_cc(trl[e.kf], pose[e.kf], &pt[3 * e.pt], Kf, e.A, e.B);
    }

    // BaseBinaryEdge::constructQuadraticForm, robust branch (base_binary_edge.hpp:55-120),
    // robustInformation (base_edge.h:96-102): W = rho' * Omega.
    void quadratic_form(Edge& e) {
        const int D = e.stereo ? 3 : 2;
        double rho[2];
        robustify(e, chi2(e), rho);
        const double w = rho[1] * e.info;  // weightedOmega diagonal
        double om_r[3];
        for (int k = 0; k < D; k++) om_r[k] = (-(e.info * e.err[k])) * rho[1];
        const int ip = 3 * e.pt;
        // from = point: b += A^T om_r, Hll += A^T W A
        for (int c = 0; c < 3; c++) {
            double s = 0;
            for (int k = 0; k < D; k++) s += e.A[3 * k + c] * om_r[k];
            b[6 * np + ip + c] += s;
        }
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += (e.A[3 * k + r] * w) * e.A[3 * k + c];
                Hll[9 * e.pt + 3 * r + c] += s;
            }
        const int h = hidx[e.kf];
        if (h < 0) return;
        // Hpl (pose row, landmark col) = B^T W A (the transposed-block write)
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += (e.B[6 * k + r] * w) * e.A[3 * k + c];
                e.Hpl[3 * r + c] = s;
            }
        for (int c = 0; c < 6; c++) {
            double s = 0;
            for (int k = 0; k < D; k++) s += e.B[6 * k + c] * om_r[k];
            b[6 * h + c] += s;
        }
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += (e.B[6 * k + r] * w) * e.B[6 * k + c];
                Hpp[36 * h + 6 * r + c] += s;
            }
    }

    // BlockSolver::buildSystem (block_solver.hpp:501-560).  Two edges between the same pose and
    // point (a KeyFrame's left and right observation, Optimizer.cc:1818-1914) write one shared
    // Hpl block: the follower's product is added to the leader's, in edge order.
    std::vector<int> lead;  // per edge: the edge whose Hpl block it accumulates into (itself = own)
    void build_system() {
        std::fill(Hpp.begin(), Hpp.end(), 0.0);
        std::fill(Hll.begin(), Hll.end(), 0.0);
        std::fill(b.begin(), b.end(), 0.0);
        for (size_t i = 0; i < E.size(); i++) {
            Edge& e = E[i];
            linearize(e);
            quadratic_form(e);
            if (lead[i] != (int)i && hidx[e.kf] >= 0)
                for (int k = 0; k < 18; k++) E[lead[i]].Hpl[k] += e.Hpl[k];
        }
    }

    // OptimizationAlgorithmLevenberg::computeLambdaInit (optimization_algorithm_levenberg.cpp:171-185)
    double lambda_init(double user) const {
        if (user > 0) return user;
        double m = 0.;
        for (int i = 0; i < np; i++)
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(Hpp[36 * i + 7 * j]), m);
        for (int i = 0; i < npt(); i++)
            for (int j = 0; j < 3; j++) m = std::max(std::fabs(Hll[9 * i + 4 * j]), m);
        return 1e-5 * m;
    }

    // Dense LDL^T of the Schur complement (deviation from SimplicialLDLT + AMD, see header).
    // Fails like Eigen's factorize when a pivot is exactly zero.
    bool ldlt_solve(std::vector<double>& A, int n, const double* rhs, double* out) {
        std::vector<double> d(n);
        for (int j = 0; j < n; j++) {
            double dj = A[(size_t)j * n + j];
            for (int k = 0; k < j; k++) dj -= A[(size_t)j * n + k] * A[(size_t)j * n + k] * d[k];
            if (dj == 0.0) return false;
            d[j] = dj;
            for (int i = j + 1; i < n; i++) {
                double s = A[(size_t)i * n + j];
                for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k] * d[k];
                A[(size_t)i * n + j] = s / dj;
            }
        }
        std::vector<double> y(rhs, rhs + n);
        for (int i = 0; i < n; i++)
            for (int k = 0; k < i; k++) y[i] -= A[(size_t)i * n + k] * y[k];
        for (int i = 0; i < n; i++) y[i] /= d[i];
        for (int i = n - 1; i >= 0; i--)
            for (int k = i + 1; k < n; k++) y[i] -= A[(size_t)k * n + i] * y[k];
        std::memcpy(out, y.data(), sizeof(double) * n);
        return true;
    }

    // BlockSolver::solve, Schur branch (block_solver.hpp:353-486), lambda already on the
    // diagonals (setLambda, :563-590).
    bool solve_system() {
        const int n = 6 * np;
        Hs.assign((size_t)n * n, 0.0);
        for (int i = 0; i < np; i++)
            for (int r = 0; r < 6; r++)
                for (int c = r; c < 6; c++) Hs[(size_t)(6 * i + r) * n + 6 * i + c] = Hpp[36 * i + 6 * r + c];
        std::vector<double> coeff(n, 0.0);
        std::vector<double> Dinv(9 * (size_t)npt());
        for (int l = 0; l < npt(); l++) {
            inverse3(&Hll[9 * l], &Dinv[9 * l]);
            const double* Di = &Dinv[9 * l];
            const double* bl = &b[n + 3 * l];
            double db[3];
            for (int r = 0; r < 3; r++) db[r] = Di[3 * r] * bl[0] + Di[3 * r + 1] * bl[1] + Di[3 * r + 2] * bl[2];
            const std::vector<int>& col = pt_edges[l];
            for (size_t a = 0; a < col.size(); a++) {
                const Edge& ei = E[col[a]];
                const int i1 = hidx[ei.kf];
                double BD[18];
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++)
                        BD[3 * r + c] = ei.Hpl[3 * r] * Di[c] + ei.Hpl[3 * r + 1] * Di[3 + c] +
                                        ei.Hpl[3 * r + 2] * Di[6 + c];
                for (int r = 0; r < 6; r++)
                    coeff[6 * i1 + r] += ei.Hpl[3 * r] * db[0] + ei.Hpl[3 * r + 1] * db[1] + ei.Hpl[3 * r + 2] * db[2];
                for (size_t bq = a; bq < col.size(); bq++) {
                    const Edge& ej = E[col[bq]];
                    const int i2 = hidx[ej.kf];
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 6; c++)
                            Hs[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -=
                                BD[3 * r] * ej.Hpl[3 * c] + BD[3 * r + 1] * ej.Hpl[3 * c + 1] +
                                BD[3 * r + 2] * ej.Hpl[3 * c + 2];
                }
            }
        }
        // the upper triangle is authoritative (SimplicialLDLT<.., Upper>): mirror it
        for (int r = 0; r < n; r++)
            for (int c = 0; c < r; c++) Hs[(size_t)r * n + c] = Hs[(size_t)c * n + r];
        std::vector<double> bs(n);
        for (int i = 0; i < n; i++) bs[i] = b[i] - coeff[i];
        if (!ldlt_solve(Hs, n, bs.data(), x.data())) return false;
        // cl = bl - Hpl^T xp ; xl = Dinv cl (block_solver.hpp:456-481)
        for (int l = 0; l < npt(); l++) {
            double cl[3] = {b[n + 3 * l], b[n + 3 * l + 1], b[n + 3 * l + 2]};
            for (int ei : pt_edges[l]) {
                const Edge& e = E[ei];
                const double* xp = &x[6 * hidx[e.kf]];
                for (int c = 0; c < 3; c++)
                    for (int r = 0; r < 6; r++) cl[c] += e.Hpl[3 * r + c] * (-xp[r]);
            }
            const double* Di = &Dinv[9 * l];
            for (int r = 0; r < 3; r++)
                x[n + 3 * l + r] = Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1] + Di[3 * r + 2] * cl[2];
        }
        return true;
    }

    // BlockSolver::setLambda(lambda, backup=true) / restoreDiagonal (block_solver.hpp:563-604)
    std::vector<double> diag_bak;
    void set_lambda(double lam) {
        diag_bak.clear();
        for (int i = 0; i < np; i++)
            for (int j = 0; j < 6; j++) {
                diag_bak.push_back(Hpp[36 * i + 7 * j]);
                Hpp[36 * i + 7 * j] += lam;
            }
        for (int i = 0; i < npt(); i++)
            for (int j = 0; j < 3; j++) {
                diag_bak.push_back(Hll[9 * i + 4 * j]);
                Hll[9 * i + 4 * j] += lam;
            }
    }
    void restore_diagonal() {
        size_t k = 0;
        for (int i = 0; i < np; i++)
            for (int j = 0; j < 6; j++) Hpp[36 * i + 7 * j] = diag_bak[k++];
        for (int i = 0; i < npt(); i++)
            for (int j = 0; j < 3; j++) Hll[9 * i + 4 * j] = diag_bak[k++];
    }

    // SparseOptimizer::update (sparse_optimizer.cpp:422-435): VertexSE3Expmap::oplusImpl
    // (types_six_dof_expmap.h:71-74) and VertexSBAPointXYZ::oplusImpl (types_sba.h:52-56).
    void update() {
        for (size_t k = 0; k < pose.size(); k++) {
            const int h = hidx[k];
            if (h >= 0) pose[k] = oplus_cc(&x[6 * h], pose[k]);  // as compiled (g2o_sites.hpp, round 6)
        }
        for (int l = 0; l < npt(); l++)
            for (int c = 0; c < 3; c++) pt[3 * l + c] += x[6 * np + 3 * l + c];
    }

    double compute_scale() const {
        double s = 0.;
        for (size_t j = 0; j < x.size(); j++) s += x[j] * (lambda * x[j] + b[j]);
        return s;
    }

    enum { OK, TERMINATE };

    // OptimizationAlgorithmLevenberg::solve (optimization_algorithm_levenberg.cpp:61-169)
    int lm_solve(int iteration, double user_lambda, double* chi_ini_out, double* chi_out) {
        double currentChi = active_errors();
        const double iniChi = currentChi;
        if (chi_ini_out) *chi_ini_out = currentChi;
        build_system();
        if (iteration == 0) {
            lambda = lambda_init(user_lambda);
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            pose_bak = pose;  // push
            pt_bak = pt;
            set_lambda(lambda);
            const bool ok2 = solve_system();
            trials++;
            update();
            restore_diagonal();
            double tempChi = active_errors();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = compute_scale();
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                pose = pose_bak;  // pop
                pt = pt_bak;
            }
            qmax++;
        } while (rho < 0 && qmax < 10 && !stop);
        *chi_out = currentChi;
        if (qmax == 10 || rho == 0) return TERMINATE;
        if ((iniChi - currentChi) * 1e3 < iniChi)
            nBad++;
        else
            nBad = 0;
        if (nBad >= 3) return TERMINATE;
        return OK;
    }

    // SparseOptimizer::optimize (sparse_optimizer.cpp:354-420)
    int optimize(int iterations, double user_lambda, double* chi_ini, double* chi_fin) {
        int it = 0;
        bool ok = true;
        for (int i = 0; i < iterations && !stop && ok; i++) {
            double ci, cf;
            const int r = lm_solve(i, user_lambda, &ci, &cf);
            if (chi_ini && i == 0) *chi_ini = ci;
            *chi_fin = cf;
            ok = r == OK;
            ++it;
        }
        return it;
    }
};

}  // namespace

// LocalBundleAdjustment's Huber deltas (Optimizer.cc:1794-1795: float sqrt, widened by setDelta)
// and outlier thresholds (:2002, :2024: double constants)
const float kThHuberMono = std::sqrt(5.991), kThHuberStereo = std::sqrt(7.815);
constexpr double kChi2Mono = 5.991, kChi2Stereo = 7.815;

extern "C" {

/* Optimizer::LocalBundleAdjustment from the vertex/edge setup on (Optimizer.cc:1722-2077).
 * kf_fixed: 0 free, 1 fixed and written back (the init KF inside lLocalKeyFrames),
 * 2 fixed camera (lFixedCameras, not written back).  stop = *pbStopFlag (static here). */
int oracle_lba_solve(const slam_lba_problem* P, const slam_lba_options* opt, int stop,
                     slam_lba_result* R) {
    Solver S;
    S.P = P;
    S.stop = stop;
    const float thMono = kThHuberMono, thStereo = kThHuberStereo;  // Optimizer.cc:1794-1795
    S.delta_mono = thMono;
    S.delta_stereo = thStereo;
    S.dsqr_mono = (float)(S.delta_mono * S.delta_mono);  // RobustKernelHuber::setDelta
    S.dsqr_stereo = (float)(S.delta_stereo * S.delta_stereo);
    const int nk = P->n_kf, npt = P->n_pt, ne = P->n_edge;
    S.pose.resize(nk);
    S.hidx.assign(nk, -1);
    // vertices without edges are not active (sparse_optimizer.cpp:262-300)
    std::vector<int> kf_edges(nk, 0);
    for (int i = 0; i < ne; i++) kf_edges[P->edge_kf[i]]++;
    S.trl.assign(nk, SE3{{0, 0, 0, 1}, {0, 0, 0}});
    S.kc.resize(nk);
    S.kc2.resize(nk);
    for (int k = 0; k < nk; k++) {
        const slam_camera& c = P->kf_cam ? P->kf_cam[k] : P->cam;
        const slam_camera& c2 = P->kf_cam2 ? P->kf_cam2[k] : P->cam2;
        S.kc[k] = KCam{c.fx, c.fy, c.cx, c.cy, c.bf};
        S.kc2[k] = KCam{c2.fx, c2.fy, c2.cx, c2.cy, 0.0};
        S.pose[k] = se3_from_cv(P->kf_Tcw + 16 * k);
        if (P->edge_body && P->kf_Trl) S.trl[k] = se3_from_cv(P->kf_Trl + 16 * k);
        if (P->kf_fixed[k] == 0 && kf_edges[k] > 0) S.hidx[k] = S.np++;
    }
    S.pt.resize(3 * (size_t)npt);
    for (int i = 0; i < 3 * npt; i++) S.pt[i] = P->pt_pos[i];
    S.E.resize(ne);
    S.pt_edges.assign(npt, {});
    for (int i = 0; i < ne; i++) {
        Edge& e = S.E[i];
        e.pt = P->edge_pt[i];
        e.kf = P->edge_kf[i];
        e.body = P->edge_body && P->edge_body[i];
        e.stereo = !e.body && P->edge_obs[3 * i + 2] >= 0;  // mvuRight < 0 -> mono (Optimizer.cc:1822, 1852)
        for (int c = 0; c < 3; c++) e.obs[c] = P->edge_obs[3 * i + c];
        e.info = P->edge_inv_sigma2[i];
        e.err[0] = e.err[1] = e.err[2] = 0;
    }
    // one Hpl block per (pose, point): an edge right after one on the same point and KeyFrame
    // (the body edge after the left edge) shares that edge's block
    S.lead.resize(ne);
    for (int i = 0; i < ne; i++) {
        const Edge& e = S.E[i];
        const bool follows = i > 0 && S.E[i - 1].pt == e.pt && S.E[i - 1].kf == e.kf;
        S.lead[i] = follows ? S.lead[i - 1] : i;
        if (S.hidx[e.kf] >= 0 && !follows) S.pt_edges[e.pt].push_back(i);
    }
    // HplCCS columns are sorted by pose row (block_solver.hpp:247, fillSparseBlockMatrixCCS)
    for (auto& col : S.pt_edges) {
        for (size_t a = 1; a < col.size(); a++)
            for (size_t b = a; b > 0 && S.hidx[S.E[col[b - 1]].kf] > S.hidx[S.E[col[b]].kf]; b--)
                std::swap(col[b - 1], col[b]);
    }
    S.Hpp.assign(36 * (size_t)S.np, 0.0);
    S.Hll.assign(9 * (size_t)npt, 0.0);
    S.b.assign(6 * (size_t)S.np + 3 * (size_t)npt, 0.0);
    S.x.assign(S.b.size(), 0.0);

    R->iterations[0] = R->iterations[1] = 0;
    R->trials = 0;
    R->chi2_initial = 0;
    R->chi2_final = 0;
    R->lambda_final = 0;
    R->n_outlier = 0;
    R->ran = stop ? 0 : 1;
    if (stop) {  // Optimizer.cc:1921-1923: return before optimizing, nothing written back
        std::memcpy(R->kf_Tcw, P->kf_Tcw, sizeof(float) * 16 * nk);
        std::memcpy(R->pt_pos, P->pt_pos, sizeof(float) * 3 * npt);
        std::memset(R->edge_outlier, 0, ne);
        return 0;
    }
    double cf = 0;
    const double ul = P->user_lambda_init > 0 ? P->user_lambda_init : opt->user_lambda_init;
    // an empty graph makes initializeOptimization / optimize fail (sparse_optimizer.cpp:282-285)
    if (ne > 0) R->iterations[0] = S.optimize(opt->iters_first, ul, &R->chi2_initial, &cf);
    if (!S.stop && ne > 0) R->iterations[1] = S.optimize(opt->iters_second, ul, nullptr, &cf);
    R->chi2_final = cf;
    R->lambda_final = S.lambda;
    R->trials = S.trials;
    int nout = 0;
    for (int i = 0; i < ne; i++) {
        const Edge& e = S.E[i];
        const double th = e.stereo ? kChi2Stereo : kChi2Mono;
        const bool bad = S.chi2(e) > th || !S.depth_positive(e);
        R->edge_outlier[i] = bad;
        nout += bad;
    }
    R->n_outlier = nout;
    for (int k = 0; k < nk; k++) {
        if (P->kf_fixed[k] == 2)
            std::memcpy(R->kf_Tcw + 16 * k, P->kf_Tcw + 16 * k, sizeof(float) * 16);
        else
            se3_to_cv(S.pose[k], R->kf_Tcw + 16 * k);
    }
    for (int i = 0; i < 3 * npt; i++) R->pt_pos[i] = (float)S.pt[i];
    return 0;
}

/* {Huber delta mono, stereo (as setDelta receives them), chi2 mono, stereo} for test_fp_sites.py */
void oracle_fp_lba_consts(double* out) {
    out[0] = (double)kThHuberMono;
    out[1] = (double)kThHuberStereo;
    out[2] = kChi2Mono;
    out[3] = kChi2Stereo;
}

}  // extern "C"
