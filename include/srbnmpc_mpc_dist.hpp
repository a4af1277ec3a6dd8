/*
 * srbnmpc_mpc_dist.hpp -- header-only C++ class with the reference's per-agent MPC_dist call
 * surface (/root/reference/include/MPC_dist.hpp:137-190) on top of the batched C ABI in
 * srbnmpc.h (srb_solve_batch with a batch of one).  Drivers written against MPC_dist
 * (src/A1_Sim.cpp:180-197, driver_scripts/qp_only_exp.cpp:156-188) compile against this class
 * unchanged; see INTEGRATION.md for the two-line switch.
 *
 * What stays on the host, as in the reference: copPlanner_eventbase (MPC_dist.cpp:702-782),
 * footholdsPlanner (:1204-1266) and the bookkeeping of gaitDomain_ / the alpha buffer
 * (:450-453, :798).  What goes to the GPU: the QP assembly + iSWIFT QP + closest-obstacle
 * scan + NLP (:99-427) and fitComTrajectory_eventbase (:784-855, fused epilogue).
 *
 * Matrix types: with Eigen available (define SRBNMPC_USE_EIGEN, or have <eigen3/Eigen/Dense>
 * on the include path) the getters return Eigen::MatrixXd / Eigen::Vector4d exactly as the
 * reference does; otherwise a minimal column-major srbnmpc::Mat with the same accessors
 * (operator()(i, j), rows(), cols(), data()).  Setters accept any type with operator()(i, j)
 * (Eigen matrices included) or raw column-major pointers.
 *
 * Errors: the C ABI never throws; this C++ layer throws std::runtime_error with
 * srb_last_error() when a context cannot be created (e.g. no GPU) or a solve call fails.
 * A non-optimal solver exit is NOT an error (the reference returns the last iterate too,
 * iswift_qp.cpp:126-151); it is reported by last_status().
 */
#ifndef SRBNMPC_MPC_DIST_HPP
#define SRBNMPC_MPC_DIST_HPP

#include <array>
#include <cmath>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "srbnmpc.h"

#if !defined(SRBNMPC_USE_EIGEN) && defined(__has_include)
#if __has_include(<eigen3/Eigen/Dense>)
#define SRBNMPC_USE_EIGEN 1
#endif
#endif
#ifdef SRBNMPC_USE_EIGEN
#include <eigen3/Eigen/Dense>
#endif

namespace srbnmpc {

#ifdef SRBNMPC_USE_EIGEN
using Mat = Eigen::MatrixXd;
using Vec4 = Eigen::Vector4d;
#else
/* Minimal column-major dense matrix (the subset of Eigen::MatrixXd the drivers use). */
class Mat {
public:
    Mat() = default;
    Mat(long r, long c) : r_(r), c_(c), v_((size_t)(r * c), 0.0) {}
    static Mat Zero(long r, long c) { return Mat(r, c); }
    void setZero(long r, long c) { *this = Mat(r, c); }
    double &operator()(long i, long j) { return v_[(size_t)(j * r_ + i)]; }
    double operator()(long i, long j) const { return v_[(size_t)(j * r_ + i)]; }
    double &operator()(long i) { return v_[(size_t)i]; }
    double operator()(long i) const { return v_[(size_t)i]; }
    long rows() const { return r_; }
    long cols() const { return c_; }
    double *data() { return v_.data(); }
    const double *data() const { return v_.data(); }

private:
    long r_ = 0, c_ = 0;
    std::vector<double> v_;
};
using Vec4 = Mat;
#endif

/* reference constants (include/global_loco_opts.h:8-31, MPC_dist.cpp:1206-1209) */
constexpr int NDOMAIN = 4;
constexpr double INIT_FOOTPRINT[4][2] = {{0.2188, -0.1320}, {0.2188, 0.1320}, {-0.1472, -0.1320}, {-0.1472, 0.1320}};

/* Horizon: the reference hard-codes N = NDOMAIN = 4 grids (MPC_dist.cpp:92, :104).  The second
 * constructor argument generalises it (BASELINE configs[0]: horizon 10): the reference window still
 * starts at column NDOMAIN * gaitDomain_ (a gait domain is NDOMAIN grids) and spans N columns, every
 * grid gets the domain's footholds, get_MPCsol() is 4N x 1 and the Bezier fit keeps using X_0..X_3;
 * the default N = NDOMAIN is the reference exactly. */
class MPC_dist {
public:
    bool use_snopt = false;       /* MPC_dist.hpp:139: false -> QP stage only (srb_solve_qp) */

    explicit MPC_dist(int device = 0, int horizon = NDOMAIN) : device_(device), N_(horizon)
    {
        if (horizon < NDOMAIN || horizon > 33) throw std::runtime_error("MPC_dist: horizon must be in [4, 33]");
        X_.assign((size_t)(4 * N_), 0.0);
    }
    MPC_dist(const MPC_dist &) = delete;
    MPC_dist &operator=(const MPC_dist &) = delete;
    ~MPC_dist()
    {
        for (auto &kv : ctx_) srb_ctx_destroy(kv.second);
    }

    /* ------------------------------------------------------------------ setters */
    void setAgentID(size_t agent_id) { agent_id_ = agent_id; }

    /* Pstart: 2*NA x 1 (x, y of every agent); sets this agent's start and alpha buffer */
    template <class V> void setPstart(const V &Pstart)
    {
        agent_initial_[0] = Pstart((long)(2 * agent_id_), 0);
        agent_initial_[1] = Pstart((long)(2 * agent_id_ + 1), 0);
        alpha_buffer_ = {agent_initial_[0], 0.0, agent_initial_[1], 0.0};
        pstart_.resize((size_t)Pstart.rows());
        for (long i = 0; i < (long)Pstart.rows(); i++) pstart_[(size_t)i] = Pstart(i, 0);
    }
    /* Pobs / Pobs_real: 2 x NOBS (MPC_dist.hpp:85-86); run_NMPC uses Pobs_real (:371-396) */
    template <class M> void setPobs(const M &P) { copy_obs(P, pobs_); }
    template <class M> void setPobs_real(const M &P) { copy_obs(P, pobs_real_); }
    void setPobs_real(const double *xy_colmajor, int n_obs)
    {
        pobs_real_.assign(xy_colmajor, xy_colmajor + 2 * n_obs);
    }

    /* MPC_dist.cpp:930-1104 on the device (srb_hl_plan): every agent from Pstart around the
     * planner obstacles Pobs; fills Pr_refined_ / Prd_refined_ (2NA x loop/40). */
    void generateReferenceTrajectory(int loop = 100000)
    {
        if (pstart_.empty()) throw std::runtime_error("MPC_dist: setPstart() not called");
        const int NA = (int)(pstart_.size() / 2), T = loop / 40;
        pr_.assign((size_t)2 * NA * T, 0.0);
        prd_.assign((size_t)2 * NA * T, 0.0);
        if (srb_hl_plan(device_, NA, pstart_.data(), pobs_.empty() ? nullptr : pobs_.data(),
                        (int)(pobs_.size() / 2), loop, pr_.data(), prd_.data()) != SRB_OK)
            throw std::runtime_error(srb_last_error());
        ref_rows_ = 2 * NA; ref_cols_ = T;
    }

    /* Output of the HL planner (generateReferenceTrajectory) when the caller already holds it:
     * Pr_refined_, Prd_refined_ as 2*NA x T column-major arrays. */
    void setReferenceTrajectory(const double *Pr, const double *Prd, int rows, int cols)
    {
        pr_.assign(Pr, Pr + (size_t)rows * cols);
        prd_.assign(Prd, Prd + (size_t)rows * cols);
        ref_rows_ = rows; ref_cols_ = cols;
    }

    /* MPC_dist.cpp:1195-1202 */
    template <class T34, class V4>
    void updateState(const double *qin, const double *dqin, const int *ind, const T34 &toePos, const V4 &state_vec)
    {
        for (int i = 0; i < 18; i++) { q_[i] = qin[i]; dq_[i] = dqin[i]; }
        for (int i = 0; i < 4; i++) contact_[i] = ind[i];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) toe_[r][c] = toePos(r, c);
        for (int i = 0; i < 4; i++) state_other_[i] = state_vec(i, 0);
    }

    /* ------------------------------------------------------------------ solve */
    /* MPC_dist.cpp:81-454 with the QP/NLP solve on the GPU (batch of one). */
    void run_NMPC()
    {
        const int N = N_;
        std::vector<double> ref((size_t)(4 * N));
        copPlanner_eventbase(ref.data());
        std::vector<double> F;                       /* 2 x C, row-major */
        const int C = footholdsPlanner(F);
        std::vector<double> foot((size_t)N * 2 * C); /* same block every grid (:1256-1260) */
        for (int k = 0; k < N; k++)
            for (int i = 0; i < 2 * C; i++) foot[(size_t)k * 2 * C + i] = F[(size_t)i];
        const double x0[4] = {q_[0], dq_[0], q_[1], dq_[1]};   /* :226-229 */
        srb_ctx *ctx = context(C, use_snopt ? 1 : 0);
        srb_params p;
        srb_params_default(&p, N, C);
        const int nv = srb_nv(&p);
        x_.assign((size_t)nv, 0.0);
        x_qp_.assign((size_t)nv, 0.0);
        double obj = 0.0;
        srb_batch b{};
        b.struct_size = sizeof b;            /* ABI check (SRB_ABI_VERSION) */
        b.x0 = x0; b.ref = ref.data(); b.foot = foot.data();
        b.obstacles = pobs_real_.empty() ? nullptr : pobs_real_.data();
        b.n_obs = (int)(pobs_real_.size() / 2);
        b.nbr_state = nullptr; b.n_all = 0; b.agent_offset = 0;
        b.x_qp = x_qp_.data(); b.x = x_.data(); b.obj = &obj; b.status = status_; b.iters = iters_;
        /* fitComTrajectory_eventbase :784-855 runs as the solve kernel's epilogue */
        b.alpha_buf = alpha_buffer_.data(); b.alpha = alpha_.data();
        const int rc = use_snopt ? srb_solve_batch(ctx, 1, &b) : srb_solve_qp(ctx, 1, &b);
        if (rc != SRB_OK) throw std::runtime_error(std::string("srb_solve_batch: ") + srb_last_error());
        /* copy-out :431-440, buffer update :798 */
        for (int i = 0; i < 4 * N; i++) X_[(size_t)i] = x_[(size_t)i];
        for (int d = 0; d < 4; d++) alpha_buffer_[(size_t)d] = X_[(size_t)(4 * (NDOMAIN - 1) + d)];   /* the domain's end */
        gaitDomain_++;
    }

    /* ------------------------------------------------------------------ getters */
    Mat get_alphaCOM() const                       /* 4 x 5 (MPC_dist.hpp:178) */
    {
        Mat a = Mat::Zero(4, 5);
        for (int d = 0; d < 4; d++)
            for (int j = 0; j < 5; j++) a(d, j) = alpha_[(size_t)(d * 5 + j)];
        return a;
    }
    Mat get_MPCsol() const                         /* 4N x 1 predicted X (16 x 1 in the reference, MPC_dist.hpp:179) */
    {
        Mat m = Mat::Zero(4 * N_, 1);
        for (int i = 0; i < 4 * N_; i++) m(i, 0) = X_[(size_t)i];
        return m;
    }
    int getDomain() const { return domain_; }
    Vec4 get_lastState() const                     /* measured, not predicted (:1272-1276) */
    {
#ifdef SRBNMPC_USE_EIGEN
        Vec4 v;
#else
        Vec4 v(4, 1);
#endif
        v(0, 0) = q_[0]; v(1, 0) = q_[1]; v(2, 0) = dq_[0]; v(3, 0) = dq_[1];
        return v;
    }
    /* MPC_dist.cpp:21-40 */
    void updateDistance_to_fail()
    {
        if (!is_success_) return;
        for (size_t i = 0; i + 1 < pobs_real_.size(); i += 2) {
            if (std::hypot(q_[0] - pobs_real_[i], q_[1] - pobs_real_[i + 1]) < 0.5) {
                is_success_ = false;
                distance_to_fail_ = std::hypot(q_[0], q_[1]);
                break;
            }
        }
    }
    double getDistance_to_fail() const { return distance_to_fail_; }

    /* extras (not in the reference surface): the full decision vectors and solver codes */
    const std::vector<double> &decision_vector() const { return x_; }
    const std::vector<double> &qp_solution() const { return x_qp_; }
    std::pair<int, int> last_status() const { return {status_[0], status_[1]}; }
    std::pair<int, int> last_iters() const { return {iters_[0], iters_[1]}; }
    /* Pr_refined_ / Prd_refined_ (2NA x T column-major) as generateReferenceTrajectory left them */
    const std::vector<double> &Pr_refined() const { return pr_; }
    const std::vector<double> &Prd_refined() const { return prd_; }
    size_t gaitDomain() const { return gaitDomain_; }
    int horizon() const { return N_; }

private:
    template <class M> static void copy_obs(const M &P, std::vector<double> &out)
    {
        out.resize((size_t)(2 * P.cols()));
        for (long j = 0; j < P.cols(); j++) { out[(size_t)(2 * j)] = P(0, j); out[(size_t)(2 * j + 1)] = P(1, j); }
    }

    srb_ctx *context(int C, int use_nlp)
    {
        const int key = C * 2 + use_nlp;            /* one horizon per object */
        auto it = ctx_.find(key);
        if (it != ctx_.end()) return it->second;
        srb_params p;
        srb_params_default(&p, N_, C);        /* K_obs = 1 (closest obstacle), K_nbr = 0 */
        p.use_nlp = use_nlp;
        srb_ctx *c = nullptr;
        if (srb_ctx_create(&p, 1, device_, &c) != SRB_OK)
            throw std::runtime_error(std::string("srb_ctx_create: ") + srb_last_error());
        /* the per-agent surface keeps the reference's QP solution (qp_solution_eventbased_, iSWIFT's
         * tolerance): the QP stage is not shortened here */
        if (srb_ctx_set_option(c, SRB_OPT_QP_WARM_TOL, 0.0) != SRB_OK)
            throw std::runtime_error(std::string("srb_ctx_set_option: ") + srb_last_error());
        ctx_[key] = c;
        return c;
    }

    /* MPC_dist.cpp:702-782: 4 x N window of the HL path from column NDOMAIN*gaitDomain_, flattened
     * column-major (x, xdot, y, ydot per grid). */
    void copPlanner_eventbase(double *ref) const
    {
        if (pr_.empty()) throw std::runtime_error("MPC_dist: setReferenceTrajectory() not called");
        const int N = N_;
        const long c0 = (long)NDOMAIN * (long)gaitDomain_;
        if (c0 + N > ref_cols_) throw std::runtime_error("MPC_dist: reference trajectory exhausted");
        const long r0 = 2 * (long)agent_id_;
        auto at = [&](const std::vector<double> &M, long r, long c) { return M[(size_t)(c * ref_rows_ + r)]; };
        for (int k = 0; k < N; k++) {
            ref[4 * k + 0] = at(pr_, r0, c0 + k);
            ref[4 * k + 1] = at(prd_, r0, c0 + k);
            ref[4 * k + 2] = at(pr_, r0 + 1, c0 + k);
            ref[4 * k + 3] = at(prd_, r0 + 1, c0 + k);
        }
    }

    /* MPC_dist.cpp:1204-1266: stance footholds, F row-major 2 x C, legs in FR,FL,RR,RL order */
    int footholdsPlanner(std::vector<double> &F)
    {
        if (gaitDomain_ <= 1)
            for (int l = 0; l < 4; l++) {
                toe_[0][l] = INIT_FOOTPRINT[l][0] + agent_initial_[0];
                toe_[1][l] = INIT_FOOTPRINT[l][1] + agent_initial_[1];
                toe_[2][l] = 0.0;
            }
        const int contacts = contact_[0] + contact_[1] + contact_[2] + contact_[3];
        int legs[4], C;
        if (contacts == 4) { C = 4; legs[0] = 0; legs[1] = 1; legs[2] = 2; legs[3] = 3; }
        else if (contacts == 2 && contact_[0] == 0) { C = 2; legs[0] = 1; legs[1] = 2; }
        else if (contacts == 2 && contact_[0] == 1) { C = 2; legs[0] = 0; legs[1] = 3; }
        else throw std::runtime_error("MPC_dist: unsupported contact pattern");
        F.assign((size_t)(2 * C), 0.0);
        for (int i = 0; i < C; i++) { F[(size_t)i] = toe_[0][legs[i]]; F[(size_t)(C + i)] = toe_[1][legs[i]]; }
        return C;
    }

    int device_;
    int N_;                                      /* horizon (grids) */
    size_t agent_id_ = 0, gaitDomain_ = 0;
    int domain_ = 0;
    bool is_success_ = true;
    double distance_to_fail_ = 10.0;             /* MPC_dist.cpp:51 */
    std::array<double, 2> agent_initial_{{0.0, 0.0}};
    std::array<double, 4> alpha_buffer_{{0.0, 0.0, 0.0, 0.0}};
    std::vector<double> pstart_, pobs_, pobs_real_, pr_, prd_;
    long ref_rows_ = 0, ref_cols_ = 0;
    double q_[18] = {0}, dq_[18] = {0};
    int contact_[4] = {1, 1, 1, 1};
    double toe_[3][4] = {{0}};
    double state_other_[4] = {0};
    std::map<int, srb_ctx *> ctx_;
    std::vector<double> x_, x_qp_;
    std::vector<double> X_;
    std::array<double, 20> alpha_{};
    int status_[2] = {0, 0}, iters_[2] = {0, 0};
};

}  // namespace srbnmpc

#endif
