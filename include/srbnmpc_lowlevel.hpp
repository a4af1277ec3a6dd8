/*
 * srbnmpc_lowlevel.hpp -- header-only C++ class with the reference's LowLevelCtrl call surface
 * (/root/reference/include/LowLevelCtrl.hpp:15-27) on top of the batched low-level C ABI in
 * srbnmpc.h (srb_ll_calc_torque), plus a batch object for many robots per call.
 *
 *   LowLevelCtrl LL;                                     // LocoWrapper.cpp:32 (new LowLevelCtrl())
 *   const LLInfo *ll = LL.getllPointer();                // LocoWrapper.cpp:42
 *   LL.calcTorque(state, dyn, kin, vcon, con, &params);  // LocoWrapper.cpp:222
 *   double *tau = LL.getTorque();                        // A1_Sim.cpp:206 via LocoWrapper
 *
 * calcTorque is a template over the reference's StateInfo / DynamicsInfo / KinematicsInfo /
 * VCInfo / ContactInfo / Settings::LL_params (global_loco_structs.hpp): it reads them only
 * through the members and accessors the reference code uses -- q(i,0), Dinv(i,j), Jc(i,j),
 * toePos(r,leg), con->ind[i], params->kp, ... -- so Eigen types and any type with the same
 * accessors work.  The GPU computes everything calcTorque computes (QP assembly, the iSWIFT
 * QP, swing PD, integration, swingInvKin); the host only packs and unpacks.
 *
 *   LowLevelBatch batch(max_agents);                     // one launch for many robots
 *   batch.set(a, state, dyn, kin, vcon, con);            // per robot
 *   batch.run(params);                                   // one srb_ll_calc_torque call
 *   batch.ll(a), batch.tau(a)
 *
 * Errors: the C ABI never throws; this layer throws std::runtime_error with srb_last_error()
 * when a context cannot be created (e.g. no GPU) or a call fails.  A non-optimal QP exit is
 * not an error (the reference keeps the returned iterate too); see last_status().
 */
#ifndef SRBNMPC_LOWLEVEL_HPP
#define SRBNMPC_LOWLEVEL_HPP

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "srbnmpc.h"

namespace srbnmpc {

/* LLInfo (global_loco_structs.hpp:74-80) with plain arrays (column vectors as in the reference);
 * as in the reference, ll.tau carries the QP torques (entries 6..17) and getTorque() the member
 * tau array with the swing-leg PD added */
struct LLInfo {
    double tau[18] = {0};
    double QP_force[12] = {0};
    double q[18] = {0}, dq[18] = {0}, ddq[18] = {0};
    double V = 0, dV = 0;
};

/* per-agent element counts of srb_ll_io's inputs (include/srbnmpc.h) */
enum : int { LL_NQ = 18, LL_NU = 12 };

class LowLevelBatch {
public:
    explicit LowLevelBatch(int max_agents, int device = 0) : max_(max_agents), device_(device)
    {
        if (max_agents <= 0) throw std::runtime_error("LowLevelBatch: max_agents must be positive");
        const size_t A = (size_t)max_agents;
        ind_.assign(4 * A, 0);
        q_.assign(A * LL_NQ, 0); dq_.assign(A * LL_NQ, 0); Dinv_.assign(A * LL_NQ * LL_NQ, 0);
        B_.assign(A * LL_NQ * LL_NU, 0); H_.assign(A * LL_NQ, 0); Jc_.assign(A * LL_NU * LL_NQ, 0);
        dJc_.assign(A * LL_NU, 0); Js_.assign(A * LL_NU * LL_NQ, 0); Jtoe_.assign(A * LL_NU * LL_NQ, 0);
        Jhip_.assign(A * LL_NU * LL_NQ, 0); toe_.assign(A * 12, 0); hip_.assign(A * 12, 0);
        H0_.assign(A * LL_NQ * LL_NQ, 0); dH0_.assign(A * LL_NQ, 0); y_.assign(A * LL_NQ, 0);
        dy_.assign(A * LL_NQ, 0); hd_.assign(A * LL_NQ, 0); dhd_.assign(A * LL_NQ, 0); fDes_.assign(A * LL_NU, 0);
        tau_.assign(A * LL_NQ, 0); F_.assign(A * 12, 0); ddq_.assign(A * LL_NQ, 0); dqo_.assign(A * LL_NQ, 0);
        qo_.assign(A * LL_NQ, 0); V_.assign(A, 0); dV_.assign(A, 0); x_.assign(A * 32, 0);
        status_.assign(A, 0); iters_.assign(A, 0);
        used_ = 0;
    }
    ~LowLevelBatch()
    {
        if (ctx_) srb_ll_ctx_destroy(ctx_);
    }
    LowLevelBatch(const LowLevelBatch &) = delete;
    LowLevelBatch &operator=(const LowLevelBatch &) = delete;

    /* pack robot a's inputs (calcTorque's arguments); tau carries over between calls */
    template <class State, class Dyn, class Kin, class VC, class Con>
    void set(int a, const State *state, const Dyn *dyn, const Kin *kin, const VC *vc, const Con *con)
    {
        if (a < 0 || a >= max_) throw std::runtime_error("LowLevelBatch::set: agent index out of range");
        if (a + 1 > used_) used_ = a + 1;
        const size_t A = (size_t)a;
        int cnt = 0;
        for (int i = 0; i < 4; i++) { ind_[4 * A + i] = con->ind[i]; cnt += (con->ind[i] == 1); }
        const int conDim = 3 * cnt, outDim = 6 + 3 * (4 - cnt), sw = 12 - conDim;
        double *D = &Dinv_[A * LL_NQ * LL_NQ], *B = &B_[A * LL_NQ * LL_NU], *H0 = &H0_[A * LL_NQ * LL_NQ];
        double *Jc = &Jc_[A * LL_NU * LL_NQ], *Js = &Js_[A * LL_NU * LL_NQ], *Jt = &Jtoe_[A * LL_NU * LL_NQ],
               *Jh = &Jhip_[A * LL_NU * LL_NQ];
        std::memset(Jc, 0, sizeof(double) * LL_NU * LL_NQ);
        std::memset(Js, 0, sizeof(double) * LL_NU * LL_NQ);
        std::memset(H0, 0, sizeof(double) * LL_NQ * LL_NQ);
        for (int t = 0; t < LL_NQ; t++) {
            q_[A * LL_NQ + t] = state->q(t, 0);
            dq_[A * LL_NQ + t] = state->dq(t, 0);
            H_[A * LL_NQ + t] = dyn->H(t, 0);
            for (int j = 0; j < LL_NQ; j++) D[j * LL_NQ + t] = dyn->Dinv(t, j);
            for (int j = 0; j < LL_NU; j++) B[j * LL_NQ + t] = dyn->B(t, j);
            for (int r = 0; r < conDim; r++) Jc[t * LL_NU + r] = kin->Jc(r, t);
            for (int r = 0; r < sw; r++) Js[t * LL_NU + r] = kin->Js(r, t);
            for (int r = 0; r < LL_NU; r++) { Jt[t * LL_NU + r] = kin->Jtoe(r, t); Jh[t * LL_NU + r] = kin->Jhip(r, t); }
            for (int r = 0; r < outDim; r++) H0[t * LL_NQ + r] = vc->H0(r, t);
            hd_[A * LL_NQ + t] = vc->hd(t, 0);
            dhd_[A * LL_NQ + t] = vc->dhd(t, 0);
        }
        for (int r = 0; r < LL_NU; r++) dJc_[A * LL_NU + r] = (r < conDim) ? kin->dJc(r, 0) : 0.0;
        for (int r = 0; r < LL_NQ; r++) {
            dH0_[A * LL_NQ + r] = (r < outDim) ? vc->dH0(r, 0) : 0.0;
            y_[A * LL_NQ + r] = (r < outDim) ? vc->y(r, 0) : 0.0;
            dy_[A * LL_NQ + r] = (r < outDim) ? vc->dy(r, 0) : 0.0;
        }
        for (int i = 0; i < 4; i++)
            for (int r = 0; r < 3; r++) {
                toe_[A * 12 + 3 * i + r] = kin->toePos(r, i);
                hip_[A * 12 + 3 * i + r] = kin->hipPos(r, i);
            }
        for (int r = 0; r < LL_NU; r++) fDes_[A * LL_NU + r] = vc->fDes(r, 0);
    }

    /* one srb_ll_calc_torque launch over robots 0 .. n-1 (default: every robot set so far) */
    template <class Params>
    void run(const Params *params, int n = -1)
    {
        srb_ll_params p;
        srb_ll_params_default(&p);
        p.mu = params->mu; p.kp = params->kp; p.kd = params->kd; p.useCLF = (int)params->useCLF;
        p.tauPen = params->tauPen; p.dfPen = params->dfPen; p.auxPen = params->auxPen; p.clfPen = params->clfPen;
        p.auxMax = params->auxMax; p.clfEps = params->clfEps;
        run_params(p, n);
    }
    void run_params(const srb_ll_params &p, int n = -1)
    {
        if (n < 0) n = used_;
        if (n > max_) throw std::runtime_error("LowLevelBatch::run: n exceeds max_agents");
        if (!ctx_ || std::memcmp(&p, &params_, sizeof p) != 0) {
            if (ctx_) { srb_ll_ctx_destroy(ctx_); ctx_ = nullptr; }
            if (srb_ll_ctx_create(&p, max_, device_, &ctx_) != SRB_OK)
                throw std::runtime_error(std::string("srb_ll_ctx_create: ") + srb_last_error());
            params_ = p;
        }
        srb_ll_io io{};
        io.struct_size = sizeof io;          /* ABI check (SRB_ABI_VERSION) */
        io.ind = ind_.data();
        io.q = q_.data(); io.dq = dq_.data(); io.Dinv = Dinv_.data(); io.B = B_.data(); io.H = H_.data();
        io.Jc = Jc_.data(); io.dJc = dJc_.data(); io.Js = Js_.data(); io.Jtoe = Jtoe_.data(); io.Jhip = Jhip_.data();
        io.toePos = toe_.data(); io.hipPos = hip_.data(); io.H0 = H0_.data(); io.dH0 = dH0_.data(); io.y = y_.data();
        io.dy = dy_.data(); io.hd = hd_.data(); io.dhd = dhd_.data(); io.fDes = fDes_.data();
        io.tau = tau_.data(); io.QP_force = F_.data(); io.ddq = ddq_.data(); io.dq_out = dqo_.data();
        io.q_out = qo_.data(); io.V = V_.data(); io.dV = dV_.data(); io.x = x_.data();
        io.status = status_.data(); io.iters = iters_.data();
        if (srb_ll_calc_torque(ctx_, n, &io) != SRB_OK)
            throw std::runtime_error(std::string("srb_ll_calc_torque: ") + srb_last_error());
        for (int a = 0; a < n; a++) unpack(a);
    }

    const LLInfo &ll(int a) const { return ll_.at((size_t)a); }
    double *tau(int a) { return &tau_[(size_t)a * LL_NQ]; }
    const double *qp_solution(int a) const { return &x_[(size_t)a * 32]; }
    int status(int a) const { return status_.at((size_t)a); }
    int iterations(int a) const { return iters_.at((size_t)a); }
    int size() const { return used_; }

private:
    void unpack(int a)
    {
        if ((int)ll_.size() < max_) ll_.resize((size_t)max_);
        LLInfo &o = ll_[(size_t)a];
        const size_t A = (size_t)a;
        int cnt = 0;
        for (int i = 0; i < 4; i++) cnt += (ind_[4 * A + i] == 1);
        /* ll.tau holds the QP torques only (LowLevelCtrl.cpp:49-53); the swing PD goes to tau */
        for (int i = 0; i < 6; i++) o.tau[i] = 0.0;
        for (int i = 0; i < LL_NU; i++) o.tau[6 + i] = x_[A * 32 + 3 * cnt + i];
        std::memcpy(o.QP_force, &F_[A * 12], sizeof o.QP_force);
        std::memcpy(o.q, &qo_[A * LL_NQ], sizeof o.q);
        std::memcpy(o.dq, &dqo_[A * LL_NQ], sizeof o.dq);
        std::memcpy(o.ddq, &ddq_[A * LL_NQ], sizeof o.ddq);
        o.V = V_[A];
        o.dV = dV_[A];
    }

    int max_, device_, used_ = 0;
    srb_ll_ctx *ctx_ = nullptr;
    srb_ll_params params_{};
    std::vector<int> ind_, status_, iters_;
    std::vector<double> q_, dq_, Dinv_, B_, H_, Jc_, dJc_, Js_, Jtoe_, Jhip_, toe_, hip_, H0_, dH0_, y_, dy_, hd_,
        dhd_, fDes_, tau_, F_, ddq_, dqo_, qo_, V_, dV_, x_;
    std::vector<LLInfo> ll_;
};

/* The reference's per-robot class: one LowLevelBatch of one (LowLevelCtrl.hpp:15-27). */
class LowLevelCtrl {
public:
    explicit LowLevelCtrl(int device = 0) : b_(1, device) {}
    template <class State, class Dyn, class Kin, class VC, class Con, class Params>
    void calcTorque(const State *state, const Dyn *dyn, const Kin *kin, const VC *vc, const Con *con, Params *params)
    {
        b_.set(0, state, dyn, kin, vc, con);
        b_.run(params, 1);
        ll_ = b_.ll(0);
    }
    const LLInfo *getllPointer() { return &ll_; }
    double *getTorque() { return b_.tau(0); }
    const double *qp_solution() const { return b_.qp_solution(0); }
    int last_status() const { return b_.status(0); }
    int last_iterations() const { return b_.iterations(0); }

private:
    LowLevelBatch b_;
    LLInfo ll_;
};

}  // namespace srbnmpc

#endif
