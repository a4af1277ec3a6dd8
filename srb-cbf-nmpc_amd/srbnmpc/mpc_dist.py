"""MPCDist -- the reference's per-agent MPC_dist call surface over the batched GPU solver.

Mirrors /root/reference/include/MPC_dist.hpp:137-190 method for method, so a driver
written against MPC_dist (src/A1_Sim.cpp:180-197, driver_scripts/qp_only_exp.cpp:156-188)
reads the same:

    mpc = MPCDist(); mpc.setAgentID(0); mpc.setPstart(Pstart); mpc.setPobs(Pobs)
    mpc.setPobs_real(Pobs_real); mpc.setReferenceTrajectory(Pr, Prd)
    mpc.updateState(q, dq, contactInd, toePos, state_other); mpc.run_NMPC()
    alpha = mpc.get_alphaCOM(); X = mpc.get_MPCsol(); last = mpc.get_lastState()

run_NMPC keeps the reference's host-side planners (copPlanner_eventbase, footholdsPlanner)
and sends the solve (with the fused Bezier fit) to the GPU as a batch of one.

Horizon: the reference hard-codes N = NDOMAIN = 4 grids (MPC_dist.cpp:92, :104).  MPCDist(horizon=N)
generalises it as SURVEY.md 5 asks (BASELINE configs[0]: horizon 10): the window still starts at
column NDOMAIN * gaitDomain_ (a gait domain is NDOMAIN grids) and spans N columns, every grid gets
the domain's footholds, get_MPCsol() is 4N x 1, and the Bezier fit keeps using X_0..X_3 (the
domain); horizon=NDOMAIN (default) is the reference exactly.

generateReferenceTrajectory (the offline HL planner, MPC_dist.cpp:930-1104) runs on the
GPU through srb_hl_plan; callers that already hold its output use setReferenceTrajectory.
"""
from __future__ import annotations

import numpy as np

NDOMAIN = 4
INIT_FOOTPRINT = np.array([[0.2188, -0.1320],   # FR   (MPC_dist.cpp:1206-1209)
                           [0.2188, 0.1320],    # FL
                           [-0.1472, -0.1320],  # RR
                           [-0.1472, 0.1320]])  # RL


class MPCDist:
    _solvers = {}

    def __init__(self, device: int = 0, horizon: int = NDOMAIN):
        if horizon < NDOMAIN:
            raise ValueError(f"horizon {horizon} < NDOMAIN = {NDOMAIN} (the Bezier fit reads X_0..X_3)")
        self.use_snopt = False            # MPC_dist.hpp:139: False -> QP only
        self.device = device
        self.N = int(horizon)
        self.agent_id_ = 0
        self.gaitDomain_ = 0
        self.domain_ = 0
        self.distance_to_fail = 10.0      # MPC_dist.cpp:51
        self.isSuccess = True
        self.Pstart_ = None
        self.Pobs = np.zeros((2, 0))
        self.Pobs_real = np.zeros((2, 0))
        self.Pr_refined_ = None
        self.Prd_refined_ = None
        self.agent_Initial_ = np.zeros(2)
        self.mpc_state_alpha_buffer_ = np.zeros(4)
        self.q = np.zeros(18); self.dq = np.zeros(18)
        self.contactInd = np.ones(4, dtype=np.int32)
        self.toePos_ = np.zeros((3, 4))
        self.state_other = np.zeros(4)
        self.alpha_COM_traj_e_ = np.zeros((4, 5))
        self.mpc_state_e_x_eventbased_ = np.zeros(4 * self.N)
        self.qp_solution_eventbased_ = None
        self.last_status = None
        self.last_iters = None

    # ------------------------------------------------------------------ setters
    def setAgentID(self, agent_id: int):
        self.agent_id_ = int(agent_id)

    def setPstart(self, Pstart):
        self.Pstart_ = np.asarray(Pstart, dtype=np.float64).ravel()
        self.agent_Initial_ = self.Pstart_[2 * self.agent_id_:2 * self.agent_id_ + 2].copy()
        self.mpc_state_alpha_buffer_ = np.array([self.agent_Initial_[0], 0.0, self.agent_Initial_[1], 0.0])

    def setPobs(self, Pobs):
        self.Pobs = np.asarray(Pobs, dtype=np.float64).reshape(2, -1)

    def setPobs_real(self, Pobs):
        self.Pobs_real = np.asarray(Pobs, dtype=np.float64).reshape(2, -1)

    def setReferenceTrajectory(self, Pr, Prd):
        """Output of generateReferenceTrajectory (Pr_refined_, Prd_refined_: 2*NA x T)."""
        self.Pr_refined_ = np.asarray(Pr, dtype=np.float64)
        self.Prd_refined_ = np.asarray(Prd, dtype=np.float64)

    def generateReferenceTrajectory(self, loop: int = 100000):
        """MPC_dist.cpp:930-1104 on the device (srb_hl_plan): all agents from Pstart_ around
        the planner obstacles Pobs (2 x n_obs); fills Pr_refined_ / Prd_refined_ (2NA x loop/40)."""
        if self.Pstart_ is None:
            raise RuntimeError("MPC_dist: setPstart() not called")
        from . import hl_plan
        self.Pr_refined_, self.Prd_refined_ = hl_plan(self.Pstart_.reshape(-1, 2), self.Pobs.T, loop,
                                                      self.device)

    def updateState(self, q, dq, ind, toePos, state_other):
        self.q = np.asarray(q, dtype=np.float64).ravel()[:18].copy()
        self.dq = np.asarray(dq, dtype=np.float64).ravel()[:18].copy()
        self.contactInd = np.asarray(ind, dtype=np.int32).ravel()[:4].copy()
        self.toePos_ = np.asarray(toePos, dtype=np.float64).reshape(3, 4).copy()
        self.state_other = np.asarray(state_other, dtype=np.float64).ravel()[:4].copy()

    # ------------------------------------------------------------------ planners (host)
    def copPlanner_eventbase(self, N: int | None = None):
        """MPC_dist.cpp:702-782: 4 x N window of the HL path from column NDOMAIN * gaitDomain_,
        flattened column-major (N = the horizon)."""
        N = self.N if N is None else N
        a = self.agent_id_
        c0 = NDOMAIN * self.gaitDomain_
        if c0 + N > self.Pr_refined_.shape[1]:
            raise RuntimeError("MPC_dist: reference trajectory exhausted")
        qref = np.zeros((4, N))
        qref[0] = self.Pr_refined_[2 * a, c0:c0 + N]
        qref[1] = self.Prd_refined_[2 * a, c0:c0 + N]
        qref[2] = self.Pr_refined_[2 * a + 1, c0:c0 + N]
        qref[3] = self.Prd_refined_[2 * a + 1, c0:c0 + N]
        return qref.T.reshape(-1)

    def footholdsPlanner(self):
        """MPC_dist.cpp:1204-1266: stance footholds (2 x C) in FR,FL,RR,RL order."""
        if self.gaitDomain_ <= 1:
            self.toePos_ = np.zeros((3, 4))
            self.toePos_[0] = INIT_FOOTPRINT[:, 0] + self.agent_Initial_[0]
            self.toePos_[1] = INIT_FOOTPRINT[:, 1] + self.agent_Initial_[1]
        ci = self.contactInd
        C = int(ci.sum())
        if C == 4:
            legs = [0, 1, 2, 3]
        elif C == 2 and ci[0] == 0:
            legs = [1, 2]
        elif C == 2 and ci[0] == 1:
            legs = [0, 3]
        else:
            raise ValueError(f"unsupported contact pattern {ci.tolist()}")
        return self.toePos_[:2, legs].copy()

    # ------------------------------------------------------------------ solve
    def _solver(self, C: int, use_nlp: bool):
        from . import BatchSolver, default_params
        key = (self.device, self.N, C, use_nlp)
        if key not in MPCDist._solvers:
            p = default_params(self.N, C, K_obs=1, K_nbr=0, use_nlp=int(use_nlp))
            MPCDist._solvers[key] = BatchSolver(p, 1, self.device)
            # the per-agent surface keeps the reference's QP solution (qp_solution_eventbased_, iSWIFT's
            # tolerance): the QP stage is not shortened here (SRB_OPT_QP_WARM_TOL = 0)
            MPCDist._solvers[key].set_option("qp_warm_tol", 0.0)
        return MPCDist._solvers[key]

    def run_NMPC(self):
        """MPC_dist.cpp:81-454 with the QP/NLP solve on the GPU."""
        N = self.N
        ref = self.copPlanner_eventbase(N)
        F = self.footholdsPlanner()
        C = F.shape[1]
        foot = np.repeat(F[None], N, 0)             # same block on every grid (:1256-1260)
        x0 = np.array([self.q[0], self.dq[0], self.q[1], self.dq[1]])
        solver = self._solver(C, bool(self.use_snopt))
        # the solve and fitComTrajectory_eventbase (:784-855, fused epilogue) in one call
        out = solver.solve(x0[None], ref[None], foot[None], self.Pobs_real.T.copy(),
                           alpha_buf=self.mpc_state_alpha_buffer_[None])
        x = out["x"][0]
        self.qp_solution_eventbased_ = out["x_qp"][0]
        self.mpc_state_e_x_eventbased_ = x[:4 * N].copy()
        self.last_status = out["status"][0]
        self.last_iters = out["iters"][0]
        X = self.mpc_state_e_x_eventbased_.reshape(N, 4)
        self.alpha_COM_traj_e_ = out["alpha"][0]
        self.mpc_state_alpha_buffer_ = X[NDOMAIN - 1].copy()    # buffer update (:798): the domain's end
        self.gaitDomain_ += 1
        return x

    # ------------------------------------------------------------------ getters
    def get_alphaCOM(self):
        return self.alpha_COM_traj_e_

    def get_MPCsol(self):
        return self.mpc_state_e_x_eventbased_.reshape(-1, 1)

    def getDomain(self):
        return self.domain_

    def get_lastState(self):
        """MPC_dist.cpp:1272-1276: measured (not predicted) [x, y, xdot, ydot]."""
        return np.array([self.q[0], self.q[1], self.dq[0], self.dq[1]])

    def updateDistance_to_fail(self):
        """MPC_dist.cpp:21-40."""
        if self.isSuccess:
            p = self.q[:2]
            for i in range(self.Pobs_real.shape[1]):
                if np.hypot(*(p - self.Pobs_real[:, i])) < 0.5:
                    self.isSuccess = False
                    self.distance_to_fail = float(np.hypot(*p))
                    break

    def getDistance_to_fail(self):
        return self.distance_to_fail
