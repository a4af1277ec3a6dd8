/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp64) of the reference's per-control-cycle NMPC path
 *   MPC_dist::run_NMPC            /root/reference/src/MPC_dist.cpp:81-454
 *   iSWIFT QP_SETUP/QP_SOLVE      /root/reference/optimization/iSWIFT/src/Prime.c:35-230
 *   NLP rows (obstacle/velocity)  /root/reference/include/dec_vars_constr_cost.h:245-395
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker.  The product (srb-cbf-nmpc_amd/csrc) never links it.
 *
 * Linear algebra is deliberately FULL-SPACE and dense (Schur complement on the
 * unreduced KKT for the QP stage, LU on [H A'; A 0] for the NLP stage) so that it
 * shares no code path with the GPU kernel's condensed (null-space) linear algebra.
 *
 * Parity pins:
 *   - QP stage == genuine vendored iSWIFT (oracle/_ref) -- same iteration count and
 *     x to ~1e-10 under a quasi-definite elimination order;
 *   - reconstructed print_file.out instance reproduces the reference's logged QP
 *     output (SNOPT start point) to 5e-10;
 *   - NLP stage (SNOPT in the reference; not vendored): KKT certificate + SciPy.
 */
#ifndef SRB_ORACLE_H
#define SRB_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_params {
    int N;          /* grid points in the horizon (reference: 4, MPC_dist.cpp:92)            */
    int C;          /* stance contacts per grid (trot 2, stand 4; MPC_dist.cpp:132)          */
    int K_obs;      /* nearest static obstacles per agent (reference: 1, MPC_dist.cpp:371-396) */
    int K_nbr;      /* nearest neighbour agents used as moving obstacles (reference: 0)       */
    double grav, hcom, Ts, mu;          /* 9.81, 0.29, 0.043, 0.7  (MPC_dist.cpp:90-104)      */
    double Qw, Pw, Rw, Sw;              /* 300, 2000, 0.1, 3000    (MPC_dist.cpp:168-178)     */
    double box;                         /* 1e3                     (MPC_dist.cpp:317-318)     */
    double eps_obs, eps_nbr;            /* (double)1.9f, (double)2.2f (dec_vars_constr_cost.h:401-402) */
    double vsat;                        /* (double)0.35f           (dec_vars_constr_cost.h:306) */
    double tol;                         /* 1e-6                    (GlobalOptions.h:24-25)    */
    int qp_maxit, nlp_maxit;            /* 25 (GlobalOptions.h:23), 50                        */
    int use_nlp;                        /* MPC_dist::use_snopt                                */
    int qp_init;                        /* QP starting point: 1 scaled (the kernel's default), 0 iSWIFT's kkt_initialize */
    double tol_qp;                      /* the QP stage's tolerance when the NLP follows (the kernel's SRB_OPT_QP_WARM_TOL,
                                           default 0.3; 0: tol) */
    int polish;                         /* 1: active-set polish of the NLP result (the kernel's SRB_OPT_POLISH, default 1) */
} orc_params;

void orc_params_default(orc_params *p, int N, int C);

/* sizes */
int orc_nv(const orc_params *p);      /* (6+C)N+1                 */
int orc_neq(const orc_params *p);     /* 7N                       */
int orc_mqp(const orc_params *p);     /* 4(N-1)+12N+2CN           */
int orc_mnlp(const orc_params *p);    /* mqp + 4N + N*(K_obs+K_nbr) */

/* LIP discretisation, MPC_dist.cpp:99-127.  Ad row-major 4x4, Bd row-major 4x2. */
void orc_lip(const orc_params *p, double Ad[16], double Bd[8]);

/*
 * Dense QP assembly exactly as MPC_dist.cpp:135-321, generalised to N grids and
 * per-grid footholds foot[N][2][C] (the reference repeats one block, :1256-1260).
 * Outputs (caller-allocated, row-major):
 *   Pd[nv] (diagonal of Q_qp), c[nv], A[neq*nv], b[neq], G[mqp*nv], h[mqp]
 */
void orc_build_qp(const orc_params *p, const double x0[4], const double *ref, const double *foot,
                  double *Pd, double *c, double *A, double *b, double *G, double *h);

/*
 * Per-grid obstacle list for the NLP rows (dec_vars_constr_cost.h:262-265 generalised):
 * K_obs nearest static obstacles by current CoM position (MPC_dist.cpp:371-396; the
 * strict '<' keeps the first index on ties) followed by K_nbr nearest other agents,
 * each predicted at constant velocity to grid k: o_k = p + v*Ts*(k+1)
 * (the intent of the commented line MPC_dist.cpp:391).
 * obs_out[N][K][2], eps_out[K]; missing entries are parked far away (1e6).
 */
void orc_select_idx(const orc_params *p, const double x0[4], const double *obstacles, int n_obs,
                    const double *nbr_state, int n_all, int self_idx, int *idx);
void orc_select_obstacles(const orc_params *p, const double x0[4],
                          const double *obstacles, int n_obs,
                          const double *nbr_state, int n_all, int self_idx,
                          double *obs_out, double *eps_out);

/* iSWIFT algorithm restated (Prime.c:127-230, Auxilary.c); returns 0..3 exit code. */
/* the NMPC's divergence rule (both stages): a dual beyond this ends the solve FATAL at its finite
 * iterate (infeasible rows; converging solves keep their duals below ~1e4) -- srb_kernels.hip,
 * srb12_kernels.hip and oracle/srb12.c apply the same threshold */
#define ORC_Z_DIV 1e10
/* qp_init: 0 = iSWIFT's kkt_initialize (Auxilary.c:680-755), 1 = scaled start (qp_ipm.c) */
int orc_qp_solve_init(int n, int m, int p, const double *Pd, const double *c, const double *A, const double *b,
                      const double *G, const double *h, int maxit, double tol, int qp_init, double *x_out, double *q_out,
                      int *iters_out);
int orc_qp_solve(int n, int m, int p, const double *Pd, const double *c,
                 const double *A, const double *b, const double *G, const double *h,
                 int maxit, double tol, double *x_out, double *q_out, int *iters_out);

int orc_qp_solve_full(int n, int m, int p, const double *P, const double *c,
                      const double *A, const double *b, const double *G, const double *h,
                      int maxit, double tol, double *x_out, int *iters_out);

/* NLP stage (replaces SnoptSolver::Solve, MPC_dist.cpp:402-427). */
int orc_nlp_solve(const orc_params *p, const double x0[4], const double *foot,
                  const double *Pd, const double *c, const double *A, const double *b,
                  const double *G, const double *h,
                  const double *obs, const double *eps,
                  const double *x_init, double *x_out, int *iters_out);

/* One agent end-to-end (run_NMPC minus planners): QP stage then (use_nlp) NLP stage. */
int orc_solve_agent(const orc_params *p, const double x0[4], const double *ref, const double *foot,
                    const double *obstacles, int n_obs, const double *nbr_state, int n_all, int self_idx,
                    double *x_qp, double *x_out, double *obj, int status[2], int iters[2]);

/* Agent batch on `nthreads` host threads (CPU baseline in bench.py). */
int orc_solve_batch(const orc_params *p, int n_agents, const double *x0, const double *ref,
                    const double *foot, const double *obstacles, int n_obs,
                    const double *nbr_state, int n_all, int agent_offset,
                    double *x_qp, double *x_out, double *obj, int *status, int *iters, int nthreads);

/* fitComTrajectory_eventbase restated (MPC_dist.cpp:784-855): alpha[4][5] (row-major)
 * from the buffer state (4) and the first 4 predicted states X[0..3]. */
void orc_fit_bezier(const double buf[4], const double *X, double alpha[20]);

/* HL reference planner (generateReferenceTrajectory, MPC_dist.cpp:930-1104) for NA agents,
 * n_obs planner obstacles Pobs [n_obs][2], `loop` steps (reference: 100000).  Pr, Prd:
 * column-major 2NA x (loop / 40). */
void orc_hl_plan(int NA, const double *Pstart, const double *Pobs, int n_obs, int loop, double *Pr, double *Prd);

/* iSWIFT without the rounding-only sigma <= sigma_d branch (see qp_ipm.c), and iSWIFT
 * semantics reporting whether that branch was taken */
int orc_qp_solve_nt(int n, int m, int p, const double *Pd, const double *c, const double *A, const double *b,
                    const double *G, const double *h, int maxit, double tol, double *x_out, int *iters_out);
int orc_qp_solve_trap(int n, int m, int p, const double *Pd, const double *c, const double *A, const double *b,
                      const double *G, const double *h, int maxit, double tol, double *x_out, int *iters_out,
                      int *trapped);

/* ---- low-level CLF-QP controller (ll_ctrl.c; LowLevelCtrl::calcTorque, LowLevelCtrl.cpp:18-113) */
typedef struct orc_ll_params {
    double mu, kp, kd;                  /* Settings::LL_params (global_loco_structs.hpp:96-111) */
    int useCLF;
    double tauPen, dfPen, auxPen, clfPen, auxMax, clfEps;
    int maxit;                          /* iSWIFT MAXIT 25, tolerance 1e-6 (GlobalOptions.h:23-25) */
    double tol;
    int iswift_trap;                    /* 1: keep iSWIFT's sigma <= sigma_d branch (default 0, as the kernel) */
} orc_ll_params;

/* one agent's inputs; column-major matrices with the leading dimensions of srb_ll_io */
typedef struct orc_ll_agent {
    int ind[4];
    const double *q, *dq, *Dinv, *B, *Hv, *Jc, *dJc, *Js, *Jtoe, *Jhip, *toePos, *hipPos;
    const double *H0, *dH0, *y, *dy, *hd, *dhd, *fDes;
} orc_ll_agent;

typedef struct orc_ll_out {
    double tau[18];        /* in/out (the reference's member array, tau[0..5] accumulate) */
    double QP_force[12], ddq[18], dq[18], q[18], V, dV, x[32];
    int status, iters;
} orc_ll_out;

void orc_ll_params_default(orc_ll_params *p);
/* dense QP of LowLevelCtrl::cost/constraints (row-major A, G); clf = {V, Veps, LfV} */
int orc_ll_build_qp(const orc_ll_params *prm, const orc_ll_agent *in,
                    int *n_out, int *p_out, int *m_out, double *Pd, double *c, double *A, double *b,
                    double *G, double *h, double clf[3], double *LgV);
int orc_ll_calc_torque(const orc_ll_params *prm, const orc_ll_agent *in, orc_ll_out *out);
int orc_ll_calc_torque_batch(const orc_ll_params *prm, int n_agents, const int *ind, const double *q, const double *dq,
                             const double *Dinv, const double *B, const double *Hv, const double *Jc, const double *dJc,
                             const double *Js, const double *Jtoe, const double *Jhip, const double *toePos,
                             const double *hipPos, const double *H0, const double *dH0, const double *y,
                             const double *dy, const double *hd, const double *dhd, const double *fDes, double *tau,
                             double *QP_force, double *ddq, double *dq_out, double *q_out, double *V, double *dV,
                             double *x, int *status, int *iters);

int orc_ll_calc_torque_batch_mt(const orc_ll_params *prm, int nthreads, int n_agents, const int *ind, const double *q,
                                const double *dq, const double *Dinv, const double *B, const double *Hv,
                                const double *Jc, const double *dJc, const double *Js, const double *Jtoe,
                                const double *Jhip, const double *toePos, const double *hipPos, const double *H0,
                                const double *dH0, const double *y, const double *dy, const double *hd,
                                const double *dhd, const double *fDes, double *tau, double *QP_force, double *ddq,
                                double *dq_out, double *q_out, double *V, double *dV, double *x, int *status,
                                int *iters);

/* ---- SRB-12 extension mode (srb12.c; the north star's 12-state SRB model, declared but never
 * implemented by the reference, include/fast_MPC.hpp:98-103: parity unpinned) */
typedef struct orc12_params {
    int N, K_obs, K_nbr;
    double Ts, mass, Ib[9], grav, mu, fmax;
    double q[12], qN[12], r[3], Sw;     /* stage / terminal state weights, force weights, slack weight */
    double eps_obs, eps_nbr, tol;
    int qp_maxit, nlp_maxit, use_nlp;
    double z0;                          /* NLP initial duals z0 / max(s, 1) */
    double tol_final;                   /* complementarity tolerance of the last stage (srb12_params) */
    int polish;                         /* 1: active-set polish of the last stage's result */
    double tol_qp;                      /* the QP stage's tolerance when the NLP follows (srb12_params) */
} orc12_params;

void orc12_params_default(orc12_params *p, int N);
int orc12_nv(const orc12_params *p);
extern int orc12_polish_stats[4];      /* polishes rejected, accepted, Newton steps, most steps of one solve */   /* 24N + 1: X (12N) | U (12N) | s */
void orc12_dynamics(const orc12_params *p, const double x0[12], const double *xref, const double *foot,
                    const int *contact, double *A, double *B, double *c);
int orc12_solve_agent(const orc12_params *p, const double x0[12], const double *xref, const double *foot,
                      const int *contact, const double *obstacles, int n_obs, const double *nbr_state, int n_all,
                      int self_idx, double *x_qp, double *x_out, double *obj, int status[2], int iters[2]);
int orc12_solve_batch(const orc12_params *p, int n_agents, const double *x0, const double *xref, const double *foot,
                      const int *contact, const double *obstacles, int n_obs, const double *nbr_state, int n_all,
                      int agent_offset, double *x_qp, double *x_out, double *obj, int *status, int *iters, int nthreads);

/* dense helpers (linalg.c) */
int orc_chol(int n, double *A);                               /* in place, lower */
void orc_chol_solve(int n, const double *L, double *x);
int orc_lu(int n, double *A, int *piv);
void orc_lu_solve(int n, const double *LU, const int *piv, double *x);

#ifdef __cplusplus
}
#endif
#endif
