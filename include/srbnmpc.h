/*
 * srbnmpc -- batched CBF-NMPC solver for AMD Instinct MI355X (gfx950).  C ABI.
 *
 * Drop-in replacement for the per-control-cycle solve of the HDSRL/SRB-CBF-NMPC
 * reference (MPC_dist::run_NMPC, /root/reference/src/MPC_dist.cpp:81-454):
 *   - the QP stage iswiftQp_e(Q_qp, f_qp, Aeq, beq, Gineq, hineq, sol)
 *       (/root/reference/optimization/iSWIFT/cpp_wrapper/iswift_qp.h:14-16, called at
 *        MPC_dist.cpp:348), and
 *   - the NLP stage nlp.AddVariableSet/AddConstraintSet/AddCostSet + SnoptSolver::Solve
 *       (MPC_dist.cpp:402-427 with include/dec_vars_constr_cost.h),
 * for a whole batch of agents per call.  Problem assembly (MPC_dist.cpp:99-321) and the
 * closest-obstacle scan (:371-396) happen on the device from the per-agent inputs below.
 *
 * Conventions: plain C, fp64, agent-major arrays, caller-owned buffers, int status
 * codes (0 = success; negative = API error), no exceptions across the ABI.  Solver exit
 * codes mirror iSWIFT's (GlobalOptions.h:31-34): 0 OPTIMAL, 1 KKTFAIL, 2 MAXIT, 3 FATAL.
 * As in the reference (iswift_qp.cpp:126-151, MPC_dist.cpp:421), a non-optimal exit
 * still returns the last iterate.
 *
 * Decision vector of one agent (the reference's mpc_state_eventbased_, MPC_dist.cpp:345):
 *   x = [ X (4N: x, xdot, y, ydot per grid) | U (2N: CoP) | lambda (C*N) | s ]
 *   nv = (6 + C) * N + 1
 */
#ifndef SRBNMPC_H
#define SRBNMPC_H

#ifdef __cplusplus
extern "C" {
#endif

#define SRB_OK 0
#define SRB_ERR_ARG (-1)
#define SRB_ERR_HIP (-2)
#define SRB_ERR_SIZE (-3)

/*
 * ABI versioning.  Every I/O struct (srb_batch, srb_prep, srb_ll_io) starts with
 * `int struct_size`, which the caller sets to sizeof(struct) of the header it was compiled
 * against; the library rejects any other value with SRB_ERR_ARG (srb_last_error() names
 * the struct), so a caller built against an older or newer layout fails loudly instead of
 * having trailing fields read from whatever follows its struct.  srb_abi_version() returns
 * the SRB_ABI_VERSION the library was built with (bumped on any layout change).
 *   srb_batch b = {sizeof(srb_batch)};      (C)      srb_batch b{}; b.struct_size = sizeof b;  (C++)
 */
#define SRB_ABI_VERSION 5
int srb_abi_version(void);

/* solver exit codes (iSWIFT GlobalOptions.h:31-34) */
#define SRB_OPTIMAL 0
#define SRB_KKTFAIL 1
#define SRB_MAXIT 2
#define SRB_FATAL 3

typedef struct srb_params {
    int N;              /* grid points in the horizon (reference: 4, MPC_dist.cpp:92)               */
    int C;              /* stance contacts per grid (trot 2, stand 4; MPC_dist.cpp:132)             */
    int K_obs;          /* nearest static obstacles per agent (reference: 1, MPC_dist.cpp:371-396)  */
    int K_nbr;          /* nearest other agents used as moving obstacles (reference: 0)             */
    double grav, hcom, Ts, mu;       /* 9.81, 0.29, 0.043, 0.7 (MPC_dist.cpp:90-104)                */
    double Qw, Pw, Rw, Sw;           /* 300, 2000, 0.1, 3000 (MPC_dist.cpp:172-175)                 */
    double box;                      /* 1e3 (MPC_dist.cpp:317-318)                                  */
    double eps_obs, eps_nbr;         /* (double)1.9f, (double)2.2f (dec_vars_constr_cost.h:401-402) */
    double vsat;                     /* (double)0.35f (dec_vars_constr_cost.h:306-307)              */
    double tol;                      /* 1e-6 (GlobalOptions.h:24-25)                                */
    int qp_maxit, nlp_maxit;         /* 25 (GlobalOptions.h:23), 50                                 */
    int use_nlp;                     /* MPC_dist::use_snopt (MPC_dist.hpp:139): 0 = QP only         */
} srb_params;

/* Reference defaults for horizon N and C contacts (K_obs = 1, K_nbr = 0, use_nlp = 1). */
void srb_params_default(srb_params *p, int N, int C);
int srb_nv(const srb_params *p);     /* (6+C)N+1 */

/*
 * One batch.  All pointers agent-major, fp64 unless noted.
 *   x0        [A][4]        x, xdot, y, ydot             (MPC_dist.cpp:226-229; q[0],dq[0],q[1],dq[1])
 *   ref       [A][4N]       com_desired_Traj_vec         (copPlanner_eventbase, MPC_dist.cpp:780)
 *   foot      [A][N][2][C]  stance footholds per grid: row 0 = x, row 1 = y of the C
 *                           contact legs in FR,FL,RR,RL order (footholdsPlanner, :1238-1260)
 *   obstacles [n_obs][2]    Pobs_real columns, shared by the batch (MPC_dist.hpp:85)
 *   nbr_state [n_all][4]    get_lastState() of every agent: x, y, xdot, ydot (MPC_dist.cpp:1272-1276);
 *                           may be NULL when K_nbr == 0.  Local agent a is global agent
 *                           agent_offset + a (itself excluded from its neighbours).
 * Outputs:
 *   x_qp      [A][nv]       QP-stage solution (qp_solution_eventbased_, :350-354); may be NULL.  With the NLP
 *                           stage on it is the NLP's warm start, solved to SRB_OPT_QP_WARM_TOL (default 0.3,
 *                           status 4 below), not to iSWIFT's 1e-6 -- set that option to 0 for the reference's
 *                           point (the MPC_dist shims do); srb_solve_qp always solves to 1e-6
 *   x         [A][nv]       final decision vector (mpc_state_eventbased_ after :423-426)
 *   obj       [A]           0.5 x'Q_qp x + f'x (ExCost::GetCost)
 *   status    [A][2] int    QP, NLP exit codes: 0 OPTIMAL, 1 KKTFAIL, 2 MAXIT, 3 FATAL (iSWIFT's);
 *                           QP also 4 QP_WARM: converged at the warm-start tolerance only (the NLP follows);
 *                           NLP also 4 ACCEPTABLE: stopped at a near-optimal iterate (primal and
 *                           complementarity met, dual residual within 100x of its threshold)
 *                           whose next step was blocked or needed an inertia shift, or met only
 *                           the loosened exit tests the polish relies on and was not polished
 *                           (rejected, or SRB_OPT_POLISH = 0); 3 FATAL also when a dual passes 1e10
 *                           (infeasible rows) -- the iterate returned is finite in every case
 *   iters     [A][2] int    QP, NLP interior-point iterations
 * Bezier fit of the predicted CoM (fitComTrajectory_eventbase, MPC_dist.cpp:784-855), fused
 * into the solve; both NULL = not fitted (needs N >= 4):
 *   alpha_buf [A][4]        mpc_state_alpha_buffer_ (the previous solve's X_3; the start
 *                           position with zero velocity before the first one, :792, :798)
 *   alpha     [A][20]       get_alphaCOM(): 4 x 5 row-major (state row, Bernstein index)
 * Selected obstacle rows (the closest-obstacle scan, MPC_dist.cpp:371-382), optional:
 *   sel       [A][Ko + Kn] int  out: the Ko = min(K_obs, n_obs) static obstacle indices, then the
 *                           Kn = min(K_nbr, n_all - 1) neighbour rows (global indices into
 *                           nbr_state; -1 = none), in the reference's scan order (sqrt distance,
 *                           lower index on ties; a static round with nothing closer than 1000 m
 *                           selects obstacle 0, as min_dist = 1000 / min_i = 0 do).  NULL = the
 *                           context's own scratch buffer.
 */
typedef struct srb_batch {
    int struct_size;         /* sizeof(srb_batch) (ABI check, see SRB_ABI_VERSION) */
    const double *x0, *ref, *foot, *obstacles, *nbr_state;
    int n_obs, n_all, agent_offset;
    double *x_qp, *x, *obj;
    int *status, *iters;
    const double *alpha_buf;
    double *alpha;
    int *sel;
    int obstacles_version;   /* != 0: the obstacle table is unchanged since the last call that passed
                                this version, pointer and n_obs (the reference's Pobs_real is set once,
                                MPC_dist::setPobs_real): its selection grid is reused; 0: rebuilt */
} srb_batch;

typedef struct srb_ctx srb_ctx;

/* Create a context on HIP device `device` for batches of up to max_agents agents. */
int srb_ctx_create(const srb_params *p, int max_agents, int device, srb_ctx **out);
int srb_ctx_destroy(srb_ctx *ctx);

/* Waves (64-lane wavefronts) per agent's workgroup: 0 = automatic (4 while the batch has no
 * more agents than the device has CUs, else 1, or 2 for problems whose row slots exceed five
 * per lane), or force 1, 2 or 4.  Results are bit-identical for a given wave count; different
 * counts sum the reduced Newton matrix in a different order (round-off differences only).
 * srb_ctx_waves() returns the count the last launch used. */
int srb_ctx_set_waves(srb_ctx *ctx, int nw);
int srb_ctx_waves(srb_ctx *ctx);

/* Context options (no environment variable changes what the library computes; every knob is one
 * of these, per context).  set returns SRB_ERR_ARG for an unknown option or a value out of range.
 *   SRB_OPT_POLISH               1 (default) polish the NLP result to the exact KKT point of its active
 *                                set, 0 off: results that met only the loosened NLP exit
 *                                tests then stay ACCEPTABLE (4)
 *   SRB_OPT_POLISH_RHO           the polish's regularisation 1 / rho (default 1e9; 1e3 .. 1e12)
 *   SRB_OPT_POLISH_WAVES         waves per agent of the polish kernel: 0 automatic (default), 1, 2, 4
 *   SRB_OPT_GRID_MIN_ROWS        tables of this many rows or more get a selection grid (default 8192)
 *   SRB_OPT_GRID_MIN_ROWS_STATIC the same for a versioned static obstacle table (default 4096)
 *   SRB_OPT_POLISH_FUSED         1 (default) the polish runs at the end of the solve kernel (problems with
 *                                N(C-1)+1 <= 16), 0 as a kernel of its own after it; the same results
 *   SRB_OPT_LAST_POLISH          read only: how the last launch polished, 0 not at all, 1 polish kernel,
 *                                2 fused into the solve kernel
 *   SRB_OPT_TIMING               1 (default): HIP events around the launch's kernels (srb_last_kernel_ms,
 *                                srb_last_polish_ms); 0: none (each event record is a marker the queue
 *                                drains to: a few us per call, measured in bench.py's timed loop)
 *   SRB_OPT_QP_WARM_TOL          the QP stage's tolerance when the NLP stage follows (default 0.3; 0: the
 *                                full tolerance, 1e-6 as iSWIFT): that point only warm-starts the NLP, whose
 *                                result is unchanged (the polish makes it exact; statuses and NLP iterations
 *                                unchanged on the bench batches) while the QP stage takes 3.0 instead of 5.8
 *                                iterations at configs[2]; x_qp is then that rougher point.  The
 *                                QP-only solve (srb_solve_qp, use_nlp = 0) always runs to the full tolerance.
 *                                Such a QP stage reports status 4 (QP_WARM: converged at this tolerance), never
 *                                0; with 0 here it reports iSWIFT's codes (0 OPTIMAL at 1e-6)
 *   SRB_OPT_SELECTION            1 (default): srb_solve_batch_device runs the obstacle / neighbour selection
 *                                itself; 0: the caller has filled batch.sel with srb_select_device (the two
 *                                tables may then be selected on either side of the neighbour all-gather)
 *   SRB_OPT_KKT_FP32_MU          0 (default): the reduced Newton matrix is inverted in fp64.  > 0: BASELINE
 *                                configs[4]'s "fp32 KKT with fp64 iterative-refine residuals" -- where the
 *                                instance has an fp32-factor variant (the configs[2] and config-5 shapes), the
 *                                matrix (assembled in fp64) is inverted in fp32 while the complementarity mu is
 *                                above this value, each solve then refined SRB_OPT_KKT_FP32_REFINE times (default
 *                                3) against the fp64 matrix; fp64 below it
 *   SRB_OPT_LAST_KKT_FP32        read only: 1 if the last launch ran an fp32-factor instance */
#define SRB_OPT_POLISH 1
#define SRB_OPT_POLISH_RHO 2
#define SRB_OPT_POLISH_WAVES 3
#define SRB_OPT_GRID_MIN_ROWS 4
#define SRB_OPT_GRID_MIN_ROWS_STATIC 5
#define SRB_OPT_POLISH_FUSED 6
#define SRB_OPT_LAST_POLISH 7
#define SRB_OPT_TIMING 8
#define SRB_OPT_QP_WARM_TOL 9
#define SRB_OPT_SELECTION 10
#define SRB_OPT_KKT_FP32_MU 11
#define SRB_OPT_KKT_FP32_REFINE 12
#define SRB_OPT_LAST_KKT_FP32 13
int srb_ctx_set_option(srb_ctx *ctx, int opt, double value);
int srb_ctx_get_option(srb_ctx *ctx, int opt, double *value);

/* QP-stage starting point: 1 (default) the scaled start s = max(h - Gx, 0.1), z = 1/s from the
 * least-squares x of iSWIFT's kkt_initialize (Auxilary.c:680-755); 0 iSWIFT's own shifted start
 * (z + 1 + max(h - Gx): ~1e3 with the +-1e3 boxes of MPC_dist.cpp:317-318), which follows the
 * genuine iSWIFT step for step (tests/test_gpu_parity.py) but needs up to twice the iterations on
 * the slowest agents.  Both end at the QP optimum to the solver tolerance. */
int srb_ctx_set_qp_init(srb_ctx *ctx, int mode);

/* Host buffers: copies in, solves, copies out, synchronises.  n_agents <= max_agents. */
int srb_solve_batch(srb_ctx *ctx, int n_agents, const srb_batch *host_io);

/* Same as srb_solve_batch with use_nlp forced to 0 (reference use_snopt == false). */
int srb_solve_qp(srb_ctx *ctx, int n_agents, const srb_batch *host_io);

/* Device buffers (all pointers in `dev_io` are device pointers), asynchronous on
 * `stream` (a hipStream_t; NULL = the HIP null stream, which orders against every blocking
 * stream, as the CUDA/HIP convention has it).  Pass the stream that produced the inputs (the
 * Python layer passes torch's current stream, whose default is that null stream).  Call
 * srb_sync() or synchronise the stream.
 *
 * Ordering.  A context executes its calls in submission order, whatever stream each call
 * names: a launch on a stream other than the previous call's first waits (hipStreamWaitEvent)
 * for that call's work, and the host entry points (srb_solve_batch / srb_solve_qp) order
 * after the last device launch the same way.  The context's scratch -- the selection grids
 * and their static-table cache, the default `sel` buffer, the staging buffers and the timing
 * events -- is therefore never used by two launches in flight.  For solves that run
 * concurrently, use one context per stream. */
int srb_solve_batch_device(srb_ctx *ctx, int n_agents, const srb_batch *dev_io, void *stream);

/* The selection alone (MPC_dist.cpp:371-396 generalised to K), asynchronous on `stream`: tables = 1 the static
 * obstacles (columns 0 .. Ko-1 of dev_io->sel), 2 the neighbour snapshot (columns Ko .. Ko+Kn-1), 3 both.
 * dev_io->sel is required; the other members are read as srb_solve_batch_device reads them.  Multi-GPU use
 * (bench.py): select the static obstacles while the neighbour all-gather is in flight, the neighbours after
 * it, then solve with SRB_OPT_SELECTION = 0.  Indices are identical to the solve's own selection. */
int srb_select_device(srb_ctx *ctx, int n_agents, const srb_batch *dev_io, int tables, void *stream);
int srb_sync(srb_ctx *ctx);

/*
 * Input assembly on the device (the planners run_NMPC calls before its solve; SURVEY.md 8(f)
 * row 2), one batch of agents, asynchronous on `stream` like srb_solve_batch_device:
 *   updateState + x0 (MPC_dist.cpp:1195-1202, :226-229), get_lastState (:1272-1276),
 *   copPlanner_eventbase (:702-782) and footholdsPlanner (:1204-1266).
 * All pointers are device pointers.  Inputs:
 *   Pr, Prd      [T][n_rows]   the HL path Pr_refined_ / Prd_refined_ (2*NA x T, column-major as
 *                              Eigen stores it); agent id uses rows 2 id, 2 id + 1
 *   agent_id     [A] int       (NULL: agent_offset + a)
 *   gait_domain  [A] int       gaitDomain_: the window starts at column 4 * gaitDomain_ (NDOMAIN
 *                              grids per domain) and spans N columns
 *   contact      [A][4] int    contactInd (FR, FL, RR, RL); must give C contacts
 *   toe          [A][3][4]     toePos (row-major 3 x 4)
 *   start        [A][2]        agent_Initial_ (default stance while gaitDomain_ <= 1)
 *   q, dq        [A][18]       generalised coordinates / velocities (q[0], q[1], dq[0], dq[1] used)
 * Outputs: x0 [A][4], ref [A][4N], foot [A][N][2][C] (the srb_batch inputs), last_state [A][4]
 * (the neighbour-snapshot row), status [A] int: 0 ok, 1 contact pattern does not give C
 * contacts, 2 reference window outside the path.
 */
typedef struct srb_prep {
    int struct_size;         /* sizeof(srb_prep) (ABI check) */
    const double *Pr, *Prd;
    int n_rows, T, agent_offset;
    const int *agent_id, *gait_domain, *contact;
    const double *toe, *start, *q, *dq;
    double *x0, *ref, *foot, *last_state;
    int *status;
} srb_prep;
int srb_prepare_batch_device(srb_ctx *ctx, int n_agents, const srb_prep *dev_io, void *stream);

/*
 * HL reference planner (generateReferenceTrajectory, MPC_dist.cpp:930-1104; SURVEY.md 8(f)
 * row 3) on HIP device `device`, host buffers, synchronous.  NA agents (1..2^20; up to 1024 in
 * one persistent workgroup, more -- one coupled swarm -- as one launch per step) starting at
 * Pstart [NA][2], planner obstacles Pobs [n_obs][2] (n_obs <= 2048), `loop` steps (reference:
 * 100000).  Outputs Pr_refined_ / Prd_refined_ as column-major 2NA x (loop / 40) arrays (the
 * layout setReferenceTrajectory / srb_prep take).  Returns 0 or a negative error code.
 */
int srb_hl_plan(int device, int NA, const double *Pstart, const double *Pobs, int n_obs, int loop, double *Pr,
                double *Prd);

/* Per-launch timing of the last srb_solve_batch_device call, measured with HIP events on
 * the stream the kernel ran on (ms): knn_ms the obstacle / neighbour selection kernel
 * (0 when nothing is selected: QP only, or K_obs = K_nbr = 0), solve_ms the solve kernel. */
int srb_last_kernel_ms(srb_ctx *ctx, float *knn_ms, float *solve_ms);
/* ... and of the active-set polish of the NLP result (srb_polish_kernel, launched right after the
 * solve kernel), ms. */
int srb_last_polish_ms(srb_ctx *ctx, float *polish_ms);

/* Dynamic LDS bytes one agent's workgroup uses (for occupancy reports). */
int srb_lds_bytes(const srb_params *p);

/* Bezier fit of the predicted CoM states (fitComTrajectory_eventbase, MPC_dist.cpp:784-855),
 * host-side: alpha[4][5] from the buffer state buf[4] and X[0..3] (4 states). */
void srb_fit_bezier(const double buf[4], const double *X, double alpha[20]);

/*
 * ---- Low-level CLF-QP controller ----------------------------------
 * Replaces LowLevelCtrl::calcTorque(state, dyn, kin, vc, con, params)
 * (/root/reference/include/LowLevelCtrl.hpp:20, src/LowLevelCtrl.cpp:18-113) for a batch of
 * agents: QP assembly (cost :115-137, constraints :139-236), the iswiftQp_e solve (:33-37,
 * iSWIFT Prime.c:127-230), the parse into ll.QP_force / tau / dV (:44-64), swing-leg PD
 * (:71-91), the integration ll.ddq / ll.dq / ll.q (:96-98) and swingInvKin (:446-488).
 * One QP per agent: numDec = 3c + 12 + outDim + useCLF (<= 31) variables
 * [F (3c, stance legs FR,FL,RR,RL) | tau (12) | aux (outDim = 6 + 3(4-c)) | d].
 */
typedef struct srb_ll_params {      /* Settings::LL_params (global_loco_structs.hpp:96-111) */
    double mu, kp, kd;
    int useCLF;
    double tauPen, dfPen, auxPen, clfPen, auxMax, clfEps;
    int maxit;                      /* iSWIFT MAXIT 25 (GlobalOptions.h:23) */
    double tol;                     /* 1e-6 (GlobalOptions.h:24-25) */
} srb_ll_params;

/* Parameters.cpp:62-75 defaults: mu 0.7, kp 700, kd 40, useCLF 1, tauPen 1, dfPen 0.1,
 * auxPen 1e6, clfPen 1e8, auxMax 100, clfEps 0.8. */
void srb_ll_params_default(srb_ll_params *p);

/*
 * One batch, agent-major.  Matrices are column-major (Eigen's storage) with FIXED leading
 * dimensions, so every agent has the same stride whatever its contact count:
 *   ind      [A][4] int      ConInf::ind (1 stance, 0 swing; other values -> status 3)
 *   q, dq    [A][18]         StateInfo::q, dq
 *   Dinv     [A][18*18]      DynamicsInfo::Dinv
 *   B        [A][12*18]      DynamicsInfo::B (18 x 12, ld 18)
 *   H        [A][18]         DynamicsInfo::H
 *   Jc, Js   [A][18*12]      KinematicsInfo::Jc (3c x 18), Js ((12-3c) x 18), ld 12
 *   dJc      [A][12]         KinematicsInfo::dJc (3c used)
 *   Jtoe, Jhip [A][18*12]    KinematicsInfo::Jtoe, Jhip (12 x 18, ld 12)
 *   toePos, hipPos [A][12]   KinematicsInfo::toePos, hipPos (3 x 4: column per leg)
 *   H0       [A][18*18]      VCInfo::H0 (outDim x 18, ld 18)
 *   dH0, y, dy [A][18]       VCInfo (outDim used)
 *   hd, dhd  [A][18]         VCInfo::hd, dhd (rows 6.. hold the swing-toe targets)
 *   fDes     [A][12]         VCInfo::fDes
 * In/out:
 *   tau      [A][18]         LowLevelCtrl::tau (the member array: entries 0..5 carry over
 *                            between calls and accumulate the swing PD, :91)
 * Outputs:
 *   QP_force [A][12], ddq, dq_out, q_out [A][18]  LLInfo (global_loco_structs.hpp:74-80)
 *   V, dV    [A]             LLInfo::V, dV
 *   x        [A][32]         QP solution (optimOut), zero-padded beyond numDec; may be NULL
 *   status   [A] int         iSWIFT exit code (0 OPTIMAL, 1 KKTFAIL, 2 MAXIT, 3 bad contact flags)
 *   iters    [A] int         interior-point iterations
 */
typedef struct srb_ll_io {
    int struct_size;         /* sizeof(srb_ll_io) (ABI check) */
    const int *ind;
    const double *q, *dq, *Dinv, *B, *H, *Jc, *dJc, *Js, *Jtoe, *Jhip, *toePos, *hipPos;
    const double *H0, *dH0, *y, *dy, *hd, *dhd, *fDes;
    double *tau, *QP_force, *ddq, *dq_out, *q_out, *V, *dV, *x;
    int *status, *iters;
} srb_ll_io;

typedef struct srb_ll_ctx srb_ll_ctx;

int srb_ll_ctx_create(const srb_ll_params *p, int max_agents, int device, srb_ll_ctx **out);
int srb_ll_ctx_destroy(srb_ll_ctx *ctx);
/* host buffers: copies in, solves, copies out, synchronises */
int srb_ll_calc_torque(srb_ll_ctx *ctx, int n_agents, const srb_ll_io *host_io);
/* device buffers, asynchronous on `stream` (NULL = the HIP null stream); call srb_ll_sync() */
int srb_ll_calc_torque_device(srb_ll_ctx *ctx, int n_agents, const srb_ll_io *dev_io, void *stream);
int srb_ll_sync(srb_ll_ctx *ctx);
/* HIP-event time of the last srb_ll_calc_torque[_device] kernel on its stream (ms) */
int srb_ll_last_kernel_ms(srb_ll_ctx *ctx, float *ms);

/* ================================================================ SRB-12 extension mode
 * The north star's 12-state single-rigid-body NMPC (state [p, roll/pitch/yaw, v, omega], inputs the
 * four leg forces, friction pyramid + f_z <= fmax, the obstacle rows of the LIP mode).  The
 * reference DECLARES this solver (FastMPC::runMPC / MPC_Cost / MPC_Constraints /
 * getLinearDynamics, include/fast_MPC.hpp:98-103) without implementing it, so these entry points
 * replace no reference binding; the problem is stated in DESIGN.md section 11, the CPU checker is
 * oracle/srb12.c (parity with the reference unpinned).  Constants: mass and inertia of FastMPC
 * (src/fast_MPC.cpp:40-43), weights and mu_MPC of the default mpc_params (src/Parameters.cpp:32-52).
 */
typedef struct srb12_params {
    int N, K_obs, K_nbr;          /* grids (<= 24), nearest static obstacles / neighbours (each <= 16) */
    double Ts, mass, Ib[9], grav, mu, fmax;
    double q[12], qN[12], r[3], Sw;     /* stage / terminal state weights, force weights (per axis), slack */
    double eps_obs, eps_nbr, tol;
    int qp_maxit, nlp_maxit, use_nlp;
    double z0;                    /* NLP initial duals z0 / max(s, 1) */
    double tol_final;             /* complementarity s'z/m < tol_final ends the LAST stage (the NLP, or the QP when
                                     use_nlp = 0; default 1e-8): far enough for the polish to identify the active
                                     set (without the polish 1e-8 leaves the forces up to 1e-3 N from
                                     the exact optimum, 1e-6 up to 3e-2 N) */
    int polish;                   /* 1 (default): the last stage's result is polished to the exact KKT point of
                                     its active set (forces within 1e-4 N of the optimum); 0 off */
    double tol_qp;                /* the QP stage's tolerance when the NLP stage follows it (default 1e-3; 0: tol):
                                     the NLP is warm-started from that point, so its accuracy does not carry into
                                     the result (QP iterations 4.1 -> 2.6 on average, 6 -> 4 at most) */
} srb12_params;

void srb12_params_default(srb12_params *p, int N);
int srb12_nv(const srb12_params *p);   /* 24N + 1: X = x_1..x_N (12N) | U = u_0..u_{N-1} (12N) | s */

/* Batch buffers, agent-major fp64 (int32 where noted):
 *   x0 [A][12]; xref [A][N][12] (x_1..x_N); foot [A][N][4][3] (world foot positions per grid, legs FR FL
 *   RR RL); contact [A][N][4] int (1 stance); obstacles / nbr_state / n_obs / n_all / agent_offset /
 *   sel / obstacles_version as in srb_batch (the neighbour snapshot rows are [x, y, xdot, ydot]);
 *   outputs x_qp (may be NULL), x [A][24N+1], obj [A], status [A][2], iters [A][2]; a FATAL (3) QP stage ends the
 *   solve before the NLP stage, whose status then reads FATAL as well (use_nlp = 1).
 *   status codes 0..3 as iSWIFT's; 4 by stage: the LAST stage (the NLP, or the QP when use_nlp = 0) converged but
 *   its polish was rejected (the interior-point result is returned); the QP stage followed by the NLP converged at
 *   tol_qp only (QP_WARM, x_qp is the NLP's warm start); with use_nlp = 0 status[1] and iters[1] read 0 */
typedef struct srb12_batch {
    int struct_size;              /* sizeof(srb12_batch) (ABI check) */
    const double *x0, *xref, *foot;
    const int *contact;
    const double *obstacles, *nbr_state;
    int n_obs, n_all, agent_offset;
    double *x_qp, *x, *obj;
    int *status, *iters;
    int *sel;                     /* optional [A][K_obs + K_nbr] selected rows */
    int obstacles_version;
} srb12_batch;

typedef struct srb12_ctx srb12_ctx;
int srb12_ctx_create(const srb12_params *p, int max_agents, int device, srb12_ctx **out);
int srb12_ctx_destroy(srb12_ctx *ctx);
/* host buffers: copies in, solves, copies out, synchronises */
int srb12_solve_batch(srb12_ctx *ctx, int n_agents, const srb12_batch *host_io);
/* device buffers, asynchronous on `stream` (NULL = the HIP null stream) */
int srb12_solve_batch_device(srb12_ctx *ctx, int n_agents, const srb12_batch *dev_io, void *stream);
/* HIP-event times of the last call's selection and solve kernels (ms) */
int srb12_last_kernel_ms(srb12_ctx *ctx, float *select_ms, float *solve_ms);
/* 1 (default): HIP events around the selection and solve kernels (srb12_last_kernel_ms); 0: none */
int srb12_ctx_set_timing(srb12_ctx *ctx, int on);
int srb12_lds_bytes(const srb12_params *p);

const char *srb_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
