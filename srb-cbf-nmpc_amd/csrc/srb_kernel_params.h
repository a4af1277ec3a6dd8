// Kernel-side parameter block (host fills it from srb_params, see srb_capi.cpp) and the
// per-instance LDS budget.
#pragma once

#define SRB_KNN_MAX 16    // nearest static obstacles / neighbours per agent (each)
#ifndef SRB_REFINE
#define SRB_REFINE 1      // iterative-refinement steps per reduced Newton solve
#endif
#ifndef SRB_KNN_WAVES
#define SRB_KNN_WAVES 2   // waves per agent in the selection kernel (srb_knn_kernel; 2: 1 % faster configs[2] step than 4, round 4)
#endif
#define SRB_GRID_CELLS 16384      // cells of the selection grid (LDS counters of srb_grid_build_kernel)
#define SRB_GRID_MIN_ROWS 8192    // tables this long get a grid (shorter: brute-force scan)
#define SRB_GRID_MIN_ROWS_STATIC 4096   // versioned static obstacle tables (grid built once, reused):
                                         // configs[2]'s 5120 rows: selection 37.8 -> 31.3 us (profiles/r02_grid_threshold.txt)
#define SRB_MAX_NZ 32     // reduced Newton system size bound: nz = N(C-1)+1 <= 32
#define SRB_MAX_N 33      // CoM-CoP slots 2(N-1) fit one 64-lane trip
// NLP stage: initial inequality duals (the oracle's ORC_NLP_Z0, oracle/nlp_ipm.c).  100 is the
// scale of the tracking weights' multipliers; on the five bench/test workloads it takes the
// NLP from 10.4-11.4 to 8.0-8.6 iterations on average and from 13-18 to 9-13 at most
// (profiles/r01_nlp_z0_scan.txt) against z = 1.
#define SRB_NLP_Z0 100.0
// NLP stage: a step (primal or dual) shorter than this from a near-optimal iterate ends the
// solve as ACCEPTABLE, status 4 (oracle ORC_NLP_BLOCKED)
#define SRB_NLP_BLOCKED 0.05
// NLP stage: OPTIMAL also needs the last primal step max |ap dx| below this (oracle
// ORC_NLP_DXTOL): the residual tests alone left 3.6 % of N = 20 solves 1e-4..5e-4 from the
// optimum along flat directions (profiles/r02_nlp_exit.txt); after SRB_NLP_NEARWAIT
// near-optimal iterates without meeting both, the solve is at its round-off floor: ACCEPTABLE
#define SRB_NLP_DXTOL 1e300     // round 3: off (the polish makes the result exact; oracle ORC_NLP_DXTOL)
// QP stage followed by the NLP stage: its point only warm-starts the NLP (the duals restart), so it runs to
// this tolerance (srb_ctx_set_option SRB_OPT_QP_WARM_TOL; 0: the reference's 1e-6).  Round 5: 1e-2 (QP
// iterations 5.8 -> 3.8 on average at configs[2], NLP iterations and statuses unchanged, the result within
// 4e-11), then 0.3 from a scan on the GPU (1e-2 / 3e-2 / 0.1 / 0.3 / 1 / 3: configs[2] 0.317 -> 0.309 ms,
// config 5 1.74 -> 1.68 ms; QP iterations 3.8 -> 3.0 and 4.4 -> 3.7, NLP iterations and every status
// unchanged; profiles/r05_qp_warm_tol_scan.txt)
#define SRB_QP_WARM_TOL 3e-1
// NLP stage: dual-residual and complementarity tests this much looser than the QP's (the polish
// after the solve lands on the exact KKT point of the active set the interior point identified;
// 15 % fewer NLP iterations on the bench batches, polished results unchanged within 4e-7)
#define SRB_NLP_EXITF 10.0
#define SRB_NLP_NEARWAIT 4
// NLP stage: active-set polish of the final iterate (oracle/nlp_ipm.c `polish`, the same rules):
// rows with s * KAPPA < z are taken as active and the equality-constrained problem is solved by at
// most IT Newton steps (fewer once a correction is <= DXTOL) on its KKT system regularised by
// 1/RHO; at most PASSES active sets (the most negative multiplier leaves, violated rows join).
// Accepted (-> OPTIMAL) only if every row is within PTOL of its bound, the active rows hold to PTOL,
// z_A >= -1e-9 max|z_A| and the last Newton correction is <= DXTOL.
#ifndef SRB_POLISH_ON
#define SRB_POLISH_ON 1
#endif
// instances whose solve kernel carries the fused polish (srb_kernels.hip; srb_capi.cpp launches the
// polish kernel for the others).  Round 5: up to NZL 24 -- with the obstacle positions moved into the
// Z'Z buffer (SRB_OBS_IN_ZZ) two N = 20 agents with the fused polish's buffer fit one CU's LDS, and
// config 5 went 2.49 -> 2.33 ms (2.12 with the horizon compiled in, SRB_N20_NC)
#ifndef SRB_FUSED_POLISH_MAX
#define SRB_FUSED_POLISH_MAX 24
#endif
#define SRB_FUSED_POLISH_OK(NZL) ((NZL) <= SRB_FUSED_POLISH_MAX)

// diagnostic trace buffer of the nlpdbg build (srb_kernels.hip, srb_capi.cpp)
#define SRB_NLP_DBG_LEN (8 * 64 + 32 * 32 + 32 + 1024 + 256 + 3 * 256)
#define SRB_POLISH_RHO 1e9
#define SRB_POLISH_KAPPA 1e4
#define SRB_POLISH_OMCAP 1e-2      // inactive rows: proximal Hessian weight min(z/s, OMCAP)
#define SRB_POLISH_IT 5
#ifndef SRB_POLISH_PASSES
#define SRB_POLISH_PASSES 4
#endif
#define SRB_POLISH_PTOL 1e-9
#define SRB_POLISH_DXTOL 1e-7
// and only where the equality rows (LIP dynamics, CoP, sum lambda) hold to this (lip_eq_res, srb_kernels.hip)
#ifndef SRB_POLISH_EQTOL
#define SRB_POLISH_EQTOL 1e-8
#endif
// and only where the Newton correction M^-1 g that the reduced stationarity residual g = Z'(grad f + J_A' z_A) implies
// is <= this (polish_stationary, srb_kernels.hip; oracle ORC_POLISH_STOL: at most 6e-8 on the accepted polishes of six
// bench workloads, round 6)
#ifndef SRB_POLISH_STOL
#define SRB_POLISH_STOL 1e-6
#endif
#ifndef SRB_POLISH_EQCHECK        // 0: diagnostic builds without the equality test
#define SRB_POLISH_EQCHECK 1
#endif
// a Newton step <= DX1 after which every active row holds to CTOL (its quadratic remainder) ends the
// pass as converged without the verifying step (oracle ORC_POLISH_DX1 / ORC_POLISH_CTOL)
#define SRB_POLISH_DX1 1e-4
#define SRB_POLISH_CTOL 1e-10
// divergence: a dual beyond this ends a stage FATAL at its finite iterate (infeasible rows; converging
// solves keep their duals below ~1e4 on every workload; oracle ORC_Z_DIV)
#define SRB_Z_DIV 1e10
// cross-wave reduction scratch: sites of up to 8 doubles per wave (srb_kernels.hip)
#define SRB_RED_SITES 10

struct SrbKParams {
    int N, C, K_obs, K_nbr;
    int n, nz, mq, use_nlp;
    int qp_maxit, nlp_maxit;
    int qp_init;                           // QP starting point: 1 scaled (s = max(h - Gx, 0.1), z = 1/s), 0 iSWIFT's kkt_initialize
    int polish_fused;                      // 1: the polish runs at the end of the solve kernel (no polish kernel)
    double polish_rho;                     // SRB_POLISH_RHO (SRB_OPT_POLISH_RHO)
    double qp_warm_tol;                    // the QP stage's tolerance when the NLP stage follows (SRB_OPT_QP_WARM_TOL)
    double kkt32_mu;                       // fp32-factor instances: fp32 inverse while mu > this (SRB_OPT_KKT_FP32_MU)
    int kkt32_ref;                         // ... and this many fp64 refinement steps per solve then (SRB_OPT_KKT_FP32_REFINE)
    double Ad[16], Bd[8];                  // LIP discretisation (MPC_dist.cpp:126-127)
    double Qw, Pw, Rw, Sw, box, fr;        // gains (:172-175), box (:317), mu*h/sqrt(2) (:315)
    double eps_obs, eps_nbr, vsat, tol, Ts;
    double Binv[25];                       // inverse 5x5 Bernstein matrix at s = 0, 1/4, .., 1 (Bezier fit)
};

// Kernel instances (NZL, TS, NW, NC, CC, KC): register bound on nz (one reduced-matrix row per
// lane), slot trips per thread, wavefronts per agent (n + 2(N-1) + 2N + N K row slots over 64 NW
// threads, see srb_kernels.hip), and the problem shape (N, C, K = K_obs + K_nbr) the instance is
// compiled for -- 0: read at run time.  A compiled shape makes every LDS offset and loop bound of
// the agent a constant (the bench shapes configs[1] and configs[2] / [3]: 12 % and 7 % faster steps;
// the N = 20 shape, configs[4] / config 5: compiled whole since round 5 -- the round-4 build of it
// returned wrong polishes on a quarter of the agents, the code-generation hazard of DESIGN.md 11 that
// tests/test_isa_hazard.py now scans every shipped kernel for; this one is clean and 9 % faster).  The
// host launches the first fitting instance of this list (an exact shape first, then the run-time
// ones) with NW = 4 for small batches (one agent per CU, all four SIMDs) and NW = 1 otherwise
// (srb_capi.cpp).
#ifndef SRB_WPE                 // extra kernel attribute of the solve instances (register-tuning builds)
#define SRB_WPE
#endif
#ifdef SRB_DEV_INSTANCES          // register-tuning builds of a few instances (make dev)
#define SRB_KERNEL_INSTANCES(X) SRB_DEV_INSTANCES(X)
#else
// the host picks the first fitting instance of this list (srb_capi.cpp), so its order matters
#ifndef SRB_N20_NC               // horizon compiled into the configs[4]-shape instance (0: read at run time)
#define SRB_N20_NC 20
#endif
#define SRB_XE(X, ...) X(__VA_ARGS__)   // expands SRB_N20_NC before X pastes it into the kernel name
#define SRB_KERNEL_INSTANCES(X) \
    X(12, 4, 1, 10, 2, 11) X(12, 1, 4, 10, 2, 3) SRB_XE(X, 24, 4, 2, SRB_N20_NC, 2, 11) \
    X(8, 1, 1, 0, 0, 0) X(16, 1, 1, 0, 0, 0) X(12, 3, 1, 0, 0, 0) X(12, 4, 1, 0, 0, 0) X(16, 4, 1, 0, 0, 0) \
    X(24, 5, 1, 0, 0, 0) X(24, 8, 1, 0, 0, 0) X(32, 4, 1, 0, 0, 0) X(32, 8, 1, 0, 0, 0) \
    X(8, 1, 4, 0, 0, 0) X(12, 1, 4, 0, 0, 0) X(16, 1, 4, 0, 0, 0) X(16, 2, 4, 0, 0, 0) X(32, 2, 4, 0, 0, 0) \
    X(12, 2, 2, 0, 0, 0) X(16, 2, 2, 0, 0, 0) X(24, 4, 2, 0, 0, 0) X(24, 2, 4, 0, 0, 0)
// the same instances in four parts of about equal compile time: the product build compiles
// srb_kernels.hip once per part (-DSRB_PART=0..3, in parallel)
#define SRB_KI_PART0(X) X(12, 4, 1, 10, 2, 11) X(12, 4, 1, 0, 0, 0) X(8, 1, 1, 0, 0, 0) X(16, 1, 1, 0, 0, 0) \
    X(12, 3, 1, 0, 0, 0) X(8, 1, 4, 0, 0, 0)
#define SRB_KI_PART1(X) SRB_XE(X, 24, 4, 2, SRB_N20_NC, 2, 11) X(24, 4, 2, 0, 0, 0) X(12, 1, 4, 0, 0, 0) X(16, 4, 1, 0, 0, 0) \
    X(12, 2, 2, 0, 0, 0)
#define SRB_KI_PART2(X) X(12, 1, 4, 10, 2, 3) X(24, 5, 1, 0, 0, 0) X(24, 8, 1, 0, 0, 0) X(16, 1, 4, 0, 0, 0) \
    X(16, 2, 4, 0, 0, 0) X(16, 2, 2, 0, 0, 0)
#define SRB_KI_PART3(X) X(32, 4, 1, 0, 0, 0) X(32, 8, 1, 0, 0, 0) X(32, 2, 4, 0, 0, 0) X(24, 2, 4, 0, 0, 0)
#endif
// fp32-factor variants of the bench shapes (srb_nmpc_kernel_f32_*, SRB_OPT_KKT_FP32_MU > 0; configs[4]'s "fp32
// KKT with fp64 iterative-refine residuals"): config 5's instance in part 3, configs[2]'s in part 2
#define SRB_KF32_PART2(X) X(12, 4, 1, 10, 2, 11)
#define SRB_KF32_PART3(X) SRB_XE(X, 24, 4, 2, SRB_N20_NC, 2, 11)
#define SRB_KF32_INSTANCES(X) SRB_KF32_PART2(X) SRB_KF32_PART3(X)
// host and device (the LDS-bounds diagnostic build checks the kernel's carve against srb_lds_doubles)
#if defined(__HIPCC__)
#define SRB_HD __host__ __device__
#else
#define SRB_HD
#endif
SRB_HD static inline int srb_slots(int N, int C, int K) { return (6 + C) * N + 1 + 2 * (N - 1) + 2 * N + N * K; }

SRB_HD static inline int srb_r4(int x) { return (x + 3) & ~3; }


// doubles of dynamic LDS one agent needs for instance bound NZL; must match the carve in
// nmpc_agent (srb_kernels.hip)
// Obstacle rows: materialised as term rows in LDS at each re-linearisation for the small instances
// (NZL <= SRB_OBS_STORED_MAX: a stored row is one LDS load per Gram element), folded per grid into three
// terms built from the grid's CoM rows for the large ones (srb_kernels.hip ObsFold: at N = 20 the Gram's
// obstacle part 14 -> 4 batches; at configs[1] / [2] the fold measured 7 % / 1.6 % slower than stored rows)
#ifndef SRB_OBS_STORED_MAX
#define SRB_OBS_STORED_MAX 16
#endif
#define SRB_OBS_STORED(NZL) ((NZL) <= SRB_OBS_STORED_MAX)

// the obstacle positions (2 N K + 2 doubles, read by the slots' setup only) share the Z'Z buffer when they
// fit there: Z'Z is first written by the NLP setup's Gram, after every slot has read its position
#define SRB_OBS_IN_ZZ(NZL, NK) (2 * (NK) + 2 <= (NZL) * ((NZL) + 1))

SRB_HD static inline int srb_lds_doubles(const SrbKParams &p, int NZL, int NW)
{
    const int NZM = ((NZL + 15) / 16) * 16, LDR = NZL + 1, LDH = NZL + 1;
    const int N = p.N, C = p.C, K = p.K_obs + p.K_nbr, n4 = srb_r4(p.n), NK = N * K;
    const int q = 16 * NW;
    const int rU = (4 * N + 2 * (N - 1) + q - 1) / q * q;                                  // X, CoM-CoP rows
    const int rO = (rU + srb_r4(p.n - 4 * N) + q - 1) / q * q;                              // stored term rows
    const int NKP = (NK + q - 1) / q * q, TT = rO + NKP;          // + the obstacle rows' W / CF / (jx, jy) entries
    const int red = (NW > 1) ? 8 * SRB_RED_SITES * NW : 0;
    const int part = (NW > 2) ? NW * ((NZM == 16) ? 1 : 3) * 256 + NW * NZM : 0;
    return (SRB_OBS_STORED(NZL) ? TT : rO) * LDR + 2 * (TT + 1) + (SRB_OBS_STORED(NZL) ? 0 : 2 * NKP + 9 * (N + 1)) +
           2 * NZL * LDH + 4 * NZM + 4 * n4 + 4 * N + 2 * C * N +
           (SRB_OBS_IN_ZZ(NZL, NK) ? 0 : 2 * NK + 2) +
           (K + 1) + srb_r4(NK) + (K + 1) + red + part + (SRB_FUSED_POLISH_OK(NZL) ? srb_r4(srb_slots(N, C, K)) : 0)
#ifdef SRB_STAMPS
           + 64
#endif
        ;
}

// ---- low-level CLF-QP (srb_llctrl.hip; LowLevelCtrl::calcTorque, src/LowLevelCtrl.cpp:18-113)
// Host fills it from srb_ll_params (srb_capi.cpp): the gains of Settings::LL_params plus the
// constants of the CLF Lyapunov matrix (LowLevelCtrl.cpp:176-185) folded once per launch.
struct SrbLLKParams {
    double mus;                       // mu / sqrt(2)                         (:157)
    double kp, kd;
    double tauPen, dfPen, auxPen, clfPen;
    double p1e2, pde, p2;             // P1/eps^2, Pd/eps, P2 of tuneMat*PP*tuneMat (:176-190)
    double cce;                       // c / eps with c = 1 / lambda_max(PP0)  (:184-185, :233)
    double tol;
    int useCLF, maxit;
    int dbg_agent;                    // >= 0: that agent records a per-iteration trace (srb_ll_debug_trace)
};

#ifndef SRB_LL_WPE        // waves per SIMD the low-level kernel is compiled for (min, max)
#define SRB_LL_WPE 2, 8
#endif

// device layout of one agent (srb_ll_io, include/srbnmpc.h): column-major matrices with fixed
// leading dimensions
#define SRB_LL_NQ 18   // TOTAL_DOF (global_loco_opts.h:24)
#define SRB_LL_NU 12   // TOTAL_IN  (global_loco_opts.h:25)

// ---- SRB-12 extension mode (srb12_kernels.hip; the north star's 12-state single rigid body,
// declared but never implemented by the reference, include/fast_MPC.hpp:98-103)
struct Srb12KParams {
    int N, K_obs, K_nbr, use_nlp;
    int qp_maxit, nlp_maxit, polish;
    double Ts, mass, grav, mus, fmax, Sw, eps_obs, eps_nbr, tol, z0, tol_final, tol_qp;
    double Ib[9];                     // body inertia (fast_MPC.cpp:41-43)
    double q[12], qN[12], r[3];       // stage / terminal state weights, force weights
    int dbg_agent;                    // >= 0: that agent records a per-iteration trace into dbg
    double *dbg;                      // [2 stages][64 iterations][8] (srb12_debug_trace)
};
#define SRB12_MAX_N 24
// active-set polish of the last stage's result (oracle/srb12.c ORC12_POL_*, the same constants)
#define SRB12_POL_RHO 1e9
#define SRB12_POL_KAPPA 1e4
// (round 5: 8 steps, 4 passes -- with 5 and 2, 1 of 1024 stand agents ended a pass still contracting
// linearly under the pass's frozen factor, or needed a third active set; the oracle at 6 x 1024 agents:
// 2 rejected -> 0, Newton steps +0.1 %)
#define SRB12_POL_IT 8
#define SRB12_POL_PASSES 4
#define SRB12_POL_PTOL 1e-9
#define SRB12_POL_DXTOL 1e-7
#define SRB12_POL_DYNTOL 1e-8      // accepted only where max_k |x_{k+1} - A_k x_k - B_k u_k - c_k| <= this
// kernel instances (TL, TO, NC, K1): leg-slot trips (4N legs over 64 lanes), obstacle-slot trips (N K
// rows), and the horizon N and rows per grid K compiled in (NC = N, K1 = K + 1) or read at run time
// (NC = K1 = 0).  The host launches the compiled-in instance of the problem's (N, K) when there is one
// (every LDS offset and e / K a constant: fewer instructions and SGPRs in the stage loops), else the
// first run-time instance whose trips fit
#define SRB12_INSTANCES(X) X(1, 2, 10, 12) X(2, 4, 20, 12) \
    X(1, 1, 0, 0) X(1, 2, 0, 0) X(1, 4, 0, 0) X(1, 8, 0, 0) X(1, 12, 0, 0) X(2, 4, 0, 0) X(2, 8, 0, 0) X(2, 12, 0, 0)
static inline int srb12_leg_trips(int N) { return (4 * N + 63) / 64; }
static inline int srb12_obs_trips(int N, int K) { return (N * K + 63) / 64 > 0 ? (N * K + 63) / 64 : 1; }
// doubles of LDS one agent needs (the carve in srb12_kernels.hip)
static inline int srb12_lds_doubles(int N, int K)
{
    return 36 * N + 2 * N + 4 * N                        // W_l, (cos, sin) psi, contact
           + 156 * N + 78 * N                           // K_k, Hu_k^-1 (packed) per grid
           + 324                                        // factor transposes (+ 24 sink entries)
           + 6 * N + 24 * N                             // (p_x, p_y, s) blocks, force blocks
           + (24 * N + 4) + 12 * N                      // iterate (X | U | s), reference
           + 50 * N                                     // rhs columns 0 and 1 (the polish's saved iterate in column 0)
           + 13 * N + 12 * N + 12 * N                   // solution, feed-forward -Hu^-1 gu
           + 16 + 16 + 28 + 16                          // vector, scalars, the weights q, qN, r, x_0
           + 2 * N * K + K + K + 2                      // obstacle positions, eps, sel (as ints)
           + 16;                                        // stamp accumulators (diagnostic build make s12st)
}
