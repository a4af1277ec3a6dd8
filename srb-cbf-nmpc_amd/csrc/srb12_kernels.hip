// SRB-12 extension mode for MI355X (gfx950): the batched CBF-NMPC of the north star on the
// 12-state single rigid body.  The reference declares this model (FastMPC::runMPC, MPC_Cost,
// MPC_Constraints, getLinearDynamics: /root/reference/include/fast_MPC.hpp:98-103) but never
// implements it, so the problem is stated in DESIGN.md section 11 and in oracle/srb12.c (the
// CPU checker this kernel is tested against); parity with the reference is UNPINNED.
//
//   state  x = [p, Theta (roll, pitch, yaw), v, omega] (12), inputs u_k = four leg forces (12);
//   x_{k+1} = A_k x_k + B_k u_k + c_k, the convex-MPC linearisation about the reference yaw:
//     A_k = I + Ts E(psi_k)  (p += Ts v, Theta += Ts Rz' omega),
//     B_k: v += Ts f / m, omega += Ts I_w^-1 (r_l x f_l) per stance leg l (W_l = Ts I_w^-1 [r_l]x);
//   cost  sum (x - x_ref)' Q (x - x_ref) / 2 + u' R u / 2 + Sw s^2 / 2;
//   rows  friction pyramid + f_z <= fmax per stance leg (LowLevelCtrl.cpp:158-162), and in the
//         NLP stage the obstacle rows -|p_k - o_kj|^2 - s <= -eps_j (dec_vars_constr_cost.h:262-302).
//
// Execution model: one 64-lane wavefront per agent runs both interior-point stages (QP without
// the obstacle rows, then the NLP warm-started from it) and the active-set polish of the last
// stage -- the iteration of oracle/srb12.c step for step.  The Newton system is solved by a Riccati
// recursion over the horizon (O(N 13^3) per iteration) instead of the oracle's dense LU.  The
// obstacle slack s rides along as a 13th state (s_{k+1} = s_k, s_0 free), so the stiff obstacle
// rows stay inside one grid's block.  Round 4 layout:
//   * rows: a LEG slot per (grid, leg) holds that leg's six friction rows in the registers of one
//     lane (its 3 x 3 Hessian block and force gradient are formed in-lane, no atomics); an OBSTACLE
//     slot per (grid, row) adds its (p_x, p_y, s) block by LDS atomics;
//   * factor, stage k: the products G = V A~, F = V B~, A~'G, B~'G, B~'F on the matrix cores
//     (v_mfma_f64_16x16x4f64; V stays in the accumulator layout from stage to stage, whose D
//     operand is directly the next product's B operand), then Hu = L D L' by a COLUMN-oriented
//     elimination of [Hu | Hux | I] (lane j holds column j: one readlane of the pivot column's
//     multipliers per entry, 37 columns over 37 lanes), Y = D^-1/2 L^-1 Hux, Z = D^-1/2 L^-1, and
//     Y'Y (the Schur update, positive semi-definite by construction), Hu^-1 = Z'Z and the gain
//     K = -Z'Y as three more MFMA products; per stage K and Hu^-1 go to LDS for the solves;
//   * solves: vectors in registers, component i = lane & 15 replicated in the four 16-lane rows;
//     each matrix-vector product is split over the rows (row g takes columns 4g..4g+3, gathered by
//     ds_bpermute), then summed across rows by two permlane swaps -- 4 LDS reads per lane and
//     product instead of 13, and a 4-long instead of a 13-long dependent chain.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "srb_kernel_params.h"

#ifndef SRB12_REFINE_PREDICTOR        // 1: refine the predictor's solve too (round-3 behaviour)
#define SRB12_REFINE_PREDICTOR 0
#endif
#ifndef SRB12_REFINE                  // 0: no iterative refinement at all (A/B builds)
#define SRB12_REFINE 1
#endif
// a second refinement step of the corrector's solve once mu < this (round 6): below
// s'z/m ~ 1e-9 the barrier weights z/s reach 1e10 and one step left the corrector at the Riccati solve's
// round-off floor (|r_d| 4e-6 -> 4e-3, the iterate wandering into MAXIT on 3 of 1024 stand agents at tol_final
// 1e-9, 20 at 1e-10); with the second step every agent converges at 1e-9 and 1e-10 (profiles/r06_s12_tolfinal.txt).
// At the default tol_final 1e-8 it never runs (results identical).  The correctly rounded 1/sqrt pivot
// (SRB12_EXACT_RSQ) was not the cause: alone it changes nothing.
#ifndef SRB12_REFINE2_MU
#define SRB12_REFINE2_MU 1e-8
#endif
#ifndef SRB12_REFINE_MU               // the corrector's solve is refined once mu < this
#define SRB12_REFINE_MU 1e-3
#endif

// one wave per SIMD is the design point (four agents per CU by LDS): the scheduler may spend every
// register on latency hiding instead of trimming live ranges for an occupancy the LDS rules out
// (Overriding it is for diagnostic builds only, make s12var, which define SRB_DIAG_BUILD: the round-4
// build without it returned wrong OPTIMAL answers -- the compiler hazard of DESIGN.md 11, which
// tests/test_isa_hazard.py now scans every shipped kernel for.)
#ifdef SRB12_WPE
#ifndef SRB_DIAG_BUILD
#error "SRB12_WPE overrides the product SRB-12 instances' attribute: diagnostic builds only (make s12var)"
#endif
#else
#define SRB12_WPE __attribute__((amdgpu_waves_per_eu(1, 1)))
#endif

// The workgroup is one wavefront (launch bound 64): its LDS accesses are executed in issue order, so a
// barrier needs no hardware wait -- a wavefront-scope fence (no s_waitcnt) and a wave barrier keep the
// compiler from moving memory accesses across it.  (__syncthreads would add an lgkmcnt(0) wait for the
// stores before every barrier.)
// What this relies on: (1) LLVM IR -- a fence, whatever its scope, orders the thread's memory
// operations: no load or store is moved across it (an acq_rel fence is a read-write of all memory for
// alias analysis), so the ISA keeps the source order of the LDS accesses around SYNC; the wave barrier
// is IntrNoMem (a convergence point only) and is not what orders them.  (2) The AMDGPU memory model
// (LLVM AMDGPUUsage, memory model for GFX942 / GFX950): the LDS operations of one wavefront are performed
// in issue order, so a ds_read by any lane observes an earlier ds_write of the same wave without an
// s_waitcnt; the compiler still waits (lgkmcnt) before a loaded value is used.
#define SYNC() do { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); __builtin_amdgcn_wave_barrier(); } while (0)
#include "srb_wave.h"

namespace {

struct Srb12Lds {
    double *Wl, *cs, *ct, *Kst, *Hst, *T, *Q3, *Rh, *Z, *xr;
    double *rX, *rU, *gX, *gU, *dX, *dU, *kff, *vv, *sc, *obs, *eps, *xsv;
    double *wq, *wqN, *wr;                                  // the weights q, qN, r (lane-indexed reads)
    double *x0l;                                            // x_0 in LDS (selected by LDS pointers only: no flat access)
    int *sel;
};

// the carve of srb12_lds_doubles (srb_kernel_params.h), same order.  The right-hand side columns:
// column 0 (rX | rU: the Newton solves) and column 1 (gX | gU: gradients, the refinement's
// correction, the polish); the polish keeps the interior-point iterate in column 0's space (xsv)
__device__ __forceinline__ Srb12Lds carve12(double *p, int N, int K)
{
    Srb12Lds L;
    L.Wl = p; p += 36 * N;  L.cs = p; p += 2 * N;  L.ct = p; p += 4 * N;
    L.Kst = p; p += 156 * N;                                // K_k = -Hu^-1 Hux, 12 x 13 row-major per grid
    L.Hst = p; p += 78 * N;                                 // Hu_k^-1, packed lower triangle per grid
    L.T = p; p += 324;                                      // factor transposes (12-entry columns) + 24 sink entries
    L.Q3 = p; p += 6 * N; L.Rh = p; p += 24 * N;
    L.Z = p; p += 24 * N + 4; L.xr = p; p += 12 * N;
    L.rX = p; L.rU = p + 13 * N; L.gX = p + 25 * N; L.gU = p + 38 * N; L.xsv = p; p += 50 * N;
    L.dX = p; p += 13 * N; L.dU = p; p += 12 * N; L.kff = p; p += 12 * N;
    L.vv = p; p += 16; L.sc = p; p += 16;
    L.wq = p; L.wqN = p + 12; L.wr = p + 24; p += 28;
    L.x0l = p; p += 16;
    L.obs = p; p += 2 * N * K; L.eps = p; p += K;
    L.sel = (int *)p;
    return L;
}

// per-phase cycle stamps of the traced agent (diagnostic build -DSRB12_STAMPS, libsrbnmpc_s12st.so):
// s_memtime deltas accumulated into prm.dbg[SRB12_DBG_TRACE + slot], read by srb12_debug_trace
#define SRB12_DBG_TRACE (2 * 64 * 8)
#define SRB12_DBG_CHECK (SRB12_DBG_TRACE + 16)      // diagnostic build -DSRB12_CHECK: 128 state checks
#ifdef SRB12_STAMPS
#define S12ST(slot)                                                                                  \
    do {                                                                                             \
        if (dstamp) {                                                                                \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            if (tid == 0) stl[slot] += (double)(t_ - tprev);  /* LDS: no global round trip per stamp */ \
            tprev = t_;                                                                              \
        }                                                                                            \
    } while (0)
#else
#define S12ST(slot) do { } while (0)
#endif

// Rz(psi)[a][b] from (cos, sin)
__device__ __forceinline__ double rzab(int a, int b, double c, double s)
{
    return (a == 2 || b == 2) ? ((a == b) ? 1.0 : 0.0) : (a == b) ? c : (a == 0 ? -s : s);
}

// (A_k x)[i], x a 12-vector in LDS
__device__ __forceinline__ double a_mul(int i, const double *x, double Ts, double c, double s)
{
    double v = x[i];
    if (i < 3) v = fma(Ts, x[6 + i], v);
    else if (i < 6) v = fma(Ts, rzab(0, i - 3, c, s) * x[9] + rzab(1, i - 3, c, s) * x[10] + rzab(2, i - 3, c, s) * x[11], v);
    return v;
}
// (B_k u)[i] (i < 12); W: the grid's 4 x 9 leg blocks (contact and Ts folded in), ct: contact flags
__device__ __forceinline__ double b_mul(int i, const double *u, const double *W, const double *ct, double tsm)
{
    double v = 0.0;
    if (i >= 6 && i < 9) {
        for (int l = 0; l < 4; l++) v = fma(ct[l] * tsm, u[3 * l + i - 6], v);
    } else if (i >= 9 && i < 12) {
        const int a = i - 9;
        for (int l = 0; l < 4; l++)
            for (int j = 0; j < 3; j++) v = fma(W[9 * l + 3 * a + j], u[3 * l + j], v);
    }
    return v;
}
// friction row q of a leg: coefficients on (f_x, f_y, f_z) (LowLevelCtrl.cpp:158-162, + f_z <= fmax)
__device__ __forceinline__ void fric_coef(int q, double mus, double &c0, double &c1, double &c2)
{
    c0 = (q == 0) ? 1.0 : (q == 1) ? -1.0 : 0.0;
    c1 = (q == 2) ? 1.0 : (q == 3) ? -1.0 : 0.0;
    c2 = (q < 4) ? -mus : (q == 4) ? -1.0 : 1.0;
}
// index of (a, b) in a symmetric 3x3 block stored as 00 01 02 11 12 22
__device__ __forceinline__ int sym3(int a, int b)
{
    const int i = a < b ? a : b, j = a < b ? b : a;
    return (i == 0) ? j : (i == 1) ? 2 + j : 5;
}
// packed lower-triangle index of (i, j)
__device__ __forceinline__ int tri(int i, int j)
{
    return (i >= j) ? (i * (i + 1)) / 2 + j : (j * (j + 1)) / 2 + i;
}
// A~_k[i][j] (13 x 13: the 12 states and the slack; zero beyond)
__device__ __forceinline__ double atil(int i, int j, double Ts, double c, double s)
{
    double v = (i == j && i < 13) ? 1.0 : 0.0;
    if (i < 3 && j == i + 6) v = Ts;
    if (i >= 3 && i < 6 && j >= 9 && j < 12) v = Ts * rzab(j - 9, i - 3, c, s);
    return v;
}
// value of x held by lane `src` (any 64-bit register): ds_bpermute, no LDS memory traffic
__device__ __forceinline__ double perm_d(double x, int src)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// sum over the four 16-lane rows (lanes l, l^16, l^32, l^48), every lane gets the total: two
// permlane-swap stages, two values interleaved
__device__ __forceinline__ void rowsum2(double &a, double &b)
{
    double a0, a1, b0, b1;
    swap_d<32>(a, a0, a1); swap_d<32>(b, b0, b1);
    a = a0 + a1; b = b0 + b1;
    swap_d<16>(a, a0, a1); swap_d<16>(b, b0, b1);
    a = a0 + a1; b = b0 + b1;
}
__device__ __forceinline__ double rowsum(double a)
{
    double a0, a1;
    swap_d<32>(a, a0, a1); a = a0 + a1;
    swap_d<16>(a, a0, a1); return a0 + a1;
}
__device__ __forceinline__ d4 mfma(double a, double b, d4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

} // namespace

template <int TL, int TO, int NC, int K1>
__device__ __forceinline__ void srb12_agent(const Srb12KParams &prm, int agent, const double *__restrict__ x0g,
        const double *__restrict__ xrefg, const double *__restrict__ footg, const int *__restrict__ contactg,
        const double *__restrict__ obstacles, const double *__restrict__ nbr_state, const int *__restrict__ sel_g,
        double *__restrict__ x_qp_out, double *__restrict__ x_out, double *__restrict__ obj_out,
        int *__restrict__ status_out, int *__restrict__ iters_out, double *lds)
{
    const int tid = threadIdx.x, lane = tid;
    const int N = NC > 0 ? NC : prm.N, K = K1 > 0 ? K1 - 1 : prm.K_obs + prm.K_nbr;
    const int NK = N * K, nv = 24 * N + 1, NL = 4 * N;
    const double Ts = prm.Ts, tsm = prm.Ts / prm.mass, mus = prm.mus;
    const double tol = prm.tol;
    const int ci = lane & 15, gi = lane >> 4;          // column / component, 16-lane row
    Srb12Lds L = carve12(lds, N, K);
    double *X = L.Z, *U = L.Z + 12 * N;
    const double *x0 = x0g + 12 * (size_t)agent;
#ifdef SRB12_STAMPS
    const bool dstamp = agent == prm.dbg_agent && prm.dbg != nullptr;
    double *stl = (double *)L.sel + K + 2;              // 16 stamp accumulators (srb12_lds_doubles)
    if (tid < 16) stl[tid] = 0.0;
    unsigned long long tprev = dstamp ? __builtin_amdgcn_s_memtime() : 0ull;
#endif

    // ---------------- inputs, per-grid model (orc12_dynamics), selected rows
    for (int i = tid; i < 12 * N; i += 64) L.xr[i] = xrefg[(size_t)agent * 12 * N + i];
    for (int i = tid; i < 4 * N; i += 64) L.ct[i] = contactg[(size_t)agent * 4 * N + i] ? 1.0 : 0.0;
    // weights indexed by lane go through LDS: a lane-indexed read of the kernel-argument arrays is a
    // vector memory load, one per use inside the factor's and the solves' stage loops
    if (tid < 12) { L.wq[tid] = prm.q[tid]; L.wqN[tid] = prm.qN[tid]; }
    if (tid < 3) L.wr[tid] = prm.r[tid];
    if (prm.use_nlp && tid < K) L.sel[tid] = sel_g[(size_t)agent * K + tid];
    if (tid < 12) L.x0l[tid] = x0[tid];
    SYNC();
    for (int e = tid; e < 4 * N; e += 64) {              // one (grid, leg) per lane: W_l = Ts Iw^-1 [r]x
        const int k = e >> 2, l = e & 3;
        // (the linearisation point: x0 for grid 0, else the reference -- both in LDS: a pointer selecting between
        // global memory and LDS compiles to flat accesses, which this kernel avoids)
        const double *ph = (k == 0) ? L.x0l : L.xr + 12 * (k - 1);
        const double ph0 = ph[0], ph1 = ph[1], ph2 = ph[2];
        const double psi = ph[5], c = cos(psi), s = sin(psi);
        double R[9], T[9], Iw[9], Iwi[9];
        for (int a = 0; a < 3; a++) for (int b = 0; b < 3; b++) R[3 * a + b] = rzab(a, b, c, s);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) T[3 * i + j] = R[3 * i] * prm.Ib[j] + R[3 * i + 1] * prm.Ib[3 + j] + R[3 * i + 2] * prm.Ib[6 + j];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Iw[3 * i + j] = T[3 * i] * R[3 * j] + T[3 * i + 1] * R[3 * j + 1] + T[3 * i + 2] * R[3 * j + 2];
        {
            const double a = Iw[0], b = Iw[1], cc = Iw[2], d = Iw[3], ee = Iw[4], f = Iw[5], g = Iw[6], h = Iw[7], ii = Iw[8];
            const double A0 = ee * ii - f * h, B0 = -(d * ii - f * g), C0 = d * h - ee * g;
            const double r = 1.0 / (a * A0 + b * B0 + cc * C0);
            Iwi[0] = A0 * r; Iwi[1] = -(b * ii - cc * h) * r; Iwi[2] = (b * f - cc * ee) * r;
            Iwi[3] = B0 * r; Iwi[4] = (a * ii - cc * g) * r; Iwi[5] = -(a * f - cc * d) * r;
            Iwi[6] = C0 * r; Iwi[7] = -(a * h - b * g) * r; Iwi[8] = (a * ee - b * d) * r;
        }
        const double *fp = footg + (size_t)agent * 12 * N + 12 * k + 3 * l;
        const double r0 = fp[0] - ph0, r1 = fp[1] - ph1, r2 = fp[2] - ph2;
        const double S[9] = {0, -r2, r1, r2, 0, -r0, -r1, r0, 0};
        const double on = L.ct[4 * k + l];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                L.Wl[36 * k + 9 * l + 3 * i + j] = on * (Ts * (Iwi[3 * i] * S[j] + Iwi[3 * i + 1] * S[3 + j] + Iwi[3 * i + 2] * S[6 + j]));
        if (l == 0) { L.cs[2 * k] = c; L.cs[2 * k + 1] = s; }
    }
    if (prm.use_nlp) {                                   // obstacle rows: the LIP mode's selection and prediction
        for (int e = tid; e < NK; e += 64) {
            const int k = e / K, j = e - k * K;
            const bool st = j < prm.K_obs;
            const int bi = L.sel[j];
            const double tt = st ? 0.0 : Ts * (k + 1);
            const size_t bj = (bi >= 0) ? bi : 0;
            const double *src = st ? obstacles + 2 * bj : nbr_state + 4 * bj;
            L.obs[2 * e] = (bi >= 0) ? src[0] + (st ? 0.0 : src[2] * tt) : x0[0] + 1000.0;
            L.obs[2 * e + 1] = (bi >= 0) ? src[1] + (st ? 0.0 : src[3] * tt) : x0[1];
        }
        if (tid < K) L.eps[tid] = (tid < prm.K_obs) ? prm.eps_obs : prm.eps_nbr;
    }
    // start: gravity-compensating forces on the stance legs, the dynamics rolled out, s = 0
    for (int e = tid; e < 12 * N; e += 64) {
        const int k = e / 12, i = e - 12 * k, l = i / 3;
        int ns = 0;
        for (int q = 0; q < 4; q++) ns += contactg[(size_t)agent * 4 * N + 4 * k + q] != 0;
        U[e] = (i % 3 == 2 && ns && contactg[(size_t)agent * 4 * N + 4 * k + l]) ? prm.mass * prm.grav / ns : 0.0;
    }
    if (tid < 12) L.vv[tid] = x0[tid];
    if (tid == 0) L.Z[24 * N] = 0.0;                    // s
    SYNC();
#pragma clang loop unroll(disable)
    for (int k = 0; k < N; k++) {                        // x_{k+1} = A_k x_k + B_k u_k + c_k
        double v = 0.0;
        if (tid < 12) {
            v = a_mul(tid, L.vv, Ts, L.cs[2 * k], L.cs[2 * k + 1]) + b_mul(tid, U + 12 * k, L.Wl + 36 * k, L.ct + 4 * k, tsm);
            if (tid == 8) v -= Ts * prm.grav;
        }
        SYNC();
        if (tid < 12) { L.vv[tid] = v; X[12 * k + tid] = v; }
        SYNC();
    }

    // ---------------- row slots (registers).  Leg slot t of this lane: leg e = lane + 64 t (grid e / 4,
    // leg e % 4), its six friction rows q (global row 6 e + q, the oracle's stage-major order) when the
    // leg is in stance.  Obstacle slot t: row e = lane + 64 t (grid e / K, row e % K; global row
    // 24 N + e), NLP stage only.  s, z and the predictor's ds, dz (kept for the corrector).
    double ls[TL][6], lz[TL][6], lsa[TL][6], lza[TL][6];
    double os[TO], oz[TO], osa[TO], oza[TO];
    bool lon[TL], oon[TO];
    bool obs_on = false;                                  // the stage has obstacle rows (uniform)
    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
    const int nstage = prm.use_nlp ? 2 : 1;
    // obstacle row e at the current iterate: g, h and the Jacobian (c0, c1) on (p_x, p_y) (-1 on s)
    auto obs_row = [&](int e, double &g, double &h, double &c0, double &c1) {
        const int k = e / K, j = e - k * K;
        const double dx = X[12 * k] - L.obs[2 * e], dy = X[12 * k + 1] - L.obs[2 * e + 1];
        c0 = -2.0 * dx; c1 = -2.0 * dy;
        g = -(dx * dx + dy * dy) - L.Z[24 * N];
        h = -L.eps[j];
    };

    // ---------------- backward Riccati factor over the 13-state with the shift delta.  false when a
    // pivot (the inertia test) or the initial slack's Schur complement is not positive.  Reads the
    // per-grid blocks (Q3, Rh), writes K_k and Hu_k^-1 per grid, sets `schur`.
    double schur = 0.0;
    auto factor = [&](double delta) -> bool {
        int fail = 0;
        // this lane's entries (i = gi + 4 q, j = ci) of Q^, branch-free: masks and clamped LDS indices (a
        // diagonal weight, an obstacle-block entry Q3); R^ likewise (a leg-block entry Rh) in the stage loop
        auto qh = [&](int k, int q) {
            const int i = gi + 4 * q, j = ci;
            const bool dg = i == j && i < 12, ob = (i < 2 || i == 12) && (j < 2 || j == 12);
            const int a = (i == 12) ? 2 : (i < 2 ? i : 0), b = (j == 12) ? 2 : (j < 2 ? j : 0);
            const int lo = a < b ? a : b, hi = a < b ? b : a;
            const double wd = ((k == N - 1) ? L.wqN : L.wq)[i < 12 ? i : 0], qo = L.Q3[6 * k + (hi * (hi + 1)) / 2 + lo];
            // masks as factors: the loads stay unconditional (a select lets the compiler sink them into branches)
            return (dg ? 1.0 : 0.0) * (wd + delta) + (ob ? 1.0 : 0.0) * qo;
        };
        d4 Vd;                                            // V in the MFMA accumulator layout: V[gi + 4 q][ci]
#pragma unroll
        for (int q = 0; q < 4; q++) Vd[q] = qh(N - 1, q);
        // per-lane index pieces of the stage operands (qh, rh, bt above, split into the LDS reads -- one
        // batch, one round trip per stage -- and the masked arithmetic after them)
        int qoi[4], rbi[4], wqi[4], wri[4];
        double qdm[4], qom[4], rdm[4], rbm[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int i = gi + 4 * q, j = ci;
            {
                const bool dg = i == j && i < 12, ob = (i < 2 || i == 12) && (j < 2 || j == 12);
                const int a = (i == 12) ? 2 : (i < 2 ? i : 0), b = (j == 12) ? 2 : (j < 2 ? j : 0);
                const int lo = a < b ? a : b, hi = a < b ? b : a;
                wqi[q] = i < 12 ? i : 0; qoi[q] = (hi * (hi + 1)) / 2 + lo;
                qdm[q] = dg ? 1.0 : 0.0; qom[q] = ob ? 1.0 : 0.0;
            }
            {
                const bool in = i < 12 && j < 12, dg = in && i == j, bl = in && i / 3 == j / 3;
                const int i3 = in ? i % 3 : 0, j3 = in ? j % 3 : 0, l = in ? i / 3 : 0;
                wri[q] = i3; rbi[q] = 6 * l + sym3(i3, j3);
                rdm[q] = dg ? 1.0 : 0.0; rbm[q] = bl ? 1.0 : 0.0;
            }
        }
        const int bl_ = (ci < 12 ? ci : 0) / 3, ba_ = (ci < 12 ? ci : 0) - 3 * bl_;
        const int i1 = 4 + gi, i2 = 8 + gi;
        const bool bv1 = ci < 12 && i1 >= 6 && i1 < 9 && ba_ == i1 - 6, bv2 = ci < 12 && i2 >= 6 && i2 < 9 && ba_ == i2 - 6;
        const bool bw2 = ci < 12 && i2 >= 9 && i2 < 12;
        const int bwi = 9 * bl_ + 3 * (bw2 ? i2 - 9 : 0) + ba_;
#pragma clang loop unroll(disable)
        for (int k = N - 1; k >= 0; k--) {
            // the stage's LDS operands in one batch (Q^_{k-1}: k = 0 reads grid 0, masked below)
            __builtin_amdgcn_sched_barrier(0);
            const int km = k > 0 ? k - 1 : 0;
            const double c = L.cs[2 * k], s = L.cs[2 * k + 1];
            const double ctl = L.ct[4 * k + bl_], wl2 = L.Wl[36 * k + bwi];
            double qd[4], qo[4], rd[4], rb[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                qd[q] = L.wq[wqi[q]]; qo[q] = L.Q3[6 * km + qoi[q]];
                rd[q] = L.wr[wri[q]]; rb[q] = L.Rh[24 * k + rbi[q]];
            }
            __builtin_amdgcn_sched_barrier(0);
            // operand values: A~[4 kb + gi][ci] (B operand of A~, A operand of A~'), B~ likewise (rows
            // 4..11 only: kb = 1, 2)
            double Ab[4];
#pragma unroll
            for (int kb = 0; kb < 4; kb++) Ab[kb] = atil(4 * kb + gi, ci, Ts, c, s);
            const double Bb1 = (bv1 ? tsm : 0.0) * ctl;
            const double Bb2 = (bv2 ? tsm : 0.0) * ctl + (bw2 ? 1.0 : 0.0) * wl2;
            d4 G = {0.0, 0.0, 0.0, 0.0}, F = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kb = 0; kb < 4; kb++) G = mfma(Vd[kb], Ab[kb], G);           // G = V A~
            F = mfma(Vd[1], Bb1, F); F = mfma(Vd[2], Bb2, F);                      // F = V B~
            d4 Vn, Hu, Hux = {0.0, 0.0, 0.0, 0.0};
            const double mk = (k > 0) ? 1.0 : 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                Vn[q] = mk * (qdm[q] * (qd[q] + delta) + qom[q] * qo[q]);
                Hu[q] = rdm[q] * (rd[q] + delta) + rbm[q] * rb[q];
            }
#pragma unroll
            for (int kb = 0; kb < 4; kb++) Vn = mfma(Ab[kb], G[kb], Vn);          // Q^_{k-1} + A~'G
            Hux = mfma(Bb1, G[1], Hux); Hux = mfma(Bb2, G[2], Hux);                // B~'G (12 x 13)
            Hu = mfma(Bb1, F[1], Hu); Hu = mfma(Bb2, F[2], Hu);                    // R^ + B~'F
            S12ST(10);  // factor: operands and the products
            // to the column layout: Hu, Hux in T, 12 entries a column, row r at position 3 (r % 4) + r / 4 so
            // that the three rows gi + 4 q an MFMA-layout lane holds are adjacent (merged LDS accesses).
            // Stores are unconditional: lanes outside a block write to the sink entries T[300..323]
            const int sink = 300;
            {
                double *bh = L.T + (ci < 12 ? 12 * ci + 3 * gi : sink), *bx = L.T + (ci < 13 ? 144 + 12 * ci + 3 * gi : sink + 4);
#pragma unroll
                for (int q = 0; q < 3; q++) { bh[q] = Hu[q]; bx[q] = Hux[q]; }
            }
            SYNC();
            // lane j < 12: column j of Hu; 12..24: column j - 12 of Hux; 25..36: column j - 25 of I
            double col[12];
            {
                const double *src = (lane < 12) ? L.T + 12 * lane : L.T + 144 + 12 * (lane < 25 ? lane - 12 : 0);
                const double mc = (lane < 25) ? 1.0 : 0.0;
#pragma unroll
                for (int r = 0; r < 12; r++) col[r] = mc * src[3 * (r % 4) + r / 4] + ((lane - 25 == r) ? 1.0 : 0.0);
            }
            SYNC();
            S12ST(11);  // factor: to the column layout
            // Hu = L D L': forward elimination, row i -= (Hu[i][kk] / d_kk) row kk for i > kk, on every column.
            // Lane kk holds column kk, whose entries below the pivot are the multipliers (readlane)
            double dinv[12];
#pragma unroll
            for (int kk = 0; kk < 12; kk++) {
                const double piv = readlane_d(col[kk], kk);
                fail |= !(piv > 0.0);
                const double t = col[kk] * rcp_d(piv);
#pragma unroll
                for (int i = kk + 1; i < 12; i++) col[i] = fma(-readlane_d(col[i], kk), t, col[i]);
                // 1 / sqrt(piv): v_rsq_f64 and two Newton steps (a failed pivot's value is never used)
#ifdef SRB12_EXACT_RSQ                // diagnostic builds: the correctly rounded 1 / sqrt
#ifndef SRB_DIAG_BUILD
#error "SRB12_EXACT_RSQ is a diagnostic-build option"
#endif
                dinv[kk] = 1.0 / sqrt(piv);
#else
                double rs = __builtin_amdgcn_rsq(piv);
                rs = fma(0.5 * rs, fma(-piv * rs, rs, 1.0), rs);
                rs = fma(0.5 * rs, fma(-piv * rs, rs, 1.0), rs);
                dinv[kk] = rs;
#endif
            }
            // (Two pivots a step -- every broadcast of the step reading values from before it, the same fma
            // forms, bit-identical -- measured slower: SRB-12 step 0.756 -> 0.793 ms, round 5.)
            S12ST(12);  // factor: elimination
            // Y = D^-1/2 L^-1 Hux (lanes 12..24), Z = D^-1/2 L^-1 (lanes 25..36), back to T column-major
            {
                double *by = L.T + ((lane >= 12 && lane < 37) ? 12 * (lane - 12) : sink + 12);
#pragma unroll
                for (int r = 0; r < 12; r++) by[3 * (r % 4) + r / 4] = col[r] * dinv[r];
            }
            SYNC();
            // Y'Y (13 x 13), Hu^-1 = Z'Z (12 x 12), Z'Y = -K (12 x 13): operands Y[4 kb + gi][ci], Z[..][ci]
            // (rows 4 kb + gi at positions 3 gi + kb: adjacent)
            d4 YY = {0.0, 0.0, 0.0, 0.0}, ZZ = {0.0, 0.0, 0.0, 0.0}, ZY = {0.0, 0.0, 0.0, 0.0};
            {
                const double *py = L.T + 12 * (ci < 13 ? ci : 12) + 3 * gi, *pz = L.T + 156 + 12 * (ci < 12 ? ci : 11) + 3 * gi;
                const double my = (ci < 13) ? 1.0 : 0.0, mz = (ci < 12) ? 1.0 : 0.0;
#pragma unroll
                for (int kb = 0; kb < 3; kb++) {
                    const double ya = my * py[kb], za = mz * pz[kb];
                    YY = mfma(ya, ya, YY); ZZ = mfma(za, za, ZZ); ZY = mfma(za, ya, ZY);
                }
            }
            Vd = Vn - YY;                                  // V_{k-1} = Q^ + A~'G - Hux' Hu^-1 Hux
            double *Kk = L.Kst + 156 * k, *Hk = L.Hst + 78 * k;
#pragma unroll
            for (int q = 0; q < 3; q++) {
                const int i = gi + 4 * q;
                *(ci < 13 ? Kk + 13 * i + ci : L.T + sink) = -ZY[q];
                *(ci <= i ? Hk + tri(i, ci) : L.T + sink + 1) = ZZ[q];
            }
            SYNC();
            S12ST(13);  // factor: Y, Z, the Schur / gain / inverse products, stores
        }
        if (fail) return false;
        // the free initial slack closes the recursion: V_-1[12][12] + Sw + delta > 0 is the last
        // pivot of the inertia test (row 12 = gi 0, q 3; column 12 = lane 12)
        schur = readlane_d(Vd[3], 12) + prm.Sw + delta;
        return schur > 0.0;
    };

    // ---------------- Riccati solve of column c (rX / gX: 13 per grid, rU / gU: 12, sc[2 + c]: the s_0
    // entry) into dX (13 per grid), dU: w solves H w = -rhs on the dynamics' null space (x_0 fixed, s_0
    // free).  Component i = ci of every vector, replicated in the four rows; row gi takes columns
    // 4 gi .. 4 gi + 3 of each matrix-vector product (perm_d gathers them), rowsum adds the rows.
    [[maybe_unused]] int sph = 4;                         // stamps: the phase a solve's set-up counts to
    // A~_k applied to a replicated 13-vector, less the identity part over Ts, branch-free (a select chain
    // over DPP results compiles to exec-mask branches inside the stage loops):
    //   atv: (A~' v)[i] - v[i] = Ts (v[i-6] for i = 6, 7, 8, 11; the Rz' rows on v[3], v[4] for i = 9, 10)
    //   apv: (A~  v)[i] - v[i] = Ts (v[i+6] for i = 0, 1, 2, 5; the Rz rows on v[9], v[10] for i = 3, 4)
    // one row shift by six brings v[i -/+ 6] to lane i, a swap of the two rotation lanes brings the other
    // component; the per-lane coefficients (1 on a copy lane, cos on a rotation lane; +-sin on the swapped
    // component) are three lane constants per form
    const double m12 = (ci < 12) ? 1.0 : 0.0, m13 = (ci < 13) ? 1.0 : 0.0, mg0 = (gi == 0) ? 1.0 : 0.0;
    const double ea0 = (ci % 3 == 0) ? 1.0 : 0.0, ea1 = (ci % 3 == 1) ? 1.0 : 0.0, ea2 = (ci % 3 == 2) ? 1.0 : 0.0;
    const double tP = (ci >= 6 && ci < 12 && ci != 9 && ci != 10) ? 1.0 : 0.0, tQ = (ci == 9 || ci == 10) ? 1.0 : 0.0;
    const double tR = (ci == 9) ? -1.0 : (ci == 10) ? 1.0 : 0.0;
    const double aP = (ci < 6 && ci != 3 && ci != 4) ? 1.0 : 0.0, aQ = (ci == 3 || ci == 4) ? 1.0 : 0.0;
    const double aR = (ci == 3) ? 1.0 : (ci == 4) ? -1.0 : 0.0;
#ifndef SRB12_DPPSHIFT
#define SRB12_DPPSHIFT 1
#endif
#if !SRB12_DPPSHIFT
    const double e0 = ci == 0 ? 1.0 : 0.0, e1 = ci == 1 ? 1.0 : 0.0, e2 = ci == 2 ? 1.0 : 0.0, e3 = ci == 3 ? 1.0 : 0.0;
    const double e4 = ci == 4 ? 1.0 : 0.0, e5 = ci == 5 ? 1.0 : 0.0, e6 = ci == 6 ? 1.0 : 0.0, e7 = ci == 7 ? 1.0 : 0.0;
    const double e8 = ci == 8 ? 1.0 : 0.0, e9 = ci == 9 ? 1.0 : 0.0, e10 = ci == 10 ? 1.0 : 0.0, e11 = ci == 11 ? 1.0 : 0.0;
    auto atv = [&](double v, double cc, double sn) {
        const double v0 = bc16(v, 0), v1 = bc16(v, 1), v2 = bc16(v, 2), v3 = bc16(v, 3), v4 = bc16(v, 4), v5 = bc16(v, 5);
        const double sel = fma(e6, v0, fma(e7, v1, fma(e8, v2, e11 * v5)));
        const double c3 = fma(e9, cc, e10 * sn), c4 = fma(e10, cc, -(e9 * sn));
        return sel + fma(c3, v3, c4 * v4);
    };
    auto apv = [&](double p, double cc, double sn) {
        const double p6 = bc16(p, 6), p7 = bc16(p, 7), p8 = bc16(p, 8), p9 = bc16(p, 9), p10 = bc16(p, 10), p11 = bc16(p, 11);
        const double sel = fma(e0, p6, fma(e1, p7, fma(e2, p8, e5 * p11)));
        const double c9 = fma(e3, cc, -(e4 * sn)), c10 = fma(e3, sn, e4 * cc);
        return sel + fma(c9, p9, c10 * p10);
    };
#else
    auto atv = [&](double v, double cc, double sn) {
        const double s6 = dpp_d<0x116>(v);                // row_shr:6 -- lane i: v[i - 6]
        const double t = dpp_d<0xD8>(s6);                 // quad_perm [0,2,1,3] -- lanes 9, 10 swapped
        return fma(fma(tQ, cc, tP), s6, (tR * sn) * t);   // 9: cc v3 - sn v4, 10: cc v4 + sn v3
    };
    auto apv = [&](double p, double cc, double sn) {
        const double s6 = dpp_d<0x106>(p);                // row_shl:6 -- lane i: p[i + 6]
        const double t = dpp_d<0x141>(s6);                // row_half_mirror -- lanes 3, 4 swapped
        return fma(fma(aQ, cc, aP), s6, (aR * sn) * t);   // 3: cc p9 + sn p10, 4: cc p10 - sn p9
    };
#endif
    // the per-stage operands of the two sweeps, read in one batch at the top of the stage (one LDS round
    // trip; scheduling barriers keep the compiler from interleaving each read with its first use), so
    // the stage's dependent chain (broadcasts, ds_bpermute gathers, permlane sums) waits on no LDS read.
    // (A variant that loaded stage k - 1's operands during stage k, two stages a trip, measured slower,
    // 0.850 against 0.828 ms a step, and failed the GPU parity tests -- cause not found.)
    struct BwOps { double ct, ru, w0, w1, w2, cc, sn, rx, kk[4], hk[4]; };
    struct FwOps { double ct, kff, w0, w1, w2, cc, sn, kk[4]; };
    auto riccati_solve = [&](int c, bool acc) {
        S12ST(sph);
        const double *rX = c ? L.gX : L.rX, *rU = c ? L.gU : L.rU;
        double *sink = L.T + 300 + ci;                      // stores of lanes outside a vector (T is free here)
        const int i = ci, g = gi, ir = (i < 12) ? i : 0, l = ir / 3, a = ir - 3 * l, i13 = (i < 13) ? i : 12;
        const int gsrc = 16 * g + 4 * g;                   // lane holding component 4 g (this row's copy)
        // (lanes i >= 13 read clamped entries: their K'gu and -Hu^-1 gu never leave the lane -- v is
        // masked, kff goes to the sink -- and the row sums stay within one component i)
        auto bw_load = [&](int k) {
            BwOps o;
            __builtin_amdgcn_sched_barrier(0);
            const double *W = L.Wl + 36 * k;
            o.ct = L.ct[4 * k + l]; o.ru = rU[12 * k + ir];
            o.w0 = W[9 * l + a]; o.w1 = W[9 * l + 3 + a]; o.w2 = W[9 * l + 6 + a];
            o.cc = L.cs[2 * k]; o.sn = L.cs[2 * k + 1];
            o.rx = rX[13 * (k > 0 ? k - 1 : 0) + i13];
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int j = 4 * g + m, jc = (j < 12) ? j : 11;
                o.kk[m] = L.Kst[156 * k + 13 * jc + i13];
                o.hk[m] = L.Hst[78 * k + tri(ir, jc)];
            }
            __builtin_amdgcn_sched_barrier(0);
            return o;
        };
        double v = (ci < 13) ? rX[13 * (N - 1) + ci] : 0.0;
        // backward stage k: gu = rhs_u + B~'v, kff = -Hu^-1 gu, v_{k-1} = rhs_x(k-1) + A~'v + K'gu
        auto bw_stage = [&](int k, const BwOps &o) {
            const double v6 = bc16(v, 6), v7 = bc16(v, 7), v8 = bc16(v, 8), v9 = bc16(v, 9), v10 = bc16(v, 10), v11 = bc16(v, 11);
            double gu = fma(o.ct * tsm, fma(ea0, v6, fma(ea1, v7, ea2 * v8)), o.ru);
            gu = fma(o.w0, v9, gu); gu = fma(o.w1, v10, gu); gu = fma(o.w2, v11, gu);
            // K'gu (state i) and -Hu^-1 gu (input i): this row's four input columns j = 4 g + m
            // (the gathers are issued together, one LDS round trip: the barrier keeps the scheduler from
            // interleaving each with its use)
            double gr[4];
#pragma unroll
            for (int m = 0; m < 4; m++) gr[m] = perm_d(gu, gsrc + m);
            __builtin_amdgcn_sched_barrier(0);
            double pk = 0.0, ph = 0.0;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const double gj = gr[m] * ((4 * g + m < 12) ? 1.0 : 0.0);
                pk = fma(o.kk[m], gj, pk);
                ph = fma(o.hk[m], gj, ph);
            }
            rowsum2(pk, ph);
            *((g == 0 && i < 12) ? L.kff + 12 * k + i : sink) = -ph;
            v = m13 * (fma(Ts, atv(v, o.cc, o.sn), v + pk) + (k > 0 ? 1.0 : 0.0) * o.rx);
        };
#pragma clang loop unroll(disable)
        for (int k = N - 1; k >= 0; k--) bw_stage(k, bw_load(k));
        const double ds0 = -(bc16(v, 12) + L.sc[2 + c]) / schur;
        SYNC();                                            // kff
        S12ST(14);  // solve: backward sweep
        const int lsrc = 16 * g + 3 * g, i9 = (i >= 9 && i < 12) ? i - 9 : 0;   // lane of leg g's first force
        const double mv = (i >= 6 && i < 9) ? 1.0 : 0.0, mw = (i >= 9 && i < 12) ? 1.0 : 0.0;
        auto fw_load = [&](int k) {
            FwOps o;
            __builtin_amdgcn_sched_barrier(0);
            const double *w = L.Wl + 36 * k + 9 * g + 3 * i9;
            o.ct = L.ct[4 * k + g]; o.kff = L.kff[12 * k + ir];
            o.w0 = w[0]; o.w1 = w[1]; o.w2 = w[2];
            o.cc = L.cs[2 * k]; o.sn = L.cs[2 * k + 1];
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int j = 4 * g + m, jc = (j < 13) ? j : 12;
                o.kk[m] = L.Kst[156 * k + 13 * ir + jc];
            }
            __builtin_amdgcn_sched_barrier(0);
            return o;
        };
        double prev = (ci == 12) ? ds0 : 0.0;
        // forward stage k: du = kff + K dx, dx_{k+1} = A~ dx + B~ du (row g adds leg g's forces, row 0
        // the A~ part)
        auto fw_stage = [&](int k, const FwOps &f) {
            double *pu = (g == 0 && i < 12) ? L.dU + 12 * k + i : sink;
            double *px = (g == 0 && i < 13) ? L.dX + 13 * k + i : sink;
            const double pu0 = acc ? *pu : 0.0, px0 = acc ? *px : 0.0;
            double gr[4];
#pragma unroll
            for (int m = 0; m < 4; m++) gr[m] = perm_d(prev, gsrc + m);
            __builtin_amdgcn_sched_barrier(0);
            double pk = 0.0;
#pragma unroll
            for (int m = 0; m < 4; m++) pk = fma(f.kk[m], gr[m] * ((4 * g + m < 13) ? 1.0 : 0.0), pk);
            const double du = m12 * (rowsum(pk) + f.kff);
            *pu = acc ? pu0 + du : du;
            const double d0 = perm_d(du, lsrc), d1 = perm_d(du, lsrc + 1), d2 = perm_d(du, lsrc + 2);
            __builtin_amdgcn_sched_barrier(0);
            const double bv = f.ct * tsm * fma(ea0, d0, fma(ea1, d1, ea2 * d2)), bw = fma(f.w0, d0, fma(f.w1, d1, f.w2 * d2));
            double pb = fma(mv, bv, mw * bw);
            pb = fma(mg0, fma(Ts, apv(prev, f.cc, f.sn), prev), pb);
            const double dx = m13 * rowsum(pb);
            *px = acc ? px0 + dx : dx;
            prev = dx;
        };
#pragma clang loop unroll(disable)
        for (int k = 0; k < N; k++) fw_stage(k, fw_load(k));
        SYNC();
        S12ST(15);  // solve: forward sweep
    };
    // one step of iterative refinement of column 0 (correction in column 1): the residual of H w = -rhs
    // on the null space is the reduced gradient -- t_u = R^ du + rhs_u + B' mu, t_s = (Sw + delta) ds_0 +
    // rhs_s + mu_0[12], costates mu from the state rows -- and the correction solves with (0, t_u, t_s)
    auto refine = [&](double delta) {
        const double *rX = L.rX, *rU = L.rU, *dX = L.dX, *dU = L.dU;
        double *tX = L.gX, *tU = L.gU;
        double *sink = L.T + 300 + ci;
        auto qdx = [&](int k, const double *dx, int i) {   // (Q^_k dx)[i], branch-free
            const double wd = ((k == N - 1) ? L.wqN : L.wq)[i < 12 ? i : 0];
            const bool ob = i < 2 || i == 12;
            const int a = (i == 12) ? 2 : (i < 2 ? i : 0);
            const double *q3 = L.Q3 + 6 * k;               // symmetric (p_x, p_y, s) block, packed lower triangle
            const double b0 = q3[tri(a, 0)], b1 = q3[tri(a, 1)], b2 = q3[tri(a, 2)];
            return (i < 12 ? 1.0 : 0.0) * (wd + delta) * dx[i < 13 ? i : 0] +
                   (ob ? 1.0 : 0.0) * fma(b0, dx[0], fma(b1, dx[1], b2 * dx[12]));
        };
        for (int e = tid; e < 13 * N; e += 64) tX[e] = 0.0;
        double m = (ci < 13) ? qdx(N - 1, dX + 13 * (N - 1), ci) + rX[13 * (N - 1) + ci] : 0.0;
        const int i = ci, ir = (i < 12) ? i : 0, l = ir / 3, a3 = ir - 3 * l, i13 = (i < 13) ? i : 12;
        const int qa = (i == 12) ? 2 : (i < 2 ? i : 0);
        const double mob = (i < 2 || i == 12) ? 1.0 : 0.0;
#pragma clang loop unroll(disable)
        for (int k = N - 1; k >= 0; k--) {
            // the stage's LDS operands in one batch (one round trip); Q^_{k-1} dx_{k-1}: k = 0 reads grid 0
            __builtin_amdgcn_sched_barrier(0);
            const int km = k > 0 ? k - 1 : 0;
            const double *W = L.Wl + 36 * k + 9 * l + a3, *du = dU + 12 * k + 3 * l, *rh = L.Rh + 24 * k + 6 * l;
            const double du0 = du[0], du1 = du[1], du2 = du[2], dua = dU[12 * k + ir];
            const double rh0 = rh[sym3(a3, 0)], rh1 = rh[sym3(a3, 1)], rh2 = rh[sym3(a3, 2)];
            const double ru = rU[12 * k + ir], ctl = L.ct[4 * k + l], wr = L.wr[a3];
            const double w0 = W[0], w1 = W[3], w2 = W[6], cc = L.cs[2 * k], sn = L.cs[2 * k + 1];
            const double *q3 = L.Q3 + 6 * km, *dx = dX + 13 * km;
            const double wd = L.wq[ir], b0 = q3[tri(qa, 0)], b1 = q3[tri(qa, 1)], b2 = q3[tri(qa, 2)];
            const double dxi = dx[i13], dx0 = dx[0], dx1 = dx[1], dx12 = dx[12], rxn = rX[13 * km + i13];
            __builtin_amdgcn_sched_barrier(0);
            const double v6 = bc16(m, 6), v7 = bc16(m, 7), v8 = bc16(m, 8), v9 = bc16(m, 9), v10 = bc16(m, 10), v11 = bc16(m, 11);
            double t = fma(wr + delta, dua, ru);
            t = fma(rh0, du0, t); t = fma(rh1, du1, t); t = fma(rh2, du2, t);
            t = fma(ctl * tsm, fma(ea0, v6, fma(ea1, v7, ea2 * v8)), t);
            t = fma(w0, v9, t); t = fma(w1, v10, t); t = fma(w2, v11, t);
            *((lane < 12) ? tU + 12 * k + i : sink) = t;
            // m_{k-1} = rhs_x(k-1) + Q^_{k-1} dx_{k-1} + A~'m (k = 0: m_0 stays)
            const double qd = m12 * (wd + delta) * dxi + mob * fma(b0, dx0, fma(b1, dx1, b2 * dx12));
            const double mn = m13 * (fma(Ts, atv(m, cc, sn), m) + qd + rxn);
            m = (k > 0) ? mn : m;
        }
        const double ms = bc16(m, 12);
        if (tid == 0) L.sc[3] = fma(prm.Sw + delta, dX[12], L.sc[2]) + ms;
        SYNC();
        riccati_solve(1, true);
    };

    // ---------------- the rows: gradient of f and J'z into column 1, the Hessian blocks (leg blocks Rh
    // written by their lanes, obstacle blocks Q3 by atomics), residual sums.  y(row): the multiplier
    // (z, or the polish's z_A + RHO c_A); w(row): the Hessian weight (z / s, or RHO / 0)
    auto grad_f = [&](double *gx, double *gu) {
        for (int e = tid; e < 12 * N; e += 64) {
            const int k = e / 12, i = e - 12 * k;
            const double w = (k == N - 1) ? L.wqN[i] : L.wq[i];
            gx[13 * k + i] = w * (X[e] - L.xr[e]);
            gu[e] = L.wr[i % 3] * U[e];
        }
        for (int k = tid; k < N; k += 64) gx[13 * k + 12] = 0.0;
    };
    // max_k |x_{k+1} - A_k x_k - B_k u_k - c_k| at the iterate (x_0 given): the dynamics every returned
    // point must satisfy (dec_vars_constr_cost.h:154-206 in the LIP mode); the polish's acceptance tests it
    auto dyn_res = [&]() -> double {
        double r = 0.0;
        for (int e = tid; e < 12 * N; e += 64) {
            const int k = e / 12, i = e - 12 * k;
            const double *xp = (k == 0) ? L.x0l : X + 12 * (k - 1);        // LDS only (no flat access)
            double v = a_mul(i, xp, Ts, L.cs[2 * k], L.cs[2 * k + 1]) + b_mul(i, U + 12 * k, L.Wl + 36 * k, L.ct + 4 * k, tsm);
            if (i == 8) v -= Ts * prm.grav;
            r = fmax(r, fabs(X[e] - v));
        }
        return wmax(r);
    };
#ifdef SRB12_CHECK
    // diagnostic build (make s12chk): state checks of the traced agent into prm.dbg[SRB12_DBG_CHECK + slot]
    const bool dchk = agent == prm.dbg_agent && prm.dbg != nullptr;
    auto lds_sum = [&](const double *p, int n) {
        double a = 0.0;
        for (int v = tid; v < n; v += 64) a += fabs(p[v]);
        return wsum(a);
    };
    // the solve's consistency: max_k |dx_{k+1} - A~ dx_k - B~ du_k| (dx_0 = 0 but its slack)
    auto sol_res = [&]() -> double {
        double r = 0.0;
        for (int e = tid; e < 12 * N; e += 64) {
            const int k = e / 12, i = e - 12 * k;
            double v = b_mul(i, L.dU + 12 * k, L.Wl + 36 * k, L.ct + 4 * k, tsm);
            if (k > 0) v += a_mul(i, L.dX + 13 * (k - 1), Ts, L.cs[2 * k], L.cs[2 * k + 1]);
            r = fmax(r, fabs(L.dX[13 * k + i] - v));
        }
        return wmax(r);
    };
#define S12CK(slot, expr) do { const double v_ = (expr); if (dchk && tid == 0) prm.dbg[SRB12_DBG_CHECK + (slot)] = v_; } while (0)
// per Newton step (the first 5 steps of the first 2 passes: slots 8..87) and per pass (the first 4: 88..119)
#define S12CKP(k, expr) do { if (pass < 2 && pit < 5) S12CK((k) + 40 * pass + 8 * pit, expr); } while (0)
#define S12CKA(k, expr) do { if (pass < 4) S12CK(88 + 8 * pass + (k), expr); } while (0)
#else
#define S12CK(slot, expr) do { } while (0)
#define S12CKP(k, expr) do { } while (0)
#define S12CKA(k, expr) do { } while (0)
#endif
    // right-hand side of pass (0 predictor, 1 corrector) into column 0:
    // rhs = grad f + sum_rows J'(z + r3 / s + W r_p), r3 = -s z (+ sigma mu - ds_a dz_a)
    auto build_rhs = [&](int pass, double smu) {
        grad_f(L.rX, L.rU);
        if (tid == 0) L.sc[2] = prm.Sw * L.Z[24 * N];
        SYNC();
        // (branch-free: a row that is not active contributes w = 0 through its mask, at a clamped index)
#pragma unroll
        for (int t = 0; t < TL; t++) {
            const int e = lane + 64 * t, ec = e < NL ? e : 0;
            const double mo = lon[t] ? 1.0 : 0.0;
            const double *u = U + 3 * ec;
            double r[3] = {0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 6; q++) {
                double c0, c1, c2;
                fric_coef(q, mus, c0, c1, c2);
                const double g = c0 * u[0] + c1 * u[1] + c2 * u[2], h = (q == 5) ? prm.fmax : 0.0;
                const double s = ls[t][q], z = lz[t][q], is = rcp_d(s);
                const double rp = g + s - h, om = z * is;
                const double r3 = -s * z + (pass ? smu - lsa[t][q] * lza[t][q] : 0.0);
                const double w = mo * (z + r3 * is + om * rp);
                r[0] = fma(w, c0, r[0]); r[1] = fma(w, c1, r[1]); r[2] = fma(w, c2, r[2]);
            }
            double *ru = (e < NL) ? L.rU + 3 * e : L.T + 300 + 4 * (lane & 3);   // (a lane past the legs: the sink,
            ru[0] += r[0]; ru[1] += r[1]; ru[2] += r[2];                           //  never row 0's entries: a plain RMW)
        }
        if (obs_on)
#pragma unroll
        for (int t = 0; t < TO; t++) {
            const int e = lane + 64 * t, ec = oon[t] ? e : 0;
            const double mo = oon[t] ? 1.0 : 0.0;
            double g, h, c0, c1;
            obs_row(ec, g, h, c0, c1);
            const double s = os[t], z = oz[t], is = rcp_d(s);
            const double rp = g + s - h, om = z * is;
            const double r3 = -s * z + (pass ? smu - osa[t] * oza[t] : 0.0);
            const double w = mo * (z + r3 * is + om * rp);
            double *rx = L.rX + 13 * (ec / K);
            __hip_atomic_fetch_add(&rx[0], w * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&rx[1], w * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&rx[12], -w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        SYNC();
    };
    // the rows' steps of the solved column: J dw, ds = -r_p - J dw, dz = (r3 - z ds) / s; step maxima
    auto row_step = [&](int pass, double smu, double (&dls)[TL][6], double (&dlz)[TL][6], double (&dos)[TO],
                        double (&doz)[TO]) {
        double ms = 0.0, mz = 0.0;
#pragma unroll
        for (int t = 0; t < TL; t++) {
            const int e = lane + 64 * t, ec = e < NL ? e : 0;
            const double mo = lon[t] ? 1.0 : 0.0;
            const double *u = U + 3 * ec, *du = L.dU + 3 * ec;
#pragma unroll
            for (int q = 0; q < 6; q++) {
                double c0, c1, c2;
                fric_coef(q, mus, c0, c1, c2);
                const double g = c0 * u[0] + c1 * u[1] + c2 * u[2], h = (q == 5) ? prm.fmax : 0.0;
                const double jd = c0 * du[0] + c1 * du[1] + c2 * du[2];
                const double s = ls[t][q], z = lz[t][q];
                const double rp = g + s - h;
                const double r3 = -s * z + (pass ? smu - lsa[t][q] * lza[t][q] : 0.0);
                const double is = rcp_d(s);
                dls[t][q] = mo * (-rp - jd); dlz[t][q] = mo * (r3 - z * dls[t][q]) * is;
                ms = fmax(ms, -dls[t][q] * is); mz = fmax(mz, -dlz[t][q] * rcp_d(z + (1.0 - mo)));
            }
        }
#pragma unroll
        for (int t = 0; t < TO; t++) {
            dos[t] = doz[t] = 0.0;
            if (!obs_on) continue;
            const int e = lane + 64 * t, ec = oon[t] ? e : 0;
            const double mo = oon[t] ? 1.0 : 0.0;
            double g, h, c0, c1;
            obs_row(ec, g, h, c0, c1);
            const double *dx = L.dX + 13 * (ec / K);
            const double jd = c0 * dx[0] + c1 * dx[1] - dx[12];
            const double s = os[t], z = oz[t];
            const double rp = g + s - h;
            const double r3 = -s * z + (pass ? smu - osa[t] * oza[t] : 0.0);
            const double is = rcp_d(s);
            dos[t] = mo * (-rp - jd); doz[t] = mo * (r3 - z * dos[t]) * is;
            ms = fmax(ms, -dos[t] * is); mz = fmax(mz, -doz[t] * rcp_d(z + (1.0 - mo)));
        }
        double rv[2] = {ms, mz};
        wred<2, 3u>(rv);
        return make_double2(rv[0] > 0.0 ? 1.0 / rv[0] : 1.0, rv[1] > 0.0 ? 1.0 / rv[1] : 1.0);
    };

    S12ST(0);   // inputs, model, rollout
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        const bool nl = stage == 1;
        obs_on = nl && NK > 0;
        // active rows and the starting slacks / duals (oracle ipm(): QP s = h - g, z = 1 / max(s, 1);
        // NLP shifted so min s = 1 when a row is violated, z = z0 / max(s, 1))
        double mcount = 0.0, mn = 1e300;
#pragma unroll
        for (int t = 0; t < TL; t++) {
            const int e = lane + 64 * t;
            lon[t] = e < NL && L.ct[e] != 0.0;
            const double *u = U + 3 * (lon[t] ? e : 0);
#pragma unroll
            for (int q = 0; q < 6; q++) {
                double c0, c1, c2;
                fric_coef(q, mus, c0, c1, c2);
                ls[t][q] = ((q == 5) ? prm.fmax : 0.0) - (c0 * u[0] + c1 * u[1] + c2 * u[2]);
                if (lon[t]) { mcount += 1.0; mn = fmin(mn, ls[t][q]); }
            }
        }
#pragma unroll
        for (int t = 0; t < TO; t++) {
            const int e = lane + 64 * t;
            oon[t] = nl && e < NK;
            double g = 0.0, h = 0.0, c0, c1;
            if (oon[t]) obs_row(e, g, h, c0, c1);
            os[t] = h - g;
            if (oon[t]) { mcount += 1.0; mn = fmin(mn, h - g); }
        }
        {
            double rv[2] = {mcount, -mn};
            wred<2, 2u>(rv);
            mcount = rv[0]; mn = -rv[1];
        }
        const double ssh = (nl && mn <= 0.0) ? 1.0 - mn : 0.0, zs = nl ? prm.z0 : 1.0;
#pragma unroll
        for (int t = 0; t < TL; t++)
#pragma unroll
            for (int q = 0; q < 6; q++) {
                double s = ls[t][q] + ssh;
                if (!nl && s < 1e-8) s = 1e-8;
                ls[t][q] = lon[t] ? s : 1.0;
                lz[t][q] = lon[t] ? zs / fmax(s, 1.0) : 0.0;
                lsa[t][q] = lza[t][q] = 0.0;
            }
#pragma unroll
        for (int t = 0; t < TO; t++) {
            double s = os[t] + ssh;
            os[t] = oon[t] ? s : 1.0;
            oz[t] = oon[t] ? zs / fmax(s, 1.0) : 0.0;
            osa[t] = oza[t] = 0.0;
        }
        const double inv_m = 1.0 / fmax(mcount, 1.0);
        const int maxit = nl ? prm.nlp_maxit : prm.qp_maxit;
        // a QP stage that the NLP follows runs to tol_qp (the NLP's warm start only); the last stage's
        // complementarity test is tol_final (the forces' accuracy: DESIGN.md 11); oracle/srb12.c the same
        const double tol_s = (!nl && prm.use_nlp && prm.tol_qp > 0.0) ? prm.tol_qp : tol, th_s = tol_s / sqrt(3.0);
        const double mtol = (stage == nstage - 1) ? prm.tol_final : tol_s;
        int flag = 2, it = 0;
        double sigma = 0.0;
#pragma clang loop unroll(disable)
        for (it = 0; it < maxit; it++) {
            // ---- gradient of f (X, U; Sw s of the slack at s_0), cleared obstacle blocks
            grad_f(L.gX, L.gU);
            for (int e = tid; e < 6 * N; e += 64) L.Q3[e] = 0.0;
            if (tid == 0) { L.sc[0] = prm.Sw * L.Z[24 * N]; L.sc[1] = prm.Sw; }    // grad_s f, H_ss (inertia scale)
            SYNC();
            S12ST(3);   // (stamps: the gradient; slot 3 also takes the factor -> predictor gap)
            // ---- rows: residuals, weights, J'z and J'WJ into the per-grid blocks
            double nrp = 0.0, sz = 0.0, zmx = 0.0;
#pragma unroll
            for (int t = 0; t < TL; t++) {
                // branch-free: a leg out of range or in swing has z = 0 (rh, gz vanish) and a masked r_p;
                // its stores go to the sink
                const int e = lane + 64 * t, ec = e < NL ? e : 0;
                const double mo = lon[t] ? 1.0 : 0.0;
                double gz[3] = {0.0, 0.0, 0.0}, rh[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                const double *u = U + 3 * ec;
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    double c0, c1, c2;
                    fric_coef(q, mus, c0, c1, c2);
                    const double g = c0 * u[0] + c1 * u[1] + c2 * u[2], h = (q == 5) ? prm.fmax : 0.0;
                    const double s = ls[t][q], z = mo * lz[t][q];
                    const double rp = mo * (g + s - h), om = z * rcp_d(s);
                    nrp = fma(rp, rp, nrp); sz = fma(s, z, sz); zmx = fmax(zmx, z);
                    const double cc[3] = {c0, c1, c2};
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        gz[a] = fma(z, cc[a], gz[a]);
#pragma unroll
                        for (int b = a; b < 3; b++) rh[sym3(a, b)] = fma(om * cc[a], cc[b], rh[sym3(a, b)]);
                    }
                }
                double *gu = (e < NL) ? L.gU + 3 * e : L.T + 300 + 4 * (lane & 3);
                gu[0] += gz[0]; gu[1] += gz[1]; gu[2] += gz[2];
                double *rhp = (e < NL) ? L.Rh + 6 * e : L.T + 300;
#pragma unroll
                for (int m = 0; m < 6; m++) rhp[m] = rh[m];
            }
            if (obs_on) {
            // (the slack's curvature sum H_ss += om goes through a wave sum: an LDS atomic to one address
            // from every lane compiles to a 64-step scalar loop)
            double oms = 0.0;
#pragma unroll
            for (int t = 0; t < TO; t++) {
                // branch-free: a lane past the last row adds zeros to row 0's grid
                const int e = lane + 64 * t, ec = oon[t] ? e : 0;
                const double mo = oon[t] ? 1.0 : 0.0;
                double g, h, c0, c1;
                obs_row(ec, g, h, c0, c1);
                const double s = os[t], z = mo * oz[t];
                const double rp = mo * (g + s - h), om = z * rcp_d(s);
                nrp = fma(rp, rp, nrp); sz = fma(s, z, sz); zmx = fmax(zmx, z);
                // obstacle row of grid k on (p_x, p_y, s): J = (c0, c1, -1), Lagrangian Hessian -2z on p_x, p_y
                const int k = ec / K;
                double *gx = L.gX + 13 * k, *q3 = L.Q3 + 6 * k;
                __hip_atomic_fetch_add(&gx[0], z * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&gx[1], z * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&gx[12], -z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[0], fma(om * c0, c0, -2.0 * z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[1], om * c0 * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[2], fma(om * c1, c1, -2.0 * z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[3], -om * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[4], -om * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&q3[5], om, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                oms += om;
            }
            oms = wsum(oms);
            if (tid == 0) L.sc[1] += oms;
            }
            SYNC();
            S12ST(8);   // (stamps: the rows; slot 8 also takes the exit test -> polish gap)
            // ---- costates and the dual residual (13-state: the slack rides along as x[12], s_{k+1} = s_k):
            //      lam_{N-1} = gX_{N-1}, lam_{k-1} = gX_{k-1} + A~_k' lam_k, r_u,k = gU_k + B_k' lam_k,
            //      r_s = Sw s + lam_0[12] (the free initial slack)
            double nrd = 0.0, gm = 1.0;
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                const double w = (k == N - 1) ? L.wqN[i] : L.wq[i];
                gm = fmax(gm, fabs(w * (X[e] - L.xr[e])));
                gm = fmax(gm, fabs(L.wr[i % 3] * U[e]));
            }
            gm = fmax(gm, fabs(prm.Sw * L.Z[24 * N]));
            {
                // (the operands of stage k in one batch of LDS reads, as in the solves)
                const int i = ci, ir = (i < 12) ? i : 0, l = ir / 3, jj = ir - 3 * l, i13 = (i < 13) ? i : 12;
                struct CsOps { double ct, gu, w0, w1, w2, cc, sn, gx; };
                auto cs_load = [&](int k) {
                    CsOps o;
                    __builtin_amdgcn_sched_barrier(0);
                    const double *W = L.Wl + 36 * k + 9 * l + jj;
                    o.ct = L.ct[4 * k + l]; o.gu = L.gU[12 * k + ir];
                    o.w0 = W[0]; o.w1 = W[3]; o.w2 = W[6];
                    o.cc = L.cs[2 * k]; o.sn = L.cs[2 * k + 1];
                    o.gx = L.gX[13 * (k > 0 ? k - 1 : 0) + i13];
                    __builtin_amdgcn_sched_barrier(0);
                    return o;
                };
                double lam = (i < 13) ? L.gX[13 * (N - 1) + i] : 0.0;
                auto cs_stage = [&](int k, const CsOps &o) {
                    const double v6 = bc16(lam, 6), v7 = bc16(lam, 7), v8 = bc16(lam, 8);
                    const double v9 = bc16(lam, 9), v10 = bc16(lam, 10), v11 = bc16(lam, 11);
                    double ru = fma(o.ct * tsm, fma(ea0, v6, fma(ea1, v7, ea2 * v8)), o.gu);
                    ru = fma(o.w0, v9, ru); ru = fma(o.w1, v10, ru); ru = fma(o.w2, v11, ru);
                    ru *= m12 * mg0;                         // one row of the four copies
                    nrd = fma(ru, ru, nrd);
                    // lam_{k-1} (k = 0: lam_0 stays, its slack entry closes r_s)
                    const double ln = m13 * (fma(Ts, atv(lam, o.cc, o.sn), lam) + o.gx);
                    lam = (k > 0) ? ln : lam;
                };
#pragma clang loop unroll(disable)
                for (int k = N - 1; k >= 0; k--) cs_stage(k, cs_load(k));
                const double l12 = bc16(lam, 12);
                if (tid == 0) { const double rs = L.sc[0] + l12; nrd = fma(rs, rs, nrd); }
            }
            {
                double rv[5] = {nrd, nrp, sz, gm, zmx};
                wred<5, 24u>(rv);
                nrd = sqrt(rv[0]); nrp = sqrt(rv[1]); sz = rv[2]; gm = rv[3]; zmx = rv[4];
            }
            const double mu = sz * inv_m;
            double *dbgrow = (agent == prm.dbg_agent && prm.dbg && it < 64) ? prm.dbg + 8 * (64 * stage + it) : nullptr;
            if (dbgrow && tid == 0) { dbgrow[0] = nrd; dbgrow[1] = th_s * gm; dbgrow[2] = nrp; dbgrow[3] = mu; }
            // divergence (the LIP mode's rule, SRB_Z_DIV; oracle/srb12.c the same): a dual beyond 1e10 means
            // infeasible rows -- FATAL at this finite iterate
            if (!isfinite(nrd) || !isfinite(nrp) || !isfinite(sz) || !(zmx <= SRB_Z_DIV)) { flag = 3; break; }
            S12ST(1);   // residuals, weights, scatter, costates
            if (nrd < th_s * gm && nrp < th_s && mu < mtol) { flag = 0; break; }

            // ---- factorisation (backward Riccati over the 13-state) with the inertia shift delta (NLP)
            double dmax = 1.0;
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                const double qd = ((k == N - 1) ? L.wqN[i] : L.wq[i]) + (i < 2 ? L.Q3[6 * k + 2 * i] : 0.0);
                const int l = i / 3, a = i % 3;
                const double rd = L.wr[a] + L.Rh[24 * k + 6 * l + sym3(a, a)];
                dmax = fmax(dmax, fmax(qd, rd));
            }
            dmax = wmax(dmax);
            dmax = fmax(dmax, L.sc[1]);
            const double dstart = 1e-10 * dmax;
            double delta = 0.0;
            int ok = 0;
            for (int tries = 0; tries < (nl ? 14 : 1); tries++) {
                if (tries > 0) delta = (delta == 0.0) ? dstart : delta * 10.0;
                if (factor(delta)) { ok = 1; break; }
            }
            S12ST(2);   // Riccati factor (all tries)
            if (!ok) { flag = 1; break; }
            S12ST(3);   // between factor and predictor
            // ---- predictor
            // (the refinement only near the optimum, mu < 1e-3, and only of the corrector: far from the
            // optimum the step's accuracy is not what limits progress, and the predictor only sets sigma
            // and the second-order term; each refinement costs a solve)
            const bool refn = mu < SRB12_REFINE_MU;
            sph = 4;
            build_rhs(0, 0.0);
            riccati_solve(0, false);
#if SRB12_REFINE_PREDICTOR
            if (refn) refine(delta);
#endif
            S12ST(4);   // predictor rhs + solve (+ refinement)
            double dls[TL][6], dlz[TL][6], dos[TO], doz[TO];
            double2 al = row_step(0, 0.0, dls, dlz, dos, doz);
#pragma unroll
            for (int t = 0; t < TL; t++)
#pragma unroll
                for (int q = 0; q < 6; q++) { lsa[t][q] = dls[t][q]; lza[t][q] = dlz[t][q]; }
#pragma unroll
            for (int t = 0; t < TO; t++) { osa[t] = dos[t]; oza[t] = doz[t]; }
            {
                double num = 0.0;
#pragma unroll
                for (int t = 0; t < TL; t++)
                    if (lon[t])
#pragma unroll
                        for (int q = 0; q < 6; q++) num = fma(fma(al.x, lsa[t][q], ls[t][q]), fma(al.y, lza[t][q], lz[t][q]), num);
#pragma unroll
                for (int t = 0; t < TO; t++)
                    if (oon[t]) num = fma(fma(al.x, osa[t], os[t]), fma(al.y, oza[t], oz[t]), num);
                num = wsum(num);
                const double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
                sigma = mr * mr * mr;
            }
            S12ST(5);   // predictor row step, sigma
            // ---- corrector
            sph = 6;
            build_rhs(1, sigma * mu);
            riccati_solve(0, false);
            if (SRB12_REFINE && refn) refine(delta);
            if (SRB12_REFINE2_MU > 0.0 && mu < SRB12_REFINE2_MU) refine(delta);
            S12ST(6);   // corrector rhs + solve (+ refinement)
            al = row_step(1, sigma * mu, dls, dlz, dos, doz);
            const double ap = fmin(1.0, 0.99 * al.x), ad = fmin(1.0, 0.99 * al.y);
            if (dbgrow && tid == 0) { dbgrow[4] = ap; dbgrow[5] = ad; dbgrow[6] = delta; dbgrow[7] = sigma; }
            // ---- update: x += ap dx (the slack: ds_0, carried in every grid's x[12]), rows s += ap ds, z += ad dz
            const double dsv = L.dX[12];
            SYNC();
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                X[e] = fma(ap, L.dX[13 * k + i], X[e]);
                U[e] = fma(ap, L.dU[e], U[e]);
            }
            if (tid == 0) L.Z[24 * N] = fma(ap, dsv, L.Z[24 * N]);
#pragma unroll
            for (int t = 0; t < TL; t++)
#pragma unroll
                for (int q = 0; q < 6; q++) { ls[t][q] = fma(ap, dls[t][q], ls[t][q]); lz[t][q] = fma(ad, dlz[t][q], lz[t][q]); }
#pragma unroll
            for (int t = 0; t < TO; t++) { os[t] = fma(ap, dos[t], os[t]); oz[t] = fma(ad, doz[t], oz[t]); }
            SYNC();
            S12ST(7);   // corrector row step + update
        }
        if (stage == 0) {
            // stopped at the warm-start tolerance tol_qp: 4, never OPTIMAL (oracle/srb12.c, same rule)
            qp_flag = (flag == 0 && tol_s > tol) ? 4 : flag; qp_it = it;
            if (x_qp_out)
                for (int v = tid; v < nv; v += 64) x_qp_out[(size_t)agent * nv + v] = L.Z[v];
            // a FATAL QP stage ends the solve: the NLP stage does not run and reports FATAL too (a
            // consumer reading the NLP status alone must not see OPTIMAL; oracle/srb12.c, same rule)
            if (flag == 3) { if (prm.use_nlp) nlp_flag = 3; break; }
        } else {
            nlp_flag = flag; nlp_it = it;
        }
    }
    // ---- active-set polish of the last stage's OPTIMAL result (oracle/srb12.c polish12, the same steps):
    // rows with s KAPPA < z form the active set A; Newton steps on the augmented Lagrangian
    //   (H_L + RHO J_A'J_A) d = -(grad f + J_A'(z_A + RHO c_A)),  z_A += RHO (c_A + J_A d)
    // through the same Riccati factor / solve (the weights RHO on the active rows, 0 on the others,
    // -2 y on (p_x, p_y) of active obstacle rows, y = z_A + RHO c_A), one factor per pass and at most IT
    // steps (fewer once |d| <= DXTOL); accepted when every row holds to PTOL, the active rows to PTOL,
    // z_A >= -1e-9 max |z_A| and the last step <= DXTOL; else the most negative multiplier leaves, the
    // violated rows join and a second pass starts from the interior-point result.  Rejected: that result
    // stands (it met tol_final).  Why: along the legs' internal-force directions only r = 1e-2 pins the
    // forces, so an interior-point iterate at s'z/m ~ 1e-9 is still up to 1e-3 N off; the active set's
    // KKT point is exact.
    const int fin_flag = prm.use_nlp ? nlp_flag : qp_flag;
    if (prm.polish && fin_flag == 0) {
        S12ST(8);
        bool lact[TL][6], oact[TO];
        double lza_[TL][6], ozz[TO], lcr[TL][6], ocr[TO];
#pragma unroll
        for (int t = 0; t < TL; t++)
#pragma unroll
            for (int q = 0; q < 6; q++) {
                lact[t][q] = lon[t] && ls[t][q] * SRB12_POL_KAPPA < lz[t][q];
                lza_[t][q] = lact[t][q] ? lz[t][q] : 0.0;
            }
#pragma unroll
        for (int t = 0; t < TO; t++) {
            oact[t] = oon[t] && os[t] * SRB12_POL_KAPPA < oz[t];
            ozz[t] = oact[t] ? oz[t] : 0.0;
        }
        SYNC();
        S12CK(0, (double)fin_flag); S12CK(1, dyn_res()); S12CK(2, lds_sum(L.Z, nv)); S12CK(3, X[0]);
        for (int v = tid; v < nv; v += 64) L.xsv[v] = L.Z[v];
        SYNC();
        S12CK(4, lds_sum(L.xsv, nv));
        bool accepted = false;
#pragma clang loop unroll(disable)
        for (int pass = 0; pass < SRB12_POL_PASSES; pass++) {
            if (pass > 0) {
                SYNC();
                for (int v = tid; v < nv; v += 64) L.Z[v] = L.xsv[v];
            }
            double lastdx = 1e300;
            bool bad = false;
#pragma clang loop unroll(disable)
            for (int pit = 0; pit < SRB12_POL_IT; pit++) {
                // gradient (column 1 of the right-hand side) and, for the pass's factor, the Hessian blocks
                SYNC();
                grad_f(L.gX, L.gU);
                if (pit == 0) for (int e = tid; e < 6 * N; e += 64) L.Q3[e] = 0.0;
                if (tid == 0) { L.sc[3] = prm.Sw * L.Z[24 * N]; L.sc[1] = prm.Sw; }
                SYNC();
#pragma unroll
                for (int t = 0; t < TL; t++) {
                    const int e = lane + 64 * t;
                    if (e >= NL) continue;
                    double gz[3] = {0.0, 0.0, 0.0}, rh[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
                    const double *u = U + 3 * (lon[t] ? e : 0);
#pragma unroll
                    for (int q = 0; q < 6; q++) {
                        double c0, c1, c2;
                        fric_coef(q, mus, c0, c1, c2);
                        lcr[t][q] = c0 * u[0] + c1 * u[1] + c2 * u[2] - ((q == 5) ? prm.fmax : 0.0);
                        if (!lact[t][q]) continue;
                        const double y = fma(SRB12_POL_RHO, lcr[t][q], lza_[t][q]);
                        const double cc[3] = {c0, c1, c2};
#pragma unroll
                        for (int a = 0; a < 3; a++) {
                            gz[a] = fma(y, cc[a], gz[a]);
#pragma unroll
                            for (int b = a; b < 3; b++) rh[sym3(a, b)] = fma(SRB12_POL_RHO * cc[a], cc[b], rh[sym3(a, b)]);
                        }
                    }
                    if (lon[t]) { double *gu = L.gU + 3 * e; gu[0] += gz[0]; gu[1] += gz[1]; gu[2] += gz[2]; }
                    if (pit == 0)
#pragma unroll
                        for (int m = 0; m < 6; m++) L.Rh[6 * e + m] = rh[m];
                }
#pragma unroll
                for (int t = 0; t < TO; t++) {
                    if (!oon[t]) continue;
                    const int e = lane + 64 * t;
                    double g, h, c0, c1;
                    obs_row(e, g, h, c0, c1);
                    ocr[t] = g - h;
                    if (!oact[t]) continue;
                    const double y = fma(SRB12_POL_RHO, ocr[t], ozz[t]), om = SRB12_POL_RHO;
                    const int k = e / K;
                    double *gx = L.gX + 13 * k, *q3 = L.Q3 + 6 * k;
                    __hip_atomic_fetch_add(&gx[0], y * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&gx[1], y * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&gx[12], -y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (pit == 0) {
                        __hip_atomic_fetch_add(&q3[0], fma(om * c0, c0, -2.0 * y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&q3[1], om * c0 * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&q3[2], fma(om * c1, c1, -2.0 * y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&q3[3], -om * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&q3[4], -om * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_add(&q3[5], om, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                // converged: a last step <= DXTOL that left the active rows within PTOL (oracle/srb12.c, same
                // rule; under the pass's frozen factor a small step can leave |c_A| above PTOL: one more step)
                if (pit > 0 && lastdx <= SRB12_POL_DXTOL) {
                    double cm = 0.0;
#pragma unroll
                    for (int t = 0; t < TL; t++)
#pragma unroll
                        for (int q = 0; q < 6; q++) cm = fmax(cm, lact[t][q] ? fabs(lcr[t][q]) : 0.0);
#pragma unroll
                    for (int t = 0; t < TO; t++) cm = fmax(cm, oact[t] ? fabs(ocr[t]) : 0.0);
                    if (wmax(cm) <= SRB12_POL_PTOL) break;
                }
                SYNC();
                if (pit == 0 && !factor(0.0)) { bad = true; break; }      // not definite: reject
                S12CKP(8, schur);
                sph = 9;
                riccati_solve(1, false);                                    // d = -H^-1 grad (column 1)
                S12CKP(9, sol_res()); S12CKP(10, L.dX[0]);
                S12CKP(11, L.dU[2]); S12CKP(12, lds_sum(L.xsv, nv));
                // multipliers z_A += RHO (c_A + J_A d) at the linearisation point; then x += d
#pragma unroll
                for (int t = 0; t < TL; t++) {
                    if (!lon[t]) continue;
                    const double *du = L.dU + 3 * (lane + 64 * t);
#pragma unroll
                    for (int q = 0; q < 6; q++) {
                        if (!lact[t][q]) continue;
                        double c0, c1, c2;
                        fric_coef(q, mus, c0, c1, c2);
                        lza_[t][q] = fma(SRB12_POL_RHO, lcr[t][q] + c0 * du[0] + c1 * du[1] + c2 * du[2], lza_[t][q]);
                    }
                }
#pragma unroll
                for (int t = 0; t < TO; t++) {
                    if (!oact[t]) continue;
                    const int e = lane + 64 * t;
                    double g, h, c0, c1;
                    obs_row(e, g, h, c0, c1);
                    const double *dx = L.dX + 13 * (e / K);
                    ozz[t] = fma(SRB12_POL_RHO, ocr[t] + c0 * dx[0] + c1 * dx[1] - dx[12], ozz[t]);
                }
                double mdx = 0.0;
                const double dsv = L.dX[12];
                SYNC();
                for (int e = tid; e < 12 * N; e += 64) {
                    const int k = e / 12, i = e - 12 * k;
                    const double dxe = L.dX[13 * k + i], due = L.dU[e];
                    X[e] += dxe; U[e] += due;
                    mdx = fmax(mdx, fmax(fabs(dxe), fabs(due)));
                }
                if (tid == 0) { L.Z[24 * N] += dsv; mdx = fmax(mdx, fabs(dsv)); }
                lastdx = wmax(mdx);
                SYNC();
                S12CKP(13, lastdx); S12CKP(14, dyn_res());
                S12CKP(15, X[0]);
            }
            S12CKA(5, bad ? 1.0 : 0.0);
            if (bad) break;
            SYNC();
            // acceptance at the polished point
            double pv = -1e300, cv = 0.0, nzmin = -1e300, zm = 1.0;
#pragma unroll
            for (int t = 0; t < TL; t++) {
                if (!lon[t]) continue;
                const double *u = U + 3 * (lane + 64 * t);
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    double c0, c1, c2;
                    fric_coef(q, mus, c0, c1, c2);
                    lcr[t][q] = c0 * u[0] + c1 * u[1] + c2 * u[2] - ((q == 5) ? prm.fmax : 0.0);
                    pv = fmax(pv, lcr[t][q]);
                    if (lact[t][q]) { cv = fmax(cv, fabs(lcr[t][q])); nzmin = fmax(nzmin, -lza_[t][q]); zm = fmax(zm, fabs(lza_[t][q])); }
                }
            }
#pragma unroll
            for (int t = 0; t < TO; t++) {
                if (!oon[t]) continue;
                double g, h, c0, c1;
                obs_row(lane + 64 * t, g, h, c0, c1);
                ocr[t] = g - h;
                pv = fmax(pv, ocr[t]);
                if (oact[t]) { cv = fmax(cv, fabs(ocr[t])); nzmin = fmax(nzmin, -ozz[t]); zm = fmax(zm, fabs(ozz[t])); }
            }
            {
                double rv[4] = {pv, cv, nzmin, zm};
                wred<4, 15u>(rv);
                pv = rv[0]; cv = rv[1]; nzmin = rv[2]; zm = rv[3];
            }
            // the dynamics too: the rows alone would pass a point the Newton steps carried off them
            const double dres = dyn_res();
            S12CKA(0, pv); S12CKA(1, cv); S12CKA(2, nzmin); S12CKA(3, zm);
            S12CKA(4, dres); S12CKA(6, lastdx); S12CKA(7, X[0]);
            if (pv <= SRB12_POL_PTOL && cv <= SRB12_POL_PTOL && nzmin <= 1e-9 * zm && lastdx <= SRB12_POL_DXTOL &&
                dres <= SRB12_POL_DYNTOL) {
                accepted = true;
                break;
            }
            // next pass: the most negative multiplier leaves (lowest row on ties, the oracle's row order:
            // friction 6 leg + q, then obstacles 24 N + e), violated rows join (multiplier 0), the others
            // keep max(z_A, 0)
            double wd = -1e-9 * zm;
            int wk = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < TL; t++)
#pragma unroll
                for (int q = 0; q < 6; q++)
                    if (lact[t][q] && lza_[t][q] < wd) lexmin(wd, wk, lza_[t][q], 6 * (lane + 64 * t) + q);
#pragma unroll
            for (int t = 0; t < TO; t++)
                if (oact[t] && ozz[t] < wd) lexmin(wd, wk, ozz[t], 24 * N + lane + 64 * t);
            if (wk == 0x7fffffff) wd = 1e300;
            wargmin(wd, wk);
            bool changed = wk != 0x7fffffff;
#pragma unroll
            for (int t = 0; t < TL; t++)
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    if (6 * (lane + 64 * t) + q == wk) lact[t][q] = false;
                    else if (lon[t] && !lact[t][q] && lcr[t][q] > SRB12_POL_PTOL) { lact[t][q] = true; changed = true; }
                    lza_[t][q] = lact[t][q] ? fmax(lza_[t][q], 0.0) : 0.0;
                }
#pragma unroll
            for (int t = 0; t < TO; t++) {
                if (24 * N + lane + 64 * t == wk) oact[t] = false;
                else if (oon[t] && !oact[t] && ocr[t] > SRB12_POL_PTOL) { oact[t] = true; changed = true; }
                ozz[t] = oact[t] ? fmax(ozz[t], 0.0) : 0.0;
            }
            if (!__builtin_amdgcn_ballot_w64(changed)) break;
        }
        SYNC();
        if (!accepted) {
            for (int v = tid; v < nv; v += 64) L.Z[v] = L.xsv[v];
            // the interior-point point stands, up to ~1e-3 N from the optimum along the legs' internal-force
            // directions: ACCEPTABLE (4), never OPTIMAL (oracle/srb12.c, same rule)
            if (prm.use_nlp) nlp_flag = 4; else qp_flag = 4;
        }
        SYNC();
        S12CK(120, accepted ? 1.0 : 0.0); S12CK(121, lds_sum(L.Z, nv)); S12CK(122, X[0]); S12CK(123, dyn_res());
        S12ST(9);
    }
#ifdef SRB12_STAMPS
    SYNC();
    if (dstamp && tid < 16) prm.dbg[SRB12_DBG_TRACE + tid] += stl[tid];
#endif
    // ---- outputs: x and 0.5 x'Px + c'x
    double f = 0.0;
    for (int v = tid; v < nv; v += 64) {
        const double xv = L.Z[v];
        x_out[(size_t)agent * nv + v] = xv;
        double w, cl = 0.0;
        if (v < 12 * N) { const int k = v / 12, i = v - 12 * k; w = (k == N - 1) ? L.wqN[i] : L.wq[i]; cl = -w * L.xr[v]; }
        else if (v < 24 * N) w = L.wr[(v - 12 * N) % 3];
        else w = prm.Sw;
        f += fma(0.5 * w * xv, xv, cl * xv);
    }
    f = wsum(f);
    if (tid == 0) {
        obj_out[agent] = f;
        status_out[2 * agent] = qp_flag; status_out[2 * agent + 1] = nlp_flag;
        iters_out[2 * agent] = qp_it; iters_out[2 * agent + 1] = nlp_it;
    }
}

#define SRB12_KERNEL(TL, TO, NC, K1)                                                                            \
    extern "C" __global__ void __launch_bounds__(64) SRB12_WPE srb12_kernel_##TL##_##TO##_##NC##_##K1(          \
        Srb12KParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ xrefg,        \
        const double *__restrict__ footg, const int *__restrict__ contactg, const double *__restrict__ obstacles, \
        const double *__restrict__ nbr_state, const int *__restrict__ sel_g, double *__restrict__ x_qp_out,      \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                \
        int *__restrict__ iters_out)                                                                          \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = xcd_agent(blockIdx.x, gridDim.x);                                                   \
        if (agent >= n_agents) return;                                                                         \
        srb12_agent<TL, TO, NC, K1>(prm, agent, x0g, xrefg, footg, contactg, obstacles, nbr_state, sel_g, x_qp_out,     \
                            x_out, obj_out, status_out, iters_out, lds);                                       \
    }
SRB12_INSTANCES(SRB12_KERNEL)

// CoM rows [x, xdot, y, ydot] of a 12-state batch: the layout the shared selection kernel
// (srb_knn_kernel) reads its query points from
extern "C" __global__ void srb12_pos_kernel(int n_agents, const double *__restrict__ x0g, double *__restrict__ pos)
{
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n_agents) return;
    const double *x = x0g + 12 * (size_t)a;
    pos[4 * (size_t)a] = x[0]; pos[4 * (size_t)a + 1] = x[6]; pos[4 * (size_t)a + 2] = x[1]; pos[4 * (size_t)a + 3] = x[7];
}
