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
// the obstacle rows, then the NLP warm-started from it), the iteration of oracle/srb12.c step for
// step.  The Newton system is solved by a Riccati recursion over the horizon instead of the
// oracle's dense LU -- O(N 12^3) per iteration, the structure the 12-state model has:
//   * every inequality row is a slot owned by one lane (registers), scattered into per-grid
//     Hessian blocks (the p_xy 2x2 block and the s border column of the obstacle rows, the 3x3
//     friction blocks of each leg) by LDS atomics;
//   * backward pass per grid: G = V A, F = V B (A, B applied through their structure: a few FMAs
//     per entry), Hu = R^ + B'F = L D L' by a register forward elimination of [Hu | Hux | I] (its
//     pivots are the reduced Hessian's: the inertia test), Z = D^-1/2 L^-1 kept for the solves
//     (Hu^-1 = Z'Z), and the Schur update V' = Q^ + A'G - Y'Y, Y = Z Hux, as a 16x16x16 product on
//     the matrix cores (v_mfma_f64_16x16x4f64), positive semi-definite by construction;
//   * the obstacle slack s rides along as a 13th state (s_{k+1} = s_k, s_0 free), so the stiff
//     obstacle rows stay inside one grid's block;
//   * the dual residual uses the costates of the backward recursion lambda_k = grad_x_k L +
//     A_k' lambda_{k+1} (the state part of r_d is zero, the input part is the reduced gradient);
//     the primal-dual step does not depend on them (oracle, same rule).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "srb_kernel_params.h"

#define SYNC() __syncthreads()
#include "srb_wave.h"

namespace {

struct Srb12Lds {
    double *Wl, *cs, *ct, *Lm, *Hx, *V0, *Gt, *Ft, *Mt, *Q3, *Rh, *Z, *xr, *gX, *gU;
    double *rX, *rU, *dX, *dU, *gus, *vv, *sc, *obs, *eps, *xsv;
    int *sel;
};

// the carve of srb12_lds_doubles (srb_kernel_params.h), same order.  State vectors carry 13 entries
// per grid (the 12 states and the slack), input vectors 12; columns 0 (solve) and 1 (its refinement)
__device__ __forceinline__ Srb12Lds carve12(double *p, int N, int K)
{
    Srb12Lds L;
    L.Wl = p; p += 36 * N;  L.cs = p; p += 2 * N;  L.ct = p; p += 4 * N;
    L.Lm = p; p += 78 * N; L.Hx = p; p += 156 * N;          // Z = D^-1/2 L^-1 packed lower triangle, Hux
    L.V0 = p; p += 169;                                     // V (the update is written over it)
    L.Gt = p; p += 169; L.Ft = p; p += 156; L.Mt = L.Ft;    // Y reuses F's storage (single wave, in order)
    L.Q3 = p; p += 6 * N; L.Rh = p; p += 24 * N;
    L.Z = p; p += 24 * N + 4; L.xr = p; p += 12 * N;
    L.rX = p; p += 26 * N; L.rU = p; p += 24 * N; L.dX = p; p += 13 * N; L.dU = p; p += 12 * N;
    L.gX = L.rX + 13 * N; L.gU = L.rU + 12 * N;              // gradients: column 1 (free until the refinement)
    L.gus = p; p += 12 * N; L.vv = p; p += 16; L.sc = p; p += 16;
    L.obs = p; p += 2 * N * K; L.eps = p; p += K;
    L.xsv = p; p += 24 * N + 1;                             // the interior-point result (polish)
    L.sel = (int *)p;
    return L;
}

// pivot-row entries of the forward elimination: every 16-lane row holds the whole matrix, so a DPP
// row broadcast (SRB12_ELIM_DPP=1) or a readlane of lane kk (0) give the same value
#ifndef SRB12_ELIM_DPP
#define SRB12_ELIM_DPP 0
#endif
#if SRB12_ELIM_DPP
#define SRB12_PIVROW(v, kk) bc16((v), (kk))
#else
#define SRB12_PIVROW(v, kk) readlane_d((v), (kk))
#endif

// per-phase cycle stamps of the traced agent (diagnostic build -DSRB12_STAMPS, libsrbnmpc_s12st.so):
// s_memtime deltas accumulated into prm.dbg[SRB12_DBG_TRACE + slot], read by srb12_debug_trace
#define SRB12_DBG_TRACE (2 * 64 * 8)
#ifdef SRB12_STAMPS
#define S12ST(slot)                                                                                  \
    do {                                                                                             \
        if (dstamp) {                                                                                \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            if (tid == 0) prm.dbg[SRB12_DBG_TRACE + (slot)] += (double)(t_ - tprev);                  \
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


} // namespace

template <int TS>
__device__ __forceinline__ void srb12_agent(const Srb12KParams &prm, int agent, const double *__restrict__ x0g,
        const double *__restrict__ xrefg, const double *__restrict__ footg, const int *__restrict__ contactg,
        const double *__restrict__ obstacles, const double *__restrict__ nbr_state, const int *__restrict__ sel_g,
        double *__restrict__ x_qp_out, double *__restrict__ x_out, double *__restrict__ obj_out,
        int *__restrict__ status_out, int *__restrict__ iters_out, double *lds)
{
    const int tid = threadIdx.x, lane = tid;
    const int N = prm.N, K = prm.K_obs + prm.K_nbr, NK = N * K, nv = 24 * N + 1;
    const int nf = 24 * N;                                  // friction row slots
    const double Ts = prm.Ts, tsm = prm.Ts / prm.mass, mus = prm.mus;
    const double tol = prm.tol, th = tol / sqrt(3.0);
    Srb12Lds L = carve12(lds, N, K);
    double *X = L.Z, *U = L.Z + 12 * N;
    const double *x0 = x0g + 12 * (size_t)agent;
#ifdef SRB12_STAMPS
    const bool dstamp = agent == prm.dbg_agent && prm.dbg != nullptr;
    unsigned long long tprev = dstamp ? __builtin_amdgcn_s_memtime() : 0ull;
#endif

    // ---------------- inputs, per-grid model (orc12_dynamics), selected rows
    for (int i = tid; i < 12 * N; i += 64) L.xr[i] = xrefg[(size_t)agent * 12 * N + i];
    for (int i = tid; i < 4 * N; i += 64) L.ct[i] = contactg[(size_t)agent * 4 * N + i] ? 1.0 : 0.0;
    if (prm.use_nlp && tid < K) L.sel[tid] = sel_g[(size_t)agent * K + tid];
    SYNC();
    for (int e = tid; e < 4 * N; e += 64) {              // one (grid, leg) per lane: W_l = Ts Iw^-1 [r]x
        const int k = e >> 2, l = e & 3;
        const double *ph = (k == 0) ? x0 : L.xr + 12 * (k - 1);
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
        const double r0 = fp[0] - ph[0], r1 = fp[1] - ph[1], r2 = fp[2] - ph[2];
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

    // ---------------- slot state (registers): row t of this lane is slot id = lane + 64 t
    double ss[TS], zz[TS], dsa[TS], dza[TS];
    int qp_flag = 3, qp_it = 0, nlp_flag = 0, nlp_it = 0;
    const int nstage = prm.use_nlp ? 2 : 1;
    int nrow = nf;                                      // rows of the current stage (row_g)
    auto row_g = [&](int id, double &g, double &h, double &c0, double &c1, double &c2, int &kind) {
        g = 0.0; h = 0.0; c0 = c1 = c2 = 0.0; kind = 0;
        if (id < nf) {
            const int k = id / 24, l = (id / 6) & 3, q = id % 6;
            if (L.ct[4 * k + l] != 0.0) {
                kind = 1;
                fric_coef(q, mus, c0, c1, c2);
                const double *u = U + 12 * k + 3 * l;
                g = c0 * u[0] + c1 * u[1] + c2 * u[2];
                h = (q == 5) ? prm.fmax : 0.0;
            }
        } else if (id < nrow) {
            const int e = id - nf, k = e / K, j = e - k * K;
            kind = 2;
            const double dx = X[12 * k] - L.obs[2 * e], dy = X[12 * k + 1] - L.obs[2 * e + 1];
            c0 = -2.0 * dx; c1 = -2.0 * dy;
            g = -(dx * dx + dy * dy) - L.Z[24 * N];
            h = -L.eps[j];
        }
    };
    // Q^_k (state block k, 13 x 13): diag(q) + delta on the 12 states, the obstacle rows' (p_x, p_y, s)
    // block; the slack's own weight Sw + delta enters once, at s_0
    auto qhat = [&](int k, int i, int j, double delta) {
        double v = (i == j && i < 12) ? ((k == N - 1) ? prm.qN[i] : prm.q[i]) + delta : 0.0;
        const bool pi = i < 2 || i == 12, pj = j < 2 || j == 12;
        if (pi && pj) {
            const double *q3 = L.Q3 + 6 * k;
            const int a = (i == 12) ? 2 : i, b = (j == 12) ? 2 : j;
            const int lo = a < b ? a : b, hi = a < b ? b : a;
            v += (lo == 0) ? (hi == 0 ? q3[0] : hi == 1 ? q3[1] : q3[3]) : (lo == 1) ? (hi == 1 ? q3[2] : q3[4]) : q3[5];
        }
        return v;
    };
    // backward Riccati factor over the 13-state with the shift delta; false when a pivot (the inertia
    // test) or the initial slack's Schur complement is not positive.  Reads the per-grid Hessian blocks
    // (Q3, Rh), writes Z = D^-1/2 L^-1 and Hux per grid and sets `schur`
    double schur = 0.0;
    auto factor = [&](double delta) -> bool {
        int fail = 0;
        for (int e = tid; e < 169; e += 64) L.V0[e] = qhat(N - 1, e / 13, e % 13, delta);
        SYNC();
        for (int k = N - 1; k >= 0; k--) {
            const double c = L.cs[2 * k], s = L.cs[2 * k + 1];
            const double *W = L.Wl + 36 * k, *ct = L.ct + 4 * k, *V = L.V0;
            // G = V A~_k (13 x 13), F = V B~_k (13 x 12)
            for (int e = tid; e < 169; e += 64) {
                const int i = e / 13, j = e - 13 * i;
                const double *Vi = V + 13 * i;
                double g = Vi[j];
                if (j >= 6 && j < 9) g = fma(Ts, Vi[j - 6], g);
                else if (j >= 9 && j < 12) g = fma(Ts, Vi[3] * rzab(j - 9, 0, c, s) + Vi[4] * rzab(j - 9, 1, c, s) + Vi[5] * rzab(j - 9, 2, c, s), g);
                L.Gt[e] = g;
            }
            for (int e = tid; e < 156; e += 64) {
                const int i = e / 12, j = e - 12 * i, l = j / 3, jj = j - 3 * l;
                const double *Vi = V + 13 * i;
                double f = ct[l] * tsm * Vi[6 + jj];
                for (int a = 0; a < 3; a++) f = fma(Vi[9 + a], W[9 * l + 3 * a + jj], f);
                L.Ft[e] = f;
            }
            SYNC();
            // Hux = B'G (12 x 13, stored), V_next = Q^_{k-1} + A~'G (then - Hux' Hu^-1 Hux); at k = 0 only
            // V_0[12][12] is used (the initial slack's Schur complement)
            double *Hx = L.Hx + 156 * k, *Vn = L.V0;
            for (int e = tid; e < 156; e += 64) {
                const int i = e / 13, j = e - 13 * i;
                const int li = i / 3, ai = i - 3 * li;
                double hx = ct[li] * tsm * L.Gt[13 * (6 + ai) + j];
                for (int a = 0; a < 3; a++) hx = fma(W[9 * li + 3 * a + ai], L.Gt[13 * (9 + a) + j], hx);
                Hx[e] = hx;
            }
            for (int e = tid; e < 169; e += 64) {
                const int i = e / 13, j = e - 13 * i;
                double w = L.Gt[e];
                if (i >= 6 && i < 9) w = fma(Ts, L.Gt[13 * (i - 6) + j], w);
                else if (i >= 9 && i < 12)
                    w = fma(Ts, rzab(i - 9, 0, c, s) * L.Gt[39 + j] + rzab(i - 9, 1, c, s) * L.Gt[52 + j] +
                                    rzab(i - 9, 2, c, s) * L.Gt[65 + j], w);
                if (k > 0) w += qhat(k - 1, i, j, delta);
                Vn[e] = w;
            }
            SYNC();
            // Hu = R^ + B'F = L D L' by a forward elimination of [Hu | Hux | I] in registers (row i16
            // per lane, replicated in every 16-lane row): its pivots are the inertia test, Z = D^-1/2 L^-1
            // (stored: the solves apply Hu^-1 = Z'Z) and Y = Z Hux, so the Schur update
            // S = Hux' Hu^-1 Hux = Y'Y is one 16x16x16 product on the matrix cores.  The product with
            // an explicit inverse, Hux'(Hu^-1 Hux), loses V's definiteness once z / s reaches ~1e7 on
            // active rows; Y'Y is positive semi-definite by construction.
            {
                const int i16 = lane & 15, q = lane >> 4;
                double Ag[37];
                {
                    const int li = (i16 < 12) ? i16 / 3 : 0, ai = (i16 < 12) ? i16 - 3 * li : 0;
#pragma unroll
                    for (int j = 0; j < 12; j++) {
                        double v = 0.0;
                        if (i16 < 12) {
                            v = ct[li] * tsm * L.Ft[12 * (6 + ai) + j];
                            for (int aa = 0; aa < 3; aa++) v = fma(W[9 * li + 3 * aa + ai], L.Ft[12 * (9 + aa) + j], v);
                            if (j == i16) v += prm.r[ai] + delta;
                            if (j / 3 == li) v += L.Rh[24 * k + 6 * li + sym3(ai, j - 3 * (j / 3))];
                        }
                        Ag[j] = v;
                    }
#pragma unroll
                    for (int j = 0; j < 13; j++) Ag[12 + j] = (i16 < 12) ? Hx[13 * i16 + j] : 0.0;
#pragma unroll
                    for (int j = 0; j < 12; j++) Ag[25 + j] = (i16 == j) ? 1.0 : 0.0;
                }
                double dk = 1.0;
#pragma unroll
                for (int kk = 0; kk < 12; kk++) {
                    const double piv = readlane_d(Ag[kk], kk);
                    fail |= !(piv > 0.0);
                    const double f = (i16 > kk && i16 < 12) ? Ag[kk] * rcp_d(piv) : 0.0;
#pragma unroll
                    for (int j = kk + 1; j < 25; j++) Ag[j] = fma(-f, SRB12_PIVROW(Ag[j], kk), Ag[j]);
#pragma unroll
                    for (int j = 0; j <= kk; j++) Ag[25 + j] = fma(-f, SRB12_PIVROW(Ag[25 + j], kk), Ag[25 + j]);
                    dk = (i16 == kk) ? piv : dk;
                }
                const double sc_ = (i16 < 12 && dk > 0.0) ? 1.0 / sqrt(dk) : 0.0;
                if (lane < 12) {
#pragma unroll
                    for (int j = 0; j < 13; j++) L.Mt[13 * lane + j] = Ag[12 + j] * sc_;
#pragma unroll
                    for (int j = 0; j < 12; j++)
                        if (j <= lane) L.Lm[78 * k + (lane * (lane + 1)) / 2 + j] = Ag[25 + j] * sc_;
                }
                SYNC();
                d4 acc2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                    const int kc = 4 * kk + q;
                    const double y = (kc < 12 && i16 < 13) ? L.Mt[13 * kc + i16] : 0.0;
                    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, acc2, 0, 0, 0);
                }
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = q + 4 * r;
                    if (row < 13 && i16 < 13) Vn[13 * row + i16] -= acc2[r];
                }
            }
            SYNC();
        }
        if (fail) return false;
        // the free initial slack closes the recursion: V_0[12][12] + Sw + delta > 0 is the last
        // pivot of the inertia test
        schur = L.V0[168] + prm.Sw + delta;
        return schur > 0.0;
    };
    // Riccati solve of column c (rX: 13 per grid, rU: 12 per grid, sc[2 + c]: the s_0 entry) into
    // dX (13 per grid), dU: w solves H w = -rhs on the dynamics' null space (x_0 fixed, s_0 free).
    // Vectors live in registers, component i = lane & 15 (each 16-lane row holds a copy), and move
    // between lanes by DPP row broadcasts: no LDS round trip or barrier inside the recursion.
    auto riccati_solve = [&](int c, bool acc) {
        const int i = lane & 15, ir = (i < 12) ? i : 0, l = ir / 3, jj = ir - 3 * l, tri = (ir * (ir + 1)) / 2;
        const double *rX = L.rX + 13 * N * c, *rU = L.rU + 12 * N * c;
        double *dX = L.dX, *dU = L.dU, *gus = L.gus;      // acc: the refinement's correction adds in
        double v = (i < 13) ? rX[13 * (N - 1) + i] : 0.0;
        for (int k = N - 1; k >= 0; k--) {
            const double *W = L.Wl + 36 * k, *ct = L.ct + 4 * k, *Zk = L.Lm + 78 * k, *Hx = L.Hx + 156 * k;
            double vb[13];
#pragma unroll
            for (int j = 0; j < 13; j++) vb[j] = bc16(v, j);
            double gu = 0.0;
            if (i < 12) {
                gu = rU[12 * k + i] + ct[l] * tsm * (jj == 0 ? vb[6] : jj == 1 ? vb[7] : vb[8]);
                for (int a = 0; a < 3; a++) gu = fma(W[9 * l + 3 * a + jj], vb[9 + a], gu);
            }
            if (lane < 12) gus[12 * k + i] = gu;
            double w = 0.0, kk = 0.0;                        // kk = -Z'(Z gu)
#pragma unroll
            for (int j = 0; j < 12; j++) w = fma((j <= ir) ? Zk[tri + j] : 0.0, bc16(gu, j), w);
            if (i >= 12) w = 0.0;
#pragma unroll
            for (int j = 0; j < 12; j++) kk = fma((ir <= j) ? -Zk[(j * (j + 1)) / 2 + ir] : 0.0, bc16(w, j), kk);
            if (i >= 12) kk = 0.0;
            const double cc = L.cs[2 * k], sn = L.cs[2 * k + 1];
            double vn = v;                                     // A~' v
            if (i >= 6 && i < 9) vn = fma(Ts, i == 6 ? vb[0] : i == 7 ? vb[1] : vb[2], vn);
            else if (i >= 9 && i < 12)
                vn = fma(Ts, i == 9 ? fma(cc, vb[3], -sn * vb[4]) : i == 10 ? fma(sn, vb[3], cc * vb[4]) : vb[5], vn);
            if (k > 0 && i < 13) vn += rX[13 * (k - 1) + i];
            if (i < 13)
#pragma unroll
                for (int j = 0; j < 12; j++) vn = fma(Hx[13 * j + i], bc16(kk, j), vn);
            v = (i < 13) ? vn : 0.0;
        }
        const double ds0 = -(bc16(v, 12) + L.sc[2 + c]) / schur;
        double prev = (i == 12) ? ds0 : 0.0;
        for (int k = 0; k < N; k++) {
            // t = Hux dx_k + gu_k ; du_k = -Hu^-1 t ; dx_{k+1} = A~_k dx_k + B~_k du_k
            const double *W = L.Wl + 36 * k, *ct = L.ct + 4 * k, *Zk = L.Lm + 78 * k, *Hr = L.Hx + 156 * k + 13 * ir;
            double pb[13];
#pragma unroll
            for (int j = 0; j < 13; j++) pb[j] = bc16(prev, j);
            double t = gus[12 * k + ir];
#pragma unroll
            for (int j = 0; j < 13; j++) t = fma(Hr[j], pb[j], t);
            if (i >= 12) t = 0.0;
            double w = 0.0, du = 0.0;                        // du = -Z'(Z t)
#pragma unroll
            for (int j = 0; j < 12; j++) w = fma((j <= ir) ? Zk[tri + j] : 0.0, bc16(t, j), w);
            if (i >= 12) w = 0.0;
#pragma unroll
            for (int j = 0; j < 12; j++) du = fma((ir <= j) ? -Zk[(j * (j + 1)) / 2 + ir] : 0.0, bc16(w, j), du);
            if (i >= 12) du = 0.0;
            if (lane < 12) dU[12 * k + i] = acc ? dU[12 * k + i] + du : du;
            double db[12];
#pragma unroll
            for (int j = 0; j < 12; j++) db[j] = bc16(du, j);
            const double cc = L.cs[2 * k], sn = L.cs[2 * k + 1];
            double dx = prev;
            if (i < 3) dx = fma(Ts, i == 0 ? pb[6] : i == 1 ? pb[7] : pb[8], dx);
            else if (i < 6)
                dx = fma(Ts, i == 3 ? fma(cc, pb[9], sn * pb[10]) : i == 4 ? fma(-sn, pb[9], cc * pb[10]) : pb[11], dx);
            else if (i < 9) {
                for (int ll = 0; ll < 4; ll++) dx = fma(ct[ll] * tsm, i == 6 ? db[3 * ll] : i == 7 ? db[3 * ll + 1] : db[3 * ll + 2], dx);
            } else if (i < 12) {
                const int a = i - 9;
                for (int ll = 0; ll < 4; ll++)
                    for (int j = 0; j < 3; j++) dx = fma(W[9 * ll + 3 * a + j], db[3 * ll + j], dx);
            }
            if (i > 12) dx = 0.0;
            if (lane < 13) dX[13 * k + i] = acc ? dX[13 * k + i] + dx : dx;
            prev = dx;
        }
        SYNC();
    };
    // one step of iterative refinement of column 0 (correction in column 1): the residual of H w = -rhs
    // on the null space is the reduced gradient -- t_u = R^ du + rhs_u + B' mu, t_s = (Sw + delta) ds_0 +
    // rhs_s + mu_0[12], costates mu from the state rows -- and the correction solves with (0, t_u, t_s).
    // Explicit Gauss-Jordan inverses lose digits once z / s reaches 1e7 on active rows.
    auto refine = [&](double delta) {
        const int i = lane & 15, ir = (i < 12) ? i : 0, l = ir / 3, a3 = ir - 3 * l;
        const double *rX = L.rX, *rU = L.rU, *dX = L.dX, *dU = L.dU;
        double *tX = L.rX + 13 * N, *tU = L.rU + 12 * N;
        auto qdx = [&](int k, const double *dx) {          // (Q^_k dx)[i]
            double v = 0.0;
            for (int j = 0; j < 13; j++) {
                const bool nz = (j == i) || ((i < 2 || i == 12) && (j < 2 || j == 12));
                if (nz) v = fma(qhat(k, i, j, delta), dx[j], v);
            }
            return v;
        };
        for (int e = tid; e < 13 * N; e += 64) tX[e] = 0.0;
        double m = (i < 13) ? qdx(N - 1, dX + 13 * (N - 1)) + rX[13 * (N - 1) + i] : 0.0;
        for (int k = N - 1; k >= 0; k--) {
            const double *W = L.Wl + 36 * k, *ct = L.ct + 4 * k;
            double vb[13];
#pragma unroll
            for (int j = 0; j < 13; j++) vb[j] = bc16(m, j);
            if (lane < 12) {
                const double *du = dU + 12 * k + 3 * l, *rh = L.Rh + 24 * k + 6 * l;
                double t = fma(prm.r[a3] + delta, du[a3], rU[12 * k + i]);
                for (int bb = 0; bb < 3; bb++) t = fma(rh[sym3(a3, bb)], du[bb], t);
                t = fma(ct[l] * tsm, a3 == 0 ? vb[6] : a3 == 1 ? vb[7] : vb[8], t);
                for (int a = 0; a < 3; a++) t = fma(W[9 * l + 3 * a + a3], vb[9 + a], t);
                tU[12 * k + i] = t;
            }
            if (k > 0) {
                const double cc = L.cs[2 * k], sn = L.cs[2 * k + 1];
                double mn = m;
                if (i >= 6 && i < 9) mn = fma(Ts, i == 6 ? vb[0] : i == 7 ? vb[1] : vb[2], mn);
                else if (i >= 9 && i < 12)
                    mn = fma(Ts, i == 9 ? fma(cc, vb[3], -sn * vb[4]) : i == 10 ? fma(sn, vb[3], cc * vb[4]) : vb[5], mn);
                m = (i < 13) ? mn + qdx(k - 1, dX + 13 * (k - 1)) + rX[13 * (k - 1) + i] : 0.0;
            }
        }
        const double m12 = bc16(m, 12);
        if (tid == 0) L.sc[3] = fma(prm.Sw + delta, dX[12], L.sc[2]) + m12;
        SYNC();
        riccati_solve(1, true);
    };
    // right-hand side of pass (0 predictor, 1 corrector) into column 0:
    // rhs = grad f + sum_rows J'(z + r3 / s + W r_p), r3 = -s z (+ sigma mu - ds_a dz_a)
    auto build_rhs = [&](int pass, double smu) {
        for (int e = tid; e < 12 * N; e += 64) {
            const int k = e / 12, i = e - 12 * k;
            const double w = (k == N - 1) ? prm.qN[i] : prm.q[i];
            L.rX[13 * k + i] = w * (X[e] - L.xr[e]);
            L.rU[e] = prm.r[i % 3] * U[e];
        }
        for (int k = tid; k < N; k += 64) L.rX[13 * k + 12] = 0.0;
        if (tid == 0) L.sc[2] = prm.Sw * L.Z[24 * N];
        SYNC();
#pragma unroll
        for (int t = 0; t < TS; t++) {
            const int id = lane + 64 * t;
            double g, h, c0, c1, c2; int kind;
            row_g(id, g, h, c0, c1, c2, kind);
            if (!kind) continue;
            const double rp = g + ss[t] - h, om = zz[t] / ss[t];
            const double r3 = -ss[t] * zz[t] + (pass ? smu - dsa[t] * dza[t] : 0.0);
            const double w = zz[t] + r3 / ss[t] + om * rp;
            if (kind == 1) {
                const int k = id / 24, l = (id / 6) & 3;
                double *ru = L.rU + 12 * k + 3 * l;
                const double cc[3] = {c0, c1, c2};
                for (int a = 0; a < 3; a++)
                    if (cc[a] != 0.0) __hip_atomic_fetch_add(&ru[a], w * cc[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                double *rx = L.rX + 13 * ((id - nf) / K);
                __hip_atomic_fetch_add(&rx[0], w * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&rx[1], w * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(&rx[12], -w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        SYNC();
    };
    // the rows' steps of the solved column: J dz, ds = -r_p - J dz, dz = (r3 - z ds) / s; step maxima
    auto row_step = [&](int pass, double smu, double (&dsl)[TS], double (&dzl)[TS]) {
        double ms = 0.0, mz = 0.0;
#pragma unroll
        for (int t = 0; t < TS; t++) {
            const int id = lane + 64 * t;
            double g, h, c0, c1, c2; int kind;
            row_g(id, g, h, c0, c1, c2, kind);
            dsl[t] = dzl[t] = 0.0;
            if (!kind) continue;
            double jd;
            if (kind == 1) {
                const int k = id / 24, l = (id / 6) & 3;
                const double *du = L.dU + 12 * k + 3 * l;
                jd = c0 * du[0] + c1 * du[1] + c2 * du[2];
            } else {
                const double *dx = L.dX + 13 * ((id - nf) / K);
                jd = c0 * dx[0] + c1 * dx[1] - dx[12];
            }
            const double rp = g + ss[t] - h;
            const double r3 = -ss[t] * zz[t] + (pass ? smu - dsa[t] * dza[t] : 0.0);
            dsl[t] = -rp - jd; dzl[t] = (r3 - zz[t] * dsl[t]) / ss[t];
            ms = fmax(ms, -dsl[t] / ss[t]); mz = fmax(mz, -dzl[t] / zz[t]);
        }
        double rv[2] = {ms, mz};
        wred<2, 3u>(rv);
        return make_double2(rv[0] > 0.0 ? 1.0 / rv[0] : 1.0, rv[1] > 0.0 ? 1.0 / rv[1] : 1.0);
    };
    S12ST(0);   // inputs, model, rollout
#pragma clang loop unroll(disable)
    for (int stage = 0; stage < nstage; stage++) {
        const bool nl = stage == 1;
        nrow = nl ? nf + NK : nf;
        // active row count m and the starting slacks / duals (oracle ipm(): QP s = h - g, z = 1 /
        // max(s, 1); NLP shifted so min s = 1 when a row is violated, z = z0 / max(s, 1))
        double mcount = 0.0, mn = 1e300;
#pragma unroll
        for (int t = 0; t < TS; t++) {
            double g, h, c0, c1, c2; int kind;
            row_g(lane + 64 * t, g, h, c0, c1, c2, kind);
            ss[t] = h - g;
            if (kind) { mcount += 1.0; mn = fmin(mn, h - g); }
        }
        {
            double rv[2] = {mcount, -mn};
            wred<2, 2u>(rv);
            mcount = rv[0]; mn = -rv[1];
        }
        const double ssh = (nl && mn <= 0.0) ? 1.0 - mn : 0.0;
#pragma unroll
        for (int t = 0; t < TS; t++) {
            double g, h, c0, c1, c2; int kind;
            row_g(lane + 64 * t, g, h, c0, c1, c2, kind);
            double s = ss[t] + ssh;
            if (!nl && s < 1e-8) s = 1e-8;
            ss[t] = kind ? s : 1.0;
            zz[t] = kind ? (nl ? prm.z0 : 1.0) / fmax(s, 1.0) : 0.0;
            dsa[t] = dza[t] = 0.0;
        }
        const double inv_m = 1.0 / fmax(mcount, 1.0);
        const int maxit = nl ? prm.nlp_maxit : prm.qp_maxit;
        // the last stage's complementarity test is tol_final (the forces' accuracy: DESIGN.md 11)
        const double mtol = (stage == nstage - 1) ? prm.tol_final : tol;
        int flag = 2, it = 0;
        double sigma = 0.0;
#pragma clang loop unroll(disable)
        for (it = 0; it < maxit; it++) {
            // ---- gradient of f (X, U; Sw s of the slack at s_0), cleared per-grid blocks
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                const double w = (k == N - 1) ? prm.qN[i] : prm.q[i];
                L.gX[13 * k + i] = w * (X[e] - L.xr[e]);
                L.gU[e] = prm.r[i % 3] * U[e];
            }
            for (int k = tid; k < N; k += 64) L.gX[13 * k + 12] = 0.0;
            for (int e = tid; e < 6 * N; e += 64) L.Q3[e] = 0.0;
            for (int e = tid; e < 24 * N; e += 64) L.Rh[e] = 0.0;
            if (tid == 0) { L.sc[0] = prm.Sw * L.Z[24 * N]; L.sc[1] = prm.Sw; }    // grad_s f, H_ss (inertia scale)
            SYNC();
            // ---- rows: residuals, weights, scatter of J'z and J'WJ into the per-grid blocks
            double nrp = 0.0, sz = 0.0, zmx = 0.0;
#pragma unroll
            for (int t = 0; t < TS; t++) {
                const int id = lane + 64 * t;
                double g, h, c0, c1, c2; int kind;
                row_g(id, g, h, c0, c1, c2, kind);
                if (!kind) continue;
                const double rp = g + ss[t] - h, om = zz[t] / ss[t];
                nrp = fma(rp, rp, nrp);
                sz = fma(ss[t], zz[t], sz);
                zmx = fmax(zmx, zz[t]);
                if (kind == 1) {
                    const int k = id / 24, l = (id / 6) & 3;
                    double *gu = L.gU + 12 * k + 3 * l, *rh = L.Rh + 24 * k + 6 * l;
                    const double cc[3] = {c0, c1, c2};
                    for (int a = 0; a < 3; a++)
                        if (cc[a] != 0.0) __hip_atomic_fetch_add(&gu[a], zz[t] * cc[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    for (int a = 0; a < 3; a++)
                        for (int b = a; b < 3; b++)
                            if (cc[a] != 0.0 && cc[b] != 0.0)
                                __hip_atomic_fetch_add(&rh[sym3(a, b)], om * cc[a] * cc[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    // obstacle row of grid k on (p_x, p_y, s): J = (c0, c1, -1), Lagrangian Hessian -2z on p_x, p_y
                    const int k = (id - nf) / K;
                    double *gx = L.gX + 13 * k, *q3 = L.Q3 + 6 * k;
                    __hip_atomic_fetch_add(&gx[0], zz[t] * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&gx[1], zz[t] * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&gx[12], -zz[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[0], fma(om * c0, c0, -2.0 * zz[t]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[1], om * c0 * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[2], fma(om * c1, c1, -2.0 * zz[t]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[3], -om * c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[4], -om * c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&q3[5], om, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&L.sc[1], om, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            SYNC();
            // ---- costates and the dual residual (13-state: the slack rides along as x[12], s_{k+1} = s_k):
            //      lam_{N-1} = gX_{N-1}, lam_{k-1} = gX_{k-1} + A~_k' lam_k, r_u,k = gU_k + B_k' lam_k,
            //      r_s = Sw s + lam_0[12] (the free initial slack)
            double nrd = 0.0, gm = 1.0;
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                const double w = (k == N - 1) ? prm.qN[i] : prm.q[i];
                gm = fmax(gm, fabs(w * (X[e] - L.xr[e])));
                gm = fmax(gm, fabs(prm.r[i % 3] * U[e]));
            }
            gm = fmax(gm, fabs(prm.Sw * L.Z[24 * N]));
            {
                const int i = lane & 15, ir = (i < 12) ? i : 0, l = ir / 3, jj = ir - 3 * l;
                double lam = (i < 13) ? L.gX[13 * (N - 1) + i] : 0.0;
                for (int k = N - 1; k >= 0; k--) {
                    const double *W = L.Wl + 36 * k, *ct = L.ct + 4 * k;
                    double vb[13];
#pragma unroll
                    for (int j = 0; j < 13; j++) vb[j] = bc16(lam, j);
                    if (lane < 12) {
                        double ru = L.gU[12 * k + i] + ct[l] * tsm * (jj == 0 ? vb[6] : jj == 1 ? vb[7] : vb[8]);
                        for (int a = 0; a < 3; a++) ru = fma(W[9 * l + 3 * a + jj], vb[9 + a], ru);
                        nrd = fma(ru, ru, nrd);
                    }
                    if (k > 0) {
                        const double cc = L.cs[2 * k], sn = L.cs[2 * k + 1];
                        double ln = lam;
                        if (i >= 6 && i < 9) ln = fma(Ts, i == 6 ? vb[0] : i == 7 ? vb[1] : vb[2], ln);
                        else if (i >= 9 && i < 12)
                            ln = fma(Ts, i == 9 ? fma(cc, vb[3], -sn * vb[4]) : i == 10 ? fma(sn, vb[3], cc * vb[4]) : vb[5], ln);
                        lam = (i < 13) ? ln + L.gX[13 * (k - 1) + i] : 0.0;
                    }
                }
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
            if (dbgrow && tid == 0) { dbgrow[0] = nrd; dbgrow[1] = th * gm; dbgrow[2] = nrp; dbgrow[3] = mu; }
            // divergence (the LIP mode's rule, SRB_Z_DIV; oracle/srb12.c the same): a dual beyond 1e10 means
            // infeasible rows -- FATAL at this finite iterate
            if (!isfinite(nrd) || !isfinite(nrp) || !isfinite(sz) || !(zmx <= SRB_Z_DIV)) { flag = 3; break; }
            S12ST(1);   // residuals, weights, scatter, costates
            if (nrd < th * gm && nrp < th && mu < mtol) { flag = 0; break; }

            // ---- factorisation (backward Riccati over the 13-state) with the inertia shift delta (NLP)
            double dmax = 1.0;
            for (int e = tid; e < 12 * N; e += 64) {
                const int k = e / 12, i = e - 12 * k;
                const double qd = ((k == N - 1) ? prm.qN[i] : prm.q[i]) + (i < 2 ? L.Q3[6 * k + 2 * i] : 0.0);
                const int l = i / 3, a = i % 3;
                const double rd = prm.r[a] + L.Rh[24 * k + 6 * l + sym3(a, a)];
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
            // (the refinement only near the optimum, mu < 1e-3: far from it the step's accuracy is not
            // what limits progress, and it costs a solve)
            const bool refn = mu < 1e-3;
            build_rhs(0, 0.0);
            riccati_solve(0, false);
            if (refn) refine(delta);
            S12ST(4);   // predictor rhs + solve (+ refinement)
            double dsl[TS], dzl[TS];
            double2 al = row_step(0, 0.0, dsl, dzl);
#pragma unroll
            for (int t = 0; t < TS; t++) { dsa[t] = dsl[t]; dza[t] = dzl[t]; }
            {
                double num = 0.0;
#pragma unroll
                for (int t = 0; t < TS; t++) {
                    double g, h, c0, c1, c2; int kind;
                    row_g(lane + 64 * t, g, h, c0, c1, c2, kind);
                    if (kind) num = fma(fma(al.x, dsa[t], ss[t]), fma(al.y, dza[t], zz[t]), num);
                }
                num = wsum(num);
                const double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
                sigma = mr * mr * mr;
            }
            S12ST(5);   // predictor row step, sigma
            // ---- corrector
            build_rhs(1, sigma * mu);
            riccati_solve(0, false);
            if (refn) refine(delta);
            S12ST(6);   // corrector rhs + solve (+ refinement)
            al = row_step(1, sigma * mu, dsl, dzl);
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
            for (int t = 0; t < TS; t++) { ss[t] = fma(ap, dsl[t], ss[t]); zz[t] = fma(ad, dzl[t], zz[t]); }
            SYNC();
            S12ST(7);   // corrector row step + update
        }
        if (stage == 0) {
            qp_flag = flag; qp_it = it;
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
        bool pact[TS];
        double za[TS], cr[TS];
#pragma unroll
        for (int t = 0; t < TS; t++) {
            double g, h, c0, c1, c2; int kind;
            row_g(lane + 64 * t, g, h, c0, c1, c2, kind);
            pact[t] = kind && ss[t] * SRB12_POL_KAPPA < zz[t];
            za[t] = pact[t] ? zz[t] : 0.0;
        }
        for (int v = tid; v < nv; v += 64) L.xsv[v] = L.Z[v];
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
                for (int e = tid; e < 12 * N; e += 64) {
                    const int k = e / 12, i = e - 12 * k;
                    const double w = (k == N - 1) ? prm.qN[i] : prm.q[i];
                    L.gX[13 * k + i] = w * (X[e] - L.xr[e]);
                    L.gU[e] = prm.r[i % 3] * U[e];
                }
                for (int k = tid; k < N; k += 64) L.gX[13 * k + 12] = 0.0;
                if (pit == 0) {
                    for (int e = tid; e < 6 * N; e += 64) L.Q3[e] = 0.0;
                    for (int e = tid; e < 24 * N; e += 64) L.Rh[e] = 0.0;
                }
                if (tid == 0) { L.sc[3] = prm.Sw * L.Z[24 * N]; L.sc[1] = prm.Sw; }
                SYNC();
#pragma unroll
                for (int t = 0; t < TS; t++) {
                    const int id = lane + 64 * t;
                    double g, h, c0, c1, c2; int kind;
                    row_g(id, g, h, c0, c1, c2, kind);
                    cr[t] = g - h;
                    if (!pact[t]) continue;
                    const double y = fma(SRB12_POL_RHO, cr[t], za[t]), om = SRB12_POL_RHO;
                    if (kind == 1) {
                        const int k = id / 24, l = (id / 6) & 3;
                        double *gu = L.gU + 12 * k + 3 * l, *rh = L.Rh + 24 * k + 6 * l;
                        const double cc[3] = {c0, c1, c2};
                        for (int a = 0; a < 3; a++)
                            if (cc[a] != 0.0) __hip_atomic_fetch_add(&gu[a], y * cc[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (pit == 0)
                            for (int a = 0; a < 3; a++)
                                for (int b = a; b < 3; b++)
                                    if (cc[a] != 0.0 && cc[b] != 0.0)
                                        __hip_atomic_fetch_add(&rh[sym3(a, b)], om * cc[a] * cc[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        const int k = (id - nf) / K;
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
                }
                SYNC();
                if (pit == 0 && !factor(0.0)) { bad = true; break; }      // not definite: reject
                riccati_solve(1, false);                                    // d = -H^-1 grad (column 1)
                // multipliers z_A += RHO (c_A + J_A d) at the linearisation point; then x += d
                double mdx = 0.0;
#pragma unroll
                for (int t = 0; t < TS; t++) {
                    const int id = lane + 64 * t;
                    double g, h, c0, c1, c2; int kind;
                    row_g(id, g, h, c0, c1, c2, kind);
                    if (!pact[t]) continue;
                    double jd;
                    if (kind == 1) {
                        const int k = id / 24, l = (id / 6) & 3;
                        const double *du = L.dU + 12 * k + 3 * l;
                        jd = c0 * du[0] + c1 * du[1] + c2 * du[2];
                    } else {
                        const double *dx = L.dX + 13 * ((id - nf) / K);
                        jd = c0 * dx[0] + c1 * dx[1] - dx[12];
                    }
                    za[t] = fma(SRB12_POL_RHO, cr[t] + jd, za[t]);
                }
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
                if (lastdx <= SRB12_POL_DXTOL) break;
            }
            if (bad) break;
            SYNC();
            // acceptance at the polished point
            double pv = -1e300, cv = 0.0, nzmin = -1e300, zm = 1.0;
#pragma unroll
            for (int t = 0; t < TS; t++) {
                double g, h, c0, c1, c2; int kind;
                row_g(lane + 64 * t, g, h, c0, c1, c2, kind);
                cr[t] = g - h;
                if (!kind) continue;
                pv = fmax(pv, cr[t]);
                if (pact[t]) { cv = fmax(cv, fabs(cr[t])); nzmin = fmax(nzmin, -za[t]); zm = fmax(zm, fabs(za[t])); }
            }
            {
                double rv[4] = {pv, cv, nzmin, zm};
                wred<4, 15u>(rv);
                pv = rv[0]; cv = rv[1]; nzmin = rv[2]; zm = rv[3];
            }
            if (pv <= SRB12_POL_PTOL && cv <= SRB12_POL_PTOL && nzmin <= 1e-9 * zm && lastdx <= SRB12_POL_DXTOL) {
                accepted = true;
                break;
            }
            // next pass: the most negative multiplier leaves (lowest row on ties, the oracle's row order),
            // violated rows join (multiplier 0), the others keep max(z_A, 0)
            double wd = -1e-9 * zm;
            int wk = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < TS; t++)
                if (pact[t] && za[t] < wd) lexmin(wd, wk, za[t], lane + 64 * t);
            if (wk == 0x7fffffff) wd = 1e300;
            wargmin(wd, wk);
            bool changed = wk != 0x7fffffff;
#pragma unroll
            for (int t = 0; t < TS; t++) {
                const int id = lane + 64 * t;
                double g, h, c0, c1, c2; int kind;
                row_g(id, g, h, c0, c1, c2, kind);
                if (id == wk) pact[t] = false;
                else if (kind && !pact[t] && cr[t] > SRB12_POL_PTOL) { pact[t] = true; changed = true; }
                za[t] = pact[t] ? fmax(za[t], 0.0) : 0.0;
            }
            if (!__builtin_amdgcn_ballot_w64(changed)) break;
        }
        SYNC();
        if (!accepted)
            for (int v = tid; v < nv; v += 64) L.Z[v] = L.xsv[v];
        SYNC();
        S12ST(9);
    }
    // ---- outputs: x and 0.5 x'Px + c'x
    double f = 0.0;
    for (int v = tid; v < nv; v += 64) {
        const double xv = L.Z[v];
        x_out[(size_t)agent * nv + v] = xv;
        double w, cl = 0.0;
        if (v < 12 * N) { const int k = v / 12, i = v - 12 * k; w = (k == N - 1) ? prm.qN[i] : prm.q[i]; cl = -w * L.xr[v]; }
        else if (v < 24 * N) w = prm.r[(v - 12 * N) % 3];
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

#define SRB12_KERNEL(TS)                                                                                        \
    extern "C" __global__ void __launch_bounds__(64) srb12_kernel_##TS(                                         \
        Srb12KParams prm, int n_agents, const double *__restrict__ x0g, const double *__restrict__ xrefg,        \
        const double *__restrict__ footg, const int *__restrict__ contactg, const double *__restrict__ obstacles, \
        const double *__restrict__ nbr_state, const int *__restrict__ sel_g, double *__restrict__ x_qp_out,      \
        double *__restrict__ x_out, double *__restrict__ obj_out, int *__restrict__ status_out,                \
        int *__restrict__ iters_out)                                                                          \
    {                                                                                                          \
        extern __shared__ __attribute__((aligned(16))) double lds[];                                           \
        const int agent = blockIdx.x;                                                                          \
        if (agent >= n_agents) return;                                                                         \
        srb12_agent<TS>(prm, agent, x0g, xrefg, footg, contactg, obstacles, nbr_state, sel_g, x_qp_out, x_out, \
                        obj_out, status_out, iters_out, lds);                                                  \
    }
SRB12_KERNEL(4)
SRB12_KERNEL(6)
SRB12_KERNEL(8)
SRB12_KERNEL(12)

// CoM rows [x, xdot, y, ydot] of a 12-state batch: the layout the shared selection kernel
// (srb_knn_kernel) reads its query points from
extern "C" __global__ void srb12_pos_kernel(int n_agents, const double *__restrict__ x0g, double *__restrict__ pos)
{
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n_agents) return;
    const double *x = x0g + 12 * (size_t)a;
    pos[4 * (size_t)a] = x[0]; pos[4 * (size_t)a + 1] = x[6]; pos[4 * (size_t)a + 2] = x[1]; pos[4 * (size_t)a + 3] = x[7];
}
