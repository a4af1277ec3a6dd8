// Batched low-level CLF-QP controller for MI355X (gfx950): LowLevelCtrl::calcTorque
// (/root/reference/src/LowLevelCtrl.cpp:18-113) for a whole batch of agents per launch --
// QP assembly (cost :115-137, constraints :139-236), the iSWIFT interior-point solve
// (iswiftQp_e, optimization/iSWIFT/src/Prime.c:127-230), the parse (:44-64), swing-leg PD
// (:71-91), the joint-acceleration integration (:96-98) and swingInvKin (:446-488).
//
// Execution model: one 64-lane wavefront (= one workgroup) per agent.  The QP has
// n = 3c + 12 + outDim + useCLF <= 31 variables (F | tau | aux | d), p = 3c + outDim = 18
// equalities and m = 5c + 24 + useCLF <= 45 inequalities, so every variable, equality row
// and inequality row has an owner lane whose registers hold its iterate for the whole solve.
//
// Linear algebra (the iterates are iSWIFT's; only the Newton solve differs):
// iSWIFT factors the unreduced KKT [P A' G'; A 0 0; G 0 -W] by sparse LDL'.  Here dz is
// eliminated (Omega = W^-1 = z/s) and the equalities are handled by a Schur complement:
//     H = P + G' Omega G  is block diagonal by structure:
//         friction block of stance leg l (3x3, five cone rows): closed-form LDL' whose pivots
//           are sums of positive terms (no cancellation when a cone row goes stiff),
//         torque variables: diagonal (the two bound rows),
//         aux / defect variables: diag(auxPen, clfPen) + omega_clf u u', u = [LgV; -1]
//           (Sherman-Morrison; the stiff CLF row's right-hand side enters through
//            v r3 / (w + u'v), never as omega * r3);
//     Y = H^-1 A' (31 x 18), S = A Y (18 x 18, SPD), inverted by register Gauss-Jordan;
//     dy = S^-1 (A H^-1 g - r2), dx = H^-1 g - Y dy, dz = Omega (G dx - r3).
// A (18 x 31) is assembled once per agent: [Jc; H0] Dinv [Jc' B] on the VALU from LDS.
//
// Inputs/outputs are agent-major fp64 arrays in HBM (srb_ll_io, include/srbnmpc.h).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "srb_kernel_params.h"
#include "srb_wave.h"

#define NQ SRB_LL_NQ
#define NU SRB_LL_NU
#define LDJ 19      // row stride of 18-column LDS matrices (odd: no bank conflicts down a column)
#define LDA 25      // row stride of the dense (F, tau) part of A
#define ZS 63       // index of the always-zero slot of the 64-entry LDS vectors
#define SYNC() __syncthreads()

struct SrbLLDev {
    const int *ind;
    const double *q, *dq, *Dinv, *B, *Hv, *Jc, *dJc, *Js, *Jtoe, *Jhip, *toePos, *hipPos, *H0, *dH0, *y, *dy, *hd,
        *dhd, *fDes;
    double *tau, *QP_force, *ddq, *dq_out, *q_out, *V, *dV, *x;
    int *status, *iters;
};

struct LLShared {
    double D[NQ * NQ];                    // Dinv, column-major as given
    union {
        struct { double J[NQ * LDJ], K[24 * NQ], M[NQ * LDJ]; } as;   // assembly / epilogue scratch
        struct { double Y[32 * LDJ], S[NQ * LDJ]; } ip;                 // interior point
    } u;
    double A[NQ * LDA];                   // dense (F, tau) columns of A, row-major
    double vx[64], vr[64], ve[64], vg[64], vt[64];   // lane-indexed exchange vectors (slot ZS stays 0)
    double Lg[32], vv[32];                // u = [LgV; -1] and v = u / diag(auxPen, clfPen), by aux index
    double vvp[48];                       // vv shifted by 12 with zeros in front (contact rows of Y)
    double leg[4][5];                     // per stance leg: a, b, sigma, l0, l1 of the friction LDL'
    double sc[8];
};

// sum of two interleaved wave reductions (helpers from srb_wave.h)
__device__ __forceinline__ void wsum2(double &a, double &b)
{
    double v[2] = {a, b};
    wred<2, 0u>(v);
    a = v[0]; b = v[1];
}

// diagnostic trace of one agent (prm.dbg_agent): per iteration the four residual sums, mu,
// both predictor steps, sigma (8 doubles), read back by srb_ll_debug_trace
__device__ double srb_ll_dbg[512];
__device__ unsigned long long srb_ll_stamp[16];   // s_memtime cycles per phase of the traced agent
#define LLST(slot)                                                                                   \
    do {                                                                                             \
        if (dstamp) {                                                                                \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();                              \
            __builtin_amdgcn_sched_barrier(0);                                                       \
            if (lane == 0) srb_ll_stamp[slot] += t_ - tprev;                                         \
            tprev = t_;                                                                              \
        }                                                                                            \
    } while (0)

extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SRB_LL_WPE))) srb_ll_kernel(SrbLLKParams prm, int n_agents, SrbLLDev io)
{
    __shared__ LLShared sh;
    const int agent = blockIdx.x;
    if (agent >= n_agents) return;
    const int lane = threadIdx.x;
    // diagnostics: prm.dbg_agent = agent | (iteration of the state dump << 16), or -1
    const int dag = prm.dbg_agent < 0 ? -1 : (prm.dbg_agent & 0xffff), dit = prm.dbg_agent < 0 ? -1 : (prm.dbg_agent >> 16);
    const bool dstamp = agent == dag;
    unsigned long long tprev = dstamp ? __builtin_amdgcn_s_memtime() : 0ull;

    // ------------------------------------------------------------------ contact pattern (uniform)
    int ind[4], cnt = 0, bad = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        ind[i] = io.ind[4 * agent + i];
        cnt += (ind[i] == 1);
        bad |= (ind[i] != 0 && ind[i] != 1);
    }
    if (bad) {   // not a contact pattern the reference can express: FATAL, outputs untouched
        if (lane == 0) { io.status[agent] = 3; io.iters[agent] = 0; }
        return;
    }
    const int useCLF = prm.useCLF ? 1 : 0;
    const int con = 3 * cnt, out = 6 + 3 * (4 - cnt), nft = con + NU, a0 = nft;
    const int n = con + NU + out + useCLF, m = 5 * cnt + 2 * NU + useCLF;
    const int rclf = useCLF ? m - 1 : ZS;

    // stance position of each leg (order FR, FL, RR, RL), swing position likewise
    int spos[4], wpos[4];
    {
        int s = 0, w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) { spos[i] = s; wpos[i] = w; s += (ind[i] == 1); w += (ind[i] == 0); }
    }

    const size_t A18 = (size_t)agent * NQ, A12 = (size_t)agent * NU;
    const double *gD = io.Dinv + A18 * NQ, *gB = io.B + A18 * NU, *gJc = io.Jc + A12 * NQ, *gH0 = io.H0 + A18 * NQ;

    // ------------------------------------------------------------------ load + assembly
    for (int e = lane; e < 64; e += 64) {
        sh.vx[e] = 0; sh.vr[e] = 0; sh.ve[e] = 0; sh.vg[e] = 0; sh.vt[e] = 0;
    }
    // every global load of the assembly is issued before the first LDS store (one HBM round
    // trip instead of one per loop trip): Dinv, J = [Jc (con rows); H0 (out rows)] down the
    // stored columns, K = [Jc' B] (18 x nft) column by column
    {
        double tD[6], tJ[6], tK[7];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const int e = lane + 64 * i;
            const int t = e / NQ, k = e - t * NQ;
            tD[i] = (e < NQ * NQ) ? gD[e] : 0.0;
            tJ[i] = (e < NQ * NQ) ? ((k < con) ? gJc[t * NU + k] : gH0[t * NQ + (k - con)]) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int e = lane + 64 * i;
            const int v = e / NQ, t = e - v * NQ;
            tK[i] = (e < nft * NQ) ? ((v < con) ? gJc[t * NU + v] : gB[(v - con) * NQ + t]) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const int e = lane + 64 * i;
            const int t = e / NQ, k = e - t * NQ;
            if (e < NQ * NQ) { sh.D[e] = tD[i]; sh.u.as.J[k * LDJ + t] = tJ[i]; }
        }
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const int e = lane + 64 * i;
            if (e < nft * NQ) sh.u.as.K[e] = tK[i];
        }
    }
    // touch the epilogue's kinematics now so that its loads hit the caches later
    double pf = 0.0;
    {
        const double *gJs = io.Js + A12 * NQ, *gJt = io.Jtoe + A12 * NQ, *gJh = io.Jhip + A12 * NQ;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int e = lane + 64 * i;
            if (e < NU * NQ) pf += gJs[e] + gJt[e] + gJh[e];
        }
    }
    SYNC();
    // M = J Dinv (18 x 18)
    for (int e = lane; e < NQ * NQ; e += 64) {
        const int k = e / NQ, j = e - k * NQ;
        double s0 = 0, s1 = 0;
#pragma unroll
        for (int t = 0; t < NQ; t += 2) {
            s0 = fma(sh.u.as.J[k * LDJ + t], sh.D[j * NQ + t], s0);
            s1 = fma(sh.u.as.J[k * LDJ + t + 1], sh.D[j * NQ + t + 1], s1);
        }
        sh.u.as.M[k * LDJ + j] = s0 + s1;
    }
    SYNC();
    // A = M K (18 x nft); b = M Hv - dJc | (-kp y - kd dy) + M Hv - dH0 (:147-152)
    for (int e = lane; e < NQ * 24; e += 64) {     // columns nft..23 are zero padding
        const int k = e / 24, v = e - k * 24;
        double s0 = 0, s1 = 0;
#pragma unroll
        for (int t = 0; t < NQ; t += 2) {
            s0 = fma(sh.u.as.M[k * LDJ + t], sh.u.as.K[v * NQ + t], s0);
            s1 = fma(sh.u.as.M[k * LDJ + t + 1], sh.u.as.K[v * NQ + t + 1], s1);
        }
        sh.A[k * LDA + v] = (v < nft) ? s0 + s1 : 0.0;
    }
    double bk = 0.0;
    if (lane < NQ) {
        const double *hv = io.Hv + A18;
        double s0 = 0, s1 = 0;
#pragma unroll
        for (int t = 0; t < NQ; t += 2) {
            s0 = fma(sh.u.as.M[lane * LDJ + t], hv[t], s0);
            s1 = fma(sh.u.as.M[lane * LDJ + t + 1], hv[t + 1], s1);
        }
        const double mh = s0 + s1;
        if (lane < con) bk = mh - io.dJc[A12 + lane];
        else {
            const int i = lane - con;
            bk = (-prm.kp * io.y[A18 + i] - prm.kd * io.dy[A18 + i]) + mh - io.dH0[A18 + i];
        }
    }

    LLST(0);   // load + assembly
    // CLF scalars in closed form (PP = tuneMat PP0 tuneMat, eta = [y; dy], :171-235):
    //   V = eta'PP eta, LfV = eta'(FF'PP + PP FF)eta, LgV_i = 2 (Pd/e y_i + P2 dy_i)
    double Vv = 0.0, LfV = 0.0, Lgi = 0.0;
    if (useCLF && lane < out) {
        const double yi = io.y[A18 + lane], dyi = io.dy[A18 + lane];
        const double py = prm.p1e2 * yi + prm.pde * dyi, pdy = prm.pde * yi + prm.p2 * dyi;
        Vv = yi * py + dyi * pdy;
        LfV = 2.0 * (py * dyi + pdy * (-prm.kp * yi - prm.kd * dyi));
        Lgi = 2.0 * pdy;
    }
    wsum2(Vv, LfV);
    const double Veps = prm.cce * Vv;
    // u = [LgV; -1], v = u ./ diag(auxPen.., clfPen): fixed for the whole solve
    if (lane < 32) { sh.Lg[lane] = 0.0; sh.vv[lane] = 0.0; }
    if (lane < 48) sh.vvp[lane] = 0.0;
    if (lane < out) { sh.Lg[lane] = Lgi; sh.vv[lane] = Lgi / prm.auxPen; sh.vvp[12 + lane] = Lgi / prm.auxPen; }
    if (lane == out) { sh.Lg[lane] = useCLF ? -1.0 : 0.0; sh.vv[lane] = useCLF ? -1.0 / prm.clfPen : 0.0; }
    double uv = (useCLF && lane < out) ? Lgi * (Lgi / prm.auxPen) : 0.0;
    double dummy = 0.0;
    wsum2(uv, dummy);
    uv += useCLF ? 1.0 / prm.clfPen : 0.0;
    if (pf == 1.2345e300) sh.sc[7] = pf;   // never true: keeps the cache-warming loads
    SYNC();

    // ------------------------------------------------------------------ lane roles
    // variable lane j < n: type 0 F (stance leg lf, axis af), 1 tau, 2 aux, 3 defect d
    const bool isv = lane < n;
    const int vtype = (lane < con) ? 0 : (lane < nft) ? 1 : (lane < nft + out) ? 2 : 3;
    const int lf = lane / 3, af = lane - 3 * (lane / 3);
    double Pj = 0.0, cj = 0.0;
    if (isv) {
        Pj = (vtype == 0) ? prm.dfPen : (vtype == 1) ? prm.tauPen : (vtype == 2) ? prm.auxPen : prm.clfPen;
        if (vtype == 0) {
            int leg = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) if (ind[i] == 1 && spos[i] == lf) leg = i;
            cj = -io.fDes[A12 + 3 * leg + af] * prm.dfPen;   // c = -Fd dfPen (:126-136)
        }
    }
    // G' columns: up to five (row, coefficient) pairs per variable
    int gti[5] = {ZS, ZS, ZS, ZS, ZS};
    double gtc[5] = {0, 0, 0, 0, 0};
    if (isv && vtype == 0) {
        const double mus = prm.mus;
#pragma unroll
        for (int q = 0; q < 5; q++) gti[q] = 5 * lf + q;
        gtc[0] = (af == 0) ? 1.0 : (af == 2) ? -mus : 0.0;
        gtc[1] = (af == 0) ? -1.0 : (af == 2) ? -mus : 0.0;
        gtc[2] = (af == 1) ? 1.0 : (af == 2) ? -mus : 0.0;
        gtc[3] = (af == 1) ? -1.0 : (af == 2) ? -mus : 0.0;
        gtc[4] = (af == 2) ? -1.0 : 0.0;
    }
    if (isv && vtype == 1) {
        gti[0] = 5 * cnt + (lane - con); gtc[0] = 1.0;
        gti[1] = 5 * cnt + NU + (lane - con); gtc[1] = -1.0;
    }
    if (isv && vtype >= 2) { gti[0] = rclf; gtc[0] = (vtype == 2) ? sh.Lg[lane - a0] : -1.0; }
    // aux / defect lane: D_j, v_j
    const double Dj = (vtype == 2) ? prm.auxPen : prm.clfPen, iDj = 1.0 / Dj;
    const double vj = (isv && vtype >= 2) ? sh.vv[lane - a0] : 0.0;

    // inequality lane r < m: three-term row (friction, torque bounds) or the CLF row
    const bool isr = lane < m;
    int gri[3] = {ZS, ZS, ZS};
    double grc[3] = {0, 0, 0};
    double hr = 0.0;
    const bool isclf = useCLF && lane == m - 1;
    if (isr && !isclf) {
        if (lane < 5 * cnt) {
            const int l = lane / 5, qq = lane - 5 * l;
            gri[0] = 3 * l; gri[1] = 3 * l + 1; gri[2] = 3 * l + 2;
            grc[0] = (qq == 0) ? 1.0 : (qq == 1) ? -1.0 : 0.0;
            grc[1] = (qq == 2) ? 1.0 : (qq == 3) ? -1.0 : 0.0;
            grc[2] = (qq == 4) ? -1.0 : -prm.mus;
        } else {
            const int i = (lane - 5 * cnt) % NU;
            const bool up = lane < 5 * cnt + NU;
            gri[0] = con + i; grc[0] = up ? 1.0 : -1.0;
            hr = (i % 3 == 0) ? 22.0 : 50.0;                 // sat = {22, 50, 50} (LowLevelCtrl.hpp:35)
        }
    }
    if (isclf) hr = -LfV - Veps;                             // (:233)
    // equality lane k < 18
    const bool ise = lane < NQ;
    // upper-triangle entries e = lane + 64 t of S -> (j << 8 | k), row-major
    int sjk[3] = {0, 0, 0};
#pragma unroll
    for (int t = 0; t < 3; t++) {
        int j = 0, rem = lane + 64 * t;
        for (int q = 0; q < NQ; q++)
            if (rem >= NQ - j) { rem -= NQ - j; j++; }
        sjk[t] = (j << 8) | (j + rem);
    }

    // G x for the inequality lanes from an LDS vector (var-indexed)
    auto grow = [&](const double *vec) -> double {
        double g = grc[0] * vec[gri[0]] + grc[1] * vec[gri[1]] + grc[2] * vec[gri[2]];
        if (isclf) {
            double s0 = 0.0;
#pragma unroll
            for (int i = 0; i <= NQ; i++) s0 = fma(sh.Lg[i], vec[a0 + i], s0);   // Lg is 0 beyond outDim+useCLF
            g = s0;
        }
        return g;
    };
    // G' t for the variable lanes from an LDS vector (row-indexed)
    auto gtcol = [&](const double *t) -> double {
        double g = 0.0;
#pragma unroll
        for (int k = 0; k < 5; k++) g = fma(gtc[k], t[gti[k]], g);
        return g;
    };
    // A x (equality lanes), x var-indexed in LDS
    auto arow = [&](const double *vec) -> double {
        double s0 = 0.0, s1 = 0.0;
        const int k = ise ? lane : 0;
#pragma unroll 4
        for (int v = 0; v < 24; v += 2) {            // A is zero-padded to 24 columns
            s0 = fma(sh.A[k * LDA + v], vec[v], s0);
            s1 = fma(sh.A[k * LDA + v + 1], vec[v + 1], s1);
        }
        return s0 + s1 + ((k >= con) ? vec[a0 + k - con] : 0.0);
    };
    // A' y (variable lanes), y eq-indexed in LDS
    auto acol = [&](const double *yv) -> double {
        if (vtype <= 1) {
            const int j = isv ? lane : 0;
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int k = 0; k < NQ; k += 2) {
                s0 = fma(sh.A[k * LDA + j], yv[k], s0);
                s1 = fma(sh.A[(k + 1) * LDA + j], yv[k + 1], s1);
            }
            return s0 + s1;
        }
        return (vtype == 2) ? yv[con + lane - a0] : 0.0;
    };

    // ------------------------------------------------------------------ factor: H, Y, S, S^-1
    double fl0 = 0, fl1 = 0, fisg = 0, fia = 0, fla = 0, hinv = 0, gam = 0;
    // component af of H_l^-1 g for the friction block of leg l by LDL' substitution
    // (L = [1 0 0; 0 1 0; -l0 -l1 1], D = diag(a, b, sigma)): backward stable when a cone row
    // is stiff, unlike a product with the explicit 3x3 inverse
    auto fsolve = [&](double g0, double g1, double g2) -> double {
        const double u2 = (g2 + fl0 * g0 + fl1 * g1) * fisg;
        const double ga = (af == 0) ? g0 : g1;
        return fma(fla, u2, ga * fia);
    };
    // om: inverse weights z/s of every inequality row, in sh.vt (row-indexed); wc = s/z of the CLF row
    auto factor = [&](double wc) -> int {
        // friction LDL' per stance leg: H = [a 0 p; 0 b q; p q c]
        if (lane < cnt) {
            const double *om = sh.vt + 5 * lane;
            const double w0 = om[0], w1 = om[1], w2 = om[2], w3 = om[3], w4 = om[4], d = prm.dfPen, mu = prm.mus;
            const double a = d + w0 + w1, b = d + w2 + w3;
            const double sig = d + w4 + mu * mu * (d * (w0 + w1) + 4.0 * w0 * w1) / a +
                               mu * mu * (d * (w2 + w3) + 4.0 * w2 * w3) / b;
            double *L = sh.leg[lane];
            L[0] = a; L[1] = b; L[2] = sig; L[3] = -mu * (w1 - w0) / a; L[4] = -mu * (w3 - w2) / b;
        }
        LLST(1);
        gam = useCLF ? 1.0 / (wc + uv) : 0.0;
        if (vtype == 1 && isv) hinv = 1.0 / (prm.tauPen + sh.vt[gti[0]] + sh.vt[gti[1]]);
        SYNC();
        if (vtype == 0 && isv) {   // leg block LDL' factors for the substitution in fsolve
            const double *L = sh.leg[lf];
            fl0 = L[3]; fl1 = L[4]; fisg = 1.0 / L[2];
            fia = (af == 0) ? 1.0 / L[0] : (af == 1) ? 1.0 / L[1] : 0.0;
            fla = (af == 0) ? fl0 : (af == 1) ? fl1 : 1.0;
        }
        LLST(2);   // friction LDL' pieces
        // Y row j = (H^-1 A')_j (18 entries)
        if (isv) {
            double *Yj = sh.u.ip.Y + lane * LDJ;
            if (vtype == 0) {
                const int c0 = 3 * lf;
#pragma unroll
                for (int k = 0; k < NQ; k++)
                    Yj[k] = fsolve(sh.A[k * LDA + c0], sh.A[k * LDA + c0 + 1], sh.A[k * LDA + c0 + 2]);
            } else if (vtype == 1) {
#pragma unroll
                for (int k = 0; k < NQ; k++) Yj[k] = sh.A[k * LDA + lane] * hinv;
            } else {
                // branch-free: vvp[12 + kk] is v_kk for output rows kk >= 0 and 0 on the contact rows
                const int i = lane - a0;
                const double gv = gam * vj;
                double vk[NQ];
#pragma unroll
                for (int k = 0; k < NQ; k++) vk[k] = sh.vvp[12 + k - con];
#pragma unroll
                for (int k = 0; k < NQ; k++) Yj[k] = fma(-gv, vk[k], (k - con == i) ? iDj : 0.0);
            }
        }
        SYNC();
        LLST(3);   // Y
        // S = A Y, upper triangle spread over the wave (171 entries)
#pragma unroll 1
        for (int t = 0; t < 3; t++) {
            const int e = lane + 64 * t;
            if (e >= NQ * (NQ + 1) / 2) break;
            const int jk = (t == 0) ? sjk[0] : (t == 1) ? sjk[1] : sjk[2];
            const int j = (jk >> 8), k = jk & 255;
            double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
            for (int v = 0; v < 24; v += 2) {
                s0 = fma(sh.A[j * LDA + v], sh.u.ip.Y[v * LDJ + k], s0);
                s1 = fma(sh.A[j * LDA + v + 1], sh.u.ip.Y[(v + 1) * LDJ + k], s1);
            }
            double s = s0 + s1;
            if (j >= con) s += sh.u.ip.Y[(a0 + j - con) * LDJ + k];
            sh.u.ip.S[j * LDJ + k] = s;
            sh.u.ip.S[k * LDJ + j] = s;
        }
        SYNC();
        LLST(4);   // S
        const int i = ise ? lane : 0;
        double Si[NQ];
#pragma unroll
        for (int j = 0; j < NQ; j++) Si[j] = ise ? sh.u.ip.S[i * LDJ + j] : ((lane == j) ? 1.0 : 0.0);
        const int gjf = gj_invert<NQ>(Si, NQ, lane, 0);
        // S^-1 goes back to LDS (row per equality lane): 36 VGPRs kept free across the loop
        if (ise) {
#pragma unroll
            for (int j = 0; j < NQ; j++) sh.u.ip.S[i * LDJ + j] = Si[j];
        }
        LLST(5);   // Gauss-Jordan
        return gjf;
    };

    // ------------------------------------------------------------------ Newton solve
    // [P A' G'; A 0 0; G 0 -W] [dx; dy; dz] = [r1; r2; r3]; om_r = z/s per row (register)
    auto kkt_solve = [&](double r1, double r2, double r3, double om, double &dx, double &dy, double &dz) {
        // t = Omega r3 (rows); the CLF row's r3 itself goes to sc[0]
        if (isr) sh.vr[lane] = om * r3;
        if (isclf) sh.sc[0] = r3;
        SYNC();
        double g = r1 + gtcol(sh.vr);
        double uj = 0.0;
        // aux / defect: u = g1 / D + gam v (r3c - v'g1), g1 = r1 (aux rows of G' are the CLF row only)
        double vg = (isv && vtype >= 2) ? vj * r1 : 0.0, d0 = 0.0;
        wsum2(vg, d0);
        if (isv) sh.vg[lane] = g;
        SYNC();
        if (isv) {
            if (vtype == 0) {
                const int c0 = 3 * lf;
                uj = fsolve(sh.vg[c0], sh.vg[c0 + 1], sh.vg[c0 + 2]);
            } else if (vtype == 1) {
                uj = g * hinv;
            } else {
                uj = r1 * iDj + gam * vj * (sh.sc[0] - vg);
            }
            sh.vx[lane] = uj;
        }
        SYNC();
        // rhs = A u - r2 -> dy = S^-1 rhs
        if (ise) sh.ve[lane] = arow(sh.vx) - r2;
        SYNC();
        double dyk = 0.0;
        if (ise) {
            const double *Sr = sh.u.ip.S + lane * LDJ;
#pragma unroll
            for (int j = 0; j < NQ; j++) dyk = fma(Sr[j], sh.ve[j], dyk);
        }
        SYNC();
        if (ise) sh.ve[lane] = dyk;
        SYNC();
        // dx = u - Y dy
        double dxj = uj;
        if (isv) {
            const double *Yj = sh.u.ip.Y + lane * LDJ;
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int k = 0; k < NQ; k += 2) { s0 = fma(Yj[k], sh.ve[k], s0); s1 = fma(Yj[k + 1], sh.ve[k + 1], s1); }
            dxj = uj - (s0 + s1);
        }
        SYNC();
        if (isv) sh.vx[lane] = dxj;
        SYNC();
        dx = isv ? dxj : 0.0;
        dy = ise ? dyk : 0.0;
        dz = isr ? (grow(sh.vx) - r3) * om : 0.0;
        SYNC();
    };

    // ------------------------------------------------------------------ kkt_initialize (Auxilary.c:680-755)
    int flag = 3, it = 0;
    double xj = 0.0, yk = 0.0, s = 0.0, z = 0.0;
    if (isr) sh.vt[lane] = 1.0;
    SYNC();
    if (factor(1.0)) {
        flag = 1;
    } else {
        double dzt;
        kkt_solve(isv ? -cj : 0.0, ise ? bk : 0.0, isr ? hr : 0.0, isr ? 1.0 : 0.0, xj, yk, dzt);
        if (isv) sh.vx[lane] = xj;
        SYNC();
        const double zi = isr ? hr - grow(sh.vx) : 0.0;
        double mm[2] = {isr ? -zi : -1e300, isr ? zi : -1e300};   // max(-zi) = -min(zi), max(zi)
        wred<2, 3u>(mm);
        const double ap = mm[0], ad = mm[1];
        s = isr ? ((ap < 0) ? zi : zi + (1 + ap)) : 1.0;
        z = isr ? ((ad < 0) ? -zi : -zi + (1 + ad)) : 1.0;
        flag = 2;
        SYNC();

        double omf = 0.0;
        const double th = prm.tol / sqrt(3.0);
        const double invm = 1.0 / (double)m;
        for (int iter = 0; iter < prm.maxit; iter++) {
            // residuals (computeresiduals, Auxilary.c:524-553)
            if (isv) sh.vx[lane] = xj;
            if (ise) sh.ve[lane] = yk;
            const double iz = isr ? 1.0 / z : 0.0, is_ = isr ? 1.0 / s : 0.0;
            if (isr) { sh.vr[lane] = z; sh.vt[lane] = z * is_; }
            if (isclf) sh.sc[1] = s * iz;
            SYNC();
            const double rx = isv ? -Pj * xj - cj - gtcol(sh.vr) - acol(sh.ve) : 0.0;
            const double ry = ise ? bk - arow(sh.vx) : 0.0;
            const double rz = isr ? hr - s - grow(sh.vx) : 0.0;
            const double lam = isr ? sqrt(s * z) : 0.0;
            const bool dbs = agent == dag && iter == dit;   // state dump at iteration dit
            if (dbs) {
                if (isv) srb_ll_dbg[256 + lane] = xj;
                if (ise) srb_ll_dbg[288 + lane] = yk;
                if (isr) { srb_ll_dbg[306 + lane] = s; srb_ll_dbg[352 + lane] = z; }
            }
            double nr[5] = {rx * rx, ry * ry, rz * rz, isr ? s * z : 0.0, lam * lam};
            wred<5, 0u>(nr);
            LLST(10);  // residuals + norms
            if (sqrt(nr[0]) < th && sqrt(nr[2]) < th && sqrt(nr[1]) < th && nr[3] * invm < prm.tol) { flag = 0; break; }
            const double mu = nr[4] * invm;
            const bool dbg = agent == dag && lane == 0 && iter < 32;
            if (dbg) { for (int q = 0; q < 5; q++) srb_ll_dbg[8 * iter + q] = nr[q]; }
            double ds, dx, dy, dz, dsv, st[2], alp, ald;
            // updatekktmatrix + kktsolve_1 (Prime.c:165-192): refactor at the current weights.
            // iSWIFT's sigma <= sigma_d branch (Prime.c:193-196: the factor is frozen for the rest
            // of the solve) is not taken: the step-length rule keeps every factor of rho's products
            // >= 0, so sigma = 0 arises only from rounding at a blocking row
            omf = isr ? sh.vt[lane] : 0.0;
            if (factor(sh.sc[1])) { flag = 1; break; }
            // predictor
            ds = -lam * lam;
            kkt_solve(rx, ry, isr ? rz - ds * iz : 0.0, omf, dx, dy, dz);
            LLST(6);   // predictor solve
            dsv = isr ? (ds - s * dz) * iz : 0.0;
            st[0] = (isr && dsv < 0) ? s / dsv : -1e300;   // max(v/dv) = -min(-v/dv) (findsteplength)
            st[1] = (isr && dz < 0) ? z / dz : -1e300;
            wred<2, 3u>(st);
            alp = (-st[0] < 1e10) ? -st[0] : 1.0;
            ald = (-st[1] < 1e10) ? -st[1] : 1.0;
            {
                double num = isr ? (s + alp * dsv) * (z + ald * dz) : 0.0, d1 = 0.0;
                wsum2(num, d1);
                const double rho = num / nr[3];
                const double mr = rho < 1 ? rho : 1;
                double sigma = mr * mr * mr;
                if (sigma < 0.0) sigma = 0.0;                   // sigma_d = 0 (iswift_qp.cpp:103)
                ds = -(lam * lam) - (dsv * dz) + sigma * mu;
                if (dbg) { srb_ll_dbg[8 * iter + 5] = alp; srb_ll_dbg[8 * iter + 6] = ald; srb_ll_dbg[8 * iter + 7] = sigma; }
            }
            LLST(7);   // predictor steps, rho
            // corrector (kktsolve_2)
            kkt_solve(rx, ry, isr ? rz - ds * iz : 0.0, omf, dx, dy, dz);
            LLST(8);   // corrector solve
            dsv = isr ? (ds - s * dz) * iz : 0.0;
            st[0] = (isr && dsv < 0) ? s / dsv : -1e300;
            st[1] = (isr && dz < 0) ? z / dz : -1e300;
            wred<2, 3u>(st);
            alp = (-st[0] < 1e10) ? -st[0] : 1.0;
            ald = (-st[1] < 1e10) ? -st[1] : 1.0;
            if (dbs) {
                if (isv) srb_ll_dbg[398 + lane] = dx;
                if (ise) srb_ll_dbg[430 + lane] = dy;
                if (isr) srb_ll_dbg[448 + lane] = dz;
            }
            alp = 0.99 * alp < 1.0 ? 0.99 * alp : 1.0;
            ald = 0.99 * ald < 1.0 ? 0.99 * ald : 1.0;
            xj += dx * alp;
            yk += dy * ald;
            if (isr) { s += dsv * alp; z += dz * ald; }
            it++;
            LLST(9);   // steps + update
        }
    }

    LLST(11);  // init point / loop exit
    // ------------------------------------------------------------------ parse + epilogue
    const double *gq = io.q + A18, *gdq = io.dq + A18;
    if (isv) sh.vx[lane] = xj;
    SYNC();
    if (lane < 32) io.x[(size_t)agent * 32 + lane] = isv ? xj : 0.0;
    // dV = LfV + Veps + LgV' aux (:57-63)
    double dvs = (useCLF && vtype == 2 && isv) ? sh.Lg[lane - a0] * xj : 0.0, d2 = 0.0;
    wsum2(dvs, d2);
    if (lane == 0) {
        io.V[agent] = useCLF ? Vv : 0.0;
        io.dV[agent] = useCLF ? LfV + Veps + dvs : 0.0;
        io.status[agent] = flag;
        io.iters[agent] = it;
    }
    // QP_force (12) into vg[0..11]; tau (18) into vt[0..17]
    if (lane < NU) {
        const int L = lane / 3;
        const double f = (ind[L] == 1) ? sh.vx[3 * spos[L] + lane % 3] : 0.0;
        sh.vg[lane] = f;
        io.QP_force[A12 + lane] = f;
    }
    // (each load through its own address space: the plain select had been merged into one generic-pointer
    // flat load -- the shipped code objects carry no flat memory instruction, tests/test_isa_hazard.py)
    double taut = 0.0;
    if (lane < NQ) {
        const __attribute__((address_space(1))) double *tg = (const __attribute__((address_space(1))) double *)(io.tau + A18);
        const __attribute__((address_space(3))) double *tl = (const __attribute__((address_space(3))) double *)(sh.vx + con);
        const double a = tg[lane < 6 ? lane : 0], b = tl[lane < 6 ? 0 : lane - 6];
        taut = (lane < 6) ? a : b;
    }
    const int sw = NU - con;
    double *sJs = sh.u.as.J, *sJD = sh.u.as.M, *sDl = sh.u.as.K;
    if (sw > 0) {
        // swing-leg PD (:71-91): Delta = (Js Dinv Js')^-1, Kp = wd^2 diag(Delta), Kd = 40
        const double *gJs = io.Js + A12 * NQ;
        SYNC();
        for (int e = lane; e < sw * NQ; e += 64) {
            const int t = e / sw, r = e - t * sw;
            sJs[r * LDJ + t] = gJs[t * NU + r];
        }
        SYNC();
        for (int e = lane; e < sw * NQ; e += 64) {
            const int r = e / NQ, j = e - r * NQ;
            double s0 = 0.0;
#pragma unroll
            for (int t = 0; t < NQ; t++) s0 = fma(sJs[r * LDJ + t], sh.D[j * NQ + t], s0);
            sJD[r * LDJ + j] = s0;
        }
        SYNC();
        for (int e = lane; e < sw * sw; e += 64) {
            const int r = e / sw, rr = e - r * sw;
            double s0 = 0.0;
#pragma unroll
            for (int t = 0; t < NQ; t++) s0 = fma(sJD[r * LDJ + t], sJs[rr * LDJ + t], s0);
            sDl[r * 16 + rr] = s0;
        }
        SYNC();
        double Dr[NU];
#pragma unroll
        for (int j = 0; j < NU; j++) Dr[j] = (lane < sw && j < sw) ? sDl[lane * 16 + j] : ((lane == j) ? 1.0 : 0.0);
        gj_invert<NU>(Dr, sw, lane, 0);
        double dg = 0.0;
#pragma unroll
        for (int j = 0; j < NU; j++) dg = (j == lane) ? Dr[j] : dg;
        if (lane < sw) {
            const int k = lane / 3, ax = lane - 3 * k;
            int L = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) if (ind[i] == 0 && wpos[i] == k) L = i;
            const double pd = io.hd[A18 + 6 + lane] - io.toePos[A12 + 3 * L + ax];
            const double *gJt = io.Jtoe + A12 * NQ;
            double jv = 0.0;
#pragma unroll
            for (int t = 0; t < NQ; t++) jv = fma(gJt[t * NU + 3 * L + ax], gdq[t], jv);
            const double vd = io.dhd[A18 + 6 + lane] - jv;
            sh.ve[lane] = 40.0 * 40.0 * dg * pd + 40.0 * vd;
        }
        SYNC();
        if (lane < NQ) {
            double s0 = 0.0;
            for (int r = 0; r < sw; r++) s0 = fma(sJs[r * LDJ + lane], sh.ve[r], s0);
            taut += s0;
        }
    }
    if (lane < NQ) { sh.vt[lane] = taut; io.tau[A18 + lane] = taut; }
    SYNC();
    // ddq = Dinv (B tau[6:] + Jtoe' F - H) (:96)
    double rhs = 0.0;
    if (lane < NQ) {
        const double *gJt = io.Jtoe + A12 * NQ;
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int j = 0; j < NU; j++) s0 = fma(gB[j * NQ + lane], sh.vt[6 + j], s0);
#pragma unroll
        for (int r = 0; r < NU; r++) s1 = fma(gJt[lane * NU + r], sh.vg[r], s1);
        rhs = s0 + s1 - io.Hv[A18 + lane];
        sh.vr[lane] = rhs;
    }
    SYNC();
    double ddq = 0.0, dqn = 0.0, qn = 0.0;
    if (lane < NQ) {
        double s0 = 0.0;
#pragma unroll
        for (int j = 0; j < NQ; j++) s0 = fma(sh.D[j * NQ + lane], sh.vr[j], s0);
        ddq = s0;
        dqn = gdq[lane] + ddq / 1000.0;                                  // LL_Hz = 1000 (global_loco_opts.h:22)
        qn = gq[lane] + dqn / 1000.0 + 0.5 / (1000.0 * 1000.0) * ddq;
    }
    // swingInvKin (:446-488): lane L < 4 solves its swing leg's 3x3 system; Jhip rows are taken
    // at the swing counter (:467) as in the reference
    if (sw > 0 && lane < 4 && ind[lane] == 0) {
        const int L = lane, cs = 3 * wpos[L];
        const double *gJt = io.Jtoe + A12 * NQ, *gJh = io.Jhip + A12 * NQ;
        double r[3], J[3][3];
#pragma unroll
        for (int a = 0; a < 3; a++) {
            double jv = 0.0;
            for (int t = 0; t < NQ; t++) jv = fma(gJh[t * NU + cs + a], gdq[t], jv);
            const double dxde = io.dhd[A18 + 6 + cs + a] - jv;
            const double xde = io.hd[A18 + 6 + cs + a] - io.hipPos[A12 + 3 * L + a];
            const double xe = io.toePos[A12 + 3 * L + a] - io.hipPos[A12 + 3 * L + a];
            double jt = 0.0;
#pragma unroll
            for (int b = 0; b < 3; b++) {
                jt = fma(gJt[(3 + b) * NU + 3 * L + a] - gJh[(3 + b) * NU + 3 * L + a], gdq[3 + b], jt);
                J[a][b] = gJt[(6 + 3 * L + b) * NU + 3 * L + a] - gJh[(6 + 3 * L + b) * NU + 3 * L + a];
            }
            r[a] = dxde + 20.0 * (xde - xe) - jt;
            // one row's loads at a time: hoisting all three rows' loads spilled 12 VGPRs to scratch,
            // whose write-back tripled the kernel's HBM writes
            __builtin_amdgcn_sched_barrier(0);
        }
        // Cramer's rule on the 3x3 leg block
        const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1], c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2],
                     c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
        const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02, id = 1.0 / det;
        const double v0 = (r[0] * c00 + r[1] * (J[0][2] * J[2][1] - J[0][1] * J[2][2]) + r[2] * (J[0][1] * J[1][2] - J[0][2] * J[1][1])) * id;
        const double v1 = (r[0] * c01 + r[1] * (J[0][0] * J[2][2] - J[0][2] * J[2][0]) + r[2] * (J[0][2] * J[1][0] - J[0][0] * J[1][2])) * id;
        const double v2 = (r[0] * c02 + r[1] * (J[0][1] * J[2][0] - J[0][0] * J[2][1]) + r[2] * (J[0][0] * J[1][1] - J[0][1] * J[1][0])) * id;
        sh.ve[32 + 3 * L] = v0; sh.ve[33 + 3 * L] = v1; sh.ve[34 + 3 * L] = v2;
    }
    SYNC();
    if (lane < NQ) {
        if (sw > 0 && lane >= 6 && ind[(lane - 6) / 3] == 0) {
            const double v = sh.ve[32 + lane - 6];
            dqn = v;
            qn = gq[lane] + v / 1000.0;
        }
        io.ddq[A18 + lane] = ddq;
        io.dq_out[A18 + lane] = dqn;
        io.q_out[A18 + lane] = qn;
    }
    LLST(12);  // epilogue
}

// diagnostics: select the traced agent (-1 = none) and read the previous launch's trace
static int g_dbg_agent = -1;
extern "C" int srb_ll_dbg_agent(void) { return g_dbg_agent; }
extern "C" int srb_ll_debug_stamps(unsigned long long *out, int reset)
{
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(srb_ll_stamp), 16 * sizeof(unsigned long long), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -2;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(srb_ll_stamp), z, sizeof z, 0, hipMemcpyHostToDevice) != hipSuccess) return -2;
    }
    return 0;
}
extern "C" int srb_ll_debug_trace(int agent, double *out)
{
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(srb_ll_dbg), 512 * sizeof(double), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -2;
    g_dbg_agent = agent;
    return 0;
}
