/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * SRB-12 extension mode: the batched CBF-NMPC of BASELINE.json's north star on the 12-state
 * single-rigid-body model, restated as a dense full-space solve.  The reference only DECLARES
 * this model (FastMPC::runMPC / MPC_Cost / MPC_Constraints / getLinearDynamics,
 * /root/reference/include/fast_MPC.hpp:98-103, no bodies anywhere), so there is no reference
 * output to pin: PARITY UNPINNED against the reference; the oracle is pinned by a
 * solver-independent KKT certificate (tests/kkt.py) and the GPU kernel
 * (srb-cbf-nmpc_amd/csrc/srb12_kernels.hip) is checked against this file.
 *
 * Problem (DESIGN.md section 11 states it in full):
 *   state  x = [p (3), Theta = roll/pitch/yaw (3), v (3), omega (3)], x_0 given;
 *   input  u_k = the ground reaction forces f_{k,i} of the four legs (FR, FL, RR, RL);
 *   constants: mass 12.453 kg and body inertia of FastMPC (/root/reference/src/fast_MPC.cpp:40-43),
 *     mu_MPC 0.7 and the 12-state weights q = 1e3, r = 1e-2 of the default mpc_params
 *     (/root/reference/src/Parameters.cpp:32-52), the friction pyramid of
 *     LowLevelCtrl::calcTorque (rows +-f_x - mu/sqrt2 f_z, +-f_y - mu/sqrt2 f_z, -f_z,
 *     /root/reference/src/LowLevelCtrl.cpp:158-162) plus f_z <= fmax, the slack weight 3000 and
 *     the obstacle rows -|p_k - o_kj|^2 - s <= -eps_j of the LIP mode
 *     (/root/reference/include/dec_vars_constr_cost.h:262-265,297-302, MPC_dist.cpp:176-178);
 *   dynamics: the convex-MPC linearisation about the reference yaw (forward Euler, Ts):
 *     p' = p + Ts v,  Theta' = Theta + Ts Rz(psi)^T omega,  v' = v + Ts (sum f / m + g),
 *     omega' = omega + Ts I_w^-1 sum r_i x f_i,  I_w = Rz I_b Rz^T,  r_i = foot_i - p_hat;
 *     swing legs (contact 0) have zero B columns (their forces go to 0 through the cost).
 * Algorithm (the kernel's, step for step): stage 0 = the QP without the obstacle rows, a
 * Mehrotra predictor-corrector (iSWIFT's rules: sigma = min(1, rho)^3, 0.99 step, exit
 * ||r_d|| < tol/sqrt3 max(1, ||grad f||_inf), ||r_p|| < tol/sqrt3, s'z/m < tol) from the
 * gravity-compensating start; stage 1 = the same iteration on all rows with the Lagrangian
 * Hessian (-2 z on p_x, p_y) and an inertia shift delta I when the reduced Hessian is not
 * positive definite, warm-started from the stage-0 point.
 * Linear algebra: dense LU on the full-space KKT [H + J'WJ + dI, A'; A, 0] (the kernel uses a
 * Riccati recursion), and a Cholesky of the explicitly condensed Hessian for the inertia test.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <stdio.h>
#include "oracle.h"

void orc12_params_default(orc12_params *p, int N)
{
    memset(p, 0, sizeof *p);
    p->N = N;
    p->K_obs = 3; p->K_nbr = 0;
    p->Ts = 43 * 0.001;                   /* the LIP mode's grid (MPC_dist.cpp:104): same neighbour prediction */
    p->mass = 12.4530;                    /* fast_MPC.cpp:40 */
    const double Ib[9] = {0.01683993, 8.3902e-5, 0.000597679,     /* fast_MPC.cpp:41-43 */
                          8.3902e-5, 0.056579028, 2.5134e-5,
                          0.000597679, 2.5134e-5, 0.064713601};
    memcpy(p->Ib, Ib, sizeof Ib);
    p->grav = 9.81;
    p->mu = 0.7;                          /* mpc_params.mu_MPC, Parameters.cpp:32 */
    p->fmax = 150.0;
    for (int i = 0; i < 12; i++) { p->q[i] = 1e3; p->qN[i] = 1e3; }   /* qpx..qwy, Parameters.cpp:34-45 */
    for (int i = 0; i < 3; i++) p->r[i] = 1e-2;                        /* rx, ry, rz, Parameters.cpp:50-52 */
    p->Sw = 3000.0;                       /* MPC_dist.cpp:176-178 */
    p->eps_obs = (double)1.9f; p->eps_nbr = (double)2.2f;              /* dec_vars_constr_cost.h:401-402 */
    p->tol = 1e-6; p->qp_maxit = 25; p->nlp_maxit = 50; p->use_nlp = 1;
    p->z0 = 100.0;                       /* the LIP mode's SRB_NLP_Z0: 6.9 NLP iterations on average at 64 trot agents, against 9.8 (z0 = 1) and 8.6 (10) */
    p->tol_final = 1e-8;                 /* last stage: the polish then lands on the exact optimum (round 5: 1e-9 -> 1e-8,
                                            NLP iterations 8.8 -> 8.3 (stand), 8.3 -> 7.7 (trot), polishes all accepted;
                                            below 1e-10 the kernel's Riccati steps reach their round-off floor) */
    p->polish = 1;
    p->tol_qp = 1e-3;                    /* QP stage before the NLP: 2.6 instead of 4.1 iterations, the result unchanged */
}

int orc12_nv(const orc12_params *p) { return 24 * p->N + 1; }

static void rz(double psi, double R[9])
{
    const double c = cos(psi), s = sin(psi);
    R[0] = c; R[1] = -s; R[2] = 0; R[3] = s; R[4] = c; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
}

static void inv3(const double M[9], double X[9])
{
    const double a = M[0], b = M[1], c = M[2], d = M[3], e = M[4], f = M[5], g = M[6], h = M[7], i = M[8];
    const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
    const double det = a * A + b * B + c * C, r = 1.0 / det;
    X[0] = A * r; X[1] = -(b * i - c * h) * r; X[2] = (b * f - c * e) * r;
    X[3] = B * r; X[4] = (a * i - c * g) * r; X[5] = -(a * f - c * d) * r;
    X[6] = C * r; X[7] = -(a * h - b * g) * r; X[8] = (a * e - b * d) * r;
}

/* per-stage A_k, B_k (row-major 12x12) and c_k (12); the kernel's srb12_stage_model, same order of
 * operations where it matters (products of the 3x3 blocks) */
void orc12_dynamics(const orc12_params *p, const double x0[12], const double *xref, const double *foot,
                    const int *contact, double *A, double *B, double *c)
{
    const int N = p->N;
    const double Ts = p->Ts;
    for (int k = 0; k < N; k++) {
        const double *ph = (k == 0) ? x0 : xref + 12 * (k - 1);
        const double psi = ph[5];
        double R[9], T[9], Iw[9], Iwi[9];
        rz(psi, R);
        for (int i = 0; i < 3; i++)            /* T = Rz Ib */
            for (int j = 0; j < 3; j++) T[3 * i + j] = R[3 * i] * p->Ib[j] + R[3 * i + 1] * p->Ib[3 + j] + R[3 * i + 2] * p->Ib[6 + j];
        for (int i = 0; i < 3; i++)            /* Iw = T Rz' */
            for (int j = 0; j < 3; j++) Iw[3 * i + j] = T[3 * i] * R[3 * j] + T[3 * i + 1] * R[3 * j + 1] + T[3 * i + 2] * R[3 * j + 2];
        inv3(Iw, Iwi);
        double *Ak = A + 144 * k, *Bk = B + 144 * k, *ck = c + 12 * k;
        memset(Ak, 0, sizeof(double) * 144); memset(Bk, 0, sizeof(double) * 144); memset(ck, 0, sizeof(double) * 12);
        for (int i = 0; i < 12; i++) Ak[13 * i] = 1.0;
        for (int i = 0; i < 3; i++) {
            Ak[12 * i + 6 + i] = Ts;
            for (int j = 0; j < 3; j++) Ak[12 * (3 + i) + 9 + j] = Ts * R[3 * j + i];      /* Ts Rz' */
        }
        for (int l = 0; l < 4; l++) {
            if (!contact[4 * k + l]) continue;
            const double *fp = foot + 12 * k + 3 * l;
            const double r0 = fp[0] - ph[0], r1 = fp[1] - ph[1], r2 = fp[2] - ph[2];
            const double S[9] = {0, -r2, r1, r2, 0, -r0, -r1, r0, 0};               /* [r]x */
            for (int i = 0; i < 3; i++) {
                Bk[12 * (6 + i) + 3 * l + i] = Ts / p->mass;
                for (int j = 0; j < 3; j++)
                    Bk[12 * (9 + i) + 3 * l + j] = Ts * (Iwi[3 * i] * S[j] + Iwi[3 * i + 1] * S[3 + j] + Iwi[3 * i + 2] * S[6 + j]);
            }
        }
        ck[8] = -Ts * p->grav;
    }
}

/* ------------------------------------------------------------------------------------------ IPM */
typedef struct {
    int N, n, p, mlin, mc;          /* variables, equalities, linear rows, obstacle rows */
    const orc12_params *prm;
    double *Pd, *cv;                /* cost diagonal and linear term */
    double *Aeq, *beq;              /* p x n, p */
    double *G, *h;                  /* mlin x n, mlin */
    const double *obs, *eps;        /* [N][K][2], [K] */
    int K;
    double *T;                      /* condensation: X = T U + xbar (12N x 12N) */
} p12_t;

/* row values g(z) (linear rows then obstacle rows), and the Jacobian J (m x n dense) */
static void rows_eval(const p12_t *P, const double *z, int nl, double *g, double *J)
{
    const int n = P->n, m = P->mlin + (nl ? P->mc : 0);
    if (J) memset(J, 0, sizeof(double) * (size_t)m * n);
    for (int r = 0; r < P->mlin; r++) {
        double v = 0;
        for (int j = 0; j < n; j++) v += P->G[(size_t)r * n + j] * z[j];
        g[r] = v;
        if (J) memcpy(J + (size_t)r * n, P->G + (size_t)r * n, sizeof(double) * n);
    }
    if (!nl) return;
    for (int k = 0; k < P->N; k++)
        for (int j = 0; j < P->K; j++) {
            const int r = P->mlin + k * P->K + j;
            const double dx = z[12 * k] - P->obs[2 * (k * P->K + j)], dy = z[12 * k + 1] - P->obs[2 * (k * P->K + j) + 1];
            g[r] = -(dx * dx + dy * dy) - z[n - 1];
            if (J) { J[(size_t)r * n + 12 * k] = -2 * dx; J[(size_t)r * n + 12 * k + 1] = -2 * dy; J[(size_t)r * n + n - 1] = -1.0; }
        }
}

static double h_of(const p12_t *P, int r) { return r < P->mlin ? P->h[r] : -P->eps[(r - P->mlin) % P->K]; }

/* Cholesky of the condensed Hessian Zb' Hf Zb (Zb: the null space of the dynamics) */
static int reduced_pd(const p12_t *P, const double *Hf)
{
    const int N = P->N, n = P->n, nu = 12 * N, nz = nu + 1;
    double *Zb = calloc((size_t)n * nz, sizeof(double)), *HZ = malloc(sizeof(double) * (size_t)n * nz);
    double *Hr = malloc(sizeof(double) * (size_t)nz * nz);
    for (int i = 0; i < nu; i++) for (int j = 0; j < nu; j++) Zb[(size_t)i * nz + j] = P->T[(size_t)i * nu + j];
    for (int i = 0; i < nu; i++) Zb[(size_t)(nu + i) * nz + i] = 1.0;
    Zb[(size_t)(n - 1) * nz + nu] = 1.0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < nz; j++) {
            double v = 0;
            for (int l = 0; l < n; l++) v += Hf[(size_t)i * n + l] * Zb[(size_t)l * nz + j];
            HZ[(size_t)i * nz + j] = v;
        }
    for (int i = 0; i < nz; i++)
        for (int j = 0; j < nz; j++) {
            double v = 0;
            for (int l = 0; l < n; l++) v += Zb[(size_t)l * nz + i] * HZ[(size_t)l * nz + j];
            Hr[(size_t)i * nz + j] = v;
        }
    const int ok = orc_chol(nz, Hr) == 0;
    free(Zb); free(HZ); free(Hr);
    return ok;
}

/* ---------------------------------------------------------------------------- active-set polish
 * The last stage's OPTIMAL iterate is polished to the exact KKT point of its active set (the LIP
 * mode's rule, oracle/nlp_ipm.c `polish`, restated for this problem; the kernel does the same steps
 * with its Riccati recursion).  Rows with s KAPPA < z form the active set A; min f s.t. dynamics,
 * g_A(x) = h_A is solved by Newton steps on the augmented Lagrangian
 *   (H_L + RHO J_A'J_A) dx = -(grad f + J_A'(z_A + RHO c_A)),
 *   z_A += RHO (c_A + J_A dx)
 * (H_L: the cost Hessian and -2 y on (p_x, p_y) of active obstacle rows, y = z_A + RHO c_A the current
 * multiplier estimate).  At most IT steps per
 * pass (fewer once |dx| <= DXTOL); accepted when every row holds to PTOL, the active rows to PTOL,
 * z_A >= -1e-9 max|z_A|, the last step is <= DXTOL and the dynamics hold to DYNTOL; otherwise the most negative multiplier
 * leaves A, violated rows join and the next pass starts again from the interior-point point (at most
 * PASSES).  The steps after a pass's first reuse its factor (the kernel's rule: one Riccati factor per
 * pass; measured no different in acceptance or accuracy from refactoring every step).  Unlike the LIP
 * polish there is no proximal term on the inactive rows: the cost alone (q, r > 0) makes the matrix
 * definite, and a proximal weight the size of r = 1e-2 slowed the Newton iteration to a crawl.  Why: the forces are pinned by the friction rows and the r = 1e-2 weight alone along the
 * legs' internal-force directions, so an interior-point iterate at s'z/m ~ 1e-9 still sits up to
 * 1e-3 N from the optimum there; the active set's KKT point is exact. */
#define ORC12_POL_RHO 1e9
#define ORC12_POL_KAPPA 1e4
#define ORC12_POL_IT 8
#define ORC12_POL_PASSES 4
#define ORC12_POL_PTOL 1e-9
#define ORC12_POL_DXTOL 1e-7
#define ORC12_POL_DYNTOL 1e-8        /* max |x_{k+1} - A_k x_k - B_k u_k - c_k| of an accepted point */

/* diagnostics for the tests: polishes rejected, accepted, Newton steps in all, most steps of one solve */
int orc12_polish_stats[4];

/* returns 1 (accepted: x replaced by the polished point) or 0; *steps: Newton steps taken */
static int polish12(const p12_t *P, int nl, double *x, const double *s, const double *zd, int *steps)
{
    const int n = P->n, p = P->p, m = P->mlin + (nl ? P->mc : 0), nk = n + p;
    double *xt = malloc(sizeof(double) * n), *g = malloc(sizeof(double) * (m ? m : 1));
    double *J = malloc(sizeof(double) * (size_t)(m ? m : 1) * n), *za = malloc(sizeof(double) * (m ? m : 1));
    double *Hf = malloc(sizeof(double) * (size_t)n * n), *KK = malloc(sizeof(double) * (size_t)nk * nk);
    double *rhs = malloc(sizeof(double) * nk);
    int *act = malloc(sizeof(int) * (m ? m : 1)), *piv = malloc(sizeof(int) * nk);
    int accepted = 0;
    *steps = 0;
    for (int r = 0; r < m; r++) { act[r] = s[r] * ORC12_POL_KAPPA < zd[r]; za[r] = act[r] ? zd[r] : 0.0; }
    for (int pass = 0; pass < ORC12_POL_PASSES && !accepted; pass++) {
        memcpy(xt, x, sizeof(double) * n);
        double lastdx = 1e300;
        int bad = 0;
        for (int it = 0; it < ORC12_POL_IT; it++) {
            rows_eval(P, xt, nl, g, J);
            /* converged: a last step <= DXTOL that left the active rows within PTOL (the kernel, same rule;
             * under the pass's frozen factor a small step can leave |c_A| above PTOL, then one more step) */
            if (it > 0 && lastdx <= ORC12_POL_DXTOL) {
                double cm = 0.0;
                for (int r = 0; r < m; r++) if (act[r]) cm = fmax(cm, fabs(g[r] - h_of(P, r)));
                if (cm <= ORC12_POL_PTOL) break;
            }
            memset(Hf, 0, sizeof(double) * (size_t)n * n);
            for (int i = 0; i < n; i++) { Hf[(size_t)i * n + i] = P->Pd[i]; rhs[i] = -(P->Pd[i] * xt[i] + P->cv[i]); }
            for (int r = 0; r < m; r++) {
                const double *Jr = J + (size_t)r * n;
                const double c = g[r] - h_of(P, r);
                const double w = act[r] ? ORC12_POL_RHO : 0.0;
                const double y = act[r] ? za[r] + ORC12_POL_RHO * c : 0.0;
                if (act[r] && r >= P->mlin) {           /* -2 y on (p_x, p_y) of the row's grid, y = z_A + RHO c_A */
                    const int k = (r - P->mlin) / P->K;
                    Hf[(size_t)(12 * k) * n + 12 * k] -= 2.0 * y; Hf[(size_t)(12 * k + 1) * n + 12 * k + 1] -= 2.0 * y;
                }
                for (int i = 0; i < n; i++) {
                    if (Jr[i] == 0.0) continue;
                    rhs[i] -= Jr[i] * y;
                    for (int j = 0; j < n; j++) if (Jr[j] != 0.0) Hf[(size_t)i * n + j] += w * Jr[i] * Jr[j];
                }
            }
            const int frz = it > 0;          /* later steps of a pass reuse the first step's factor */
            if (!frz && !reduced_pd(P, Hf)) { bad = 1; break; }          /* the kernel's Riccati pivots fail there */
            if (!frz) memset(KK, 0, sizeof(double) * (size_t)nk * nk);
            if (!frz) for (int i = 0; i < n; i++) memcpy(KK + (size_t)i * nk, Hf + (size_t)i * n, sizeof(double) * n);
            for (int r = 0; r < p; r++) {
                double v = -P->beq[r];
                for (int j = 0; j < n; j++) {
                    if (!frz) { KK[(size_t)(n + r) * nk + j] = P->Aeq[(size_t)r * n + j]; KK[(size_t)j * nk + n + r] = P->Aeq[(size_t)r * n + j]; }
                    v += P->Aeq[(size_t)r * n + j] * xt[j];
                }
                rhs[n + r] = -v;
            }
            if (!frz && orc_lu(nk, KK, piv) != 0) { bad = 1; break; }
            orc_lu_solve(nk, KK, piv, rhs);
            double mdx = 0.0;
            for (int r = 0; r < m; r++)
                if (act[r]) {
                    const double *Jr = J + (size_t)r * n;
                    double jd = 0.0;
                    for (int i = 0; i < n; i++) if (Jr[i] != 0.0) jd += Jr[i] * rhs[i];
                    za[r] += ORC12_POL_RHO * (g[r] - h_of(P, r) + jd);
                }
            for (int i = 0; i < n; i++) { xt[i] += rhs[i]; mdx = fmax(mdx, fabs(rhs[i])); }
            (*steps)++;
            lastdx = mdx;
            if (getenv("ORC12_TRACE")) fprintf(stderr, "        polish step %d |dx| %.3e\n", it, mdx);
        }
        if (bad) break;
        /* acceptance at the polished point */
        rows_eval(P, xt, nl, g, NULL);
        double pv = -1e300, cv = 0.0, nzmin = -1e300, zm = 1.0;
        for (int r = 0; r < m; r++) {
            const double v = g[r] - h_of(P, r);
            pv = fmax(pv, v);
            if (act[r]) { cv = fmax(cv, fabs(v)); nzmin = fmax(nzmin, -za[r]); zm = fmax(zm, fabs(za[r])); }
        }
        /* and the dynamics: the rows alone would pass a point the Newton steps carried off them (the
         * kernel's SRB12_POL_DYNTOL test; the LU step keeps them to round-off here) */
        double dres = 0.0;
        for (int r = 0; r < p; r++) {
            double v = -P->beq[r];
            for (int j = 0; j < n; j++) v += P->Aeq[(size_t)r * n + j] * xt[j];
            dres = fmax(dres, fabs(v));
        }
        if (getenv("ORC12_TRACE"))
            fprintf(stderr, "      polish pass %d: primal %.2e |c_A| %.2e -min z_A %.2e last dx %.2e dyn %.2e\n", pass, pv, cv, nzmin, lastdx, dres);
        if (pv <= ORC12_POL_PTOL && cv <= ORC12_POL_PTOL && nzmin <= 1e-9 * zm && lastdx <= ORC12_POL_DXTOL &&
            dres <= ORC12_POL_DYNTOL) {
            memcpy(x, xt, sizeof(double) * n);
            accepted = 1;
            break;
        }
        /* next pass: the most negative multiplier leaves, violated rows join (multiplier 0) */
        int wk = -1;
        double wd = -1e-9 * zm;
        for (int r = 0; r < m; r++) if (act[r] && za[r] < wd) { wd = za[r]; wk = r; }
        int changed = 0;
        for (int r = 0; r < m; r++) {
            if (r == wk) { act[r] = 0; changed = 1; }
            else if (!act[r] && g[r] - h_of(P, r) > ORC12_POL_PTOL) { act[r] = 1; changed = 1; }
            za[r] = act[r] ? fmax(za[r], 0.0) : 0.0;
        }
        if (!changed) break;
    }
    free(xt); free(g); free(J); free(za); free(Hf); free(KK); free(rhs); free(act); free(piv);
    return accepted;
}

/* one interior-point stage; z (n), lam (p) in/out; returns 0 OPTIMAL, 1 KKTFAIL, 2 MAXIT, 3 FATAL, and for the
 * polished last stage 4 ACCEPTABLE (met tol_final, polish rejected) */
static int ipm(const p12_t *P, int nl, double *z, double *lam, int *iters)
{
    const orc12_params *prm = P->prm;
    const int n = P->n, p = P->p, m = P->mlin + (nl ? P->mc : 0), nk = n + p;
    /* a QP stage that the NLP follows runs to tol_qp (its point is only the NLP's warm start); the last
     * stage (the NLP, or the QP alone) ends at s'z/m < tol_final: the forces' accuracy */
    const double tol = (!nl && prm->use_nlp && prm->tol_qp > 0.0) ? prm->tol_qp : prm->tol, th = tol / sqrt(3.0);
    const double mtol = (nl || !prm->use_nlp) ? prm->tol_final : tol;
    double *g = malloc(sizeof(double) * m), *J = malloc(sizeof(double) * (size_t)m * n);
    double *s = malloc(sizeof(double) * m), *zd = malloc(sizeof(double) * m);
    double *rd = malloc(sizeof(double) * n), *rp = malloc(sizeof(double) * m), *req = malloc(sizeof(double) * p);
    double *Hf = malloc(sizeof(double) * (size_t)n * n), *KK = malloc(sizeof(double) * (size_t)nk * nk);
    double *rhs = malloc(sizeof(double) * nk), *om = malloc(sizeof(double) * m), *r3 = malloc(sizeof(double) * m);
    double *dz = malloc(sizeof(double) * n), *dl = malloc(sizeof(double) * p), *ds = malloc(sizeof(double) * m);
    double *dzd = malloc(sizeof(double) * m), *dsa = malloc(sizeof(double) * m), *dza = malloc(sizeof(double) * m);
    int *piv = malloc(sizeof(int) * nk);
    int flag = 2, it = 0;
    /* slacks and duals: QP start s = h - g (the gravity-compensating start is strictly feasible),
     * z = 1 / max(s, 1); NLP start shifted so that min s = 1 when a row is violated, z = z0 / max(s, 1) */
    rows_eval(P, z, nl, g, NULL);
    double mn = 1e300;
    for (int r = 0; r < m; r++) mn = fmin(mn, h_of(P, r) - g[r]);
    const double ssh = (nl && mn <= 0.0) ? 1.0 - mn : 0.0;
    for (int r = 0; r < m; r++) {
        s[r] = h_of(P, r) - g[r] + ssh;
        if (!nl && s[r] < 1e-8) s[r] = 1e-8;
        zd[r] = (nl ? prm->z0 : 1.0) / fmax(s[r], 1.0);
    }
    double sigma = 0.0;
    for (it = 0; it < (nl ? prm->nlp_maxit : prm->qp_maxit); it++) {
        rows_eval(P, z, nl, g, J);
        /* equality multipliers: the costates that zero the state part of r_d (the kernel's backward
         * recursion lambda_k = grad_x_k L + A_k' lambda_{k+1}; the primal-dual step does not depend on
         * them, the dual residual test does): (Aeq' lam)_{x_j} = lam_{j-1} - A_j' lam_j = -grad_{x_j} */
        {
            const int N = P->N;
            double gx[12];
            for (int j = N; j >= 1; j--) {
                for (int i = 0; i < 12; i++) {
                    const int v = 12 * (j - 1) + i;
                    double gv = P->Pd[v] * z[v] + P->cv[v];
                    for (int r = 0; r < m; r++) gv += J[(size_t)r * n + v] * zd[r];
                    gx[i] = gv;
                }
                for (int i = 0; i < 12; i++) {
                    double v = -gx[i];
                    if (j < N) for (int q = 0; q < 12; q++) v -= P->Aeq[(size_t)(12 * j + q) * n + 12 * (j - 1) + i] * lam[12 * j + q];
                    lam[12 * (j - 1) + i] = v;
                }
            }
        }
        /* residuals: r_d = grad f + Aeq' lam + J' z ; r_p = g + s - h ; r_eq = Aeq z - beq */
        double gm = 1.0, nrd = 0, nrp = 0, sz = 0;
        for (int i = 0; i < n; i++) {
            const double gf = P->Pd[i] * z[i] + P->cv[i];
            gm = fmax(gm, fabs(gf));
            double v = gf;
            for (int r = 0; r < p; r++) v += P->Aeq[(size_t)r * n + i] * lam[r];
            for (int r = 0; r < m; r++) v += J[(size_t)r * n + i] * zd[r];
            rd[i] = v; nrd += v * v;
        }
        for (int r = 0; r < m; r++) { rp[r] = g[r] + s[r] - h_of(P, r); nrp += rp[r] * rp[r]; sz += s[r] * zd[r]; }
        for (int r = 0; r < p; r++) {
            double v = -P->beq[r];
            for (int j = 0; j < n; j++) v += P->Aeq[(size_t)r * n + j] * z[j];
            req[r] = v;
        }
        nrd = sqrt(nrd); nrp = sqrt(nrp);
        const double mu = sz / (m > 0 ? m : 1);
        {                                          /* divergence: ORC_Z_DIV (the LIP mode's rule) */
            double zm = 0.0;
            for (int r = 0; r < m; r++) zm = fmax(zm, zd[r]);
            if (!isfinite(nrd) || !isfinite(nrp) || !isfinite(sz) || !(zm <= ORC_Z_DIV)) { flag = 3; break; }
        }
        if (getenv("ORC12_TRACE"))
            fprintf(stderr, "  %s it %2d |rd| %.3e (th %.3e) |rp| %.3e mu %.3e sigma %.3e\n", nl ? "nlp" : "qp ", it, nrd, th * gm, nrp, mu, sigma);
        if (nrd < th * gm && nrp < th && mu < mtol) { flag = 0; break; }
        /* Hessian of the Lagrangian + J' W J */
        memset(Hf, 0, sizeof(double) * (size_t)n * n);
        for (int i = 0; i < n; i++) Hf[(size_t)i * n + i] = P->Pd[i];
        if (nl)
            for (int k = 0; k < P->N; k++)
                for (int j = 0; j < P->K; j++) {
                    const double w = -2.0 * zd[P->mlin + k * P->K + j];
                    Hf[(size_t)(12 * k) * n + 12 * k] += w; Hf[(size_t)(12 * k + 1) * n + 12 * k + 1] += w;
                }
        for (int r = 0; r < m; r++) om[r] = zd[r] / s[r];
        for (int r = 0; r < m; r++) {
            const double *Jr = J + (size_t)r * n;
            for (int i = 0; i < n; i++) {
                if (Jr[i] == 0.0) continue;
                const double a = om[r] * Jr[i];
                for (int j = 0; j < n; j++) if (Jr[j] != 0.0) Hf[(size_t)i * n + j] += a * Jr[j];
            }
        }
        /* inertia: delta I until the condensed Hessian is positive definite (NLP; the QP's is) */
        double delta = 0.0;
        if (nl) {
            double dm = 1.0;
            for (int i = 0; i < n; i++) dm = fmax(dm, Hf[(size_t)i * n + i]);
            const double dstart = 1e-10 * dm;
            int ok = 0;
            for (int tries = 0; tries < 14; tries++) {
                if (tries > 0) {
                    const double nd = (delta == 0.0) ? dstart : delta * 10.0;
                    for (int i = 0; i < n; i++) Hf[(size_t)i * n + i] += nd - delta;
                    delta = nd;
                }
                if (reduced_pd(P, Hf)) { ok = 1; break; }
            }
            if (!ok) { flag = 1; break; }
        }
        memset(KK, 0, sizeof(double) * (size_t)nk * nk);
        for (int i = 0; i < n; i++) memcpy(KK + (size_t)i * nk, Hf + (size_t)i * n, sizeof(double) * n);
        for (int r = 0; r < p; r++)
            for (int j = 0; j < n; j++) { KK[(size_t)(n + r) * nk + j] = P->Aeq[(size_t)r * n + j]; KK[(size_t)j * nk + n + r] = P->Aeq[(size_t)r * n + j]; }
        if (orc_lu(nk, KK, piv) != 0) { flag = 1; break; }
        double ap = 1, ad = 1;
        for (int pass = 0; pass < 2; pass++) {
            /* complementarity target r3 = -s z (predictor), - s z - ds_a dz_a + sigma mu (corrector) */
            for (int r = 0; r < m; r++) r3[r] = -s[r] * zd[r] + (pass ? sigma * mu - dsa[r] * dza[r] : 0.0);
            /* (H + J'WJ) dz + Aeq' dl = -r_d - J'(r3 / s + W r_p) ; Aeq dz = -r_eq */
            for (int i = 0; i < n; i++) rhs[i] = -rd[i];
            for (int r = 0; r < m; r++) {
                const double w = r3[r] / s[r] + om[r] * rp[r];
                const double *Jr = J + (size_t)r * n;
                for (int i = 0; i < n; i++) if (Jr[i] != 0.0) rhs[i] -= Jr[i] * w;
            }
            for (int r = 0; r < p; r++) rhs[n + r] = -req[r];
            orc_lu_solve(nk, KK, piv, rhs);
            memcpy(dz, rhs, sizeof(double) * n); memcpy(dl, rhs + n, sizeof(double) * p);
            double mxs = 0, mxz = 0;
            for (int r = 0; r < m; r++) {
                double jd = 0;
                const double *Jr = J + (size_t)r * n;
                for (int i = 0; i < n; i++) if (Jr[i] != 0.0) jd += Jr[i] * dz[i];
                ds[r] = -rp[r] - jd;
                dzd[r] = (r3[r] - zd[r] * ds[r]) / s[r];
                mxs = fmax(mxs, -ds[r] / s[r]); mxz = fmax(mxz, -dzd[r] / zd[r]);
            }
            ap = mxs > 0 ? 1.0 / mxs : 1.0; ad = mxz > 0 ? 1.0 / mxz : 1.0;
            if (pass == 0) {
                double num = 0;
                for (int r = 0; r < m; r++) num += (s[r] + ap * ds[r]) * (zd[r] + ad * dzd[r]);
                const double rho = num / sz, mr = rho < 1.0 ? rho : 1.0;
                sigma = mr * mr * mr;
                memcpy(dsa, ds, sizeof(double) * m); memcpy(dza, dzd, sizeof(double) * m);
            }
        }
        ap = fmin(1.0, 0.99 * ap); ad = fmin(1.0, 0.99 * ad);
        if (getenv("ORC12_TRACE")) fprintf(stderr, "      ap %.4e ad %.4e delta %.3e\n", ap, ad, delta);
        for (int i = 0; i < n; i++) z[i] += ap * dz[i];
        for (int r = 0; r < m; r++) { s[r] += ap * ds[r]; zd[r] += ad * dzd[r]; }
    }
    *iters = it;
    if (flag == 0 && (nl || !prm->use_nlp) && prm->polish) {         /* the last stage: exact active-set point */
        int steps = 0;
        const int acc = polish12(P, nl, z, s, zd, &steps);
        /* a rejected polish leaves the interior-point point, up to ~1e-3 N from the optimum along the legs'
         * internal-force directions: ACCEPTABLE (4), never OPTIMAL (the kernel, same rule) */
        if (!acc) flag = 4;
        __atomic_fetch_add(&orc12_polish_stats[acc], 1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&orc12_polish_stats[2], steps, __ATOMIC_RELAXED);
        int old = orc12_polish_stats[3];
        while (steps > old && !__atomic_compare_exchange_n(&orc12_polish_stats[3], &old, steps, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
    }
    free(g); free(J); free(s); free(zd); free(rd); free(rp); free(req); free(Hf); free(KK); free(rhs); free(om); free(r3);
    free(dz); free(dl); free(ds); free(dzd); free(dsa); free(dza); free(piv);
    return flag;
}

int orc12_solve_agent(const orc12_params *p_in, const double x0[12], const double *xref, const double *foot,
                      const int *contact, const double *obstacles, int n_obs, const double *nbr_state, int n_all,
                      int self_idx, double *x_qp, double *x_out, double *obj, int status[2], int iters[2])
{
    orc12_params pc = *p_in;
    if (pc.K_obs > n_obs) pc.K_obs = n_obs > 0 ? n_obs : 0;
    { const int others = nbr_state ? n_all - 1 : 0; if (pc.K_nbr > others) pc.K_nbr = others > 0 ? others : 0; }
    const orc12_params *prm = &pc;
    const int N = prm->N, n = orc12_nv(prm), p = 12 * N, K = prm->K_obs + prm->K_nbr;
    p12_t P;
    memset(&P, 0, sizeof P);
    P.N = N; P.n = n; P.p = p; P.prm = prm; P.K = K; P.mc = N * K;
    double *A = malloc(sizeof(double) * 144 * N), *B = malloc(sizeof(double) * 144 * N), *c = malloc(sizeof(double) * 12 * N);
    orc12_dynamics(prm, x0, xref, foot, contact, A, B, c);
    /* cost */
    P.Pd = calloc(n, sizeof(double)); P.cv = calloc(n, sizeof(double));
    for (int k = 0; k < N; k++)
        for (int i = 0; i < 12; i++) {
            const double w = (k == N - 1) ? prm->qN[i] : prm->q[i];
            P.Pd[12 * k + i] = w; P.cv[12 * k + i] = -w * xref[12 * k + i];
            P.Pd[12 * N + 12 * k + i] = prm->r[i % 3];
        }
    P.Pd[n - 1] = prm->Sw;
    /* dynamics rows: x_{k+1} - A_k x_k - B_k u_k = c_k (+ A_0 x0 for k = 0) */
    P.Aeq = calloc((size_t)p * n, sizeof(double)); P.beq = calloc(p, sizeof(double));
    for (int k = 0; k < N; k++)
        for (int i = 0; i < 12; i++) {
            double *row = P.Aeq + (size_t)(12 * k + i) * n;
            row[12 * k + i] = 1.0;
            for (int j = 0; j < 12; j++) {
                if (k > 0) row[12 * (k - 1) + j] -= A[144 * k + 12 * i + j];
                row[12 * N + 12 * k + j] -= B[144 * k + 12 * i + j];
            }
            double b = c[12 * k + i];
            if (k == 0) for (int j = 0; j < 12; j++) b += A[12 * i + j] * x0[j];
            P.beq[12 * k + i] = b;
        }
    /* friction pyramid + fz <= fmax per stance leg (LowLevelCtrl.cpp:158-162), stage-major */
    int mlin = 0;
    for (int k = 0; k < N; k++) for (int l = 0; l < 4; l++) mlin += contact[4 * k + l] ? 6 : 0;
    P.mlin = mlin;
    P.G = calloc((size_t)(mlin ? mlin : 1) * n, sizeof(double)); P.h = calloc(mlin ? mlin : 1, sizeof(double));
    const double mus = prm->mu / sqrt(2.0);
    int r = 0;
    for (int k = 0; k < N; k++)
        for (int l = 0; l < 4; l++) {
            if (!contact[4 * k + l]) continue;
            const int f0 = 12 * N + 12 * k + 3 * l;
            const double gc[6][3] = {{1, 0, -mus}, {-1, 0, -mus}, {0, 1, -mus}, {0, -1, -mus}, {0, 0, -1}, {0, 0, 1}};
            for (int q = 0; q < 6; q++, r++) {
                for (int d = 0; d < 3; d++) P.G[(size_t)r * n + f0 + d] = gc[q][d];
                P.h[r] = (q == 5) ? prm->fmax : 0.0;
            }
        }
    /* condensation X = T U + xbar (inertia test) */
    P.T = calloc((size_t)144 * N * N, sizeof(double));
    {
        const int nu = 12 * N;
        double *M = malloc(sizeof(double) * 144), *M2 = malloc(sizeof(double) * 144);
        for (int j = 0; j < N; j++) {              /* column block j: x_{k+1} = A_k..A_{j+1} B_j */
            memcpy(M, B + 144 * j, sizeof(double) * 144);
            for (int k = j; k < N; k++) {
                if (k > j) {
                    for (int a = 0; a < 12; a++)
                        for (int b = 0; b < 12; b++) {
                            double v = 0;
                            for (int q = 0; q < 12; q++) v += A[144 * k + 12 * a + q] * M[12 * q + b];
                            M2[12 * a + b] = v;
                        }
                    memcpy(M, M2, sizeof(double) * 144);
                }
                for (int a = 0; a < 12; a++)
                    for (int b = 0; b < 12; b++) P.T[(size_t)(12 * k + a) * nu + 12 * j + b] = M[12 * a + b];
            }
        }
        free(M); free(M2);
    }
    /* start: gravity-compensating forces on the stance legs, the dynamics rolled out, s = 0 */
    double *z = calloc(n, sizeof(double)), *lam = calloc(p, sizeof(double));
    {
        double x[12], xn[12];
        memcpy(x, x0, sizeof x);
        for (int k = 0; k < N; k++) {
            int ns = 0;
            for (int l = 0; l < 4; l++) ns += contact[4 * k + l] != 0;
            double *u = z + 12 * N + 12 * k;
            for (int l = 0; l < 4; l++) u[3 * l + 2] = (ns && contact[4 * k + l]) ? prm->mass * prm->grav / ns : 0.0;
            for (int i = 0; i < 12; i++) {
                double v = c[12 * k + i];
                for (int j = 0; j < 12; j++) v += A[144 * k + 12 * i + j] * x[j] + B[144 * k + 12 * i + j] * u[j];
                xn[i] = v;
            }
            memcpy(x, xn, sizeof x);
            memcpy(z + 12 * k, x, sizeof x);
        }
    }
    status[0] = ipm(&P, 0, z, lam, &iters[0]);
    if (status[0] == 0 && prm->use_nlp && prm->tol_qp > prm->tol) status[0] = 4;   /* warm-start tolerance only (kernel rule) */
    if (x_qp) memcpy(x_qp, z, sizeof(double) * n);
    status[1] = (prm->use_nlp && status[0] == 3) ? 3 : 0;      /* FATAL QP: the NLP stage is not run (kernel, same rule) */
    iters[1] = 0;
    double *obs = NULL, *eps = NULL;
    if (prm->use_nlp && K > 0 && status[0] != 3) {
        /* the selection and prediction of the LIP mode, on the CoM position / velocity */
        orc_params op;
        orc_params_default(&op, N, 2);
        op.K_obs = prm->K_obs; op.K_nbr = prm->K_nbr; op.Ts = prm->Ts; op.eps_obs = prm->eps_obs; op.eps_nbr = prm->eps_nbr;
        const double xl[4] = {x0[0], x0[6], x0[1], x0[7]};
        obs = malloc(sizeof(double) * 2 * N * K); eps = malloc(sizeof(double) * K);
        orc_select_obstacles(&op, xl, obstacles, n_obs, nbr_state, n_all, self_idx, obs, eps);
        P.obs = obs; P.eps = eps;
        status[1] = ipm(&P, 1, z, lam, &iters[1]);
    } else if (prm->use_nlp && status[0] != 3) {
        P.mc = 0;
        status[1] = ipm(&P, 1, z, lam, &iters[1]);
    }
    memcpy(x_out, z, sizeof(double) * n);
    double f = 0;
    for (int i = 0; i < n; i++) f += 0.5 * P.Pd[i] * z[i] * z[i] + P.cv[i] * z[i];
    *obj = f;
    free(A); free(B); free(c); free(P.Pd); free(P.cv); free(P.Aeq); free(P.beq); free(P.G); free(P.h); free(P.T);
    free(z); free(lam); free(obs); free(eps);
    return status[0] | (status[1] << 4);
}

typedef struct {
    const orc12_params *p; int lo, hi;
    const double *x0, *xref, *foot, *obstacles, *nbr; const int *contact; int n_obs, n_all, off;
    double *x_qp, *x_out, *obj; int *status, *iters;
} job12_t;

static void *worker12(void *arg)
{
    job12_t *j = (job12_t *)arg;
    const int nv = orc12_nv(j->p), N = j->p->N;
    for (int a = j->lo; a < j->hi; a++)
        orc12_solve_agent(j->p, j->x0 + 12 * (size_t)a, j->xref + (size_t)12 * N * a, j->foot + (size_t)12 * N * a,
                          j->contact + (size_t)4 * N * a, j->obstacles, j->n_obs, j->nbr, j->n_all, j->off + a,
                          j->x_qp ? j->x_qp + (size_t)nv * a : NULL, j->x_out + (size_t)nv * a, j->obj + a,
                          j->status + 2 * a, j->iters + 2 * a);
    return NULL;
}

int orc12_solve_batch(const orc12_params *p, int n_agents, const double *x0, const double *xref, const double *foot,
                      const int *contact, const double *obstacles, int n_obs, const double *nbr_state, int n_all,
                      int agent_offset, double *x_qp, double *x_out, double *obj, int *status, int *iters, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n_agents) nthreads = n_agents > 0 ? n_agents : 1;
    pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
    job12_t *jobs = malloc(sizeof(job12_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        job12_t *j = &jobs[t];
        j->p = p; j->lo = (int)((long)n_agents * t / nthreads); j->hi = (int)((long)n_agents * (t + 1) / nthreads);
        j->x0 = x0; j->xref = xref; j->foot = foot; j->contact = contact; j->obstacles = obstacles; j->nbr = nbr_state;
        j->n_obs = n_obs; j->n_all = n_all; j->off = agent_offset;
        j->x_qp = x_qp; j->x_out = x_out; j->obj = obj; j->status = status; j->iters = iters;
        pthread_create(&th[t], NULL, worker12, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}
