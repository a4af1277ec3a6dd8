/*
 * ORACLE (test infrastructure only): problem assembly restated from
 * /root/reference/src/MPC_dist.cpp:81-321 (QP) and :371-396 (closest obstacle).
 */
#include <math.h>
#include <string.h>
#include <float.h>
#include "oracle.h"

#ifndef ORC_POLISH_DEFAULT
#define ORC_POLISH_DEFAULT 1           /* the kernel's SRB_POLISH_ON */
#endif

void orc_params_default(orc_params *p, int N, int C)
{
    memset(p, 0, sizeof(*p));
    p->N = N; p->C = C; p->K_obs = 1; p->K_nbr = 0;
    p->grav = 9.81; p->hcom = 0.29;
    p->Ts = 43 * 0.001;                  /* ts_OptTick_*0.001, MPC_dist.cpp:104 */
    p->mu = 0.7;                         /* MPC_dist.cpp:90 */
    p->Qw = 3e2; p->Pw = 2e3; p->Rw = 1e-1; p->Sw = 0.3e4;   /* :172-175 */
    p->box = 1e3;                        /* :317-318 */
    p->eps_obs = (double)1.9f;           /* dec_vars_constr_cost.h:401 (float) */
    p->eps_nbr = (double)2.2f;           /* dec_vars_constr_cost.h:402 (robot-to-robot value) */
    p->vsat = (double)0.35f;             /* dec_vars_constr_cost.h:306-307 (float) */
    p->tol = 1e-6;                       /* GlobalOptions.h:24-25 */
    p->qp_maxit = 25;                    /* GlobalOptions.h:23 */
    p->nlp_maxit = 50;
    p->use_nlp = 1;
    p->qp_init = 1;                      /* scaled QP start (qp_ipm.c); 0 = iSWIFT's kkt_initialize */
    p->polish = ORC_POLISH_DEFAULT;
    p->tol_qp = 3e-1;                    /* QP stage before the NLP: its point only warm-starts the NLP */
}

int orc_nv(const orc_params *p) { return (6 + p->C) * p->N + 1; }
int orc_neq(const orc_params *p) { return 7 * p->N; }
int orc_mqp(const orc_params *p) { return 4 * (p->N - 1) + 12 * p->N + 2 * p->C * p->N; }
int orc_mnlp(const orc_params *p) { return orc_mqp(p) + 4 * p->N + p->N * (p->K_obs + p->K_nbr); }

static void mm4(const double *X, const double *Y, double *Z)   /* Z = X*Y, 4x4 */
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += X[i * 4 + k] * Y[k * 4 + j];
            Z[i * 4 + j] = s;
        }
}

void orc_lip(const orc_params *p, double Ad[16], double Bd[8])
{
    /* A, B of the LIP, MPC_dist.cpp:117-122 */
    double w2 = p->grav / p->hcom, T = p->Ts;
    double A[16] = {0}, B[8] = {0};
    A[0 * 4 + 1] = 1; A[1 * 4 + 0] = w2; A[2 * 4 + 3] = 1; A[3 * 4 + 2] = w2;
    B[1 * 2 + 0] = -w2; B[3 * 2 + 1] = -w2;
    /* Ad = I + A T + 0.5 A A T^2 + A A A T^3 / 6   (MPC_dist.cpp:126) */
    double A2[16], A3[16];
    mm4(A, A, A2); mm4(A2, A, A3);
    for (int i = 0; i < 16; i++)
        Ad[i] = (i % 5 == 0 ? 1.0 : 0.0) + A[i] * T + 0.5 * A2[i] * T * T + A3[i] * T * T * T / 6;
    /* Bd = A^{-1} (Ad - I) B   (MPC_dist.cpp:127); A^{-1} of the LIP in closed form */
    double Ai[16] = {0};
    Ai[0 * 4 + 1] = 1.0 / w2; Ai[1 * 4 + 0] = 1.0; Ai[2 * 4 + 3] = 1.0 / w2; Ai[3 * 4 + 2] = 1.0;
    double AdI[16], M[16];
    for (int i = 0; i < 16; i++) AdI[i] = Ad[i] - (i % 5 == 0 ? 1.0 : 0.0);
    mm4(Ai, AdI, M);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 2; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += M[i * 4 + k] * B[k * 2 + j];
            Bd[i * 2 + j] = s;
        }
}

void orc_build_qp(const orc_params *p, const double x0[4], const double *ref, const double *foot,
                  double *Pd, double *c, double *A, double *b, double *G, double *h)
{
    const int N = p->N, C = p->C, nv = orc_nv(p), neq = orc_neq(p), m = orc_mqp(p);
    const int oU = 4 * N, oL = 6 * N, oS = nv - 1;
    double Ad[16], Bd[8];
    orc_lip(p, Ad, Bd);

    /* cost: Q_qp = blkdiag(Pbig, Rbig, 0, sl_gain), f = -Pbig' ref   (MPC_dist.cpp:190-210) */
    for (int i = 0; i < nv; i++) { Pd[i] = 0; c[i] = 0; }
    for (int k = 0; k < N; k++) {
        double q = (k == N - 1) ? p->Pw : p->Qw;
        for (int d = 0; d < 4; d++) { Pd[4 * k + d] = q; c[4 * k + d] = -q * ref[4 * k + d]; }
        Pd[oU + 2 * k] = p->Rw; Pd[oU + 2 * k + 1] = p->Rw;
    }
    Pd[oS] = p->Sw;

    /* equalities (MPC_dist.cpp:249-261) */
    memset(A, 0, sizeof(double) * (size_t)neq * nv);
    memset(b, 0, sizeof(double) * neq);
    for (int k = 0; k < N; k++) {
        for (int d = 0; d < 4; d++) {
            int r = 4 * k + d;
            A[(size_t)r * nv + 4 * k + d] += -1.0;                       /* Abig - I */
            if (k >= 1)
                for (int e = 0; e < 4; e++) A[(size_t)r * nv + 4 * (k - 1) + e] += Ad[d * 4 + e];
            for (int e = 0; e < 2; e++) A[(size_t)r * nv + oU + 2 * k + e] += Bd[d * 2 + e];   /* Bbig */
            if (k == 0) {                                                /* beq = -Abigx0*x0 */
                double s = 0;
                for (int e = 0; e < 4; e++) s += Ad[d * 4 + e] * x0[e];
                b[r] = -s;
            }
        }
        for (int d = 0; d < 2; d++) {                                    /* u_k - F_k lambda_k = 0 */
            int r = 4 * N + 2 * k + d;
            A[(size_t)r * nv + oU + 2 * k + d] = 1.0;
            for (int j = 0; j < C; j++) A[(size_t)r * nv + oL + C * k + j] = -foot[(k * 2 + d) * C + j];
        }
        int r = 6 * N + k;                                               /* sum lambda_k = 1 */
        for (int j = 0; j < C; j++) A[(size_t)r * nv + oL + C * k + j] = 1.0;
        b[r] = 1.0;
    }

    /* inequalities G x <= h (MPC_dist.cpp:278-321) */
    memset(G, 0, sizeof(double) * (size_t)m * nv);
    const double fr = p->mu * p->hcom / sqrt(2.0);
    int r = 0;
    for (int sgn = 1; sgn >= -1; sgn -= 2)                               /* +-(Gsubx - Gsubu) */
        for (int i = 0; i < N - 1; i++)
            for (int d = 0; d < 2; d++, r++) {
                G[(size_t)r * nv + 4 * i + 2 * d] = sgn;
                G[(size_t)r * nv + oU + 2 * (i + 1) + d] = -sgn;
                h[r] = fr;
            }
    for (int sgn = 1; sgn >= -1; sgn -= 2)                               /* +-X <= 1e3 */
        for (int j = 0; j < 4 * N; j++, r++) { G[(size_t)r * nv + j] = sgn; h[r] = p->box; }
    for (int sgn = 1; sgn >= -1; sgn -= 2)                               /* +-U <= 1e3 */
        for (int j = 0; j < 2 * N; j++, r++) { G[(size_t)r * nv + oU + j] = sgn; h[r] = p->box; }
    for (int j = 0; j < C * N; j++, r++) { G[(size_t)r * nv + oL + j] = -1.0; h[r] = 0.0; }  /* -lambda <= 0 */
    for (int j = 0; j < C * N; j++, r++) { G[(size_t)r * nv + oL + j] = 1.0; h[r] = 1.0; }   /*  lambda <= 1 */
}

/* Indices of the selected rows: idx[0..K_obs) static obstacles, idx[K_obs..K) agents.
 *
 * Static obstacles: MPC_dist.cpp:371-382 -- min_dist = 1000, min_i = 0, then a strict '<'
 * scan over sqrt distances (the first index wins ties, including ties created by sqrt
 * rounding).  Generalised to K_obs rounds over the not yet chosen rows; a round that finds
 * no row closer than 1000 m keeps the reference's default index 0 (as the reference does
 * when every obstacle is 1000 m or more away, or its distance is NaN).
 * Neighbours (the reference reads one state_other, MPC_dist.cpp:385): the K_nbr nearest
 * other agents by the same sqrt / first-index order, no distance cap; -1 when fewer finite
 * rows exist. */
void orc_select_idx(const orc_params *p, const double x0[4], const double *obstacles, int n_obs,
                    const double *nbr_state, int n_all, int self_idx, int *idx)
{
    const double px = x0[0], py = x0[2];
    for (int j = 0; j < p->K_obs; j++) {
        double best = 1000.0; int bi = n_obs > 0 ? 0 : -1;
        for (int i = 0; i < n_obs; i++) {
            int used = 0;
            for (int t = 0; t < j; t++) used |= (idx[t] == i);
            if (used) continue;
            double dx = px - obstacles[2 * i], dy = py - obstacles[2 * i + 1];
            double d = sqrt(dx * dx + dy * dy);
            if (d < best) { best = d; bi = i; }
        }
        idx[j] = bi;
    }
    for (int j = 0; j < p->K_nbr; j++) {
        double best = DBL_MAX; int bi = -1;
        for (int i = 0; i < n_all; i++) {
            if (i == self_idx) continue;
            int used = 0;
            for (int t = 0; t < j; t++) used |= (idx[p->K_obs + t] == i);
            if (used) continue;
            double dx = px - nbr_state[4 * i], dy = py - nbr_state[4 * i + 1];
            double d = sqrt(dx * dx + dy * dy);
            if (d < best) { best = d; bi = i; }
        }
        idx[p->K_obs + j] = bi;
    }
}

/* obstacle positions per grid (static: fixed; agents: constant-velocity prediction
 * o_k = p + v Ts (k+1)) and their clearances; a row with no selection (-1: fewer finite
 * neighbours than K_nbr) sits 1000 m from the agent along +x, the reference's "no obstacle"
 * distance (min_dist = 1000, MPC_dist.cpp:371): inactive, and small enough that its
 * residual |p - o|^2 ~ 1e6 keeps full precision */
void orc_select_obstacles(const orc_params *p, const double x0[4],
                          const double *obstacles, int n_obs,
                          const double *nbr_state, int n_all, int self_idx,
                          double *obs_out, double *eps_out)
{
    const int N = p->N, K = p->K_obs + p->K_nbr;
    int chosen[64];
    orc_select_idx(p, x0, obstacles, n_obs, nbr_state, n_all, self_idx, chosen);
    for (int j = 0; j < K; j++) {
        const int st = j < p->K_obs, bi = chosen[j];
        eps_out[j] = st ? p->eps_obs : p->eps_nbr;
        for (int k = 0; k < N; k++) {
            const double t = st ? 0.0 : p->Ts * (k + 1);
            const double *row = st ? obstacles + 2 * (size_t)bi : nbr_state + 4 * (size_t)bi;
            obs_out[(k * K + j) * 2 + 0] = bi >= 0 ? row[0] + (st ? 0.0 : row[2] * t) : x0[0] + 1000.0;
            obs_out[(k * K + j) * 2 + 1] = bi >= 0 ? row[1] + (st ? 0.0 : row[3] * t) : x0[2];
        }
    }
}

/* fitComTrajectory_eventbase, MPC_dist.cpp:784-855, N == NDOMAIN branch:
 * 24x24 KKT of  min |B a - [buf; X0..X3]|^2  s.t. first 4 rows of the end-point
 * constraint (the reference's 20x8 -> 20x4 block assignment keeps only s=0). */
void orc_fit_bezier(const double buf[4], const double *X, double alpha[20])
{
    double Bm[20 * 20], Q[24 * 24], rhs[24], pts[20];
    memset(Bm, 0, sizeof Bm); memset(Q, 0, sizeof Q); memset(rhs, 0, sizeof rhs);
    static const int fact[5] = {1, 1, 2, 6, 24};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 5; j++) {
            double s = i * (1.0 / 4.0);
            double mck = (double)(fact[4] / (fact[j] * fact[4 - j]));
            double v = mck * pow(s, j) * pow(1 - s, 4 - j);
            for (int d = 0; d < 4; d++) Bm[(i * 4 + d) * 20 + j * 4 + d] = v;
        }
    for (int d = 0; d < 4; d++) pts[d] = buf[d];
    for (int i = 0; i < 4; i++) for (int d = 0; d < 4; d++) pts[4 + i * 4 + d] = X[i * 4 + d];
    for (int a = 0; a < 20; a++) {
        for (int bb = 0; bb < 20; bb++) {
            double s = 0;
            for (int r = 0; r < 20; r++) s += Bm[r * 20 + a] * Bm[r * 20 + bb];
            Q[a * 24 + bb] = s;
        }
        double s = 0;
        for (int r = 0; r < 20; r++) s += Bm[r * 20 + a] * pts[r];
        rhs[a] = s;
    }
    for (int e = 0; e < 4; e++)
        for (int a = 0; a < 20; a++) { Q[a * 24 + 20 + e] = Bm[e * 20 + a]; Q[(20 + e) * 24 + a] = Bm[e * 20 + a]; }
    for (int e = 0; e < 4; e++) rhs[20 + e] = buf[e];
    int piv[24];
    orc_lu(24, Q, piv);
    orc_lu_solve(24, Q, piv, rhs);
    /* alpha_mtx (4x5, column-major map of the 20-vector): alpha[d][j] = vec[j*4+d] */
    for (int d = 0; d < 4; d++) for (int j = 0; j < 5; j++) alpha[d * 5 + j] = rhs[j * 4 + d];
}
