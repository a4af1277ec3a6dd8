/*
 * ORACLE (test infrastructure only): the low-level CLF-QP controller restated from
 *   LowLevelCtrl::calcTorque   /root/reference/src/LowLevelCtrl.cpp:18-113
 *   LowLevelCtrl::cost         :115-137
 *   LowLevelCtrl::constraints  :139-236
 *   LowLevelCtrl::swingInvKin  :446-488
 * with the QP solved by the iSWIFT restatement in qp_ipm.c (iswiftQp_e, Prime.c:127-230).
 *
 * Matrices are column-major (Eigen's default), with the fixed leading dimensions of the
 * batched ABI (include/srbnmpc.h, srb_ll_io): Dinv 18x18, B 18x12, H0 18x18 (outDim rows
 * used), Jc / Js / Jtoe / Jhip 12x18 (leading dimension 12; 3c / 12-3c / 12 / 12 rows
 * used), toePos / hipPos 3x4.
 *
 * Decision vector (numDec = 3c + 12 + outDim + useCLF, always 31 with the CLF):
 *   [F (3c, stance legs in FR,FL,RR,RL order) | tau (12) | aux (outDim = 6 + 3(4-c)) | d].
 *
 * Dense assembly follows the reference's Eigen expressions literally (products formed
 * as in the source, the CLF quadratic forms with explicit PP/FF/GG matrices).
 * Deliberate difference: the reference's h_QP member is never cleared, so when the
 * contact count grows between calls its friction rows inherit stale torque-bound values
 * from the previous call (:159-168 write rows 5c.. only); here every call starts from
 * h = 0 on the friction rows, which is what the reference computes for a first call or a
 * constant contact count.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "oracle.h"

#define NQ 18   /* TOTAL_DOF (global_loco_opts.h:24) */
#define NU 12   /* TOTAL_IN  (global_loco_opts.h:25) */
#define LLHZ 1000.0   /* LL_Hz (global_loco_opts.h:22) */

void orc_ll_params_default(orc_ll_params *p)
{
    /* Parameters.cpp:62-75 (default low level) */
    p->mu = 0.7; p->kp = 700; p->kd = 40; p->useCLF = 1;
    p->tauPen = 1e0; p->dfPen = 1e-1; p->auxPen = 1e6; p->clfPen = 1e8;
    p->auxMax = 100; p->clfEps = 0.8;
    p->maxit = 25; p->tol = 1e-6;             /* GlobalOptions.h:23-25 */
    p->iswift_trap = 0;
}

/* C (r x k, ldc r) = A (r x n, lda) * B (n x k, ldb), column-major */
static void mm(int r, int n, int k, const double *A, int lda, const double *B, int ldb, double *C)
{
    for (int j = 0; j < k; j++)
        for (int i = 0; i < r; i++) {
            double s = 0;
            for (int t = 0; t < n; t++) s += A[t * lda + i] * B[j * ldb + t];
            C[j * r + i] = s;
        }
}

/* transpose of (r x c, ld) into (c x r, ld c) */
static void tr(int r, int c, const double *A, int lda, double *T)
{
    for (int i = 0; i < r; i++)
        for (int j = 0; j < c; j++) T[i * c + j] = A[j * lda + i];
}

static int ll_count(const int ind[4]) { return (ind[0] == 1) + (ind[1] == 1) + (ind[2] == 1) + (ind[3] == 1); }

int orc_ll_build_qp(const orc_ll_params *prm, const orc_ll_agent *in,
                    int *n_out, int *p_out, int *m_out, double *Pd, double *c, double *A, double *b,
                    double *G, double *h, double clf[3], double *LgV)
{
    const int cnt = ll_count(in->ind), useCLF = prm->useCLF ? 1 : 0;
    const int conDim = 3 * cnt, outDim = 6 + 3 * (4 - cnt), numDec = conDim + NU + outDim + useCLF;
    const int p = conDim + outDim, m = 5 * cnt + 2 * NU + useCLF;
    *n_out = numDec; *p_out = p; *m_out = m;
    memset(Pd, 0, sizeof(double) * numDec); memset(c, 0, sizeof(double) * numDec);
    memset(A, 0, sizeof(double) * p * numDec); memset(b, 0, sizeof(double) * p);
    memset(G, 0, sizeof(double) * m * numDec); memset(h, 0, sizeof(double) * m);
    clf[0] = clf[1] = clf[2] = 0.0;
    for (int i = 0; i < NQ; i++) LgV[i] = 0.0;

    /* ---- cost (LowLevelCtrl.cpp:115-137) */
    for (int i = 0; i < conDim; i++) Pd[i] = prm->dfPen;
    for (int i = 0; i < NU; i++) Pd[conDim + i] = prm->tauPen;
    for (int i = 0; i < outDim; i++) Pd[conDim + NU + i] = prm->auxPen;
    if (useCLF) Pd[numDec - 1] = prm->clfPen;
    {
        int k = 0;
        for (int i = 0; i < 4; i++)
            if (in->ind[i] == 1) { for (int j = 0; j < 3; j++) c[k + j] = -in->fDes[3 * i + j] * prm->dfPen; k += 3; }
    }

    /* ---- equalities (:147-152): Jc Dinv [Jc' B], H0 Dinv [Jc' B] I; b = Jc Dinv H - dJc, ... */
    double JcT[NQ * NU], JcD[NU * NQ], H0D[NQ * NQ], t1[NQ * NU], t2[NQ * NU], v1[NQ], v2[NQ];
    tr(conDim, NQ, in->Jc, NU, JcT);                       /* 18 x conDim, ld 18 */
    mm(conDim, NQ, NQ, in->Jc, NU, in->Dinv, NQ, JcD);      /* Jc Dinv: conDim x 18, ld conDim */
    mm(outDim, NQ, NQ, in->H0, NQ, in->Dinv, NQ, H0D);      /* H0 Dinv: outDim x 18, ld outDim */
    /* rows 0..conDim-1 */
    mm(conDim, NQ, conDim, JcD, conDim, JcT, NQ, t1);
    mm(conDim, NQ, NU, JcD, conDim, in->B, NQ, t2);
    for (int i = 0; i < conDim; i++) {
        for (int j = 0; j < conDim; j++) A[i * numDec + j] = t1[j * conDim + i];
        for (int j = 0; j < NU; j++) A[i * numDec + conDim + j] = t2[j * conDim + i];
    }
    mm(conDim, NQ, 1, JcD, conDim, in->Hv, NQ, v1);
    for (int i = 0; i < conDim; i++) b[i] = v1[i] - in->dJc[i];
    /* rows conDim.. */
    mm(outDim, NQ, conDim, H0D, outDim, JcT, NQ, t1);
    mm(outDim, NQ, NU, H0D, outDim, in->B, NQ, t2);
    for (int i = 0; i < outDim; i++) {
        double *row = A + (size_t)(conDim + i) * numDec;
        for (int j = 0; j < conDim; j++) row[j] = t1[j * outDim + i];
        for (int j = 0; j < NU; j++) row[conDim + j] = t2[j * outDim + i];
        row[conDim + NU + i] = 1.0;
    }
    mm(outDim, NQ, 1, H0D, outDim, in->Hv, NQ, v2);
    for (int i = 0; i < outDim; i++)
        b[conDim + i] = (-prm->kp * in->y[i] - prm->kd * in->dy[i]) + v2[i] - in->dH0[i];

    /* ---- friction cone (:157-165, repdiag of gc over the stance legs) */
    const double mus = prm->mu / sqrt(2.0);
    const double gc[5][3] = {{1, 0, -mus}, {-1, 0, -mus}, {0, 1, -mus}, {0, -1, -mus}, {0, 0, -1}};
    for (int l = 0; l < cnt; l++)
        for (int r = 0; r < 5; r++)
            for (int j = 0; j < 3; j++) G[(size_t)(5 * l + r) * numDec + 3 * l + j] = gc[r][j];
    /* ---- torque bounds (:167-172): sat = {22, 50, 50} per leg (LowLevelCtrl.hpp:35) */
    const double sat[3] = {22, 50, 50};
    for (int i = 0; i < NU; i++) {
        G[(size_t)(5 * cnt + i) * numDec + conDim + i] = 1.0;
        G[(size_t)(5 * cnt + NU + i) * numDec + conDim + i] = -1.0;
        h[5 * cnt + i] = sat[i % 3];
        h[5 * cnt + NU + i] = sat[i % 3];
    }

    /* ---- CLF row (:171-235): Lyapunov P of the IO-linearised outputs, explicit matrices */
    if (useCLF) {
        const int d2 = 2 * outDim;
        const double kp = prm->kp, kd = prm->kd, eps = prm->clfEps;
        const double P1 = (kd * kd + kp * kp + kp) / (2 * kp * kd), Pdd = 1 / (2 * kp), P2 = (kp + 1) / (2 * kd * kp);
        const double cc = 1.0 / (0.5 * (P1 + P2 + sqrt(P1 * P1 - 2 * P1 * P2 + P2 * P2 + 4 * Pdd * Pdd)));
        double *PP = calloc((size_t)d2 * d2, sizeof(double)), *FF = calloc((size_t)d2 * d2, sizeof(double));
        double *TT = calloc((size_t)d2 * d2, sizeof(double)), *M1 = calloc((size_t)d2 * d2, sizeof(double));
        double *M2 = calloc((size_t)d2 * d2, sizeof(double)), *eta = calloc(d2, sizeof(double));
        double *ve = calloc(d2, sizeof(double));
        for (int i = 0; i < outDim; i++) {
            PP[i * d2 + i] = P1; PP[(outDim + i) * d2 + i] = Pdd;
            PP[i * d2 + outDim + i] = Pdd; PP[(outDim + i) * d2 + outDim + i] = P2;
        }
        for (int i = 0; i < d2; i++) TT[i * d2 + i] = (i < outDim) ? 1.0 / eps : 1.0;
        mm(d2, d2, d2, TT, d2, PP, d2, M1);             /* tuneMat * PP * tuneMat */
        mm(d2, d2, d2, M1, d2, TT, d2, PP);
        for (int i = 0; i < outDim; i++) {
            FF[(outDim + i) * d2 + i] = 1.0;            /* block (0, outDim) = I   */
            FF[i * d2 + outDim + i] = -kp;              /* block (outDim, 0) = -kp */
            FF[(outDim + i) * d2 + outDim + i] = -kd;   /* block (outDim, outDim) = -kd */
            eta[i] = in->y[i]; eta[outDim + i] = in->dy[i];
        }
        /* V = eta' PP eta ; LfV = eta' (FF' PP + PP FF) eta ; LgV = 2 eta' PP GG */
        double FFt[36 * 36];
        tr(d2, d2, FF, d2, FFt);
        mm(d2, d2, d2, FFt, d2, PP, d2, M1);
        mm(d2, d2, d2, PP, d2, FF, d2, M2);
        for (int i = 0; i < d2 * d2; i++) M1[i] += M2[i];
        double V = 0, LfV = 0;
        mm(d2, d2, 1, PP, d2, eta, d2, ve);
        for (int i = 0; i < d2; i++) V += eta[i] * ve[i];
        mm(d2, d2, 1, M1, d2, eta, d2, ve);
        for (int i = 0; i < d2; i++) LfV += eta[i] * ve[i];
        /* (eta' PP)_j for j in the lower block; GG = [0; I] picks those columns */
        for (int j = 0; j < outDim; j++) {
            double s = 0;
            for (int i = 0; i < d2; i++) s += eta[i] * PP[(outDim + j) * d2 + i];
            LgV[j] = 2 * s;
        }
        const int row = 2 * NU + 5 * cnt;
        for (int j = 0; j < outDim; j++) G[(size_t)row * numDec + conDim + NU + j] = LgV[j];
        G[(size_t)row * numDec + numDec - 1] = -1.0;
        h[row] = -LfV - cc / eps * V;
        clf[0] = V; clf[1] = cc / eps * V; clf[2] = LfV;
        free(PP); free(FF); free(TT); free(M1); free(M2); free(eta); free(ve);
    }
    return 0;
}

int orc_ll_calc_torque(const orc_ll_params *prm, const orc_ll_agent *in, orc_ll_out *out)
{
    const int cnt = ll_count(in->ind), useCLF = prm->useCLF ? 1 : 0;
    const int conDim = 3 * cnt, outDim = 6 + 3 * (4 - cnt);
    double Pd[32], c[32], A[18 * 32], b[18], G[45 * 32], h[45], clf[3], LgV[NQ], x[32];
    int n, p, m, it = 0;
    orc_ll_build_qp(prm, in, &n, &p, &m, Pd, c, A, b, G, h, clf, LgV);
    /* the kernel's solve: iSWIFT minus the rounding-only sigma <= sigma_d branch (qp_ipm.c) */
    const int flag = prm->iswift_trap ? orc_qp_solve(n, m, p, Pd, c, A, b, G, h, prm->maxit, prm->tol, x, NULL, &it)
                                      : orc_qp_solve_nt(n, m, p, Pd, c, A, b, G, h, prm->maxit, prm->tol, x, &it);
    out->status = flag; out->iters = it;
    for (int i = 0; i < 32; i++) out->x[i] = (i < n) ? x[i] : 0.0;

    /* ---- parse (:44-64) */
    int k = 0;
    for (int i = 0; i < 12; i++) out->QP_force[i] = 0.0;
    for (int i = 0; i < 4; i++)
        if (in->ind[i] == 1) for (int j = 0; j < 3; j++) out->QP_force[3 * i + j] = x[k++];
    double *tau = out->tau;                       /* in/out: tau[0..5] carries the caller's state */
    for (int i = 0; i < NU; i++) tau[6 + i] = x[k++];
    double dV = 0;
    if (useCLF) {
        dV = clf[2] + clf[1];
        for (int i = 0; i < outDim; i++) dV += LgV[i] * x[k++];
    }
    out->V = useCLF ? clf[0] : 0.0;
    out->dV = dV;

    /* ---- swing-leg PD (:71-91) */
    if (conDim < 12) {
        const int sw = 12 - conDim;
        double JsD[12 * NQ], JsT[NQ * 12], Dl[12 * 12], pdv[12], vdv[12], kv[12];
        int piv[12];
        mm(sw, NQ, NQ, in->Js, NU, in->Dinv, NQ, JsD);
        tr(sw, NQ, in->Js, NU, JsT);
        mm(sw, NQ, sw, JsD, sw, JsT, NQ, Dl);      /* Delta_temp (sw x sw, col-major) */
        /* Delta = Delta_temp^-1: diagonal only is used; LU solve with unit vectors */
        double Dt[12 * 12];
        for (int i = 0; i < sw; i++) for (int j = 0; j < sw; j++) Dt[i * sw + j] = Dl[j * sw + i];   /* row-major */
        orc_lu(sw, Dt, piv);
        double diag[12];
        for (int j = 0; j < sw; j++) {
            double e[12] = {0};
            e[j] = 1.0;
            orc_lu_solve(sw, Dt, piv, e);
            diag[j] = e[j];
        }
        const double Kd = 40, wd = 40;
        int cs = 0;
        for (int i = 0; i < 4; i++)
            if (in->ind[i] == 0) {
                for (int r = 0; r < 3; r++) {
                    pdv[cs + r] = in->hd[6 + cs + r] - in->toePos[3 * i + r];
                    double jv = 0;
                    for (int t = 0; t < NQ; t++) jv += in->Jtoe[t * NU + 3 * i + r] * in->dq[t];
                    vdv[cs + r] = in->dhd[6 + cs + r] - jv;
                    kv[cs + r] = wd * wd * diag[cs + r];
                }
                cs += 3;
            }
        for (int t = 0; t < NQ; t++) {
            double s = 0;
            for (int r = 0; r < sw; r++) s += JsT[r * NQ + t] * (kv[r] * pdv[r] + Kd * vdv[r]);
            tau[t] += s;
        }
    }

    /* ---- joint accelerations / integration (:96-98) */
    double rhs[NQ];
    for (int t = 0; t < NQ; t++) {
        double s = 0;
        for (int j = 0; j < NU; j++) s += in->B[j * NQ + t] * tau[6 + j];
        double s2 = 0;
        for (int r = 0; r < 12; r++) s2 += in->Jtoe[t * NU + r] * out->QP_force[r];
        rhs[t] = s + s2 - in->Hv[t];
    }
    for (int t = 0; t < NQ; t++) {
        double s = 0;
        for (int j = 0; j < NQ; j++) s += in->Dinv[j * NQ + t] * rhs[j];
        out->ddq[t] = s;
    }
    for (int t = 0; t < NQ; t++) out->dq[t] = in->dq[t] + out->ddq[t] / LLHZ;
    for (int t = 0; t < NQ; t++) out->q[t] = in->q[t] + out->dq[t] / LLHZ + 0.5 / (LLHZ * LLHZ) * out->ddq[t];

    /* ---- swingInvKin (:446-488); Jhip rows are taken at the swing counter (:467), as in
     *      the reference */
    if (conDim != 12) {
        int cs = 0;
        for (int i = 0; i < 4; i++)
            if (in->ind[i] == 0) {
                double dxde[3], xde[3], xe[3], Jth[3][3], Jq[3][3];
                for (int r = 0; r < 3; r++) {
                    double jv = 0;
                    for (int t = 0; t < NQ; t++) jv += in->Jhip[t * NU + cs + r] * in->dq[t];
                    dxde[r] = in->dhd[6 + cs + r] - jv;
                    xde[r] = in->hd[6 + cs + r] - in->hipPos[3 * i + r];
                    xe[r] = in->toePos[3 * i + r] - in->hipPos[3 * i + r];
                    for (int j = 0; j < 3; j++) {
                        Jth[r][j] = in->Jtoe[(3 + j) * NU + 3 * i + r] - in->Jhip[(3 + j) * NU + 3 * i + r];
                        Jq[r][j] = in->Jtoe[(6 + 3 * i + j) * NU + 3 * i + r] - in->Jhip[(6 + 3 * i + j) * NU + 3 * i + r];
                    }
                }
                double rv[3];
                for (int r = 0; r < 3; r++) {
                    double s = 0;
                    for (int j = 0; j < 3; j++) s += Jth[r][j] * in->dq[3 + j];
                    rv[r] = dxde[r] + 20 * (xde[r] - xe[r]) - s;
                }
                /* Jq is block diagonal over the swing legs: its inverse is the blockwise inverse */
                double L[9]; int pv[3];
                for (int r = 0; r < 3; r++) for (int j = 0; j < 3; j++) L[r * 3 + j] = Jq[r][j];
                orc_lu(3, L, pv);
                orc_lu_solve(3, L, pv, rv);
                for (int r = 0; r < 3; r++) {
                    out->dq[6 + 3 * i + r] = rv[r];
                    out->q[6 + 3 * i + r] = in->q[6 + 3 * i + r] + rv[r] / LLHZ;
                }
                cs += 3;
            }
    }
    return flag;
}

/* agent-major flat arrays, strides of srb_ll_io (include/srbnmpc.h) */
int orc_ll_calc_torque_batch(const orc_ll_params *prm, int n_agents, const int *ind, const double *q, const double *dq,
                             const double *Dinv, const double *B, const double *Hv, const double *Jc, const double *dJc,
                             const double *Js, const double *Jtoe, const double *Jhip, const double *toePos,
                             const double *hipPos, const double *H0, const double *dH0, const double *y,
                             const double *dy, const double *hd, const double *dhd, const double *fDes, double *tau,
                             double *QP_force, double *ddq, double *dq_out, double *q_out, double *V, double *dV,
                             double *x, int *status, int *iters)
{
    for (int a = 0; a < n_agents; a++) {
        orc_ll_agent in;
        for (int i = 0; i < 4; i++) in.ind[i] = ind[4 * a + i];
        in.q = q + NQ * a; in.dq = dq + NQ * a;
        in.Dinv = Dinv + NQ * NQ * a; in.B = B + NQ * NU * a; in.Hv = Hv + NQ * a;
        in.Jc = Jc + NU * NQ * a; in.dJc = dJc + NU * a; in.Js = Js + NU * NQ * a;
        in.Jtoe = Jtoe + NU * NQ * a; in.Jhip = Jhip + NU * NQ * a;
        in.toePos = toePos + 12 * a; in.hipPos = hipPos + 12 * a;
        in.H0 = H0 + NQ * NQ * a; in.dH0 = dH0 + NQ * a; in.y = y + NQ * a; in.dy = dy + NQ * a;
        in.hd = hd + NQ * a; in.dhd = dhd + NQ * a; in.fDes = fDes + NU * a;
        orc_ll_out o;
        for (int i = 0; i < NQ; i++) o.tau[i] = tau[NQ * a + i];
        orc_ll_calc_torque(prm, &in, &o);
        for (int i = 0; i < NQ; i++) {
            tau[NQ * a + i] = o.tau[i]; ddq[NQ * a + i] = o.ddq[i];
            dq_out[NQ * a + i] = o.dq[i]; q_out[NQ * a + i] = o.q[i];
        }
        for (int i = 0; i < 12; i++) QP_force[12 * a + i] = o.QP_force[i];
        for (int i = 0; i < 32; i++) x[32 * a + i] = o.x[i];
        V[a] = o.V; dV[a] = o.dV; status[a] = o.status; iters[a] = o.iters;
    }
    return 0;
}

/* the same, split over nthreads pthreads by contiguous agent ranges (bench.py cpu_baseline) */
typedef struct {
    const orc_ll_params *prm; int n;
    const int *ind; const double *in[19]; double *tau, *QP_force, *ddq, *dq_out, *q_out, *V, *dV, *x;
    int *status, *iters;
} ll_job;

static void *ll_worker(void *arg)
{
    ll_job *j = (ll_job *)arg;
    const double *const *i = j->in;
    orc_ll_calc_torque_batch(j->prm, j->n, j->ind, i[0], i[1], i[2], i[3], i[4], i[5], i[6], i[7], i[8], i[9], i[10],
                             i[11], i[12], i[13], i[14], i[15], i[16], i[17], i[18], j->tau, j->QP_force, j->ddq,
                             j->dq_out, j->q_out, j->V, j->dV, j->x, j->status, j->iters);
    return NULL;
}

int orc_ll_calc_torque_batch_mt(const orc_ll_params *prm, int nthreads, int n_agents, const int *ind, const double *q,
                                const double *dq, const double *Dinv, const double *B, const double *Hv,
                                const double *Jc, const double *dJc, const double *Js, const double *Jtoe,
                                const double *Jhip, const double *toePos, const double *hipPos, const double *H0,
                                const double *dH0, const double *y, const double *dy, const double *hd,
                                const double *dhd, const double *fDes, double *tau, double *QP_force, double *ddq,
                                double *dq_out, double *q_out, double *V, double *dV, double *x, int *status,
                                int *iters)
{
    static const int per[19] = {NQ, NQ, NQ * NQ, NQ * NU, NQ, NU * NQ, NU, NU * NQ, NU * NQ, NU * NQ, 12, 12,
                                NQ * NQ, NQ, NQ, NQ, NQ, NQ, NU};
    const double *in[19] = {q, dq, Dinv, B, Hv, Jc, dJc, Js, Jtoe, Jhip, toePos, hipPos, H0, dH0, y, dy, hd, dhd, fDes};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    ll_job jobs[64];
    int created[64] = {0};
    for (int t = 0; t < nthreads; t++) {
        const int lo = (int)((long long)n_agents * t / nthreads), hi = (int)((long long)n_agents * (t + 1) / nthreads);
        ll_job *j = &jobs[t];
        j->prm = prm; j->n = hi - lo; j->ind = ind + 4 * lo;
        for (int k = 0; k < 19; k++) j->in[k] = in[k] + (size_t)per[k] * lo;
        j->tau = tau + NQ * lo; j->QP_force = QP_force + 12 * lo; j->ddq = ddq + NQ * lo; j->dq_out = dq_out + NQ * lo;
        j->q_out = q_out + NQ * lo; j->V = V + lo; j->dV = dV + lo; j->x = x + 32 * lo; j->status = status + lo;
        j->iters = iters + lo;
        if (j->n <= 0) continue;
        if (pthread_create(&th[t], NULL, ll_worker, j) == 0) created[t] = 1;
        else ll_worker(j);
    }
    for (int t = 0; t < nthreads; t++)
        if (created[t]) pthread_join(th[t], NULL);
    return 0;
}
