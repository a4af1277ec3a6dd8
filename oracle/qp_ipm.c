/*
 * ORACLE (test infrastructure only): the iSWIFT primal-dual interior-point method
 * restated step for step from /root/reference/optimization/iSWIFT/src/Prime.c:127-230
 * and src/Auxilary.c (kkt_initialize :680-755, computeresiduals :524-553,
 * formlambda :462-465, form_ds :250-267, findsteplength :271-294, formrho :600-609,
 * kktsolve_1/2 :334-398, updatevariables :224-227).
 *
 * Only the linear algebra differs: iSWIFT factors the sparse unreduced KKT
 *     [P A' G'; A 0 0; G 0 -W]
 * with a regularised up-looking LDL' (ldl.c:254-326); here dz is eliminated (W is
 * diagonal) and the full-space [P + G'W^-1 G, A'; A, 0] is factored densely by LU with
 * partial pivoting.  In exact arithmetic both give the same Newton step.  (A Schur
 * complement on dy is NOT used: with interior contact weights the lambda block of
 * P + G'W^-1 G is O(mu) and A H^-1 A' loses definiteness to round-off near convergence.)
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

typedef struct {
    int n, m, p;
    const double *Pd, *Pf, *A, *G;   /* P diagonal (Pd) or full row-major (Pf, when non-NULL) */
    int gk;        /* max nonzeros of a G row */
    int *gnz;      /* [m][gk] column indices of row r's nonzeros (-1 padded) */
    double *gval;  /* [m][gk] */
    double *H, *t1, *t2;
    double *K; int *piv;
} kktws;

static void ws_init(kktws *w, int n, int m, int p, const double *Pd, const double *A, const double *G)
{
    w->n = n; w->m = m; w->p = p; w->Pd = Pd; w->Pf = NULL; w->A = A; w->G = G;
    int gk = 1;
    for (int r = 0; r < m; r++) {
        int k = 0;
        for (int j = 0; j < n; j++) k += (G[(size_t)r * n + j] != 0.0);
        if (k > gk) gk = k;
    }
    w->gk = gk;
    w->gnz = (int *)malloc(sizeof(int) * (size_t)gk * (size_t)(m > 0 ? m : 1));
    w->gval = (double *)malloc(sizeof(double) * (size_t)gk * (size_t)(m > 0 ? m : 1));
    for (int r = 0; r < m; r++) {
        int k = 0;
        for (int j = 0; j < gk; j++) { w->gnz[gk * r + j] = -1; w->gval[gk * r + j] = 0; }
        for (int j = 0; j < n; j++)
            if (G[(size_t)r * n + j] != 0.0) { w->gnz[gk * r + k] = j; w->gval[gk * r + k] = G[(size_t)r * n + j]; k++; }
    }
    w->H = (double *)malloc(sizeof(double) * n * n);
    w->t1 = (double *)malloc(sizeof(double) * (n + p + m + 8));
    w->t2 = (double *)malloc(sizeof(double) * (n + p + m + 8));
    w->K = (double *)malloc(sizeof(double) * (size_t)(n + p) * (n + p));
    w->piv = (int *)malloc(sizeof(int) * (n + p));
}

static void ws_free(kktws *w)
{
    free(w->gnz); free(w->gval); free(w->H); free(w->t1); free(w->t2);
    free(w->K); free(w->piv);
}

static void gmul(const kktws *w, const double *x, double *y)   /* y = G x */
{
    for (int r = 0; r < w->m; r++) {
        double s = 0;
        for (int k = 0; k < w->gk; k++) if (w->gnz[w->gk * r + k] >= 0) s += w->gval[w->gk * r + k] * x[w->gnz[w->gk * r + k]];
        y[r] = s;
    }
}

static void gtmul_add(const kktws *w, const double *v, double *y)   /* y += G' v */
{
    for (int r = 0; r < w->m; r++)
        for (int k = 0; k < w->gk; k++) if (w->gnz[w->gk * r + k] >= 0) y[w->gnz[w->gk * r + k]] += w->gval[w->gk * r + k] * v[r];
}

/* factor for weights wgt (W = diag(wgt)); returns 0 on success */
static int kkt_factor(kktws *w, const double *wgt)
{
    const int n = w->n, m = w->m, p = w->p;
    double *H = w->H;
    memset(H, 0, sizeof(double) * n * n);
    if (w->Pf) memcpy(H, w->Pf, sizeof(double) * n * n);
    else for (int i = 0; i < n; i++) H[i * n + i] = w->Pd[i];
    for (int r = 0; r < m; r++) {
        double iw = 1.0 / wgt[r];
        for (int a = 0; a < w->gk; a++) {
            int ia = w->gnz[w->gk * r + a]; if (ia < 0) continue;
            for (int bb = 0; bb < w->gk; bb++) {
                int ib = w->gnz[w->gk * r + bb]; if (ib < 0) continue;
                H[ia * n + ib] += iw * w->gval[w->gk * r + a] * w->gval[w->gk * r + bb];
            }
        }
    }
    {
        const int d = n + p;
        memset(w->K, 0, sizeof(double) * (size_t)d * d);
        for (int i = 0; i < n; i++) for (int j = 0; j < n; j++) w->K[(size_t)i * d + j] = H[i * n + j];
        for (int k = 0; k < p; k++)
            for (int j = 0; j < n; j++) {
                w->K[(size_t)(n + k) * d + j] = w->A[(size_t)k * n + j];
                w->K[(size_t)j * d + n + k] = w->A[(size_t)k * n + j];
            }
        return orc_lu(d, w->K, w->piv);
    }
}

/* solve [P A' G'; A 0 0; G 0 -W][dx;dy;dz] = [r1;r2;r3] with the current factor */
static void kkt_solve(kktws *w, const double *wgt, const double *r1, const double *r2, const double *r3,
                      double *dx, double *dy, double *dz)
{
    const int n = w->n, m = w->m, p = w->p;
    double *g = w->t1, *t = w->t2;
    for (int i = 0; i < n; i++) g[i] = r1[i];
    for (int r = 0; r < m; r++) t[r] = r3[r] / wgt[r];
    gtmul_add(w, t, g);                                   /* g = r1 + G' W^-1 r3 */
    for (int i = 0; i < n; i++) t[i] = g[i];
    for (int k = 0; k < p; k++) t[n + k] = r2[k];
    orc_lu_solve(n + p, w->K, w->piv, t);
    for (int i = 0; i < n; i++) dx[i] = t[i];
    for (int k = 0; k < p; k++) dy[k] = t[n + k];
    gmul(w, dx, dz);
    for (int r = 0; r < m; r++) dz[r] = (dz[r] - r3[r]) / wgt[r];
}

static double norm2(const double *v, int n) { double s = 0; for (int i = 0; i < n; i++) s += v[i] * v[i]; return sqrt(s); }
static double dot(const double *a, const double *b, int n) { double s = 0; for (int i = 0; i < n; i++) s += a[i] * b[i]; return s; }

/* findsteplength, Auxilary.c:271-294 */
static double steplen(const double *v, const double *dv, int m)
{
    double a = 1e10; int f = 0;
    for (int i = 0; i < m; i++)
        if (dv[i] < 0 && (-v[i] / dv[i]) < a) { a = -(v[i] / dv[i]); f = 1; }
    return f ? a : 1.0;
}

static int qp_solve_impl(int n, int m, int p, const double *Pd, const double *Pf, const double *c,
                         const double *A, const double *b, const double *G, const double *h,
                         int maxit, double tol, double *x_out, double *q_out, int *iters_out, int no_trap,
                         int *trapped, int qp_init, double zdiv)
{
    kktws w;
    ws_init(&w, n, m, p, Pd, A, G);
    w.Pf = Pf;
    double *x = calloc(n, sizeof(double)), *y = calloc(p + 1, sizeof(double));
    double *s = calloc(m, sizeof(double)), *z = calloc(m, sizeof(double));
    double *rx = calloc(n, sizeof(double)), *ry = calloc(p + 1, sizeof(double)), *rz = calloc(m, sizeof(double));
    double *dx = calloc(n, sizeof(double)), *dy = calloc(p + 1, sizeof(double)), *dz = calloc(m, sizeof(double));
    double *dsv = calloc(m, sizeof(double)), *ds = calloc(m, sizeof(double)), *lam = calloc(m, sizeof(double));
    double *wgt = calloc(m, sizeof(double)), *r3 = calloc(m, sizeof(double)), *zi = calloc(m, sizeof(double));
    double *nc = calloc(n, sizeof(double));
    int flag = 3, it = 0;

    /* kkt_initialize (Auxilary.c:680-755): W = I, rhs [-c; b; h] */
    for (int r = 0; r < m; r++) wgt[r] = 1.0;
    if (kkt_factor(&w, wgt)) { flag = 1; goto done; }
    for (int i = 0; i < n; i++) nc[i] = -c[i];
    kkt_solve(&w, wgt, nc, b, h, x, y, dz);
    gmul(&w, x, zi);
    for (int r = 0; r < m; r++) zi[r] = h[r] - zi[r];     /* z_inter = h - G x */
    {
        double mn = zi[0], mx = zi[0];
        for (int r = 1; r < m; r++) { if (zi[r] < mn) mn = zi[r]; if (zi[r] > mx) mx = zi[r]; }
        double ap = -mn, ad = mx;
        for (int r = 0; r < m; r++) s[r] = (ap < 0) ? zi[r] : zi[r] + (1 + ap);
        for (int r = 0; r < m; r++) z[r] = (ad < 0) ? -zi[r] : -zi[r] + (1 + ad);
        /* scaled start (qp_init = 1, the kernel's default): the same x, s_r = max(h_r - (Gx)_r, 0.1),
         * z_r = 1 / s_r.  iSWIFT shifts every z by 1 + max_r(h - Gx)_r, which the +-1e3 boxes on X
         * and U (MPC_dist.cpp:317-318) make ~1e3: mu starts near 5e4, the dual steps stay blocked
         * (alpha_d 0.01-0.1) for many iterations, and the slowest bench agents need 18-19; from the
         * scaled start the same QPs take at most 9 and end within 4e-8 of iSWIFT's point
         * (DESIGN.md 3).  iSWIFT's start stays available (qp_init = 0) for step-for-step checks. */
        if (qp_init == 1)
            for (int r = 0; r < m; r++) { s[r] = fmax(zi[r], 0.1); z[r] = 1.0 / s[r]; }
    }

    double sigma = 100.0;                  /* options->sigma = SIGMA (GlobalOptions.h:26) */
    const double sigma_d = 0.0;            /* iswift_qp.cpp:103 */
    double alpha_p = 0, alpha_d = 0;
    flag = 2;
    for (int i = 0; i < maxit; i++) {
        /* computeresiduals: rx = -Px - G'z - A'y - c; ry = -Ax + b; rz = -s - Gx + h */
        for (int j = 0; j < n; j++) {
            double px = 0;
            if (Pf) for (int k = 0; k < n; k++) px += Pf[(size_t)j * n + k] * x[k];
            else px = Pd[j] * x[j];
            rx[j] = -px - c[j];
        }
        for (int r = 0; r < m; r++) lam[r] = -z[r];
        gtmul_add(&w, lam, rx);
        for (int k = 0; k < p; k++) {
            double sy = 0;
            for (int j = 0; j < n; j++) sy += A[(size_t)k * n + j] * x[j];
            ry[k] = b[k] - sy;
            for (int j = 0; j < n; j++) rx[j] -= A[(size_t)k * n + j] * y[k];
        }
        gmul(&w, x, rz);
        for (int r = 0; r < m; r++) rz[r] = h[r] - s[r] - rz[r];
        const double th = tol / sqrt(3.0);
        /* divergence (zdiv > 0: the NMPC's QP stage, ORC_Z_DIV): a dual beyond zdiv means the rows
         * are infeasible -- the duals of converging solves stay below ~1e4 on every workload, those of
         * infeasible ones pass 1e10 within a few iterations and then overflow.  FATAL at this
         * (finite) iterate, as the kernel (srb_kernels.hip, the same rule and threshold) */
        if (zdiv > 0) {
            double zm = 0.0;
            for (int r = 0; r < m; r++) zm = fmax(zm, z[r]);
            if (!(zm <= zdiv)) { flag = 3; break; }
        }
        if (norm2(rx, n) < th && norm2(rz, m) < th && (p == 0 || norm2(ry, p) < th) && dot(s, z, m) / m < tol) {
            flag = 0; break;
        }
        for (int r = 0; r < m; r++) lam[r] = sqrt(s[r] * z[r]);
        double mu = dot(lam, lam, m) / m;
        if (sigma > sigma_d || no_trap) {
            /* updatekktmatrix(indicator 0) + ldl_numeric inside kktsolve_1 (Prime.c:165-177) */
            for (int r = 0; r < m; r++) wgt[r] = s[r] / z[r];
            if (kkt_factor(&w, wgt)) { flag = 1; break; }
            for (int r = 0; r < m; r++) { ds[r] = -lam[r] * lam[r]; r3[r] = rz[r] - ds[r] / z[r]; }
            kkt_solve(&w, wgt, rx, ry, r3, dx, dy, dz);       /* kktsolve_1: only dz, ds used */
            for (int r = 0; r < m; r++) dsv[r] = (ds[r] - s[r] * dz[r]) / z[r];
            alpha_p = steplen(s, dsv, m); alpha_d = steplen(z, dz, m);
            double num = 0;
            for (int r = 0; r < m; r++) num += (s[r] + alpha_p * dsv[r]) * (z[r] + alpha_d * dz[r]);
            double rho = num / dot(s, z, m);
            double mr = rho < 1 ? rho : 1;
            sigma = mr * mr * mr; if (sigma < sigma_d) sigma = sigma_d;
            for (int r = 0; r < m; r++) ds[r] = -(lam[r] * lam[r]) - (dsv[r] * dz[r]) + sigma * mu;
        } else {
            /* Prime.c:193-196: no refactorisation -- kktsolve_2 reuses the previous factor */
            sigma = sigma_d;
            if (trapped) *trapped = 1;
            for (int r = 0; r < m; r++) ds[r] = -(lam[r] * lam[r]) + sigma * mu;
        }
        for (int r = 0; r < m; r++) r3[r] = rz[r] - ds[r] / z[r];
        kkt_solve(&w, wgt, rx, ry, r3, dx, dy, dz);           /* kktsolve_2 */
        for (int r = 0; r < m; r++) dsv[r] = (ds[r] - s[r] * dz[r]) / z[r];
        alpha_p = steplen(s, dsv, m); alpha_d = steplen(z, dz, m);
        if (getenv("ORC_QP_TRACE"))
            fprintf(stderr, "  qp %2d  |rx| %.2e |rz| %.2e |ry| %.2e  mu %.2e  ap %.3f ad %.3f sigma %.2e\n", i, norm2(rx, n),
                    norm2(rz, m), norm2(ry, p), dot(s, z, m) / m, alpha_p, alpha_d, sigma);
        alpha_p = 0.99 * alpha_p < 1.0 ? 0.99 * alpha_p : 1.0;
        alpha_d = 0.99 * alpha_d < 1.0 ? 0.99 * alpha_d : 1.0;
        for (int j = 0; j < n; j++) x[j] += dx[j] * alpha_p;
        for (int k = 0; k < p; k++) y[k] += dy[k] * alpha_d;
        for (int r = 0; r < m; r++) { s[r] += dsv[r] * alpha_p; z[r] += dz[r] * alpha_d; }
        it++;
    }
done:
    memcpy(x_out, x, sizeof(double) * n);
    if (q_out) {                                   /* q = A' y (equality multipliers in x-space) */
        for (int j = 0; j < n; j++) q_out[j] = 0;
        for (int k = 0; k < p; k++) for (int j = 0; j < n; j++) q_out[j] += A[(size_t)k * n + j] * y[k];
    }
    if (iters_out) *iters_out = it;
    free(x); free(y); free(s); free(z); free(rx); free(ry); free(rz); free(dx); free(dy); free(dz);
    free(dsv); free(ds); free(lam); free(wgt); free(r3); free(zi); free(nc);
    ws_free(&w);
    return flag;
}

int orc_qp_solve_init(int n, int m, int p, const double *Pd, const double *c, const double *A, const double *b,
                      const double *G, const double *h, int maxit, double tol, int qp_init, double *x_out, double *q_out,
                      int *iters_out)
{
    return qp_solve_impl(n, m, p, Pd, NULL, c, A, b, G, h, maxit, tol, x_out, q_out, iters_out, 0, NULL, qp_init, ORC_Z_DIV);
}

int orc_qp_solve(int n, int m, int p, const double *Pd, const double *c,
                 const double *A, const double *b, const double *G, const double *h,
                 int maxit, double tol, double *x_out, double *q_out, int *iters_out)
{
    return qp_solve_impl(n, m, p, Pd, NULL, c, A, b, G, h, maxit, tol, x_out, q_out, iters_out, 0, NULL, 0, 0.0);
}

/* iSWIFT with the sigma <= sigma_d branch (Prime.c:193-196) disabled.  The step-length rule keeps
 * both factors of every product in rho non-negative, so rho <= 0 (sigma = 0) arises only from
 * rounding at a blocking row; iSWIFT then freezes the KKT factor for the rest of the solve and
 * usually ends at MAXIT.  The low-level controller's kernel keeps the predictor-corrector path
 * instead; this is its oracle. */
int orc_qp_solve_nt(int n, int m, int p, const double *Pd, const double *c,
                    const double *A, const double *b, const double *G, const double *h,
                    int maxit, double tol, double *x_out, int *iters_out)
{
    return qp_solve_impl(n, m, p, Pd, NULL, c, A, b, G, h, maxit, tol, x_out, NULL, iters_out, 1, NULL, 0, 0.0);
}

/* iSWIFT semantics, reporting whether the sigma <= sigma_d branch was taken */
int orc_qp_solve_trap(int n, int m, int p, const double *Pd, const double *c,
                      const double *A, const double *b, const double *G, const double *h,
                      int maxit, double tol, double *x_out, int *iters_out, int *trapped)
{
    *trapped = 0;
    return qp_solve_impl(n, m, p, Pd, NULL, c, A, b, G, h, maxit, tol, x_out, NULL, iters_out, 0, trapped, 0, 0.0);
}

/* general (full, symmetric) P -- used for iSWIFT's own test QP (Matrices_small.h) */
int orc_qp_solve_full(int n, int m, int p, const double *P, const double *c,
                      const double *A, const double *b, const double *G, const double *h,
                      int maxit, double tol, double *x_out, int *iters_out)
{
    return qp_solve_impl(n, m, p, NULL, P, c, A, b, G, h, maxit, tol, x_out, NULL, iters_out, 0, NULL, 0, 0.0);
}
