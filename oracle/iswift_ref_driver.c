/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * Thin driver around the *genuine* vendored iSWIFT solver compiled from
 * /root/reference/optimization/iSWIFT/{src,ldl/src} by oracle/Makefile into
 * oracle/_ref/libiswift_ref.so.  It plays the role of the reference's
 * Eigen wrapper `iswiftQp` (optimization/iSWIFT/cpp_wrapper/iswift_qp.cpp:78-162):
 *   dense -> CCS (`ccstorage`, iswift_qp.cpp:164-182; exact zeros dropped like
 *   Eigen::sparseView), a fill-reducing ordering of the full KKT pattern
 *   (`permutation`, iswift_qp.cpp:184-210 uses Eigen AMDOrdering; here a
 *   plain minimum-degree ordering written for this harness -- the ordering
 *   only changes round-off), then QP_SETUP / QP_SOLVE /
 *   memcpy(x) / QP_CLEANUP with sigma_d = 0.0 (iswift_qp.cpp:103,127-151).
 *
 * This file is our own code; the reference sources are compiled where they
 * lie and are never copied into the repository.
 */
#include <stdlib.h>
#include <string.h>
#include "Prime.h"

/* dense row-major (rows x cols) -> CCS with sorted row indices, zeros dropped */
static int to_ccs(int rows, int cols, const double *D, idxint **jc, idxint **ir, realqp **pr)
{
    int nnz = 0;
    for (int i = 0; i < rows * cols; i++) nnz += (D[i] != 0.0);
    *jc = (idxint *)malloc((cols + 1) * sizeof(idxint));
    *ir = (idxint *)malloc((nnz > 0 ? nnz : 1) * sizeof(idxint));
    *pr = (realqp *)malloc((nnz > 0 ? nnz : 1) * sizeof(realqp));
    int k = 0;
    (*jc)[0] = 0;
    for (int j = 0; j < cols; j++) {
        for (int i = 0; i < rows; i++) {
            double v = D[(size_t)i * cols + j];
            if (v != 0.0) { (*ir)[k] = i; (*pr)[k] = v; k++; }
        }
        (*jc)[j + 1] = k;
    }
    return nnz;
}

/*
 * Minimum-degree ordering on the symmetric pattern of
 *   K = [P A' G'; A 0 0; G 0 -I]
 * using an explicit dense boolean elimination graph (dim <= a few thousand).
 * perm[k] = original index eliminated k-th (the convention ldl_numeric's
 * P argument expects: "kk = P[k]: kth original column").
 */
static void min_degree(int dim, unsigned char *adj, idxint *perm)
{
    unsigned char *done = (unsigned char *)calloc(dim, 1);
    int *deg = (int *)calloc(dim, sizeof(int));
    int *nbr = (int *)malloc(dim * sizeof(int));
    for (int i = 0; i < dim; i++)
        for (int j = 0; j < dim; j++)
            if (i != j && adj[(size_t)i * dim + j]) deg[i]++;
    for (int k = 0; k < dim; k++) {
        int best = -1;
        for (int i = 0; i < dim; i++)
            if (!done[i] && (best < 0 || deg[i] < deg[best])) best = i;
        perm[k] = best;
        done[best] = 1;
        int cnt = 0;
        for (int j = 0; j < dim; j++)
            if (!done[j] && adj[(size_t)best * dim + j]) nbr[cnt++] = j;
        /* eliminate: neighbours become a clique */
        for (int a = 0; a < cnt; a++) {
            int u = nbr[a];
            adj[(size_t)u * dim + best] = 0;
            for (int b = 0; b < cnt; b++) {
                int v = nbr[b];
                if (u != v && !adj[(size_t)u * dim + v]) { adj[(size_t)u * dim + v] = 1; deg[u]++; }
            }
            deg[u]--; /* lost edge to `best` */
        }
    }
    free(done); free(deg); free(nbr);
}

/*
 * Solve  min 0.5 x'Px + c'x  s.t. A x = b, G x <= h  with the genuine iSWIFT.
 * All matrices dense row-major. Returns the iSWIFT exit flag (0..3).
 */
int iswift_ref_solve(int n, int m, int p,
                     const double *P, const double *c,
                     const double *A, const double *b,
                     const double *G, const double *h,
                     double *x_out, int *iters_out,
                     double *t_setup_out, double *t_solve_out)
{
    idxint *Pjc, *Pir, *Ajc, *Air, *Gjc, *Gir;
    realqp *Ppr, *Apr, *Gpr;
    to_ccs(n, n, P, &Pjc, &Pir, &Ppr);
    to_ccs(p, n, A, &Ajc, &Air, &Apr);
    to_ccs(m, n, G, &Gjc, &Gir, &Gpr);

    int dim = n + p + m;
    unsigned char *adj = (unsigned char *)calloc((size_t)dim * dim, 1);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            if (P[(size_t)i * n + j] != 0.0) adj[(size_t)i * dim + j] = 1;
    for (int r = 0; r < p; r++)
        for (int j = 0; j < n; j++)
            if (A[(size_t)r * n + j] != 0.0) {
                adj[(size_t)(n + r) * dim + j] = 1; adj[(size_t)j * dim + n + r] = 1;
            }
    for (int r = 0; r < m; r++)
        for (int j = 0; j < n; j++)
            if (G[(size_t)r * n + j] != 0.0) {
                adj[(size_t)(n + p + r) * dim + j] = 1; adj[(size_t)j * dim + n + p + r] = 1;
            }
    idxint *perm = (idxint *)malloc(dim * sizeof(idxint));
    min_degree(dim, adj, perm);
    free(adj);

    /* iSWIFT keeps pointers to c/h/b without copying (Prime.c:57-59) */
    realqp *cc = (realqp *)malloc(n * sizeof(realqp));
    realqp *hh = (realqp *)malloc((m > 0 ? m : 1) * sizeof(realqp));
    realqp *bb = (realqp *)malloc((p > 0 ? p : 1) * sizeof(realqp));
    memcpy(cc, c, n * sizeof(double));
    if (m) memcpy(hh, h, m * sizeof(double));
    if (p) memcpy(bb, b, p * sizeof(double));

    QP *qp = QP_SETUP(n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, cc, hh, bb, 0.0, perm);
    idxint flag = QP_SOLVE(qp);
    memcpy(x_out, qp->x, n * sizeof(double));
    if (iters_out) *iters_out = qp->stats->IterationCount;
    if (t_setup_out) *t_setup_out = qp->stats->tsetup;
    if (t_solve_out) *t_solve_out = qp->stats->tsolve;
    QP_CLEANUP(qp);

    free(Pjc); free(Pir); free(Ppr); free(Ajc); free(Air); free(Apr);
    free(Gjc); free(Gir); free(Gpr); free(perm); free(cc); free(hh); free(bb);
    return (int)flag;
}

/* Same as above but with a caller-supplied permutation (used for KAT-1, whose
 * fixture ships the reference's own ordering, Matrices_small.h `P[72]`). */
int iswift_ref_solve_ccs(int n, int m, int p,
                         int *Pjc, int *Pir, double *Ppr,
                         int *Ajc, int *Air, double *Apr,
                         int *Gjc, int *Gir, double *Gpr,
                         double *c, double *h, double *b, int *perm,
                         double *x_out, int *iters_out)
{
    QP *qp = QP_SETUP(n, m, p, Pjc, Pir, Ppr, Ajc, Air, Apr, Gjc, Gir, Gpr, c, h, b, 0.0, perm);
    idxint flag = QP_SOLVE(qp);
    memcpy(x_out, qp->x, n * sizeof(double));
    if (iters_out) *iters_out = qp->stats->IterationCount;
    QP_CLEANUP(qp);
    return (int)flag;
}
