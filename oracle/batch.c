/* ORACLE (test infrastructure only): one agent end to end + a pthread batch driver. */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "oracle.h"

int orc_solve_agent(const orc_params *p_in, const double x0[4], const double *ref, const double *foot,
                    const double *obstacles, int n_obs, const double *nbr_state, int n_all, int self_idx,
                    double *x_qp, double *x_out, double *obj, int status[2], int iters[2])
{
    /* "up to K nearest": clamp to what exists, as the product's C ABI does */
    orc_params pc = *p_in;
    const orc_params *p = &pc;
    if (pc.K_obs > n_obs) pc.K_obs = n_obs > 0 ? n_obs : 0;
    {
        int others = nbr_state ? n_all - 1 : 0;
        if (pc.K_nbr > others) pc.K_nbr = others > 0 ? others : 0;
    }
    const int nv = orc_nv(p), neq = orc_neq(p), mq = orc_mqp(p), K = p->K_obs + p->K_nbr;
    double *Pd = malloc(sizeof(double) * nv), *c = malloc(sizeof(double) * nv);
    double *A = malloc(sizeof(double) * (size_t)neq * nv), *b = malloc(sizeof(double) * neq);
    double *G = malloc(sizeof(double) * (size_t)mq * nv), *h = malloc(sizeof(double) * mq);
    double *xq = malloc(sizeof(double) * nv);
    orc_build_qp(p, x0, ref, foot, Pd, c, A, b, G, h);
    /* the QP stage that the NLP follows runs to tol_qp: its point only warm-starts the NLP (the kernel's
     * SRB_OPT_QP_WARM_TOL; the reference runs iSWIFT to 1e-6 there -- a documented deviation) */
    const double tq = (p->use_nlp && p->tol_qp > 0.0) ? p->tol_qp : p->tol;
    status[0] = orc_qp_solve_init(nv, mq, neq, Pd, c, A, b, G, h, p->qp_maxit, tq, p->qp_init, xq, NULL, &iters[0]);
    if (status[0] == 0 && tq > p->tol) status[0] = 4;      /* converged at the warm-start tolerance only (the kernel's rule) */
    if (x_qp) memcpy(x_qp, xq, sizeof(double) * nv);
    status[1] = 0; iters[1] = 0;
    if (p->use_nlp) {
        double *obs = malloc(sizeof(double) * (size_t)p->N * (K ? K : 1) * 2), *eps = malloc(sizeof(double) * (K ? K : 1));
        orc_select_obstacles(p, x0, obstacles, n_obs, nbr_state, n_all, self_idx, obs, eps);
        status[1] = orc_nlp_solve(p, x0, foot, Pd, c, A, b, G, h, obs, eps, xq, x_out, &iters[1]);
        free(obs); free(eps);
    } else {
        memcpy(x_out, xq, sizeof(double) * nv);
    }
    double f = 0;
    for (int i = 0; i < nv; i++) f += 0.5 * Pd[i] * x_out[i] * x_out[i] + c[i] * x_out[i];   /* ExCost::GetCost */
    *obj = f;
    free(Pd); free(c); free(A); free(b); free(G); free(h); free(xq);
    return status[0] | (status[1] << 4);
}

typedef struct {
    const orc_params *p; int lo, hi;
    const double *x0, *ref, *foot, *obstacles, *nbr; int n_obs, n_all, off;
    double *x_qp, *x_out, *obj; int *status, *iters;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    const orc_params *p = j->p;
    const int nv = orc_nv(p), N = p->N, C = p->C;
    for (int a = j->lo; a < j->hi; a++)
        orc_solve_agent(p, j->x0 + 4 * a, j->ref + (size_t)4 * N * a, j->foot + (size_t)2 * N * C * a,
                        j->obstacles, j->n_obs, j->nbr, j->n_all, j->off + a,
                        j->x_qp ? j->x_qp + (size_t)nv * a : NULL, j->x_out + (size_t)nv * a, j->obj + a,
                        j->status + 2 * a, j->iters + 2 * a);
    return NULL;
}

int orc_solve_batch(const orc_params *p, int n_agents, const double *x0, const double *ref,
                    const double *foot, const double *obstacles, int n_obs,
                    const double *nbr_state, int n_all, int agent_offset,
                    double *x_qp, double *x_out, double *obj, int *status, int *iters, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n_agents) nthreads = n_agents > 0 ? n_agents : 1;
    pthread_t *th = malloc(sizeof(pthread_t) * nthreads);
    job_t *jobs = malloc(sizeof(job_t) * nthreads);
    for (int t = 0; t < nthreads; t++) {
        job_t *j = &jobs[t];
        j->p = p; j->lo = (int)((long)n_agents * t / nthreads); j->hi = (int)((long)n_agents * (t + 1) / nthreads);
        j->x0 = x0; j->ref = ref; j->foot = foot; j->obstacles = obstacles; j->nbr = nbr_state;
        j->n_obs = n_obs; j->n_all = n_all; j->off = agent_offset;
        j->x_qp = x_qp; j->x_out = x_out; j->obj = obj; j->status = status; j->iters = iters;
        pthread_create(&th[t], NULL, worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}
