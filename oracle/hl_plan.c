/*
 * ORACLE (test infrastructure only): the offline HL reference planner
 * MPC_dist::generateReferenceTrajectory, /root/reference/src/MPC_dist.cpp:930-1104, restated
 * for NA agents (the reference hard-codes NUMBER_OF_AGENTS = 4 in F and Pr, :982, :1057).
 *
 * Per step i < loop, for every agent k from the positions of step i:
 *   F_att   = -alpha (p_k - g) / |p_k - g|                                  (:1002)
 *   F_rep   = sum_{j: d_j < dmin} eta (1/d_j - 1/dmin) (1/d_j^2) (p_k - o_j)/|p_k - o_j|   (:1011-1019)
 *   F_agent = - sum_{j != k} 4 eps (6 s^6 / d^7 - 12 s^12 / d^13) (p_k - p_j)/|p_k - p_j|   (:1022-1032)
 *   F = F_att + F_rep + F_agent, or 0 F_att within 1 mm of the goal         (:1034-1039)
 *   q_{i+1} = Ad q_i + (Bd F) scale, scale = i / 1000 for i < 1000           (:1042-1044)
 * with the reference's numeric Ad, Bd (:939-961; state x, y, xdot, ydot).  Output (:1047-1067):
 * every 40th state, read from column 2 of the in-place subsampled q -- so the last two output
 * columns are the UNsampled states T and T+1 (T = loop / 40), reproduced here.
 *   Pr, Prd: column-major 2NA x T (Eigen layout): element (row, col) at col * 2NA + row.
 * Arithmetic is written out operation by operation with no contraction (the HIP kernel
 * mirrors it, so the two agree bit for bit); pow(d, 7) / pow(d, 13) are evaluated as
 * products (within a few ulp of libm pow, the only departure from the reference).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

/* built with -ffp-contract=off (oracle/Makefile) */

void orc_hl_plan(int NA, const double *Pstart, const double *Pobs, int n_obs, int loop, double *Pr, double *Prd)
{
    const double epsilon = 60, sigma = 1.0, alpha = 150.0, eta = 400.0, dmin = 1.0;
    const double gx = 10.0, gy = 0.0;                       /* GOAL_X, GOAL_Y (global_loco_opts.h:12-13) */
    const double a01 = 0.001025061239872, a22 = 0.929527039758809;
    const double b00 = 0.000000068070472960, b20 = 0.000128132654983983;
    const int T = loop / 40, R = 2 * NA;
    const double s6 = 6 * (sigma * sigma * sigma * sigma * sigma * sigma);
    const double s12 = 12 * (sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma);
    double *q = (double *)calloc((size_t)4 * NA, sizeof(double)), *qn = (double *)calloc((size_t)4 * NA, sizeof(double));
    for (int k = 0; k < NA; k++) { q[4 * k] = Pstart[2 * k]; q[4 * k + 1] = Pstart[2 * k + 1]; }
    for (int i = 0; i <= loop; i++) {
        /* record: output column j = (2 + j < T) ? state 40 (2 + j) : state 2 + j (a state can
         * land in two columns, e.g. state T when T is a multiple of 40) */
        int cols[2], nc = 0;
        if (i % 40 == 0 && i / 40 >= 2 && i / 40 < T) cols[nc++] = i / 40 - 2;
        if (T >= 2 && i == T) cols[nc++] = T - 2;
        if (T >= 1 && i == T + 1) cols[nc++] = T - 1;
        for (int c = 0; c < nc; c++)
            for (int k = 0; k < NA; k++) {
                const int j = cols[c];
                Pr[(size_t)j * R + 2 * k] = q[4 * k]; Pr[(size_t)j * R + 2 * k + 1] = q[4 * k + 1];
                Prd[(size_t)j * R + 2 * k] = q[4 * k + 2]; Prd[(size_t)j * R + 2 * k + 1] = q[4 * k + 3];
            }
        if (i == loop) break;
        const double scale = (i < 1000) ? ((double)i / 1000) : 1.0;
        for (int k = 0; k < NA; k++) {
            const double px = q[4 * k], py = q[4 * k + 1];
            const double ex = px - gx, ey = py - gy;
            const double dg = sqrt(ex * ex + ey * ey);
            const double fax = -alpha * (ex / dg), fay = -alpha * (ey / dg);
            double frx = 0.0, fry = 0.0;
            for (int o = 0; o < n_obs; o++) {
                const double vx = px - Pobs[2 * o], vy = py - Pobs[2 * o + 1];
                const double d = sqrt(vx * vx + vy * vy);
                if (d < dmin) {
                    const double c = (eta * (1 / d - 1 / dmin)) * (1 / (d * d));
                    frx = frx + c * (vx / d); fry = fry + c * (vy / d);
                }
            }
            double fgx = 0.0, fgy = 0.0;
            for (int jn = 0; jn < NA; jn++) {
                if (jn == k) continue;
                const double vx = px - q[4 * jn], vy = py - q[4 * jn + 1];
                const double d = sqrt(vx * vx + vy * vy);
                const double d2 = d * d, d3 = d2 * d, d6 = d3 * d3, d7 = d6 * d, d13 = d6 * d7;
                const double c = (4 * epsilon) * (s6 / d7 - s12 / d13);
                fgx = fgx - c * (vx / d); fgy = fgy - c * (vy / d);
            }
            double fx = (fax + frx) + fgx, fy = (fay + fry) + fgy;
            if (dg < 0.001) { fx = 0 * fax; fy = 0 * fay; }
            const double x = q[4 * k], y = q[4 * k + 1], xd = q[4 * k + 2], yd = q[4 * k + 3];
            qn[4 * k] = (x + a01 * xd) + (b00 * fx) * scale;
            qn[4 * k + 1] = (y + a01 * yd) + (b00 * fy) * scale;
            qn[4 * k + 2] = (a22 * xd) + (b20 * fx) * scale;
            qn[4 * k + 3] = (a22 * yd) + (b20 * fy) * scale;
        }
        double *t = q; q = qn; qn = t;
    }
    free(q); free(qn);
}
