// HL reference planner on the device: MPC_dist::generateReferenceTrajectory
// (/root/reference/src/MPC_dist.cpp:930-1104) for NA agents, every agent of the swarm in one
// workgroup (one thread per agent, up to 1024).  Per step each thread evaluates its agent's
// goal attraction, obstacle repulsion and Lennard-Jones interaction with every other agent
// from the positions of the step (double-buffered in LDS, read as wave-wide broadcasts) and
// advances its own state; one barrier per step.  The arithmetic is written out operation by
// operation with contraction off, mirroring oracle/hl_plan.c, so the path is reproduced bit for
// bit (pow(d, 7) / pow(d, 13) as products, within a few ulp of the reference's libm pow).
// Output: every 40th state from column 2 of the reference's in-place subsampled q, whose last
// two columns are the unsampled states T and T+1 (T = loop / 40), reproduced (:1047-1067).
#include <hip/hip_runtime.h>
#include "srbnmpc.h"

#pragma clang fp contract(off)

#define HL_MAX_OBS 2048

extern "C" __global__ void __launch_bounds__(1024) srb_hlplan_kernel(int NA, const double *__restrict__ Pstart,
                                                                     const double *__restrict__ Pobs, int n_obs,
                                                                     int loop, double *__restrict__ Pr,
                                                                     double *__restrict__ Prd)
{
    extern __shared__ double hl_lds[];
    double *pos = hl_lds;                    // [2][NA][2] positions, double-buffered
    double *ob = hl_lds + 4 * NA;            // [n_obs][2]
    const int k = threadIdx.x;
    const double epsilon = 60, sigma = 1.0, alpha = 150.0, eta = 400.0, dmin = 1.0;
    const double gx = 10.0, gy = 0.0;
    const double a01 = 0.001025061239872, a22 = 0.929527039758809;
    const double b00 = 0.000000068070472960, b20 = 0.000128132654983983;
    const double s6 = 6 * (sigma * sigma * sigma * sigma * sigma * sigma);
    const double s12 = 12 * (sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma);
    const int T = loop / 40, R = 2 * NA;
    for (int i = k; i < 2 * n_obs; i += blockDim.x) ob[i] = Pobs[i];
    const bool act = k < NA;
    double x = act ? Pstart[2 * k] : 0.0, y = act ? Pstart[2 * k + 1] : 0.0, xd = 0.0, yd = 0.0;
    if (act) { pos[2 * k] = x; pos[2 * k + 1] = y; }
    __syncthreads();
    int cur = 0;
    for (int i = 0; i <= loop; i++) {
        // output column j = (2 + j < T) ? state 40 (2 + j) : state 2 + j (state T can land in two)
        const int j0 = (i % 40 == 0 && i / 40 >= 2 && i / 40 < T) ? i / 40 - 2 : -1;
        const int j1 = (T >= 2 && i == T) ? T - 2 : ((T >= 1 && i == T + 1) ? T - 1 : -1);
        if (act) {
            if (j0 >= 0) {
                Pr[(size_t)j0 * R + 2 * k] = x; Pr[(size_t)j0 * R + 2 * k + 1] = y;
                Prd[(size_t)j0 * R + 2 * k] = xd; Prd[(size_t)j0 * R + 2 * k + 1] = yd;
            }
            if (j1 >= 0) {
                Pr[(size_t)j1 * R + 2 * k] = x; Pr[(size_t)j1 * R + 2 * k + 1] = y;
                Prd[(size_t)j1 * R + 2 * k] = xd; Prd[(size_t)j1 * R + 2 * k + 1] = yd;
            }
        }
        if (i == loop) break;
        const double scale = (i < 1000) ? ((double)i / 1000) : 1.0;
        const double *pc = pos + 2 * NA * cur;
        double xn = 0.0, yn = 0.0, xdn = 0.0, ydn = 0.0;
        if (act) {
            const double ex = x - gx, ey = y - gy;
            const double dg = sqrt(ex * ex + ey * ey);
            const double fax = -alpha * (ex / dg), fay = -alpha * (ey / dg);
            double frx = 0.0, fry = 0.0;
            for (int o = 0; o < n_obs; o++) {
                const double vx = x - ob[2 * o], vy = y - ob[2 * o + 1];
                const double d = sqrt(vx * vx + vy * vy);
                if (d < dmin) {
                    const double c = (eta * (1 / d - 1 / dmin)) * (1 / (d * d));
                    frx = frx + c * (vx / d); fry = fry + c * (vy / d);
                }
            }
            double fgx = 0.0, fgy = 0.0;
            for (int jn = 0; jn < NA; jn++) {
                if (jn == k) continue;
                const double vx = x - pc[2 * jn], vy = y - pc[2 * jn + 1];
                const double d = sqrt(vx * vx + vy * vy);
                const double d2 = d * d, d3 = d2 * d, d6 = d3 * d3, d7 = d6 * d, d13 = d6 * d7;
                const double c = (4 * epsilon) * (s6 / d7 - s12 / d13);
                fgx = fgx - c * (vx / d); fgy = fgy - c * (vy / d);
            }
            double fx = (fax + frx) + fgx, fy = (fay + fry) + fgy;
            if (dg < 0.001) { fx = 0 * fax; fy = 0 * fay; }
            xn = (x + a01 * xd) + (b00 * fx) * scale;
            yn = (y + a01 * yd) + (b00 * fy) * scale;
            xdn = (a22 * xd) + (b20 * fx) * scale;
            ydn = (a22 * yd) + (b20 * fy) * scale;
            pos[2 * NA * (cur ^ 1) + 2 * k] = xn; pos[2 * NA * (cur ^ 1) + 2 * k + 1] = yn;
        }
        x = xn; y = yn; xd = xdn; yd = ydn;
        cur ^= 1;
        __syncthreads();
    }
}

// Swarms beyond one workgroup (NA > 1024, or on request): one launch per step, one thread per
// agent over as many 64-thread workgroups as the swarm needs, every agent coupled to every
// other through the step's position snapshot in global memory (pos_cur, read as wave-wide
// broadcasts through L2) -- no grid-wide barrier, the launch boundary orders the steps.  The
// per-agent arithmetic is the kernel above, operation for operation, so both paths (and
// oracle/hl_plan.c) agree bit for bit.  st = [NA][4] (x, y, xd, yd), updated in place.
extern "C" __global__ void __launch_bounds__(64) srb_hlplan_step_kernel(int NA, int i, int loop,
                                                                        const double *__restrict__ Pobs, int n_obs,
                                                                        const double *__restrict__ pos_cur,
                                                                        double *__restrict__ pos_next, double *__restrict__ st,
                                                                        double *__restrict__ Pr, double *__restrict__ Prd)
{
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= NA) return;
    const double epsilon = 60, sigma = 1.0, alpha = 150.0, eta = 400.0, dmin = 1.0;
    const double gx = 10.0, gy = 0.0;
    const double a01 = 0.001025061239872, a22 = 0.929527039758809;
    const double b00 = 0.000000068070472960, b20 = 0.000128132654983983;
    const double s6 = 6 * (sigma * sigma * sigma * sigma * sigma * sigma);
    const double s12 = 12 * (sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma * sigma);
    const int T = loop / 40, R = 2 * NA;
    double x = st[4 * k], y = st[4 * k + 1], xd = st[4 * k + 2], yd = st[4 * k + 3];
    const int j0 = (i % 40 == 0 && i / 40 >= 2 && i / 40 < T) ? i / 40 - 2 : -1;
    const int j1 = (T >= 2 && i == T) ? T - 2 : ((T >= 1 && i == T + 1) ? T - 1 : -1);
    if (j0 >= 0) {
        Pr[(size_t)j0 * R + 2 * k] = x; Pr[(size_t)j0 * R + 2 * k + 1] = y;
        Prd[(size_t)j0 * R + 2 * k] = xd; Prd[(size_t)j0 * R + 2 * k + 1] = yd;
    }
    if (j1 >= 0) {
        Pr[(size_t)j1 * R + 2 * k] = x; Pr[(size_t)j1 * R + 2 * k + 1] = y;
        Prd[(size_t)j1 * R + 2 * k] = xd; Prd[(size_t)j1 * R + 2 * k + 1] = yd;
    }
    if (i == loop) return;
    const double scale = (i < 1000) ? ((double)i / 1000) : 1.0;
    const double ex = x - gx, ey = y - gy;
    const double dg = sqrt(ex * ex + ey * ey);
    const double fax = -alpha * (ex / dg), fay = -alpha * (ey / dg);
    double frx = 0.0, fry = 0.0;
    for (int o = 0; o < n_obs; o++) {
        const double vx = x - Pobs[2 * o], vy = y - Pobs[2 * o + 1];
        const double d = sqrt(vx * vx + vy * vy);
        if (d < dmin) {
            const double c = (eta * (1 / d - 1 / dmin)) * (1 / (d * d));
            frx = frx + c * (vx / d); fry = fry + c * (vy / d);
        }
    }
    double fgx = 0.0, fgy = 0.0;
    for (int jn = 0; jn < NA; jn++) {
        if (jn == k) continue;
        const double vx = x - pos_cur[2 * jn], vy = y - pos_cur[2 * jn + 1];
        const double d = sqrt(vx * vx + vy * vy);
        const double d2 = d * d, d3 = d2 * d, d6 = d3 * d3, d7 = d6 * d, d13 = d6 * d7;
        const double c = (4 * epsilon) * (s6 / d7 - s12 / d13);
        fgx = fgx - c * (vx / d); fgy = fgy - c * (vy / d);
    }
    double fx = (fax + frx) + fgx, fy = (fay + fry) + fgy;
    if (dg < 0.001) { fx = 0 * fax; fy = 0 * fay; }
    const double xn = (x + a01 * xd) + (b00 * fx) * scale;
    const double yn = (y + a01 * yd) + (b00 * fy) * scale;
    const double xdn = (a22 * xd) + (b20 * fx) * scale;
    const double ydn = (a22 * yd) + (b20 * fy) * scale;
    pos_next[2 * k] = xn; pos_next[2 * k + 1] = yn;
    st[4 * k] = xn; st[4 * k + 1] = yn; st[4 * k + 2] = xdn; st[4 * k + 3] = ydn;
}
