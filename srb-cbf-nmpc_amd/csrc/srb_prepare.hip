// Input assembly on the device: the per-agent planners that run_NMPC
// calls before its solve, for a whole batch, one thread per agent.
//   updateState / get_lastState   MPC_dist.cpp:1195-1202, 1272-1276 (x0 :226-229)
//   copPlanner_eventbase          MPC_dist.cpp:702-782 (reference window of the HL path)
//   footholdsPlanner              MPC_dist.cpp:1204-1266 (stance footholds, default stance
//                                 before locomotion starts)
// Outputs land in the agent-major arrays srb_solve_batch_device consumes, plus the
// neighbour-snapshot row (get_lastState) that the multi-GPU all-gather exchanges.
#include <hip/hip_runtime.h>
#include "srbnmpc.h"

// MPC_dist.cpp:1206-1209: FR, FL, RR, RL offsets from the start position
__constant__ double c_init_foot[4][2] = {{0.2188, -0.1320}, {0.2188, 0.1320}, {-0.1472, -0.1320}, {-0.1472, 0.1320}};

extern "C" __global__ void __launch_bounds__(256) srb_prepare_kernel(
    int n_agents, int N, int C, int n_rows, int T, int agent_offset, const double *__restrict__ Pr,
    const double *__restrict__ Prd, const int *__restrict__ agent_id, const int *__restrict__ gait_domain,
    const int *__restrict__ contact, const double *__restrict__ toe, const double *__restrict__ start,
    const double *__restrict__ q, const double *__restrict__ dq, double *__restrict__ x0, double *__restrict__ ref,
    double *__restrict__ foot, double *__restrict__ last_state, int *__restrict__ status)
{
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n_agents) return;
    int st = 0;
    // updateState + x0 (:226-229) + get_lastState (:1272-1276)
    const double qx = q[18 * (size_t)a], qy = q[18 * (size_t)a + 1], vx = dq[18 * (size_t)a], vy = dq[18 * (size_t)a + 1];
    x0[4 * (size_t)a + 0] = qx; x0[4 * (size_t)a + 1] = vx; x0[4 * (size_t)a + 2] = qy; x0[4 * (size_t)a + 3] = vy;
    last_state[4 * (size_t)a + 0] = qx; last_state[4 * (size_t)a + 1] = qy;
    last_state[4 * (size_t)a + 2] = vx; last_state[4 * (size_t)a + 3] = vy;
    // copPlanner_eventbase: rows 2 id, 2 id + 1 of Pr / Prd (column-major, Eigen layout) from
    // the current gait domain's first column (4 grids per domain, NDOMAIN), x xdot y ydot
    const int id = agent_id ? agent_id[a] : agent_offset + a;
    const int gd = gait_domain[a];
    const int c0 = 4 * gd;
    if (2 * id + 1 >= n_rows || c0 < 0 || c0 + N > T) st = 2;
    for (int k = 0; k < N; k++) {
        const int c = (st == 2) ? 0 : c0 + k;
        const size_t col = (size_t)c * n_rows;
        const int r0 = (st == 2) ? 0 : 2 * id;
        ref[(size_t)a * 4 * N + 4 * k + 0] = Pr[col + r0];
        ref[(size_t)a * 4 * N + 4 * k + 1] = Prd[col + r0];
        ref[(size_t)a * 4 * N + 4 * k + 2] = Pr[col + r0 + 1];
        ref[(size_t)a * 4 * N + 4 * k + 3] = Prd[col + r0 + 1];
    }
    // footholdsPlanner: default stance around the start position while gaitDomain <= 1
    double tx[4], ty[4];
    for (int l = 0; l < 4; l++) {
        tx[l] = (gd <= 1) ? c_init_foot[l][0] + start[2 * (size_t)a] : toe[12 * (size_t)a + l];
        ty[l] = (gd <= 1) ? c_init_foot[l][1] + start[2 * (size_t)a + 1] : toe[12 * (size_t)a + 4 + l];
    }
    const int *ci = contact + 4 * (size_t)a;
    const int nc = ci[0] + ci[1] + ci[2] + ci[3];
    int legs[4] = {0, 1, 2, 3};
    if (nc == 2 && ci[0] == 0) { legs[0] = 1; legs[1] = 2; }        // 0 1 1 0
    else if (nc == 2 && ci[0] == 1) { legs[0] = 0; legs[1] = 3; }   // 1 0 0 1
    if (nc != C || (nc != 2 && nc != 4)) st = st ? st : 1;
    for (int k = 0; k < N; k++)                                      // same block every grid (:1256-1260)
        for (int i = 0; i < C; i++) {
            foot[((size_t)a * N + k) * 2 * C + i] = tx[legs[i]];
            foot[((size_t)a * N + k) * 2 * C + C + i] = ty[legs[i]];
        }
    status[a] = st;
}
