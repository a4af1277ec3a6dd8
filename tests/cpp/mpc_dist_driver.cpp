// Reference-style driver for the C++ MPC_dist shim (include/srbnmpc_mpc_dist.hpp): the
// HL block of src/A1_Sim.cpp:180-197 (updateState -> run_NMPC -> getters) on one agent.
//   mpc_dist_driver <input.txt> <use_snopt 0|1> [horizon N (4)] [trot|stand (stand)]
// input.txt: x0[4] (x, xdot, y, ydot) | ref[4N] (N grids x (x, xdot, y, ydot)) | n_obs | obs xy...
// stdout: status qp nlp, then get_MPCsol (4N), qp_solution (nv = (6 + C)N + 1), get_alphaCOM (20,
// row-major).  trot: contactInd {1, 0, 0, 1} (FR + RL stance, C = 2), stand: all four (C = 4).
//   mpc_dist_driver hl <loop>
// HL planner (src/A1_Sim.cpp:1152-1156): setPstart / setPobs / generateReferenceTrajectory for
// the reference's 4-agent start and 3 obstacles; stdout: Pr_refined_ then Prd_refined_.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>
#include "srbnmpc_mpc_dist.hpp"

static int hl_mode(int loop)
{
    srbnmpc::MPC_dist mpc;
    mpc.setAgentID(0);
    srbnmpc::Mat Pstart = srbnmpc::Mat::Zero(8, 1);
    const double ps[8] = {0.0, 0.0, 0.0, -0.9, -1, 0, -1, -0.9};   // src/A1_Sim.cpp:1013
    for (int i = 0; i < 8; i++) Pstart(i, 0) = ps[i];
    srbnmpc::Mat Pobs = srbnmpc::Mat::Zero(2, 3);
    const double po[6] = {3.0, 0.2, 5.0, -0.6, 7.0, 0.4};
    for (int j = 0; j < 3; j++) { Pobs(0, j) = po[2 * j]; Pobs(1, j) = po[2 * j + 1]; }
    try {
        mpc.setPstart(Pstart);
        mpc.setPobs(Pobs);
        mpc.generateReferenceTrajectory(loop);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    for (double v : mpc.Pr_refined()) std::printf("%.17g\n", v);
    for (double v : mpc.Prd_refined()) std::printf("%.17g\n", v);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 3 && std::string(argv[1]) == "hl") return hl_mode(std::atoi(argv[2]));
    if (argc < 3) { std::fprintf(stderr, "usage: %s input.txt use_snopt\n", argv[0]); return 2; }
    const int H = argc >= 4 ? std::atoi(argv[3]) : 4;
    const bool trot = argc >= 5 && std::string(argv[4]) == "trot";
    std::ifstream in(argv[1]);
    double x0[4];
    std::vector<double> ref((size_t)(4 * H));
    for (double &v : x0) in >> v;
    for (double &v : ref) in >> v;
    int n_obs = 0;
    in >> n_obs;
    srbnmpc::Mat Pobs = srbnmpc::Mat::Zero(2, n_obs);
    for (int j = 0; j < n_obs; j++) in >> Pobs(0, j) >> Pobs(1, j);
    if (!in) { std::fprintf(stderr, "bad input\n"); return 2; }
    // HL path of one agent: 2 x (H + 4) columns, the window the first run_NMPC reads (gaitDomain 0)
    const int rows = 2, cols = H + 4;
    std::vector<double> Pr(rows * cols, 0.0), Prd(rows * cols, 0.0);
    for (int k = 0; k < H; k++) {
        Pr[k * rows + 0] = ref[4 * k + 0]; Prd[k * rows + 0] = ref[4 * k + 1];
        Pr[k * rows + 1] = ref[4 * k + 2]; Prd[k * rows + 1] = ref[4 * k + 3];
    }
    try {
        srbnmpc::MPC_dist mpc(0, H);
        mpc.setAgentID(0);
        srbnmpc::Mat Pstart = srbnmpc::Mat::Zero(8, 1);
        mpc.setPstart(Pstart);
        mpc.setPobs(Pobs);
        mpc.setPobs_real(Pobs);
        mpc.setReferenceTrajectory(Pr.data(), Prd.data(), rows, cols);
        double q[18] = {0}, dq[18] = {0};
        q[0] = x0[0]; dq[0] = x0[1]; q[1] = x0[2]; dq[1] = x0[3];
        int ind[4] = {1, trot ? 0 : 1, trot ? 0 : 1, 1};
        srbnmpc::Mat toe = srbnmpc::Mat::Zero(3, 4), other = srbnmpc::Mat::Zero(4, 1);
        mpc.updateState(q, dq, ind, toe, other);
        mpc.use_snopt = std::atoi(argv[2]) != 0;
        mpc.run_NMPC();
        auto st = mpc.last_status();
        std::printf("%d %d\n", st.first, st.second);
        srbnmpc::Mat X = mpc.get_MPCsol();
        for (int i = 0; i < 4 * H; i++) std::printf("%.17g\n", X(i, 0));
        for (double v : mpc.qp_solution()) std::printf("%.17g\n", v);
        srbnmpc::Mat a = mpc.get_alphaCOM();
        for (int d = 0; d < 4; d++)
            for (int j = 0; j < 5; j++) std::printf("%.17g\n", a(d, j));
        srbnmpc::Vec4 last = mpc.get_lastState();
        std::fprintf(stderr, "last_state %g %g %g %g domain %d\n", last(0, 0), last(1, 0), last(2, 0), last(3, 0),
                     mpc.getDomain());
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    return 0;
}
