// Reference-style driver for the C++ LowLevelCtrl shim (include/srbnmpc_lowlevel.hpp): the
// low-level block of LocoWrapper.cpp:32-42, 222 (new LowLevelCtrl -> getllPointer ->
// calcTorque -> getTorque) on one robot, with stand-in structs that expose the reference's
// member names and Eigen-style accessors (global_loco_structs.hpp:12-111).
//   lowlevel_driver <input.txt> <calls>
// input.txt: ind[4] then the srb_ll_io arrays of one agent in IN order (q, dq, Dinv, B, H, Jc,
// dJc, Js, Jtoe, Jhip, toePos, hipPos, H0, dH0, y, dy, hd, dhd, fDes; fixed leading
// dimensions) and tau[18].  stdout per call: status iters, then tau (18), ll.QP_force (12),
// ll.ddq, ll.dq, ll.q (18 each), ll.V, ll.dV, ll.tau (18).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>
#include "srbnmpc_lowlevel.hpp"

struct M {   // column-major matrix with Eigen's (i, j) accessor
    int r = 0, c = 0;
    std::vector<double> v;
    M() = default;
    M(int rr, int cc) : r(rr), c(cc), v((size_t)rr * cc, 0.0) {}
    double &operator()(int i, int j) { return v[(size_t)j * r + i]; }
    double operator()(int i, int j) const { return v[(size_t)j * r + i]; }
};
struct StateInfo { M q{18, 1}, dq{18, 1}; };
struct DynamicsInfo { M Dinv{18, 18}, B{18, 12}, H{18, 1}; };
struct KinematicsInfo { M toePos{3, 4}, Jtoe{12, 18}, hipPos{3, 4}, Jhip{12, 18}, Jc, dJc, Js; };
struct VCInfo { M y, dy, H0, dH0, hd{18, 1}, dhd{18, 1}, fDes{12, 1}; };
struct ContactInfo { int ind[4] = {1, 1, 1, 1}; int cnt = 4; };
struct LL_params {   // Settings::LL_params, Parameters.cpp:62-75 defaults
    double mu = 0.7, kp = 700, kd = 40;
    int useCLF = 1;
    double tauPen = 1e0, dfPen = 1e-1, auxPen = 1e6, clfPen = 1e8, auxMax = 100, clfEps = 0.8;
};

int main(int argc, char **argv)
{
    if (argc < 3) { std::fprintf(stderr, "usage: %s input.txt calls\n", argv[0]); return 2; }
    std::ifstream in(argv[1]);
    ContactInfo con;
    con.cnt = 0;
    for (int &i : con.ind) { in >> i; con.cnt += (i == 1); }
    const int cd = 3 * con.cnt, od = 6 + 3 * (4 - con.cnt), sw = 12 - cd;
    StateInfo st; DynamicsInfo dyn; KinematicsInfo kin; VCInfo vc;
    kin.Jc = M(cd, 18); kin.dJc = M(cd, 1); kin.Js = M(sw, 18);
    vc.y = M(od, 1); vc.dy = M(od, 1); vc.H0 = M(od, 18); vc.dH0 = M(od, 1);
    double t;
    auto vec = [&](M &m, int n) { for (int i = 0; i < n; i++) { in >> t; if (i < m.r) m(i, 0) = t; } };
    auto cm = [&](M &m, int ld, int cols) {   // fixed-ld column-major block
        for (int j = 0; j < cols; j++)
            for (int i = 0; i < ld; i++) { in >> t; if (i < m.r && j < m.c) m(i, j) = t; }
    };
    vec(st.q, 18); vec(st.dq, 18);
    cm(dyn.Dinv, 18, 18); cm(dyn.B, 18, 12); vec(dyn.H, 18);
    cm(kin.Jc, 12, 18); vec(kin.dJc, 12); cm(kin.Js, 12, 18); cm(kin.Jtoe, 12, 18); cm(kin.Jhip, 12, 18);
    cm(kin.toePos, 3, 4); cm(kin.hipPos, 3, 4);
    cm(vc.H0, 18, 18); vec(vc.dH0, 18); vec(vc.y, 18); vec(vc.dy, 18); vec(vc.hd, 18); vec(vc.dhd, 18);
    vec(vc.fDes, 12);
    LL_params prm;
    try {
        srbnmpc::LowLevelCtrl LL;                          // LocoWrapper.cpp:32
        const srbnmpc::LLInfo *ll = LL.getllPointer();     // LocoWrapper.cpp:42
        double *tau = LL.getTorque();
        for (int i = 0; i < 18; i++) in >> tau[i];         // the member array's carried-over state
        for (int call = 0; call < std::atoi(argv[2]); call++) {
            LL.calcTorque(&st, &dyn, &kin, &vc, &con, &prm);   // LocoWrapper.cpp:222
            std::printf("%d %d\n", LL.last_status(), LL.last_iterations());
            for (int i = 0; i < 18; i++) std::printf("%.17g\n", LL.getTorque()[i]);
            for (double v : ll->QP_force) std::printf("%.17g\n", v);
            for (double v : ll->ddq) std::printf("%.17g\n", v);
            for (double v : ll->dq) std::printf("%.17g\n", v);
            for (double v : ll->q) std::printf("%.17g\n", v);
            std::printf("%.17g\n%.17g\n", ll->V, ll->dV);
            for (double v : ll->tau) std::printf("%.17g\n", v);
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 3;
    }
    return 0;
}
