"""Diagnostics for the SRB-12 polish: solve the N = 20, 3 + 8 row case of
test_srb12_variants_vs_oracle with a given build, compare with the oracle (polish on and off), and
print the polish state checks that a -DSRB12_CHECK build records for one traced agent
(srb12_kernels.hip S12CK slots; srb12_debug_check).

    python tools/srb12_check.py --lib libsrbnmpc_chknowpe.so [--agent 0] [--N 20] [--agents 32]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="libsrbnmpc.so")
    ap.add_argument("--agent", type=int, default=0)
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--agents", type=int, default=32)
    ap.add_argument("--seed", type=int, default=31)
    ap.add_argument("--gait", default="trot")
    a = ap.parse_args()
    srbnmpc.use_library(a.lib)
    import oracle
    from srbnmpc import srb12, workload
    L = srb12._lib()
    L.srb12_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.srb12_debug_check.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
    N, A = a.N, a.agents
    b = workload.make_batch12(A, N, a.gait, seed=a.seed)
    args = (b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    print(f"lib {a.lib}  N {N}  agents {A}  gait {a.gait}  seed {a.seed}")
    for pol in (1, 0):
        s = srb12.Solver12(srb12.default_params(N, K_obs=3, K_nbr=8, polish=pol), A)
        L.srb12_debug_trace(s._h, a.agent, None)
        out = s.solve(*args)
        chk = np.zeros(128)
        L.srb12_debug_check(s._h, chk.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        s.close()
        r = oracle.solve_batch12(oracle.params12(N, K_obs=3, K_nbr=8, polish=pol), *args)
        ex = np.abs(out["x"][:, :12 * N] - r["x"][:, :12 * N]).max(1)
        eq = np.abs(out["x_qp"][:, :12 * N] - r["x_qp"][:, :12 * N]).max(1)
        print(f"polish {pol}: status equal {bool((out['status'] == r['status']).all())}, "
              f"iters equal {float((out['iters'] == r['iters']).all(1).mean()):.2f}; "
              f"x_qp max err {eq.max():.2e}; x max err {ex.max():.2e}, agents > 1e-6: {int((ex > 1e-6).sum())}")
        print("   agent errors:", " ".join(f"{e:.1e}" for e in ex[:16]))
        if pol and ex[a.agent] > 1e-6:
            np.set_printoptions(linewidth=180, precision=6, suppress=False)
            g, o = out["x"][a.agent], r["x"][a.agent]
            print("   agent x (gpu / oracle), entries off by > 1e-6:", int((np.abs(g - o) > 1e-6).sum()), "of", g.size,
                  " exact zeros in gpu:", np.where(g == 0.0)[0].tolist()[:64])
            for k in range(0, g.size, 12):
                print(f"   [{k:4d}] gpu ", g[k:k + 12])
                print(f"          orc ", o[k:k + 12])
        if pol:
            print("   agent0 X[0:3] gpu", out["x"][a.agent, :3], "oracle", r["x"][a.agent, :3])
            names = {0: "fin_flag", 1: "dyn_res(ipm)", 2: "sum|Z| start", 3: "X0 start", 4: "sum|xsv| saved"}
            for i in range(5):
                print(f"   [{i:3d}] {names[i]:18s} {chk[i]: .6e}")
            for pas in range(2):
                for pit in range(5):
                    base = 8 + 40 * pas + 8 * pit
                    v = chk[base:base + 8]
                    if not v.any():
                        continue
                    print(f"   pass {pas} step {pit}: schur {v[0]: .3e} sol_res {v[1]: .2e} dX0 {v[2]: .3e} dU2 {v[3]: .3e} "
                          f"sum|xsv| {v[4]: .6e} lastdx {v[5]: .2e} dyn_res {v[6]: .2e} X0 {v[7]: .6e}")
            for pas in range(4):
                v = chk[88 + 8 * pas:96 + 8 * pas]
                if v.any():
                    print(f"   pass {pas} bad {v[5]:.0f} accept-test: pv {v[0]: .2e} cv {v[1]: .2e} nzmin {v[2]: .2e} "
                          f"zm {v[3]: .2e} dyn {v[4]: .2e} lastdx {v[6]: .2e} X0 {v[7]: .6e}")
            print(f"   end: accepted {chk[120]:.0f} sum|Z| {chk[121]: .6e} X0 {chk[122]: .6e} dyn_res {chk[123]: .2e}")


if __name__ == "__main__":
    main()
