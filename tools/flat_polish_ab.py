"""Diagnostic (round 6): where does the round-5 generic-pointer build (c2a5ce8, rebuilt
unchanged as libsrbnmpc_r05c.so) go wrong?  Run options only, no rebuild (a rebuild moves the defect):
the K = 3 + 0 batch of test_knn_matches_bruteforce with the polish fused (default), in its own kernel
(polish_fused 0) and off (polish 0), on the failing build and on the same source with the round-5 final
lip_eq_res (libsrbnmpc_r05cfix.so); the interior-point results of the two builds compared bit for bit.
    python tools/flat_polish_ab.py"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
OUT = os.path.join(ROOT, "gpurun_out")

if len(sys.argv) > 2 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
    import srbnmpc
    srbnmpc.use_library(sys.argv[2])
    from srbnmpc import workload
    N, C, A = 10, 2, 512
    b = workload.make_batch(A, N, C, seed=3)
    res = {}
    for mode, opts in (("fused", {}), ("kernel", {"polish_fused": 0}), ("off", {"polish": 0})):
        s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=3, K_nbr=0, use_nlp=1), A)
        for k, v in opts.items():
            s.set_option(k, v)
        o = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
        s.close()
        for k in ("x", "x_qp", "status", "iters", "obj"):
            res[f"{mode}_{k}"] = o[k]
    np.savez(os.path.join(OUT, f"r06_ab_{sys.argv[2]}.npz"), **res)
    sys.exit(0)

libs = ["libsrbnmpc_r05c.so", "libsrbnmpc_r05cfix.so"]
for lib in libs:                              # one process per library (a process loads one)
    subprocess.run([sys.executable, __file__, "--child", lib], check=True, timeout=300)
r = {lib: dict(np.load(os.path.join(OUT, f"r06_ab_{lib}.npz"))) for lib in libs}
a, f = r[libs[0]], r[libs[1]]
for mode in ("fused", "kernel", "off"):
    print(f"{mode:7s} NLP statuses r05c {np.bincount(a[mode + '_status'][:, 1], minlength=5).tolist()}  "
          f"r05cfix {np.bincount(f[mode + '_status'][:, 1], minlength=5).tolist()}")
    for k in ("x_qp", "x"):
        d = np.abs(a[f"{mode}_{k}"] - f[f"{mode}_{k}"])
        print(f"        {k:5s} bit-identical agents {int((d.max(1) == 0).sum())}/512, max |diff| {d.max():.3e}")
    print(f"        iterations identical {int((a[mode + '_iters'] == f[mode + '_iters']).all(1).sum())}/512")
