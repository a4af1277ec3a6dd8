"""Round 6: BASELINE configs[4]'s "fp32 KKT with fp64 iterative-refine residuals" as SRB_OPT_KKT_FP32_MU (the
reduced Newton matrix inverted in fp32 while the complementarity mu is above a threshold, each solve refined in fp64
against the fp64 matrix).  Per threshold and refinement count: NLP statuses, iterations and X, U, s against the fp64
kernel and the oracle on the config-5 batch (configs[4]'s shape) and the configs[2] batch, plus kernel time.
    python tools/kkt32_check.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import bench  # noqa: E402
import oracle  # noqa: E402
import srbnmpc  # noqa: E402

for cfg in (5, 3):
    c = bench.CONFIGS[cfg]
    N, C = c["N"], c["C"]
    A, b, _, _ = bench.rank_batch(cfg, c["agents"], 1, 0)
    args = (b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    xus = np.r_[0:6 * N, (6 + C) * N]
    r = oracle.solve_batch(oracle.params(N, C, K_obs=c["K_obs"], K_nbr=c["K_nbr"]), *args, nthreads=16)
    ref = None
    for mu, nref in ((0.0, 3), (1e-1, 2), (1e-1, 3), (1e-2, 3), (1e-3, 3), (1e-4, 4)):
        s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=c["K_obs"], K_nbr=c["K_nbr"], use_nlp=1), A)
        s.set_option("kkt_fp32_mu", mu)
        s.set_option("kkt_fp32_refine", nref)
        out = s.solve(*args)
        used = s.get_option("last_kkt_fp32")
        ks = []
        for _ in range(10):
            s.solve(*args)
            ks.append(s.last_kernel_ms()[1])
        s.close()
        if ref is None:
            ref = out
        st = out["status"]
        e_or = np.abs(out["x"][:, xus] - r["x"][:, xus]).max(1)
        e_64 = np.abs(out["x"][:, xus] - ref["x"][:, xus]).max(1)
        print(f"config {cfg} mu {mu:g} refine {nref} (fp32 instance {int(used)}): kernel {np.median(ks):.4f} ms; NLP statuses "
              f"{np.bincount(st[:, 1], minlength=5).tolist()} (oracle {np.bincount(r['status'][:, 1], minlength=5).tolist()}); "
              f"statuses == oracle {int((st == r['status']).all(1).sum())}/{A}; iters mean {st.shape and out['iters'].mean(0).round(2).tolist()} "
              f"max {out['iters'].max(0).tolist()}; |x - oracle| max {e_or.max():.2e}; |x - fp64| max {e_64.max():.2e}", flush=True)
