"""Diagnostic (round 6): the round-4 N = 20 whole-shape failure.  Runs one build of the
ROUND-4 package (extracted from commit b64117e into a scratch directory; the base build ships 24_4_2_0_2_11,
the whole-shape build 24_4_2_20_2_11) on the config-5 batch, with the polish kernel on and off, and saves x,
x_qp, status and iterations for tools/r04_n20_compare.py.
    python tools/r04_n20_run.py <scratch-root> <tag>"""
import os
import sys

import numpy as np

root, tag = sys.argv[1], sys.argv[2]
sys.path[:0] = [os.path.join(root, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402   (the round-4 package of <scratch-root>)
from srbnmpc import workload  # noqa: E402

N, C, A, Ko, Kn = 20, 2, 2048, 3, 8
b = workload.make_batch(A, N, C, seed=0)
out = {}
for mode, pol in (("on", 1), ("off", 0)):
    s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1), A)
    s.set_option("polish", pol)
    r = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    s.close()
    for k in ("x", "x_qp", "status", "iters"):
        out[f"{mode}_{k}"] = np.asarray(r[k])
    print(f"{tag} polish {mode}: NLP statuses {np.bincount(r['status'][:, 1], minlength=5).tolist()}, "
          f"iterations mean {np.asarray(r['iters']).mean(0).round(3).tolist()}", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/r06_r04n20_{tag}.npz", **out)
