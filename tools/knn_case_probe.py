"""Diagnostic: status histogram and oracle distance of the (Ko, Kn) selection test's batch shape
(tests/test_gpu_parity.py::test_knn_matches_bruteforce) at every wave count.
    python tools/knn_case_probe.py Ko Kn [A]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))
import oracle  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

if os.environ.get("PROBE_LIB"):           # e.g. libsrbnmpc_nlpdbg.so
    srbnmpc.LIB_PATH = os.path.join(os.path.dirname(srbnmpc.__file__), os.environ["PROBE_LIB"])

Ko, Kn = int(sys.argv[1]), int(sys.argv[2])
A = int(sys.argv[3]) if len(sys.argv) > 3 else 512
N, C = 10, 2
b = workload.make_batch(A, N, C, seed=3)
op = oracle.params(N, C, K_obs=Ko, K_nbr=Kn)
r = oracle.solve_batch(op, b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"], nthreads=16)
xus = lambda x: np.concatenate([x[:, :6 * N], x[:, -1:]], 1)
for nw in map(int, os.environ.get("PROBE_WAVES", "0 1 2 4").split()):
    s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn), A)
    s.set_waves(nw)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    st = out["status"]
    e = np.abs(xus(out["x"]) - xus(r["x"])).max(1)
    print(f"waves {nw} (picked {s.waves()}): qp status {np.bincount(st[:, 0], minlength=5).tolist()} nlp status "
          f"{np.bincount(st[:, 1], minlength=5).tolist()} iters max {st.shape and out['iters'].max(0).tolist()} "
          f"max |x - oracle| {np.nanmax(e):.3e}, non-finite agents {np.where(~np.isfinite(e))[0][:12].tolist()}", flush=True)
    s.close()
