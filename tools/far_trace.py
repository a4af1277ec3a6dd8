"""Diagnostic: NLP traces (GPU nlpdbg build and oracle) of the far-obstacle instance of
tests/test_gpu_parity.py::test_knn_sentinel_and_missing_rows.   python tools/far_trace.py agent"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

N, C, A, Ko, Kn = 10, 2, 32, 2, 4
b = workload.make_batch(A, N, C, seed=12)
ob = np.array([[2500.0, 0.0], [0.0, -1200.0], [1001.0, 1001.0]])
nb = b["nbr_state"].copy(); nb[3:, :2] = np.nan; nb[:3] = b["nbr_state"][:3]
ag = int(sys.argv[1]) if len(sys.argv) > 1 else 5
if len(sys.argv) > 2 and sys.argv[2] == "oracle":
    import oracle
    os.environ["ORC_NLP_TRACE"] = "1"
    r = oracle.solve_batch(oracle.params(N, C, K_obs=Ko, K_nbr=Kn), b["x0"][ag:ag + 1], b["ref"][ag:ag + 1],
                           b["foot"][ag:ag + 1], ob, nb, agent_offset=ag)
    print("oracle", r["status"], r["iters"])
    sys.exit(0)
srbnmpc.LIB_PATH = os.path.join(os.path.dirname(srbnmpc.__file__), "libsrbnmpc_nlpdbg.so")
s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn), A)
L = srbnmpc.lib()
L.srb_debug_nlp_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
buf = np.zeros(8 * 64)
L.srb_debug_nlp_trace(ag, None)
out = s.solve(b["x0"], b["ref"], b["foot"], ob, nb)
L.srb_debug_nlp_trace(-1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
print(f"GPU agent {ag}: status {out['status'][ag].tolist()} iters {out['iters'][ag].tolist()}")
for i in range(min(int(out["iters"][ag, 1]) + 1, 64)):
    print(f"  {i:2d} " + " ".join(f"{v:10.3e}" for v in buf[8 * i:8 * i + 8]), flush=True)
