"""Diagnostic: NLP traces (nlpdbg build) of one agent under different waves-per-agent.
    python tools/trace_nw.py N C Ko Kn A seed agent"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402
import srbnmpc  # noqa: E402
from srbnmpc import workload  # noqa: E402

srbnmpc.LIB_PATH = os.path.join(os.path.dirname(srbnmpc.__file__), "libsrbnmpc_nlpdbg.so")
N, C, Ko, Kn, A, seed, ag = map(int, sys.argv[1:8])
b = workload.make_batch(A, N, C, seed=seed)
L = srbnmpc.lib()
L.srb_debug_nlp_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
buf = np.zeros(8 * 64)
for nw in (4, 2, 1):
    s = srbnmpc.BatchSolver(srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn), A)
    s.set_waves(nw)
    L.srb_debug_nlp_trace(ag, None)
    out = s.solve(b["x0"], b["ref"], b["foot"], b["obstacles"], b["nbr_state"])
    L.srb_debug_nlp_trace(-1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    print(f"nw={s.waves()} agent {ag}: status {out['status'][ag].tolist()} iters {out['iters'][ag].tolist()}")
    for i in range(min(int(out["iters"][ag, 1]) + 1, 12)):
        print(f"  {i:2d} " + " ".join(f"{v:10.3e}" for v in buf[8 * i:8 * i + 8]), flush=True)
    s.close()
