"""Diagnostic: per-phase cycle stamps of chosen agents of an SRB-12 batch (configs[2] swarm, 1024
agents), from the -DSRB12_STAMPS build:
    python tools/srb12_stamps.py agent [agent ...]     (loads libsrbnmpc_s12st.so, make s12st)"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402

import srbnmpc  # noqa: E402
srbnmpc.use_library("libsrbnmpc_s12st.so")
from srbnmpc import srb12, workload  # noqa: E402

PHASES = ["inputs/model/rollout", "costates+norms+exit", "Riccati factor", "gradient (+factor->pred)",
          "predictor rhs+solve", "predictor step+sigma", "corrector rhs+solve", "corrector step+update",
          "row loops (+exit->polish)", "active-set polish", "factor: products", "factor: to columns",
          "factor: elimination", "factor: Y Z products, stores", "solve: backward sweep", "solve: forward sweep"]
A, N = 1024, 10
b = workload.make_batch12(A, N, "trot", seed=0)
s = srb12.Solver12(srb12.default_params(N, K_obs=3, K_nbr=8), A)
L = srb12._lib()
L.srb12_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
buf = np.zeros(2 * 64 * 8 + 16)
s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])   # warm-up
for ag in map(int, sys.argv[1:]):
    L.srb12_debug_trace(s._h, ag, None)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    L.srb12_debug_trace(s._h, -1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    st = buf[2 * 64 * 8:2 * 64 * 8 + len(PHASES)]
    its = int(out["iters"][ag].sum())
    tot = st.sum()
    print(f"agent {ag}: iters {out['iters'][ag].tolist()}, total {tot:.0f} s_memtime cycles, "
          f"per iteration {tot / max(its, 1):.0f}")
    for name, v in zip(PHASES, st):
        print(f"   {name:24s} {v:10.0f}  {v / max(its, 1):9.0f} /iter  {100 * v / tot:5.1f} %")
s.close()
