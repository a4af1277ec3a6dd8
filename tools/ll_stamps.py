"""Diagnostic: per-phase s_memtime cycles of one agent of the low-level CLF-QP kernel
(srb_ll_debug_stamps), in a batch of A agents (default 8192, the bench workload).

    python tools/ll_stamps.py [A] [agent]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import srbnmpc  # noqa: E402
from srbnmpc import ll_workload, lowlevel  # noqa: E402

A = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
agent = int(sys.argv[2]) if len(sys.argv) > 2 else 0
NAMES = ["load+assembly", "factor: om/leg reads", "factor: friction LDL'", "factor: Y", "factor: S",
         "factor: Gauss-Jordan", "predictor solve", "predictor steps+rho", "corrector solve", "steps+update",
         "residuals+norms", "init / exit", "epilogue"]
pool = ll_workload.make_batch(min(512, A), seed=4321)
reps = -(-A // pool["ind"].shape[0])
b = {k: np.concatenate([v] * reps)[:A] for k, v in pool.items()}
L = srbnmpc.lib()
L.srb_ll_debug_trace.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
L.srb_ll_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
c = srbnmpc.LowLevelCtrl(lowlevel.default_params(), A)
c.calc_torque(b)                       # warm-up
L.srb_ll_debug_trace(agent | (31 << 16), None)
L.srb_ll_debug_stamps(None, 1)
out = c.calc_torque(b)
st = np.zeros(16, np.uint64)
L.srb_ll_debug_stamps(st.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 0)
L.srb_ll_debug_trace(-1, None)
it = int(out["iters"][agent])
tot = int(st[:13].sum())
print(f"agent {agent} of {A}: contacts {int(b['ind'][agent].sum())}, {it} iterations, {tot} cycles total "
      f"({tot / max(it, 1):.0f} per iteration incl. setup)")
for i, n in enumerate(NAMES):
    v = int(st[i])
    print(f"  {n:24s} {v:9d}  {v / max(it, 1):8.0f}/it  {100.0 * v / max(tot, 1):5.1f}%")
