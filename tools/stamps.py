"""Diagnostic: per-phase s_memtime cycles of agent 0 (libsrbnmpc_stamps.so).

    python tools/stamps.py [N C K_obs K_nbr agents]
"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'srb-cbf-nmpc_amd'))
import numpy as np
import srbnmpc
srbnmpc.LIB_PATH = os.path.join(os.path.dirname(srbnmpc.__file__), 'libsrbnmpc_stamps.so')
from srbnmpc import workload
N, C, Ko, Kn, A = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (10, 2, 3, 0, 64))]
p = srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn)
b = workload.make_batch(A, N, C, seed=1234)
s = srbnmpc.BatchSolver(p, A)
L = srbnmpc.lib(); L.srb_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 64)()
s.solve(b['x0'], b['ref'], b['foot'], b['obstacles'], b['nbr_state'])
L.srb_debug_stamps(buf, 1)
reps = 5
for _ in range(reps):
    out = s.solve(b['x0'], b['ref'], b['foot'], b['obstacles'], b['nbr_state'])
L.srb_debug_stamps(buf, 1)
v = np.array(buf[:], dtype=float) / reps
it = out['iters'][0]
names = ['resid+norms', 'om', 'build_D', "Z'HZ (mfma)", 'chol', 'pred rhs',
         'P: om*r3 + J\'w', "P: Z'v", 'P: tri-solves', 'P: Z xi', 'P: J dx',
         'step/rho/corr rhs',
         'C: om*r3 + J\'w', "C: Z'v", 'C: tri-solves', 'C: Z xi', 'C: J dx', 'dq+update']
print(f"agent0 iters qp={it[0]} nlp={it[1]}; kernel ms {s.last_kernel_ms()}")
print("setup", v[28], "qp-init", v[29], "nlp-init", v[30], "output", v[31], "init-solve", v[20:25].sum())
for stage, base, nit in (("QP", 0, it[0]), ("NLP", 32, it[1])):
    tot = v[base:base + 18].sum()
    print(stage, "total cycles", tot, "per iter", tot / max(nit, 1))
    for i, nm in enumerate(names):
        print(f"   {nm:20s} {v[base + i] / max(nit, 1):10.0f} cyc/iter  {100 * v[base + i] / max(tot, 1):5.1f}%")
