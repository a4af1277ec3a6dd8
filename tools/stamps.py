"""Diagnostic: per-phase s_memtime cycles of agent 0 (libsrbnmpc_stamps.so, make stamps).

    python tools/stamps.py [N C K_obs K_nbr agents]
"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'srb-cbf-nmpc_amd'))
import numpy as np
import srbnmpc
srbnmpc.use_library('libsrbnmpc_stamps.so')
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
names = {0: 'setup', 1: 'qp-init', 2: 'nlp-init', 18: 'resid loop', 3: 'resid reduce', 16: 'weights', 17: 'P: rhs',
         4: 'gram', 5: 'factor (GJ)', 6: 'P: rhs', 7: 'P: rmul', 8: 'P: solve', 21: 'P: Jdx', 9: 'P: steplen',
         10: 'rho + C: rhs', 11: 'C: rmul', 12: 'C: solve', 22: 'C: Jdx', 13: 'C: steplen', 19: 'update: s z',
         20: 'update: x rx', 14: 'update: hess', 15: 'output', 23: 'setup: inputs', 24: 'setup: obstacles',
         25: 'setup: basis', 26: 'fused polish'}
periter = set(range(3, 15)) | set(range(16, 23))
print(f"agent0 iters qp={it[0]} nlp={it[1]}; kernel ms {s.last_kernel_ms()[1]:.4f}")
tot_all = v.sum()
for stage, nit in ((0, it[0]), (1, it[1])):
    blk = v[32 * stage:32 * stage + 32]
    per = sum(blk[i] for i in periter) / max(nit, 1)
    print(f"{'QP' if stage == 0 else 'NLP'}: total {blk.sum():.0f} cyc, per iteration {per:.0f}")
    for i, nm in names.items():
        if stage == 1 and i == 6:
            nm = 'kNN selection'
        if blk[i] > 0:
            print(f"   {nm:18s} {blk[i]:10.0f} cyc  {blk[i] / max(nit, 1) if i in periter else 0:8.0f} /iter  {100 * blk[i] / tot_all:5.1f}%")
