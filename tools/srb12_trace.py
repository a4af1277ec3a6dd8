"""Diagnostic: per-iteration trace of chosen agents of an SRB-12 batch, GPU kernel
(srb12_debug_trace) next to the oracle (ORC12_TRACE=1 on stderr).
    python tools/srb12_trace.py [--lib libsrbnmpc_<tag>.so] gait seed A agent [agent ...]
    (agent "auto": the first five agents the GPU does not report OPTIMAL)"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from srbnmpc import srb12, workload  # noqa: E402

import srbnmpc  # noqa: E402
argv = sys.argv[1:]
if argv[0] == "--lib":
    srbnmpc.use_library(argv[1])
    argv = argv[2:]
gait, seed, A = argv[0], int(argv[1]), int(argv[2])
N = 10
b = workload.make_batch12(A, N, gait, seed=seed)
s = srb12.Solver12(srb12.default_params(N, K_obs=3, K_nbr=8), A)
L = srb12._lib()
L.srb12_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
buf = np.zeros(2 * 64 * 8 + 16)
p = oracle.params12(N, K_obs=3, K_nbr=8)
agents = argv[3:]
if agents == ["auto"]:
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    bad = np.where((out["status"] != 0).any(1))[0]
    print("not OPTIMAL:", [(int(a), out["status"][a].tolist(), out["iters"][a].tolist()) for a in bad], flush=True)
    agents = bad[:5]
for ag in map(int, agents):
    L.srb12_debug_trace(s._h, ag, None)
    out = s.solve(b["x0"], b["xref"], b["foot"], b["contact"], b["obstacles"], b["nbr_state"])
    L.srb12_debug_trace(s._h, -1, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    print(f"agent {ag}: GPU status {out['status'][ag].tolist()} iters {out['iters'][ag].tolist()}")
    for st in range(2):
        print("  stage", st, "  it   |rd|       th         |rp|       mu         ap         ad         delta      sigma")
        for i in range(min(int(out["iters"][ag, st]) + 1, 64)):
            r = buf[8 * (64 * st + i):8 * (64 * st + i) + 8]
            print(f"          {i:2d} " + " ".join(f"{v:10.3e}" for v in r), flush=True)
    os.environ["ORC12_TRACE"] = "1"
    r = oracle.solve_batch12(p, b["x0"][ag:ag + 1], b["xref"][ag:ag + 1], b["foot"][ag:ag + 1], b["contact"][ag:ag + 1],
                             b["obstacles"], b["nbr_state"], agent_offset=ag, nthreads=1)
    del os.environ["ORC12_TRACE"]
    print(f"  oracle status {r['status'][0].tolist()} iters {r['iters'][0].tolist()}  max|x - x_oracle| "
          f"{np.abs(out['x'][ag] - r['x'][0]).max():.3e}", flush=True)
s.close()
