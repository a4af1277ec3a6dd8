"""Diagnostic (round 6): compare the two round-4 N = 20 builds saved by tools/r04_n20_run.py -- which stage
differs (the interior point with the polish off; the polish kernel with it on), on how many agents, by how much;
and whether the whole-shape build's accepted polishes are the base build's points (feasible but wrong?).
    python tools/r04_n20_compare.py gpurun_out/r06_r04n20_base.npz gpurun_out/r06_r04n20_whole.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
N, C = 20, 2
xus = np.r_[0:6 * N, (6 + C) * N]
for mode in ("off", "on"):
    xa, xb = a[f"{mode}_x"], b[f"{mode}_x"]
    same = (xa == xb).all(1)
    print(f"polish {mode}: x_qp bit-identical {int((a[f'{mode}_x_qp'] == b[f'{mode}_x_qp']).all(1).sum())}/{len(xa)}, "
          f"x bit-identical {int(same.sum())}/{len(xa)}, iterations identical "
          f"{int((a[f'{mode}_iters'] == b[f'{mode}_iters']).all(1).sum())}/{len(xa)}, max |dx| (X, U, s) "
          f"{np.abs(xa[:, xus] - xb[:, xus]).max():.3e}")
    print(f"   NLP statuses base {np.bincount(a[f'{mode}_status'][:, 1], minlength=5).tolist()} whole "
          f"{np.bincount(b[f'{mode}_status'][:, 1], minlength=5).tolist()}")
# polish on: the whole build's OPTIMAL agents against the base build's (polished) points
sa, sb = a["on_status"][:, 1], b["on_status"][:, 1]
both = (sa == 0) & (sb == 0)
e = np.abs(a["on_x"][:, xus] - b["on_x"][:, xus]).max(1)
print(f"both OPTIMAL {int(both.sum())}: |x_base - x_whole| max {e[both].max() if both.any() else 0:.3e}, "
      f"> 1e-6 on {int((e[both] > 1e-6).sum())}, > 1e-4 on {int((e[both] > 1e-4).sum())}")
rej = (sa == 0) & (sb != 0)
print(f"base OPTIMAL, whole not: {int(rej.sum())}; whole's result = its interior-point result on "
      f"{int((b['on_x'][rej] == b['off_x'][rej]).all(1).sum())} of them")
