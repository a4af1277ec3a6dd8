import os, sys
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
import numpy as np, torch
import srbnmpc
from srbnmpc import workload
dev = torch.device("cuda:0")
def run(A, Kn, n_all, Ko=3, N=10, C=2):
    p = srbnmpc.default_params(N, C, K_obs=Ko, K_nbr=Kn, use_nlp=1)
    b = workload.make_batch(max(A, n_all), N, C, seed=1234)
    s = srbnmpc.BatchSolver(p, A)
    t = {k: torch.as_tensor(np.ascontiguousarray(v[:A] if k not in ("obstacles", "nbr_state") else v).reshape((v[:A] if k not in ("obstacles", "nbr_state") else v).shape[0], -1), dtype=torch.float64, device=dev) for k, v in b.items()}
    out = dict(x_qp=None, x=torch.zeros((A, p.nv), dtype=torch.float64, device=dev), obj=torch.zeros(A, dtype=torch.float64, device=dev),
               status=torch.zeros((A, 2), dtype=torch.int32, device=dev), iters=torch.zeros((A, 2), dtype=torch.int32, device=dev))
    st = torch.cuda.Stream(dev); torch.cuda.set_stream(st)
    ks = []
    for i in range(6):
        s.solve_device(t["x0"], t["ref"], t["foot"], t["obstacles"], t["nbr_state"][:n_all] if Kn else None, out, stream=st.cuda_stream)
        ks.append(s.last_kernel_ms())
    print(f"A={A} Ko={Ko} Kn={Kn} n_all={n_all}: knn_ms {np.median([k[0] for k in ks[2:]]):.4f} solve_ms {np.median([k[1] for k in ks[2:]]):.4f}", flush=True)
for Kn in (0, 1, 4, 8):
    run(1024, Kn, 1024)
for n_all in (2048, 4096):
    run(1024, 8, n_all)
run(256, 8, 1024); run(4096, 8, 4096)
run(1024, 0, 1024, Ko=0)
