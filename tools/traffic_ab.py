"""Attribution of the configs[2] solve kernel's HBM fetch: the same 1024-agent
batch and tables, solved for its first A agents (A = 128, 256, 512, 1024) under
`rocprofv3 --pmc FETCH_SIZE` (and WRITE_SIZE in a pass of its own).  Per-dispatch traffic against A
separates what every launch fetches once per XCD (code, kernel arguments, the obstacle / neighbour tables
read through L2) from what each agent adds (its inputs, gathers, outputs).

    rocprofv3 --pmc FETCH_SIZE -d <dir> -o run --output-format csv -- python3 tools/traffic_ab.py
    python tools/traffic_ab.py --fit <fetch_dir> <write_dir> <calib.json> <out.json>
"""
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "srb-cbf-nmpc_amd")]
SIZES = (128, 256, 512, 1024)
REPS = 4


def run():
    import torch
    import bench
    import srbnmpc
    cfg = bench.CONFIGS[3]
    A, b, sh, _ = bench.rank_batch(3, 1024, 1, 0)
    N, C = cfg["N"], cfg["C"]
    p = srbnmpc.default_params(N, C, K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=1)
    s = srbnmpc.BatchSolver(p, A)
    s.set_waves(1)                     # the configs[2] instance (12_4_1_10_2_11) at every size
    dev = torch.device("cuda:0")
    T = lambda v: torch.as_tensor(np.ascontiguousarray(v), dtype=torch.float64, device=dev)
    x0, ref, foot, ob, nb = T(b["x0"]), T(b["ref"]), T(b["foot"]), T(b["obstacles"]), T(b["nbr_state"])
    for n in SIZES:
        out = dict(x_qp=None, x=torch.zeros((n, p.nv), dtype=torch.float64, device=dev),
                   obj=torch.zeros(n, dtype=torch.float64, device=dev),
                   status=torch.zeros((n, 2), dtype=torch.int32, device=dev),
                   iters=torch.zeros((n, 2), dtype=torch.int32, device=dev))
        for _ in range(REPS):
            s.solve_device(x0[:n], ref[:n], foot[:n], ob, nb, out, obstacles_version=1)
            torch.cuda.synchronize()
    s.close()


def per_dispatch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or "srb_nmpc_kernel" not in r["Kernel_Name"]:
            continue
        per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def fit(fdir, wdir, calib, out):
    cal = json.load(open(calib))
    f = np.array(per_dispatch(fdir, "FETCH_SIZE")) / cal["fetch_units_per_byte_read8"]
    w = np.array(per_dispatch(wdir, "WRITE_SIZE")) / cal["write_units_per_byte_write8"]
    n = np.repeat(SIZES, REPS)[:len(f)]
    res = {"agents": n.tolist(), "fetch_bytes": f.tolist(), "write_bytes": w.tolist()}
    for name, v in (("fetch", f), ("write", w)):
        med = np.array([np.median(v[n == a]) for a in SIZES])
        slope, icpt = np.polyfit(np.array(SIZES, float), med, 1)
        res[name] = {"median_per_size": med.tolist(), "bytes_per_agent": slope, "bytes_per_launch_fixed": icpt}
        print(f"{name}: per agent {slope:.0f} B, fixed per launch {icpt / 1e6:.3f} MB; medians (MB) "
              + " ".join(f"{a}:{m / 1e6:.3f}" for a, m in zip(SIZES, med)))
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--fit":
        fit(*sys.argv[2:6])
    else:
        run()
