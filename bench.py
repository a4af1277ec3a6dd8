#!/usr/bin/env python3
"""Benchmark: batched CBF-NMPC solves on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--config 2] [--agents A]

--gpus N > 1 without a launcher starts N ranks itself (torch.distributed.run on 127.0.0.1, one
process per GPU); under a launcher WORLD_SIZE must equal N or the run exits non-zero.

One "step" = one pass of the hot path over one batch: (configs with inter-agent rows:
all-gather of the neighbour snapshot over RCCL) + kNN + QP stage + NLP stage + Bezier fit
(alpha_COM) for every agent of the batch, inputs resident in HBM.  Multi-GPU: one process per GPU (torchrun),
agents sharded agent-major, weak scaling (fixed agents per GPU).  Rank 0 prints one JSON
line.  Configs (BASELINE.json "configs"):
    1  1 agent, N=4 reference mode (KAT-2 shape)            -- CPU plumbing case
    2  64 agents/GPU, N=10, trot, 3 static obstacles        -- configs[1]
    3  1024 agents/GPU, N=10, 3 static + 8 nearest agents   -- configs[2], the default (the
                                                               largest single-GPU config)
    4  1024 agents/GPU, as 3 with the RCCL all-gather       -- configs[3] (8 GPUs = 8192)
    5  2048 agents/GPU, N=20, 3 static + 8 nearest agents   -- configs[4] shape, fp64

    python bench.py --path ll [--agents A]

The low-level CLF-QP (LowLevelCtrl::calcTorque): one step = QP
assembly + iSWIFT solve + swing PD + integration for every agent (default 8192 per GPU,
trot / stand mix), inputs resident in HBM; its own metric and roofline, not the headline.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "srb-cbf-nmpc_amd"))

import srbnmpc  # noqa: E402
from srbnmpc import dist as sdist, workload  # noqa: E402

METRIC = "NMPC solves/sec (whole node) + p99 solve latency, N-agent batch horizon=10"
FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 (vector and matrix) dense peak, spec
SCLK_GHZ = 2.4               # MI355X peak engine clock (MI355X_MICROARCH.md)
CONFIGS = {
    1: dict(agents=1, N=4, C=4, K_obs=1, K_nbr=0, name="1 agent, N=4, stand (reference mode, KAT-2 shape)"),
    2: dict(agents=64, N=10, C=2, K_obs=3, K_nbr=0, name="64 agents/GPU, horizon 10, trot, 3 static CBF obstacles, fp64"),
    3: dict(agents=1024, N=10, C=2, K_obs=3, K_nbr=8, name="1024 agents/GPU, horizon 10, 3 static + 8-nearest inter-agent CBF, fp64"),
    4: dict(agents=1024, N=10, C=2, K_obs=3, K_nbr=8, name="1024 agents/GPU + RCCL all-gather of neighbour CoM states, horizon 10, fp64"),
    5: dict(agents=2048, N=20, C=2, K_obs=3, K_nbr=8, name="2048 agents/GPU, horizon 20, 3 static + 8-nearest, fp64"),
}


def dense_equiv_flops(p, iters):
    """SURVEY.md §8d per-iteration figure: (2/3) d^3 + 4 d^2 with d = nv + neq (the unreduced
    dense KKT of the north-star formulation), times the actual per-agent iteration counts.
    A work-equivalence figure for comparison with a dense-KKT solver, NOT executed flops."""
    d = p.nv + 7 * p.N
    return float(iters.sum()) * ((2.0 / 3.0) * d ** 3 + 4.0 * d ** 2)


def executed_flops(p, iters, K):
    """fp64 flops the kernel's algorithm performs (useful work), per IPM
    iteration of one agent, with nz = N(C-1)+1 reduced unknowns, `terms` term rows and S row
    slots:  Gram 2 nz^2 terms + two right-hand sides 4 nz terms + Gauss-Jordan 2 nz^3 + two
    refined solves 12 nz^2 + slot work S (4 nz + 60) (+ obstacle re-linearisation 3 nz N K),
    summed over the actual QP and NLP iteration counts."""
    N, C = p.N, p.C
    nz, n, NE, NK = N * (C - 1) + 1, p.nv, 2 * (N - 1), N * K

    def per_iter(terms, S, nk):
        return 2 * nz * nz * terms + 4 * nz * terms + 2 * nz ** 3 + 12 * nz * nz + S * (4 * nz + 60) + 3 * nz * nk
    qp = per_iter(n + NE, n + NE, 0)
    nlp = per_iter(n + NE + NK, n + NE + 2 * N + NK, NK)
    return float(iters[:, 0].sum()) * qp + float(iters[:, 1].sum()) * nlp


def io_bytes(p, n_agents, n_obs, n_all):
    """Algorithmic HBM bytes per launch: inputs + outputs once."""
    per = 8 * (4 + 4 * p.N + 2 * p.C * p.N + 4) + 8 * (p.nv + 1 + 20) + 16
    return n_agents * per + 16 * n_obs + 32 * n_all


def host_threads():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS, 16 on the GPU
    boxes; os.cpu_count() there reports the whole machine), else every core here."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, os.cpu_count() or 1)


def cpu_baseline(cfg, b, budget_s):
    """CPU baselines on this host's cores, on bounded samples of the same workload, in this run:
      * the port (oracle/: the same QP + NLP algorithm in C, dense LU on the full-space KKT),
        "kind" "port" -- the headline cpu_baseline value (the reference's NLP solver, SNOPT, is
        proprietary and absent: there is no reference QP + NLP rate to time);
      * reference_qp: the reference's OWN QP solver -- the vendored iSWIFT compiled unchanged from
        /root/reference (oracle/_ref/libiswift_ref.so, iswift_qp.cpp:44-162 / Prime.c:127-230 with
        its dense -> CCS conversion and a fill-reducing ordering of the full KKT every call, as the
        Eigen wrapper does) on the QP stage of the same instances, same threads ("kind" "reference");
      * port_qp: the port's QP stage alone on those instances (the like-for-like ratio to
        reference_qp; replaces round 2's build-container calibration)."""
    sys.path.insert(0, ROOT)
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    nthreads = host_threads()
    p = oracle.params(cfg["N"], cfg["C"], K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"])
    A = b["x0"].shape[0]
    sample = min(A, max(nthreads * 2, 16))

    def timed(fn, budget):
        t0 = time.perf_counter(); done = 0
        while True:
            done += fn()
            if time.perf_counter() - t0 > budget:
                return done, time.perf_counter() - t0

    def port_batch():
        oracle.solve_batch(p, b["x0"][:sample], b["ref"][:sample], b["foot"][:sample], b["obstacles"],
                           b["nbr_state"], nthreads=nthreads)
        return sample
    solved, dt = timed(port_batch, budget_s)
    line = {"value": solved / dt, "unit": "solves/s", "cores": nthreads, "kind": "port",
            "sample": f"{solved} solves ({sample}-agent slices of the same batch) in {dt:.1f} s, QP+NLP, "
                      f"{nthreads} threads"}
    # the QP stage (a few ms per solve, so larger slices keep the per-call thread start-up out of the
    # rate): the port (use_nlp = 0) and the genuine iSWIFT on the same instances
    qs = min(A, 32 * nthreads)
    pq = oracle.params(cfg["N"], cfg["C"], K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=0)

    def port_qp():
        oracle.solve_batch(pq, b["x0"][:qs], b["ref"][:qs], b["foot"][:qs], b["obstacles"], b["nbr_state"],
                           nthreads=nthreads)
        return qs
    qsolved, qdt = timed(port_qp, budget_s / 3)
    line["port_qp"] = {"value": qsolved / qdt, "unit": "QP-stage solves/s", "cores": nthreads, "kind": "port",
                       "sample": f"{qsolved} QP stages ({qs}-agent slices of the same batch) in {qdt:.1f} s"}
    try:
        R = oracle.ref_lib()
    except OSError as e:                       # oracle/_ref not built (no /root/reference where it was built)
        line["reference_qp"] = {"value": None, "error": f"oracle/_ref/libiswift_ref.so unavailable: {e}"}
        return line
    import ctypes
    import scipy.sparse as sps
    ip, dp = ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)
    probs = []
    for a in range(qs):          # dense QPs (MPC_dist.cpp:135-321) -> CCS, built once, untimed
        Pd, c, Aq, bq, G, h = oracle.build_qp(p, b["x0"][a], b["ref"][a], b["foot"][a])
        n, m, pp = Pd.size, G.shape[0], Aq.shape[0]
        keep = []
        for M in (np.diag(Pd), Aq, G):
            S = sps.csc_matrix(M); S.eliminate_zeros(); S.sort_indices()
            keep += [np.ascontiguousarray(S.indptr, np.int32), np.ascontiguousarray(S.indices, np.int32),
                     np.ascontiguousarray(S.data, np.float64)]
        # elimination order z | x | y: quasi-definite, so no pivot needs iSWIFT's regularisation (the
        # reference's Eigen AMD order is a one-off symbolic cost next to QP_SETUP's factorisation)
        perm = np.r_[np.arange(n + pp, n + pp + m), np.arange(n), np.arange(n, n + pp)].astype(np.int32)
        vecs = [np.ascontiguousarray(v, np.float64).copy() for v in (c, h, bq)]
        args = [v.ctypes.data_as(ip if v.dtype == np.int32 else dp) for v in keep] + \
               [v.ctypes.data_as(dp) for v in vecs] + [perm.ctypes.data_as(ip)]
        probs.append((n, m, pp, args, np.zeros(n), keep, vecs, perm))
    flags = []

    def solve_range(lo, hi):
        it = ctypes.c_int()
        for k in range(lo, hi):
            n, m, pp, args, x = probs[k][:5]
            flags.append(R.iswift_ref_solve_ccs(n, m, pp, *args, x.ctypes.data_as(dp), ctypes.byref(it)))
        return hi - lo
    cuts = [qs * t // nthreads for t in range(nthreads + 1)]
    with ThreadPoolExecutor(nthreads) as ex:  # ctypes releases the GIL: one host thread per slice
        def ref_batch():
            return sum(ex.map(lambda t: solve_range(cuts[t], cuts[t + 1]), range(nthreads)))
        rsolved, rdt = timed(ref_batch, budget_s / 3)
    line["reference_qp"] = {
        "value": rsolved / rdt, "unit": "QP-stage solves/s", "cores": nthreads, "kind": "reference",
        "sample": f"{rsolved} QP stages ({qs}-agent slices, as port_qp) in {rdt:.1f} s: the genuine vendored iSWIFT "
                  f"(oracle/_ref; QP_SETUP + QP_SOLVE + QP_CLEANUP per call as iswift_qp.cpp:78-162 does, "
                  f"CCS inputs and a quasi-definite elimination order prepared once), "
                  f"{sum(f == 0 for f in flags)}/{len(flags)} OPTIMAL"}
    line["port_qp_over_reference_qp"] = line["port_qp"]["value"] / line["reference_qp"]["value"]
    return line


LL_METRIC = "low-level CLF-QP controller solves/sec (LowLevelCtrl::calcTorque, batched)"
LL_IN_DOUBLES = 18 + 18 + 324 + 216 + 18 + 216 + 12 + 216 + 216 + 216 + 12 + 12 + 324 + 18 * 5 + 12
LL_OUT_DOUBLES = 18 + 12 + 18 * 3 + 2 + 32


def ll_executed_flops(cnt, iters):
    """fp64 flops of srb_ll_kernel per agent: assembly [Jc;H0] Dinv (2*18^3)
    and (.)[Jc' B] (2*18*18*nft); per IPM iteration Y = H^-1 A' (~6*18*nft), S = A Y upper
    triangle (171 * 2 nft), Gauss-Jordan 2*18^3, two Newton solves (A u, S^-1, Y dy:
    2*(2*18*nft + 2*18^2 + 2*n*18 + 12 n)), residuals (A'y, A x: 4*18*nft + 12 n)."""
    nft = 3 * cnt + 12
    n = nft + 6 + 3 * (4 - cnt) + 1
    asm = 2 * 18 ** 3 + 2 * 18 * 18 * nft
    it = 6 * 18 * nft + 171 * 2 * nft + 2 * 18 ** 3 + 2 * (2 * 18 * nft + 2 * 18 * 18 + 2 * n * 18 + 12 * n) + \
        4 * 18 * nft + 12 * n
    return float(np.sum(asm + it * iters))


def main_ll(args, world, rank, local_rank, dev):
    from srbnmpc import ll_workload, lowlevel
    A_local = args.agents or 8192
    A_total = A_local * world
    lo, hi = sdist.shard_range(A_total, world, rank)
    n_loc = hi - lo
    # a pool of 512 distinct synthetic agents tiled over the batch (generation is host Python)
    pool = ll_workload.make_batch(min(512, A_total), seed=4321)
    reps = -(-A_total // pool["ind"].shape[0])
    full = {k: np.concatenate([v] * reps)[:A_total] for k, v in pool.items()}
    d = {"ind": torch.as_tensor(np.ascontiguousarray(full["ind"][lo:hi], np.int32), device=dev)}
    for k in lowlevel.IN_KEYS:
        d[k] = torch.as_tensor(np.ascontiguousarray(full[k][lo:hi]).reshape(n_loc, -1), dtype=torch.float64, device=dev)
    tau0 = torch.as_tensor(np.ascontiguousarray(full["tau"][lo:hi]), dtype=torch.float64, device=dev)
    out = {k: torch.zeros((n_loc, s), dtype=torch.float64, device=dev) for k, s in lowlevel.OUT_SIZE.items()}
    out["status"] = torch.zeros(n_loc, dtype=torch.int32, device=dev)
    out["iters"] = torch.zeros(n_loc, dtype=torch.int32, device=dev)
    ctrl = srbnmpc.LowLevelCtrl(lowlevel.default_params(), n_loc, local_rank)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def step():
        out["tau"].copy_(tau0)        # tau is in/out (LowLevelCtrl::tau), restore the input state
        ctrl.calc_torque_device(d, out, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    kern = []
    for _ in range(3):
        step()
        kern.append(ctrl.last_kernel_ms())
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_step = np.array([a.elapsed_time(bb) for a, bb in ev])
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    status = out["status"].cpu().numpy(); iters = out["iters"].cpu().numpy()
    cnt = full["ind"][lo:hi].sum(1)
    kms = float(np.median(kern))
    flops = ll_executed_flops(cnt, iters)
    achieved = flops / (kms * 1e-3) / 1e12
    io = n_loc * (8 * (LL_IN_DOUBLES + 18 + LL_OUT_DOUBLES) + 16 + 8)
    line = {
        "metric": LL_METRIC, "value": A_total * args.steps / elapsed, "unit": "solves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{A_local} agents/GPU, A1-sized LL QP (numDec <= 31), trot/stand mix, useCLF=1",
                   "agents_per_gpu": A_local, "agents_total": A_total, "parallelism": f"agents sharded x{world}"},
        "p50_ms": float(np.percentile(per_step, 50)), "p99_ms": float(np.percentile(per_step, 99)),
        "optimal_frac": float((status == 0).mean()), "iters_mean": float(iters.mean()),
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic_from("ll", n_loc)[0],
                     "traffic_source": traffic_from("ll", n_loc)[1], "kernel": "srb_ll_kernel",
                     "kernel_ms": kms, "flop_model": "bench.ll_executed_flops (DESIGN.md 6b); latency-bound",
                     "io_bytes_per_launch": io, "hbm_GBps": io / (kms * 1e-3) / 1e9},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        import oracle
        p = oracle.ll_params()
        nthreads = host_threads()
        sample = {k: v[:512] for k, v in full.items()}
        t1 = time.perf_counter(); n = 0
        while time.perf_counter() - t1 < args.cpu_seconds:
            oracle.ll_calc_torque(p, sample, nthreads=nthreads)
            n += 512
        dt = time.perf_counter() - t1
        line["cpu_baseline"] = {"value": n / dt, "unit": "solves/s", "cores": nthreads, "kind": "port",
                                "sample": f"{n} calcTorque calls (512-agent slices of the same batch) in {dt:.1f} s, "
                                          f"oracle/ll_ctrl.c, {nthreads} threads"}
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctrl.close()


def srb12_executed_flops(N, K, iters):
    """Executed fp64 flops of the SRB-12 Riccati interior-point method per solve, summed over the
    batch: per iteration the backward factorisation (G, F, Hux, A'G by their
    structure ~ 3 x 13^2 x 8, B'F 12^2 x 8, the 12 x 12 Gauss-Jordan 2 x 12^3, the two 16x16x16
    MFMA products 2 x 2 x 16^3) per grid, four Riccati vector solves (predictor, corrector, their
    refinements: ~ 2 x (12 x 12 + 13 x 12) x 2 + 300 per grid each) and the row work (~40 per row)."""
    fac = 3 * 169 * 8 + 144 * 8 + 2 * 12 ** 3 + 2 * 2 * 16 ** 3
    sol = 2 * (144 + 156) * 2 + 300
    rows = 40 * (24 * N + N * K)
    it = N * (fac + 4 * sol) + rows
    return float(np.sum(iters.sum(1) * it))


def traffic_from(name, agents):
    """roofline.traffic of a non-default path: hbm bytes per launch of its PMC summary
    (tools/pmc_traffic.py, profiles/r06_pmc_traffic_<name>.json, else round 5's; the LL kernel, unchanged
    since, also r04's and r03's) when it matches the batch."""
    for rnd in ("r06", "r05", "r04", "r03") if name == "ll" else ("r06", "r05"):
        f = os.path.join(ROOT, "profiles", f"{rnd}_pmc_traffic_{name}.json")
        try:
            tj = json.load(open(f))
            if tj.get("agents") in (agents, 0):
                return tj.get("hbm_bytes_per_launch"), os.path.relpath(f, ROOT)
        except Exception:
            pass
    return None, None


def main_srb12(args, world, rank, local_rank, dev):
    """SRB-12 extension mode: the north star's 12-state SRB NMPC on the
    configs[2]-shaped swarm (1024 agents per GPU, N = 10, trot, 3 static + 8 neighbour rows);
    its own line, not the headline."""
    from srbnmpc import srb12
    A_local = args.agents or 1024
    A_total = A_local * world
    N, Ko_, Kn_ = 10, 3, 8
    b = workload.make_batch12(A_total, N, "trot", seed=1234)
    lo, hi = sdist.shard_range(A_total, world, rank)
    n_loc = hi - lo
    T = lambda v, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(v), dtype=dt, device=dev)
    x0, xref, foot = T(b["x0"][lo:hi]), T(b["xref"][lo:hi]), T(b["foot"][lo:hi])
    contact, obst = T(b["contact"][lo:hi], torch.int32), T(b["obstacles"])
    nbr_all = T(b["nbr_state"])
    nbr_local = nbr_all[lo:hi].contiguous()
    prm = srb12.default_params(N, K_obs=Ko_, K_nbr=Kn_)
    if args.qp_warm_tol is not None:                     # diagnostics: the QP stage's tolerance before the NLP
        prm.tol_qp = args.qp_warm_tol
    solver = srb12.Solver12(prm, n_loc, local_rank)
    Ko, Kn = srb12.n_selected(prm, obst.shape[0], A_total)
    out = dict(x_qp=None, x=torch.zeros((n_loc, prm.nv), dtype=torch.float64, device=dev),
               obj=torch.zeros(n_loc, dtype=torch.float64, device=dev),
               status=torch.zeros((n_loc, 2), dtype=torch.int32, device=dev),
               iters=torch.zeros((n_loc, 2), dtype=torch.int32, device=dev),
               sel=torch.zeros((n_loc, Ko + Kn), dtype=torch.int32, device=dev))
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    exchange = sdist.NeighbourExchange(A_total, world, rank, dev) if world > 1 else None

    def step():
        nb = exchange(nbr_local) if exchange is not None else nbr_all
        solver.solve_device(x0, xref, foot, contact, obst, nb, out, agent_offset=lo, stream=stream.cuda_stream,
                            obstacles_version=1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    kern = []
    for _ in range(3):
        step()
        kern.append(solver.last_kernel_ms())
    # the timed loop runs without the library's own timing events (srb12_ctx_set_timing): each event
    # record is a marker the queue drains to; the kernel times above came from the same launches
    solver.set_timing(False)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_step = np.array([a.elapsed_time(bb) for a, bb in ev])
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    status = out["status"].cpu().numpy(); iters = out["iters"].cpu().numpy()
    sel_ms = float(np.median([k[0] for k in kern])); solve_ms = float(np.median([k[1] for k in kern]))
    flops = srb12_executed_flops(N, Ko + Kn, iters)
    achieved = flops / (solve_ms * 1e-3) / 1e12
    io = n_loc * 8 * (12 + 24 * N + 12 * N + (24 * N + 1) + 1) + n_loc * 4 * (4 * N + 4)
    line = {
        "metric": "SRB-12 NMPC solves/sec (extension mode, DESIGN.md section 11)", "value": A_total * args.steps / elapsed,
        "unit": "solves/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{A_local} agents/GPU, 12-state SRB, horizon {N}, trot, 3 static + 8-nearest "
                               "inter-agent CBF, fp64", "agents_per_gpu": A_local, "agents_total": A_total,
                   "parallelism": f"agents sharded x{world}"},
        "p50_ms": float(np.percentile(per_step, 50)), "p99_ms": float(np.percentile(per_step, 99)),
        "optimal_frac": float((np.isin(status[:, 0], (0, 4)) & (status[:, 1] == 0)).mean()), "iters_mean": iters.mean(0).tolist(),
        "iters_max": iters.max(0).tolist(),
        "roofline": {"bound": "mfma", "limiter": "latency", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic_from("s12", n_loc)[0],
                     "traffic_source": traffic_from("s12", n_loc)[1], "kernel": "srb12_kernel",
                     "kernel_ms": solve_ms, "select_ms": sel_ms, "io_bytes_per_launch": io,
                     "flop_model": "bench.srb12_executed_flops (Riccati IPM, DESIGN.md 11); latency-bound"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, ROOT)
        import oracle
        op = oracle.params12(N, K_obs=Ko_, K_nbr=Kn_)
        nthreads = host_threads()
        t1 = time.perf_counter(); n = 0
        while time.perf_counter() - t1 < args.cpu_seconds:
            sl = slice(n % A_total, n % A_total + 32)
            oracle.solve_batch12(op, b["x0"][sl], b["xref"][sl], b["foot"][sl], b["contact"][sl], b["obstacles"],
                                 b["nbr_state"], agent_offset=sl.start, nthreads=nthreads)
            n += b["x0"][sl].shape[0]
        dt = time.perf_counter() - t1
        line["cpu_baseline"] = {"value": n / dt, "unit": "solves/s", "cores": nthreads, "kind": "port",
                                "sample": f"{n} solves (32-agent slices of the same batch) in {dt:.1f} s, "
                                          f"oracle/srb12.c (dense full-space LU), {nthreads} threads"}
    if rank == 0:
        print(json.dumps(line), flush=True)
    solver.close()


def rank_batch(config, agents_per_gpu, world, rank, seed=1234):
    """The swarm of a `world`-GPU run of `config` and this rank's block of it: (A_total, the whole
    batch as host arrays, lo, hi).  Every rank generates the whole swarm identically and keeps
    agents [lo, hi); the obstacle arena and the neighbour snapshot (get_lastState rows of every
    agent, MPC_dist.cpp:1272-1276) stay whole.  tests/test_gpu_shards.py solves exactly this."""
    cfg = CONFIGS[config]
    A_total = agents_per_gpu * world
    b = workload.make_batch(A_total, cfg["N"], cfg["C"], seed=seed)
    lo, hi = sdist.shard_range(A_total, world, rank)
    return A_total, b, lo, hi


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: run this script as N ranks (one per GPU) under
    torch.distributed.run on 127.0.0.1, as the driver does, and return their exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def plumbing(args, world, rank):
    """The launch / barrier / max-over-ranks path of main() on CPU (gloo), without a solve: every
    rank reports, rank 0 prints the JSON line with n_gpus = WORLD_SIZE and value null."""
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    t0 = time.perf_counter()
    elapsed = time.perf_counter() - t0
    seen = torch.zeros(world, dtype=torch.int64)
    seen[rank] = 1
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dist.all_reduce(seen)
    print(f"bench.py rank {rank}/{world} reporting", file=sys.stderr, flush=True)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "plumbing": True, "ranks_reporting": int(seen.sum())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", choices=["nmpc", "ll", "srb12"], default="nmpc")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--agents", type=int, default=0, help="agents per GPU (override)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--waves", type=int, default=0, help="waves per agent (0 automatic; srb_ctx_set_waves)")
    ap.add_argument("--qp-init", type=int, default=1,
                    help="QP-stage start: 1 scaled (default), 0 iSWIFT's kkt_initialize (srb_ctx_set_qp_init)")
    ap.add_argument("--kkt-fp32-mu", type=float, default=0.0,
                    help="SRB_OPT_KKT_FP32_MU: invert the reduced Newton matrix in fp32 while mu > this, refined in fp64 "
                         "(BASELINE configs[4] 'fp32 KKT with fp64 iterative-refine residuals'); 0 = fp64 throughout")
    ap.add_argument("--kkt-fp32-refine", type=int, default=3, help="SRB_OPT_KKT_FP32_REFINE")
    ap.add_argument("--qp-warm-tol", type=float, default=None,
                    help="diagnostics: the QP stage's tolerance before the NLP (SRB_OPT_QP_WARM_TOL; default: the library's)")
    ap.add_argument("--polish-fused", type=int, default=1,
                    help="1 (default): the active-set polish runs at the end of the solve kernel where the instance "
                         "allows (NZL <= 16), 0: as srb_polish_kernel (SRB_OPT_POLISH_FUSED)")
    ap.add_argument("--emulate-shards", type=int, default=1,
                    help="diagnostic: solve rank 0's shard of a swarm this many GPUs wide on one GPU (the whole "
                         "neighbour snapshot and obstacle arena of that swarm, no collective)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_traffic.py); default profiles/r06_pmc_traffic_c<config>.json, else r05's")
    ap.add_argument("--lib", default=None,
                    help="diagnostics: time the variant build libsrbnmpc_<tag>.so instead of the product library")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU check of the multi-process launch only (gloo, no GPU, no solve; tests/test_bench_launch.py)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start N ranks under torch.distributed.run as CHILD processes (no
        # GPU has been touched in this process; never exec over it) and exit with their status
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a number for another "
              f"GPU count", file=sys.stderr)
        sys.exit(2)
    if args.plumbing:
        plumbing(args, world, rank)
        return
    if args.lib:
        srbnmpc.use_library(args.lib)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if args.path in ("ll", "srb12"):
        (main_ll if args.path == "ll" else main_srb12)(args, world, rank, local_rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return

    cfg = dict(CONFIGS[args.config])
    A_local = args.agents or cfg["agents"]
    N, C = cfg["N"], cfg["C"]
    p = srbnmpc.default_params(N, C, K_obs=cfg["K_obs"], K_nbr=cfg["K_nbr"], use_nlp=1)
    A_total, b, lo, hi = rank_batch(args.config, A_local, max(world, args.emulate_shards), rank)
    sh = {k: (v[lo:hi] if k not in ("obstacles", "nbr_state") else v) for k, v in b.items()}
    t = {k: torch.as_tensor(np.ascontiguousarray(v).reshape(v.shape[0], -1), dtype=torch.float64, device=dev)
         for k, v in sh.items()}
    nbr_local = t["nbr_state"][lo:hi].contiguous()
    nbr_all = t["nbr_state"] if cfg["K_nbr"] > 0 else None
    n_loc = hi - lo
    # Bezier buffer state (fitComTrajectory_eventbase runs fused in the solve kernel): start
    # position with zero velocity, as before an agent's first solve (MPC_dist.cpp:792)
    alpha_buf = torch.stack([t["x0"][:, 0], torch.zeros_like(t["x0"][:, 0]), t["x0"][:, 2],
                             torch.zeros_like(t["x0"][:, 0])], 1).contiguous()
    out = dict(x_qp=None, alpha=torch.zeros((n_loc, 20), dtype=torch.float64, device=dev),
               x=torch.zeros((n_loc, p.nv), dtype=torch.float64, device=dev),
               obj=torch.zeros(n_loc, dtype=torch.float64, device=dev),
               status=torch.zeros((n_loc, 2), dtype=torch.int32, device=dev),
               iters=torch.zeros((n_loc, 2), dtype=torch.int32, device=dev))
    solver = srbnmpc.BatchSolver(p, n_loc, local_rank)
    solver.set_waves(args.waves)
    solver.set_qp_init(args.qp_init)
    solver.set_option("polish_fused", args.polish_fused)
    if args.qp_warm_tol is not None:
        solver.set_option("qp_warm_tol", args.qp_warm_tol)
    if args.kkt_fp32_mu > 0:
        solver.set_option("kkt_fp32_mu", args.kkt_fp32_mu)
        solver.set_option("kkt_fp32_refine", args.kkt_fp32_refine)
    # one explicit stream for the collective, both kernels and the timing events (the C ABI
    # launches on the stream it is handed; the null stream would not order against it)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    exchange = sdist.NeighbourExchange(A_total, world, rank, dev) if cfg["K_nbr"] > 0 and world > 1 else None
    Ko, Kn = solver.n_selected(sh["obstacles"].shape[0], A_total if cfg["K_nbr"] > 0 else 0)
    out["sel"] = torch.zeros((n_loc, Ko + Kn), dtype=torch.int32, device=dev)

    if exchange is not None:
        solver.set_option("selection", 0)          # the step selects around the collective (below)

    def step():
        if exchange is None:
            solver.solve_device(t["x0"], t["ref"], t["foot"], t["obstacles"], nbr_all, out, agent_offset=lo,
                                stream=stream.cuda_stream, alpha_buf=alpha_buf, obstacles_version=1)
            return
        # multi-GPU: the all-gather of the neighbour snapshot is issued first (RCCL on its own
        # stream), the static obstacles -- which need no neighbour row -- are selected on the compute stream
        # while it is in flight, then the compute stream waits for the collective (no host block) and the
        # neighbour selection and the solve follow
        pend = exchange.start(nbr_local)
        solver.select_device(t["x0"], t["obstacles"], exchange.out, out["sel"], tables=1, agent_offset=lo,
                             stream=stream.cuda_stream, obstacles_version=1)
        nb = pend.wait()
        solver.select_device(t["x0"], t["obstacles"], nb, out["sel"], tables=2, agent_offset=lo,
                             stream=stream.cuda_stream)
        solver.solve_device(t["x0"], t["ref"], t["foot"], t["obstacles"], nb, out, agent_offset=lo,
                            stream=stream.cuda_stream, alpha_buf=alpha_buf, obstacles_version=1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    kern, pol = [], []
    for _ in range(3):            # kernel duration on the stream it runs on (HIP events in the C ABI)
        step()
        kern.append(solver.last_kernel_ms())
        pol.append(solver.last_polish_ms())
    # the timed loop runs without the library's own timing events (SRB_OPT_TIMING): each event record
    # is a marker the queue drains to, a few us a step; the kernel times above came from the same launches
    solver.set_option("timing", 0)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_step = np.array([a.elapsed_time(bb) for a, bb in ev])
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        lat = torch.as_tensor(per_step, dtype=torch.float64, device=dev)
        gl = [torch.empty_like(lat) for _ in range(world)]
        dist.all_gather(gl, lat)
        per_step = torch.cat(gl).cpu().numpy()
    ms_per_step = elapsed * 1e3 / args.steps
    value = (hi - lo) * world * args.steps / elapsed if args.emulate_shards > 1 else A_total * args.steps / elapsed

    status = out["status"].cpu().numpy(); iters = out["iters"].cpu().numpy()
    solve_ms = float(np.median([k[1] for k in kern]))
    flops = executed_flops(p, iters, cfg["K_obs"] + cfg["K_nbr"])
    achieved = flops / (solve_ms * 1e-3) / 1e12
    dense_per_solve = dense_equiv_flops(p, iters) / max(1, iters.shape[0])
    cyc_iter = solve_ms * 1e-3 * SCLK_GHZ * 1e9 / max(1, int(iters.sum(1).max()))
    traffic = traffic_polish = None
    fused = solver.polish_fused_active()
    if args.traffic_json is None:           # this round's PMC summary of the config, else round 5's
        args.traffic_json = next((f for f in (os.path.join(ROOT, "profiles", f"{r}_pmc_traffic_c{args.config}.json")
                                              for r in ("r06", "r05")) if os.path.exists(f)),
                                 os.path.join(ROOT, "profiles", f"r06_pmc_traffic_c{args.config}.json"))
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("config") == args.config and tj.get("agents") == n_loc and \
                    tj.get("polish_fused", 0) == int(fused):
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_polish = tj.get("kernels", {}).get("srb_polish_kernel", {}).get("hbm_bytes")
        except Exception:
            traffic = None
    kkt32 = args.kkt_fp32_mu > 0 and solver.get_option("last_kkt_fp32") == 1.0
    line = {
        "metric": METRIC, "value": value, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("f64 (reduced Newton matrix inverted in fp32 while mu > %g, %d fp64 refinement steps per solve)"
                  % (args.kkt_fp32_mu, args.kkt_fp32_refine)) if kkt32 else "f64", "data": "synthetic",
        "config": {"workload": cfg["name"], "agents_per_gpu": A_local, "agents_total": A_total, "horizon": N,
                   "contacts": C, "K_obs": cfg["K_obs"], "K_nbr": cfg["K_nbr"], "parallelism": f"agents sharded x{world}",
                   "emulated_shards": args.emulate_shards, "n_obs": int(sh["obstacles"].shape[0]),
                   "nbr_rows": int(A_total if cfg["K_nbr"] else 0)},
        "p50_ms": float(np.percentile(per_step, 50)), "p99_ms": float(np.percentile(per_step, 99)),
        "optimal_frac": float((np.isin(status[:, 0], (0, 4)) & (status[:, 1] == 0)).mean()),
        "acceptable_frac": float((np.isin(status[:, 0], (0, 4)) & (status[:, 1] == 4)).mean()),
        "iters_mean": [float(iters[:, 0].mean()), float(iters[:, 1].mean())],
        "iters_max": [int(iters[:, 0].max()), int(iters[:, 1].max())],
        "qp_init": args.qp_init,
        "dense_kkt_flops_per_solve": dense_per_solve,
        "dense_kkt_flops_note": "SURVEY.md 8(d) work-equivalence figure: (2/3) d^3 + 4 d^2 per IPM iteration of the "
                                "unreduced dense KKT (d = nv + neq) x this batch's iterations, per solve; a "
                                "comparison with a dense-KKT solver, not executed flops and not a rate",
        "roofline": {"bound": "mfma", "limiter": "latency", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "traffic_source": os.path.relpath(args.traffic_json, ROOT) if traffic is not None else None,
                     "cycles_per_iter": cyc_iter,
                     "cycles_per_iter_note": "solve-kernel HIP-event time x 2.4 GHz / IPM iterations (QP + NLP) of "
                                             "the slowest agent: the critical-path cost of one iteration; per-phase "
                                             "split in profiles/r06_c3_stamps.txt (r05_*_stamps.txt)",
                     "kernel": "srb_nmpc_kernel", "waves_per_agent": solver.waves(), "kernel_ms": solve_ms, "knn_ms": float(np.median([k[0] for k in kern])),
                     "flop_model": "executed fp64 flops of the condensed IPM (bench.executed_flops, DESIGN.md 6) over "
                                   "the fp64 peak; the kernel is latency-bound (dependent FMA / cross-lane chains per "
                                   "agent), neither MFMA- nor HBM-throughput-bound",
                     "polish_ms": float(np.median(pol)),
                     "polish_kernel": "fused into srb_nmpc_kernel" if fused else "srb_polish_kernel",
                     "polish_traffic": traffic_polish,
                     "io_bytes_per_launch": io_bytes(p, n_loc, sh["obstacles"].shape[0], A_total if cfg["K_nbr"] else 0)},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(cfg, sh, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    solver.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
