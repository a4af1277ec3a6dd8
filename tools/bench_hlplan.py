"""Bench of the HL reference planner (generateReferenceTrajectory, MPC_dist.cpp:930-1104) on
one GPU against the CPU restatement (oracle/hl_plan.c, 1 thread) timed on a bounded sample.

    python tools/bench_hlplan.py [--agents 4,256,1024] [--loop 100000] [--cpu-seconds 10]
"""
import argparse, json, os, sys, time
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'srb-cbf-nmpc_amd'))
import numpy as np
import srbnmpc

ap = argparse.ArgumentParser()
ap.add_argument('--agents', default='4,256,1024,4096')
ap.add_argument('--loop', type=int, default=100000)
ap.add_argument('--cpu-seconds', type=float, default=10.0)
args = ap.parse_args()
for NA in [int(v) for v in args.agents.split(',')]:
    rng = np.random.default_rng(NA)
    Ps = np.array([0.0, 0.0, 0.0, -0.9, -1, 0, -1, -0.9]) if NA == 4 else \
        np.stack([rng.uniform(-4 * np.sqrt(NA / 4), 0, NA), rng.uniform(-3, 3, NA) * np.sqrt(NA / 4)], 1).ravel()
    Po = np.stack([rng.uniform(0, 9, 20), rng.uniform(-2, 2, 20)], 1)
    srbnmpc.hl_plan(Ps, Po, loop=400)                       # warm-up (module load)
    t0 = time.perf_counter(); srbnmpc.hl_plan(Ps, Po, loop=args.loop); g = time.perf_counter() - t0
    line = {"bench": "hl_planner", "agents": NA, "steps": args.loop, "gpu_s": g,
            "gpu_agent_steps_per_s": NA * args.loop / g}
    if os.path.exists(os.path.join(ROOT, 'oracle', 'liboracle.so')):
        import oracle
        steps = 400
        while True:                                          # bounded CPU sample
            t0 = time.perf_counter(); oracle.hl_plan(Ps, Po, loop=steps); c = time.perf_counter() - t0
            if c > args.cpu_seconds / 4 or steps >= args.loop:
                break
            steps = min(args.loop, steps * 4)
        line.update(cpu_s_sample=c, cpu_sample_steps=steps, cpu_agent_steps_per_s=NA * steps / c, cpu_threads=1,
                    speedup=(NA * args.loop / g) / (NA * steps / c))
    print(json.dumps(line), flush=True)
