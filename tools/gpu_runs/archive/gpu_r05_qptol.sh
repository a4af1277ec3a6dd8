#!/bin/bash
# QP warm-start tolerance scan (SRB_OPT_QP_WARM_TOL) on config 5 and configs[2]: step time, iterations, statuses
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for c in 5 3; do
  for t in 3e-1 1 3; do
    timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --qp-warm-tol $t > $O/qptol_c${c}_$t.json 2> $O/qptol.err || { tail -5 $O/qptol.err; exit 1; }
    python -c "import json; d=json.load(open('$O/qptol_c${c}_$t.json')); print('c$c tol=$t', round(d['ms_per_step'],4), round(d['p99_ms'],4), d['iters_mean'], d['iters_max'], d['optimal_frac'])"
  done
done
