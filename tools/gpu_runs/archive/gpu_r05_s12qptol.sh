#!/bin/bash
# SRB-12 QP-stage tolerance scan (srb12_params.tol_qp) on the SRB-12 bench line
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for t in 1e-3 1e-2 1e-1 3e-1; do
  timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline --qp-warm-tol $t > $O/s12qptol_$t.json 2> $O/s12qptol.err || { tail -5 $O/s12qptol.err; exit 1; }
  python -c "import json; d=json.load(open('$O/s12qptol_$t.json')); print('s12 tol=$t', round(d['ms_per_step'],4), round(d['p99_ms'],4), d['iters_mean'], d['iters_max'], d['optimal_frac'])"
done
