#!/bin/bash
# A/B of the polish kernel's waves per agent (SRB_POLISH_NW) on bench configs 3 / 2 / 5, after the
# GPU suite.  Every GPU step time-limited; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in 3 2 5; do
  for pnw in 0 1 2 4; do
    SRB_POLISH_NW=$pnw timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 30 > $O/pnw_c${c}_$pnw.json 2> $O/pnw.err || { tail -5 $O/pnw.err; exit 1; }
    python -c "import json;d=json.load(open('$O/pnw_c${c}_$pnw.json'));r=d['roofline'];print('config $c polish_nw $pnw', round(d['value']), 'solves/s ms/step', round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'polish', round(r['polish_ms'],4), 'knn', round(r['knn_ms'],4), 'opt', d['optimal_frac'])"
  done
done
