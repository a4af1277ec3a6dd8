#!/bin/bash
# selection inside the solve kernel (SRB_OPT_SELECT_FUSED): GPU suite, then bench A/B against the
# selection kernel on configs[2], configs[1] and config 5, alternating
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r05_sel_pytest_gpu.log 2>&1; rc=$?
tail -4 $O/r05_sel_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  for c in 3 2 5; do
    for sf in 1 0; do
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --select-fused $sf > $O/sel_c${c}_${sf}_${rep}.json 2> $O/sel_c${c}_${sf}.err || { tail -5 $O/sel_c${c}_${sf}.err; exit 1; }
      python -c "import json; d=json.load(open('$O/sel_c${c}_${sf}_${rep}.json')); r=d['roofline']; print('c$c sf=$sf', round(d['ms_per_step'],4), round(d['p99_ms'],4), round(r['kernel_ms'],4), round(r.get('knn_ms') or 0,4))"
    done
  done
done
