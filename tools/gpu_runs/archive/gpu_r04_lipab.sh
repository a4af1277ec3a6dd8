#!/bin/bash
# LIP-mode A/B: bench lines of configs 3, 2 and 5 for the product build and variant builds (alternating,
# twice), then the whole GPU suite on the product build.   usage: tools/gpu_r04_lipab.sh <tag> <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; shift
for rep in 1 2; do
  for lib in libsrbnmpc.so "$@"; do
    for cfg in 3 2 5; do
      SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline > $O/r04_lipab_${T}_${lib}_c$cfg.json 2> $O/r04_lipab_${T}.err || { tail -20 $O/r04_lipab_${T}.err; exit 1; }
      python -c "import json; d=json.load(open('$O/r04_lipab_${T}_${lib}_c$cfg.json')); r=d['roofline']; print('$rep $lib c$cfg', round(d['ms_per_step'],4), round(d['p99_ms'],4), round(r['kernel_ms'],4), r.get('polish_ms'), d['iters_mean'], d['optimal_frac'])"
    done
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/r04_lipab_${T}_tests.log 2>&1
rc=$?; tail -3 $O/r04_lipab_${T}_tests.log; exit $rc
