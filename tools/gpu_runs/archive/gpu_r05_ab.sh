#!/bin/bash
# A/B of a variant build against the product on the bench lines (configs[2] = --config 3, configs[1] = 2,
# N = 20 = 5), alternating, plus the variant's GPU parity tests.  usage: gpu_r05_ab.sh <tag> [configs] [tests-k]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; CF=${2:-"3 2 5"}; KX=${3:-""}
if [ -n "$KX" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --srbnmpc-lib libsrbnmpc_$T.so -k "$KX" > $O/ab_${T}_tests.log 2>&1; rc=$?
  tail -3 $O/ab_${T}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for rep in 1 2; do
  for c in $CF; do
    for lib in product $T; do
      a=""; [ $lib != product ] && a="--lib libsrbnmpc_$lib.so"
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline $a > $O/ab_${T}_${lib}_c${c}_$rep.json 2> $O/ab_${T}_${lib}_c${c}_$rep.err || { tail -5 $O/ab_${T}_${lib}_c${c}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/ab_${T}_${lib}_c${c}_$rep.json')); r=d['roofline']; print('c$c $lib', round(d['ms_per_step'],4), round(d.get('p99_ms') or 0,4), round(r.get('kernel_ms') or 0,4), round(r.get('polish_ms') or 0,4), d.get('iters_mean'), d.get('optimal_frac'))"
    done
  done
done
