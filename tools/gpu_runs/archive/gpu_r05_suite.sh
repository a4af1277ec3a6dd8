#!/bin/bash
# round 5: GPU suite on the product build, then the bench lines (default = configs[2] with the CPU baseline;
# configs[1]; configs[4] shape; SRB-12; LL)   usage: tools/gpu_runs/gpu_r05_suite.sh <tag> [nosuite]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1
if [ "$2" != "nosuite" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r05_${T}_pytest_gpu.log 2>&1; rc=$?
  tail -4 $O/r05_${T}_pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $O/r05_${T}_bench_c3.json 2> $O/r05_${T}_bench_c3.err || { tail -5 $O/r05_${T}_bench_c3.err; exit 1; }
for c in 2 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/r05_${T}_bench_c$c.json 2> $O/r05_${T}_bench_c$c.err || { tail -5 $O/r05_${T}_bench_c$c.err; exit 1; }
done
timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r05_${T}_bench_srb12.json 2> $O/r05_${T}_bench_srb12.err || exit 1
for f in c3 c2 c5 srb12; do
  python -c "import json; d=json.load(open('$O/r05_${T}_bench_$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], d.get('p99_ms'), r.get('kernel_ms'), r.get('polish_ms'), d.get('iters_mean'), d.get('iters_max'), d.get('optimal_frac'))"
done
