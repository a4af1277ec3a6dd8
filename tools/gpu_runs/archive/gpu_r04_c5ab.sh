#!/bin/bash
# N = 20 (bench config 5) A/B of a variant build: bench lines (alternating, twice), then the config-5
# full-size test against the oracle with the variant.   usage: tools/gpu_r04_c5ab.sh <tag> <lib>
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; V=$2
for rep in 1 2; do
  for lib in libsrbnmpc.so $V; do
    SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline > $O/r04_c5ab_${T}_$lib.json 2> $O/r04_c5ab_${T}.err || { tail -20 $O/r04_c5ab_${T}.err; exit 1; }
    python -c "import json; d=json.load(open('$O/r04_c5ab_${T}_$lib.json')); r=d['roofline']; print('$rep $lib', round(d['ms_per_step'],4), round(d['p99_ms'],4), round(r['kernel_ms'],4), r.get('polish_ms'), d['iters_mean'], d['optimal_frac'])"
  done
done
SRBNMPC_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "config5 or full_size or matches_oracle" > $O/r04_c5ab_${T}_tests.log 2>&1
rc=$?; tail -3 $O/r04_c5ab_${T}_tests.log; exit $rc
