#!/bin/bash
# A/B of an SRB-12 variant build: bench lines (product, variant, twice) and the SRB-12 GPU tests on the
# variant.   usage: tools/gpu_r04_s12libab.sh <variant.so> <tag>
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; V=$1; T=$2
for lib in libsrbnmpc.so $V libsrbnmpc.so $V; do
  SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r04_s12ab_${T}_$lib.json 2> $O/r04_s12ab_${T}.err || { tail -20 $O/r04_s12ab_${T}.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r04_s12ab_${T}_$lib.json')); r=d['roofline']; print('$lib', d['ms_per_step'], d['p99_ms'], r['kernel_ms'], d['iters_mean'], d['iters_max'], d['optimal_frac'])"
done
SRBNMPC_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -q --timeout 150 --timeout-method thread > $O/r04_s12ab_${T}_tests.log 2>&1
rc=$?; tail -6 $O/r04_s12ab_${T}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
