#!/bin/bash
# SRB-12 check of the product build: bench lines (product, then variant builds for the A/B), the SRB-12
# GPU tests, per-phase stamps of the product's stamps build and of variant stamps builds.
#   usage: tools/gpu_r04_s12new.sh <tag> "<variant libs>" "<variant stamps libs>"
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1
for lib in libsrbnmpc.so $2; do
  SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r04_s12n_${T}_$lib.json 2> $O/r04_s12n_${T}.err || { tail -20 $O/r04_s12n_${T}.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r04_s12n_${T}_$lib.json')); r=d['roofline']; print('$lib', d['ms_per_step'], d['p99_ms'], r['kernel_ms'], d['iters_mean'], d['iters_max'], d['optimal_frac'])"
done
timeout -k 10 400 python -u -m pytest tests/test_srb12.py -m gpu -v --timeout 150 --timeout-method thread > $O/r04_s12n_${T}_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $O/r04_s12n_${T}_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in libsrbnmpc_s12st.so $3; do
  SRBNMPC_LIB=$lib timeout -k 10 120 python tools/srb12_stamps.py 0 24 > $O/r04_s12_stamps_${T}_$lib.txt 2>&1 || exit 1
  echo "== $lib"; head -18 $O/r04_s12_stamps_${T}_$lib.txt
done
