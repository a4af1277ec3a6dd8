#!/bin/bash
# SRB-12 bench lines and GPU tests of several variant builds.   usage: tools/gpu_r04_s12multi.sh <tag> <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; shift
for lib in libsrbnmpc.so "$@"; do
  SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r04_s12m_${T}_$lib.json 2> $O/r04_s12m_${T}.err || { tail -20 $O/r04_s12m_${T}.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r04_s12m_${T}_$lib.json')); r=d['roofline']; print('$lib', d['ms_per_step'], d['p99_ms'], r['kernel_ms'], d['iters_mean'], d['iters_max'], d['optimal_frac'])"
done
for lib in "$@"; do
  SRBNMPC_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -q --timeout 150 --timeout-method thread > $O/r04_s12m_${T}_${lib}_tests.log 2>&1
  rc=$?; echo "== $lib"; tail -3 $O/r04_s12m_${T}_${lib}_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
