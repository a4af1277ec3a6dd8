#!/bin/bash
# Round-3 polish check: GPU suite (no -x: every failure listed), then configs[2] / config 5 bench
# lines with and without the active-set polish (SRBNMPC_LIB A/B).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -30
for c in 3 5 2; do
  for v in "libsrbnmpc.so 1" "libsrbnmpc.so 0" "libsrbnmpc_nopolish.so 1"; do
    set -- $v
    SRBNMPC_LIB=$1 timeout -k 10 200 python bench.py --config $c --qp-init $2 --no-cpu-baseline > gpurun_out/bench_c${c}_$1_$2.json 2> gpurun_out/bench_c${c}_$1_$2.err || { tail gpurun_out/bench_c${c}_$1_$2.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_c${c}_$1_$2.json')); print('$c $1 qp_init=$2', round(d['value']), round(d['ms_per_step'], 4), 'solve', round(d['roofline']['kernel_ms'], 4), 'polish', d['roofline'].get('polish_ms'), d['optimal_frac'], d['acceptable_frac'], d['iters_mean'], d.get('iters_max'))"
  done
done
exit $rc
