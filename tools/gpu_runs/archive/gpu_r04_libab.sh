#!/bin/bash
# A/B of a variant build against the product library: configs[2] and configs[5] bench lines, then the
# LIP GPU parity tests on the variant.   usage: tools/gpu_r04_libab.sh <variant.so> <tag>
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; V=$1; T=$2
for lib in libsrbnmpc.so $V libsrbnmpc.so $V; do
  SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline > $O/r04_ab_${T}_$lib.json 2> $O/r04_ab_${T}.err || { tail -20 $O/r04_ab_${T}.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/r04_ab_${T}_$lib.json')); r=d['roofline']; print('$lib', d['ms_per_step'], d['p99_ms'], r['kernel_ms'], r['cycles_per_iter'], d['iters_max'])"
done
SRBNMPC_LIB=$V timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline > $O/r04_ab_${T}_c5.json 2>> $O/r04_ab_${T}.err || exit 1
python -c "import json; d=json.load(open('$O/r04_ab_${T}_c5.json')); r=d['roofline']; print('c5 $V', d['ms_per_step'], r['kernel_ms'], r['polish_ms'])"
SRBNMPC_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread > $O/r04_ab_${T}_tests.log 2>&1
rc=$?; tail -4 $O/r04_ab_${T}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
