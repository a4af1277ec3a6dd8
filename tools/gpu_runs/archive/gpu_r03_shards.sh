#!/bin/bash
# Round-3: the RCCL single-rank test, and rank 0's shard of the 8-GPU configs[3] / configs[4] swarms
# solved on this GPU (bench.py --emulate-shards 8: the whole snapshot and arena, no collective).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py -v -m gpu -k rccl --timeout 200 --timeout-method thread > $O/pytest_rccl.log 2>&1; rc=$?
tail -3 $O/pytest_rccl.log
for c in 4 5; do
  timeout -k 10 200 python bench.py --config $c --emulate-shards 8 --no-cpu-baseline --steps 30 > $O/r03_bench_c${c}_shard8.json 2> $O/sh.err || { tail -5 $O/sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/r03_bench_c${c}_shard8.json'));r=d['roofline'];print('config $c shard of 8', round(d['value']), 'per GPU, ms/step', round(d['ms_per_step'],4), 'solve', round(r['kernel_ms'],4), 'knn', round(r['knn_ms'],4), 'polish', round(r['polish_ms'],4), 'opt', d['optimal_frac'])"
done

timeout -k 10 200 python bench.py --path srb12 > $O/r03_bench_srb12.json 2> $O/sh.err || { tail -5 $O/sh.err; exit 1; }
cat $O/r03_bench_srb12.json
exit $rc
