#!/bin/bash
# Development GPU run: quick parity subset, bench lines, rocprofv3 kernel trace of config 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in 2 3 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_c$c.json'));r=d['roofline'];print($c, round(d['value']), 'solves/s', round(d['ms_per_step'],3),'ms/step p99',round(d['p99_ms'],3),'kernel',round(r['kernel_ms'],3),'knn',round(r['knn_ms'],3),'iters',d['iters_mean'],'opt',d['optimal_frac'])"
done
rm -rf gpurun_out/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --config 2 --no-cpu-baseline --steps 20 > gpurun_out/prof_c2.log 2>&1 || exit 1
find gpurun_out/prof_c2 -name "*stats*" | head
