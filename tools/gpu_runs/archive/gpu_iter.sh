#!/bin/bash
# Development GPU run: full gpu test suite, per-phase stamps, bench lines for configs 2/3/5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python tools/stamps.py 10 2 3 0 64 > gpurun_out/stamps.log 2>&1 || exit 1
cat gpurun_out/stamps.log
for c in 2 3 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_c$c.json'));r=d['roofline'];print($c, round(d['value']), 'solves/s', round(d['ms_per_step'],3),'ms/step p99',round(d['p99_ms'],3),'kernel',round(r['kernel_ms'],3),'iters',d['iters_mean'],'opt',d['optimal_frac'])"
done
