#!/bin/bash
# Development GPU run: gpu parity suite (stop at first failure), then bench lines for configs 2/3/5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log | grep -v "^$" | tail -25
[ $rc -eq 0 ] || exit $rc
for c in 2 3 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { tail -5 gpurun_out/bench_c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_c$c.json'));r=d['roofline'];print($c, round(d['value']), 'solves/s', round(d['ms_per_step'],3),'ms/step p99',round(d['p99_ms'],3),'kernel',round(r['kernel_ms'],3),'iters',d['iters_mean'],'opt',d['optimal_frac'])"
done
if [ -f srb-cbf-nmpc_amd/srbnmpc/libsrbnmpc_stamps.so ]; then
  timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { tail -5 gpurun_out/stamps.log; exit 1; }
  cat gpurun_out/stamps.log
fi
