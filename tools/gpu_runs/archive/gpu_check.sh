#!/bin/bash
# Development GPU run: tests, smoke, bench, kernel trace.  Every GPU step time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 200 python bench.py --config 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
cat gpurun_out/bench_c2.json
timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1
cat gpurun_out/bench_c3.json
