#!/bin/bash
# Round GPU run: gpu test suite, smoke, bench lines (configs 2/3/5), rocprofv3 kernel-trace
# stats and HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) for the default config.
# Every GPU step has its own time limit; the script stops at the first failure.
#   usage: tools/gpu_runs/gpu_round.sh [tag] [skip_tests]
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
if [ -z "$2" ]; then
  timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for c in 3 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { tail gpurun_out/bench_c$c.err; exit 1; }
  cat gpurun_out/bench_c$c.json
done
timeout -k 10 300 python bench.py --path ll > gpurun_out/bench_ll.json 2> gpurun_out/bench_ll.err || { tail gpurun_out/bench_ll.err; exit 1; }
cat gpurun_out/bench_ll.json
for c in 2 3 5; do
  rm -rf gpurun_out/prof_c$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o run --output-format csv -- \
      python3 bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/prof_c$c.log 2>&1 || { tail gpurun_out/prof_c$c.log; exit 1; }
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$ctr
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc_$ctr -o run --output-format csv -- \
      python3 bench.py --config 2 --no-cpu-baseline --steps 10 > gpurun_out/pmc_$ctr.log 2>&1 || { tail gpurun_out/pmc_$ctr.log; exit 1; }
done
rm -rf gpurun_out/prof_ll
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ll -o run --output-format csv -- \
    python3 bench.py --path ll --no-cpu-baseline --steps 20 > gpurun_out/prof_ll.log 2>&1 || { tail gpurun_out/prof_ll.log; exit 1; }
find gpurun_out -name "*stats*.csv" -o -name "*counter_collection*.csv" | sort
