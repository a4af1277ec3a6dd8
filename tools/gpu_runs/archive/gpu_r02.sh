#!/bin/bash
# Round-2 GPU run: gpu test suite, smoke, bench lines (default = configs[2]; configs[1], N=20,
# LL), rocprofv3 kernel stats + FETCH/WRITE PMC passes for the default config, stamps, and
# raw GPU outputs of config 5 for offline analysis.  Every GPU step time-limited; stops at
# the first failure.   usage: tools/gpu_runs/gpu_r02.sh [skip_tests]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
if [ -z "$1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -4 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -30; exit $rc; }
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for c in 2 5; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { tail gpurun_out/bench_c$c.err; exit 1; }
  cat gpurun_out/bench_c$c.json
done
timeout -k 10 200 python bench.py --path ll --no-cpu-baseline > gpurun_out/bench_ll.json 2> gpurun_out/bench_ll.err || { tail gpurun_out/bench_ll.err; exit 1; }
cat gpurun_out/bench_ll.json
timeout -k 10 120 python tools/dump_gpu.py 5 gpurun_out/c5_gpu.npz || exit 1
rm -rf gpurun_out/prof_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 > gpurun_out/prof_c3.log 2>&1 || { tail gpurun_out/prof_c3.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc3_$ctr
  timeout -k 10 120 rocprofv3 --pmc $ctr -d gpurun_out/pmc3_$ctr -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/pmc3_$ctr.log 2>&1 || { tail gpurun_out/pmc3_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py gpurun_out/pmc3_FETCH_SIZE gpurun_out/pmc3_WRITE_SIZE 3 1024 gpurun_out/r02_pmc_traffic_c3.json || exit 1
for a in "10 2 3 0 64" "10 2 3 8 1024"; do
  timeout -k 10 120 python tools/stamps.py $a > "gpurun_out/stamps_${a// /_}.log" 2>&1 || { tail "gpurun_out/stamps_${a// /_}.log"; exit 1; }
  cat "gpurun_out/stamps_${a// /_}.log"
done
find gpurun_out -name "*stats*.csv" | sort
echo "round script done"
