#!/bin/bash
# LL CLF-QP: bench line (with CPU baseline), rocprofv3 kernel stats, HBM PMC passes.
# Every GPU step time-limited; stops at the first failure.   usage: tools/gpu_runs/gpu_ll_prof.sh [tag]
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 300 python bench.py --path ll > gpurun_out/bench_ll.json 2> gpurun_out/bench_ll.err || { tail gpurun_out/bench_ll.err; exit 1; }
cat gpurun_out/bench_ll.json
rm -rf gpurun_out/prof_ll
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ll -o run --output-format csv -- \
    python3 bench.py --path ll --no-cpu-baseline --steps 20 > gpurun_out/prof_ll.log 2>&1 || { tail gpurun_out/prof_ll.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_ll_$ctr
  timeout -k 10 300 rocprofv3 --pmc $ctr -d gpurun_out/pmc_ll_$ctr -o run --output-format csv -- \
      python3 bench.py --path ll --no-cpu-baseline --steps 5 > gpurun_out/pmc_ll_$ctr.log 2>&1 || { tail gpurun_out/pmc_ll_$ctr.log; exit 1; }
done
find gpurun_out -path "*ll*" -name "*stats*.csv" -o -path "*ll*" -name "*counter_collection*.csv" | sort
