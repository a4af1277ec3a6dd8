#!/bin/bash
# LL kernel after the spill fix: LL GPU tests, FETCH_SIZE / WRITE_SIZE passes
# (separate runs), kernel-trace stats and the bench line.  Every GPU step time-limited, chained.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ll_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r03_pytest_ll.log 2>&1 || { tail -20 $O/r03_pytest_ll.log; exit 1; }
tail -2 $O/r03_pytest_ll.log
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/pmc_ll_$ctr
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmc_ll_$ctr -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --path ll > $O/pmc_ll_$ctr.log 2>&1 || { tail -5 $O/pmc_ll_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py $O/pmc_ll_FETCH_SIZE $O/pmc_ll_WRITE_SIZE ll 0 $O/r03_pmc_traffic_ll.json profiles/r03_pmc_calib.json || exit 1
cp $O/r03_pmc_traffic_ll.json profiles/ && rm -rf $O/prof_ll
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ll -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 --path ll > $O/prof_ll.log 2>&1 || { tail -5 $O/prof_ll.log; exit 1; }
timeout -k 10 200 python bench.py --path ll --no-cpu-baseline > $O/r03_bench_ll.json 2> $O/bench_ll.err || { tail $O/bench_ll.err; exit 1; }
cat $O/r03_pmc_traffic_ll.json $O/r03_bench_ll.json
find $O/prof_ll -name "*kernel_stats.csv"
echo "ll script done"
