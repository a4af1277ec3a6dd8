#!/bin/bash
# Round-6 measurement run of the final build: FETCH_SIZE / WRITE_SIZE passes (separate runs) of bench configs 3, 2,
# 5 and the SRB-12 path (calibrated, tools/pmc_traffic.py -> r06_pmc_traffic_*.json); rocprofv3 kernel-trace stats of
# the same commands; then the bench lines reading the traffic files (the default line with its cpu_baseline).
# Every GPU step time-limited and chained: the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
pmc() {   # pmc <tag> <bench args...>: one FETCH_SIZE pass and one WRITE_SIZE pass
  local tag=$1; shift
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmc_${tag}_$ctr
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmc_${tag}_$ctr -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" > $O/pmc_${tag}_$ctr.log 2>&1 || { tail -5 $O/pmc_${tag}_$ctr.log; return 1; }
  done
}
stats() { # stats <tag> <bench args...>: kernel-trace summary of the bench command
  local tag=$1; shift
  rm -rf $O/prof_$tag
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 20 "$@" > $O/prof_$tag.log 2>&1 || { tail -5 $O/prof_$tag.log; return 1; }
}
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/cal_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/cal_$ctr -o run --output-format csv -- ./tools/ubench/fetch_calib > $O/cal_$ctr.log 2>&1 || { tail -5 $O/cal_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py calib $O/cal_FETCH_SIZE $O/cal_WRITE_SIZE $O/r06_pmc_calib.json || exit 1
C=$O/r06_pmc_calib.json
pmc c3 --config 3 && python tools/pmc_traffic.py $O/pmc_c3_FETCH_SIZE $O/pmc_c3_WRITE_SIZE 3 1024 $O/r06_pmc_traffic_c3.json $C 1 || exit 1
pmc c2 --config 2 && python tools/pmc_traffic.py $O/pmc_c2_FETCH_SIZE $O/pmc_c2_WRITE_SIZE 2 64 $O/r06_pmc_traffic_c2.json $C 1 || exit 1
pmc c5 --config 5 && python tools/pmc_traffic.py $O/pmc_c5_FETCH_SIZE $O/pmc_c5_WRITE_SIZE 5 2048 $O/r06_pmc_traffic_c5.json $C 1 || exit 1
pmc s12 --path srb12 && python tools/pmc_traffic.py $O/pmc_s12_FETCH_SIZE $O/pmc_s12_WRITE_SIZE s12 1024 $O/r06_pmc_traffic_s12.json $C 0 || exit 1
stats c3 --config 3 && stats c2 --config 2 && stats c5 --config 5 && stats s12 --path srb12 || exit 1
cp $O/r06_pmc_traffic_*.json profiles/ || exit 1
timeout -k 10 300 python3 bench.py > $O/r06_bench_c3.json 2> $O/r06_bench_c3.err || { tail $O/r06_bench_c3.err; exit 1; }
timeout -k 10 200 python3 bench.py --config 5 --no-cpu-baseline > $O/r06_bench_c5.json 2> $O/r06_bench_c5.err || { tail $O/r06_bench_c5.err; exit 1; }
timeout -k 10 200 python3 bench.py --config 2 --no-cpu-baseline > $O/r06_bench_c2.json 2> $O/r06_bench_c2.err || { tail $O/r06_bench_c2.err; exit 1; }
timeout -k 10 200 python3 bench.py --path srb12 > $O/r06_bench_srb12.json 2> $O/r06_bench_s12.err || { tail $O/r06_bench_s12.err; exit 1; }
cat $O/r06_bench_c3.json $O/r06_bench_c5.json $O/r06_bench_c2.json $O/r06_bench_srb12.json
find $O -name "*kernel_stats.csv" -newer $C | sort
echo "round script done"
