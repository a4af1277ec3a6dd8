#!/bin/bash
# Round-3 measurement run: counter calibration (tools/ubench/fetch_calib), FETCH_SIZE / WRITE_SIZE
# passes (separate runs) of bench configs 3 (default instance and the spill-free 2-wave instance,
# for the scratch share of WRITE_SIZE), 5, 2 and the LL path, rocprofv3 kernel-trace stats of the
# same commands, then the bench lines reading the traffic files.  Every GPU step time-limited and
# chained: the first failure ends the script.   usage: tools/gpu_runs/gpu_r03_prof.sh
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
python tools/pmc_traffic.py calib $O/cal_FETCH_SIZE $O/cal_WRITE_SIZE $O/r03_pmc_calib.json || exit 1
pmc c3 --config 3 && python tools/pmc_traffic.py $O/pmc_c3_FETCH_SIZE $O/pmc_c3_WRITE_SIZE 3 1024 $O/r03_pmc_traffic_c3.json $O/r03_pmc_calib.json || exit 1
pmc c3w2 --config 3 --waves 2 && python tools/pmc_traffic.py $O/pmc_c3w2_FETCH_SIZE $O/pmc_c3w2_WRITE_SIZE c3-waves2 1024 $O/r03_pmc_traffic_c3_waves2.json $O/r03_pmc_calib.json || exit 1
pmc c5 --config 5 && python tools/pmc_traffic.py $O/pmc_c5_FETCH_SIZE $O/pmc_c5_WRITE_SIZE 5 2048 $O/r03_pmc_traffic_c5.json $O/r03_pmc_calib.json || exit 1
pmc c2 --config 2 && python tools/pmc_traffic.py $O/pmc_c2_FETCH_SIZE $O/pmc_c2_WRITE_SIZE 2 64 $O/r03_pmc_traffic_c2.json $O/r03_pmc_calib.json || exit 1
pmc ll --path ll && python tools/pmc_traffic.py $O/pmc_ll_FETCH_SIZE $O/pmc_ll_WRITE_SIZE ll 0 $O/r03_pmc_traffic_ll.json $O/r03_pmc_calib.json || exit 1
pmc s12 --path srb12 && python tools/pmc_traffic.py $O/pmc_s12_FETCH_SIZE $O/pmc_s12_WRITE_SIZE s12 1024 $O/r03_pmc_traffic_s12.json $O/r03_pmc_calib.json || exit 1
stats c3 --config 3 && stats c5 --config 5 && stats c2 --config 2 && stats ll --path ll && stats s12 --path srb12 || exit 1
timeout -k 10 300 python bench.py --traffic-json $O/r03_pmc_traffic_c3.json > $O/r03_bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
for c in 5 2; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --traffic-json $O/r03_pmc_traffic_c$c.json > $O/r03_bench_c$c.json 2> $O/bench_c$c.err || { tail $O/bench_c$c.err; exit 1; }
done
timeout -k 10 200 python bench.py --path ll --no-cpu-baseline > $O/r03_bench_ll.json 2> $O/bench_ll.err || { tail $O/bench_ll.err; exit 1; }
timeout -k 10 200 python bench.py --path srb12 > $O/r03_bench_srb12.json 2> $O/bench_s12.err || { tail $O/bench_s12.err; exit 1; }
SRB_STAMPS_LIB=libsrbnmpc_stamps.so timeout -k 10 120 python tools/stamps.py 10 2 3 8 1024 > $O/r03_c3_stamps.txt 2>&1 || exit 1
cat $O/r03_bench_c3.json $O/r03_bench_c5.json $O/r03_bench_c2.json $O/r03_bench_ll.json $O/r03_bench_srb12.json
find $O -name "*kernel_stats.csv" | sort
echo "round script done"
