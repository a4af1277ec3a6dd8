#!/bin/bash
# configs[2] A/B of solve-kernel variants: bench lines (alternating, twice), then FETCH_SIZE / WRITE_SIZE
# passes of each library (calibrated as in tools/gpu_r04_prof.sh).   usage: tools/gpu_r04_c3ab.sh <tag> <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out; T=$1; shift
for rep in 1 2; do
  for lib in libsrbnmpc.so "$@"; do
    SRBNMPC_LIB=$lib timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline > $O/r04_c3ab_${T}_$lib.json 2> $O/r04_c3ab_${T}.err || { tail -20 $O/r04_c3ab_${T}.err; exit 1; }
    python -c "import json; d=json.load(open('$O/r04_c3ab_${T}_$lib.json')); r=d['roofline']; print('$rep $lib', round(d['ms_per_step'],4), round(d['p99_ms'],4), round(r['kernel_ms'],4), d['iters_mean'], d['optimal_frac'])"
  done
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/cal_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/cal_$ctr -o run --output-format csv -- ./tools/ubench/fetch_calib > $O/cal_$ctr.log 2>&1 || { tail -5 $O/cal_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py calib $O/cal_FETCH_SIZE $O/cal_WRITE_SIZE $O/c3ab_calib.json > /dev/null || exit 1
for lib in libsrbnmpc.so "$@"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmcab_${lib}_$ctr
    SRBNMPC_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmcab_${lib}_$ctr -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config 3 > $O/pmcab_${lib}_$ctr.log 2>&1 || { tail -5 $O/pmcab_${lib}_$ctr.log; exit 1; }
  done
  python tools/pmc_traffic.py $O/pmcab_${lib}_FETCH_SIZE $O/pmcab_${lib}_WRITE_SIZE 3 1024 $O/c3ab_traffic_$lib.json $O/c3ab_calib.json 1 > /dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c3ab_traffic_$lib.json')); print('$lib traffic', d['hbm_bytes_per_launch'])"
done
