#!/bin/bash
# Round 6, call t: calibrated PMC traffic of the final build at configs[2] and config 5 (the selection kernel's
# bytes after the thresholded scan; the solve kernel for reference).  Separate FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/calt_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/calt_$ctr -o run --output-format csv -- ./tools/ubench/fetch_calib > $O/calt_$ctr.log 2>&1 || { tail -5 $O/calt_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py calib $O/calt_FETCH_SIZE $O/calt_WRITE_SIZE $O/r06_final_pmc_calib.json || exit 1
C=$O/r06_final_pmc_calib.json
for c in 3 5; do
  A=1024; [ $c = 5 ] && A=2048
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmct_c${c}_$ctr
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmct_c${c}_$ctr -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config $c > $O/pmct_c${c}_$ctr.log 2>&1 || { tail -5 $O/pmct_c${c}_$ctr.log; exit 1; }
  done
  python tools/pmc_traffic.py $O/pmct_c${c}_FETCH_SIZE $O/pmct_c${c}_WRITE_SIZE $c $A $O/r06_final_pmc_traffic_c$c.json $C 1 || exit 1
done
echo "done"
