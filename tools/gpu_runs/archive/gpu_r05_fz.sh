#!/bin/bash
# N = 20 with the fused polish and the compiled horizon (24_4_2_20_2_11): GPU suite + bench lines, then
# FETCH / WRITE passes and kernel-trace stats of config 5 and configs[1] (the obstacle-position aliasing)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_runs/gpu_r05_suite.sh fz || exit 1
C=profiles/r05_pmc_calib.json
for cfg in 5 2; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmcf_c${cfg}_$ctr
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmcf_c${cfg}_$ctr -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config $cfg > $O/pmcf_c${cfg}_$ctr.log 2>&1 || { tail -5 $O/pmcf_c${cfg}_$ctr.log; exit 1; }
  done
done
python tools/pmc_traffic.py $O/pmcf_c5_FETCH_SIZE $O/pmcf_c5_WRITE_SIZE 5 2048 $O/r05f_pmc_traffic_c5.json $C 1 &&
python tools/pmc_traffic.py $O/pmcf_c2_FETCH_SIZE $O/pmcf_c2_WRITE_SIZE 2 64 $O/r05f_pmc_traffic_c2.json $C 1 || exit 1
rm -rf $O/prof_fz_c5
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_fz_c5 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 --config 5 > $O/prof_fz_c5.log 2>&1 || { tail -5 $O/prof_fz_c5.log; exit 1; }
