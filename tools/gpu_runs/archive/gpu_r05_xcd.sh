#!/bin/bash
# XCD-aware agent mapping (csrc/srb_wave.h xcd_agent): GPU suite + bench lines, the traffic A/B of the
# configs[2] solve kernel, and bench-based FETCH/WRITE of configs[2] and N = 20
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_runs/gpu_r05_suite.sh xcd || exit 1
bash tools/gpu_runs/gpu_r05_traffic.sh xcd || exit 1
C=profiles/r05_pmc_calib.json
for cfg in 3 5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmcx_c${cfg}_$ctr
    timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmcx_c${cfg}_$ctr -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 --config $cfg > $O/pmcx_c${cfg}_$ctr.log 2>&1 || { tail -5 $O/pmcx_c${cfg}_$ctr.log; exit 1; }
  done
done
python tools/pmc_traffic.py $O/pmcx_c3_FETCH_SIZE $O/pmcx_c3_WRITE_SIZE 3 1024 $O/r05x_pmc_traffic_c3.json $C 1 &&
python tools/pmc_traffic.py $O/pmcx_c5_FETCH_SIZE $O/pmcx_c5_WRITE_SIZE 5 2048 $O/r05x_pmc_traffic_c5.json $C 0
