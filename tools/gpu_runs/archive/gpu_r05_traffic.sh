#!/bin/bash
# per-agent vs per-launch HBM traffic of the configs[2] solve kernel (tools/traffic_ab.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/tab_$ctr
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/tab_$ctr -o run --output-format csv -- python3 tools/traffic_ab.py > $O/tab_$ctr.log 2>&1 || { tail -5 $O/tab_$ctr.log; exit 1; }
done
python tools/traffic_ab.py --fit $O/tab_FETCH_SIZE $O/tab_WRITE_SIZE profiles/r05_pmc_calib.json $O/r05_traffic_ab_c3${1:+_$1}.json
