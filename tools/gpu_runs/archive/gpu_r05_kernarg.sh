#!/bin/bash
# is the solve kernel's per-agent fetch beyond its inputs the kernel-argument block
# (read per workgroup) or fills of partially written output lines?  (tools/ubench/kernarg_fetch.hip)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/ka_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/ka_$ctr -o run --output-format csv -- ./tools/ubench/kernarg_fetch > $O/ka_$ctr.log 2>&1 || { tail -5 $O/ka_$ctr.log; exit 1; }
done
python tools/ubench/kernarg_fit.py $O/ka_FETCH_SIZE $O/ka_WRITE_SIZE profiles/r05_pmc_calib.json $O/r05_kernarg_fetch.json
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/cf_$ctr
  timeout -s KILL 60 rocprofv3 --pmc $ctr -d $O/cf_$ctr -o run --output-format csv -- ./tools/ubench/code_fetch > $O/cf_$ctr.log 2>&1 || { tail -5 $O/cf_$ctr.log; exit 1; }
done
python tools/ubench/kernarg_fit.py $O/cf_FETCH_SIZE $O/cf_WRITE_SIZE profiles/r05_pmc_calib.json $O/r05_code_fetch.json code_big,code_small
