#!/bin/bash
# the SRB-12 N = 20 polish of the variant builds against the oracle, with the
# polish state checks of -DSRB12_CHECK builds (tools/srb12_check.py), then the SRB-12 GPU tests of
# the no-waves_per_eu variant.   usage: tools/gpu_runs/gpu_r05_chk.sh <tag> <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; shift
for lib in "$@"; do
  echo "=== $lib"
  timeout -k 10 240 python -u tools/srb12_check.py --lib $lib > $O/r05_chk_${T}_$lib.txt 2>&1; rc=$?
  cat $O/r05_chk_${T}_$lib.txt | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
done
