#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for c in 5 3; do
  for r in 1e8 1e9 1e10 1e7; do
    SRB_POLISH_RHO=$r timeout -k 10 120 python tools/polish_probe.py $c || exit 1
  done
done
