#!/bin/bash
# SRB-12 GPU tests against variant builds (SRBNMPC_LIB).   usage: tools/gpu_r04_var.sh <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  SRBNMPC_LIB=$v timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r04_var_$v.log 2>&1
  rc=$?; echo "== $v"; tail -8 gpurun_out/r04_var_$v.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
