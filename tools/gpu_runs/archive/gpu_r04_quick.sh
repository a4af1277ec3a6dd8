#!/bin/bash
# quick GPU check: a few LIP parity tests and the SRB-12 parity tests.   usage: tools/gpu_r04_quick.sh <tag>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 150 --timeout-method thread -k "test_gpu_matches_oracle or kat2" > gpurun_out/r04_quick_lip_$1.log 2>&1
rc=$?; tail -5 gpurun_out/r04_quick_lip_$1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r04_quick_s12_$1.log 2>&1
rc=$?; tail -5 gpurun_out/r04_quick_s12_$1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
