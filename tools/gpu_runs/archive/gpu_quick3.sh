#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for c in 3 5 2; do timeout -k 10 120 python tools/polish_probe.py $c || exit 1; done
timeout -k 10 300 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -30
exit $rc
