#!/bin/bash
# Round-3 check: GPU suite (no -x, every failure listed), polish probe at configs 5 / 3, NLP traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
grep -E "^FAILED|^ERROR" gpurun_out/pytest_gpu.log | head -30
for c in 5 3 2; do timeout -k 10 120 python tools/polish_probe.py $c || exit 1; done
[ -n "$TRACE" ] && { timeout -k 10 120 python tools/nlp_trace.py $TRACE > gpurun_out/nlp_trace.log 2>&1 || exit 1; }
exit $rc
