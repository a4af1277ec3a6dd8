#!/bin/bash
# SRB-12 extension mode on the GPU: its parity tests, a per-iteration trace of two agents, then a
# short bench line of the mode.  Each GPU step time-limited; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_srb12.py -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_srb12.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_srb12.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/srb12_trace.py stand 21 64 24 31 > gpurun_out/srb12_trace.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --path srb12 --steps 20 --cpu-seconds 6 > gpurun_out/bench_srb12.json 2> gpurun_out/bench_srb12.err || { tail gpurun_out/bench_srb12.err; exit 1; }
cat gpurun_out/bench_srb12.json
exit $rc
