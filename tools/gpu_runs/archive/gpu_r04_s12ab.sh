#!/bin/bash
# SRB-12 iteration: its GPU tests, the bench line, the per-phase stamps.   usage: tools/gpu_r04_s12ab.sh <tag>
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -q -x --timeout 150 --timeout-method thread > $O/r04_s12_tests_$1.log 2>&1
rc=$?; tail -3 $O/r04_s12_tests_$1.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r04_s12_bench_$1.json 2> $O/r04_s12_bench_$1.err || { tail -20 $O/r04_s12_bench_$1.err; exit 1; }
cat $O/r04_s12_bench_$1.json
SRBNMPC_LIB=libsrbnmpc_s12st.so timeout -k 10 120 python tools/srb12_stamps.py 0 24 > $O/r04_s12_stamps_$1.txt 2>&1 || { tail -20 $O/r04_s12_stamps_$1.txt; exit 1; }
cat $O/r04_s12_stamps_$1.txt
