#!/bin/bash
# Round-4 full check: the whole GPU suite (no -x: every failure listed), smoke(), the default bench line,
# the SRB-12 and N = 20 bench lines, SRB-12 stamps.  Each GPU step time-limited; a crash ends the script.
#   usage: tools/gpu_r04_full.sh <tag>
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/r04_pytest_gpu_$T.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/r04_pytest_gpu_$T.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke_$T.log 2>&1 || { tail -20 $O/r04_smoke_$T.log; exit 1; }
tail -1 $O/r04_smoke_$T.log
timeout -k 10 300 python bench.py > $O/r04_bench_c3_$T.json 2> $O/r04_bench_c3_$T.err || { tail -20 $O/r04_bench_c3_$T.err; exit 1; }
cat $O/r04_bench_c3_$T.json
timeout -k 10 300 python bench.py --path srb12 > $O/r04_bench_s12_$T.json 2> $O/r04_bench_s12_$T.err || { tail -20 $O/r04_bench_s12_$T.err; exit 1; }
cat $O/r04_bench_s12_$T.json
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline > $O/r04_bench_c5_$T.json 2> $O/r04_bench_c5_$T.err || { tail -20 $O/r04_bench_c5_$T.err; exit 1; }
cat $O/r04_bench_c5_$T.json
SRBNMPC_LIB=libsrbnmpc_s12st.so timeout -k 10 120 python tools/srb12_stamps.py 0 24 31 > $O/r04_s12_stamps_$T.txt 2>&1 || exit 1
head -20 $O/r04_s12_stamps_$T.txt
