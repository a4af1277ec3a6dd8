#!/bin/bash
# Round 4, first check: the whole GPU suite (no -x: every failure listed), smoke(), the default bench
# and the SRB-12 bench.  Each GPU step time-limited and chained.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/r04_pytest_gpu_a.log 2>&1
rc=$?
tail -40 $O/r04_pytest_gpu_a.log | grep -E "passed|failed|FAILED|ERROR" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke_a.log 2>&1 || { tail -20 $O/r04_smoke_a.log; exit 1; }
tail -1 $O/r04_smoke_a.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 9 > $O/r04_bench_a.json 2> $O/r04_bench_a.err || { tail -20 $O/r04_bench_a.err; exit 1; }
cat $O/r04_bench_a.json
timeout -k 10 300 python bench.py --path srb12 --steps 20 --warmup 3 --no-cpu-baseline > $O/r04_bench_s12_a.json 2> $O/r04_bench_s12_a.err || { tail -20 $O/r04_bench_s12_a.err; exit 1; }
cat $O/r04_bench_s12_a.json
