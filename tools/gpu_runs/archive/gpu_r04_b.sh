#!/bin/bash
# Round 4: the rewritten SRB-12 kernel first (its GPU tests + a stamps-free bench), then the whole GPU
# suite (no -x: every failure listed), smoke(), the default bench.  Each GPU step time-limited; a crash
# (status other than 0 / 1 from pytest) ends the script.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_srb12.py -m gpu -v --timeout 150 --timeout-method thread > $O/r04_pytest_s12_b.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|ERROR|Error" $O/r04_pytest_s12_b.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --path srb12 --steps 20 --warmup 3 --no-cpu-baseline > $O/r04_bench_s12_b.json 2> $O/r04_bench_s12_b.err || { tail -20 $O/r04_bench_s12_b.err; exit 1; }
cat $O/r04_bench_s12_b.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread --deselect tests/test_srb12.py > $O/r04_pytest_gpu_b.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/r04_pytest_gpu_b.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke_b.log 2>&1 || { tail -20 $O/r04_smoke_b.log; exit 1; }
tail -1 $O/r04_smoke_b.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 9 > $O/r04_bench_b.json 2> $O/r04_bench_b.err || { tail -20 $O/r04_bench_b.err; exit 1; }
cat $O/r04_bench_b.json
