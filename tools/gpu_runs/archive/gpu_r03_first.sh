#!/bin/bash
# Round-3 first GPU pass on the restored tree: full GPU suite (no -x, every failure listed),
# smoke(), the default bench line and a rocprofv3 kernel-trace summary of the same command.
# Each GPU step time-limited; the first hard failure (fault / abort / timeout) ends the script.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
cat $O/bench_default.json
rm -rf $O/prof_c3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 > $O/prof_c3.log 2>&1 || { tail -5 $O/prof_c3.log; exit 1; }
find $O/prof_c3 -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
