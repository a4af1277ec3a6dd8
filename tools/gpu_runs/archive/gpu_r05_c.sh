#!/bin/bash
# round 5: the GPU suite on the product build, the SRB-12 bench line, and traces of any non-OPTIMAL agent of
# the 1024-agent stand batch
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=${1:-c}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/r05_${T}_pytest_gpu.log 2>&1; rc=$?
tail -5 $O/r05_${T}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/r05_${T}_bench_srb12.json 2> $O/r05_${T}_bench_srb12.err || { tail -5 $O/r05_${T}_bench_srb12.err; exit 1; }
python -c "import json; d=json.load(open('$O/r05_${T}_bench_srb12.json')); print('srb12', d['ms_per_step'], d['p99_ms'], d.get('iters_mean'), d.get('optimal_frac'))"
timeout -k 10 300 python -u tools/srb12_trace.py stand 21 1024 auto > $O/r05_${T}_trace_stand21.txt 2>&1
grep -E "not OPTIMAL|^agent|oracle status" $O/r05_${T}_trace_stand21.txt
exit $rc
