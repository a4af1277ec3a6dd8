#!/bin/bash
# Round 6, call s: one knn_select call site per wave count (code object 445 -> 158 KB), two waves a SIMD -- selection tests, per-table timing,
# bench A/B against the previous build (libsrbnmpc_thr.so), alternating, same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "knn or split_selection or sharded or shards or sentinel" > $O/r06_s_pytest_knn.log 2>&1 || { echo "knn tests failed"; tail -40 $O/r06_s_pytest_knn.log; exit 1; }
tail -2 $O/r06_s_pytest_knn.log
timeout -k 10 200 python3 -u tools/knn_split_timing.py > $O/r06_s_knn_split.txt 2>&1 || { tail $O/r06_s_knn_split.txt; exit 1; }
grep -v amdgpu.ids $O/r06_s_knn_split.txt
for rep in 1 2; do
  for lib in libsrbnmpc_thr.so libsrbnmpc.so; do
    for c in 3 5 2; do
      timeout -k 10 200 python3 -u bench.py --lib $lib --config $c --steps 50 --warmup 10 --no-cpu-baseline > $O/r06_s_${lib}_c$c.json 2> $O/r06_s_c$c.err || { echo "bench failed"; tail -5 $O/r06_s_c$c.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/r06_s_${lib}_c$c.json')); r=d['roofline']; print('$rep $lib c$c', round(d['ms_per_step'],4), 'p99', round(d['p99_ms'],4), 'kernel', round(r['kernel_ms'],4), 'knn', round(r['knn_ms'],4), 'opt', d['optimal_frac'])"
    done
  done
done
