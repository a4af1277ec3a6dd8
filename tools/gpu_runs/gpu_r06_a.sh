#!/bin/bash
# Round 6, first call: (1) the round-5 generic-pointer polish failure reproduced and instrumented
# (tools/flat_polish_diag.py on libsrbnmpc_flat / _flateq / _baseeq), (2) SQ counters of the product
# solve kernel at configs[2], instruction fetch included (gpu_r06_sq.sh), (3) a product bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in flat flateq baseeq; do
  timeout -k 10 240 python3 -u tools/flat_polish_diag.py libsrbnmpc_$t.so > gpurun_out/r06_a_$t.txt 2>&1 || { echo "diag $t failed"; tail -5 gpurun_out/r06_a_$t.txt; exit 1; }
  echo "== $t"; cat gpurun_out/r06_a_$t.txt
done
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r06_a_bench.json 2> gpurun_out/r06_a_bench.err || { echo bench failed; tail -5 gpurun_out/r06_a_bench.err; exit 1; }
cat gpurun_out/r06_a_bench.json
timeout -k 10 500 bash tools/gpu_runs/gpu_r06_sq.sh 3 c3 > gpurun_out/r06_a_sq.log 2>&1 || { echo sq failed; tail -20 gpurun_out/r06_a_sq.log; exit 1; }
cat gpurun_out/r06_a_sq.log
