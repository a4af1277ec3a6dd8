#!/bin/bash
# Round 6: the round-5 generic-pointer failure on its own source (c2a5ce8 built unchanged: r05c; with the
# round-5 final lip_eq_res: r05cfix; with the polish diagnostics outputs: r05ceq).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in r05c r05cfix r05ceq; do
  timeout -k 10 240 python3 -u tools/flat_polish_diag.py libsrbnmpc_$t.so > gpurun_out/r06_b_$t.txt 2>&1 || { echo "diag $t failed"; tail -5 gpurun_out/r06_b_$t.txt; exit 1; }
  echo "== $t"; cat gpurun_out/r06_b_$t.txt
done
timeout -k 10 60 ./tools/ubench/flat_lds_order > gpurun_out/r06_b_flat_lds_order.txt 2>&1 || { echo "ubench failed"; cat gpurun_out/r06_b_flat_lds_order.txt; exit 1; }
cat gpurun_out/r06_b_flat_lds_order.txt
