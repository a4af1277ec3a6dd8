#!/bin/bash
# the LIP K = 3 + 0 polish rejections with the equality test on / disabled (SRB_POLISH_EQTOL = 1e300) / compiled
# out (SRB_POLISH_EQCHECK = 0); then the SRB-12 GPU tests (polish convergence rule on |c_A|)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for lib in libsrbnmpc.so libsrbnmpc_eqoff.so libsrbnmpc_eqnone.so; do
  echo "== $lib"
  timeout -k 10 300 python -u tools/lip_eq_check.py --lib $lib > $O/r05_f_lipeq_$lib.txt 2>&1 || { tail $O/r05_f_lipeq_$lib.txt; exit 1; }
  grep -v amdgpu.ids $O/r05_f_lipeq_$lib.txt
done
timeout -k 10 600 python -u -m pytest tests/test_srb12.py -m gpu -q --timeout 300 --timeout-method thread > $O/r05_f_s12tests.log 2>&1; rc=$?
tail -4 $O/r05_f_s12tests.log
exit $rc
