#!/bin/bash
# round-4 SRB-12 kernel rebuilt with the current host objects: the no-waves_per_eu variant that failed
# the N = 20 test, the same with the polish state checks, and the round-4 product; then the traces of the
# 1024-agent stand batch's non-OPTIMAL agents (product build)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
for lib in libsrbnmpc_r04.so libsrbnmpc_r04nowpe.so libsrbnmpc_r04chknowpe.so; do
  echo "=== $lib"
  timeout -k 10 240 python -u tools/srb12_check.py --lib $lib > $O/r05_chk_b_$lib.txt 2>&1; rc=$?
  grep -v amdgpu.ids $O/r05_chk_b_$lib.txt
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u tools/srb12_trace.py stand 21 1024 auto > $O/r05_trace_stand21.txt 2>&1; rc=$?
head -c 20000 $O/r05_trace_stand21.txt | grep -v amdgpu.ids | head -150
exit $rc
