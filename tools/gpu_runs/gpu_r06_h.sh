#!/bin/bash
# Round 6: stationarity of the accepted polishes (stdiag), the guard against the round-5 defect class
# (corrupt / corruptns), the LDS-bounds build over every instance family (ldsck), configs[2] stamps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/stationarity_scan.py libsrbnmpc_stdiag.so > gpurun_out/r06_h_stscan.txt 2>&1 || { echo "stscan failed"; tail gpurun_out/r06_h_stscan.txt; exit 1; }
cat gpurun_out/r06_h_stscan.txt
for t in corrupt corruptns; do
  timeout -k 10 200 python3 -u tools/stationarity_guard_check.py libsrbnmpc_$t.so > gpurun_out/r06_h_$t.txt 2>&1 || { echo "guard $t failed"; tail gpurun_out/r06_h_$t.txt; exit 1; }
  cat gpurun_out/r06_h_$t.txt
done
timeout -k 10 300 python3 -u tools/lds_check_scan.py libsrbnmpc_ldsck.so > gpurun_out/r06_h_ldsck.txt 2>&1; rc=$?
cat gpurun_out/r06_h_ldsck.txt
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python3 -u tools/stamps.py 10 2 3 8 1024 > gpurun_out/r06_h_c3_stamps.txt 2>&1 || { echo "stamps failed"; tail gpurun_out/r06_h_c3_stamps.txt; exit 1; }
cat gpurun_out/r06_h_c3_stamps.txt
