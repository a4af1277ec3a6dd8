#!/bin/bash
# Round 6: the SRB-12 accuracy floor (tol_final 1e-9 / 1e-10 on the product and three variants), fp32 storage of the
# term rows and reduced matrix (r32), the LDS-bounds build over every instance family, the guard's slipping agents,
# the low-level kernel's rocprof stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in "" _s12ref2 _s12rsq _s12both; do
  timeout -k 10 300 python3 -u tools/srb12_tolfinal.py libsrbnmpc$t.so > gpurun_out/r06_k_tolfinal$t.txt 2>&1 || { echo "tolfinal $t failed"; tail gpurun_out/r06_k_tolfinal$t.txt; exit 1; }
  cat gpurun_out/r06_k_tolfinal$t.txt | grep -v amdgpu.ids
done
timeout -k 10 300 python3 -u tools/round32_check.py libsrbnmpc_r32.so > gpurun_out/r06_k_r32.txt 2>&1 || { echo "r32 failed"; tail gpurun_out/r06_k_r32.txt; exit 1; }
cat gpurun_out/r06_k_r32.txt | grep -v amdgpu.ids
timeout -k 10 300 python3 -u tools/lds_check_scan.py libsrbnmpc_ldsck.so > gpurun_out/r06_k_ldsck.txt 2>&1; rc=$?
cat gpurun_out/r06_k_ldsck.txt | grep -v amdgpu.ids
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python3 -u tools/stationarity_guard_check.py libsrbnmpc_corrupt.so > gpurun_out/r06_k_corrupt.txt 2>&1 || { echo "guard failed"; exit 1; }
cat gpurun_out/r06_k_corrupt.txt | grep -v amdgpu.ids
rm -rf gpurun_out/r06_ll_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_ll_prof -o run --output-format csv -- python3 bench.py --path ll --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06_k_ll_bench.json 2> gpurun_out/r06_k_ll_bench.err || { echo "ll prof failed"; tail gpurun_out/r06_k_ll_bench.err; exit 1; }
cat gpurun_out/r06_k_ll_bench.json
