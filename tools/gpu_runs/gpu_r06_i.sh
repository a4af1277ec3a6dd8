#!/bin/bash
# Round 6: kernel stationarity distribution (stdiag), the guard on the corrupted build, the GPU suite and smoke,
# the bench lines, and the fp32-factor option (tools/kkt32_check.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/stationarity_scan.py libsrbnmpc_stdiag.so > gpurun_out/r06_i_stscan.txt 2>&1 || { echo "stscan failed"; tail gpurun_out/r06_i_stscan.txt; exit 1; }
cat gpurun_out/r06_i_stscan.txt
timeout -k 10 200 python3 -u tools/stationarity_guard_check.py libsrbnmpc_corrupt.so > gpurun_out/r06_i_corrupt.txt 2>&1 || { echo "guard failed"; tail gpurun_out/r06_i_corrupt.txt; exit 1; }
cat gpurun_out/r06_i_corrupt.txt
bash tools/gpu_runs/gpu_r06_suite.sh i || exit 1
bash tools/gpu_runs/gpu_r06_bench.sh i --no-cpu-baseline || exit 1
timeout -k 10 400 python3 -u tools/kkt32_check.py > gpurun_out/r06_i_kkt32.txt 2>&1 || { echo "kkt32 failed"; tail gpurun_out/r06_i_kkt32.txt; exit 1; }
cat gpurun_out/r06_i_kkt32.txt
