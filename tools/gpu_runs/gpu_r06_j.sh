#!/bin/bash
# Round 6: the completed KKT guard (stationarity distance + multiplier signs) on the corrupted build and its
# distribution on the product shapes; the GPU suite; bench lines; the selection split timing
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/stationarity_guard_check.py libsrbnmpc_corrupt.so > gpurun_out/r06_j_corrupt.txt 2>&1 || { echo "guard failed"; tail gpurun_out/r06_j_corrupt.txt; exit 1; }
cat gpurun_out/r06_j_corrupt.txt
timeout -k 10 200 python3 -u tools/stationarity_scan.py libsrbnmpc_stdiag.so > gpurun_out/r06_j_stscan.txt 2>&1 || { echo "stscan failed"; tail gpurun_out/r06_j_stscan.txt; exit 1; }
cat gpurun_out/r06_j_stscan.txt
bash tools/gpu_runs/gpu_r06_suite.sh j || exit 1
bash tools/gpu_runs/gpu_r06_bench.sh j --no-cpu-baseline || exit 1
timeout -k 10 120 python3 -u tools/knn_split_timing.py > gpurun_out/r06_j_knn_split.txt 2>&1 || { echo "knn split failed"; tail gpurun_out/r06_j_knn_split.txt; exit 1; }
cat gpurun_out/r06_j_knn_split.txt
