#!/bin/bash
# Round 6: the round-5 failing build under run-time options only (tools/flat_polish_ab.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/flat_polish_ab.py > gpurun_out/r06_c_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/r06_c_ab.txt; exit 1; }
cat gpurun_out/r06_c_ab.txt
