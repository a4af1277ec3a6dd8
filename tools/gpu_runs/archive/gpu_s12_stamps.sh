#!/bin/bash
# SRB-12: GPU tests on the product library, then per-phase stamps of three agents (stamps build).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03_pytest_srb12.log 2>&1 || { tail -20 $O/r03_pytest_srb12.log; exit 1; }
tail -1 $O/r03_pytest_srb12.log
SRBNMPC_LIB=libsrbnmpc_s12st.so timeout -k 10 200 python tools/srb12_stamps.py 0 24 31 > $O/r03_s12_stamps.txt 2>&1 || { tail -20 $O/r03_s12_stamps.txt; exit 1; }
cat $O/r03_s12_stamps.txt
