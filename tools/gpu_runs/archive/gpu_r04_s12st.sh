#!/bin/bash
# SRB-12 per-phase stamps (make s12st) of bench agents 0, 24, 31.   usage: tools/gpu_r04_s12st.sh <tag>
set -o pipefail
mkdir -p gpurun_out
SRBNMPC_LIB=libsrbnmpc_s12st.so timeout -k 10 120 python tools/srb12_stamps.py 0 24 31 > gpurun_out/r04_s12_stamps_$1.txt 2>&1 || { tail -20 gpurun_out/r04_s12_stamps_$1.txt; exit 1; }
cat gpurun_out/r04_s12_stamps_$1.txt
