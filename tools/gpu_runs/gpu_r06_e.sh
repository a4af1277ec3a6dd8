#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/flat_lds_order > gpurun_out/r06_e_flat_lds_order.txt 2>&1 || { echo "ubench failed"; cat gpurun_out/r06_e_flat_lds_order.txt; exit 1; }
cat gpurun_out/r06_e_flat_lds_order.txt
