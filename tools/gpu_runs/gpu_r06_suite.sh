#!/bin/bash
# Round 6: the GPU suite (pytest -m gpu) on the product library, then smoke(); log per tag
#   usage: tools/gpu_runs/gpu_r06_suite.sh <tag>
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
t=${1:-x}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_${t}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r06_${t}_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r06_${t}_pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_${t}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06_${t}_smoke.log; exit 1; }
tail -1 gpurun_out/r06_${t}_smoke.log
