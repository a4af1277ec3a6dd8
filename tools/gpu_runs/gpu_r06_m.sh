#!/bin/bash
# Round 6, call m: GPU suite + smoke + bench lines of the build with the SRB-12 second refinement
set -o pipefail
bash tools/gpu_runs/gpu_r06_suite.sh m && bash tools/gpu_runs/gpu_r06_bench.sh m --no-cpu-baseline
