#!/bin/bash
# Round 6: calls k and l in one box session (the pool was short of boxes)
set -o pipefail
bash tools/gpu_runs/gpu_r06_k.sh && bash tools/gpu_runs/gpu_r06_l.sh
