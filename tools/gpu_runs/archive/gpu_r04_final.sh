#!/bin/bash
# Round-4 closing run: the whole GPU suite, smoke and bench lines (gpu_r04_full.sh), then the profiles
# (gpu_r04_prof.sh).   usage: tools/gpu_r04_final.sh <tag>
set -o pipefail
bash tools/gpu_r04_full.sh "$1" && bash tools/gpu_r04_prof.sh
