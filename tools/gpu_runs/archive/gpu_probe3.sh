#!/bin/bash
# Timing probe (solve / polish kernel ms, statuses) of configs 5, 3, 2 with the product library.
set -o pipefail
mkdir -p gpurun_out
for c in 5 3 2; do timeout -k 10 120 python tools/polish_probe.py $c || exit 1; done
