#!/bin/bash
# Polish regularisation scan at config 5 (tuning aid): polish_probe.py under SRB_POLISH_RHO.
set -o pipefail
mkdir -p gpurun_out
for r in ${RHOS:-1e6 1e7 1e9 1e10}; do SRB_POLISH_RHO=$r timeout -k 10 120 python tools/polish_probe.py 5 || exit 1; done
