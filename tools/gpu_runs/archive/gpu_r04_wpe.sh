#!/bin/bash
set -o pipefail
bash tools/gpu_r04_s12multi.sh w libsrbnmpc_s12nowpe.so && bash tools/gpu_r04_c3ab.sh w libsrbnmpc_lipwpe.so
