#!/bin/bash
# SRB-12 A/B: the product build against variant builds (bench lines, SRB-12 GPU tests), then the
# per-phase stamps of the product's stamps build and of variant stamps builds.
#   usage: tools/gpu_r04_pf.sh <tag> "<stamps libs>" <lib> [<lib> ...]
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out; T=$1; ST=$2; shift 2
bash tools/gpu_r04_s12multi.sh $T "$@" || exit $?
for lib in libsrbnmpc_s12st.so $ST; do
  SRBNMPC_LIB=$lib timeout -k 10 120 python tools/srb12_stamps.py 0 24 > $O/r04_s12_stamps_${T}_$lib.txt 2>&1 || exit 1
  echo "== $lib"; head -18 $O/r04_s12_stamps_${T}_$lib.txt
done
