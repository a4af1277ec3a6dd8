#!/bin/bash
# Selection time of alternative builds (srbnmpc/libsrbnmpc*.so named on the command line),
# twice each, interleaved: configs[2] and the emulated 8-GPU shard.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for L in "$@"; do
  for c in "3" "4 --emulate-shards 8"; do
    SRBNMPC_LIB=$L timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 30 > gpurun_out/kab.json 2> gpurun_out/kab.err || { tail -3 gpurun_out/kab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/kab.json'));r=d['roofline'];print('$L', '$c'[:1], round(d['value']), 'knn_us', round(1000*r['knn_ms'],1), 'kernel', round(r['kernel_ms'],4))"
  done
done
done
