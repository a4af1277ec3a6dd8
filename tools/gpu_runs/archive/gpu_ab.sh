#!/bin/bash
# A/B timing of alternative builds (srbnmpc/libsrbnmpc*.so named on the command line):
# quick oracle check, bench configs 2 / 3 / 5 and (if built) stamps, per library.
#   usage: tools/gpu_runs/gpu_ab.sh libsrbnmpc.so libsrbnmpc_b.so ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "$@"; do
  echo "=== $L"
  timeout -k 10 100 python tools/quick_nw.py $L > gpurun_out/ab_quick_$L.log 2>&1 || { tail -5 gpurun_out/ab_quick_$L.log; exit 1; }
  grep -c "status ok True" gpurun_out/ab_quick_$L.log
  for c in 2 3 5; do
    SRBNMPC_LIB=$L timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 30 > gpurun_out/ab_${L}_c$c.json 2> gpurun_out/ab_c$c.err || { tail -5 gpurun_out/ab_c$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${L}_c$c.json'));r=d['roofline'];print($c, round(d['value']), 'solves/s kernel', round(r['kernel_ms'],4), 'knn', round(r['knn_ms'],4), 'iters', [round(v,2) for v in d['iters_mean']], 'opt', d['optimal_frac'], 'cyc/it', round(r['cycles_per_iter']))"
  done
done
