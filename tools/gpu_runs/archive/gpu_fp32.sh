#!/bin/bash
# fp32-KKT experiment (BASELINE configs[4] wording): product build vs the fp32-factor build
# (libsrbnmpc_fp32.so: reduced Newton matrix inverted in fp32, 3 fp64 refinement steps) on
# configs 3 and 5; statuses, iterations and max |X,U,s| error against the oracle.
set -o pipefail
mkdir -p gpurun_out
for L in libsrbnmpc.so libsrbnmpc_fp32.so; do
  for c in 3 5; do
    SRBNMPC_LIB=$L timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/fp_${L}_$c.json 2> gpurun_out/fp.err || { tail -3 gpurun_out/fp.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/fp_${L}_$c.json'));r=d['roofline'];print('$L', 'config $c', round(d['value']), 'solves/s kernel', round(r['kernel_ms'],4), 'iters', [round(v,2) for v in d['iters_mean']], 'opt', d['optimal_frac'], 'acc', d['acceptable_frac'])"
  done
  SRBNMPC_LIB=$L timeout -k 10 100 python tools/dump_gpu.py 5 gpurun_out/c5_$L.npz || exit 1
  SRBNMPC_LIB=$L timeout -k 10 100 python tools/dump_gpu.py 3 gpurun_out/c3_$L.npz || exit 1
done
