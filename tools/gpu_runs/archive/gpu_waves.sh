#!/bin/bash
# Bench one config across builds x waves per agent:  tools/gpu_runs/gpu_waves.sh <config> lib:nw [lib:nw ...]
set -o pipefail
mkdir -p gpurun_out
c=$1; shift
for spec in "$@"; do
  L=${spec%%:*}; W=${spec##*:}
  SRBNMPC_LIB=$L timeout -k 10 120 python bench.py --config $c --waves $W --no-cpu-baseline --steps 30 > gpurun_out/w.json 2> gpurun_out/w.err || { tail -5 gpurun_out/w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/w.json'));r=d['roofline'];print('$L', 'cfg $c nw', r['waves_per_agent'], round(d['value']), 'solves/s kernel', round(r['kernel_ms'],4), 'opt', d['optimal_frac'], 'cyc/it', round(r['cycles_per_iter']))"
done
