#!/bin/bash
# Round 6: product bench lines (configs[2] default, config 5 = configs[4] shape, configs[1], SRB-12)
#   usage: tools/gpu_runs/gpu_r06_bench.sh <tag> [extra bench.py args]
set -o pipefail
mkdir -p gpurun_out
t=${1:-x}; shift
for c in 3 5 2; do
  timeout -k 10 200 python3 -u bench.py --config $c --steps 50 --warmup 10 "$@" > gpurun_out/r06_${t}_bench_c$c.json 2> gpurun_out/r06_${t}_bench_c$c.err || { echo "bench c$c failed"; tail -5 gpurun_out/r06_${t}_bench_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r06_${t}_bench_c$c.json')); print('c$c', round(d['ms_per_step'],4), 'ms p99', round(d['p99_ms'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'opt', d['optimal_frac'], 'iters', d['iters_mean'], d['iters_max'])"
done
timeout -k 10 200 python3 -u bench.py --path srb12 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r06_${t}_bench_srb12.json 2> gpurun_out/r06_${t}_bench_srb12.err || { echo "bench srb12 failed"; tail -5 gpurun_out/r06_${t}_bench_srb12.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06_${t}_bench_srb12.json')); print('srb12', round(d['ms_per_step'],4), 'ms p99', round(d['p99_ms'],4), 'opt', d['optimal_frac'])"
