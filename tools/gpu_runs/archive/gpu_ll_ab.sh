#!/bin/bash
# A/B of low-level CLF-QP builds: bench --path ll and the PMC WRITE_SIZE pass per library.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in "$@"; do
  SRBNMPC_LIB=$L timeout -k 10 120 python bench.py --path ll --no-cpu-baseline --steps 20 > gpurun_out/ll_$L.json 2> gpurun_out/ll.err || { tail -3 gpurun_out/ll.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ll_$L.json'));r=d['roofline'];print('$L', round(d['value']), 'kernel_ms', round(r['kernel_ms'],4), 'iters', d['iters_mean'], 'opt', d['optimal_frac'])"
  for ctr in WRITE_SIZE FETCH_SIZE; do
    rm -rf gpurun_out/llpmc_$ctr
    SRBNMPC_LIB=$L timeout -k 10 120 rocprofv3 --pmc $ctr -d gpurun_out/llpmc_$ctr -o run --output-format csv -- python3 bench.py --path ll --no-cpu-baseline --steps 5 > gpurun_out/llpmc.log 2>&1 || { tail -3 gpurun_out/llpmc.log; exit 1; }
  done
  python tools/pmc_traffic.py gpurun_out/llpmc_FETCH_SIZE gpurun_out/llpmc_WRITE_SIZE ll 8192 gpurun_out/ll_pmc_$L.json srb_ll_kernel > /dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ll_pmc_$L.json'));print('$L', 'write KiB', d['write_kib_per_launch'], 'fetch KiB', d['fetch_kib_per_launch'])"
done
