#!/bin/bash
# Selection-kernel changes: the selection / grid / shard parity tests, then the selection time
# at configs[2] and on rank 0's shard of an emulated 8-GPU configs[3] swarm.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle all || exit 1
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "knn or sharded or device_api or sentinel" > gpurun_out/pt_knn.log 2>&1; rc=$?
tail -2 gpurun_out/pt_knn.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pt_knn.log | head; exit 1; }
timeout -k 10 120 python bench.py --config 3 --no-cpu-baseline --steps 30 > gpurun_out/kc3.json 2> gpurun_out/kc.err || { tail -3 gpurun_out/kc.err; exit 1; }
timeout -k 10 120 python bench.py --config 4 --emulate-shards 8 --no-cpu-baseline --steps 20 > gpurun_out/kc4.json 2>> gpurun_out/kc.err || { tail -3 gpurun_out/kc.err; exit 1; }
for f in kc3 kc4; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));r=d['roofline'];print('$f', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'knn_ms', round(r['knn_ms'],4), 'kernel', round(r['kernel_ms'],4), 'opt', d['optimal_frac'])"; done
