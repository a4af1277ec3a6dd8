#!/bin/bash
# A/B of the product library against libsrbnmpc_base.so (the previous product, built from the
# previous commit's sources): bit-identity on configs[2] / configs[1] batches, bench times on
# configs[2], configs[1] and N = 20, then the GPU test suite on the product.
set -o pipefail
mkdir -p gpurun_out
for c in 3 2; do
  for L in libsrbnmpc.so libsrbnmpc_base.so; do
    SRBNMPC_LIB=$L timeout -k 10 120 python tools/dump_gpu.py $c gpurun_out/c${c}_$L.npz || exit 1
  done
done
python -c "
import numpy as np
for c in ('3','2'):
    a=np.load('gpurun_out/c%s_libsrbnmpc.so.npz'%c); b=np.load('gpurun_out/c%s_libsrbnmpc_base.so.npz'%c)
    print('cfg',c,'product vs base bit-identical:', {k: bool(np.array_equal(a[k],b[k])) for k in a.files})
" || exit 1
bash tools/gpu_runs/gpu_waves.sh 3 libsrbnmpc_base.so:1 libsrbnmpc.so:1 libsrbnmpc_base.so:1 libsrbnmpc.so:1 || exit 1
bash tools/gpu_runs/gpu_waves.sh 2 libsrbnmpc_base.so:4 libsrbnmpc.so:4 || exit 1
bash tools/gpu_runs/gpu_waves.sh 5 libsrbnmpc_base.so:2 libsrbnmpc.so:2 || exit 1
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ab.log; exit $rc
