#!/bin/bash
# A/B of the staged obstacle-row relinearisation (product) and the two-chain Gram
# (libsrbnmpc_gc2.so) against the previous product (libsrbnmpc_base.so): bit-identity,
# parity of the variant, bench times, then the GPU test suite on the product.
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
bash tools/gpu_runs/gpu_waves.sh 3 libsrbnmpc_base.so:1 libsrbnmpc.so:1 libsrbnmpc_gc2.so:1 libsrbnmpc_base.so:1 libsrbnmpc.so:1 libsrbnmpc_gc2.so:1 || exit 1
bash tools/gpu_runs/gpu_waves.sh 2 libsrbnmpc_base.so:4 libsrbnmpc.so:4 libsrbnmpc_gc2.so:4 || exit 1
bash tools/gpu_runs/gpu_waves.sh 5 libsrbnmpc_base.so:2 libsrbnmpc.so:2 libsrbnmpc_gc2.so:2 || exit 1
timeout -k 10 200 python tools/quick_nw.py libsrbnmpc_gc2.so || exit 1
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_relin.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_relin.log; exit $rc
