set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/dump_gpu.py 3 gpurun_out/c3_split.npz && \
SRBNMPC_LIB=libsrbnmpc_gj0.so timeout -k 10 120 python tools/dump_gpu.py 3 gpurun_out/c3_gj0.npz && \
timeout -k 10 120 python tools/dump_gpu.py 2 gpurun_out/c2_split.npz && \
SRBNMPC_LIB=libsrbnmpc_gj0.so timeout -k 10 120 python tools/dump_gpu.py 2 gpurun_out/c2_gj0.npz && \
python -c "
import numpy as np
for c in ('c3','c2'):
    a=np.load('gpurun_out/%s_split.npz'%c); b=np.load('gpurun_out/%s_gj0.npz'%c)
    print(c, {k: bool(np.array_equal(a[k],b[k])) for k in a.files})
" && \
bash tools/gpu_runs/gpu_waves.sh 3 libsrbnmpc.so:1 libsrbnmpc_gj0.so:1 libsrbnmpc.so:1 libsrbnmpc_gj0.so:1 && \
bash tools/gpu_runs/gpu_waves.sh 2 libsrbnmpc.so:4 libsrbnmpc_gj0.so:4 && \
bash tools/gpu_runs/gpu_waves.sh 5 libsrbnmpc.so:2 libsrbnmpc_gj0.so:2 && \
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_split.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_split.log; exit $rc
