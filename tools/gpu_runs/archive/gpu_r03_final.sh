#!/bin/bash
# End-of-round check of the committed tree: the whole GPU suite and smoke().  Time-limited, chained.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/r03_pytest_gpu_final.log 2>&1 || { tail -30 $O/r03_pytest_gpu_final.log; exit 1; }
tail -3 $O/r03_pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r03_smoke_final.log 2>&1 || { tail -20 $O/r03_smoke_final.log; exit 1; }
tail -2 $O/r03_smoke_final.log
