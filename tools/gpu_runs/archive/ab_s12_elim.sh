#!/bin/bash
# SRB-12 forward elimination: readlane (product) vs DPP row broadcast (libsrbnmpc_s12dpp.so, -DSRB12_ELIM_DPP=1).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
SRBNMPC_LIB=libsrbnmpc_s12dpp.so timeout -k 10 300 python -u -m pytest tests/test_srb12.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ab_s12_dpp_tests.log 2>&1 || { tail -20 $O/ab_s12_dpp_tests.log; exit 1; }
tail -1 $O/ab_s12_dpp_tests.log
timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/ab_s12_rl.json 2> $O/ab_s12_rl.err || { tail $O/ab_s12_rl.err; exit 1; }
SRBNMPC_LIB=libsrbnmpc_s12dpp.so timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline > $O/ab_s12_dpp.json 2> $O/ab_s12_dpp.err || { tail $O/ab_s12_dpp.err; exit 1; }
cat $O/ab_s12_rl.json $O/ab_s12_dpp.json
