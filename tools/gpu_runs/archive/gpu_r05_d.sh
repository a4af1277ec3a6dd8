#!/bin/bash
# LIP equality residuals by status (the polish's new equality test), and the SRB-12 polish state checks of
# agent 100 of the 1024-agent stand batch (GPU polish rejected, oracle accepted)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u tools/lip_eq_check.py > $O/r05_d_lipeq.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/r05_d_lipeq.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/srb12_check.py --lib libsrbnmpc_chk.so --N 10 --agents 1024 --gait stand --seed 21 --agent 100 > $O/r05_d_chk100.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/r05_d_chk100.txt | grep -v "^\s*\[ *[0-9]*\] gpu\|^\s*orc" | head -60
exit $rc
