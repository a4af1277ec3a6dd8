#!/bin/bash
# the LIP K = 3 + 0 polish rejections (test_knn_matches_bruteforce[3-0]): rejected agents, then their NLP and
# polish traces (nlpdbg build: per-pass equality residual, x after each Newton step); the SRB-12 agent 100
# polish state checks over four passes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u tools/lip_eq_check.py > $O/r05_e_lipeq.txt 2>&1 || { tail $O/r05_e_lipeq.txt; exit 1; }
grep -v amdgpu.ids $O/r05_e_lipeq.txt
AG=$(cat $O/r05_rej_agents.txt)
NLPTRACE_SPEC="10 2 3 0 512 3" timeout -k 10 300 python -u tools/nlp_trace.py custom $AG > $O/r05_e_nlptrace.txt 2>&1 || { tail $O/r05_e_nlptrace.txt; exit 1; }
grep -v amdgpu.ids $O/r05_e_nlptrace.txt | grep -v "^ *[0-9]* [ -][0-9]" | head -60
timeout -k 10 300 python -u tools/srb12_check.py --lib libsrbnmpc_chk.so --N 10 --agents 1024 --gait stand --seed 21 --agent 100 > $O/r05_e_chk100.txt 2>&1 || exit 1
grep -E "pass|end:|polish" $O/r05_e_chk100.txt | head -30
