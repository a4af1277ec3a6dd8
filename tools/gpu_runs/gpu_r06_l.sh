#!/bin/bash
# Round 6, call l: the round-4 N = 20 whole-shape failure -- the round-4 package built as
# shipped (r04ab: 24_4_2_0_2_11) and with the whole shape (r04abw: 24_4_2_20_2_11), polish on and off, compared;
# then the LDS-check build (with the Z'Z / obstacle-position assertion, bit 7) over every instance family.
# Every GPU step time-limited; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u tools/r04_n20_run.py r04ab base > $O/r06_l_r04base.txt 2>&1 || { tail -20 $O/r06_l_r04base.txt; exit 1; }
timeout -k 10 300 python -u tools/r04_n20_run.py r04abw whole > $O/r06_l_r04whole.txt 2>&1 || { tail -20 $O/r06_l_r04whole.txt; exit 1; }
python tools/r04_n20_compare.py $O/r06_r04n20_base.npz $O/r06_r04n20_whole.npz > $O/r06_l_r04cmp.txt 2>&1 || { tail -20 $O/r06_l_r04cmp.txt; exit 1; }
cat $O/r06_l_r04base.txt $O/r06_l_r04whole.txt $O/r06_l_r04cmp.txt
timeout -k 10 400 python -u tools/lds_check_scan.py libsrbnmpc_ldsck.so > $O/r06_l_ldsck.txt 2>&1 || { tail -20 $O/r06_l_ldsck.txt; exit 1; }
tail -3 $O/r06_l_ldsck.txt
