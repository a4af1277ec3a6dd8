#!/bin/bash
# Round 6: rebuild the ROUND-4 package (commit b64117e) in two scratch trees for
# tools/r04_n20_run.py -- r04ab as shipped (N = 20 instance 24_4_2_0_2_11) and r04abw with the whole shape compiled
# (24_4_2_20_2_11, the round-4 failure).  Both directories are git-ignored scratch.
set -e
cd "$(dirname "$0")/.."
for d in r04ab r04abw; do
  rm -rf $d && mkdir -p $d && git archive b64117e srb-cbf-nmpc_amd include oracle | tar -x -C $d
done
sed -i 's/X(24, 4, 2, 0, 2, 11)/X(24, 4, 2, 20, 2, 11)/' r04abw/srb-cbf-nmpc_amd/csrc/srb_kernel_params.h
make -C r04ab/srb-cbf-nmpc_amd -j8
make -C r04abw/srb-cbf-nmpc_amd -j8
