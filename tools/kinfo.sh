#!/bin/bash
# Per-kernel code size, VGPR/AGPR counts and spills of the built product library.
set -e
LIB=${1:-/root/repo/srb-cbf-nmpc_amd/srbnmpc/libsrbnmpc.so}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin $LIB
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf -s $T/k.co | grep FUNC | sort -u -k8 | awk '{print $8, "bytes", $3}'
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | grep -E "^ +(- )?\.(name|vgpr_count|agpr_count|sgpr_spill_count|vgpr_spill_count|private_segment_fixed_size):" | sed 's/^ *- //;s/^ *//' | awk '{printf "%s %s  ", $1, $2} /vgpr_spill_count/ {print ""}'
cp $T/k.co /tmp/k.co
rm -rf $T
