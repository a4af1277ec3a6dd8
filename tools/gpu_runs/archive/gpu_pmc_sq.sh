#!/bin/bash
# SQ counters of the solve kernel (one rocprofv3 --pmc pass per counter group, kernel trace
# only): where a wave's cycles go at configs[2].   usage: tools/gpu_runs/gpu_pmc_sq.sh [config]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
c=${1:-3}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_ANY" \
           "SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1)); rm -rf gpurun_out/sq_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/sq_$i -o run --output-format csv -- \
      python3 bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/sq_$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 gpurun_out/sq_$i.log; continue; }
done
python - <<'PY'
import csv, glob, statistics
for d in sorted(glob.glob("gpurun_out/sq_*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs: continue
    per = {}
    for r in csv.DictReader(open(fs[0])):
        if "srb_nmpc_kernel" in r["Kernel_Name"]:
            per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in per.items():
        print(f"{k:28s} {statistics.median(list(v.values())):16.0f}")
PY
