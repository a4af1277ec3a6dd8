#!/bin/bash
# SQ counters of the solve kernel at configs[2]: where a wave's cycles go, instruction
# fetch included.  One rocprofv3 --pmc pass per group (at most 8 SQ counters a pass), kernel trace only.
#   usage: tools/gpu_runs/gpu_r06_sq.sh [config] [tag]     -> gpurun_out/r06_sq_<tag>.txt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
c=${1:-3}
tag=${2:-c$c}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_MFMA SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_INPUT_VALID_READYB" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1)); rm -rf gpurun_out/r06sq_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp -d gpurun_out/r06sq_$i -o run --output-format csv -- \
      python3 bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r06sq_$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 gpurun_out/r06sq_$i.log; exit 1; }
done
python3 - "$tag" <<'PY'
import csv, glob, statistics, sys
rows = {}
for d in sorted(glob.glob("gpurun_out/r06sq_*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs: continue
    per = {}
    for r in csv.DictReader(open(fs[0])):
        if "srb_nmpc_kernel" in r["Kernel_Name"]:
            per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            rows["kernel"] = r["Kernel_Name"]
    for k, v in per.items():
        rows[k] = statistics.median(list(v.values()))
w = rows.get("SQ_WAVES", 1.0) or 1.0
with open(f"gpurun_out/r06_sq_{sys.argv[1]}.txt", "w") as f:
    f.write(f"kernel {rows.pop('kernel', '?')}; median over dispatches, summed over XCDs; per wave = / SQ_WAVES\n")
    for k in sorted(rows):
        f.write(f"  {k:32s} {rows[k]:16.0f}   per wave {rows[k] / w:12.1f}\n")
print(open(f"gpurun_out/r06_sq_{sys.argv[1]}.txt").read())
PY
