#!/bin/bash
# Phase stamps (tools/stamps.py) of several stamps builds on one config.
#   usage: tools/gpu_runs/gpu_stamps_ab.sh "N C Ko Kn A" libsrbnmpc_stX.so ...
set -o pipefail
mkdir -p gpurun_out
cfg=$1; shift
for L in "$@"; do
  SRB_STAMPS_LIB=$L timeout -k 10 120 python tools/stamps.py $cfg > gpurun_out/stab_$L.txt 2>&1 || { tail -5 gpurun_out/stab_$L.txt; exit 1; }
done
python - "$@" <<'PY'
import sys, re
rows = {}
for L in sys.argv[1:]:
    stage = None
    for line in open(f"gpurun_out/stab_{L}.txt"):
        if line.startswith("QP") or line.startswith("NLP"):
            stage = line.split(":")[0]; rows.setdefault((stage, "per iteration"), {})[L] = line.split()[-1]
        m = re.match(r"\s+(.+?)\s{2,}(\d+) cyc\s+(\d+) /iter", line)
        if m and stage == "NLP":
            rows.setdefault((stage, m.group(1)), {})[L] = m.group(3)
print("phase".ljust(22), " ".join(L[-10:].rjust(10) for L in sys.argv[1:]))
for (st, nm), d in rows.items():
    print(f"{st}:{nm}"[:22].ljust(22), " ".join(str(d.get(L, "")).rjust(10) for L in sys.argv[1:]))
PY
