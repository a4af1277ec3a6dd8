set -o pipefail
mkdir -p gpurun_out
for c in 3 5; do for nw in 1 2 4; do
  SRB_NMPC_NW=$nw timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 20 > gpurun_out/t.json 2>/dev/null || { echo fail $c $nw; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/t.json'));print($c,$nw,round(d['value']),round(d['roofline']['kernel_ms'],3),d['optimal_frac'])"
done; done
for nw in 2 4; do
  SRB_NMPC_NW=$nw timeout -k 10 120 python bench.py --config 2 --no-cpu-baseline --steps 50 > gpurun_out/t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/t.json'));print(2,$nw,round(d['value']),round(d['roofline']['kernel_ms'],4),d['optimal_frac'])"
done
