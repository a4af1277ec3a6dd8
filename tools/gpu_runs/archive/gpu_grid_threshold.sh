set -o pipefail
for m in 8192 4096 1000; do
  SRB_GRID_MIN_ROWS=$m timeout -k 10 120 python bench.py --config 3 --no-cpu-baseline --steps 30 > gpurun_out/gm_$m.json 2> gpurun_out/gm.err || { tail -3 gpurun_out/gm.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/gm_$m.json'));r=d['roofline'];print($m, round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'knn_ms', round(r['knn_ms'],4), 'kernel', round(r['kernel_ms'],4), 'opt', d['optimal_frac'])"
done
