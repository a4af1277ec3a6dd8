set -o pipefail
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "knn or hl_planner or sharded or device_api" > gpurun_out/pytest_grid.log 2>&1; tail -3 gpurun_out/pytest_grid.log
for e in 8; do
  timeout -k 10 120 python bench.py --config 4 --emulate-shards $e --no-cpu-baseline --steps 20 > gpurun_out/emu_grid.json 2>gpurun_out/emu.err || { tail -3 gpurun_out/emu.err; exit 1; }
  SRB_GRID_MIN_ROWS=100000000 timeout -k 10 120 python bench.py --config 4 --emulate-shards $e --no-cpu-baseline --steps 20 > gpurun_out/emu_brute.json 2>>gpurun_out/emu.err || exit 1
  for f in emu_grid emu_brute; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));r=d['roofline'];c=d['config'];print('$f', c['emulated_shards'], c['n_obs'], c['nbr_rows'], round(d['value']), 'knn_ms', round(r['knn_ms'],4), 'kernel', round(r['kernel_ms'],4), 'opt', d['optimal_frac'])"; done
done
timeout -k 10 300 python tools/bench_hlplan.py --agents 1024,4096 --loop 4000 --cpu-seconds 4
