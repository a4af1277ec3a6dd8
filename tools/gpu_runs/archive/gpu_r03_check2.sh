#!/bin/bash
# Round-3 re-check after a kernel change: GPU suite, smoke, bench lines of configs 3 / 5 / 2 and the
# SRB-12 path, and the FETCH / WRITE passes of configs[2] (scratch traffic).  Chained, time-limited.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in 3 5 2; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 30 > $O/chk_c$c.json 2> $O/chk.err || { tail $O/chk.err; exit 1; }
done
timeout -k 10 200 python bench.py --path srb12 --no-cpu-baseline --steps 20 > $O/chk_s12.json 2> $O/chk.err || { tail $O/chk.err; exit 1; }
for f in c3 c5 c2 s12; do python -c "import json;d=json.load(open('$O/chk_$f.json'));r=d['roofline'];print('$f', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'polish', r.get('polish_ms'), 'opt', d['optimal_frac'], 'iters', d['iters_mean'], d.get('iters_max'))"; done
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/pmc2_c3_$ctr
  timeout -s KILL 150 rocprofv3 --pmc $ctr -d $O/pmc2_c3_$ctr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/pmc2_c3_$ctr.log 2>&1 || { tail -5 $O/pmc2_c3_$ctr.log; exit 1; }
done
python tools/pmc_traffic.py $O/pmc2_c3_FETCH_SIZE $O/pmc2_c3_WRITE_SIZE 3 1024 $O/r03_pmc_traffic_c3_b.json profiles/r03_pmc_calib.json > /dev/null || exit 1
python -c "import json;d=json.load(open('$O/r03_pmc_traffic_c3_b.json'));print({k:round(v['hbm_bytes']/1e6,3) for k,v in d['kernels'].items()})"
