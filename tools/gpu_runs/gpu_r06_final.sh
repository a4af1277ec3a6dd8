#!/bin/bash
# Round 6, final tree: GPU suite + smoke, the bench lines (the default one with its cpu_baseline), rocprofv3
# kernel statistics of configs[2] and config 5.  Every GPU step time-limited and chained.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
bash tools/gpu_runs/gpu_r06_suite.sh final || exit 1
timeout -k 10 300 python3 bench.py > $O/r06_final_bench_c3.json 2> $O/r06_final_bench_c3.err || { tail $O/r06_final_bench_c3.err; exit 1; }
for c in 5 2; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/r06_final_bench_c$c.json 2> $O/r06_final_bench_c$c.err || { tail $O/r06_final_bench_c$c.err; exit 1; }
done
timeout -k 10 200 python3 bench.py --path srb12 --no-cpu-baseline > $O/r06_final_bench_srb12.json 2> $O/r06_final_bench_srb12.err || { tail $O/r06_final_bench_srb12.err; exit 1; }
timeout -k 10 200 python3 bench.py --path ll --no-cpu-baseline > $O/r06_final_bench_ll.json 2> $O/r06_final_bench_ll.err || { tail $O/r06_final_bench_ll.err; exit 1; }
for c in 3 5; do
  rm -rf $O/prof_final_c$c
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_final_c$c -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 20 --config $c > $O/prof_final_c$c.log 2>&1 || { tail -5 $O/prof_final_c$c.log; exit 1; }
done
for f in c3 c5 c2 srb12 ll; do python3 -c "import json; d=json.load(open('$O/r06_final_bench_$f.json')); print('$f', d['value'], round(d['ms_per_step'],4), 'p99', round(d['p99_ms'],4), 'opt', d.get('optimal_frac'))"; done
grep -h "srb_nmpc\|srb_knn" $O/prof_final_c3/run_kernel_stats.csv $O/prof_final_c5/run_kernel_stats.csv | cut -d, -f1-4
echo "final script done"
