set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline > $O/ab5_w2.json 2> $O/ab5_w2.err || { tail $O/ab5_w2.err; exit 1; }
timeout -k 10 200 python bench.py --config 5 --no-cpu-baseline --waves 4 > $O/ab5_w4.json 2> $O/ab5_w4.err || { tail $O/ab5_w4.err; exit 1; }
cat $O/ab5_w2.json $O/ab5_w4.json
