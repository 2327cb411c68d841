#!/bin/bash
# A/B of where the half-pair NT's B prep runs: inside K1's launch (default), inside the NT call,
# on a side stream; then rocprof kernel stats of the default.
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_k1prep.log" 2>&1 || { tail -5 "$OUT/bench_k1prep.log"; exit 1; }
GNNMP_K1_PREP=0 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_ntprep.log" 2>&1 || exit 1

for f in k1prep ntprep; do python3 -c "
import json; d=json.loads(open('$OUT/bench_$f.log').read().strip().splitlines()[-1])
t=d['roofline']['timed_kernels']; print('$f', round(d['ms_per_step'],4), d['roofline']['frac'], {k: v['us_per_launch'] for k,v in t.items()})"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt.log" 2>&1
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    if 'gnnmp' in r['Name'] and int(r['Calls']) > 5: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1000,1))"
