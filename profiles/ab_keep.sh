#!/bin/bash
# A/B of the half-pair NT's dropout: K1's keep bits vs the NT's own hash; then rocprof kernel stats
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
GNNMP_KEEP_MASK=1 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_mask.log" 2>&1 || { tail -5 "$OUT/bench_mask.log"; exit 1; }
GNNMP_KEEP_MASK=0 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_hash.log" 2>&1 || { tail -5 "$OUT/bench_hash.log"; exit 1; }
GNNMP_H2=0 timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_bf16planes.log" 2>&1 || { tail -5 "$OUT/bench_bf16planes.log"; exit 1; }
for f in mask hash bf16planes; do python3 -c "
import json,sys; d=json.loads(open('$OUT/bench_$f.log').read().strip().splitlines()[-1])
t=d['roofline']['timed_kernels']; print('$f', round(d['ms_per_step'],4), {k: v['us_per_launch'] for k,v in t.items()})"; done
GNNMP_KEEP_MASK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt.log" 2>&1
find "$OUT/kt" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;

GNNMP_KEEP_MASK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_hash" -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt_hash.log" 2>&1
find "$OUT/kt_hash" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_hash.csv" \;
for f in kernel_stats kernel_stats_hash; do python3 -c "
import csv
for r in csv.DictReader(open('$OUT/$f.csv')):
    if 'gnnmp' in r['Name']: print('$f', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))"; done
