#!/bin/bash
# Per-GPU compute of a strong-scaling run: the largest shard of the N-way partition on one GPU.
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for N in 1 2 4 8; do
  timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/shard_$N.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/shard_$N.json')); print('shard of $N:', d['config']['max_nodes_per_gpu'], 'nodes', d['config']['max_edges_per_gpu'], 'edges', round(d['ms_per_step'],4), 'ms/step')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt8 -o run --output-format csv -- python3 bench.py --rehearse-shard 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt8.log 2>&1 || exit $?
find $OUT/kt8 -name "*kernel_stats.csv" -exec cp {} $OUT/shard8_kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/shard8_kernel_stats.csv')))
for r in rows[:16]: print('%9.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:100]))"
