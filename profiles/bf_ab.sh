#!/bin/bash
# configs[4] (scaled 2 M / 8 M, bf16 storage): U = 16 vs 8 neighbour rows in flight in the bf16
# one-pass gathers (GNNMP_BF_U), alternating, then kernel stats of the default.
export TMPDIR=/tmp; OUT=gpurun_out/${1:-rXX}; mkdir -p $OUT
for rep in 1 2; do for u in 16 8; do
  GNNMP_BF_U=$u timeout -k 10 400 python bench.py --arch sage_scaled --no-cpu-baseline --no-roofline > $OUT/bf_u${u}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/bf_u${u}_$rep.json')); print('U=$u rep $rep', round(d['ms_per_step'],4))"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --arch sage_scaled --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $OUT/kt.log 2>&1 || exit 1
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/kernel_stats.csv')))[:14]: print('%9.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:100]))"
