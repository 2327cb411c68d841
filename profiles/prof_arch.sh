#!/bin/bash
# Kernel stats of one --arch config: bash profiles/prof_arch.sh <arch> <tag>
ARCH=$1; OUT=gpurun_out/$2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --arch $ARCH --no-cpu-baseline --no-roofline > $OUT/bench.json 2>$OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --arch $ARCH --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/kernel_stats.csv')))
for r in rows[:40]: print('%9.1f us x%4s %8.1f us tot  %s' % (float(r['AverageNs'])/1e3, r['Calls'], float(r['TotalDurationNs'])/1e3, r['Name'][:110]))"
