#!/bin/bash
# GCN F <= 2 on the slot-parallel narrow LDS kernel (tree's library) vs the 8-lane group kernel
# (ab_libs/libgnnmp_old.so): GCN tests on the new library, then same-box bench A/B
OUT=gpurun_out/${1:-gcnnarrow}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -k "gcn or GCN or parity or order or explain or fullsize" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for lib in old new; do
    if [ $lib = old ]; then export GNNMP_LIB=$PWD/ab_libs/libgnnmp_old.so; else unset GNNMP_LIB; fi
    timeout -k 10 300 python bench.py --arch gcn --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('gcn $lib', round(d['ms_per_step'],4))"
  done
done
unset GNNMP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --arch gcn --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt.log 2>&1 || exit $?
python3 -c "
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$OUT/kt/**/*kernel_stats.csv', recursive=True)[0])))
for r in rows[:16]: print('%9.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))"
