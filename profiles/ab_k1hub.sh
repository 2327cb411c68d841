#!/bin/bash
# K1 hub form A/B: the half-pair tests, then shard steps and the full graph with the hub form
# (default) and without (GNNMP_K1_HUB_N=0), a kernel profile of 8 shards.
OUT=gpurun_out/${1:-k1hub}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for rep in 1 2; do
  for N in 8 4 2; do
    for H in 100000000 0; do
      GNNMP_K1_HUB_N=$H timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/s${N}_$H.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$OUT/s${N}_$H.json')); print('shard of $N hub_n=$H:', d['config']['max_nodes_per_gpu'], 'nodes', round(d['ms_per_step'],4), 'ms/step')"
    done
  done
  for H in 0 100000000; do
    GNNMP_K1_HUB_N=$H timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $OUT/full_$H.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/full_$H.json')); print('full hub_n=$H:', round(d['ms_per_step'],4), 'ms/step')"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt8 -o run --output-format csv -- python3 bench.py --rehearse-shard 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt8.log 2>&1 || exit $?
find $OUT/kt8 -name "*kernel_stats.csv" -exec cp {} $OUT/shard8_kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/shard8_kernel_stats.csv')))
for r in rows[:12]: print('%9.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:100]))"
