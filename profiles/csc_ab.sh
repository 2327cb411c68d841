#!/bin/bash
# ABI 26 A/B: the layer-1 TN forming dz's CSC half itself (GNNMP_TN_CSC=1, default) vs the separate
# CSC-sum launch (GNNMP_TN_CSC=0) — parity tests, then the headline and the 8-shard rehearsal both
# ways on the same box, then kernel stats of the folded step.
#   bash profiles/csc_ab.sh r105
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_tn_csc.py tests/test_gpu_fused_ce.py -x -v --timeout 200 \
    --timeout-method thread > $OUT/pytest_csc.txt 2>&1 || { tail -30 $OUT/pytest_csc.txt; exit 1; }
tail -3 $OUT/pytest_csc.txt
for rep in 1 2; do
  for v in 1 0; do
    GNNMP_TN_CSC=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_csc${v}_$rep.json 2>$OUT/bench_csc${v}_$rep.err || exit $?
    GNNMP_TN_CSC=$v timeout -k 10 200 python bench.py --rehearse-shard 8 --no-cpu-baseline --no-roofline > $OUT/shard8_csc${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; a=json.load(open('$OUT/bench_csc${v}_$rep.json')); b=json.load(open('$OUT/shard8_csc${v}_$rep.json')); print('TN_CSC=$v rep $rep: full', round(a['ms_per_step'],4), 'ms (frac', a['roofline']['frac'], ') shard8', round(b['ms_per_step'],4), 'ms')"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt8 -o run --output-format csv -- python3 bench.py --rehearse-shard 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt8.log 2>&1 || exit $?
find $OUT/kt8 -name "*kernel_stats.csv" -exec cp {} $OUT/shard8_kernel_stats.csv \;
for f in kernel_stats shard8_kernel_stats; do
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/$f.csv')))
print('$f')
for r in rows[:10]: print('%9.2f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:90]))"
done
