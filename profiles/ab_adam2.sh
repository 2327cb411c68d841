#!/bin/bash
# one-launch clip + Adam vs the two launches: per-kernel times on GCN / ResBN, optimizer tests
OUT=gpurun_out/${1:-adam2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_grad_sq_fold.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for arch in gcn sage_resbn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$arch -o run --output-format csv -- python3 bench.py --arch $arch --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt_$arch.log 2>&1 || exit $?
  python3 -c "
import csv,glob
rows=list(csv.DictReader(open(glob.glob('$OUT/kt_$arch/**/*kernel_stats.csv', recursive=True)[0])))
for r in rows:
  if 'adam' in r['Name'] or 'grad_sq' in r['Name']: print('$arch %.1f us x%s %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:80]))"
done
for rep in 1 2; do
  for arch in gcn gat sage_resbn; do
    timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-roofline > $OUT/$arch.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/$arch.json')); print('$arch', round(d['ms_per_step'],4))"
  done
done
