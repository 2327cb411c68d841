#!/bin/bash
# GCN: bias gradient from the skinny NT's column sums vs a separate colsum pass (GNNMP_NT_COLSUM=0)
OUT=gpurun_out/${1:-ntcolsum}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_fullsize.py -k "colsum or gcn or GCN" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for C in 1 0; do
    GNNMP_NT_COLSUM=$C timeout -k 10 300 python bench.py --arch gcn --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('gcn colsum_in_nt=$C', round(d['ms_per_step'],4))"
  done
done
