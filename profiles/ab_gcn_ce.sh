#!/bin/bash
# GCN: output aggregation + masked CE in one launch (gnn_gcn_out_ce_f32) vs two (GNNMP_GCN_CE=0)
OUT=gpurun_out/${1:-gcnce}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_ce.py tests/test_gpu_train_ops.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for C in 1 0; do
    GNNMP_GCN_CE=$C timeout -k 10 300 python bench.py --arch gcn --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('gcn fused_ce=$C', round(d['ms_per_step'],4))"
  done
done
