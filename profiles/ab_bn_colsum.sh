#!/bin/bash
# SAGE-ResBN: layer 0's conv bias gradient from K12's backward column sums vs a colsum pass
OUT=gpurun_out/${1:-bncolsum}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_ce.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -k "resbn or ResBN or sage_resbn or fused_ce" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for C in 1 0; do
    GNNMP_BN_COLSUM=$C timeout -k 10 300 python bench.py --arch sage_resbn --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('sage_resbn bn_colsum=$C', round(d['ms_per_step'],4))"
  done
done
