#!/bin/bash
# SAGE-ResBN: the output conv's mean + masked CE in one launch (default) vs two (GNNMP_OUT_CE=0)
OUT=gpurun_out/${1:-outce}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_ce.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for C in 1 0; do
    GNNMP_OUT_CE=$C timeout -k 10 300 python bench.py --arch sage_resbn --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('sage_resbn out_ce=$C', round(d['ms_per_step'],4))"
  done
done
