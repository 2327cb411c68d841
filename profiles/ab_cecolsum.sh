#!/bin/bash
# bias gradients from the kernels' column sums: tests, then GCN / GAT / SAGE-ResBN with the CE's and
# the skinny NT's sums (default) vs separate colsum passes (GNNMP_CE_COLSUM=0 GNNMP_NT_COLSUM=0)
OUT=gpurun_out/${1:-cecolsum}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do
  for arch in gcn gat sage_resbn; do
    for C in 1 0; do
      GNNMP_CE_COLSUM=$C GNNMP_NT_COLSUM=$C timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$OUT/r.json')); print('$arch kernel_colsums=$C', round(d['ms_per_step'],4))"
    done
  done
done
