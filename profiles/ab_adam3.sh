#!/bin/bash
OUT=gpurun_out/${1:-adam3}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_grad_sq_fold.py tests/test_gpu_capture.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for arch in gcn gat sage_resbn; do
  timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-roofline > $OUT/$arch.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/$arch.json')); print('$arch', round(d['ms_per_step'],4))"
done
