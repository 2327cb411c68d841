#!/bin/bash
OUT=gpurun_out/${1:-rows8}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_fullsize.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
  python3 -c "import json; print('sage', round(json.load(open('$OUT/r.json'))['ms_per_step'],4))"
  timeout -k 10 200 python bench.py --rehearse-shard 8 --no-cpu-baseline --no-roofline > $OUT/s.json 2>/dev/null || exit $?
  python3 -c "import json; print('shard8', round(json.load(open('$OUT/s.json'))['ms_per_step'],4))"
done
