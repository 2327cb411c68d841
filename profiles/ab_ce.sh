#!/bin/bash
# Fused output mean + CE vs the separate CE launch: tests, then alternating bench runs.
set -o pipefail
OUT=gpurun_out/${1:-r30}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_ce.py tests/test_gpu_capture.py tests/test_gpu_train_ops.py \
    -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1
rc=$?
tail -4 "$OUT/pytest.txt"
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for v in fused separate; do
    f=""; [ $v = separate ] && f="--separate-ce"
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 10 $f > "$OUT/b_$v$i.json" 2>> "$OUT/bench.err" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/b_$v$i.json')); print('$v', round(d['ms_per_step'],4))"
  done
done
