#!/bin/bash
# The whole -m gpu suite, then bench lines of the given archs (no CPU baseline), under gpurun_out/<tag>/
set -o pipefail
TAG=${1:-rXX}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -4 "$OUT/pytest_gpu.txt"
if [ $rc -ne 0 ]; then exit $rc; fi
for arch in "$@"; do
  timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --steps 50 --warmup 10 > "$OUT/$arch.json" 2>> "$OUT/err.txt" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/$arch.json')); print('$arch', round(d['ms_per_step'],4))"
done
