#!/bin/bash
# One GPU call: the -m gpu suite, then the default bench line (stops at the first abnormal exit).
#   bash profiles/gpu_check.sh <tag> [pytest selection]
TAG=${1:-rXX}
SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${SUITE_LIMIT:-600} python -u -m pytest $SEL -m gpu -q -rfs -x --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.txt"
if [ $rc -ne 0 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 420 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
