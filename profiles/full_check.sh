#!/bin/bash
# One GPU call: GEMM lab (half-pair), the whole -m gpu suite, the default bench line.
#   bash profiles/full_check.sh <tag>
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -x elliptic_gnn_project_amd/_lab/lab_h2 ]; then
  timeout -k 10 200 elliptic_gnn_project_amd/_lab/lab_h2 5 > "$OUT/lab.txt" 2>&1
  rc=$?; tail -25 "$OUT/lab.txt"; [ $rc -ne 0 ] && { echo "lab rc=$rc"; exit $rc; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfs --timeout 600 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 420 python bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
