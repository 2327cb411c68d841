#!/bin/bash
# The whole -m gpu suite (one process), output under gpurun_out/<tag>/
#   bash profiles/gpu_suite.sh r23 [pytest args...]
TAG=${1:-rXX}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${SUITE_LIMIT:-900} python -u -m pytest ${@:-tests} -m gpu -q -rf --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -25 "$OUT/pytest_gpu.txt"
exit $rc
