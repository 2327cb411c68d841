#!/bin/bash
# Round GPU run: the full -m gpu suite, then the profile collection (collect.sh) unless the suite
# ended abnormally (a fault, abort, time limit: rc other than 0 = pass / 1 = test failures).
#   bash profiles/round.sh r14
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 ${SUITE_LIMIT:-500} python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
tail -15 "$OUT/pytest_gpu.txt"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
bash profiles/collect.sh "$TAG"
