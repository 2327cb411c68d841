#!/bin/bash
# SAGE-ResBN: the identity residual's gradient in conv 1's meanᵀ store (default) vs autograd's add
set -o pipefail
OUT=gpurun_out/${1:-r40}
mkdir -p "$OUT"
for i in 1 2 3; do
  for v in 1 0; do
    GNNMP_RES_FOLD=$v timeout -k 10 300 python bench.py --arch sage_resbn --no-cpu-baseline --steps 50 --warmup 10 > "$OUT/res$v$i.json" 2>> "$OUT/err.txt" || exit $?
    python3 -c "import json; d=json.load(open('$OUT/res$v$i.json')); print('fold=$v', round(d['ms_per_step'],4))"
  done
done
