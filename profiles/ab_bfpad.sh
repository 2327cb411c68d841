#!/bin/bash
# bf16-storage SAGE (configs[4]): layer-0 K1 over the image's zero-padded A2 half (default) vs over
# x itself (GNNMP_K1_PAD=0), after the bf16 and full-size GPU tests.
#   bash profiles/ab_bfpad.sh r20b
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -rf > "$OUT/t.txt" 2>&1
rc=$?
tail -3 "$OUT/t.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --arch sage_scaled --no-cpu-baseline > "$OUT/pad.log" 2>&1 || exit 1
GNNMP_K1_PAD=0 timeout -k 10 300 python bench.py --arch sage_scaled --no-cpu-baseline > "$OUT/nopad.log" 2>&1 || exit 1
for f in pad nopad; do python3 -c "
import json; d=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1])
t=d['roofline']['timed_kernels']; print('$f', round(d['ms_per_step'],4), {k: v['us_per_launch'] for k,v in t.items() if 'agg' in k})"; done
