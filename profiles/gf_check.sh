#!/bin/bash
# g-form TN with the running block scale: its tests, the configs using it, GCN / GAT / ResBN benches
set -o pipefail
OUT=gpurun_out/${1:-r34}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py ${EXTRA_TESTS:-} -m gpu -x -q -rf \
    --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1
rc=$?
tail -3 "$OUT/pytest.txt"
if [ $rc -ne 0 ]; then exit $rc; fi
for arch in ${ARCHS:-gcn gat sage_resbn}; do
  timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --steps 30 --warmup 10 > "$OUT/$arch.json" 2>> "$OUT/err.txt" || exit $?
  python3 -c "
import json; d=json.load(open('$OUT/$arch.json')); r=d['roofline']
tn=[(k,v['us_per_launch']) for k,v in r['timed_kernels'].items() if 'tn' in k]
print('$arch', round(d['ms_per_step'],4), tn)"
done
