#!/bin/bash
# A/B of the g-form TN's ring depths (GNNMP_TN_GF_LAB builds in _lab/): GCN and SAGE-ResBN benches
set -o pipefail
OUT=gpurun_out/${1:-r32}
mkdir -p "$OUT"
export TMPDIR=/tmp
for arch in ${ARCHS:-gcn sage_resbn}; do
  for v in ${VARS:-0 16 32 48}; do
    lib=""; [ $v != 0 ] && lib=elliptic_gnn_project_amd/_lab/libgnnmp_gf$v.so
    GNNMP_LIB=$lib timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --steps 30 --warmup 10 > "$OUT/$arch$v.json" 2>> "$OUT/err.txt" || exit $?
    python3 -c "
import json; d=json.load(open('$OUT/$arch$v.json')); r=d['roofline']
tn=[(k,v['us_per_launch']) for k,v in r['timed_kernels'].items() if 'tn' in k]
print('$arch', $v, round(d['ms_per_step'],4), tn)"
  done
done
