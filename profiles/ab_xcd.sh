#!/bin/bash
# K1 with the XCD-aware block order (_lab/libgnnmp_xcd.so, -DGNNMP_K1_XCD=1) vs the product order
set -o pipefail
OUT=gpurun_out/${1:-r45}
mkdir -p "$OUT"
for i in 1 2 3; do
  for v in xcd base; do
    lib=""; [ $v = xcd ] && lib=elliptic_gnn_project_amd/_lab/libgnnmp_xcd.so
    GNNMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > "$OUT/$v$i.json" 2>> "$OUT/err.txt" || exit $?
    python3 -c "
import json; d=json.load(open('$OUT/$v$i.json')); r=d['roofline']['timed_kernels']
print('$v', round(d['ms_per_step'],4), [(k[:22], v['us_per_launch']) for k,v in r.items() if 'F=166' in k])"
  done
done
