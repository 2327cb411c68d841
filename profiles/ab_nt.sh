#!/bin/bash
# A/B of the headline NT forms in the real step (same box, alternating): the 16-row ring NT
# (default) vs the 32-row NT (GNNMP_AB_NT32=1), then the NT lab.
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in 0 1; do
    GNNMP_AB_NT32=$v timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > "$OUT/ab_$v_$i.json" 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/ab_$v_$i.json')); t=d['roofline']['timed_kernels']; print('nt32=$v', round(d['ms_per_step'],4), [ (k[:14], v['us_per_launch']) for k,v in t.items() if 'gemm' in k])"
  done
done
timeout -k 10 200 elliptic_gnn_project_amd/_lab/lab_nt16 9 > "$OUT/lab_nt16.txt" 2>&1 || exit $?
cat "$OUT/lab_nt16.txt"
