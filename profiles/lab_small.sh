#!/bin/bash
# Small-M GEMM lab under rocprofv3 (csrc/lab/lab_small.hip): per-kernel averages at shard sizes.
#   bash profiles/lab_small.sh r64 [M ...]
TAG=${1:-rXX}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for M in ${@:-27196 52466 203769}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ls_$M -o run --output-format csv -- ./elliptic_gnn_project_amd/_lab/lab_small $M 20 > $OUT/ls_$M.log 2>&1 || exit $?
  f=$(find $OUT/ls_$M -name "*kernel_stats.csv" | head -1)
  echo "== M $M"
  python3 - "$f" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    m = re.search(r'(gemm_\w+_kernel|lab_reduce_kernel|split_h2_kernel|ws_prep_h2_kernel)<?([^>(]*)', n)
    print('%9.2f us x%4s  %s<%s>' % (float(r['AverageNs'])/1e3, r['Calls'], m.group(1) if m else n[:60], m.group(2) if m else ''))
PY
done
