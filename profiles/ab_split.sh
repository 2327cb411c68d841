#!/bin/bash
# long-segment split (GNNMP_SPLIT) and degree order (GNNMP_ORDER) of the wide gathers, per arch
OUT=gpurun_out/${1:-split}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for A in gcn sage_resbn; do
    for S in 1 0; do
      GNNMP_SPLIT=$S timeout -k 10 300 python bench.py --arch $A --no-cpu-baseline --no-roofline > $OUT/r.json 2>$OUT/r.err || { tail -5 $OUT/r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/r.json')); print('$A split=$S', round(d['ms_per_step'],4))"
    done
  done
done
