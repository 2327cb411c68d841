#!/bin/bash
# same-box A/B: clip + Adam two launches (ab_libs/libgnnmp_old.so) vs one launch (the tree's library)
OUT=gpurun_out/${1:-adamlib}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3; do
  for arch in gcn gat; do
    for lib in old new; do
      if [ $lib = old ]; then export GNNMP_LIB=$PWD/ab_libs/libgnnmp_old.so; else unset GNNMP_LIB; fi
      timeout -k 10 300 python bench.py --arch $arch --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$OUT/r.json')); print('$arch $lib', round(d['ms_per_step'],4))"
    done
  done
done
