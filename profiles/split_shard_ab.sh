#!/bin/bash
# Long-segment split (GNNMP_SPLIT) A/B on the strong-scaling shards of the wide-gather nets.
#   bash profiles/split_shard_ab.sh r112
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for arch in sage_resbn gcn; do
    for N in 8 4; do
      for v in 1 0; do
        GNNMP_SPLIT=$v timeout -k 10 200 python bench.py --arch $arch --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/${arch}_s${N}_split${v}_$rep.json 2>/dev/null || exit $?
        python3 -c "import json; b=json.load(open('$OUT/${arch}_s${N}_split${v}_$rep.json')); print('rep $rep $arch shard $N split=$v', round(b['ms_per_step'],4), 'ms')"
      done
    done
  done
done
