#!/bin/bash
# Split-K TN threshold (GNNMP_TN_KSPLIT_MAXM, default 32768) A/B on the 4- and 8-way shards with the
# folded CSC sum (ABI 26).
#   bash profiles/ksplit_ab.sh r113
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for N in 4 8; do
    for m in 0 32768 65536; do
      GNNMP_TN_KSPLIT_MAXM=$m timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/s${N}_m${m}_$rep.json 2>/dev/null || exit $?
      python3 -c "import json; b=json.load(open('$OUT/s${N}_m${m}_$rep.json')); print('rep $rep shard $N ksplit_maxm=$m', round(b['ms_per_step'],4), 'ms')"
    done
  done
done
