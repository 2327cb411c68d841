#!/bin/bash
# K1 hub form parameters: hub threshold (GNNMP_K1_HUB_DEG) and average rows per balanced wave
# (GNNMP_K1_WAVE_ROWS), on the 8- / 4-way shards and the full graph
OUT=gpurun_out/${1:-k1waves}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "32 16" "16 16" "64 16" "32 8" "32 12" "32 24"; do
    set -- $cfg
    line="hub_deg=$1 rows=$2:"
    for N in 8 4 1; do
      GNNMP_K1_HUB_DEG=$1 GNNMP_K1_WAVE_ROWS=$2 timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
      line="$line $(python3 -c "import json; d=json.load(open('$OUT/r.json')); print('N%d %.4f' % ($N, d['ms_per_step']))")"
    done
    echo "$line"
  done
done
