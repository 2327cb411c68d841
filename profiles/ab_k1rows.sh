#!/bin/bash
# K1 hub form: average rows per balanced wave 16 (default) vs 8 / 12, full graph, interleaved
OUT=gpurun_out/${1:-k1rows}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2 3 4; do
  line="rep $rep:"
  for R in 16 8 12; do
    GNNMP_K1_WAVE_ROWS=$R timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $OUT/r.json 2>/dev/null || exit $?
    line="$line rows=$R $(python3 -c "import json; print('%.4f' % json.load(open('$OUT/r.json'))['ms_per_step'])")"
  done
  echo "$line"
done
