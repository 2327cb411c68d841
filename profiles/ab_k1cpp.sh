#!/bin/bash
# K1's riding B prep, columns per pass (ws_prep_h2_body CPP 1 / 2 / 4): shard steps and the full graph
OUT=gpurun_out/${1:-k1cpp}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for N in 8 4; do
    for C in 1 2 4; do
      GNNMP_K1_PREP_CPP=$C timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/s${N}_$C.json 2>/dev/null || exit $?
      python3 -c "import json; d=json.load(open('$OUT/s${N}_$C.json')); print('shard of $N cpp=$C:', round(d['ms_per_step'],4), 'ms/step')"
    done
  done
  for C in 1 2 4; do
    GNNMP_K1_PREP_CPP=$C timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > $OUT/full_$C.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.load(open('$OUT/full_$C.json')); print('full cpp=$C:', round(d['ms_per_step'],4), 'ms/step')"
  done
done
