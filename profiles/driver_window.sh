#!/bin/bash
# The driver's window (--steps 20 --warmup 5) vs 50 steps, with per-step HIP-event times, and a
# longer clock settle — where the 20-step line's extra us/step come from
OUT=gpurun_out/${1:-drvwin}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "20 5 300" "50 10 300" "20 5 1000" "20 5 3000"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps $1 --warmup $2 --settle-ms $3 --no-cpu-baseline --no-roofline --step-trace > $OUT/r.json 2> $OUT/r.err || exit $?
    python3 -c "
import json
d=json.load(open('$OUT/r.json'))
g=[l for l in open('$OUT/r.err') if l.startswith('step-trace gpu')][0].split()[3:]
g=[float(x) for x in g]
print('steps=$1 warmup=$2 settle=$3: %.4f ms/step; gpu events first5 %s mean %.4f' % (d['ms_per_step'], ' '.join('%.4f'%x for x in g[:5]), sum(g)/len(g)))"
  done
done
