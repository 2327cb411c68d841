#!/bin/bash
# 8-shard rehearsal lines of the other configs (the largest shard of the 8-way timestep partition)
OUT=gpurun_out/${1:-sharda}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for A in "$@"; do
  timeout -k 10 300 python bench.py --arch $A --rehearse-shard 8 --no-cpu-baseline --no-roofline > $OUT/shard8_$A.json 2>$OUT/shard8_$A.err || { tail -5 $OUT/shard8_$A.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/shard8_$A.json')); print('$A shard 8:', d['config']['max_nodes_per_gpu'], 'nodes', round(d['ms_per_step'],4), 'ms/step')"
done
