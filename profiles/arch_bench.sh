#!/bin/bash
# Per-architecture bench lines (with the CPU baseline) on the MI355X box:
#   bash profiles/arch_bench.sh r09 gcn gat sage_resbn sage_scaled
# Each line goes to gpurun_out/<tag>/bench_<arch>.json.  Stops at the first failure.
set -eo pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for ARCH in "$@"; do
  timeout -k 10 300 python bench.py --arch "$ARCH" > "$OUT/bench_$ARCH.log" 2>&1
  tail -1 "$OUT/bench_$ARCH.log" > "$OUT/bench_$ARCH.json"
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$ARCH.json')); print('$ARCH', round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,1), 'M edges/s')"
done
