#!/bin/bash
# Driver-vs-builder timing probe: the driver's exact bench command beside
# longer windows, with and without the pre-warm-up clock settle, and per-step event traces.
#   bash profiles/timing_probe.sh r22b
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 240 python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?; echo "$name: $(python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(round(d['ms_per_step'],4))")"; }
NC="--no-cpu-baseline --no-roofline"
run drv_settle --gpus 1 --steps 20 --warmup 5 $NC --step-trace
run drv_nosettle --gpus 1 --steps 20 --warmup 5 $NC --settle-ms 0 --step-trace
run long_settle --gpus 1 --steps 50 --warmup 10 $NC
run drv_settle2 --gpus 1 --steps 20 --warmup 5 $NC --step-trace
run drv_full --gpus 1 --steps 20 --warmup 5
grep step-trace "$OUT"/*.err | grep "gpu ms"
