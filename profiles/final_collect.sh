#!/bin/bash
# smoke(), the driver's exact bench command, then collect.sh (bench line with CPU baseline, rocprof
# kernel stats, FETCH / WRITE PMC passes, traffic summary) for the headline.
set -o pipefail
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { tail -5 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 420 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_cmd.json" 2> "$OUT/driver_cmd.err" || exit $?
python3 -c "import json; d=json.loads(open('$OUT/driver_cmd.json').read().strip().splitlines()[-1]); print('driver cmd', round(d['ms_per_step'],4), d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline']['value'])"
bash profiles/collect.sh "$TAG"
