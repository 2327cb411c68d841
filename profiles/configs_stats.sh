#!/bin/bash
# Bench lines + rocprofv3 kernel stats of the non-headline BASELINE configs on the final code.
#   bash profiles/configs_stats.sh r21
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for A in gcn gat sage_resbn sage_scaled; do
  timeout -k 10 300 python bench.py --arch $A --no-cpu-baseline > "$OUT/bench_$A.log" 2>&1 || { tail -5 "$OUT/bench_$A.log"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_$A" -o run --output-format csv \
      -- python3 bench.py --arch $A --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt_$A.log" 2>&1 || exit 1
  find "$OUT/kt_$A" -name "*kernel_stats.csv" -exec cp {} "$OUT/${A}_kernel_stats.csv" \;
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$A.log').read().strip().splitlines()[-1])
print('$A', round(d['ms_per_step'],4), round(d['value']/1e6,1), d['roofline']['kernel'], d['roofline']['frac'])"
done
