#!/bin/bash
# Kernel trace of the bench step with the split-image path on (1) and off (0): bash profiles/ab_planes_kt.sh <tag>
set -eo pipefail
OUT=gpurun_out/${1:-rXX}
mkdir -p "$OUT"
export TMPDIR=/tmp
for P in 1 0; do
  GNNMP_PLANES=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$P" -o run --output-format csv \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/kt$P.log" 2>&1
  echo "planes=$P"; python3 profiles/kstats.py "$OUT/kt$P/run_kernel_stats.csv" 4
done
