#!/bin/bash
# A/B of the split-image (planes) layer-1 path vs the in-kernel split, same box (run via gpurun):
#   bash profiles/ab_planes.sh r14b
set -eo pipefail
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 240 --timeout-method thread > "$OUT/planes.log" 2>&1
for P in 1 0; do
  GNNMP_PLANES=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/kt$P" -o run --output-format csv \
      -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/kt$P.log" 2>&1
  python3 profiles/kstats.py "$OUT/kt$P/run_kernel_stats.csv" 8
done
tail -2 "$OUT/planes.log"
