#!/bin/bash
# Per-architecture kernel-trace profiles on the MI355X box (run through gpurun from the repo root):
#   bash profiles/arch_kt.sh r07 gat gcn
# For each arch: rocprofv3 --kernel-trace --stats of a short bench run (no CPU baseline), its
# kernel_stats.csv copied to gpurun_out/<tag>/<arch>_kernel_stats.csv.  Stops at the first failure.
set -eo pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for ARCH in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_$ARCH" -o run --output-format csv \
      -- python3 bench.py --arch "$ARCH" --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt_$ARCH.log" 2>&1
  find "$OUT/kt_$ARCH" -name "*kernel_stats.csv" -exec cp {} "$OUT/${ARCH}_kernel_stats.csv" \;
  tail -1 "$OUT/kt_$ARCH.log"
done
