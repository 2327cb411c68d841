#!/bin/bash
# Round profile collection on the MI355X box (run through gpurun from the repo root):
#   bash profiles/collect.sh r01
# 1. the default bench line, 2. rocprofv3 kernel-trace + stats of the same bench,
# 3./4. separate PMC passes for FETCH_SIZE and WRITE_SIZE (they do not fit one pass on gfx950),
# 5. per-kernel traffic summary (profiles/pmc_summary.py).  Every GPU step has its own time
# limit and the chain stops at the first failure.
set -eo pipefail
TAG=${1:-rXX}
ARCH=${ARCH:-sage}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --arch $ARCH --steps 20 --warmup 5 --no-cpu-baseline"

timeout -k 10 420 python bench.py --arch $ARCH > "$OUT/bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 $BENCH > "$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
    -- python3 bench.py --arch $ARCH --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
    -- python3 bench.py --arch $ARCH --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > "$OUT/write.log" 2>&1
python3 profiles/pmc_summary.py --fetch "$OUT/fetch" --write "$OUT/write" --out "$OUT/traffic.json" \
    > "$OUT/traffic.txt"
cp "$OUT/traffic.json" "$OUT/traffic_${ARCH}.json"  # commit as profiles/traffic_<arch>.json (bench.py reads it)
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
tail -1 "$OUT/bench.log"
cat "$OUT/traffic.txt"
