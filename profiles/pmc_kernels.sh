#!/bin/bash
# SQ issue/wait and HBM-traffic PMC passes over the libgnnmp kernels of one bench arch:
#   bash profiles/pmc_kernels.sh <tag> <arch> <kernel-regex>
# Each pass is its own short rocprofv3 run (counters never combined with traces); the summary
# prints per-dispatch averages of every counter for the kernels whose name matches the regex.
set -o pipefail
TAG=$1; ARCH=$2; RX=$3
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
PB="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
i=0
for P in "$PA" "$PB" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv \
      -- python3 bench.py --arch $ARCH --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline > $OUT/p$i.log 2>&1 \
      || { echo FAIL pass $i; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "$RX" <<'PY'
import csv, glob, collections, re, sys
out, rx = sys.argv[1], re.compile(sys.argv[2])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not rx.search(name):
            continue
        m = re.search(r"(\w+_kernel(<[^()]*>)?)", name)
        key = m.group(1) if m else name[:70]
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[key][r["Counter_Name"]] += 1
for k in agg:
    print(k)
    for c in sorted(agg[k]):
        print(f"   {c:24s} {agg[k][c] / cnt[k][c]:.4g}")
PY
