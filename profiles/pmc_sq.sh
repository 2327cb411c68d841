#!/bin/bash
# SQ issue / wait picture of the bench's GEMM and K1 kernels (one rocprofv3 pass per counter
# set, never combined with traces):  bash profiles/pmc_sq.sh <tag> [arch]
set -o pipefail
TAG=$1; ARCH=${2:-sage}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
PA="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
PB="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o run --output-format csv \
      -- python3 bench.py --arch $ARCH --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline > $OUT/p$i.log 2>&1 \
      || { echo FAIL pass $i; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, re, sys
out = sys.argv[1]
rx = re.compile(r"gemm_tn|gemm_nt|agg_wave")
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
    d = {c: agg[k][c] / cnt[k][c] for c in agg[k]}
    waves = d.get("SQ_WAVES", 1)
    print(k)
    for c in sorted(d):
        print(f"   {c:26s} {d[c]:.4g}")
    if "SQ_WAVE_CYCLES" in d:  # quad-cycles summed over waves -> cycles per wave
        wc = 4 * d["SQ_WAVE_CYCLES"] / waves
        print(f"   cycles/wave {wc:.0f}: active {4 * d.get('SQ_ACTIVE_INST_ANY', 0) / waves / wc:.2f}"
              f" wait {4 * d.get('SQ_WAIT_ANY', 0) / waves / wc:.2f} stall {4 * d.get('SQ_WAIT_INST_ANY', 0) / waves / wc:.2f}"
              f" valu {4 * d.get('SQ_ACTIVE_INST_VALU', 0) / waves / wc:.2f}"
              f" mfma-busy/SIMD {d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / wc:.2f}")
PY
