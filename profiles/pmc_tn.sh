#!/bin/bash
# PMC passes over single TN lab variants (bench_gemm LAB_TN_ONLY): SQ issue/wait picture.
#   bash profiles/pmc_tn.sh "0 7"
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmctn
mkdir -p $OUT
B=elliptic_gnn_project_amd/_build/bench_gemm
PA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
PC="TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE"
for v in ${1:-0 7}; do
  i=0
  for P in "$PA" "$PB" "$PC"; do
    i=$((i+1))
    LAB_TN_ONLY=$v timeout -s KILL 60 rocprofv3 --pmc $P -d $OUT/v${v}_p$i -o run --output-format csv -- $B 203769 3 > $OUT/v${v}_p$i.log 2>&1 || { echo FAIL $v $i; tail -5 $OUT/v${v}_p$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmctn/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "gemm_tn" not in r["Kernel_Name"]: continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[2], {k: round(v / max(n[k], 1) / 1e6, 3) for k, v in sorted(agg.items())}, "(1e6 per dispatch)")
PY
echo ok
