#!/bin/bash
# PMC passes over single lab variants
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmclab
mkdir -p $OUT
B=elliptic_gnn_project_amd/_build/bench_gemm
PA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU"
PC="TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE"
for v in 0 11w 16w 17w; do
  i=0
  for P in "$PA" "$PB" "$PC"; do
    i=$((i+1))
    LAB_ONLY=$v timeout -k 10 60 rocprofv3 --pmc $P -d $OUT/v${v}_p$i -o run --output-format csv -- $B 203769 3 > $OUT/v${v}_p$i.log 2>&1 || { echo FAIL $v $i; tail -5 $OUT/v${v}_p$i.log; exit 1; }
  done
done
echo ok
