#!/bin/bash
# (ABI 25) GAT lin TN block scales from the attention backward's row-group maxima vs its own scan
# (GNNMP_GAT_ROWMAX); the rowmax / GAT / g-form tests first
OUT=gpurun_out/${1:-rowmax}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gat_rowmax.py tests/test_gpu_gat_proj.py tests/test_gpu_h2.py tests/test_host.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do
  for C in 1 0; do
    GNNMP_GAT_ROWMAX=$C timeout -k 10 300 python bench.py --arch gat --no-cpu-baseline --no-roofline > $OUT/r.json 2>$OUT/r.err || { tail -5 $OUT/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('gat rowmax=$C', round(d['ms_per_step'],4))"
  done
done
bash profiles/arch_kstats.sh $1_ks gat | grep -E "gemm_tn_h2|gat_bwd_cols|rowmax"
