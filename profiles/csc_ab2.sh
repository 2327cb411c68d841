#!/bin/bash
# ABI 26 A/B by shard size: the CSC sum inside the TN (GNNMP_TN_CSC_INKERNEL=1) vs the separate
# launch (=0) on the largest 2- / 4- / 8-way shard and on the full graph.
#   bash profiles/csc_ab2.sh r106
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tn_csc.py tests/test_gpu_fused_ce.py tests/test_gpu_fullsize.py -k 'csc or sage or ce' -x -v --timeout 200 \
    --timeout-method thread > $OUT/pytest_csc.txt 2>&1 || { tail -30 $OUT/pytest_csc.txt; exit 1; }
tail -2 $OUT/pytest_csc.txt
for rep in 1 2; do
  for N in 8 4 2; do
    for v in 1 0; do
      GNNMP_TN_CSC_INKERNEL=$v timeout -k 10 200 python bench.py --rehearse-shard $N --no-cpu-baseline --no-roofline > $OUT/shard${N}_k${v}_$rep.json 2>/dev/null || exit $?
      python3 -c "import json; b=json.load(open('$OUT/shard${N}_k${v}_$rep.json')); print('rep $rep shard $N inkernel=$v', round(b['ms_per_step'],4), 'ms')"
    done
  done
  for v in 1 0; do
    GNNMP_TN_CSC_INKERNEL=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/full_k${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json; a=json.load(open('$OUT/full_k${v}_$rep.json')); print('rep $rep full inkernel=$v', round(a['ms_per_step'],4), 'ms frac', a['roofline']['frac'])"
  done
done
