#!/bin/bash
# r15 check: bf16 + planes tests, GEMM lab, headline and scaled kernel traces (one GPU call)
set -eo pipefail
OUT=gpurun_out/${1:-r15}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_planes.py tests/test_gpu_fused.py -q -x --timeout 240 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 200 elliptic_gnn_project_amd/_lab/lab_gemm 7 > "$OUT/lab.txt" 2>&1
grep -E "TN production|NT production" "$OUT/lab.txt"
bash profiles/arch_kt.sh "${1:-r15}" sage sage_scaled > /dev/null
for a in sage sage_scaled; do
  echo "$a"; python3 profiles/kstats.py "$OUT/${a}_kernel_stats.csv" 8
  grep -h "^{" "$OUT/kt_$a.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value']/1e6)"
done
