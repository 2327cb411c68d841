#!/bin/bash
# Planes parity tests, the GEMM ablation lab and the planes on/off kernel trace, one GPU call:
#   bash profiles/lab_run.sh <tag>
set -eo pipefail
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_planes.py -x -q --timeout 240 --timeout-method thread > "$OUT/planes.log" 2>&1 \
  || { tail -30 "$OUT/planes.log"; exit 1; }
tail -1 "$OUT/planes.log"
timeout -k 10 200 elliptic_gnn_project_amd/_lab/lab_gemm 7 > "$OUT/lab.txt" 2>&1
cat "$OUT/lab.txt"
bash profiles/ab_planes_kt.sh "$TAG"
