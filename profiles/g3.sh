set -o pipefail
OUT=gpurun_out/r27; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_fullsize.py tests/test_gpu_planes.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; tail -4 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
for A in gcn gat sage_resbn; do
  timeout -k 10 300 python bench.py --arch $A --no-cpu-baseline > $OUT/bench_$A.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$A.json')); r=d['roofline']; print('$A', round(d['ms_per_step'],4), [(k[:40], v['us_per_launch']) for k,v in r['timed_kernels'].items() if 'gemm_tn' in k])"
done
for v in 1 0 1 0; do
  GNNMP_AB_WS64=$v timeout -k 10 300 python bench.py --arch sage_resbn --no-cpu-baseline --no-roofline > $OUT/ab_ws64_$v.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/ab_ws64_$v.json')); print('ws64=$v', round(d['ms_per_step'],4))"
done
