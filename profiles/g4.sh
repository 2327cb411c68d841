set -o pipefail
OUT=gpurun_out/r30; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_planes.py tests/test_gpu_fused.py tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -ne 0 ] && exit $rc
bash profiles/shard_probe.sh r30
