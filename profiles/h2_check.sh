mkdir -p gpurun_out/h2t
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_planes.py -x -q -rfs --timeout 200 --timeout-method thread > gpurun_out/h2t/pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/h2t/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/h2t/bench.log 2>&1 || { tail -20 gpurun_out/h2t/bench.log; exit 1; }
tail -1 gpurun_out/h2t/bench.log
