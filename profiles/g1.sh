set -o pipefail
mkdir -p gpurun_out/r22b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_train_ops.py tests/test_gpu_capture.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r22b/pytest_sel.txt 2>&1
rc=$?
tail -5 gpurun_out/r22b/pytest_sel.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/timing_probe.sh r22b
