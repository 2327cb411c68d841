export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "tests/test_gpu_fullsize.py::test_full_size_sage_resbn_train_step" -m gpu -q -rf --timeout 200 --timeout-method thread 2>&1 | grep -E "^E |passed|failed" | head -8
GNNMP_H2=0 timeout -k 10 300 python -u -m pytest "tests/test_gpu_fullsize.py::test_full_size_sage_resbn_train_step" -m gpu -q -rf --timeout 200 --timeout-method thread 2>&1 | grep -E "^E |passed|failed" | head -8
