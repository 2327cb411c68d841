#!/bin/bash
# K12's merge + finalize in one launch: BN / ResBN tests, then the configs[3] bench and kernel stats
OUT=gpurun_out/${1:-bn}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -k "bn or resbn or ResBN or k14 or k8 or k9" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --arch sage_resbn --no-cpu-baseline --no-roofline > $OUT/r.json 2>$OUT/r.err || { tail -5 $OUT/r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/r.json')); print('sage_resbn', round(d['ms_per_step'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 bench.py --arch sage_resbn --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/kt.log" 2>&1 || exit $?
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
grep -c bn_ "$OUT/kernel_stats.csv"
