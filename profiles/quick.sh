#!/bin/bash
# Quick GPU iteration: selected tests, the headline bench, rocprof kernel stats of the bench.
#   bash profiles/quick.sh r24 "tests/test_gpu_h2.py tests/test_gpu_fused.py" [arch]
set -o pipefail
TAG=${1:-rXX}
TESTS=${2:-tests/test_gpu_h2.py}
ARCH=${3:-sage}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -rf --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1
rc=$?
tail -4 "$OUT/pytest.txt"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --arch $ARCH --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('ms/step', round(d['ms_per_step'],4), 'dominant', r['kernel'], r['avg_us'], r['frac']); [print('  ', k, v['us_per_launch'], v.get('hbm_frac')) for k,v in r['timed_kernels'].items()]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv \
    -- python3 bench.py --arch $ARCH --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || exit $?
find "$OUT" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/kernel_stats.csv')))
for r in rows[:14]: print('%9.1f us x%4s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:110]))"
