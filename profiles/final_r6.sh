#!/bin/bash
# Round-6 closing run: the whole -m gpu suite, smoke(), the headline bench line (driver defaults and
# the driver's exact command), the 1/2/4/8-shard rehearsals and the 8-shard kernel stats.
#   bash profiles/final_r6.sh r107
TAG=${1:-rXX}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2>$OUT/bench.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/driver_cmd.json 2>/dev/null || exit $?
python3 -c "import json; a=json.load(open('$OUT/bench.json')); b=json.load(open('$OUT/driver_cmd.json')); print('bench', round(a['ms_per_step'],4), 'ms', round(a['value']/1e9,4), 'G edges/s frac', a['roofline']['frac'], '| driver cmd', round(b['ms_per_step'],4))"
bash profiles/shard_probe.sh $TAG
