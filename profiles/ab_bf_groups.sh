#!/bin/bash
# bf16 gathers at F = 128 (configs[4]): one slot per load instruction (GNNMP_BF_GROUPS=1, 32 of 64
# lanes) vs two slots per instruction (=2, VEC 4, agg_wave_group_bf16_kernel; the default)
OUT=gpurun_out/${1:-bfg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -k "bf16 or scaled" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
echo "groups=2 $(tail -1 $OUT/pytest.txt)"
for rep in 1 2; do
  for G in 1 2; do
    GNNMP_BF_GROUPS=$G timeout -k 10 300 python bench.py --arch sage_scaled --no-cpu-baseline --no-roofline > $OUT/r.json 2>$OUT/r.err || { tail -5 $OUT/r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/r.json')); print('sage_scaled groups=$G', round(d['ms_per_step'],4))"
  done
done
for G in 1 2; do
  GNNMP_BF_GROUPS=$G timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt$G" -o run --output-format csv \
      -- python3 bench.py --arch sage_scaled --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > "$OUT/kt$G.log" 2>&1 || exit $?
  python3 - "$OUT/kt$G" $G <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "agg_wave" in r["Name"]:
        print("groups=%s %8.1f us x%s %s" % (sys.argv[2], float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:90]))
PY
done
