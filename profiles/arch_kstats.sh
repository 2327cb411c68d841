#!/bin/bash
# rocprofv3 kernel stats of bench.py --arch A (per-step kernel list) for each arch given
OUT=gpurun_out/${1:-ks}; shift; mkdir -p $OUT; export TMPDIR=/tmp
for A in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_$A" -o run --output-format csv \
      -- python3 bench.py --arch $A --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/kt_$A.log" 2>&1 || exit $?
  python3 - "$OUT/kt_$A" $A <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    c = int(r["Calls"])
    if c >= 25 and "spin" not in r["Name"] and "rocclr" not in r["Name"]:
        print("%s %8.1f us x%.1f %s" % (sys.argv[2], float(r["AverageNs"]) / 1e3, c / 25, r["Name"][:120]))
PY
done
