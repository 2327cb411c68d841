set -eo pipefail
mkdir -p gpurun_out/r86; export TMPDIR=/tmp
for m in 65536 0; do
GNNMP_TN_KSPLIT_MAXM=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r86/kt_$m -o run --output-format csv -- python3 bench.py --rehearse-shard 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r86/kt_$m.log 2>&1
f=$(find gpurun_out/r86/kt_$m -name "*kernel_stats.csv" | head -1)
python3 - "$f" $m <<'PY'
import csv, sys
print("== maxm", sys.argv[2])
for r in csv.DictReader(open(sys.argv[1])):
    n=r["Name"]
    if ("gemm_tn" in n or "slab_reduce" in n) and int(r["Calls"])>=20:
        print('%7.2f %4s %s' % (float(r["AverageNs"])/1e3, r["Calls"], n[:110]))
PY
done
