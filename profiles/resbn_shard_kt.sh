OUT=gpurun_out/r111; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --arch sage_resbn --rehearse-shard 8 --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/resbn_shard8_kernel_stats.csv \;
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/resbn_shard8_kernel_stats.csv')))
tot=0
for r in rows:
  c=int(r['Calls'])
  if c>=25 and 'copyBuffer' not in r['Name']:
    tot+=float(r['TotalDurationNs'])/28e3
    print('%8.2f us x%4d  %s' % (float(r['AverageNs'])/1e3, c, r['Name'][:110]))
print('sum per step (28 steps)', round(tot,1))"
