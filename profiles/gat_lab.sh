export TMPDIR=/tmp
mkdir -p gpurun_out/r71
for L in 0 1 2 4 7; do
  GNNMP_GAT_LAB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r71/l$L -o run --output-format csv -- python3 bench.py --arch gat --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r71/l$L.log 2>&1 || exit 1
  f=$(find gpurun_out/r71/l$L -name "*kernel_stats.csv" | head -1)
  echo "lab $L: $(grep gat_out_narrow $f | cut -d, -f4)"
done
