set -u
# r06: the 1M protocol crawl's kernel stats on SoftSpoken k = 2 and 4 (bench --gc ot --base-ot --ot-ss-k k)
O=gpurun_out/${1:-r06ss2}; mkdir -p $O
export TMPDIR=/tmp
for k in 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp$k -o run -- python3 bench.py --gc ot --base-ot --ot-ss-k $k --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo bench k$k failed; exit 1; }
  find $O/tmp$k -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_k$k.csv \;
  rm -rf $O/tmp$k
done
echo done
