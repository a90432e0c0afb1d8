set -u
# r06: 1M protocol crawl wall (no profiler, one warm-up crawl) for IKNP and SoftSpoken k = 2, 4
O=gpurun_out/${1:-r06ss3}; mkdir -p $O
for k in 1 4 2; do
  timeout -k 10 300 python3 bench.py --gc ot --base-ot --ot-ss-k $k --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_k$k.json 2> $O/bench_k$k.err || { echo bench k$k failed; exit 1; }
done
echo done
