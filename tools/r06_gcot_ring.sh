set -u
# r06: 1M protocol crawl kernel stats, SoftSpoken k = 2 + Z_2^32 table (the bench's protocol form)
O=gpurun_out/${1:-r06gring}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp -o run -- python3 bench.py --gc ot --base-ot --ot-ss-k 2 --table-ring32 --steps 1 --warmup 1 --no-cpu-baseline > $O/gcot1m.json 2> $O/gcot1m.err || { echo gcot failed; exit 1; }
find $O/tmp -name "*kernel_stats.csv" -exec cp {} $O/gcot1m_kernel_stats.csv \;
rm -rf $O/tmp
echo done
