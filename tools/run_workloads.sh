set -e
O=${1:-gpurun_out/wl}; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
$B --workload coords --clients 1000000 --dims 2 --data-len 16 --threshold 0.075 --steps 5 > $O/coords.json 2> $O/coords.err
$B --clients 125000 --steps 10 > $O/zipf_125k.json 2> $O/zipf_125k.err
$B --clients 100000 --steps 10 > $O/zipf_100k.json 2> $O/zipf_100k.err
$B --clients 100000 --mode fe --gc ot --steps 2 > $O/gc_ot_100k.json 2> $O/gc_ot_100k.err
$B --workload sketch --steps 3 > $O/sketch.json 2> $O/sketch.err
echo done
