set -u
# r06: configs[3] with kMwItemsPerWave 2 / 4 (default) / 8 / 16 (item_layout's narrow-level items per wave), 2 rounds
O=gpurun_out/r06ipw; mkdir -p $O
for r in 1 2; do for v in 4 8 16 2; do
  FHH_LIB_PATH=ab_builds/libfhh_ipw$v.so timeout -k 10 200 python3 bench.py --workload coords --steps 20 --warmup 2 --no-cpu-baseline > $O/ipw${v}_$r.json 2> $O/ipw${v}_$r.err || { echo ipw $v failed; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ipw${v}_$r.json').read().strip().splitlines()[-1]); print('ipw $v r $r', round(d['roofline']['frac'],4), round(d['ms_per_step'],3))"
done; done
