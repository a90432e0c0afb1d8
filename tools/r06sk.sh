set -u
# r06: k_sketch_fe A/B forms at configs[4] (fhh_sketch_set_impl 0 default, 5 = 512 threads x 4 blocks, 6 = 512 x 3,
# 7 = 1024 x 3), two rounds
O=gpurun_out/${1:-r06sk}; mkdir -p $O
for rep in 1 2; do for i in 0 5 6 7; do
  timeout -k 10 200 python3 bench.py --workload sketch --sketch-impl $i --steps 5 --warmup 2 > $O/sk_${i}_$rep.json 2> $O/sk_${i}_$rep.err || { echo impl $i failed; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sk_${i}_$rep.json').read().strip().splitlines()[-1]); print('impl $i rep $rep', d['ms_per_step'])"
done; done
echo done
