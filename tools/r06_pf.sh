set -u
# r06: the table kernels' next-tile L2 touch (FHH_GT_PF 0 / 2 = evaluator / 3 = both), 1M protocol crawl kernel stats
O=gpurun_out/r06pf; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for v in 0 2 3; do
  FHH_LIB_PATH=ab_builds/libfhh_pf$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tmp -o run -- python3 bench.py --gc ot --base-ot --steps 1 --warmup 1 --no-cpu-baseline > $O/pf${v}_$r.json 2> $O/pf${v}_$r.err || { echo pf $v failed; exit 1; }
  find $O/tmp -name "*kernel_stats.csv" -exec cp {} $O/pf${v}_${r}_stats.csv \;
  rm -rf $O/tmp
  python3 - $O/pf${v}_${r}_stats.csv $v $r <<'PY'
import csv, sys
rows = {r["Name"]: r for r in csv.DictReader(open(sys.argv[1]))}
g = [v for k, v in rows.items() if "k_gt_garble_tm" in k][0]
e = [v for k, v in rows.items() if "k_gt_eval_tm" in k][0]
print("pf", sys.argv[2], "round", sys.argv[3], "garble avg us", round(float(g["AverageNs"]) / 1e3, 1), "eval avg us", round(float(e["AverageNs"]) / 1e3, 1))
PY
done; done
