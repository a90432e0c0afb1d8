#!/bin/bash
# Same-box A/B of k_expand variants through bench.py (interleaved rounds), per workload.
# Usage: tools/ab_bench_variants.sh <outdir> <variantA> <variantB> [rounds]
set -u
O=${1:-gpurun_out/ab}; A=${2:-34}; B=${3:-51}; R=${4:-2}
mkdir -p $O
run() {  # tag, variant, args...
  local tag=$1 v=$2; shift 2
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant $v "$@" > $O/${tag}_v${v}_r$r.json 2> $O/${tag}_v${v}_r$r.err
  local rc=$?
  echo "$tag v$v r$r rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
}
for r in $(seq 1 $R); do
  for v in $A $B; do
    run coords $v --workload coords --steps 10
    run z100k $v --clients 100000 --steps 10
    run z125k $v --clients 125000 --steps 10
    run z1m $v --steps 3
  done
done
echo done
