#!/bin/bash
# One parameterised GPU-box session (replaces r02-r03's per-session lease scripts). Run from the repo
# root on the box:   tools/gpu_session.sh <outdir> <step> [<step> ...]
# Steps (each under its own time limit; the session stops at the first failing step):
#   tests        pytest -m gpu, the whole suite                     -> gpu_tests.log
#   smoke        __graft_entry__.smoke()                             -> smoke.log
#   bench        the driver's line: bench.py --gpus 1 --steps 20 --warmup 5   -> bench.json / bench.err
#   final        tests + smoke + bench (the driver's round-end sequence)
#   stats        rocprofv3 --kernel-trace --stats of bench.py --steps 5 --warmup 1 -> kernel_stats.csv
#   pmc          the PMC passes of tools/pmc_passes.sh on the default bench  -> gpurun_out/pmc_<basename outdir>/
#   gcot1m       bench.py --gc ot --base-ot at the metric's 1M clients (kernel stats)  -> gcot1m_*
#   sketch       bench.py --workload sketch (configs[4]) under rocprofv3 --stats        -> sketch_*
#   dropin       bench.py --workload dropin --clients 100000 (configs[1])              -> dropin.json
#   dropin1m     the same at the metric's 1M clients (chunked party protocol), 1 warm-up + 1 timed rep  -> dropin1m.json
#   workloads    configs[1], configs[3], bincode, gc one-level lines                   -> wl_*.json
set -u
O=${1:?outdir}; shift
mkdir -p "$O"
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
stats_of() {   # stats_of <tag> <limit s> <bench args...>: rocprofv3 kernel stats of one bench.py run
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tmp_$tag" -o run \
      -- python3 bench.py "$@" > "$O/${tag}.json" 2> "$O/${tag}.err" || return $?
  find "$O/tmp_$tag" -name "*kernel_stats.csv" -exec cp {} "$O/${tag}_kernel_stats.csv" \;
  rm -rf "$O/tmp_$tag"
}
for s in "$@"; do
  case $s in
    tests) step tests bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1" ;;
    smoke) step smoke bash -c "timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" ;;
    bench) step bench bash -c "timeout -k 10 580 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err" ;;
    final) "$0" "$O" tests smoke bench || exit $? ;;
    stats) step stats stats_of stats 400 --steps 5 --warmup 1 --no-protocol-crawl ;;
    pmc) step pmc bash tools/pmc_passes.sh "$(basename "$O")" --steps 2 --warmup 1 --no-cpu-baseline --no-protocol-crawl ;;
    gcot1m) step gcot1m stats_of gcot1m 400 --gc ot --base-ot --steps 1 --warmup 0 --no-cpu-baseline ;;
    sketch) step sketch stats_of sketch 300 --workload sketch --steps 3 --warmup 1 ;;
    dropin) step dropin bash -c "timeout -k 10 600 python3 bench.py --workload dropin --clients 100000 --steps 2 --warmup 1 > $O/dropin.json 2> $O/dropin.err" ;;
    dropin1m) step dropin1m bash -c "timeout -k 10 1000 python3 -u bench.py --workload dropin --clients 1000000 --steps 1 --warmup 1 > $O/dropin1m.json 2> $O/dropin1m.err" ;;
    workloads)
      step configs1 bash -c "timeout -k 10 300 python3 bench.py --clients 100000 --steps 5 --warmup 1 --no-cpu-baseline > $O/wl_configs1.json 2> $O/wl_configs1.err"
      step configs3 bash -c "timeout -k 10 300 python3 bench.py --workload coords --steps 5 --warmup 1 --no-cpu-baseline > $O/wl_configs3.json 2> $O/wl_configs3.err"
      step bincode bash -c "timeout -k 10 300 python3 bench.py --workload bincode --clients 1000000 --steps 3 --warmup 1 > $O/wl_bincode.json 2> $O/wl_bincode.err"
      step gc bash -c "timeout -k 10 300 python3 bench.py --workload gc --steps 5 --warmup 1 > $O/wl_gc.json 2> $O/wl_gc.err" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
