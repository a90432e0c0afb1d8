#!/bin/bash
# r03k: end-to-end same-box A/B, session-start build (ab_builds/libfhh_base.so, commit 37a1703) vs
# the current tree (libfhh_new.so), no profiler: configs[1] crawl with GC + OT every level, and configs[4].
set -u
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step gcot bash tools/ab_builds.sh e2e_gcot 2 --clients 100000 --gc ot --steps 3 --warmup 1 --no-cpu-baseline
step sketch bash tools/ab_builds.sh e2e_sketch 2 --workload sketch --steps 3 --warmup 1
echo done
