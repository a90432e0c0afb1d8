#!/bin/bash
# configs[2] rehearsal on one GPU: bench.py's N = 8 path (1M clients sharded over 8 ranks, the
# per-level all-reduce through the hosted communicator) against the N = 1 run of the same
# population. Usage: tools/rehearse_n8.sh <outdir> [ranks] [mode]; mode --rehearse (default) or
# --rehearse-rccl (the ranks first bootstrap the RCCL communicator, which then refuses N ranks on one
# GPU, and fall back together to the hosted all-reduce).
set -u
O=${1:-gpurun_out/reh8}; N=${2:-8}; MODE=${3:---rehearse}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/n1.json 2> $O/n1.err || exit $?
echo "n1 rc=0"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 29611 bench.py --gpus $N $MODE --steps 1 --warmup 1 --no-cpu-baseline \
    > $O/n$N.json 2> $O/n$N.err || exit $?
echo "n$N rc=0"
python - "$O" "$N" <<'PY'
import json, sys
o, n = sys.argv[1], sys.argv[2]
a = json.loads(open(f"{o}/n1.json").read().strip().splitlines()[-1])
b = json.loads(open(f"{o}/n{n}.json").read().strip().splitlines()[-1])
keys = ("final_heavy_hitters", "children_total", "levels", "aes_blocks_per_step")
same = all(a[k] == b[k] for k in keys)
print(json.dumps({"same": same, **{k: (a[k], b[k]) for k in keys}, "ranks": b["config"]["collective"]}))
sys.exit(0 if same else 1)
PY
