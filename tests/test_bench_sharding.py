"""bench.py's multi-rank plan on the CPU: the strong-scaling shard of the 1M-client population
(configs[2] at 8 ranks), the per-rank workload slices, and the max-over-ranks / sum-over-ranks
aggregation over a gloo world of 2 (the control group bench.py uses at N > 1)."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("n,world", [(1_000_000, 8), (1_000_000, 3), (100_000, 2), (7, 4), (1000, 1)])
def test_shard_covers_population(n, world):
    import bench
    ranges = [bench.shard(n, world, r) for r in range(world)]
    assert ranges[0][0] == 0
    for (b0, n0), (b1, _) in zip(ranges, ranges[1:]):
        assert b0 + n0 == b1
    assert sum(k for _, k in ranges) == n
    assert max(k for _, k in ranges) - min(k for _, k in ranges) <= 1


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from fuzzyheavyhitters_amd import workload
        n = 1000
        base, k = bench.shard(n, world, rank)
        wl = workload.zipf_workload(k, 64, 1, num_sites=50, seed=0x5EED, client_offset=base)
        parts = [None] * world
        dist.all_gather_object(parts, (base, wl.left, wl.root_seeds))
        elapsed = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        blocks = torch.tensor([10 * (rank + 1)], dtype=torch.int64)
        dist.all_reduce(blocks)
        if rank == 0:
            q.put((parts, float(elapsed.item()), int(blocks.item())))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_plan_and_aggregation():
    import socket
    from fuzzyheavyhitters_amd import workload
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    parts, elapsed, blocks = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = workload.zipf_workload(1000, 64, 1, num_sites=50, seed=0x5EED)
    assert [b for b, _, _ in parts] == [0, 500]
    assert np.array_equal(np.concatenate([l for _, l, _ in parts]), full.left)
    assert np.array_equal(np.concatenate([r for _, _, r in parts]), full.root_seeds)
    assert elapsed == 1.5 and blocks == 30


def _bench_line(cmd, timeout=240):
    import json
    import subprocess
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_equals_one_rank():
    """bench.py's N > 1 path end to end on one GPU: two torchrun ranks share the device
    (--rehearse: the per-level all-reduce through the hosted communicator, RCCL cannot put two
    ranks on one GPU). The sharded crawl must recover exactly the single-rank run's frontier and
    heavy hitters, and the JSON line must aggregate over both ranks."""
    import random
    import sys as _sys
    common = ["--clients", "20000", "--data-len", "128", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench_line([_sys.executable, "-u", "bench.py", *common])
    port = str(29600 + random.randrange(300))
    two = _bench_line([_sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2", "--rehearse",
                       *common])
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["collective"]["comm_ranks"] == 2 and "rehearsal" in two
    for k in ("final_heavy_hitters", "children_total", "levels", "aes_blocks_per_step"):
        assert two[k] == one[k], k
    assert two["config"]["clients_total"] == one["config"]["clients_total"] == 20000
    # the real protocol's crawl (GC + OT + real base OTs every level) over the two ranks' shards with
    # the per-level all-reduce: the same heavy hitters as the plaintext headline and as one rank
    for line in (one, two):
        assert line["protocol_crawl"]["heavy_hitters_equal_headline"], line["protocol_crawl"]
    assert two["protocol_crawl"]["heavy_hitters"] == one["protocol_crawl"]["heavy_hitters"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_configs2_eight_rank_rehearsal_equals_golden():
    """configs[2] — the metric's 1M Zipf clients sharded over 8 ranks — through bench.py's own N = 8
    path on one GPU (--rehearse: 8 torchrun ranks share the device, the per-level all-reduce of the
    partials through the hosted communicator): the sharded crawl recovers the north star's output
    exactly as the committed 1M golden fixture holds it (tests/golden/zipf_1m_L512.npz: 101 998
    children over the 512 levels, 206 heavy hitters), and the line aggregates the 8 ranks. Only
    RCCL's xGMI transport differs on an 8-GPU node."""
    import random
    import sys as _sys
    g = np.load(os.path.join(ROOT, "tests", "golden", "zipf_1m_L512.npz"), allow_pickle=False)
    port = str(29000 + random.randrange(300))
    line = _bench_line([_sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "8", "--rehearse",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-protocol-crawl"], timeout=540)
    assert line["n_gpus"] == 8 and line["config"]["collective"]["comm_ranks"] == 8
    assert line["config"]["clients_total"] == 1_000_000 and line["config"]["clients_per_gpu"] == 125_000
    assert line["levels"] == 512
    assert line["children_total"] == int(g["level_children"].sum()) == 101_998
    assert line["final_heavy_hitters"] == len(g["paths"]) == 206
    assert line["aes_blocks_per_step"] == 101_998 * 1_000_000 * 4   # children x clients x 2 sides x 2 servers


@pytest.mark.gpu
def test_bench_two_rank_rccl_bootstrap_and_fallback():
    """The RCCL leg of bench.py's N > 1 path on one GPU (--rehearse-rccl): two torchrun ranks build
    the RCCL communicator over the loopback bootstrap bench.py configures; RCCL then refuses two ranks
    on one device (its duplicate-GPU check runs after the bootstrap's all-gather, so reaching it means
    the unique id, the sockets and the rank exchange worked), both ranks see the error and fall back
    together to the hosted communicator, and the crawl still equals the single-rank run."""
    import random
    import sys as _sys
    common = ["--clients", "20000", "--data-len", "128", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
    one = _bench_line([_sys.executable, "-u", "bench.py", *common])
    port = str(29300 + random.randrange(300))
    two = _bench_line([_sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                       "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "2",
                       "--rehearse-rccl", *common])
    col = two["config"]["collective"]
    assert "RCCL init failed" in col["kind"], col
    assert "ncclCommInitRank" in col["rccl_error"], col
    assert col["comm_ranks"] == 2
    for k in ("final_heavy_hitters", "children_total", "levels", "aes_blocks_per_step"):
        assert two[k] == one[k], k


def test_launch_plan_refuses_a_world_that_differs_from_gpus():
    """bench.py decides how it runs before any GPU call: a torchrun world that is not --gpus, or more
    GPUs than the node shows, exits non-zero; --gpus N > 1 without a torchrun world relaunches itself
    as N ranks (one node, rendezvous on 127.0.0.1)."""
    import bench
    assert bench.launch_plan(1, {}, 1, False) == ("run", None)
    assert bench.launch_plan(1, {}, 0, False) == ("run", None)
    assert bench.launch_plan(8, {}, 8, False) == ("relaunch", None)
    assert bench.launch_plan(8, {}, 1, True) == ("relaunch", None)          # rehearsal shares the GPU
    how, why = bench.launch_plan(8, {}, 1, False)
    assert how == "error" and "only 1 GPU" in why
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}, 8, False) == ("run", None)
    how, why = bench.launch_plan(8, {"WORLD_SIZE": "1"}, 8, False)
    assert how == "error" and "WORLD_SIZE=1" in why
    how, _ = bench.launch_plan(1, {"WORLD_SIZE": "4"}, 8, False)
    assert how == "error"
    how, _ = bench.launch_plan(4, {"WORLD_SIZE": "4"}, 1, False)
    assert how == "error"
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, 1, True) == ("run", None)
    cmd = bench.relaunch_cmd(["--gpus", "8", "--steps", "3"], 8, 29555)
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_rccl_init_failure_fails_the_measurement():
    """An RCCL init error on any rank ends every rank with a non-zero exit unless the run is the
    one-GPU --rehearse-rccl rehearsal (which falls back to the hosted all-reduce and says so)."""
    import bench
    assert bench.collective_after_init([None, None], False) == ("rccl", None)
    assert bench.collective_after_init([None, "ncclCommInitRank: invalid usage"], False) == \
        ("fail", "ncclCommInitRank: invalid usage")
    assert bench.collective_after_init(["x", "x"], True) == ("hosted", "x")


@pytest.mark.parametrize("world,gpus", [("3", "2"), ("1", "8")])
def test_bench_exits_nonzero_on_world_mismatch(world, gpus):
    """The guard runs before any GPU call: on this GPU-less container the process exits 2 with the
    reason, no JSON line."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", gpus, "--steps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r.stderr[-2000:]
    assert f"WORLD_SIZE={world} but --gpus={gpus}" in r.stderr
    assert r.stdout.strip() == ""
