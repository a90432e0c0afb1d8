"""Client-sharded crawl across ranks: each rank holds both servers' keys for a
contiguous client range; per level the per-child partial sums are all-reduced before the
leader's keep decision. CPU tests run the protocol with gloo (world_size 2) over the oracle;
the GPU test runs fhh_sim_crawl's all-reduce hook with 2 ranks sharing cuda:0."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _collect(procs, q, timeout):
    """Wait for rank 0's result, failing fast if any rank dies."""
    import queue
    import time
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            return q.get(timeout=1.0)
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                for p in procs:
                    if p.is_alive():
                        p.kill()
                raise AssertionError(f"a rank failed: exit codes {[p.exitcode for p in procs]}")
    raise AssertionError("timed out waiting for rank 0")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def sharded_oracle_crawl(rank, world, wl_args, thr, mode, out):
    """The leader level loop of fhh_sim_crawl, restated over the oracle with torch.distributed
    partial-sum all-reduce (u64 limbs, then one modular reduction)."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from fuzzyheavyhitters_amd import workload
    from oracle import oracle as O
    n_total = wl_args["n"]
    n_local = n_total // world
    base = rank * n_local
    wl = workload.zipf_workload(n_local, wl_args["L"], wl_args["d"], num_sites=wl_args["sites"],
                                seed=wl_args["seed"], client_offset=base)
    k0, k1 = O.gen_keys(wl.left, wl.right, wl.root_seeds, nthreads=1)
    d, L = wl_args["d"], wl_args["L"]
    thr64 = max(1, int(thr * n_total))
    s0, s1 = O.tree_init(k0), O.tree_init(k1)
    parents = np.zeros(1, np.uint64)
    counts_all, children = [], []
    final = []
    paths = [tuple(() for _ in range(d))]
    for lvl in range(L):
        last = lvl == L - 1
        c0, _ = O.level_expand(k0, s0, parents, lvl, nthreads=1)
        c1, _ = O.level_expand(k1, s1, parents, lvl, nthreads=1)
        C = c0.t.shape[0]
        eqm = np.all(O.share_bits(c0) == O.share_bits(c1), axis=-1)
        if mode == "count":
            part = torch.tensor(eqm.sum(axis=1).astype(np.int64))
            dist.all_reduce(part)
            vals = part.numpy().astype(np.uint64)
        else:   # FE limbs of the simulated OT shares, global client indices
            r0 = O.sim_r0_fe(7, lvl, C, base + n_local)[:, base:]
            r1 = (r0 + np.uint64(1)) % np.uint64(O.FE_P)
            v1 = np.where(eqm, r0, r1)
            limbs = np.stack([(r1 & np.uint64(0xFFFFFFFF)).sum(1), (r1 >> np.uint64(32)).sum(1),
                              (v1 & np.uint64(0xFFFFFFFF)).sum(1), (v1 >> np.uint64(32)).sum(1)], 1)
            part = torch.tensor(limbs.astype(np.int64))
            dist.all_reduce(part)
            p = part.numpy().astype(object)
            a = [(int(p[c, 0]) + (int(p[c, 1]) << 32)) % O.FE_P for c in range(C)]
            b = [(int(p[c, 2]) + (int(p[c, 3]) << 32)) % O.FE_P for c in range(C)]
            vals = np.array([(x - y) % O.FE_P for x, y in zip(a, b)], np.uint64)
        keep = vals >= thr64
        counts_all.append(vals)
        children.append(C)
        child_paths = [tuple(p[j] + ((i >> j) & 1,) for j in range(d)) for p in paths for i in range(1 << d)]
        kept = np.nonzero(keep)[0]
        paths = [child_paths[k] for k in kept]
        parents = kept.astype(np.uint64)
        s0, s1 = c0, c1
        if last:
            final = paths
    if rank == 0:
        out.put((children, [v.tolist() for v in counts_all], final))


def _worker(rank, world, port, wl_args, thr, mode, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sharded_oracle_crawl(rank, world, wl_args, thr, mode, q)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["count", "fe"])
def test_sharded_crawl_equals_single_process(oracle, mode):
    from fuzzyheavyhitters_amd import workload
    wl_args = {"n": 96, "L": 40, "d": 1, "sites": 5, "seed": 31}
    thr = 0.03
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, wl_args, thr, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    children, counts, final = _collect(procs, q, 240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    wl = workload.zipf_workload(wl_args["n"], wl_args["L"], 1, num_sites=wl_args["sites"], seed=wl_args["seed"])
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ref = oracle.crawl(k0, k1, thr, mode="count")
    assert children == list(ref.n_children)
    assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in ref.counts]
    assert sorted(final) == sorted(tuple(tuple(int(b) for b in pj) for pj in p) for p in ref.final_paths)


def _gpu_worker(rank, world, port, wl_args, thr, mode, q, host_loop=False, init_capacity=0, gc=False,
                hosted_comm=False, tight_rank1=False):
    import sys
    sys.path.insert(0, ROOT)
    if tight_rank1:
        # rank 0 sees ample memory, rank 1 none: the growth choice must be agreed over the callback
        # all-reduce (loop_entry_cap), or the ranks' collectives would stop pairing up
        os.environ["FHH_TEST_TABLE_BYTES"] = f"{1 << 40},0"
        os.environ["FHH_TEST_RANK"] = str(rank)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        import fuzzyheavyhitters_amd as fhh
        from fuzzyheavyhitters_amd import workload
        n_local = wl_args["n"] // world
        wl = workload.zipf_workload(n_local, wl_args["L"], wl_args["d"], num_sites=wl_args["sites"],
                                    seed=wl_args["seed"], client_offset=rank * n_local)
        c0 = fhh.KeyCollection(wl_args["L"], wl_args["d"])
        c1 = fhh.KeyCollection(wl_args["L"], wl_args["d"])
        fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
        c0.set_client_base(rank * n_local)
        c1.set_client_base(rank * n_local)
        comm = fhh.HostedComm(0) if hosted_comm else None
        if comm is not None:
            assert comm.info() == (world, rank)
        res = fhh.sim_crawl(c0, c1, thr, nclients_total=wl_args["n"], mode=mode, prf_seed=7,
                            distributed=comm is None, comm=comm, host_loop=host_loop, init_capacity=init_capacity,
                            gc=gc)
        if rank == 0:
            q.put((res.level_children.tolist(), [c.tolist() for c in res.counts],
                   sorted(tuple(tuple(int(b) for b in pj) for pj in r.path) for r in res.final)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,loop", [("count", "device_grow"), ("count", "host"), ("fe", "device_grow"),
                                       ("fe", "host"), ("fe", "device_gc_ot"), ("count", "comm_grow"),
                                       ("fe", "comm_grow"), ("fe", "comm_host"), ("count", "device_grow_tight"),
                                       ("fe", "comm_grow_tight")])
def test_gpu_two_ranks_allreduce_hook(oracle, mode, loop):
    """Two ranks share one GPU over the host all-reduce hook. device_grow starts the device
    loop at capacity 2 so it aborts and resumes several times: the cross-rank sum of an
    aborted level must not be applied twice (out-of-place reduction). comm_* drive the level
    loop's native-communicator path (cfg.comm, the path bench.py takes at N > 1) with a hosted
    communicator (fhh_comm_create_hosted: the sum over gloo instead of RCCL, which cannot put two
    ranks on one GPU). *_tight: rank 1 has no memory for table growth (FHH_TEST_TABLE_BYTES /
    FHH_TEST_RANK), so the growth capacity must be agreed over the reduction — the callback hook's
    (device_grow_tight) as well as the communicator's (comm_grow_tight)."""
    from fuzzyheavyhitters_amd import workload
    wl_args = {"n": 256, "L": 48, "d": 1, "sites": 6, "seed": 77}
    thr = 0.02
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    kw = {"host_loop": loop in ("host", "comm_host"), "init_capacity": 2 if "grow" in loop else 0,
          "gc": "ot" if loop == "device_gc_ot" else False, "hosted_comm": loop.startswith("comm"),
          "tight_rank1": loop.endswith("_tight")}
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, wl_args, thr, mode, q), kwargs=kw) for r in range(2)]
    for p in procs:
        p.start()
    children, counts, final = _collect(procs, q, 300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    wl = workload.zipf_workload(wl_args["n"], wl_args["L"], 1, num_sites=wl_args["sites"], seed=wl_args["seed"])
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ref = oracle.crawl(k0, k1, thr, mode=mode, sim_seed=7)
    assert children == list(ref.n_children)
    if mode == "count":
        assert [list(map(int, c)) for c in counts] == [list(map(int, c)) for c in ref.counts]
    assert final == sorted(tuple(tuple(int(b) for b in pj) for pj in p) for p in ref.final_paths)
