"""Native RCCL communicator (include/fhh.h fhh_comm_*).

One GPU per box here, and RCCL refuses two ranks on one device, so the native path is
exercised at world size 1 (identity sum, and a crawl through the comm equals the crawl
without it); the 2-rank exchange semantics are covered by test_distributed.py through the
host hook, and the N-GPU path by the driver's multi-GPU bench."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def world1():
    import torch
    import torch.distributed as dist
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    torch.cuda.set_device(0)
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_comm_allreduce_identity(world1):
    import torch
    import fuzzyheavyhitters_amd as fhh
    comm = fhh.RcclComm(0)
    try:
        t = torch.arange(1000, dtype=torch.int64, device="cuda:0") * 3 + (1 << 40)
        ref = t.clone()
        comm.allreduce_u64_(t)
        torch.cuda.synchronize()
        assert torch.equal(t, ref)
    finally:
        comm.close()


@pytest.mark.parametrize("mode", ["count", "fe"])
def test_sim_crawl_through_comm(world1, mode):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(300, 64, 1, num_sites=8, seed=91)
    c0, c1 = fhh.KeyCollection(64, 1), fhh.KeyCollection(64, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    ref = fhh.sim_crawl(c0, c1, 0.02, mode=mode, prf_seed=3)
    comm = fhh.RcclComm(0)
    try:
        for host_loop, cap in ((False, 2), (False, 0), (True, 0)):
            got = fhh.sim_crawl(c0, c1, 0.02, mode=mode, prf_seed=3, comm=comm, host_loop=host_loop,
                                init_capacity=cap)
            tag = f"host_loop={host_loop} init_capacity={cap}"
            assert np.array_equal(got.level_children, ref.level_children), \
                (tag, got.level_children[:24].tolist(), ref.level_children[:24].tolist())
            for lv, (a, b) in enumerate(zip(got.counts, ref.counts)):
                assert np.array_equal(a, b), (tag, lv, a[:8].tolist(), b[:8].tolist())
            assert [(r.path, r.value) for r in got.final] == [(r.path, r.value) for r in ref.final]
    finally:
        comm.close()
