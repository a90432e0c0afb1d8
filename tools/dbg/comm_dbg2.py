import os, sys, socket
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch, torch.distributed as dist
sk = socket.socket(); sk.bind(("127.0.0.1", 0)); port = sk.getsockname()[1]; sk.close()
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
dist.init_process_group("gloo", rank=0, world_size=1)
torch.cuda.set_device(0)
import fuzzyheavyhitters_amd as fhh
from fuzzyheavyhitters_amd import workload
wl = workload.zipf_workload(300, 64, 1, num_sites=8, seed=91)
comm = fhh.RcclComm(0)
for name, kw in [("plain", {}), ("comm", dict(comm=comm)), ("callback", dict(distributed=True))]:
    c0, c1 = fhh.KeyCollection(64, 1), fhh.KeyCollection(64, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    print("==", name, flush=True)
    got = fhh.sim_crawl(c0, c1, 0.02, mode="count", prf_seed=3, init_capacity=2, **kw)
    print(name, got.level_children[:40].tolist(), flush=True)
    print(name, [c.tolist() for c in got.counts[:8]], flush=True)
comm.close()
dist.destroy_process_group()
