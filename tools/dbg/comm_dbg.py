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
c0, c1 = fhh.KeyCollection(64, 1), fhh.KeyCollection(64, 1)
fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
ref = fhh.sim_crawl(c0, c1, 0.02, mode="count", prf_seed=3)
print("ref children", ref.level_children[:20].tolist())
pre = fhh.RcclComm(0)
t = torch.arange(1000, dtype=torch.int64, device="cuda:0"); pre.allreduce_u64_(t); torch.cuda.synchronize(); pre.close()
comm = fhh.RcclComm(0)
for name, kw in [("dist-callback", dict(distributed=True)), ("comm-device", dict(comm=comm)),
                 ("comm-host", dict(comm=comm, host_loop=True))]:
    got = fhh.sim_crawl(c0, c1, 0.02, mode="count", prf_seed=3, **kw)
    ok = np.array_equal(got.level_children, ref.level_children)
    print(name, ok, got.level_children[:20].tolist())
    if not ok:
        for lv, (a, b) in enumerate(zip(got.counts, ref.counts)):
            if not np.array_equal(a, b):
                print("  first diff level", lv, "got", a[:8].tolist(), "ref", b[:8].tolist()); break
comm.close()
dist.destroy_process_group()
