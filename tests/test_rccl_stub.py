"""The in-process RCCL branch of one KeyCollection over several GPUs (fhh_create_multi: one
ncclCommInitAll clique, the grouped ncclGroupStart / ncclAllReduce / ncclGroupEnd of the node sums, the
device loop's per-level all-reduce from one thread per shard, ncclCommAbort when a shard fails —
fhh_comm.cpp, fhh_group.cpp; north_star: per-GPU partial counts combined by an RCCL all-reduce;
src/bin/server.rs:44-52,332-335 holds the one KeyCollection). Real RCCL refuses two ranks on one GPU,
so on a one-GPU box this branch runs against tests/stubs/librccl_stub.so, a test-only stand-in with
RCCL's signatures that sums on the host (loaded through fhh_rccl_load, FHH_GROUP_REDUCE=rccl forcing
the branch on a repeated device). Each run is a child process: a process loads one RCCL."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "stubs", "librccl_stub.so")


def test_stub_exports_what_fhh_comm_resolves():
    """The stand-in defines the 11 nccl* symbols fhh_comm.cpp dlsyms (CPU: symbol table only)."""
    import ctypes
    if not os.path.exists(STUB):
        pytest.skip("stub not built (__graft_entry__.build())")
    src = open(os.path.join(ROOT, "fuzzyheavyhitters_amd", "csrc", "fhh_comm.cpp")).read()
    import re
    wanted = set(re.findall(r'dlsym\(h, "(nccl\w+)"\)', src))
    assert len(wanted) == 11
    lib = ctypes.CDLL(STUB)
    for name in wanted:
        getattr(lib, name)   # raises AttributeError if missing


def _env(tmp_path, **extra):
    env = dict(os.environ)
    env.update({"FHH_TEST_RCCL_STUB": STUB, "FHH_GROUP_REDUCE": "rccl",
                "FHH_TEST_RCCL_STUB_STATS": str(tmp_path / "stub_stats.json")})
    env.update(extra)
    return env


@pytest.mark.gpu
def test_group_suite_through_the_rccl_branch(tmp_path):
    """test_group.py's GPU tests (drop-in path level by level, the device level loop in count / FE /
    GC + OT mode on 2 and 4 shards, placement, device-value sums, growth agreement) with the RCCL branch
    taken: the same results as one GPU. The stand-in's record shows both call shapes ran — grouped node
    sums (one op per shard, one ncclGroupEnd each) and the per-shard-thread level all-reduces — on
    the shards' own streams."""
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_group.py")], cwd=ROOT, env=_env(tmp_path),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    st = json.load(open(tmp_path / "stub_stats.json"))
    assert st["init_all"] >= 1 and st["grouped"] > 0 and st["group_ends"] > 0
    assert st["grouped"] % st["group_ends"] == 0 or st["grouped"] >= 2 * st["group_ends"]
    assert st["calls"] > st["grouped"]            # the device loop's ungrouped per-shard all-reduces
    assert st["streams"] >= 2                     # each shard on its own stream
    assert st["aborts"] == 0 and st["failed"] == 0
    print("rccl stand-in:", st)


_ABORT = r"""
import json, os, sys
sys.path.insert(0, {root!r})
import numpy as np
import fuzzyheavyhitters_amd as fhh
from fuzzyheavyhitters_amd import workload
from fuzzyheavyhitters_amd._lib import lib
import ctypes
assert lib().fhh_rccl_load({stub!r}.encode()) == 0
n, L = 64 * 13 + 5, 40
wl = workload.zipf_workload(n, L, 1, num_sites=20, seed=21)
s0, s1 = fhh.KeyCollection(L, 1), fhh.KeyCollection(L, 1)
g0, g1 = fhh.KeyCollection(L, 1, devices=[0, 0, 0]), fhh.KeyCollection(L, 1, devices=[0, 0, 0])
fhh.gen_keys_pair(s0, s1, wl.left, wl.right, wl.root_seeds)
fhh.gen_keys_pair(g0, g1, wl.left, wl.right, wl.root_seeds)
assert g0.shard_info()[1] == "rccl"
ref = fhh.sim_crawl(s0, s1, 0.01, mode="fe", prf_seed=9)
os.environ["FHH_RCCL_STUB_FAIL"] = "1:5"        # shard 1's 6th level all-reduce fails
err = None
try:
    fhh.sim_crawl(g0, g1, 0.01, mode="fe", prf_seed=9)
except fhh.FhhError as e:
    err = str(e)
del os.environ["FHH_RCCL_STUB_FAIL"]
st = (ctypes.c_uint64 * 10)()
S = ctypes.CDLL({stub!r})
S.fhh_rccl_stub_stats(st)
after_fail = list(st)
again = fhh.sim_crawl(g0, g1, 0.01, mode="fe", prf_seed=9)   # the aborted communicators are rebuilt
S.fhh_rccl_stub_stats(st)
same = (list(ref.level_children) == list(again.level_children) and
        [(r.path, r.value) for r in ref.final] == [(r.path, r.value) for r in again.final])
print(json.dumps({{"err": err, "after_fail": after_fail, "final": list(st), "same": same}}))
"""


@pytest.mark.gpu
def test_failing_shard_aborts_its_peers_and_the_collection_recovers(tmp_path):
    """One shard's all-reduce fails mid-crawl (injected): the failing shard's thread aborts every
    communicator of the clique once (ncclCommAbort), which releases the peers blocked in that level's
    collective; the crawl reports FHH_E_COMM instead of hanging, and the next crawl on the same
    collection rebuilds its communicators (a second ncclCommInitAll) and equals the one-GPU crawl."""
    code = _ABORT.format(root=ROOT, stub=STUB)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=_env(tmp_path), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # the error names the root cause: the shard whose all-reduce failed, not a peer it aborted
    assert out["err"] is not None and "shard 1 " in out["err"] and "injected" in out["err"], out
    init_all, _, _, _, _, aborts, _, _, _, failed = out["after_fail"]
    assert failed == 1 and aborts >= 2 and init_all >= 1, out   # every rank's communicator aborted once
    assert out["final"][0] == init_all + 1, out                  # rebuilt on the next use
    assert out["same"], out
