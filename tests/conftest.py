import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    # tests/test_rccl_stub.py runs test_group.py in a child process with the test-only RCCL stand-in
    # (tests/stubs/librccl_stub.so) as the process's RCCL and FHH_GROUP_REDUCE=rccl, so the in-process
    # RCCL branch of a multi-device collection executes on one GPU
    stub = os.environ.get("FHH_TEST_RCCL_STUB")
    if stub:
        from fuzzyheavyhitters_amd._lib import lib
        rc = lib().fhh_rccl_load(stub.encode())
        assert rc == 0, lib().fhh_comm_last_error()


def pytest_sessionfinish(session, exitstatus):
    out = os.environ.get("FHH_TEST_RCCL_STUB_STATS")
    if out and os.environ.get("FHH_TEST_RCCL_STUB"):
        import ctypes
        import json
        st = (ctypes.c_uint64 * 10)()
        ctypes.CDLL(os.environ["FHH_TEST_RCCL_STUB"]).fhh_rccl_stub_stats(st)
        keys = ["init_all", "init_rank", "calls", "grouped", "group_ends", "aborts", "destroys", "max_count",
                "streams", "failed"]
        with open(out, "w") as f:
            json.dump(dict(zip(keys, list(st))), f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def fhh():
    import fuzzyheavyhitters_amd as f
    return f
