"""fuzzyheavyhitters_amd — MI355X-native evaluator for the per-level client-key evaluation of
sks-codes/fuzzyheavyhitters (ibDCF tree crawl). See DESIGN.md.

The compute path is libfhh.so (hand-written HIP kernels for gfx950 behind the C ABI in
include/fhh.h); this package is the host-side mirror of the reference's KeyCollection API.
"""
from ._lib import FhhError, build, lib
from .comm import HostedComm, RcclComm, load_rccl
from .collection import KeyCollection, Result, gen_keys_pair, sim_eq_count, sim_ot_sums
from .fields import FE255_P, FE_P
from .sim import SimResult, sim_crawl
from .party import TwoPartyResult, two_party_crawl

__all__ = ["FhhError", "build", "lib", "KeyCollection", "Result", "gen_keys_pair", "sim_eq_count", "sim_ot_sums",
           "FE_P", "FE255_P", "SimResult", "sim_crawl",
           "RcclComm", "HostedComm", "load_rccl", "TwoPartyResult", "two_party_crawl", "shard_plan"]


def shard_plan(n_clients: int, n_shards: int):
    """[(client_base, n_clients)] per shard of a multi-device collection (fhh_shard_plan)."""
    import ctypes
    import numpy as np
    from ._lib import check, u64p
    b = np.zeros(n_shards, np.uint64)
    c = np.zeros(n_shards, np.uint64)
    check(lib().fhh_shard_plan(n_clients, n_shards, b.ctypes.data_as(u64p), c.ctypes.data_as(u64p)))
    return [(int(x), int(y)) for x, y in zip(b, c)]
