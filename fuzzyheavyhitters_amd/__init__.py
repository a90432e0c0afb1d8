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

__all__ = ["FhhError", "build", "lib", "KeyCollection", "Result", "gen_keys_pair", "sim_eq_count", "sim_ot_sums",
           "FE_P", "FE255_P", "SimResult", "sim_crawl",
           "RcclComm", "HostedComm", "load_rccl"]
