"""Native RCCL communicator for client-sharded crawls (include/fhh.h `fhh_comm_*`).

The per-level exchange (collect.rs:487-501 -> leader.rs:182-197: each server's Vec<FE> of
per-child sums) becomes, with clients sharded over GPUs, one ncclAllReduce(sum, u64) of the
per-child limb partials. The library enqueues it on the engine's own stream, so the
device-resident level loop runs a whole crawl with no host synchronisation per level.

The unique id is created by rank 0 and broadcast over torch.distributed's default group;
RCCL itself is the copy torch already loaded (so one RCCL instance serves the process).
"""
from __future__ import annotations

import ctypes
import os

from ._lib import FhhError, lib, u8p


def _comm_check(rc: int):
    if rc != 0:
        msg = lib().fhh_comm_last_error()
        raise FhhError(f"fhh comm error {rc}: {msg.decode() if msg else ''}")


def load_rccl() -> None:
    """Load the RCCL torch uses (torch/lib/librccl.so) if present, else the system one."""
    path = None
    try:
        import torch
        cand = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if os.path.exists(cand):
            path = cand
    except ImportError:  # pragma: no cover
        pass
    _comm_check(lib().fhh_rccl_load(path.encode() if path else None))


class RcclComm:
    """One RCCL communicator over all ranks of the default torch.distributed group."""

    def __init__(self, device: int, rank: int | None = None, world: int | None = None):
        import torch.distributed as dist
        load_rccl()
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.device = device
        uid = (ctypes.c_uint8 * 128)()
        if self.rank == 0:
            _comm_check(lib().fhh_comm_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        _comm_check(lib().fhh_comm_create(ctypes.byref(h), self.world, self.rank,
                                          ctypes.cast(uid, u8p), device))
        self.handle = h

    def allreduce_u64_(self, t) -> None:
        """In-place sum of a cuda int64/uint64 torch tensor across ranks (on its current stream)."""
        import torch
        stream = torch.cuda.current_stream(t.device).cuda_stream
        _comm_check(lib().fhh_comm_allreduce_u64(self.handle, ctypes.c_void_p(t.data_ptr()),
                                                 ctypes.c_void_p(t.data_ptr()), t.numel(), ctypes.c_void_p(stream)))

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().fhh_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort at interpreter exit
        try:
            self.close()
        except Exception:
            pass
