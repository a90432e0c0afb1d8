"""Native RCCL communicator for client-sharded crawls (include/fhh.h `fhh_comm_*`).

The per-level exchange (collect.rs:487-501 -> leader.rs:182-197: each server's Vec<FE> of
per-child sums) becomes, with clients sharded over GPUs, one ncclAllReduce(sum, u64) of the
per-child limb partials. The library enqueues it on the engine's own stream, so the
device-resident level loop runs a whole crawl with no host synchronisation per level.

The unique id is created by rank 0 and broadcast over torch.distributed's default group (the
bench uses a gloo group for this control traffic, so RCCL carries only the data path);
RCCL itself is the copy torch already loaded (so one RCCL instance serves the process).
"""
from __future__ import annotations

import ctypes
import os

from ._lib import ALLREDUCE_FN, FhhError, lib, u8p


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

    def info(self):
        """(ranks, rank) as RCCL reports them for this communicator."""
        nr, rk = ctypes.c_int(), ctypes.c_int()
        _comm_check(lib().fhh_comm_info(self.handle, ctypes.byref(nr), ctypes.byref(rk)))
        return nr.value, rk.value

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().fhh_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort at interpreter exit
        try:
            self.close()
        except Exception:
            pass


class HostedComm(RcclComm):
    """The level loop's `cfg.comm` path without RCCL (fhh_comm_create_hosted): partials are summed
    on the host through torch.distributed (e.g. gloo). For multi-rank tests on one GPU, where
    RCCL cannot place two ranks on one device."""

    def __init__(self, device: int):
        import numpy as np
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.device = dist.get_rank(), dist.get_world_size(), device
        self.err = None

        def _sum(buf, count, user):
            try:
                a = np.ctypeslib.as_array(buf, shape=(count,))
                t = torch.from_numpy(a.view(np.int64).copy())
                dist.all_reduce(t)
                a[:] = t.numpy().view(np.uint64)
                return 0
            except Exception as e:  # pragma: no cover - surfaced as FHH_E_CALLBACK
                self.err = e
                return 1

        self._cb = ALLREDUCE_FN(_sum)
        h = ctypes.c_void_p()
        _comm_check(lib().fhh_comm_create_hosted(ctypes.byref(h), self.world, self.rank, device, self._cb, None))
        self.handle = h
