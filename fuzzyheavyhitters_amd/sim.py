"""In-process leader + two servers (the reference's leader level loop, leader.rs:417-440),
with the servers' garbled-circuit equality test + OT (collect.rs:419-482, out of scope)
replaced by either plaintext equality of the two share strings (mode "count") or simulated
OT share values (mode "fe": r0 from a fixed PRF, r1 = r0 + 1, v0 = r1, v1 = eq ? r0 : r1).

Clients may be sharded across GPUs (one process per GPU): each rank holds both servers'
keys for its client range, and the per-child partial sums are all-reduced over RCCL (native
communicator on the engine stream, comm.py; or torch.distributed in a host callback) before
the leader's keep decision.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ._lib import ALLREDUCE_FN, FhhSimConfig, check, lib, u64p
from .collection import KeyCollection


@dataclass
class SimResult:
    level_children: np.ndarray
    level_kept: np.ndarray
    counts: list = field(default_factory=list)     # per level np.ndarray (mode count: counts; fe: v0-v1)
    final: list = field(default_factory=list)      # Result(path, value) from server 0's final_shares
    # probe: level -> (seeds [2][C][m][d][2][16], t [2][C][m][d][2], y [2][C][m][d][2]) of the
    # probed clients (server 0, server 1), read inside the device loop right after k_expand
    probe: dict = field(default_factory=dict)


class _TorchAllReduce:
    """Sum a device buffer across ranks with torch.distributed (backend nccl = RCCL)."""

    def __init__(self, capacity: int, device: int):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.buf = torch.zeros(capacity, dtype=torch.int64, device=f"cuda:{device}")
        self.cb = ALLREDUCE_FN(self._call)
        self.err = None

    def _call(self, ptr, count, user):
        try:
            view = self.buf[:count]
            if self.dist.get_backend() == "gloo":      # CPU rehearsal path: gloo reduces host tensors
                host = view.cpu()
                self.dist.all_reduce(host)
                view.copy_(host)
            else:
                self.dist.all_reduce(view)             # RCCL over xGMI; u64 partials fit
            self.torch.cuda.current_stream().synchronize()
            return 0
        except Exception as e:  # pragma: no cover - surfaced as FHH_E_CALLBACK
            self.err = e
            return 1


def sim_crawl(c0: KeyCollection, c1: KeyCollection, threshold: float, nclients_total: int | None = None,
              mode: str = "count", prf_seed: int = 0, levels: int = 0, record: bool = True,
              distributed: bool = False, xchg_capacity: int = 1 << 20, host_loop: bool = False,
              init_capacity: int = 0, comm=None, gc=False, probe: dict | None = None,
              base_ot: bool = False, ot_ss_k: int = 1, table_ring32: bool = False) -> SimResult:
    """Leader level loop over both servers' collections. Multi-rank runs (clients sharded)
    sum per-child partials across ranks either natively (`comm`: an RcclComm, all-reduce on
    the engine stream) or, with `distributed=True`, through torch.distributed in a host
    callback (synchronises once per level; the gloo rehearsal path uses this). `gc` (mode "fe",
    device loop) takes each (child, client) equality bit from the GPU garbled-circuit equality
    test (server 0 garbles, server 1 evaluates) instead of comparing shares: `True` / "ot" with
    the evaluator's labels and the FE shares moved by the GPU OT extension (base OTs ideal),
    "ideal" with both OTs ideal; "ot-circuit" as "ot" but the half-gates circuit (+ the output-label
    share) at every level instead of the FE levels' garbled table. `ot_ss_k` (gc "ot" / "ot-circuit", r06):
    1 = IKNP OT extension, 2 / 4 = SoftSpoken with k = ot_ss_k (128 / k rows of U on the wire). `table_ring32`
    (gc "ot", d = 1, r06): the FE levels' garbled table carries Z_2^32 shares (4-B rows) instead of FE ones.

    `probe` (parity tests) = {"levels": [...], "clients": [...], "capacity": C_max}: the device
    loop gathers those clients' EvalStates of every pending child right after each listed
    level's k_expand (res.probe)."""
    if ot_ss_k not in (1, 2, 4):
        raise ValueError("sim_crawl: ot_ss_k must be 1 (IKNP), 2 or 4 (SoftSpoken)")
    L = levels or c0.depth
    n_local = c0.num_clients()
    cfg = FhhSimConfig()
    cfg.threshold = threshold
    cfg.nclients_total = nclients_total if nclients_total is not None else n_local
    cfg.mode = {"count": 0, "fe": 1}[mode]
    cfg.levels = L
    cfg.prf_seed = prf_seed
    cfg.host_loop = 1 if host_loop else 0
    cfg.init_capacity = init_capacity
    cfg.gc = {False: 0, None: 0, "ideal": 1, True: 2, "ot": 2, "ot-circuit": 3}[gc]
    cfg.base_ot = 1 if base_ot else 0   # gc = "ot": Chou–Orlandi base OTs on the host (else ideal)
    cfg.ot_ss_k = ot_ss_k
    cfg.table_ring32 = 1 if table_ring32 else 0
    ar = None
    if comm is not None:
        cfg.comm = comm.handle
        cfg.allreduce = ALLREDUCE_FN()
    elif distributed:
        ar = _TorchAllReduce(xchg_capacity, c0.device)
        cfg.allreduce = ar.cb
        cfg.xchg_dev = ctypes.cast(ctypes.c_void_p(ar.buf.data_ptr()), u64p)
        cfg.xchg_capacity = xchg_capacity
    else:
        cfg.allreduce = ALLREDUCE_FN()
    lc = np.zeros(L, np.uint64)
    lk = np.zeros(L, np.uint64)
    cap = 1 << 22 if record else 0
    counts = np.zeros(max(cap, 1), np.uint64)
    cfg.level_children = lc.ctypes.data_as(u64p)
    cfg.level_kept = lk.ctypes.data_as(u64p)
    if record:
        cfg.counts = counts.ctypes.data_as(u64p)
        cfg.counts_capacity = cap
    if probe:
        d = c0.n_dims
        p_lv = np.ascontiguousarray(np.asarray(probe["levels"], np.uint32))
        p_cl = np.ascontiguousarray(np.asarray(probe["clients"], np.uint64))
        p_cap = int(probe["capacity"])
        m = p_cl.size
        p_seeds = np.zeros((p_lv.size, 2, p_cap, m, d, 2, 16), np.uint8)
        p_ty = np.zeros((p_lv.size, 2, p_cap, m, d, 2), np.uint8)
        p_C = np.zeros(p_lv.size, np.uint64)
        cfg.probe_n_levels = p_lv.size
        cfg.probe_n_clients = m
        cfg.probe_levels = p_lv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        cfg.probe_clients = p_cl.ctypes.data_as(u64p)
        cfg.probe_capacity = p_cap
        cfg.probe_seeds = p_seeds.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.probe_ty = p_ty.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.probe_children = p_C.ctypes.data_as(u64p)
    rc = lib().fhh_sim_crawl(c0.handle, c1.handle, ctypes.byref(cfg))
    if ar is not None and ar.err is not None:
        raise ar.err
    check(rc, c0.handle)
    res = SimResult(lc, lk)
    if probe:
        for k, lv in enumerate(p_lv):
            C = int(p_C[k])
            if C > p_cap:
                raise ValueError(f"probe: level {lv} has {C} children > capacity {p_cap}")
            res.probe[int(lv)] = (p_seeds[k, :, :C], p_ty[k, :, :C] & 1, p_ty[k, :, :C] >> 1)
    if record:
        off = 0
        for C in lc:
            res.counts.append(counts[off:off + int(C)].copy())
            off += int(C)
    if mode == "fe":
        # the leader's output: v0 - v1 mod p of the two servers' FieldElm shares (collect.rs:1007-1029)
        res.final = KeyCollection.final_values(c0.final_shares(), c1.final_shares())
    else:
        res.final = c0.final_shares()   # plaintext harness: server 0 holds the counts
    return res
