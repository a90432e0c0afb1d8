#!/usr/bin/env python3
"""Benchmark of the per-level ibDCF client-key evaluation (BASELINE.json metric:
"client x prefix key evals/sec (AES blocks/s) + full-crawl wall time, 1M clients").

One step = one full crawl (data_len levels) of the in-process leader + both servers:
GPU keys already resident in HBM; per level: k_expand for both servers (one launch),
the plaintext equality count standing in for the GC/OT step, [RCCL all-reduce of the
per-child partial counts when N > 1], leader keep decision, prune. Default workload = the
metric's: 1M Zipf clients IN TOTAL (num_sites 10000, s = 1.03), data_len 512, d = 1, ball 1,
threshold 0.001, sharded by client over the ranks (strong scaling; at 8 GPUs this is
configs[2]). `--clients 100000` is configs[1]. The CPU baseline is configs[0] exactly.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LDS_PEAK_GBPS = 75_000.0       # ds_read_b32 aggregate, MI355X_MICROARCH.md §LDS (≈75 TB/s)
HBM_PEAK_GBPS = 8_000.0        # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TOPS = 78.64         # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (confirmed by fhh_microbench)
LDS_BYTES_PER_BLOCK = 160 * 4  # T-table AES-128: 10 rounds x 16 ds_read_b32 lookups
VALU_OPS_PER_BLOCK = 400       # SURVEY §8d canonical int32 ops per AES block
HBM_BYTES_PER_BLOCK = 42       # SURVEY §8d algorithmic bytes per AES block


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Threads the CPU baselines use, and why: the CPUs this process may run on
    (os.sched_getaffinity), capped by OMP_NUM_THREADS when the environment sets it — the GPU box
    exports 16, one GPU's share of its host, and the box's other CPUs belong to the other GPUs'
    jobs."""
    avail = len(os.sched_getaffinity(0))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        n = min(env, avail)
        return n, (f"OMP_NUM_THREADS={env} (one GPU's share of the host's {os.cpu_count()} CPUs), "
                   f"{avail} CPUs in this process's affinity mask")
    return avail, f"every CPU in this process's affinity mask ({avail} of {os.cpu_count()})"


def shard(n_total: int, world: int, rank: int):
    """Contiguous client range of `rank` (strong scaling: the population is fixed)."""
    base = n_total * rank // world
    return base, n_total * (rank + 1) // world - base


def cpu_baseline(args):
    """configs[0] exactly — the reference's own CPU configuration (leader.rs:299-443, SURVEY §8d
    Config A: 1000 Zipf clients over num_sites 10000, s = 1.03, data_len 512, d = 1, ball 1,
    threshold 0.001) — as a full two-server crawl of the oracle restatement (AES-NI, one
    non-pipelined block per eval_bit, reference child order, OpenMP over clients). Rank 0, N = 1
    only; the Rust reference is not buildable here (no cargo, crates not vendored)."""
    from fuzzyheavyhitters_amd import workload
    from oracle import oracle as O
    O.build()
    n_cpu, L = 1000, 512
    wl = workload.zipf_workload(n_cpu, L, 1, num_sites=10_000, zipf_s=1.03, ball_size=1, seed=args.seed)
    k0, k1 = O.gen_keys(wl.left, wl.right, wl.root_seeds)
    threads, why = host_threads()
    sample_levels = list(range(1, L, 64))   # the protocol sample's levels (states kept for these)
    t0 = time.perf_counter()
    log("cpu baseline: configs[0] crawl")
    res = O.crawl(k0, k1, 0.001, mode="count", nthreads=threads, max_seconds=args.cpu_baseline_seconds,
                  keep_levels=sample_levels)
    dt = time.perf_counter() - t0
    log(f"cpu baseline: configs[0] crawl {dt:.1f} s")
    done = len(res.n_children)
    protocol = cpu_protocol_baseline(args, O, res, n_cpu, threads, L)
    if protocol:   # the configs[0] keys of r05's line
        protocol["configs0_crawl_s_extrapolated"] = protocol["crawl_s_extrapolated"]
    # the CPU path at 1 000 / 100 000 / 1 000 000 clients (the larger two sampled)
    import numpy as np
    sizes = {"1000": {"value": res.aes_blocks / dt, "crawl_s": dt if done == L else None,
                      "crawl_s_extrapolated": (protocol or {}).get("crawl_s_extrapolated"), "kind": "full crawl"}}
    gold = {100_000: "oracle_zipf_100k_L512.npz", 1_000_000: "zipf_1m_L512.npz"}
    if not args.no_cpu_sizes:
        for n_s, fx in gold.items():
            lc = np.load(os.path.join(ROOT, "tests", "golden", fx), allow_pickle=False)["level_children"]
            sizes[str(n_s)] = cpu_size_sample(args, O, n_s, threads, int(lc.sum()), budget=max(4.0, args.cpu_baseline_seconds / 15))
    return {
        "value": res.aes_blocks / dt,
        "unit": "AES blocks/s",
        "cores": threads,
        "cores_why": why,
        "host_cpus": os.cpu_count(),
        "host_cpus_in_affinity": len(os.sched_getaffinity(0)),
        "kind": "port",
        "cpu_model": cpu_model(),
        "full_crawl_wall_s": dt if done == L else None,
        "sample": (f"configs[0]: 1000 Zipf clients (num_sites 10000, s 1.03, seed {args.seed:#x}), data_len 512, d 1, "
                   f"threshold 0.001 (count 1), levels 0..{done - 1} of {L}, both servers, {sum(res.n_children)} "
                   f"children, {res.aes_blocks} AES blocks in {dt:.2f} s, {len(res.final_paths)} heavy hitters "
                   f"(oracle/fhh_oracle.c: AES-NI single block per eval_bit, reference child order, OpenMP "
                   f"{threads} threads on {cpu_model()})"),
        "protocol": protocol,
        "sizes": sizes,
        "sizes_note": ("the oracle's eval crawl (AES blocks/s) and the reference-form protocol at each client count "
                       "of BASELINE.md; 1000 = configs[0] crawled in full, 100000 / 1000000 sampled over their first "
                       "levels and extrapolated (cpu_size_sample)"),
    }


def cpu_protocol_baseline(args, O, res, n_cpu: int, threads: int, L: int, crawl_tests: int | None = None,
                          budget: float | None = None, what: str = "configs[0]"):
    """The reference's dominant per-level cost on the host cores: tree_crawl's GC equality test + OTs
    (collect.rs:419-482, equalitytest.rs:25-106) in the REFERENCE's protocol form — the garbler labels
    every wire (2 bits + 1 AES-CTR labels), the evaluator's labels and the FE shares go by plain OT
    extension (ocelot AlszSender::send with both messages: 6 AES per OT) — on the oracle restatement
    with AES-NI (swanky's fixed-key AES runs on AES-NI), OpenMP over the host threads. Bounded sample:
    the share strings of configs[0]'s levels 1, 65, 129, ... (states from the crawl above) until
    ~cpu_baseline_seconds / 6 of protocol time; tests/s extrapolated to the configs[0] crawl's tests.
    Every sampled level's v0 - v1 equals the plaintext count (checked)."""
    import numpy as np
    if budget is None:
        budget = max(5.0, args.cpu_baseline_seconds / 6)
    rng = np.random.default_rng(args.seed)
    FE_P = O.FE_P
    tests = 0
    spent = 0.0
    levels = []
    for lv in sorted(res.level_states):
        s0, s1 = res.level_states[lv]
        g = O.share_bits(s0)   # [C][n][bits]
        e = O.share_bits(s1)
        C, n, bits = g.shape
        if C == 0:
            continue
        T = C * n
        gb = g.reshape(T, bits)
        ev = e.reshape(T, bits)
        key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        delta = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        delta[0] |= 1
        delta = bytes(delta)
        D = np.frombuffer(delta, np.uint8)
        mask = int(rng.integers(0, 2))
        seeds = [rng.integers(0, 256, (128, 2, 16), dtype=np.uint8) for _ in range(2)]
        sch = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(2)]
        r0 = rng.integers(0, FE_P, T, dtype=np.uint64)
        r1 = (r0 + np.uint64(1)) % np.uint64(FE_P)
        t0 = time.perf_counter()
        # garbler: labels + half-gates (the evaluator's active labels come out for the OT's check only)
        tables, gbl, evl, dec = O.gc_garble_eq(gb, ev, mask, key, delta)
        zero = evl ^ (ev[:, :, None] * D)          # the OT sender's x0: the evaluator's zero labels
        # the labels OT (plain OT of (x0, x0 ^ Delta), gb_set_fancy_inputs, equalitytest.rs:67-82)
        lab = O.ot_extend(ev.reshape(-1), zero.reshape(-1, 16), None, delta, seeds[0], sch[0], prg="aes")
        out = O.gc_eval_eq(tables, gbl, lab.reshape(T, bits, 16), dec)
        # the share OT (collect.rs:439-471): (r0, r1) if mask else (r1, r0), choice = the GC output
        blk = lambda v: np.concatenate([v.view(np.uint8).reshape(T, 8), np.zeros((T, 8), np.uint8)], axis=1)
        m0, m1 = (r0, r1) if mask else (r1, r0)
        got = O.ot_extend(out, blk(m0), blk(m1), None, seeds[1], sch[1], prg="aes")
        dt = time.perf_counter() - t0
        v1 = np.ascontiguousarray(got[:, :8]).view(np.uint64).reshape(C, n)
        diff = (r1.reshape(C, n).astype(object).sum(axis=1) - v1.astype(object).sum(axis=1)) % FE_P
        assert [int(x) for x in diff] == [int(x) for x in res.counts[lv]], f"CPU protocol level {lv} != plaintext"
        spent += dt
        tests += T
        levels.append(lv)
        if spent >= budget:
            break
    if not tests:
        return None
    rate = tests / spent
    full = crawl_tests is not None or len(res.n_children) == L   # the crawl above finished inside its time bound
    if crawl_tests is None:
        crawl_tests = int(sum(res.n_children)) * n_cpu
    aes = (2 * bits + 1) + 8 * (bits - 1) + 4 * (bits - 1) + 6 * bits + 6
    return {
        "value": rate, "unit": "GC equality tests + OTs per s", "cores": threads, "kind": "port",
        "aes_blocks_per_test": aes,
        "crawl_tests": crawl_tests if full else None,
        "crawl_s_extrapolated": crawl_tests / rate if full else None,
        "levels_crawled": len(res.n_children),
        "sample": (f"{what} levels {levels} ({tests} tests, {spent:.2f} s): the reference's protocol form "
                   f"(garbler labels all {2 * bits + 1} wires, half-gates + TCCR, plain ALSZ OT for the labels and "
                   f"the FE share; {aes} AES per test) on oracle/fhh_oracle.c with AES-NI, OpenMP {threads} "
                   f"threads; v0 - v1 per child = the plaintext count at every sampled level; extrapolated to the "
                   f"crawl's {crawl_tests} tests"),
    }


def cpu_size_sample(args, O, n: int, threads: int, crawl_children: int, budget: float):
    """BASELINE.md's CPU crawl at a larger client count (100k = configs[1], 1M = the metric's), sampled: the
    metric's Zipf workload at n clients (seed args.seed), its first 32 levels (the strings' first 32 bits:
    the same children as the full crawl's first levels) keyed by the oracle's keygen and crawled by the
    oracle (AES-NI single-block eval_bit, reference child order, OpenMP) until `budget` seconds, in count
    mode with the plaintext equality — the eval path the GPU headline runs. AES blocks/s of that sample,
    extrapolated to the full crawl's children (`crawl_children`: the committed golden's level_children sum)
    and labelled as such; then the reference-form protocol on the sampled levels' share strings
    (cpu_protocol_baseline), extrapolated the same way."""
    from fuzzyheavyhitters_amd import workload
    t0 = time.perf_counter()
    wl = workload.zipf_workload(n, 512, 1, num_sites=10_000, zipf_s=1.03, ball_size=1, seed=args.seed)
    K = 32
    left, right = wl.left[:, :, :K].copy(), wl.right[:, :, :K].copy()
    roots = wl.root_seeds
    del wl
    k0, k1 = O.gen_keys(left, right, roots, nthreads=threads)
    del left, right
    t_setup = time.perf_counter() - t0
    log(f"cpu baseline: {n} clients, workload + keys {t_setup:.1f} s")
    t0 = time.perf_counter()
    # at most 6 (1M) / 9 (100k) levels: a level's States are ~36 B per (child, client) and server
    res = O.crawl(k0, k1, 0.001, mode="count", nthreads=threads, max_seconds=budget, keep_levels=[1, 2, 3],
                  levels=6 if n >= 1_000_000 else 9)
    dt = time.perf_counter() - t0
    done = len(res.n_children)
    log(f"cpu baseline: {n} clients, {done} levels in {dt:.1f} s")
    per_child_client = res.aes_blocks / (sum(res.n_children) * n)
    full_blocks = per_child_client * crawl_children * n
    rate = res.aes_blocks / dt
    proto = cpu_protocol_baseline(args, O, res, n, threads, K, crawl_tests=crawl_children * n,
                                  budget=budget / 2, what=f"{n} clients")
    return {
        "clients": n, "value": rate, "unit": "AES blocks/s", "cores": threads, "kind": "port",
        "levels_sampled": done, "children_sampled": int(sum(res.n_children)), "aes_blocks_sampled": int(res.aes_blocks),
        "sample_s": dt, "setup_s": t_setup,
        "crawl_aes_blocks": int(full_blocks), "crawl_s_extrapolated": full_blocks / rate,
        "extrapolation": (f"sampled levels 0..{done - 1} ({sum(res.n_children)} children); the full crawl's "
                          f"{crawl_children} children from the committed golden level counts x {n} clients x "
                          f"{per_child_client:.0f} AES per (child, client) at the sampled rate"),
        "protocol": proto,
    }


def sketch_bench(args, world, rank, local_rank, dist):
    """configs[4]: one step = the sketch verification of a whole data_len-level crawl
    (--sketch-levels, default 1024): levels 0..L-2 over FE (sketch_at + MulState with the level's
    triples, main.rs:14-70 verify_sketches per level, batched in one call) and the last level over
    FieldElm (sketch_at_last + MulState<FieldElm>), for --sketch-keys keys per GPU x
    --sketch-nodes frontier nodes, both servers in-process. Inputs resident in HBM: the one-hot
    vectors are the same at every level (the work is not: every level has its own PrgStream and
    triples). Keys shard by GPU (weak scaling, no collective: every key's check is independent)."""
    import numpy as np
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    L = max(1, args.sketch_levels)
    if fhh.lib().fhh_sketch_set_impl(args.sketch_impl) != 0:
        raise SystemExit(f"--sketch-impl {args.sketch_impl}: no such k_sketch_fe form")
    wl = S.sketch_workload(args.sketch_keys, args.sketch_nodes, seed=args.seed + rank, bad_fraction=0.01)
    kc = fhh.KeyCollection(8, 1, device=local_rank)
    b = S.DeviceSketchBatch(wl, device=local_rank)
    if L > 1:
        S.deal_triples(kc, b, levels=L - 1, seed=args.seed + 17 * rank)
    wl255 = S.sketch_workload255(args.sketch_keys, args.sketch_nodes, seed=args.seed + 1000 + rank, bad_fraction=0.01)
    b255 = S.DeviceSketchBatch255(wl255, device=local_rank)

    def step():
        if L > 1:
            S.sim_sketch_verify(kc, b, level=0, n_levels=L - 1)
        S.sim_sketch_verify_fe255(kc, b255, level=L - 1)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)   # gloo control group: host tensors
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ok = b.ok.cpu().numpy().astype(bool)[: max(L - 1, 1)]
    assert (L == 1 or np.array_equal(ok, np.broadcast_to(wl.honest, ok.shape))), \
        "FE sketch verification disagrees with the workload's ground truth"
    ok255 = b255.ok.cpu().numpy().astype(bool)
    assert np.array_equal(ok255, wl255.honest), "FieldElm sketch verification disagrees with the ground truth"
    keys = args.sketch_keys * world * args.steps
    elems = keys * args.sketch_nodes * 2 * L   # both servers, every level
    blocks = keys * 2 * ((L - 1) * ((args.sketch_nodes + 4) // 2) + 2 * (args.sketch_nodes + 3))
    if rank == 0:
        print(json.dumps({
            "metric": "sketch key x node evaluations/sec (configs[4] sketch + Beaver verification, all levels)",
            "value": elems / elapsed, "unit": "key-node evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64 (GF(2^62-2^30-1)) + 8 x u32 (GF(2^255-19))",
            "data": ("synthetic one-hot frontier vectors (the same at every level), MAC keys, and Beaver triples "
                     "dealt per level on the GPU (sketch.rs:84-150 shape)"),
            "config": {"workload": f"configs[4]: {L - 1} FE levels + 1 FieldElm level of sketch_at + MulState "
                                   f"verify, both servers in-process",
                       "keys_per_gpu": args.sketch_keys, "nodes": args.sketch_nodes, "levels": L,
                       "sketch_impl": args.sketch_impl, "parallelism": f"key-shard x{world}"},
            "keys_verified_per_s": keys * L / elapsed, "aes_blocks_per_s": blocks / elapsed,
            "ms_per_level": elapsed / args.steps / L * 1e3,
            "accepted_per_level": int(wl.honest.sum()), "rejected_per_level": int((~wl.honest).sum()),
        }), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def bincode_bench(args, world, rank, local_rank, dist):
    """Row f4: the add_keys RPC payload (rpc.rs:12-15, bincode 1.x legacy encoding of
    Vec<Vec<(ibDCFKey, ibDCFKey)>>) of --clients clients per GPU (data_len 512, d 1: 10 265 B per
    key, ibDCFbench.csv) decoded straight into the device layout by fhh_add_keys_bincode. One step =
    one server's payload from host memory to decoded device keys (the H2D copy included, since the
    payload arrives in host memory from the RPC layer). Keys from GPU keygen, serialized once on
    the host before the timed region."""
    import numpy as np
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n = args.clients
    wl = workload.zipf_workload(n, args.data_len, args.dims, num_sites=args.num_sites, zipf_s=args.zipf,
                                ball_size=args.ball, seed=args.seed + rank)
    c0 = fhh.KeyCollection(args.data_len, args.dims, device=local_rank)
    c1 = fhh.KeyCollection(args.data_len, args.dims, device=local_rank)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    ki, rs, cw, cb = c0.export_keys()
    req = workload.add_keys_request_bincode(ki, rs, cw, cb)
    del c1, wl

    def step():
        c = fhh.KeyCollection(args.data_len, args.dims, device=local_rank)
        t0 = time.perf_counter()
        c.add_keys_bincode(req)   # pageable host memory, as a deserializer hands it over
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        return c, dt

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    times = []
    for _ in range(args.steps):
        c, dt = step()
        times.append(dt)
    # check the last decode against the keys it came from (bit-exact round trip)
    k2 = c.export_keys()
    assert all(np.array_equal(a, b) for a, b in zip(k2, (ki, rs, cw, cb))), "bincode round trip differs"
    elapsed = sum(times)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        nbytes = req.size * world * args.steps
        print(json.dumps({
            "metric": "add_keys payload decoded to device keys (bincode, host memory in)", "value": nbytes / elapsed / 1e9,
            "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic: GPU-keygen ibDCF keys serialized as AddKeysRequest.keys",
            "config": {"workload": f"row f4: {n} clients x {args.dims} dims x 2 keys, data_len {args.data_len}",
                       "payload_bytes": int(req.size), "bytes_per_key": 25 + 20 * args.data_len,
                       "parallelism": f"client-shard x{world}"},
            "keys_per_s": n * args.dims * 2 * world * args.steps / elapsed,
        }), flush=True)
    return 0


def dropin_bench(args, world, rank, local_rank, dist):
    """The KeyCollection ABI path a Rust server runs per level (collect.rs:370-507 through
    include/fhh.h; server.rs:96-118), timed against the fused device loop of the
    same protocol, --clients clients (configs[1] = 100000), data_len 512, both servers on one GPU.
    One step = one full crawl with the GPU garbled-circuit equality test and both OT extensions in
    every level (ideal base-OT material in both, so the legs do the same work):
      fused     fhh_sim_crawl(gc = 2): both parties inside one device-resident level loop
      dropin    per level, each server on its own ctx: fhh_tree_crawl (share planes stay on the
                device), the party halves fhh_gb_* / fhh_ev_* with the five messages read where the
                sender produced them (the channel's bytes are counted, not moved), fhh_party_node_sums
                on each server's device-resident OT outputs, fhh_keep_values (C), fhh_tree_prune
      dropin-2shard   the same on a two-shard fhh_create_multi collection per server (both shards on
                this GPU, host reduction), each shard its own protocol instance
      dropin-copy     (--dropin-copy) dropin with every message copied into the receiver's buffer
      host-values     (--dropin-host-values) r03's leg: share planes to the host, the leader's count
                standing in for the GC + OT, host OT values summed by fhh_node_sums_fe
    Every leg's heavy hitters are checked against the fused crawl's."""
    import numpy as np
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L, d = args.clients, args.data_len, args.dims
    wl = workload.zipf_workload(n, L, d, num_sites=args.num_sites, zipf_s=args.zipf, ball_size=args.ball,
                                seed=args.seed)

    def pair(devices=None):
        c0 = fhh.KeyCollection(L, d, device=local_rank, devices=devices)
        c1 = fhh.KeyCollection(L, d, device=local_rank, devices=devices)
        fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
        return c0, c1

    runs = {}

    cold = {}

    def timed(fn, reps, warm=1):
        for w in range(warm):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if w == 0:
                cold[id(fn)] = dt   # the first crawl on fresh collections: every buffer allocated on the way
            print(f"dropin:   warm-up run {dt:.2f} s", file=sys.stderr, flush=True)
        times, out = [], None
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"dropin:   timed run {dt:.2f} s", file=sys.stderr, flush=True)
            times.append(dt)
        runs[id(fn)] = times
        return float(np.median(times)), out   # the median run: a typical crawl, not the best one

    reps = max(1, args.steps)
    warm = max(0, args.warmup)
    out = {
        "metric": "drop-in KeyCollection ABI path (two parties, GC + OT every level) vs the fused device loop: "
                  "full-crawl wall time",
        "unit": "s per crawl", "n_gpus": 1, "steps": reps, "warmup": warm, "higher_is_better": False,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic Zipf workload (leader.rs shape), GPU keygen",
        "config": {"workload": f"{n} Zipf clients, data_len {L}, d {d}, threshold {args.threshold}, both servers, "
                               "GC + correlated OTs every level; drop-in legs: each server's own material and "
                               "real Chou-Orlandi base OTs over the channel; fused leg: one-seed material, ideal "
                               "base OTs", "parallelism": "single GPU"},
    }
    ssk = args.protocol_ot_ss_k
    leg_runs = {}
    leg_cold = {}

    def dropin_leg(devices=None, channel="inplace"):
        p0, p1 = pair(devices)
        tm = {}
        last = {}

        def run():
            tm.clear()
            r = fhh.two_party_crawl(p0, p1, args.threshold, channel=channel, timing=tm, record=False,
                                    material="fresh", ot_ss_k=ssk)
            last["r"] = r
            return r
        t, r = timed(run, reps, warm)
        leg_runs[(tuple(devices) if devices else None, channel)] = runs[id(run)]
        leg_cold[(tuple(devices) if devices else None, channel)] = cold.get(id(run))
        if hh is not None:
            assert len(r.final) == hh, f"drop-in ({devices}, {channel}) found {len(r.final)} heavy hitters, fused {hh}"
        tot = {k: sum(lb.get(k, 0) for lb in r.level_bytes) for k in ("gc", "u1", "y1", "u2", "y2")}
        tot["base_ot"] = r.base_ot_bytes
        print(f"dropin: leg devices={devices} channel={channel}: {t:.2f} s ({r.base_ot_runs} CO15 runs, "
              f"crawl waited {r.base_ot_wait_s:.3f} s for them)", file=sys.stderr, flush=True)
        return t, {k: v / L * 1e3 for k, v in tm.items()}, tot, r

    # the drop-in leg first: its cold crawl is a server process's first crawl. Run after the fused leg, the
    # drop-in's first crawl paid +3.1 s at 1M for allocating over the fused pair's freed memory, against +0.03 s
    # in a fresh process (tools/r06_cold.py, profiles/r06/cold/)
    hh = None
    t_d, per_d, bytes_d, r_d = dropin_leg()
    c0, c1 = pair()
    fused_fn = lambda: fhh.sim_crawl(c0, c1, args.threshold, mode="fe", prf_seed=7, gc="ot", record=False,  # noqa: E731
                                     ot_ss_k=ssk)
    t_fused, res = timed(fused_fn, reps, warm)
    fused_runs = runs[id(fused_fn)]
    hh = len(res.final)
    del c0, c1
    print(f"dropin: fused protocol crawl {t_fused:.2f} s, {hh} heavy hitters", file=sys.stderr, flush=True)
    assert len(r_d.final) == hh, f"drop-in found {len(r_d.final)} heavy hitters, fused {hh}"
    out.update({
        "value": t_d, "ms_per_step": t_d * 1e3,
        "fused_protocol_crawl_s": t_fused, "dropin_crawl_s": t_d, "dropin_over_fused": t_d / t_fused,
        "timing_stat": "median of the timed runs per leg (every run listed in *_runs_s)",
        "fused_runs_s": fused_runs, "dropin_runs_s": leg_runs[(None, "inplace")],
        "fused_cold_crawl_s": cold.get(id(fused_fn)), "dropin_cold_crawl_s": leg_cold[(None, "inplace")],
        "dropin_cold_over_warm": (leg_cold[(None, "inplace")] / t_d) if leg_cold[(None, "inplace")] else None,
        "cold_note": ("cold = the first (warm-up) crawl on freshly built collections, buffers allocated as the crawl "
                      "grows; the drop-in leg runs first in the process (a server's first crawl), the fused leg after it"),
        "dropin_ms_per_level": per_d,
        "dropin_overhead_ms_per_level": (t_d - t_fused) / L * 1e3,
        "channel": "in place (the receiver reads the sender's device buffer; bytes counted, not moved)",
        "channel_bytes_per_crawl": bytes_d, "channel_bytes_total": sum(bytes_d.values()),
        "ot_extension": "IKNP" if ssk == 1 else f"SoftSpoken k={ssk} (--protocol-ot-ss-k)",
        "heavy_hitters": hh,
        "dropin_material": "each server its own (os.urandom: mask per chunk; Delta = the labels base-OT run's s, one "
                           "per level, the chunks kept apart by disjoint row-PRG ranges and the gate tweaks; CO15 "
                           "seeds and s); every "
                           "level's labels OT extension on Chou-Orlandi base OTs between the servers over the "
                           "channel (1 CO15 run per level, 2 at the FieldElm level: its share OT; the FE levels' "
                           "shares come from one garbled table per test)",
        "dropin_base_ot_runs": r_d.base_ot_runs, "dropin_base_ot_wait_s": r_d.base_ot_wait_s,
    })
    if not args.no_party:
        t_2, per_2, _, _ = dropin_leg(devices=[local_rank, local_rank])
        out.update({"dropin_2shard_crawl_s": t_2, "dropin_2shard_over_fused": t_2 / t_fused,
                    "dropin_2shard_runs_s": leg_runs[((local_rank, local_rank), "inplace")],
                    "dropin_2shard_ms_per_level": per_2,
                    "dropin_2shard_note": "fhh_create_multi over [this GPU, this GPU]: host reduction of the shards' "
                                          "device-resident sums, one protocol instance per shard"})
    if args.dropin_copy:
        t_c, per_c, _, _ = dropin_leg(channel="copy")
        out.update({"dropin_copy_crawl_s": t_c, "dropin_copy_over_fused": t_c / t_fused,
                    "dropin_copy_runs_s": leg_runs[(None, "copy")],
                    "dropin_copy_ms_per_level": per_c})
    if args.dropin_host_values:
        c0, c1 = pair()
        nw = (n + 63) // 64
        valid = np.full(nw, np.uint64(0xFFFFFFFFFFFFFFFF))
        if n % 64:
            valid[-1] = np.uint64((1 << (n % 64)) - 1)
        thr = max(1, int(args.threshold * n))
        vals = np.random.default_rng(1).integers(0, 1 << 62, (512, n), dtype=np.uint64)   # host OT outputs
        per = {"crawl_planes": 0.0, "leader": 0.0, "node_sums": 0.0, "prune": 0.0}

        def host_values_crawl():
            for k in per:
                per[k] = 0.0
            c0.tree_init()
            c1.tree_init()
            final = 0
            for lv in range(L):
                last = lv == L - 1
                t0 = time.perf_counter()
                C, p0 = (c0.tree_crawl_last if last else c0.tree_crawl)(share_planes=True)
                _, p1 = (c1.tree_crawl_last if last else c1.tree_crawl)(share_planes=True)
                t1 = time.perf_counter()
                diff = np.zeros((C, nw), np.uint64)
                for j in range(2 * d):
                    diff |= p0[:, j] ^ p1[:, j]
                keep = np.bitwise_count(~diff & valid).sum(axis=1) >= thr
                t2 = time.perf_counter()
                if C > vals.shape[0]:
                    raise SystemExit(f"dropin: {C} children > the {vals.shape[0]} rows of host values")
                if not last:
                    c0.node_sums_fe(vals[:C])
                    c1.node_sums_fe(vals[:C])
                t3 = time.perf_counter()
                if last:
                    c0.tree_prune_last(keep)
                    c1.tree_prune_last(keep)
                    final = int(keep.sum())
                else:
                    c0.tree_prune(keep)
                    c1.tree_prune(keep)
                t4 = time.perf_counter()
                per["crawl_planes"] += t1 - t0
                per["leader"] += t2 - t1
                per["node_sums"] += t3 - t2
                per["prune"] += t4 - t3
            return final
        t_h, hh_h = timed(host_values_crawl, reps, warm)
        assert hh_h == hh, f"host-values leg found {hh_h} heavy hitters, fused {hh}"
        out.update({"host_values_crawl_s": t_h, "host_values_ms_per_level": {k: v / L * 1e3 for k, v in per.items()}})
    print(json.dumps(out), flush=True)
    return 0


def gc_bench(args, world, rank, local_rank, dist):
    """Row f1: one step = the garbled-circuit equality tests of one crawl level at configs[1]
    scale (--gc-groups children x --clients clients per GPU, 2d-bit share strings):
    k_gc_garble (server 0: labels, 2 half-gate ciphertexts per AND) then k_gc_eval (server 1),
    transcript through HBM, inputs resident. Tests shard by client across GPUs (weak scaling, no
    collective)."""
    import numpy as np
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    G, N, bits = args.gc_groups, args.gc_clients, 2 * args.dims
    rng = np.random.default_rng(args.seed + rank)
    nw = (N + 63) // 64
    gb = rng.integers(0, 1 << 63, (G, bits, nw), dtype=np.uint64)
    ev = gb.copy()
    # about one client in eight differs (unequal strings) in each child
    ev[:, 0, :] ^= rng.integers(0, 1 << 63, (G, nw), dtype=np.uint64) & rng.integers(0, 1 << 63, (G, nw), dtype=np.uint64) \
        & rng.integers(0, 1 << 63, (G, nw), dtype=np.uint64)
    kc = fhh.KeyCollection(8, 1, device=local_rank)
    key, delta = rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    b = gc.DeviceGcBatch(gb, ev, N, 1, key, delta, device=local_rank)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        gc.equality_device(kc, b)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        gc.equality_device(kc, b)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)   # gloo control group: host tensors
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # ground truth: eq = all planes equal at the client's bit
    out = b.out.cpu().numpy().reshape(G, N)
    diff = np.zeros((G, nw), np.uint64)
    for j in range(bits):
        diff |= gb[:, j] ^ ev[:, j]
    eq = ((np.unpackbits(diff.view(np.uint8).reshape(G, nw, 8), axis=2, bitorder="little").reshape(G, nw * 64)[:, :N])
          == 0)
    assert np.array_equal((out ^ 1).astype(bool), eq), "GC outputs disagree with plaintext equality"
    tests = G * N * world * args.steps
    ands = tests * (bits - 1)
    aes_per_test = (2 * bits + 1) + 12 * (bits - 1)   # labels + 8 (garble) + 4 (eval) per AND
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle import oracle as O
        O.build()
        m = min(G * N, 1 << 18)
        g_s = rng.integers(0, 2, (m, bits), dtype=np.uint8)
        t1 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t1 < args.cpu_baseline_seconds / 3 or reps == 0:
            tb, gl, el, dc = O.gc_garble_eq(g_s, g_s, 1, key, delta)
            O.gc_eval_eq(tb, gl, el, dc)
            reps += 1
        cpu_t = time.perf_counter() - t1
        cpu = {"value": m * reps / cpu_t, "unit": "equality tests/s", "cores": host_threads()[0],
               "kind": "port", "sample": f"{m} tests x {reps} reps, oracle garble+eval (AES-NI as swanky, OpenMP), ni={O.gc_get_ni()}"}
    if rank == 0:
        lds_bytes = tests * aes_per_test * LDS_BYTES_PER_BLOCK
        print(json.dumps({
            "metric": "garbled-circuit equality tests/sec (garble + evaluate, one crawl level)",
            "value": tests / elapsed, "unit": "equality tests/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32 (AES-128 blocks)",
            "data": "synthetic share planes (1 in 8 clients unequal per child), random garbler key and Delta",
            "config": {"workload": "row f1: GC equality tests of one configs[1] level", "groups": G,
                       "clients_per_gpu": N, "bits": bits, "parallelism": f"client-shard x{world}"},
            "and_gates_per_s": ands / elapsed, "aes_blocks_per_s": tests * aes_per_test / elapsed,
            "roofline": {"bound": "lds", "achieved": lds_bytes / elapsed / 1e9, "peak": LDS_PEAK_GBPS, "unit": "GB/s",
                         "frac": lds_bytes / elapsed / 1e9 / LDS_PEAK_GBPS, "traffic": None,
                         "kernel": "k_gc_garble + k_gc_eval (whole step)",
                         "algorithmic": f"640 B of ds_read_b32 per AES block, {aes_per_test} blocks per test"},
            "cpu_baseline": cpu,
        }), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def launch_plan(gpus: int, env, device_count: int, rehearse: bool):
    """How this invocation runs, decided before any GPU call: ("run", None), ("relaunch", None) —
    `python bench.py --gpus N` with N > 1 and no torchrun environment starts itself under
    torch.distributed.run as N ranks (a child process; this one exits with its code) — or
    ("error", message). A torchrun world that differs from --gpus, or more GPUs asked for than the
    node shows (outside --rehearse), is an error: a line that timed fewer GPUs than it names must
    not exist."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return "run", None
        if not rehearse and device_count < gpus:
            return "error", f"--gpus {gpus}: only {device_count} GPU(s) visible on this node"
        return "relaunch", None
    world = int(ws)
    if world != gpus:
        return "error", (f"WORLD_SIZE={world} but --gpus={gpus}: the line would time {world} rank(s) while "
                         f"naming {gpus}")
    if not rehearse and device_count and world > device_count:
        return "error", f"{world} ranks but only {device_count} GPU(s) visible (use --rehearse to share devices)"
    return "run", None


def relaunch_cmd(argv, gpus: int, port: int):
    """The torchrun command `python bench.py --gpus N` re-launches itself with (one node, one rank
    per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def collective_after_init(errs, rehearse_rccl: bool):
    """Every rank's RCCL init error (None = ok), gathered. ("rccl", None) when all succeeded;
    under --rehearse-rccl (ranks share a GPU, RCCL refuses them) ("hosted", error) — the ranks fall
    back together to the hosted all-reduce; otherwise ("fail", error): a measurement without RCCL's
    data path is not the measurement asked for, so every rank exits non-zero."""
    err = next((e for e in errs if e), None)
    if err is None:
        return "rccl", None
    return ("hosted" if rehearse_rccl else "fail"), err


def crawl_sig(res):
    """What a crawl recovers (leader.rs:417-440, collect.rs:945-1029): every level's child count and counts
    (count mode: counts; fe mode: v0 - v1, the same integers) and the sorted (path, value) heavy hitters."""
    import numpy as np
    counts = np.concatenate([np.asarray(c, np.uint64) for c in res.counts]) if res.counts else np.zeros(0, np.uint64)
    final = sorted((tuple(tuple(int(b) for b in dim) for dim in r.path), int(r.value)) for r in res.final)
    return {"level_children": [int(x) for x in res.level_children], "counts": counts, "final": final}


def sig_equal(a, b):
    import numpy as np
    return (a["level_children"] == b["level_children"] and np.array_equal(a["counts"], b["counts"])
            and a["final"] == b["final"])


def golden_sig(args, n_total):
    """tests/golden/zipf_1m_L512.npz (tests/golden/make_zipf_1m.py: the plaintext recount of the metric's
    workload) as a crawl signature, when this run's workload is that one; else None."""
    import numpy as np
    if not (args.workload == "zipf" and n_total == 1_000_000 and args.data_len == 512 and args.dims == 1 and
            args.num_sites == 10_000 and args.zipf == 1.03 and args.ball == 1 and args.seed == 0x5EED and
            args.threshold == 0.001):
        return None
    g = np.load(os.path.join(ROOT, "tests", "golden", "zipf_1m_L512.npz"), allow_pickle=False)
    L = int(g["data_len"])
    paths = np.unpackbits(g["paths"], axis=1, bitorder="big")[:, :L]
    return {"level_children": [int(x) for x in g["level_children"]], "counts": g["counts"].astype(np.uint64),
            "final": sorted(((tuple(int(b) for b in p),), int(v)) for p, v in zip(paths, g["values"]))}


CHACHA12_OPS_PER_BLOCK = 608   # 6 double rounds x 8 quarter rounds x 12 add/xor/rotate + 32 (state, feed-forward)


def protocol_work(level_children, n: int, d: int, circuit: bool = False, ss_k: int = 1):
    """Executed work of one real-protocol crawl on this rank (n clients), by phase, from the kernels' work
    decomposition (fhh_host.cpp level loop; fhh_gc.hip, fhh_ot.hip). Returns (aes, chacha, transpose_bytes):
    AES blocks per phase — FE levels with b = 2d <= 2 run the tile-major garbled table (2^b rows per test
    garbled, 1 evaluated, padding tests of the 512-client tiles included), b = 4 the row-major table (64-client
    words) after k_ot_rows_out, the FieldElm level the half-gates circuit (TCCR: 8 AES per AND gate garbled, 4
    evaluated) + the share C-OT's hashes (2 OTs per test: 2 + 1 per OT); circuit = the half-gates circuit + the
    output-label share (2 AES garbled, 1 evaluated per test) at the FE levels too — and ChaCha12 blocks of the
    labels / share OTs' row PRG (since r06: 64 B per row and 512-OT tile; receiver 2, sender 1 per row), and the
    bytes of the remaining row transposes (32 B per OT and party)."""
    b = 2 * d
    npad64 = (n + 63) // 64 * 64
    npad_tm = (n + 511) // 512 * 512
    aes = {"table_garble": 0, "table_eval": 0, "circuit_garble": 0, "circuit_eval": 0, "share_ot_hash": 0}
    cc = {"ot_recv_expand": 0, "ot_send_expand": 0}
    transpose_bytes = 0
    L = len(level_children)

    def expands(m):   # m OTs: 128 rows x ceil(m / 512) tiles, 2 blocks (receiver) + 1 (sender) each
        tiles = (m + 511) // 512
        if ss_k > 1:   # SoftSpoken: 128 / k chunks, 2^k blocks (receiver) and 2^k - 1 (sender) per tile
            cc["ot_recv_expand"] += (128 // ss_k) * (1 << ss_k) * tiles
            cc["ot_send_expand"] += (128 // ss_k) * ((1 << ss_k) - 1) * tiles
            return
        cc["ot_recv_expand"] += 2 * 128 * tiles
        cc["ot_send_expand"] += 128 * tiles

    for lv, C in enumerate(int(x) for x in level_children):
        if lv + 1 < L and circuit:
            m1 = C * b * npad64
            expands(m1)
            aes["circuit_garble"] += (8 * (b - 1) + 2) * C * n
            aes["circuit_eval"] += (4 * (b - 1) + 1) * C * n
            transpose_bytes += 2 * 32 * m1
        elif lv + 1 < L:
            tm = b <= 2
            npad = npad_tm if tm else npad64
            m1 = C * b * npad
            expands(m1)
            aes["table_garble"] += (1 << b) * C * (npad if tm else n)
            aes["table_eval"] += C * (npad if tm else n)
            if not tm:
                transpose_bytes += 2 * 32 * m1
        else:
            m1 = C * b * npad64
            expands(m1)
            aes["circuit_garble"] += 8 * (b - 1) * C * n
            aes["circuit_eval"] += 4 * (b - 1) * C * n
            m2 = 2 * C * n
            expands(m2)
            aes["share_ot_hash"] += 2 * m2 + m2
            transpose_bytes += 2 * 32 * m1
    return aes, cc, transpose_bytes


def protocol_bytes(level_children, n: int, d: int, circuit: bool = False, ss_k: int = 1, ring32: bool = False):
    """Server-to-server bytes of one real-protocol crawl on this rank (n clients), by message, as the party ABI
    counts them (fhh_gcot.cpp u_bytes / gc_bytes / y2_bytes; the base OTs' CO15 messages excluded): the labels
    OT's U (16 / ss_k B per OT: 128 / ss_k rows; SoftSpoken adds 4 KiB of GGM corrections per base-OT session),
    the FE levels' garbled table (2^b - 1 rows of 8 B per test) or circuit (2 (b - 1) blocks + decode + the 8-B
    share per test), the FieldElm level's circuit and its share OT (U and 16 B of y per OT, 2 OTs per test);
    ring32 (d = 1 table): the table's rows are 4-B Z_2^32 messages."""
    b = 2 * d
    npad64 = (n + 63) // 64 * 64
    npad_tm = (n + 511) // 512 * 512
    L = len(level_children)
    out = {"u_labels": 0, "u_shares": 0, "ggm_corrections": 0, "table": 0, "circuit": 0, "y_shares": 0}
    corr = 4096 if ss_k > 1 else 0
    for lv, C in enumerate(int(x) for x in level_children):
        if C == 0:
            continue
        tests = C * n
        if lv + 1 < L:
            tm = (not circuit) and b <= 2
            m1 = C * b * (npad_tm if tm else npad64)
            out["u_labels"] += 16 * m1 // ss_k
            out["ggm_corrections"] += corr
            if circuit:
                out["circuit"] += tests * (2 * (b - 1) * 16 + 1 + 8)
            else:
                out["table"] += tests * ((1 << b) - 1) * (4 if ring32 and b <= 2 else 8)
        else:
            m1 = C * b * npad64
            m2 = 2 * tests
            out["u_labels"] += 16 * m1 // ss_k
            out["u_shares"] += 16 * m2 // ss_k
            out["ggm_corrections"] += 2 * corr
            out["circuit"] += tests * (2 * (b - 1) * 16 + 1)
            out["y_shares"] += 16 * m2
    out["total"] = sum(out.values())
    return out


def protocol_crawl(args, c0, c1, n_total, comm, dist, headline_sig, gc="ot", expand_rate=None, ot_ss_k=1,
                   ring32=False):
    """The real protocol's crawl on the headline's keys (tree_crawl with gc_sender per level,
    collect.rs:419-482, with OtSender/OtReceiver::init per channel and level, :454-471; the leader's
    loop leader.rs:422-440): the GPU garbled-circuit equality test and both OT extensions in every
    level, each OT extension (and each chunk of a level's children) on its own 128 real Chou–Orlandi
    base OTs from host threads. One warm-up crawl over the first 32 levels (allocates the GC + OT
    buffers at this capacity), then one timed full crawl, bracketed like the headline."""
    import torch
    import fuzzyheavyhitters_amd as fhh

    def run(levels=None):
        # record: every level's v0 - v1 comes back to the host (a few KB per level) for the output check
        return fhh.sim_crawl(c0, c1, args.threshold, nclients_total=n_total, mode="fe", prf_seed=7, record=True,
                             comm=comm, gc=gc, base_ot=True, levels=levels, ot_ss_k=ot_ss_k,
                             table_ring32=ring32 and gc == "ot")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    tag = (gc if ot_ss_k == 1 else f"{gc}, SoftSpoken k={ot_ss_k}") + (", Z_2^32 table" if ring32 and gc == "ot" else "")
    run(levels=min(32, args.data_len))
    barrier()
    log(f"protocol crawl ({tag}): warm-up done")
    c0.reset_stats()
    c1.reset_stats()
    t0 = time.perf_counter()
    res = run()
    barrier()
    wall = time.perf_counter() - t0
    log(f"protocol crawl ({tag}): {wall:.2f} s, {len(res.final)} heavy hitters")
    s0 = c0.stats()
    if dist is not None:
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    hh = len(res.final)
    sig = crawl_sig(res)
    aes, cc, tr_bytes = protocol_work(res.level_children, c0.num_clients(), args.dims, circuit=gc == "ot-circuit",
                                      ss_k=ot_ss_k)
    wire = protocol_bytes(res.level_children, c0.num_clients(), args.dims, circuit=gc == "ot-circuit", ss_k=ot_ss_k,
                          ring32=ring32 and gc == "ot")
    n_aes, n_cc = sum(aes.values()), sum(cc.values())
    gpu_s = s0["gcot_ms"] / 1e3
    ops = n_aes * VALU_OPS_PER_BLOCK + n_cc * CHACHA12_OPS_PER_BLOCK
    tops = ops / gpu_s / 1e12 if gpu_s > 0 else 0.0
    roof = {
        "executed_aes_blocks": n_aes,
        "executed_aes_blocks_by_phase": aes,
        "executed_chacha12_blocks": n_cc,
        "executed_chacha12_blocks_by_phase": cc,
        "work_note": ("executed on this rank, from the kernels' work decomposition (bench.protocol_work): padding "
                      "tests of the 512-client tiles included; the OT row PRG is ChaCha12 since r06 (64-B blocks)"),
        "gcot_gpu_s": gpu_s,
        "aes_blocks_per_s_if_alone": n_aes / gpu_s if gpu_s > 0 else 0.0,
        "valu_tops": tops,
        "frac": tops / VALU_PEAK_TOPS,
        "frac_basis": (f"{VALU_OPS_PER_BLOCK} int32 ops per AES block (SURVEY 8d) + {CHACHA12_OPS_PER_BLOCK} per "
                       f"ChaCha12 block (add/xor/rotate) / the GC + OT steps' GPU time (HIP events) over "
                       f"{VALU_PEAK_TOPS} T ops/s"),
        "vs_k_expand_in_kernel": (ops / VALU_OPS_PER_BLOCK / gpu_s) / expand_rate if expand_rate and gpu_s > 0 else None,
        "vs_k_expand_note": "the steps' work in AES-block equivalents (ops / 400) per s over k_expand's in-kernel blocks/s",
        "transpose_hbm_bytes": tr_bytes,
        "transpose_note": ("k_ot_rows_out's bytes (32 B per OT and party): since r06 only the FieldElm level's "
                           "circuit (and d = 2's table) transposes; d = 1's FE levels read Q / T tile-major"),
    }
    return {
        "wall_s": wall,
        "heavy_hitters": hh,
        "heavy_hitters_equal_headline": sig_equal(sig, headline_sig) if headline_sig else None,
        "ot_extension": "IKNP (128 rows of U)" if ot_ss_k == 1 else
                        f"SoftSpoken k={ot_ss_k} ({128 // ot_ss_k} rows of U, GGM trees from the base OTs)",
        "table_shares": ("Z_2^32 (4-B rows)" if ring32 and gc == "ot" and args.dims == 1 else "FE (8-B rows)")
                        if gc == "ot" else None,
        "channel_bytes": wire,
        "channel_bytes_note": ("server-to-server bytes of this crawl on this rank by message, as the party ABI "
                               "counts them (bench.protocol_bytes; CO15 base-OT messages excluded)"),
        "output_check": ("every level's child count and v0 - v1 per child, and the sorted (path, value) heavy "
                         "hitters, equal the headline crawl's (recorded in its untimed warm-up)"),
        "roofline": roof,
        "sig": sig,
        "base_ot": "chou-orlandi over P-256 (host threads, a fresh instance per level for the labels OT and one "
                   "for the FieldElm level's share OT; chunks on disjoint row-PRG counters)",
        "base_ot_instances": s0["base_ot_instances"],
        "base_ot_compute_ms": s0["base_ot_ms"],
        "base_ot_stall_ms": s0["base_ot_stall_ms"],
        "base_ot_note": "compute = summed per-instance CO15 + key-schedule time over the host threads; stall = time "
                        "the level loop waited for an instance it needed (the base OTs on the critical path)",
        "protocol": ("the evaluator's labels as the IKNP correlation (Delta = the labels OT's s, no reply); every "
                     "level: half-gates GC (TCCR; the garbler's string and mask folded in); FE levels: the share "
                     "from the circuit's output labels (cr_hash of W_0, W_0 ^ Delta); the FieldElm level: ALSZ "
                     "correlated OT for the share (15 AES blocks per d=1 FE-level test: garble 8 + 2, evaluate "
                     "4 + 1; the labels OT's row PRG ChaCha12, 3 blocks of 64 B per row and 512 OTs)") if gc == "ot-circuit" else
                    "the evaluator's labels as the IKNP correlation (Delta = the labels OT's s, no reply); FE "
                    "levels: equality + share as one garbled table per test (Yao's garbled gate with "
                    "point-and-permute over the 2d input labels, rows keyed by cr_hash, 8 B per row; the "
                    "garbler's string and mask folded in); the FieldElm level: half-gates GC (TCCR) + ALSZ "
                    "correlated OT for the share (5 AES blocks per d=1 FE-level test: table 4 + 1; the labels OT's "
                    "row PRG ChaCha12 (r06), 3 blocks of 64 B per row and 512 OTs; the table kernels read the OT's "
                    "tile-major matrices, no row transposes)",
        "gcot_gpu_ms": s0["gcot_ms"], "gcot_levels_timed": s0["gcot_timed"],
        "expand_gpu_ms": s0["expand_ms"],
        "allreduce_ms": s0["allreduce_ms"] if comm is not None else None,
        "timing": "HIP events on the engine stream around every level's GC + OT step and k_expand (rank 0)",
        "warmup": "one 32-level protocol crawl before the timed one",
        "workload": "the headline's keys and clients, mode fe (FE shares, FieldElm last level), GC + OT every level",
    }


def load_pmc(config: str):
    """Committed rocprofv3 PMC summary of k_expand for this workload (tools/profile.sh +
    tools/pmc_summary.py -> profiles/pmc_expand.json, keyed by workload)."""
    path = os.path.join(ROOT, "profiles", "pmc_expand.json")
    try:
        allp = json.load(open(path))
    except (OSError, ValueError):
        return None
    return allp.get(config)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--clients", type=int, default=1_000_000,
                    help="clients in total, sharded over the ranks (strong scaling; 1M = the metric's "
                         "configuration and, at 8 GPUs, configs[2]; 100000 = configs[1])")
    ap.add_argument("--data-len", type=int, default=512)
    ap.add_argument("--dims", type=int, default=1)
    ap.add_argument("--num-sites", type=int, default=10_000)
    ap.add_argument("--zipf", type=float, default=1.03)
    ap.add_argument("--ball", type=int, default=1)
    ap.add_argument("--threshold", type=float, default=0.001)
    ap.add_argument("--mode", default="count", choices=["count", "fe"])
    ap.add_argument("--no-party", action="store_true", help="--workload dropin: skip the two-shard leg")
    ap.add_argument("--dropin-copy", action="store_true",
                    help="--workload dropin: also time the drop-in path with every message copied to the receiver")
    ap.add_argument("--dropin-host-values", action="store_true",
                    help="--workload dropin: also time r03's host-values leg (planes to the host, host OT values)")
    ap.add_argument("--workload", default="zipf", choices=["zipf", "coords", "sketch", "gc", "bincode", "dropin"],
                    help="zipf = the metric's Zipf crawl (default 1M clients; --clients 100000 = configs[1]); "
                         "coords = configs[3] (d=2 lat/lon, data_len 16); sketch = configs[4] (sketch + Beaver "
                         "verification); gc = row f1 (garbled-circuit equality tests of one level); "
                         "bincode = row f4 (add_keys payload decoded on the GPU, --clients per GPU); "
                         "dropin = the KeyCollection ABI path per level and the two-party GC + OT split vs the "
                         "fused loops (--clients 100000 = configs[1])")
    ap.add_argument("--gc-groups", type=int, default=256, help="--workload gc: children per level")
    ap.add_argument("--gc-clients", type=int, default=100_000, help="--workload gc: clients per GPU")
    ap.add_argument("--gc", default="none", choices=["none", "ot", "ideal"],
                    help="crawl with the GPU garbled-circuit equality test (mode fe): ot = labels and FE shares "
                         "by GPU OT extension, ideal = ideal OT")
    ap.add_argument("--base-ot", action="store_true",
                    help="--gc ot: real Chou-Orlandi base OTs for every level's OT extensions (host threads, "
                         "overlapped with the crawl) instead of ideal ones")
    ap.add_argument("--sketch-keys", type=int, default=100_000, help="configs[4] sketch_batch_size (per GPU)")
    ap.add_argument("--sketch-impl", type=int, default=0,
                    help="k_sketch_fe form: 0 = round keys in LDS / 1024 threads (default), 1 = r01 kernel, "
                         "2 = round keys expanded on the fly")
    ap.add_argument("--sketch-nodes", type=int, default=256, help="frontier nodes per sketched vector")
    ap.add_argument("--sketch-levels", type=int, default=1024,
                    help="configs[4]: data_len levels verified per step (L-1 over FE, the last over FieldElm)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=150.0,
                    help="upper bound on the configs[0] CPU crawl (it normally completes well inside)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-sizes", action="store_true", help="cpu_baseline: configs[0] only (no 100k / 1M samples)")
    ap.add_argument("--microbench", action="store_true", help="measure VALU/LDS peaks on this device")
    ap.add_argument("--variant", type=int, default=-1, help="k_expand variant (-1 = library default)")
    ap.add_argument("--rehearse", action="store_true",
                    help="N>1 rehearsal on fewer GPUs than ranks: ranks share devices (local_rank mod the "
                         "device count) and the per-level all-reduce runs through the hosted communicator "
                         "(the same cfg.comm path, partials summed by gloo) instead of RCCL, which cannot "
                         "place two ranks on one GPU. Never a measurement.")
    ap.add_argument("--rehearse-rccl", action="store_true",
                    help="as --rehearse (ranks share devices), but the ranks first try the RCCL communicator: "
                         "its socket bootstrap completes and RCCL then refuses two ranks on one GPU, which "
                         "exercises the init-failure fallback to the hosted communicator. Never a measurement.")
    ap.add_argument("--timing-every", type=int, default=1,
                    help="time every K-th k_expand launch with HIP events (roofline.avg_launch_us)")
    ap.add_argument("--no-protocol-circuit", action="store_true",
                    help="skip the second protocol crawl with the half-gates circuit at every level")
    ap.add_argument("--table-ring32", action="store_true",
                    help="--gc ot: the FE levels' garbled table in Z_2^32 (4-B rows) instead of FE")
    ap.add_argument("--ot-ss-k", type=int, default=1, choices=(1, 2, 4),
                    help="--gc ot: the OT extension of the timed crawl (1 IKNP, 2 / 4 SoftSpoken)")
    ap.add_argument("--protocol-ot-ss-k", type=int, default=2, choices=(1, 2, 4),
                    help="the protocol crawl's OT extension: 1 IKNP, 2 / 4 SoftSpoken (default 2: half of IKNP's U "
                         "bytes for ~1.5x the sender's ChaCha work, profiles/r06/softspoken/)")
    ap.add_argument("--protocol-table-fe", action="store_true",
                    help="the protocol crawl's FE-level garbled table with FE shares (8-B rows) instead of the "
                         "default Z_2^32 shares (4-B rows; d = 1)")
    ap.add_argument("--protocol-ss-k", default="1,4",
                    help="comma list of further OT extensions (1 IKNP, 2 / 4 SoftSpoken) to run the protocol crawl "
                         "with beside it ('' = none)")
    ap.add_argument("--no-protocol-crawl", action="store_true",
                    help="skip the real protocol's crawl (GC + OT + real base OTs every level) that follows the "
                         "headline's timed region on the zipf workload")
    args = ap.parse_args()
    if args.rehearse_rccl:
        args.rehearse = True

    import torch
    # before any GPU call (torch.cuda.device_count does not initialise the GPU on this image)
    plan, why = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), args.rehearse)
    if plan == "error":
        log(f"bench.py: {why}")
        return 2
    if plan == "relaunch":
        import socket
        import subprocess
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = relaunch_cmd(sys.argv[1:], args.gpus, port)
        log("bench.py: --gpus", args.gpus, "without a torchrun world: relaunching as", " ".join(cmd))
        return subprocess.run(cmd).returncode

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse:
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        # control plane only (barriers, the communicator id, max-over-ranks timing): gloo on the
        # host. The data path's one collective is the native RCCL communicator below — one RCCL
        # communicator per rank, nothing else touches RCCL.
        import torch.distributed as dist
        dist.init_process_group("gloo")

    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload

    if args.workload == "sketch":
        return sketch_bench(args, world, rank, local_rank, dist)
    if args.workload == "gc":
        return gc_bench(args, world, rank, local_rank, dist)
    if args.workload == "bincode":
        return bincode_bench(args, world, rank, local_rank, dist)
    if args.workload == "dropin":
        return dropin_bench(args, world, rank, local_rank, dist)
    if args.gc != "none" and args.mode != "fe":
        args.mode = "fe"   # the GC equality test feeds the OT share conversion (collect.rs:419-482)

    n_total = args.clients
    base, n_local = shard(n_total, world, rank)
    t_gen = time.perf_counter()
    if args.workload == "coords":
        # configs[3]: src/bin/config.json (data_len 16, n_dims 2, ball 1, threshold 0.075)
        args.data_len, args.dims = 16, 2
        if args.threshold == 0.001:
            args.threshold = 0.075
        wl = workload.coords_workload(n_local, ball_size=args.ball, zipf_s=args.zipf, seed=args.seed,
                                      client_offset=base)
    else:
        wl = workload.zipf_workload(n_local, args.data_len, args.dims, num_sites=args.num_sites, zipf_s=args.zipf,
                                    ball_size=args.ball, seed=args.seed, client_offset=base)
    c0 = fhh.KeyCollection(args.data_len, args.dims, device=local_rank)
    c1 = fhh.KeyCollection(args.data_len, args.dims, device=local_rank)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    del wl
    if args.variant >= 0:
        c0.set_variant(args.variant)
        c1.set_variant(args.variant)
    c0.set_client_base(base)
    c1.set_client_base(base)
    c0.set_timing(args.timing_every)
    log(f"[rank {rank}] {n_local} clients from {base}: workload+keygen {time.perf_counter() - t_gen:.2f}s "
        f"(GPU keygen {c0.stats()['keygen_ms']:.1f} ms)")

    comm, collective = None, {"kind": "none"}
    if world > 1 and args.rehearse and not args.rehearse_rccl:
        comm = fhh.HostedComm(local_rank)
        collective = {"kind": "REHEARSAL: hosted communicator (gloo all-reduce of the partials), not RCCL",
                      "comm_ranks": world, "comm_rank": rank}
    elif world > 1:
        # native RCCL all-reduce on the engine stream (no host sync per level); the id travels
        # over the gloo group. One node (the driver's torchrun --nnodes=1): RCCL's bootstrap
        # sockets stay on loopback unless the environment says otherwise (the data path is xGMI)
        if int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world:
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        err = None
        try:
            comm = fhh.RcclComm(local_rank)
        except fhh.FhhError as e:   # an RCCL init error (not a hang) on any rank
            err = str(e)
        errs = [None] * world
        dist.all_gather_object(errs, err)
        how, rccl_err = collective_after_init(errs, args.rehearse_rccl)
        if how == "fail":
            # every rank saw the same gathered errors: all leave together, no line is printed
            log(f"[rank {rank}] RCCL init failed ({rccl_err}); refusing to measure N>1 without RCCL")
            if comm is not None:
                comm.close()
            dist.barrier()
            dist.destroy_process_group()
            return 3
        if how == "hosted":
            # --rehearse-rccl: every rank falls back together: the same level loop with the per-level
            # sum of the partials through the hosted communicator (gloo), labelled as such in the line
            if comm is not None:
                comm.close()
            comm = fhh.HostedComm(local_rank)
            collective = {"kind": "hosted communicator (gloo all-reduce of the partials): RCCL init failed",
                          "rccl_error": rccl_err, "comm_ranks": world, "comm_rank": rank}
            log(f"[rank {rank}] RCCL init failed ({rccl_err}); hosted all-reduce instead (rehearsal)")
        else:
            nr, rk = comm.info()
            collective = {"kind": "rccl ncclAllReduce(sum, u64) of per-child partials on the engine stream",
                          "comm_ranks": nr, "comm_rank": rk}
            log(f"[rank {rank}] RCCL communicator: {nr} ranks, rank {rk}")

    def step(record=False):
        return fhh.sim_crawl(c0, c1, args.threshold, nclients_total=n_total, mode=args.mode, prf_seed=7,
                             record=record, comm=comm, gc={"none": False, "ot": "ot", "ideal": "ideal"}[args.gc],
                             base_ot=args.base_ot, ot_ss_k=args.ot_ss_k if args.gc == "ot" else 1,
                             table_ring32=args.table_ring32 and args.gc == "ot")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # the warm-up crawls record every level's counts (D2H per level; untimed): the output the timed steps
    # and the protocol crawl are checked against
    res_ref = None
    for _ in range(args.warmup):
        res_ref = step(record=True)
    barrier()
    log(f"[rank {rank}] warm-up done ({args.warmup} recorded crawls)")
    c0.reset_stats()
    c1.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    barrier()
    elapsed = time.perf_counter() - t0
    log(f"[rank {rank}] timed: {args.steps} crawls in {elapsed:.2f} s")
    s0, s1 = c0.stats(), c1.stats()
    blocks = s0["aes_blocks"] + s1["aes_blocks"]
    ref_evals = s0["ref_evals"] + s1["ref_evals"]
    # per-level cross-rank all-reduce (HIP events around ncclAllReduce on the engine stream)
    ar_us = s0["allreduce_ms"] * 1e3 / s0["allreduce_timed"] if s0["allreduce_timed"] else None
    ar_us_max = ar_us
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        b = torch.tensor([blocks, ref_evals], dtype=torch.int64)
        dist.all_reduce(b)
        blocks, ref_evals = int(b[0].item()), int(b[1].item())
        a = torch.tensor([ar_us or 0.0], dtype=torch.float64)
        dist.all_reduce(a, op=dist.ReduceOp.MAX)
        ar_us_max = float(a.item()) if ar_us is not None else None
    run_proto = args.workload == "zipf" and args.gc == "none" and not args.no_protocol_crawl
    if res_ref is None and run_proto:   # no warm-up: one recorded crawl after the timed region
        res_ref = step(record=True)
    ref_sig = crawl_sig(res_ref) if res_ref is not None else None
    gold = golden_sig(args, n_total)
    checks = None if ref_sig is None else {
        "timed_final_equal_reference": sorted((tuple(tuple(int(b) for b in d) for d in r.path), int(r.value))
                                              for r in res.final) == ref_sig["final"],
        "reference_equal_golden": sig_equal(ref_sig, gold) if gold else None,
        "golden": "tests/golden/zipf_1m_L512.npz (plaintext recount of the metric's workload)" if gold else None,
        "note": ("the headline's recorded warm-up crawl: every level's child count and counts and the sorted "
                 "(path, value) heavy hitters; the timed steps' heavy hitters equal it"),
    }
    launches0 = max(1, s0["expand_launches_timed"])
    expand_rate = (s0["expand_blocks_timed"] / launches0) / (s0["expand_ms"] / launches0 / 1e3) if s0["expand_ms"] else None
    proto = None
    if run_proto:
        ring = not args.protocol_table_fe
        proto = protocol_crawl(args, c0, c1, n_total, comm, dist, ref_sig, expand_rate=expand_rate,
                               ot_ss_k=args.protocol_ot_ss_k, ring32=ring)
        psig = proto.pop("sig")   # (not JSON: the crawl's signature arrays)
        proto["output_equal_golden"] = sig_equal(psig, gold) if gold else None
        if not args.no_protocol_circuit:
            # the same crawl with the half-gates circuit at every level (the reference's construction,
            # r05c form) beside the default garbled table: what the table buys, on the same box
            circ = protocol_crawl(args, c0, c1, n_total, comm, dist, ref_sig, gc="ot-circuit", expand_rate=expand_rate,
                                  ot_ss_k=args.protocol_ot_ss_k)
            proto["circuit_form"] = {k: circ[k] for k in ("wall_s", "heavy_hitters", "heavy_hitters_equal_headline",
                                                          "gcot_gpu_ms", "expand_gpu_ms", "protocol", "roofline",
                                                          "channel_bytes")}
        # r06: the same crawl on the other OT extensions (IKNP: 128 rows of U; SoftSpoken k: 128 / k rows of U,
        # 2^k ChaCha12 blocks per chunk and tile) — the wire bytes against the GPU time
        proto["ot_extension_forms"] = {}
        for k in [int(x) for x in args.protocol_ss_k.split(",") if x.strip()]:
            if k == args.protocol_ot_ss_k:
                continue
            ss = protocol_crawl(args, c0, c1, n_total, comm, dist, ref_sig, expand_rate=expand_rate, ot_ss_k=k,
                                ring32=ring)
            proto["ot_extension_forms"][f"k{k}"] = {key: ss[key] for key in (
                "wall_s", "heavy_hitters", "heavy_hitters_equal_headline", "gcot_gpu_ms", "ot_extension",
                "table_shares", "channel_bytes", "roofline")}
            proto["ot_extension_forms"][f"k{k}"]["output_equal_golden"] = sig_equal(ss["sig"], gold) if gold else None

    if rank == 0:
        launches = max(1, s0["expand_launches_timed"])
        avg_launch_s = s0["expand_ms"] / launches / 1e3
        blocks_per_launch = s0["expand_blocks_timed"] / launches
        rate = blocks_per_launch / avg_launch_s if avg_launch_s > 0 else 0.0     # in-kernel blocks/s
        valu_tops = rate * VALU_OPS_PER_BLOCK / 1e12
        lds_gbps = rate * LDS_BYTES_PER_BLOCK / 1e9
        hbm_gbps = rate * HBM_BYTES_PER_BLOCK / 1e9
        cfg_key = f"n{n_local}_L{args.data_len}_d{args.dims}"
        pmc = load_pmc(cfg_key) if args.workload == "zipf" and args.variant < 0 else None
        traffic = pmc_rates = None
        if pmc:
            traffic = pmc.get("hbm_bytes_per_launch")
            t = pmc["k_expand_avg_ns"] * 1e-9
            lds_exec = pmc["sq_insts_lds_per_launch"] * 64 * 4      # ds_read_b32: 4 B per lane
            pmc_rates = {
                "source": f"profiles/pmc_expand.json[{cfg_key}] ({pmc.get('tag')}, rocprofv3 --pmc passes)",
                "k_expand_avg_us": pmc["k_expand_avg_ns"] / 1e3,
                "valu_lane_ops_per_s": pmc["sq_insts_valu_per_launch"] * 64 / t,
                "valu_frac": pmc["sq_insts_valu_per_launch"] * 64 / t / (VALU_PEAK_TOPS * 1e12),
                "lds_executed_bytes_per_launch": lds_exec,
                "lds_executed_frac": lds_exec / t / (LDS_PEAK_GBPS * 1e9),
                "hbm_bytes_per_s": traffic / t,
                "hbm_frac": traffic / t / (HBM_PEAK_GBPS * 1e9),
                "lds_insts_per_block": pmc["sq_insts_lds_per_launch"] * 64 / blocks_per_launch,
                "valu_insts_per_block": pmc["sq_insts_valu_per_launch"] * 64 / blocks_per_launch,
                "lds_bank_conflict_cycles": pmc.get("sq_lds_bank_conflict"),
                "effective_clock_ghz": pmc.get("effective_clock_ghz"),
            }
        if args.workload == "zipf":
            wl_name = (f"Zipf ibDCF tree crawl, {n_total} clients, data_len {args.data_len}, d {args.dims}, both "
                       f"servers in-process" + (" (= configs[2] sharded over 8 GPUs)" if n_total == 1_000_000 else "")
                       + (" (= configs[1])" if n_total == 100_000 else ""))
        else:
            wl_name = ("configs[3]: lat/lon l-inf balls around the reference's county centroids "
                       "(data/county_centroids.csv, Zipf-weighted, 8 km uniform_in_square jitter), d=2, data_len 16")
        metric = ("client×prefix key evals/sec (AES blocks/s) + full-crawl wall time, 1M clients"
                  if n_total == 1_000_000 and args.workload == "zipf" else
                  f"client×prefix key evals/sec (AES blocks/s) + full-crawl wall time, {n_total} clients")
        out = {
            "metric": metric,
            "value": blocks / elapsed,
            "unit": "AES blocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": ("synthetic: seeded Zipf workload shaped like leader.rs (num_sites strings + 8-bit augmentation), "
                     "keys by GPU keygen, resident in HBM before the timed region"
                     if args.workload == "zipf" else
                     "synthetic clients over the reference's real county centroids (data/county_centroids.csv via "
                     "tests/golden/county_centroids.npz): Zipf-weighted county draw, uniform_in_square jitter of "
                     "side 8 km, i16 centidegrees; keys by GPU keygen"),
            "config": {
                "workload": wl_name,
                "clients_total": n_total, "clients_per_gpu": n_local, "data_len": args.data_len,
                "n_dims": args.dims, "num_sites": args.num_sites, "zipf_s": args.zipf, "ball_size": args.ball,
                "threshold": args.threshold, "mode": args.mode, "gc": args.gc,
                "ot_extension": None if args.gc != "ot" else ("IKNP" if args.ot_ss_k == 1 else f"SoftSpoken k={args.ot_ss_k}"),
                "base_ot": "chou-orlandi (host)" if args.base_ot else ("ideal" if args.gc == "ot" else None),
                "parallelism": f"client-shard x{world}", "collective": collective,
                "variant": args.variant if args.variant >= 0 else "default",
            },
            "full_crawl_wall_s": elapsed / args.steps,
            "full_crawl_note": "both servers' evaluation fused in one k_expand launch per level, plus the "
                               "plaintext equality count, leader keep and prune on the GPU",
            "ref_equiv_evals_per_s": ref_evals / elapsed,
            "aes_blocks_per_step": blocks / args.steps,
            "base_ot_ms_per_step": s0.get("base_ot_ms", 0.0) / args.steps if args.base_ot else None,
            "allreduce_us_per_level": ar_us,
            "allreduce_us_per_level_max_rank": ar_us_max,
            "allreduce_note": ("HIP events around the per-level cross-rank all-reduce on the engine stream (rank 0; "
                               "max over ranks beside it); null on one GPU"),
            "protocol_crawl_wall_s": proto["wall_s"] if proto else None,
            "protocol_crawl": proto,
            "final_heavy_hitters": len(res.final),
            "output_checks": checks,
            "levels": int(len(res.level_children)),
            "children_total": int(res.level_children.sum()),
            "roofline": {
                "bound": "valu", "achieved": valu_tops, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
                "frac": valu_tops / VALU_PEAK_TOPS, "traffic": traffic,
                "kernel": "k_expand",
                "algorithmic": (f"{VALU_OPS_PER_BLOCK} int32 ops per AES block (SURVEY 8d) x blocks per launch / "
                                f"average launch time (HIP events on the engine stream)"),
                "peak_basis": "256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md; fhh_microbench)",
                "avg_launch_us": avg_launch_s * 1e6, "blocks_per_launch": blocks_per_launch,
                "in_kernel_blocks_per_s": rate,
                "traffic_note": "HBM bytes per launch from rocprofv3 FETCH_SIZE (x2, gfx950) + WRITE_SIZE",
            },
            "roofline_lds": {
                "achieved_algorithmic": lds_gbps, "peak": LDS_PEAK_GBPS, "unit": "GB/s",
                "frac_algorithmic": lds_gbps / LDS_PEAK_GBPS,
                "algorithmic": f"{LDS_BYTES_PER_BLOCK} B of ds_read_b32 T-table lookups per AES block",
                "frac_executed": pmc_rates["lds_executed_frac"] if pmc_rates else None,
                "executed": "SQ_INSTS_LDS x 64 lanes x 4 B per launch / rocprof launch time (pmc_executed)",
            },
            "roofline_hbm": {"achieved": hbm_gbps, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                             "frac": hbm_gbps / HBM_PEAK_GBPS,
                             "algorithmic": f"{HBM_BYTES_PER_BLOCK} B per AES block (SURVEY 8d)"},
            "pmc_executed": pmc_rates,
        }
        if args.rehearse:
            out["rehearsal"] = (f"{world} ranks on {torch.cuda.device_count()} GPU(s), hosted all-reduce: "
                                "checks the N>1 path (sharding, per-level partial sums, timing), not a measurement")
        if args.microbench:
            import ctypes
            r = ctypes.c_double()
            fhh.lib().fhh_microbench(local_rank, 0, ctypes.byref(r))
            out["measured_valu_peak_tops"] = r.value / 1e12
            fhh.lib().fhh_microbench(local_rank, 1, ctypes.byref(r))
            out["measured_lds_peak_gbps"] = r.value / 1e9
        if world == 1 and not args.no_cpu_baseline and args.workload == "zipf":
            out["cpu_baseline"] = cpu_baseline(args)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if comm is not None:
        if dist is not None:
            dist.barrier()
        comm.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
