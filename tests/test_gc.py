"""Row f1: the garbled-circuit equality test (equalitytest.rs:25-219).

swanky (`fancy-garbling` @553ede0) is not vendored, so the wire format is parity-unpinned; the
oracle restates the published half-gates + TCCR scheme (fhh_oracle.c) and is pinned by the
reference's own functional test `eq_gc` (equalitytest.rs:222-266: masks[i] ^ results[i] ==
(gb_value[i] == ev_value[i])) and by garbling's defining properties; the HIP path is then
checked bit-exact against the oracle (tables, labels, decoding bits, outputs) and, inside the
level loop, against the plaintext-equality crawl."""
import numpy as np
import pytest

# equalitytest.rs:224-225
GB_VALUE = [[0, 1, 1, 0], [0, 0, 0, 0], [1, 1, 1, 0]]
EV_VALUE = [[0, 1, 1, 0], [0, 0, 0, 0], [1, 1, 1, 0]]
KEY = bytes(range(16))
DELTA = bytes(range(100, 116))


def _cases(rng, n, bits, p_equal=0.5):
    g = rng.integers(0, 2, (n, bits), dtype=np.uint8)
    e = g.copy()
    flip = rng.random(n) >= p_equal
    if bits:
        e[flip, rng.integers(0, bits, int(flip.sum()))] ^= 1
    return g, e


def test_oracle_eq_gc_reference_vectors(oracle):
    g = np.array(GB_VALUE, np.uint8)
    e = np.array(EV_VALUE, np.uint8)
    expected = (g == e).all(axis=1)
    for mask in (0, 1):
        tables, gbl, evl, dec = oracle.gc_garble_eq(g, e, mask, KEY, DELTA)
        results = oracle.gc_eval_eq(tables, gbl, evl, dec)
        masks = np.full(len(results), mask, np.uint8)
        assert np.array_equal((masks ^ results).astype(bool), expected)
    # and with the evaluator's strings changed, the unequal tests come out unequal
    e2 = e.copy()
    e2[0, 3] ^= 1
    e2[2, 0] ^= 1
    t, gl, el, d = oracle.gc_garble_eq(g, e2, 1, KEY, DELTA)
    assert np.array_equal((oracle.gc_eval_eq(t, gl, el, d) ^ 1).astype(bool), [False, True, False])


@pytest.mark.parametrize("bits", [1, 2, 3, 4, 6, 8])
def test_oracle_functional_random(oracle, bits):
    rng = np.random.default_rng(bits)
    g, e = _cases(rng, 700, bits)
    for mask in (0, 1):
        t, gl, el, d = oracle.gc_garble_eq(g, e, mask, KEY, DELTA, label_nonce=5, gate_base=9)
        out = oracle.gc_eval_eq(t, gl, el, d, gate_base=9)
        assert np.array_equal(out ^ mask, (g == e).all(axis=1).astype(np.uint8))


def test_oracle_garbling_is_input_independent(oracle):
    """The garbled tables and decoding bits depend on the key / Delta / tweaks only, never on
    the inputs (what lets the garbler send them before OT), and the active labels differ from
    the zero labels by exactly Delta (with its colour bit forced to 1) on the set bits."""
    rng = np.random.default_rng(3)
    g, e = _cases(rng, 200, 4)
    t0, gl0, el0, d0 = oracle.gc_garble_eq(np.zeros_like(g), np.zeros_like(e), 0, KEY, DELTA)
    t1, gl1, el1, d1 = oracle.gc_garble_eq(g, e, 1, KEY, DELTA)
    assert np.array_equal(t0, t1) and np.array_equal(d0, d1)
    D = np.frombuffer(DELTA, np.uint8).copy()
    D[0] |= 1
    assert np.array_equal(gl0[:, :4] ^ gl1[:, :4], g[:, :, None] * D)
    assert np.array_equal(el0 ^ el1, e[:, :, None] * D)
    assert np.array_equal(gl0[:, 4] ^ gl1[:, 4], np.broadcast_to(D, (200, 16)))   # mask wire, mask = 1
    # a wrong evaluator label (the other wire value) flips the result of a single-gate test
    tests = np.array([[0, 0], [1, 1]], np.uint8)
    t, gl, el, d = oracle.gc_garble_eq(tests, tests, 0, KEY, DELTA)
    assert oracle.gc_eval_eq(t, gl, el, d).tolist() == [1, 1]
    el_bad = el.copy()
    el_bad[:, 1] ^= D
    assert oracle.gc_eval_eq(t, gl, el_bad, d).tolist() == [0, 0]


# ---- HIP path -------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 1), (3, 4), (63, 2), (64, 2), (65, 3), (1000, 2), (4097, 8), (20000, 4),
                                    (500, 5), (300, 6), (130, 7)])
def test_gpu_gc_bit_exact(oracle, n, bits):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(n * 10 + bits)
    g, e = _cases(rng, n, bits)
    kc = fhh.KeyCollection(8, 1)
    # label_nonce 0 / 1 << 20 (multiples of the label counter stride: the label passes share AES
    # rounds 1-2) and 123 (unaligned: some lanes' counters carry out of byte 0, full rounds)
    for nonce, mask in ((123, 0), (123, 1), (0, 1), (1 << 20, 0)):
        out, tr = gc.equality_test(kc, g, e, mask, KEY, DELTA, label_nonce=nonce, gate_base=77, transcript=True)
        t, gl, el, d = oracle.gc_garble_eq(g, e, mask, KEY, DELTA, label_nonce=nonce, gate_base=77)
        assert np.array_equal(tr.tables, t)
        assert np.array_equal(tr.gb_labels, gl)
        assert np.array_equal(tr.ev_labels, el)
        assert np.array_equal(tr.decode, d)
        assert np.array_equal(out, oracle.gc_eval_eq(t, gl, el, d, gate_base=77))
        assert np.array_equal(out ^ mask, (g == e).all(axis=1).astype(np.uint8))


@pytest.mark.gpu
def test_gpu_eq_gc_reference_vectors():
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    kc = fhh.KeyCollection(8, 1)
    expected = [a == b for a, b in zip(GB_VALUE, EV_VALUE)]
    for seed in range(4):
        masks, results = gc.multiple_equality_test(kc, GB_VALUE, EV_VALUE, seed=seed)
        assert len(set(masks)) == 1   # one mask per call (equalitytest.rs:38-43)
        assert [m ^ r for m, r in zip(masks, results)] == expected


@pytest.mark.gpu
def test_gpu_gc_device_groups(oracle):
    """Device-resident batch, G groups x N clients (N not a multiple of 64), planes input."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(11)
    G, N, bits = 5, 1000, 2
    g = rng.integers(0, 2, (G, N, bits), dtype=np.uint8)
    e = g.copy()
    flip = rng.random((G, N)) < 0.3
    e[flip, 0] ^= 1
    kc = fhh.KeyCollection(8, 1)
    b = gc.DeviceGcBatch(gc.planes_from_bits(g), gc.planes_from_bits(e), N, 1, KEY, DELTA, label_nonce=3,
                         gate_base=4)
    gc.equality_device(kc, b)
    out = b.out.cpu().numpy()
    t, gl, el, d = oracle.gc_garble_eq(g.reshape(G * N, bits), e.reshape(G * N, bits), 1, KEY, DELTA,
                                       label_nonce=3, gate_base=4)
    assert np.array_equal(out, oracle.gc_eval_eq(t, gl, el, d, gate_base=4))
    assert np.array_equal(out ^ 1, (g == e).all(axis=2).reshape(-1).astype(np.uint8))
    # SoA tables on the device == the oracle's AoS ones
    assert np.array_equal(b.tables.cpu().numpy().reshape(bits - 1, 2, G * N, 16).transpose(2, 0, 1, 3), t)


def _pair(left, right, roots):
    import fuzzyheavyhitters_amd as fhh
    n, d, L = left.shape
    c0, c1 = fhh.KeyCollection(L, d), fhh.KeyCollection(L, d)
    fhh.gen_keys_pair(c0, c1, left, right, roots)
    return c0, c1


def _sig(res):
    return (res.level_children.tolist(), res.level_kept.tolist(), [c.tolist() for c in res.counts],
            [(r.path, r.value) for r in res.final])


@pytest.mark.gpu
@pytest.mark.parametrize("gc_mode", ["ideal", "ot", "ot+co15", "ot-circuit", "ot-circuit+co15"])
@pytest.mark.parametrize("kind", ["zipf_d1", "coords_d2"])
def test_gpu_crawl_with_gc_equals_plain(kind, gc_mode):
    """tree_crawl with the GC equality test (collect.rs:419-482) gives the same FE sums, keep
    decisions and heavy hitters as the plaintext-equality harness, level by level; "ot+co15" runs
    both OT extensions of every level on real Chou–Orlandi base OTs (host threads)."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    if kind == "zipf_d1":
        wl = workload.zipf_workload(3000, 64, 1, num_sites=40, seed=5)
        thr = 0.01
    else:
        wl = workload.coords_workload(1500, ball_size=3, num_centroids=40, side_km=4.0)
        thr = 0.01
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    plain = sim_crawl(c0, c1, thr, mode="fe", prf_seed=9)
    with_gc = sim_crawl(c0, c1, thr, mode="fe", prf_seed=9, gc=gc_mode.split("+")[0], init_capacity=2,
                        base_ot=gc_mode.endswith("co15"))
    assert _sig(with_gc) == _sig(plain)
    assert len(with_gc.final) > 0
    if gc_mode.endswith("co15"):
        assert c0.stats()["base_ot_ms"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("ss_k", [2, 4])
@pytest.mark.parametrize("gc_mode", ["ot", "ot+co15", "ot-circuit"])
@pytest.mark.parametrize("kind", ["zipf_d1", "coords_d2"])
def test_gpu_crawl_with_softspoken_equals_plain(kind, gc_mode, ss_k):
    """r06: both OT kinds of every level on SoftSpoken OT extension (k = 2, 4: 128 / k rows of U) give the
    same sums, keep decisions and heavy hitters as the plaintext harness, with ideal and with real
    Chou-Orlandi base OTs, the garbled table (d = 1: tile-major, d = 2: row form) and the circuit."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    if kind == "zipf_d1":
        wl = workload.zipf_workload(3000, 64, 1, num_sites=40, seed=5)
    else:
        wl = workload.coords_workload(1500, ball_size=3, num_centroids=40, side_km=4.0)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    plain = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=9)
    got = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=9, gc=gc_mode.split("+")[0], init_capacity=2,
                    base_ot=gc_mode.endswith("co15"), ot_ss_k=ss_k)
    assert _sig(got) == _sig(plain)
    assert len(got.final) > 0


def test_sim_crawl_rejects_bad_ss_k():
    from fuzzyheavyhitters_amd import sim_crawl
    with pytest.raises(ValueError):
        sim_crawl(None, None, 0.01, mode="fe", gc="ot", ot_ss_k=3)


@pytest.mark.gpu
@pytest.mark.parametrize("gc_mode", ["ideal", "ot", "ot+co15", "ot-circuit"])
def test_gpu_crawl_with_gc_in_chunks(monkeypatch, gc_mode):
    """A level's GC + OT split into chunks of children, each a fresh protocol instance (the
    reference spreads a level's tests over its channels, collect.rs:423-430; the device loop
    chunks so the GC and OT buffers of 1M clients stay bounded): FHH_GC_CHUNK_BYTES small enough
    for 3 children per chunk -> the same sums, keep decisions and heavy hitters as the plaintext
    harness (the last chunk of a level partial, chunks past C no-ops). "ot+co15": every chunk's two
    OT extensions start from their own real Chou–Orlandi base OTs (the metric's 1M crawl runs ~7
    chunks per level), with capacity growth and resumed levels (init_capacity 2)."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(1000, 48, 1, num_sites=30, seed=17)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    plain = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=3)
    npad = (1000 + 63) // 64 * 64
    monkeypatch.setenv("FHH_GC_CHUNK_BYTES", str(3 * 402 * npad))   # 3 children x ~402 B per test (d = 1)
    co15 = gc_mode.endswith("co15")
    with_gc = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=3, gc=gc_mode.split("+")[0], base_ot=co15,
                        init_capacity=2 if co15 else 0)
    assert _sig(with_gc) == _sig(plain)
    assert max(plain.level_children) > 6 and len(with_gc.final) > 0
    if co15:
        assert c0.stats()["base_ot_ms"] > 0


@pytest.mark.gpu
def test_gpu_crawl_gc_rejects_count_mode():
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(200, 40, 1, num_sites=10, seed=1)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    with pytest.raises(fhh.FhhError):
        sim_crawl(c0, c1, 0.01, mode="count", gc=True)


# ---- r05: the evaluator's labels by correlated OT, the garbler's string folded in --------------------
def _oracle_cot_chain(oracle, g, e, mask, seeds, s, gate_base=0, ctr_off=0, share=False):
    """The labels OT (r05b: the IKNP correlation itself; choice bits: the evaluator's bits at OT index
    j npad + i), garbling on its zero labels q_j with Delta = s and the garbler's string and mask folded
    in, evaluation on the evaluator's t_j — all in the oracle."""
    n, bits = g.shape
    npad = (n + 63) // 64 * 64
    ch = np.zeros(bits * npad, np.uint8)
    for k in range(bits):
        ch[k * npad: k * npad + n] = e[:, k]
    q, t_rows, u, _ = oracle.cot_extend(oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
    ev_zero = np.stack([q[k * npad: k * npad + n] for k in range(bits)], axis=1)
    ev_act = np.stack([t_rows[k * npad: k * npad + n] for k in range(bits)], axis=1)
    if share:   # r05c: the FE share from the output labels
        t, d, gv, y = oracle.gc_garble_eq_cot(g, ev_zero, mask, s, gate_base=gate_base, share=True)
        res, ev = oracle.gc_eval_eq_cot(t, ev_act, d, gate_base=gate_base, share_y=y)
        return res, dict(tables=t, ev_zero=ev_zero, ev_active=ev_act, decode=d, gb_share=gv, ev_share=ev,
                         share_y=y)
    t, d = oracle.gc_garble_eq_cot(g, ev_zero, mask, s, gate_base=gate_base)
    res = oracle.gc_eval_eq_cot(t, ev_act, d, gate_base=gate_base)
    return res, dict(tables=t, ev_zero=ev_zero, ev_active=ev_act, decode=d)


def _colour_s(rng):
    """The garbler's labels-kind s: the circuit's free-XOR Delta, so its colour bit (bit 0) is 1."""
    s = rng.integers(0, 256, 16, dtype=np.uint8)
    s[0] |= 1
    return s.tobytes()


@pytest.mark.parametrize("bits", [1, 2, 4, 8])
def test_oracle_cot_labels_chain_functional(oracle, bits):
    """eq_gc's assertion (equalitytest.rs:258-265) through the r05 labels step: masks ^ results ==
    (gb == ev), for both masks and for complemented evaluator strings; the evaluator's active labels
    differ from the labels OT's zero labels by Delta = s exactly on its set bits."""
    rng = np.random.default_rng(40 + bits)
    g, e = _cases(rng, 300, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    for mask in (0, 1):
        out, tr = _oracle_cot_chain(oracle, g, e, mask, seeds, s, gate_base=5, ctr_off=256)
        assert np.array_equal(out ^ mask, (g == e).all(axis=1).astype(np.uint8))
        D = np.frombuffer(s, np.uint8)   # Delta = s
        assert np.array_equal(tr["ev_zero"] ^ tr["ev_active"], e[:, :, None] * D)
        out2, _ = _oracle_cot_chain(oracle, g, 1 - e, mask, seeds, s, gate_base=5, ctr_off=256)
        assert np.array_equal(out2 ^ mask, (g == 1 - e).all(axis=1).astype(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 1), (63, 2), (65, 2), (1000, 2), (4097, 4), (300, 6), (130, 8)])
def test_gpu_cot_labels_chain_bit_exact(oracle, n, bits):
    """fhh_gc_cot_host (the labels OT + garble + evaluate of one batch) = the oracle chain: zero labels,
    active labels, tables, decoding bits, outputs; an s without the colour bit is refused."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(n * 3 + bits)
    g, e = _cases(rng, n, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    kc = fhh.KeyCollection(8, 1)
    with pytest.raises(fhh.FhhError):   # Delta = s needs the colour bit
        gc.equality_test_cot(kc, g, e, 0, seeds, bytes([s[0] & 0xFE]) + s[1:])
    for mask, ctr in ((0, 0), (1, 256), (1, 512)):
        out, tr = gc.equality_test_cot(kc, g, e, mask, seeds, s, gate_base=7, ctr_off=ctr)
        exp, etr = _oracle_cot_chain(oracle, g, e, mask, seeds, s, gate_base=7, ctr_off=ctr)
        for k in ("ev_zero", "ev_active", "tables", "decode"):
            assert np.array_equal(tr[k], etr[k]), k
        assert np.array_equal(out, exp)
        assert np.array_equal(out ^ mask, (g == e).all(axis=1).astype(np.uint8))


# ---- r05c: the FE share from the circuit's output labels (no second OT at the FE levels) -----------
FE_P = (1 << 62) - (1 << 30) - 1


@pytest.mark.parametrize("bits", [2, 4])
def test_oracle_output_label_share_functional(oracle, bits):
    """The share pair of collect.rs:437-452 from the output labels: gb_share - ev_share = eq (mod p) for
    every test and both masks (so the level sums reconstruct the plaintext counts): the evaluator's value
    is pair[o] of the garbler's (v, mask ? v + 1 : v - 1) and gb_share = v + mask; values are canonical
    FE (< p); y depends on Delta."""
    rng = np.random.default_rng(70 + bits)
    g, e = _cases(rng, 500, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    for mask in (0, 1):
        out, tr = _oracle_cot_chain(oracle, g, e, mask, seeds, s, gate_base=3, share=True)
        eq = (g == e).all(axis=1)
        assert np.array_equal(out ^ mask, eq.astype(np.uint8))
        gv, ev = tr["gb_share"].astype(object), tr["ev_share"].astype(object)
        assert all(int(x) < FE_P for x in tr["gb_share"]) and all(int(x) < FE_P for x in tr["ev_share"])
        assert np.array_equal(((gv - ev) % FE_P).astype(np.uint64), eq.astype(np.uint64))
        # y hides pair[1] behind H(W_1): a different Delta gives different messages
        s2 = bytes([s[0]]) + bytes((b ^ 0x5A) for b in s[1:])
        _, tr2 = _oracle_cot_chain(oracle, g, e, mask, seeds, s2, gate_base=3, share=True)
        assert not np.array_equal(tr2["share_y"], tr["share_y"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 2), (65, 2), (1000, 2), (4097, 4), (130, 8)])
def test_gpu_output_label_share_bit_exact(oracle, n, bits):
    """fhh_gc_cot_host's share outputs (k_gc_garble_cot's node values and y, k_gc_eval's node values)
    = the oracle's, bit for bit, with the rest of the transcript unchanged; gb - ev = eq mod p."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(n * 5 + bits)
    g, e = _cases(rng, n, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    kc = fhh.KeyCollection(8, 1)
    for mask, ctr in ((0, 0), (1, 256)):
        out, tr = gc.equality_test_cot(kc, g, e, mask, seeds, s, gate_base=9, ctr_off=ctr, share=True)
        exp, etr = _oracle_cot_chain(oracle, g, e, mask, seeds, s, gate_base=9, ctr_off=ctr, share=True)
        for k in ("ev_zero", "ev_active", "tables", "decode", "gb_share", "share_y", "ev_share"):
            assert np.array_equal(tr[k], etr[k]), k
        assert np.array_equal(out, exp)
        eq = (g == e).all(axis=1).astype(np.uint64)
        assert np.array_equal(((tr["gb_share"].astype(object) - tr["ev_share"].astype(object)) % FE_P)
                              .astype(np.uint64), eq)


# ---- r05d: the FE levels' garbled table (one b-input garbled gate per test) ------------------------
def _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=0, ctr_off=0):
    """The labels OT (the IKNP correlation), then the garbled table on its zero labels and the
    evaluator's row on its t_j — all in the oracle. OT index k npad + i: npad = n rounded up to 512 for
    b <= 2 (r06: the GPU's table kernels read the tile-major Q / T, one client range per 512-OT tile), to 64
    for b = 3, 4."""
    n, bits = g.shape
    npad = (n + 511) // 512 * 512 if bits <= 2 else (n + 63) // 64 * 64
    ch = np.zeros(bits * npad, np.uint8)
    for k in range(bits):
        ch[k * npad: k * npad + n] = e[:, k]
    q, t_rows, _, _ = oracle.cot_extend(oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
    ev_zero = np.stack([q[k * npad: k * npad + n] for k in range(bits)], axis=1)
    ev_act = np.stack([t_rows[k * npad: k * npad + n] for k in range(bits)], axis=1)
    msgs, gv = oracle.gt_garble(g, ev_zero, mask, s, gate_base=gate_base)
    ev = oracle.gt_eval(ev_act, msgs, gate_base=gate_base)
    return dict(ev_zero=ev_zero, ev_active=ev_act, msgs=msgs, gb_share=gv, ev_share=ev)


@pytest.mark.parametrize("bits", [1, 2, 3, 4])
def test_oracle_garbled_table_functional(oracle, bits):
    """The garbled table's share: gb_share - ev_share = eq (mod p) for every test and both masks; values
    canonical; the evaluator's row is named by its labels' colours (each row is reached); messages depend
    on Delta and on the tweak."""
    rng = np.random.default_rng(90 + bits)
    g, e = _cases(rng, 600, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    for mask in (0, 1):
        tr = _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=21)
        eq = (g == e).all(axis=1).astype(np.uint64)
        assert all(int(x) < FE_P for x in tr["gb_share"]) and all(int(x) < FE_P for x in tr["ev_share"])
        diff = (tr["gb_share"].astype(object) - tr["ev_share"].astype(object)) % FE_P
        assert np.array_equal(diff.astype(np.uint64), eq)
        rows = sum(((tr["ev_active"][:, k, 0] & 1).astype(int) << k) for k in range(bits))
        assert len(set(rows.tolist())) == 1 << bits
        tr2 = _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=22)
        assert not np.array_equal(tr2["msgs"], tr["msgs"])


def _oracle_table_chain_ring32(oracle, g, e, mask, seeds, s, gate_base=0, ctr_off=0):
    """_oracle_table_chain with the table's shares in Z_2^32 (r06, orc_gt_*_ring32)."""
    tr = _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=gate_base, ctr_off=ctr_off)
    msgs, gv = oracle.gt_garble_ring32(g, tr["ev_zero"], mask, s, gate_base=gate_base)
    ev = oracle.gt_eval_ring32(tr["ev_active"], msgs, gate_base=gate_base)
    return dict(ev_zero=tr["ev_zero"], ev_active=tr["ev_active"], msgs=msgs, gb_share=gv, ev_share=ev)


@pytest.mark.parametrize("bits", [1, 2])
def test_oracle_garbled_table_ring32_functional(oracle, bits):
    """r06: the Z_2^32 table — gb_share - ev_share = eq (mod 2^32) for every test and both masks; row 0's value
    and every message are the FE form's low 32 bits' counterparts (same hashes, same rows)."""
    rng = np.random.default_rng(190 + bits)
    g, e = _cases(rng, 600, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    for mask in (0, 1):
        tr = _oracle_table_chain_ring32(oracle, g, e, mask, seeds, s, gate_base=21)
        eq = (g == e).all(axis=1).astype(np.uint32)
        assert np.array_equal((tr["gb_share"] - tr["ev_share"]).astype(np.uint32), eq)
        fe = _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=21)
        rows = sum(((tr["ev_active"][:, k, 0] & 1).astype(int) << k) for k in range(bits))
        # a test whose row is r > 0 reads message r: the low 32 bits of the FE message's hash part agree
        assert tr["msgs"].shape == fe["msgs"].shape and (rows > 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 2), (65, 1), (1000, 2), (4097, 2)])
def test_gpu_garbled_table_ring32_bit_exact(oracle, n, bits):
    """r06: fhh_gt_cot_ring32_host (the tile-major table kernels with Z_2^32 shares) = the oracle chain bit for
    bit: every 4-B message and both parties' values; gb - ev = eq mod 2^32."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(n * 11 + bits)
    g, e = _cases(rng, n, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    kc = fhh.KeyCollection(8, 1)
    for mask, ctr in ((0, 0), (1, 256)):
        tr = gc.table_cot(kc, g, e, mask, seeds, s, gate_base=13, ctr_off=ctr, ring32=True)
        etr = _oracle_table_chain_ring32(oracle, g, e, mask, seeds, s, gate_base=13, ctr_off=ctr)
        for k in ("ev_zero", "ev_active", "msgs", "gb_share", "ev_share"):
            assert np.array_equal(tr[k], etr[k].astype(tr[k].dtype)), k
        eq = (g == e).all(axis=1).astype(np.uint64)
        assert np.array_equal((tr["gb_share"] - tr["ev_share"]) & 0xFFFFFFFF, eq)


@pytest.mark.gpu
@pytest.mark.parametrize("gc_mode", ["ot", "ot+co15"])
@pytest.mark.parametrize("ss_k", [1, 2])
def test_gpu_crawl_with_ring32_table_equals_plain(gc_mode, ss_k):
    """r06: the level loop with the FE levels' table in Z_2^32 (d = 1) gives the plaintext harness's counts, keep
    decisions and heavy hitters level by level, chunked (3 children per protocol instance) and whole."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(3000, 64, 1, num_sites=40, seed=5)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    plain = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=9)
    got = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=9, gc="ot", init_capacity=2, base_ot=gc_mode.endswith("co15"),
                    ot_ss_k=ss_k, table_ring32=True)
    assert _sig(got) == _sig(plain)
    assert len(got.final) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits", [(1, 2), (65, 1), (1000, 2), (777, 3), (4097, 4)])
def test_gpu_garbled_table_bit_exact(oracle, n, bits):
    """fhh_gt_cot_host (labels OT + k_gt_garble + k_gt_eval) = the oracle chain bit for bit: zero and
    active labels, every row's message, both parties' node values; gb - ev = eq mod p."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import gc
    rng = np.random.default_rng(n * 7 + bits)
    g, e = _cases(rng, n, bits)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = _colour_s(rng)
    kc = fhh.KeyCollection(8, 1)
    for mask, ctr in ((0, 0), (1, 256)):
        tr = gc.table_cot(kc, g, e, mask, seeds, s, gate_base=13, ctr_off=ctr)
        etr = _oracle_table_chain(oracle, g, e, mask, seeds, s, gate_base=13, ctr_off=ctr)
        for k in ("ev_zero", "ev_active", "msgs", "gb_share", "ev_share"):
            assert np.array_equal(tr[k], etr[k]), k
        eq = (g == e).all(axis=1).astype(np.uint64)
        assert np.array_equal(((tr["gb_share"].astype(object) - tr["ev_share"].astype(object)) % FE_P)
                              .astype(np.uint64), eq)
