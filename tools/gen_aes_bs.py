#!/usr/bin/env python3
"""Generate fuzzyheavyhitters_amd/csrc/aes_bs_gen.h: a bitsliced AES-128 with the fixed
all-zero key (the PRG of src/prg.rs:185-234) expressed as gfx950 `v_bitop3_b32` ops.

Bitsliced layout: state word i (0..127) holds bit i of 32 blocks (one block per bit
position of the u32); block bit i = bit (i & 7) of byte (i >> 3), byte k = 4*column + row
(the FIPS-197 input order, the same little-endian column words the T-table path uses).

Pipeline (all checked here in Python before anything is emitted):
  1. S-box = the Boyar-Peralta 113-gate circuit (+2 shared temporaries), checked against the
     FIPS-197 S-box on all 256 inputs;
  2. MixColumns per column as t_r = a_r ^ a_{r+1} and out_r = xtime(t_r) ^ a_{r+1} ^ t_{r+2};
  3. each network is technology-mapped to 3-input LUTs (cut enumeration + area flow) — one
     LUT = one v_bitop3_b32 with the LUT's truth table as the immediate;
  4. AddRoundKey with the zero key's round keys (compile-time constants) folds into the
     truth tables of the producing LUTs (complemented outputs), so it costs nothing;
  5. a full 10-round bitsliced evaluation of the emitted program is compared with a
     byte-oriented AES-128 on random blocks and the FIPS-197 zero-key vector.

v_bitop3_b32 D = imm[(S0 << 2) | (S1 << 1) | S2] per bit (the convention of LLVM's
AMDGPU BitOp3 matcher: S0 = 0xF0, S1 = 0xCC, S2 = 0xAA); emitted as Ops::template b3<imm>(S0, S1, S2).

Usage: python tools/gen_aes_bs.py [--check-only]
"""
from __future__ import annotations

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fuzzyheavyhitters_amd", "csrc", "aes_bs_gen.h")

# Boyar-Peralta S-box circuit (J. Boyar, R. Peralta, "A small depth-16 circuit for the AES
# S-box", 2012), in the well-known bitsliced form; x0 = MSB of the input byte, s0 = MSB out.
BP = """
y14 = x3 ^ x5
y13 = x0 ^ x6
y9 = x0 ^ x3
y8 = x0 ^ x5
t0 = x1 ^ x2
y1 = t0 ^ x7
y4 = y1 ^ x3
y12 = y13 ^ y14
y2 = y1 ^ x0
y5 = y1 ^ x6
y3 = y5 ^ y8
t1 = x4 ^ y12
y15 = t1 ^ x5
y20 = t1 ^ x1
y6 = y15 ^ x7
y10 = y15 ^ t0
y11 = y20 ^ y9
y7 = x7 ^ y11
y17 = y10 ^ y11
y19 = y10 ^ y8
y16 = t0 ^ y11
y21 = y13 ^ y16
y18 = x0 ^ y16
t2 = y12 & y15
t3 = y3 & y6
t4 = t3 ^ t2
t5 = y4 & x7
t6 = t5 ^ t2
t7 = y13 & y16
t8 = y5 & y1
t9 = t8 ^ t7
t10 = y2 & y7
t11 = t10 ^ t7
t12 = y9 & y11
t13 = y14 & y17
t14 = t13 ^ t12
t15 = y8 & y10
t16 = t15 ^ t12
t17 = t4 ^ t14
t18 = t6 ^ t16
t19 = t9 ^ t14
t20 = t11 ^ t16
t21 = t17 ^ y20
t22 = t18 ^ y19
t23 = t19 ^ y21
t24 = t20 ^ y18
t25 = t21 ^ t22
t26 = t21 & t23
t27 = t24 ^ t26
t28 = t25 & t27
t29 = t28 ^ t22
t30 = t23 ^ t24
t31 = t22 ^ t26
t32 = t31 & t30
t33 = t32 ^ t24
t34 = t23 ^ t33
t35 = t27 ^ t33
t36 = t24 & t35
t37 = t36 ^ t34
t38 = t27 ^ t36
t39 = t29 & t38
t40 = t25 ^ t39
t41 = t40 ^ t37
t42 = t29 ^ t33
t43 = t29 ^ t40
t44 = t33 ^ t37
t45 = t42 ^ t41
z0 = t44 & y15
z1 = t37 & y6
z2 = t33 & x7
z3 = t43 & y16
z4 = t40 & y1
z5 = t29 & y7
z6 = t42 & y11
z7 = t45 & y17
z8 = t41 & y10
z9 = t44 & y12
z10 = t37 & y3
z11 = t33 & y4
z12 = t43 & y13
z13 = t40 & y5
z14 = t29 & y2
z15 = t42 & y9
z16 = t45 & y14
z17 = t41 & y8
t46 = z15 ^ z16
t47 = z10 ^ z11
t48 = z5 ^ z13
t49 = z9 ^ z10
t50 = z2 ^ z12
t51 = z2 ^ z5
t52 = z7 ^ z8
t53 = z0 ^ z3
t54 = z6 ^ z7
t55 = z16 ^ z17
t56 = z12 ^ t48
t57 = t50 ^ t53
t58 = z4 ^ t46
t59 = z3 ^ t54
t60 = t46 ^ t57
t61 = z14 ^ t57
t62 = t52 ^ t58
t63 = t49 ^ t58
t64 = z4 ^ t59
t65 = t61 ^ t62
t66 = z1 ^ t63
s0 = t59 ^ t63
s6 = t56 ^ ~t62
s7 = t48 ^ ~t60
t67 = t64 ^ t65
s3 = t53 ^ t66
s4 = t51 ^ t66
s5 = t47 ^ t65
s1 = t64 ^ ~s3
s2 = t55 ^ ~t67
"""


# ---------------------------------------------------------------------------------------
# byte-oriented AES-128 (FIPS-197) for the checks
# ---------------------------------------------------------------------------------------
def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ 0x11B) if a & 0x80 else a << 1
        b >>= 1
    return r


def make_sbox():
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if gmul(a, b) == 1:
                inv[a] = b
                break
    sb = []
    for a in range(256):
        x, s = inv[a], 0x63
        for _ in range(5):
            s ^= x
            x = ((x << 1) | (x >> 7)) & 0xFF
        sb.append(s)
    return sb


SBOX = make_sbox()


def key_expand(key):
    rcon = [0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36]
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [SBOX[b] for b in t]
            t[0] ^= rcon[i // 4 - 1]
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [sum((w[4 * r + c] for c in range(4)), []) for r in range(11)]   # 11 x 16 bytes


RK = key_expand([0] * 16)


def aes_ref(block):
    s = [b ^ k for b, k in zip(block, RK[0])]
    for r in range(1, 11):
        s = [SBOX[b] for b in s]
        s = [s[4 * ((c + row) % 4) + row] for c in range(4) for row in range(4)]   # ShiftRows
        if r < 10:
            out = []
            for c in range(4):
                a = s[4 * c:4 * c + 4]
                for row in range(4):
                    out.append(gmul(a[row], 2) ^ gmul(a[(row + 1) % 4], 3) ^ a[(row + 2) % 4] ^ a[(row + 3) % 4])
            s = out
        s = [b ^ k for b, k in zip(s, RK[r])]
    return s


# ---------------------------------------------------------------------------------------
# 3-LUT technology mapping
# ---------------------------------------------------------------------------------------
def opf(op, a, b):
    return {"^": a ^ b, "&": a & b, "xnor": 1 ^ a ^ b}[op]


class Net:
    def __init__(self):
        self.pis, self.gates, self.order, self.pos = [], {}, [], []

    def pi(self, n):
        self.pis.append(n)
        return n

    def g(self, n, op, a, b):
        assert n not in self.gates
        self.gates[n] = (op, a, b)
        self.order.append(n)
        return n


def truth(net, node, leaves):
    """truth table of `node` over `leaves` (<= 3); minterm m = sum(leaf_i << i)"""
    tt = 0
    for m in range(8):
        env = {l: (m >> i) & 1 for i, l in enumerate(leaves)}

        def ev(n):
            if n in env:
                return env[n]
            op, a, b = net.gates[n]
            v = opf(op, ev(a), ev(b))
            env[n] = v
            return v

        tt |= ev(node) << m
    return tt


def lut_map(net, K=3, iters=6, rng=None):
    fanout = {n: 0 for n in net.pis + net.order}
    for n in net.order:
        _, a, b = net.gates[n]
        fanout[a] += 1
        fanout[b] += 1
    for o in net.pos:
        fanout[o] += 1
    cuts = {p: [frozenset([p])] for p in net.pis}
    for n in net.order:
        _, a, b = net.gates[n]
        cs = {c1 | c2 for c1 in cuts[a] for c2 in cuts[b] if len(c1 | c2) <= K}
        keep = []
        for c in sorted(cs, key=lambda c: (len(c), sorted(c))):
            if not any(k <= c for k in keep):
                keep.append(c)
        keep.sort(key=lambda c: (len(c), sorted(c)))
        if rng is not None:
            rng.shuffle(keep)
        cuts[n] = keep + [frozenset([n])]
    est = {n: max(1, fanout[n]) for n in fanout}
    best_sel, best = None, None
    for _ in range(iters):
        af, choice = {p: 0.0 for p in net.pis}, {}
        for n in net.order:
            bc, bv = None, 1e18
            for c in cuts[n]:
                if c == frozenset([n]):
                    continue
                v = 1 + sum(af[u] / est[u] for u in c)
                if v < bv - 1e-9 or (abs(v - bv) < 1e-9 and len(c) < len(bc)):
                    bv, bc = v, c
            af[n], choice[n] = bv, bc
        sel, stack = set(), list(net.pos)
        while stack:
            n = stack.pop()
            if n in net.pis or n in sel:
                continue
            sel.add(n)
            stack.extend(choice[n])
        refs = {n: 0 for n in fanout}
        for n in sel:
            for u in choice[n]:
                refs[u] += 1
        for o in net.pos:
            refs[o] += 1
        est = {n: max(1, refs[n]) for n in fanout}
        if best_sel is None or len(sel) < len(best_sel):
            best_sel, best = sel, dict(choice)
    prog = []
    for n in net.order:
        if n in best_sel:
            leaves = sorted(best[n], key=lambda x: (net.pis + net.order).index(x))
            prog.append((n, leaves, truth(net, n, leaves)))
    return prog


def run_prog(prog, env):
    env = dict(env)
    for n, leaves, tt in prog:
        m = 0
        for i, l in enumerate(leaves):
            m |= env[l] << i
        env[n] = (tt >> m) & 1
    return env


# ---------------------------------------------------------------------------------------
# networks
# ---------------------------------------------------------------------------------------
def parse_bp():
    gates = []
    for line in BP.strip().splitlines():
        o, e = [s.strip() for s in line.split("=")]
        a, op, b = e.split()
        neg = b.startswith("~")
        gates.append((o, "xnor" if neg else op, a, b.lstrip("~")))
    return gates


def sbox_net():
    net = Net()
    for i in range(8):
        net.pi(f"x{i}")
    for o, op, a, b in parse_bp():
        net.g(o, op, a, b)
    net.pos = [f"s{i}" for i in range(8)]
    return net


def mixcol_net():
    """one column: inputs a{r}_{k} (row r, bit k LSB-first), outputs o{r}_{k}"""
    net = Net()
    for r in range(4):
        for k in range(8):
            net.pi(f"a{r}_{k}")
    for r in range(4):
        for k in range(8):
            net.g(f"t{r}_{k}", "^", f"a{r}_{k}", f"a{(r + 1) % 4}_{k}")
    outs = []
    for r in range(4):
        for k in range(8):
            terms = [f"a{(r + 1) % 4}_{k}", f"t{(r + 2) % 4}_{k}"]
            if k > 0:
                terms.append(f"t{r}_{k - 1}")
            if k in (1, 3, 4) or k == 0:
                terms.append(f"t{r}_7")
            cur = terms[0]
            for j, x in enumerate(terms[1:]):
                cur = net.g(f"m{r}_{k}_{j}", "^", cur, x)
            outs.append(cur)
    net.pos = outs
    return net


def peak_live(prog, inputs, outputs):
    """max simultaneously live values (inputs until their last use, outputs to the end)"""
    uses = {}
    for _, leaves, _ in prog:
        for l in set(leaves):
            uses[l] = uses.get(l, 0) + 1
    live = set(inputs)
    peak = len(live)
    outs = set(outputs)
    for n, leaves, _ in prog:
        for l in set(leaves):
            uses[l] -= 1
            if uses[l] == 0 and l not in outs:
                live.discard(l)
        live.add(n)
        peak = max(peak, len(live))
    return peak


def schedule(prog, inputs, outputs, trials, rng):
    """reorder a LUT program (topologically) to minimise peak register pressure: randomised
    greedy list scheduling that prefers ops freeing the most operands"""
    best, best_peak = list(prog), peak_live(prog, inputs, outputs)
    byname = {n: (n, leaves, tt) for n, leaves, tt in prog}
    outs = set(outputs)
    for _ in range(trials):
        uses = {}
        for _, leaves, _ in prog:
            for l in set(leaves):
                uses[l] = uses.get(l, 0) + 1
        avail = set(inputs)
        pending = {n for n, _, _ in prog}
        order = []
        while pending:
            ready = [n for n in pending if all(l in avail for l in byname[n][1])]
            def score(n):
                freed = sum(1 for l in set(byname[n][1]) if uses[l] == 1 and l not in outs)
                return freed - 1 + rng.random() * 0.9
            n = max(ready, key=score)
            pending.discard(n)
            for l in set(byname[n][1]):
                uses[l] -= 1
            avail.add(n)
            order.append(byname[n])
        pk = peak_live(order, inputs, outputs)
        if pk < best_peak:
            best, best_peak = order, pk
    return best, best_peak


class Program:
    """LUT program with named inputs/outputs; outputs may be complemented at emission."""

    def __init__(self, net, trials=1, sched_trials=0):
        self.net = net
        self.prog = lut_map(net)
        rng = random.Random(12345)
        for _ in range(trials - 1):   # randomised tie-breaking; keep the smallest cover
            p = lut_map(net, rng=rng)
            if len(p) < len(self.prog):
                self.prog = p
        self.inputs = list(net.pis)
        self.outputs = list(net.pos)
        self.peak = peak_live(self.prog, self.inputs, self.outputs)
        if sched_trials:
            self.prog, self.peak = schedule(self.prog, self.inputs, self.outputs, sched_trials, rng)

    def __len__(self):
        return len(self.prog)


# ---------------------------------------------------------------------------------------
# emission + bitsliced simulation (the simulation runs exactly the op list that is emitted)
# ---------------------------------------------------------------------------------------
class Emitter:
    def __init__(self):
        self.lines = []
        self.ops = []     # (dst, a, b, c, imm) with operand names
        self.n = 0
        self.units = 0

    def new(self):
        self.n += 1
        return f"v{self.n}"

    def fence(self):
        self.lines.append(f"    Ops::template fence<{self.units}>();")
        self.units += 1

    def b3(self, a, b, c, imm):
        d = self.new()
        self.ops.append((d, a, b, c, imm))
        self.lines.append(f"    const uint32_t {d} = Ops::template b3<0x{imm:02X}>({a}, {b}, {c});")
        return d


def imm_for(leaves_vals, tt):
    """operands (S0, S1, S2) and immediate for a LUT over 1..3 leaves (leaf i = minterm bit i)"""
    k = len(leaves_vals)
    if k == 3:
        return leaves_vals[2], leaves_vals[1], leaves_vals[0], tt
    if k == 2:
        # S0 = S1 = leaf1, S2 = leaf0: index = 6*l1 + l0
        imm = 0
        for m in range(8):
            l0, l1 = m & 1, (m >> 1) & 1
            imm |= ((tt >> (l0 | (l1 << 1))) & 1) << m
        return leaves_vals[1], leaves_vals[1], leaves_vals[0], imm
    if k == 1:
        imm = 0
        for m in range(8):
            imm |= ((tt >> (m & 1)) & 1) << m
        return leaves_vals[0], leaves_vals[0], leaves_vals[0], imm
    raise ValueError(k)


def emit_prog(em, P, inmap, comp):
    """emit LUT program P with inputs bound to operand names in `inmap`; outputs whose
    name is in `comp` are complemented. Returns {output name: operand}."""
    env = dict(inmap)
    used_as_leaf = {l for _, leaves, _ in P.prog for l in leaves}
    out = {}
    for n, leaves, tt in P.prog:
        flip = n in comp and n not in used_as_leaf
        a, b, c, imm = imm_for([env[l] for l in leaves], tt ^ (0xFF if flip else 0))
        env[n] = em.b3(a, b, c, imm)
        if flip:
            out[n] = env[n]
    for o in P.outputs:
        if o in out:
            continue
        if o in comp:   # internal fanout: complement with one extra op
            out[o] = em.b3(env[o], env[o], env[o], 0x0F)
        else:
            out[o] = env[o]
    return out


def gen_aes(em, SB, MC, rounds=range(1, 11), keyed=True):
    """state operands st[i] (bit i) -> AES_0 rounds `rounds` (round 0 key is zero); keyed=False
    leaves AddRoundKey out (the rolled form applies it at run time)."""
    st = [f"s[{i}]" for i in range(128)]
    for r in rounds:
        rk_bits = [(RK[r][i >> 3] >> (i & 7)) & 1 if keyed else 0 for i in range(128)]
        sub = [None] * 128
        for byte in range(16):
            inmap = {f"x{i}": st[8 * byte + (7 - i)] for i in range(8)}
            # ShiftRows: byte (row, col) lands at (row, col - row)
            row, col = byte % 4, byte // 4
            dst = 4 * ((col - row) % 4) + row
            comp = set()
            if r == 10:
                comp = {f"s{i}" for i in range(8) if rk_bits[8 * dst + (7 - i)]}
            o = emit_prog(em, SB, inmap, comp)
            em.fence()
            for i in range(8):
                sub[8 * dst + (7 - i)] = o[f"s{i}"]
        if r == 10:
            st = sub
            break
        new = [None] * 128
        for c in range(4):
            inmap = {f"a{row}_{k}": sub[8 * (4 * c + row) + k] for row in range(4) for k in range(8)}
            names = MC.outputs   # order: r-major, k
            comp = {names[8 * row + k] for row in range(4) for k in range(8) if rk_bits[8 * (4 * c + row) + k]}
            o = emit_prog(em, MC, inmap, comp)
            em.fence()
            for row in range(4):
                for k in range(8):
                    new[8 * (4 * c + row) + k] = o[names[8 * row + k]]
        st = new
    return st


def run_words(em, final, words):
    """run the emitted op list on 128 bitsliced words; returns the 128 output words"""
    M = 0xFFFFFFFF
    env = {f"s[{i}]": w for i, w in enumerate(words)}
    for d, a, b, c, imm in em.ops:
        A, B, C = env[a], env[b], env[c]
        r = 0
        for m in range(8):
            if (imm >> m) & 1:
                r |= (A if m & 4 else ~A & M) & (B if m & 2 else ~B & M) & (C if m & 1 else ~C & M)
        env[d] = r
    return [env[f] for f in final]


def simulate(em, final, blocks):
    """run the emitted op list on 32 bitsliced blocks (python ints as u32)"""
    M = 0xFFFFFFFF
    env = {}
    for i in range(128):
        w = 0
        for j, blk in enumerate(blocks):
            w |= ((blk[i >> 3] >> (i & 7)) & 1) << j
        env[f"s[{i}]"] = w
    for d, a, b, c, imm in em.ops:
        A, B, C = env[a], env[b], env[c]
        r = 0
        for m in range(8):
            if (imm >> m) & 1:
                r |= (A if m & 4 else ~A & M) & (B if m & 2 else ~B & M) & (C if m & 1 else ~C & M)
        env[d] = r
    outs = []
    for j in range(len(blocks)):
        out = [0] * 16
        for i in range(128):
            out[i >> 3] |= ((env[final[i]] >> j) & 1) << (i & 7)
        outs.append(out)
    return outs


def main():
    check_only = "--check-only" in sys.argv
    sb = sbox_net()
    bad = [x for x in range(256)
           if sum(run_prog([(n, [a, b], truth(sb, n, [a, b])) for n, (op, a, b) in sb.gates.items()],
                           {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)})[f"s{i}"] << (7 - i) for i in range(8))
           != SBOX[x]]
    assert not bad, f"S-box circuit wrong on {len(bad)} inputs"
    SB = Program(sb, trials=300, sched_trials=400)
    for x in range(256):
        e = run_prog(SB.prog, {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)})
        assert sum(e[f"s{i}"] << (7 - i) for i in range(8)) == SBOX[x]
    MC = Program(mixcol_net(), trials=50, sched_trials=400)
    em = Emitter()
    final = gen_aes(em, SB, MC)
    rnd = random.Random(1)
    blocks = [[0] * 16] + [[rnd.randrange(256) for _ in range(16)] for _ in range(31)]
    got = simulate(em, final, blocks)
    for blk, g in zip(blocks, got):
        assert g == aes_ref(blk), "bitsliced program disagrees with AES reference"
    assert bytes(got[0]).hex() == "66e94bd4ef8a2c3b884cfa59ca342b2e"
    # rolled form: 9 x (keyless round, then AddRoundKey at run time) + keyed last round
    em_r, em_l = Emitter(), Emitter()
    fin_r = gen_aes(em_r, SB, MC, rounds=[1], keyed=False)
    fin_l = gen_aes(em_l, SB, MC, rounds=[10], keyed=True)
    words = [0] * 128
    for i in range(128):
        for j, blk in enumerate(blocks):
            words[i] |= ((blk[i >> 3] >> (i & 7)) & 1) << j
    for r in range(1, 10):
        words = run_words(em_r, fin_r, words)
        words = [w ^ (0xFFFFFFFF if (RK[r][i >> 3] >> (i & 7)) & 1 else 0) for i, w in enumerate(words)]
    words = run_words(em_l, fin_l, words)
    for j, blk in enumerate(blocks):
        out = [0] * 16
        for i in range(128):
            out[i >> 3] |= ((words[i] >> j) & 1) << (i & 7)
        assert out == aes_ref(blk), "rolled bitsliced program disagrees with AES reference"
    nops = len(em.ops)
    print(f"S-box {len(SB)} LUTs (peak live {SB.peak}), MixColumns {len(MC)} LUTs/column (peak live {MC.peak}), total {nops} v_bitop3 per 32 blocks "
          f"= {nops / 32:.1f} per block", file=sys.stderr)
    if check_only:
        return
    body = "\n".join(em.lines)
    outs = ", ".join(final)
    body_r, outs_r = "\n".join(em_r.lines), ", ".join(fin_r)
    body_l, outs_l = "\n".join(em_l.lines), ", ".join(fin_l)
    hdr = f"""// GENERATED by tools/gen_aes_bs.py — do not edit.
// Bitsliced AES-128 with the all-zero key (src/prg.rs:185-234 FixedKeyPrgStream's cipher):
// s[i] holds bit i of 32 blocks (bit i = bit (i & 7) of byte (i >> 3)); on return s holds
// AES_0 of each block (no feed-forward). {nops} v_bitop3_b32 per call = {nops / 32:.1f} per block
// (S-box: Boyar-Peralta circuit mapped to {len(SB)} 3-LUTs; MixColumns {len(MC)} per column;
// AddRoundKey folded into the truth tables). Ops::fence<unit>() follows every S-box / MixColumns
// column (unit 0..{em.units - 1}) so a device Ops can bound the scheduler's reordering.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhh {{

constexpr int kAesBsOps = {nops};

template <class Ops>
__host__ __device__ __forceinline__ void aes0_bs(uint32_t (&s)[128]) {{
{body}
    const uint32_t out_[128] = {{{outs}}};
#pragma unroll
    for (int i = 0; i < 128; i++) s[i] = out_[i];
}}

// Rolled form (code ~1/8 the size): rounds 1..9 = aes0_bs_round + AddRoundKey applied by the
// caller at run time; then aes0_bs_last (round 10, its key folded). {len(em_r.ops)} + {len(em_l.ops)} ops.
template <class Ops>
__host__ __device__ __forceinline__ void aes0_bs_round(uint32_t (&s)[128]) {{
{body_r}
    const uint32_t out_[128] = {{{outs_r}}};
#pragma unroll
    for (int i = 0; i < 128; i++) s[i] = out_[i];
}}

template <class Ops>
__host__ __device__ __forceinline__ void aes0_bs_last(uint32_t (&s)[128]) {{
{body_l}
    const uint32_t out_[128] = {{{outs_l}}};
#pragma unroll
    for (int i = 0; i < 128; i++) s[i] = out_[i];
}}

}}  // namespace fhh
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
