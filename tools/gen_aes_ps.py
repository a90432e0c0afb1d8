#!/usr/bin/env python3
"""Generate fuzzyheavyhitters_amd/csrc/aes_ps_gen.h: the zero-key AES-128 (src/prg.rs:185-234)
"pair-sliced" over two lanes, for the VALU waves of the hybrid k_expand.

A lane pair (lane 2k = "A", lane 2k+1 = "B") holds 32 blocks bitsliced: lane A the 64 bits of
state columns 0 and 1, lane B those of columns 2 and 3, so a lane needs 64 state registers
instead of the 128 of the one-lane bitsliced form (tools/gen_aes_bs.py) and the kernel stays at
<= 128 VGPRs (4 waves per SIMD beside the T-table waves). Local word i (0..63) = bit (i & 7) of
local byte i >> 3; local byte lb = 4 l + row is global byte lb (A) or lb + 8 (B).

Per round both lanes run the same instruction stream:
  SubBytes    8 local S-boxes (the Boyar-Peralta circuit mapped to 3-LUTs, as gen_aes_bs.py);
  ShiftRows   row 0 stays; row 1: l0 <- own l1, l1 <- partner's l0; row 2: l0, l1 <- partner's
              l0, l1; row 3: l0 <- partner's l1, l1 <- own l0 — the same moves in both lanes, so
              one DPP quad_perm [1,0,3,2] move per word that crosses (32 per round);
  MixColumns  the two local columns (76 LUTs each);
  AddRoundKey the zero key's round-key bits: equal in both lanes -> folded into the producing
              LUT's truth table; different -> XOR with the lane-parity mask `isb` (0 in A,
              ~0 in B), folded into the producing LUT when it has a free input, else one op.
The emitted op list is simulated here on two lanes (swap = exchange) against a byte AES.

Usage: python tools/gen_aes_ps.py [--check-only]
"""
from __future__ import annotations

import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_aes_bs as G   # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "fuzzyheavyhitters_amd", "csrc", "aes_ps_gen.h")
M32 = 0xFFFFFFFF


class PsEmitter:
    def __init__(self):
        self.lines, self.ops = [], []   # ops: ("b3", d, a, b, c, imm) | ("swap", d, a)
        self.n = 0
        self.count = {"b3": 0, "swap": 0, "lanexor": 0}

    def new(self):
        self.n += 1
        return f"v{self.n}"

    def b3(self, a, b, c, imm, kind="b3"):
        d = self.new()
        self.ops.append(("b3", d, a, b, c, imm))
        self.lines.append(f"    const uint32_t {d} = Ops::template b3<0x{imm:02X}>({a}, {b}, {c});")
        self.count[kind] += 1
        return d

    def fence(self):
        self.lines.append("    Ops::fence();")

    def swap(self, a):
        d = self.new()
        self.ops.append(("swap", d, a))
        self.lines.append(f"    const uint32_t {d} = Ops::swap({a});")
        self.count["swap"] += 1
        return d


def emit_prog_ps(em, P, inmap, keys):
    """LUT program P; keys[o] = (kA, kB) round-key bits applied to output o (None: none).
    Returns {output: operand}."""
    env = dict(inmap)
    used_as_leaf = {l for _, leaves, _ in P.prog for l in leaves}
    out = {}
    for n, leaves, tt in P.prog:
        k = keys.get(n)
        if k is not None and n not in used_as_leaf:
            ka, kb = k
            if ka == kb:
                a, b, c, imm = G.imm_for([env[l] for l in leaves], tt ^ (0xFF if ka else 0))
                env[n] = out[n] = em.b3(a, b, c, imm)
                continue
            if len(leaves) <= 2:
                # add isb as the new leaf 2 (S0): f' = f(leaves) ^ isb ^ ka
                tt3 = 0
                for m in range(8):
                    l0, l1, lb = m & 1, (m >> 1) & 1, (m >> 2) & 1
                    mm = l0 | (l1 << 1) if len(leaves) == 2 else l0
                    tt3 |= (((tt >> mm) & 1) ^ lb ^ ka) << m
                ops = [env[leaves[0]], env[leaves[1]] if len(leaves) == 2 else env[leaves[0]], "isb"]
                env[n] = out[n] = em.b3(ops[2], ops[1], ops[0], tt3)
                continue
        a, b, c, imm = G.imm_for([env[l] for l in leaves], tt)
        env[n] = em.b3(a, b, c, imm)
    for o in P.outputs:
        if o in out:
            continue
        k = keys.get(o)
        if k is None or k == (0, 0):
            out[o] = env[o]
        elif k == (1, 1):
            out[o] = em.b3(env[o], env[o], env[o], 0x0F)
        else:
            out[o] = lane_xor(em, env[o], k[0])
    return out


def lane_xor(em, w, ka):
    """w ^ isb ^ ka (a word whose key bit differs between the lanes)"""
    # S0 = isb, S1 = S2 = w: index = 4 isb + 3 w -> value w ^ isb ^ ka
    imm = 0
    for m in range(8):
        isb, wv = (m >> 2) & 1, m & 1
        imm |= (wv ^ isb ^ ka) << m
    return em.b3("isb", w, w, imm, kind="lanexor")


def rk_pair(r, lb, k):
    return ((G.RK[r][lb] >> k) & 1, (G.RK[r][lb + 8] >> k) & 1)


def gen_aes_ps(em, SB, MC):
    st = [f"s[{i}]" for i in range(64)]
    for r in range(1, 11):
        # SubBytes (round-10 keys folded at the S-box outputs, keyed by the DESTINATION byte)
        sub = [None] * 64
        for lb in range(8):
            l, row = lb // 4, lb % 4
            inmap = {f"x{i}": st[8 * lb + (7 - i)] for i in range(8)}
            keys = {}
            if r == 10:
                dl = {0: l, 1: 1 - l, 2: l, 3: 1 - l}[row]   # local column the byte lands in
                dlb = 4 * dl + row
                cross = row == 2 or (row == 1 and l == 0) or (row == 3 and l == 1)
                # a word that crosses is computed in the other lane: its key pair swaps
                keys = {f"s{i}": rk_pair(10, dlb, 7 - i)[::-1 if cross else 1] for i in range(8)}
            o = emit_prog_ps(em, SB, inmap, keys)
            em.fence()
            for i in range(8):
                sub[8 * lb + (7 - i)] = o[f"s{i}"]
        # ShiftRows
        sh = [None] * 64

        def mv(row, dst_l, src_l, cross):
            for k in range(8):
                w = sub[8 * (4 * src_l + row) + k]
                sh[8 * (4 * dst_l + row) + k] = em.swap(w) if cross else w

        mv(0, 0, 0, False)
        mv(0, 1, 1, False)
        mv(1, 0, 1, False)
        mv(1, 1, 0, True)
        mv(2, 0, 0, True)
        mv(2, 1, 1, True)
        mv(3, 0, 1, True)
        mv(3, 1, 0, False)
        if r == 10:
            return sh
        new = [None] * 64
        names = MC.outputs
        for l in range(2):
            inmap = {f"a{row}_{k}": sh[8 * (4 * l + row) + k] for row in range(4) for k in range(8)}
            keys = {names[8 * row + k]: rk_pair(r, 4 * l + row, k) for row in range(4) for k in range(8)}
            o = emit_prog_ps(em, MC, inmap, keys)
            em.fence()
            for row in range(4):
                for k in range(8):
                    new[8 * (4 * l + row) + k] = o[names[8 * row + k]]
        st = new
    raise AssertionError


def simulate_ps(em, final, blocks):
    """run the op list on two lanes holding 32 blocks; returns the 32 output blocks"""
    lanes = []
    for p in range(2):
        env = {"isb": M32 if p else 0}
        for i in range(64):
            w = 0
            for j, blk in enumerate(blocks):
                w |= ((blk[8 * p + (i >> 3)] >> (i & 7)) & 1) << j
            env[f"s[{i}]"] = w
        lanes.append(env)
    for op in em.ops:
        if op[0] == "swap":
            _, d, a = op
            va, vb = lanes[0][a], lanes[1][a]
            lanes[0][d], lanes[1][d] = vb, va
            continue
        _, d, a, b, c, imm = op
        for env in lanes:
            A, B, C = env[a], env[b], env[c]
            r = 0
            for m in range(8):
                if (imm >> m) & 1:
                    r |= (A if m & 4 else ~A & M32) & (B if m & 2 else ~B & M32) & (C if m & 1 else ~C & M32)
            env[d] = r
    outs = []
    for j in range(len(blocks)):
        out = [0] * 16
        for p in range(2):
            for i in range(64):
                out[8 * p + (i >> 3)] |= ((lanes[p][final[i]] >> j) & 1) << (i & 7)
        outs.append(out)
    return outs


def main():
    check_only = "--check-only" in sys.argv
    SB = G.Program(G.sbox_net(), trials=300, sched_trials=400)
    for x in range(256):
        e = G.run_prog(SB.prog, {f"x{i}": (x >> (7 - i)) & 1 for i in range(8)})
        assert sum(e[f"s{i}"] << (7 - i) for i in range(8)) == G.SBOX[x]
    MC = G.Program(G.mixcol_net(), trials=50, sched_trials=400)
    em = PsEmitter()
    final = gen_aes_ps(em, SB, MC)
    rnd = random.Random(2)
    blocks = [[0] * 16] + [[rnd.randrange(256) for _ in range(16)] for _ in range(31)]
    got = simulate_ps(em, final, blocks)
    for blk, g in zip(blocks, got):
        assert g == G.aes_ref(blk), "pair-sliced program disagrees with AES reference"
    assert bytes(got[0]).hex() == "66e94bd4ef8a2c3b884cfa59ca342b2e"
    nops = len(em.ops)
    per_block = 2 * nops / 32
    print(f"pair-sliced AES: {nops} ops per lane ({em.count}) = {per_block:.1f} lane-ops per block", file=sys.stderr)
    if check_only:
        return
    body = "\n".join(em.lines)
    outs = ", ".join(final)
    hdr = f"""// GENERATED by tools/gen_aes_ps.py — do not edit.
// Pair-sliced AES-128 with the all-zero key (src/prg.rs:185-234 FixedKeyPrgStream's cipher) for
// the VALU waves of the hybrid k_expand: lanes 2k ("A", isb = 0) and 2k + 1 ("B", isb = ~0)
// hold 32 blocks; s[i] = bit (i & 7) of local byte i >> 3 of all 32 blocks, local byte lb =
// global byte lb (A) or lb + 8 (B). On return s holds AES_0 of the blocks (no feed-forward).
// {nops} ops per lane = {per_block:.1f} lane-ops per block: {em.count['b3']} LUTs
// (S-box {len(SB)}, MixColumns {len(MC)} per column, round keys folded), {em.count['swap']} DPP
// swaps (ShiftRows across the pair), {em.count['lanexor']} lane-parity XORs (round-key bits that
// differ between the two lanes' bytes and could not be folded). Ops::fence() follows every S-box
// and MixColumns column (a scheduling barrier: the register peak stays that of this order).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhh {{

constexpr int kAesPsOps = {nops};

template <class Ops>
__device__ __forceinline__ void aes0_ps(uint32_t (&s)[64], const uint32_t isb) {{
{body}
    const uint32_t out_[64] = {{{outs}}};
#pragma unroll
    for (int i = 0; i < 64; i++) s[i] = out_[i];
}}

}}  // namespace fhh
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
