"""Deterministic synthetic workloads shaped like the reference leader's (src/bin/leader.rs).

The reference draws everything from `thread_rng` (irreproducible); here a seeded numpy
Generator stands in, with the same shapes:
  * sites: `num_sites` strings of (data_len - aug_len) bits per dim, each an alphanumeric
    ASCII string turned into bits LSB-first per byte (`string_to_bits`, lib.rs:90-98;
    `generate_random_bit_vectors`, leader.rs:45-58; `generate_strings`, leader.rs:60-66);
  * clients: a Zipf(s) draw over sites (leader.rs:140-147; inverse-CDF here instead of the
    `zipf` crate's rejection sampler) plus an `aug_len`-bit alphanumeric augmentation per
    dim (`augment_string`, leader.rs:78-87);
  * key bounds: l = a - ball, r = a + ball on MSB-first bit strings of width
    max(len, 32) (`gen_l_inf_ball`, ibDCF.rs:175-188; lib.rs:131-183).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

ALNUM = np.frombuffer(b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", np.uint8)


def chars_to_bits(chars: np.ndarray) -> np.ndarray:
    """uint8 ASCII [..., m] -> bits [..., 8m], LSB first per byte (lib.rs:90-98)."""
    b = (chars[..., None] >> np.arange(8, dtype=np.uint8)) & 1
    return b.reshape(*chars.shape[:-1], chars.shape[-1] * 8).astype(np.uint8)


def random_alnum(rng: np.random.Generator, shape) -> np.ndarray:
    return ALNUM[rng.integers(0, ALNUM.size, size=shape)]


def zipf_indices(rng: np.random.Generator, n: int, num_sites: int, s: float) -> np.ndarray:
    """P(k) ∝ k^-s for k = 1..num_sites; returns k-1."""
    w = np.arange(1, num_sites + 1, dtype=np.float64) ** (-s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    u = rng.random(n)
    return np.minimum(np.searchsorted(cdf, u, side="right"), num_sites - 1)


def _add_small(bits: np.ndarray, delta: int, sign: int) -> np.ndarray:
    """MSB-first bit strings [..., W] +/- delta (< 2^32) with wrap (subtract) or carry check."""
    W = bits.shape[-1]
    nwords = (W + 63) // 64
    pad = nwords * 64 - W
    b = np.concatenate([np.zeros(bits.shape[:-1] + (pad,), np.uint8), bits], axis=-1)
    # pack big-endian into u64 words (word 0 most significant)
    words = np.packbits(b, axis=-1, bitorder="big").view(">u8").astype(np.uint64)
    carry = np.full(bits.shape[:-1], np.uint64(delta), np.uint64)
    for wi in range(nwords - 1, -1, -1):
        x = words[..., wi]
        if sign > 0:
            nx = x + carry
            carry = (nx < x).astype(np.uint64)
        else:
            nx = x - carry
            carry = (nx > x).astype(np.uint64)
        words[..., wi] = nx
    if sign > 0 and np.any(carry) or (sign > 0 and pad and np.any(words[..., 0] >> np.uint64(64 - pad))):
        raise ValueError("carry out of add_bitstrings: the reference panics on this input (ibDCF.rs:182)")
    out = np.unpackbits(np.ascontiguousarray(words.astype(">u8")).view(np.uint8), axis=-1, bitorder="big")
    return np.ascontiguousarray(out[..., pad:])


def l_inf_ball_bounds(alpha: np.ndarray, ball: int):
    """alpha [n][d][L] MSB-first bits -> (left, right) [n][d][max(L,32)] (ibDCF.rs:175-188)."""
    L = alpha.shape[-1]
    if L < 32:
        alpha = np.concatenate([np.zeros(alpha.shape[:-1] + (32 - L,), np.uint8), alpha], axis=-1)
    return _add_small(alpha, ball, -1), _add_small(alpha, ball, +1)


def i16_to_bits(v: np.ndarray) -> np.ndarray:
    """sample_driving_data.rs:25-28: i16 -> 16 bits MSB first (two's complement)."""
    u = v.astype(np.int64) & 0xFFFF
    return ((u[..., None] >> np.arange(15, -1, -1)) & 1).astype(np.uint8)


@dataclass
class Workload:
    alpha: np.ndarray        # [n][d][L] client points (bits)
    left: np.ndarray         # [n][d][L] interval lower bounds
    right: np.ndarray        # [n][d][L] interval upper bounds
    root_seeds: np.ndarray   # [n][d][2 side][2 server][16]
    site_of_client: np.ndarray

    @property
    def n(self):
        return self.alpha.shape[0]


def zipf_workload(n: int, data_len: int = 512, n_dims: int = 1, num_sites: int = 10000, zipf_s: float = 1.03,
                  ball_size: int = 1, aug_len: int = 8, seed: int = 0x5EED, client_offset: int = 0,
                  sites_seed: int | None = None) -> Workload:
    """Config 'zipf' of the reference leader (leader.rs:331-365). `client_offset` draws the
    clients [client_offset, client_offset + n) of one global stream, so shards of a
    multi-GPU run are slices of the single-GPU population (the site table is shared)."""
    if data_len < 32:
        raise ValueError("zipf workload needs data_len >= 32 (gen_l_inf_ball pads to 32 bits, ibDCF.rs:178)")
    if aug_len % 8 or (data_len - aug_len) % 8:
        raise ValueError("data_len and aug_len must be multiples of 8 (leader.rs:306)")
    srng = np.random.default_rng(sites_seed if sites_seed is not None else seed)
    site_bits = chars_to_bits(random_alnum(srng, (num_sites, n_dims, (data_len - aug_len) // 8)))
    # per-client draws: generate the global stream up to client_offset + n and slice, so
    # any client range is reproducible
    sites = zipf_indices(np.random.default_rng([seed, 1]), client_offset + n, num_sites, zipf_s)[client_offset:]
    arng = np.random.default_rng([seed, 2])
    aug = random_alnum(arng, (client_offset + n, n_dims, aug_len // 8))[client_offset:]
    alpha = np.concatenate([site_bits[sites], chars_to_bits(aug)], axis=-1)
    left, right = l_inf_ball_bounds(alpha, ball_size)
    rrng = np.random.default_rng([seed, 3])
    roots = rrng.integers(0, 256, size=(client_offset + n, n_dims, 2, 2, 16), dtype=np.uint8)[client_offset:]
    return Workload(alpha, left, right, np.ascontiguousarray(roots), sites)


def synthetic_centroids(num: int = 3233, seed: int = 0xC0DE) -> np.ndarray:
    """County-centroid-shaped points (lat, lon) in degrees: mostly the contiguous US, a few in
    Alaska, Hawaii and the territories — the shape of data/county_centroids.csv (3 233 rows,
    lat -14.5..69.3, lon -171..145.8), synthesised here (the reference's file is not used)."""
    rng = np.random.default_rng(seed)
    n_ak, n_hi, n_terr = (num * 30) // 3233, (num * 5) // 3233, (num * 78) // 3233
    n_us = num - n_ak - n_hi - n_terr
    us = np.stack([rng.uniform(25.0, 49.0, n_us), rng.uniform(-124.5, -67.0, n_us)], 1)
    ak = np.stack([rng.uniform(55.0, 69.3, n_ak), rng.uniform(-171.0, -130.0, n_ak)], 1)
    hi = np.stack([rng.uniform(19.0, 22.2, n_hi), rng.uniform(-160.0, -155.0, n_hi)], 1)
    terr = np.stack([rng.uniform(-14.5, 18.5, n_terr),
                     np.where(rng.random(n_terr) < 0.8, rng.uniform(-67.3, -64.5, n_terr),
                              rng.uniform(144.6, 145.8, n_terr))], 1)
    return np.concatenate([us, ak, hi, terr])


def geo_to_int(lat: np.ndarray, lon: np.ndarray):
    """sample_driving_data.rs:11-15: centidegrees, rounded, as i16."""
    return np.round(lat * 100.0).astype(np.int16), np.round(lon * 100.0).astype(np.int16)


def reference_centroids() -> np.ndarray:
    """The reference's county centroids (data/county_centroids.csv, 3 233 rows, file order) as
    [num][lat, lon] degrees, from the committed data fixture tests/golden/county_centroids.npz
    (made by tests/golden/make_county_centroids.py; load_centroids, sample_covid_data.rs:17-30)."""
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "county_centroids.npz")
    z = np.load(path, allow_pickle=False)
    return np.stack([z["lat"], z["lon"]], 1)


def coords_workload(n: int, ball_size: int = 1, num_centroids: int = 3233, zipf_s: float = 1.03,
                    side_km: float = 8.0, seed: int = 0x5EED, client_offset: int = 0,
                    centroids: str = "reference") -> Workload:
    """Config D: d = 2 (lat, lon), data_len = 16. Points = the reference's county
    centroids (`centroids="reference"`, data/county_centroids.csv; "synthetic" = the r01/r02
    stand-in of the same shape) drawn Zipf-weighted over counties, jittered uniformly in a square
    of side aug_len = 8 km (`uniform_in_square`, sample_covid_data.rs:45-62, called with
    Some(aug_len) by leader.rs:67-75, aug_len = 8 at leader.rs:331), converted to i16 centidegrees
    (sample_driving_data.rs:11-15); keys per `gen_l_inf_ball_from_coords` (ibDCF.rs:189-205):
    bounds (c -/+ ball) clamped to +-9000 (lat) / +-18000 (lon), i16 -> 16 bits MSB first (two's
    complement, sample_driving_data.rs:25-28). The reference weighs counties by COVID case records
    (a CSV it does not ship); the Zipf weight over the file order stands in for it."""
    if centroids == "reference":   # num_centroids < 3233: the file's first rows (small tests)
        cents = reference_centroids()[:num_centroids]
        num_centroids = cents.shape[0]
    else:
        cents = synthetic_centroids(num_centroids)
    idx = zipf_indices(np.random.default_rng([seed, 11]), client_offset + n, num_centroids, zipf_s)[client_offset:]
    jr = np.random.default_rng([seed, 12])
    u = jr.random((client_offset + n, 2))[client_offset:]
    lat0, lon0 = cents[idx, 0], cents[idx, 1]
    a_lat = (side_km / 2.0) / 111.32
    a_lon = (side_km / 2.0) / (111.32 * np.cos(np.radians(lat0)))
    lat = np.clip(lat0 + (2 * u[:, 0] - 1) * a_lat, -90.0, 90.0)
    lon = np.clip(lon0 + (2 * u[:, 1] - 1) * a_lon, -180.0, 180.0)
    la, lo = geo_to_int(lat, lon)
    la32, lo32 = la.astype(np.int32), lo.astype(np.int32)
    b = int(ball_size)
    left = np.stack([i16_to_bits(np.clip(la32 - b, -9000, 9000)), i16_to_bits(np.clip(lo32 - b, -18000, 18000))], 1)
    right = np.stack([i16_to_bits(np.clip(la32 + b, -9000, 9000)), i16_to_bits(np.clip(lo32 + b, -18000, 18000))], 1)
    alpha = np.stack([i16_to_bits(la32), i16_to_bits(lo32)], 1)
    rrng = np.random.default_rng([seed, 13])
    roots = rrng.integers(0, 256, size=(client_offset + n, 2, 2, 2, 16), dtype=np.uint8)[client_offset:]
    return Workload(alpha, np.ascontiguousarray(left), np.ascontiguousarray(right), np.ascontiguousarray(roots),
                    idx)


def plaintext_heavy_hitters(alpha_left: np.ndarray, alpha_right: np.ndarray, threshold_count: int):
    """Brute-force recount (no crypto): heavy prefixes of the full depth whose box is
    contained in at least `threshold_count` clients' [l, r] boxes, crawled level by level
    exactly as the leader prunes (keep iff count >= threshold at every level). Returns
    the sorted list of final paths as tuples of d bit-tuples. For tests only at small n."""
    n, d, L = alpha_left.shape
    frontier = [tuple(() for _ in range(d))]
    for lvl in range(L):
        children = []
        for p in frontier:
            for i in range(1 << d):
                children.append(tuple(p[j] + ((i >> j) & 1,) for j in range(d)))
        kept = []
        for ch in children:
            k = lvl + 1
            cnt = 0
            for c in range(n):
                ok = True
                for j in range(d):
                    pre = ch[j]
                    lo = tuple(int(x) for x in alpha_left[c, j, :k])
                    hi = tuple(int(x) for x in alpha_right[c, j, :k])
                    if not (lo <= pre <= hi):
                        ok = False
                        break
                cnt += ok
            if cnt >= threshold_count:
                kept.append(ch)
        frontier = kept
    return sorted(frontier)


def plaintext_crawl(left: np.ndarray, right: np.ndarray, thr: int, thr_last: int, levels: int | None = None):
    """Full-size plaintext crawl (no crypto, no oracle): what the two-server protocol computes,
    level by level in the leader's child order (parents in frontier order x all_bit_vectors,
    collect.rs:379-391, lib.rs:125-129), keep iff count >= threshold (collect.rs:945-989).
    A client is inside a node iff in every dim l[:k] <= prefix <= r[:k]; the per-(node, dim)
    "still equal to l / to r" flags are bit-packed over clients, so a level is a handful of
    word ops per (child, 64 clients). Returns (per-level child counts, final paths, final
    counts); paths as tuples of d bit-tuples."""
    n, d, L = left.shape
    levels = levels or L
    nw = (n + 63) // 64

    def pack(a):   # [n] 0/1 -> [nw] u64 over clients
        b = np.zeros(nw * 64, np.uint8)
        b[:n] = a
        return np.packbits(b.reshape(nw, 64), axis=1, bitorder="little").view(np.uint64).reshape(nw)

    ones = np.full(nw, np.uint64(0xFFFFFFFFFFFFFFFF))
    valid = pack(np.ones(n, np.uint8))
    # frontier state: alive [F][nw], lo/hi tight [F][d][nw]
    alive = valid[None, :].copy()
    lo_t = np.broadcast_to(ones, (1, d, nw)).copy()
    hi_t = lo_t.copy()
    paths = [tuple(() for _ in range(d))]
    counts_per_level = []
    for k in range(levels):
        lb = np.stack([pack(left[:, j, k]) for j in range(d)])    # [d][nw]
        rb = np.stack([pack(right[:, j, k]) for j in range(d)])
        F = alive.shape[0]
        C = F << d
        c_alive = np.repeat(alive, 1 << d, axis=0)                  # child c = f * 2^d + i
        c_lo = np.repeat(lo_t, 1 << d, axis=0)
        c_hi = np.repeat(hi_t, 1 << d, axis=0)
        i_idx = np.tile(np.arange(1 << d), F)
        for j in range(d):
            b = ((i_idx >> j) & 1).astype(bool)[:, None]
            lo, hi = c_lo[:, j], c_hi[:, j]
            ok = np.where(b, ~hi | rb[j][None, :], ~lo | ~lb[j][None, :])
            c_alive &= ok
            c_lo[:, j] = np.where(b, lo & lb[j][None, :], lo & ~lb[j][None, :])
            c_hi[:, j] = np.where(b, hi & rb[j][None, :], hi & ~rb[j][None, :])
        cnt = np.bitwise_count(c_alive).sum(axis=1).astype(np.uint64) if C else np.zeros(0, np.uint64)
        counts_per_level.append(cnt)
        keep = np.nonzero(cnt >= (thr_last if k == levels - 1 else thr))[0]
        new_paths = []
        for c in keep:
            f, i = divmod(int(c), 1 << d)
            new_paths.append(tuple(paths[f][j] + ((i >> j) & 1,) for j in range(d)))
        paths = new_paths
        alive, lo_t, hi_t = c_alive[keep], c_lo[keep], c_hi[keep]
        final_counts = cnt[keep]
    return counts_per_level, paths, [int(v) for v in final_counts]


def add_keys_request_bincode(key_idx: np.ndarray, root_seed: np.ndarray, cw_seed: np.ndarray,
                             cw_bits: np.ndarray) -> np.ndarray:
    """Serialize keys (add_keys layout: [n][d][2], [n][d][2][16], [n][d][2][L][16],
    [n][d][2][L] nibbles) as `AddKeysRequest.keys` (rpc.rs:12-15) in bincode 1.x legacy
    encoding: u64 n; per client u64 d, then d (left, right) ibDCFKeys = key_idx bool,
    root_seed[16], u64 L, L x (seed[16], bits.0, bits.1, y_bits.0, y_bits.1)."""
    n, d, _, L = cw_bits.shape
    KB = 25 + 20 * L
    rec = np.zeros((n, 8 + 2 * d * KB), np.uint8)
    rec[:, 0:8] = np.frombuffer(np.uint64(d).tobytes(), np.uint8)
    keys = rec[:, 8:].reshape(n, 2 * d, KB)
    keys[:, :, 0] = key_idx.reshape(n, 2 * d)
    keys[:, :, 1:17] = root_seed.reshape(n, 2 * d, 16)
    keys[:, :, 17:25] = np.frombuffer(np.uint64(L).tobytes(), np.uint8)
    cw = keys[:, :, 25:].reshape(n, 2 * d, L, 20)
    cw[:, :, :, 0:16] = cw_seed.reshape(n, 2 * d, L, 16)
    nib = cw_bits.reshape(n, 2 * d, L)
    for b in range(4):
        cw[:, :, :, 16 + b] = (nib >> b) & 1
    return np.concatenate([np.frombuffer(np.uint64(n).tobytes(), np.uint8), rec.reshape(-1)])
