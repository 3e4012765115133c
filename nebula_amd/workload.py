"""Deterministic synthetic batches for the BASELINE.json configs.

Everything derives from one 64-bit seed through SplitMix64, so the bench, the tests and the CPU
baseline see identical (key, nonce, AAD, plaintext) tuples:
  keys          32 B each
  remote index  one uint32 per key
  key per pkt   uniform over the keys (1 key: all 0)
  counters      per key, starting at 3 (first data counter after the IX handshake,
                connection_state_test.go:135-144), incrementing in emission order
  AAD           header.Encode(1, Message, 0, remoteIndex, counter) (header/header.go:102-110)
  plaintext     uniform random bytes
  IMIX          sizes {90, 576, 1300} in a 7:4:1 count ratio, deterministically shuffled

Arena layout (the TX SendBatch slot shape, inside.go:226-227): slot = [hdr 16 | payload | tag 16],
slot stride = 16 + maxlen + 16 rounded up to 64 B, payload 16-B aligned. Seal and open are both in
place: seal turns PT into CT and writes the tag; open turns CT back into PT.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .header import encode_many

SEED = 0x6E6562756C61  # "nebula"
GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, n: int) -> np.ndarray:
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & (2**64 - 1)) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def random_bytes(seed: int, n: int) -> np.ndarray:
    return splitmix64(seed, (n + 7) // 8).view(np.uint8)[:n].copy()


@dataclass
class Batch:
    alg: int
    keys: np.ndarray        # (nkeys*32,) uint8
    remote_index: np.ndarray
    desc: np.ndarray        # DESC_DTYPE
    arena: np.ndarray       # uint8, plaintext slots (hdr | PT | tag space)
    stride: int
    name: str

    @property
    def n(self) -> int:
        return len(self.desc)

    @property
    def nkeys(self) -> int:
        return len(self.keys) // 32

    @property
    def payload_bytes(self) -> int:
        return int(self.desc["len"].astype(np.int64).sum())

    @property
    def algorithmic_bytes(self) -> int:
        """Per seal or per open: read AAD + payload, write payload + tag (2p + 32)."""
        return int((2 * self.desc["len"].astype(np.int64) + 2 * 16).sum())


def key_ids(npkt: int, nkeys: int, seed: int = SEED) -> np.ndarray:
    """Each packet's tunnel key: uniform over nkeys (a Poisson(npkt / nkeys) count per key)."""
    if nkeys == 1:
        return np.zeros(npkt, np.uint32)
    return (splitmix64(seed ^ 0x4B494453, npkt) % np.uint64(nkeys)).astype(np.uint32)


def payload_lens(npkt: int, sizes=(1300,), ratio=(1,), seed: int = SEED) -> np.ndarray:
    """Payload sizes: one size, or a mix in the given ratio (IMIX 90/576/1300 at 7:4:1), shuffled."""
    if len(sizes) == 1:
        return np.full(npkt, sizes[0], np.uint32)
    pool = np.repeat(np.asarray(sizes, np.uint32), ratio)
    reps = -(-npkt // len(pool))
    lens = np.tile(pool, reps)[:npkt]
    order = np.argsort(splitmix64(seed ^ 0x494D4958, npkt), kind="stable")
    return lens[order]


def make_batch(alg: int, npkt: int, nkeys: int, sizes=(1300,), ratio=(1,), seed: int = SEED,
               name: str = "") -> Batch:
    keys = random_bytes(seed ^ 0x4B455953, 32 * nkeys)                      # "KEYS"
    remote_index = (splitmix64(seed ^ 0x52494458, nkeys) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    kid = key_ids(npkt, nkeys, seed)
    lens = payload_lens(npkt, sizes, ratio, seed)
    # per-key counters in emission order
    order = np.argsort(kid, kind="stable")
    sk = kid[order]
    start = np.r_[0, np.flatnonzero(np.diff(sk)) + 1]
    run_id = np.repeat(np.arange(len(start)), np.diff(np.r_[start, len(sk)]))
    rank = np.arange(len(sk)) - start[run_id]
    ctr = np.empty(npkt, np.uint64)
    ctr[order] = rank.astype(np.uint64) + np.uint64(3)

    maxlen = int(lens.max())
    stride = -(-(16 + maxlen + 16) // 64) * 64
    arena = np.zeros(npkt * stride, np.uint8)
    slots = arena.reshape(npkt, stride)
    slots[:, :16] = encode_many(remote_index[kid], ctr)
    pt = random_bytes(seed ^ 0x50544558, int(lens.astype(np.int64).sum()))
    if len(sizes) == 1:
        slots[:, 16:16 + maxlen] = pt.reshape(npkt, maxlen)
    else:
        off = np.r_[0, np.cumsum(lens.astype(np.int64))[:-1]]
        for s in sizes:
            idx = np.flatnonzero(lens == s)
            src = off[idx][:, None] + np.arange(s)[None, :]
            slots[idx, 16:16 + s] = pt[src]
    desc = np.zeros(npkt, L.DESC_DTYPE)
    base = np.arange(npkt, dtype=np.uint64) * np.uint64(stride)
    desc["aad_off"] = base
    desc["src_off"] = base + np.uint64(16)
    desc["dst_off"] = base + np.uint64(16)
    desc["counter"] = ctr
    desc["len"] = lens
    desc["aad_len"] = 16
    desc["key_id"] = kid
    return Batch(alg, keys, remote_index, desc, arena, stride, name)


def relay_batch(alg: int, npkt: int, nkeys: int, aad_len: int = 1348, seed: int = SEED, name: str = "relay") -> Batch:
    """GMAC-only relay packets (ConnectionState.VerifyRelay, connection_state.go:121-148; the relay
    seal at inside.go:491): the AD is the whole relayed packet but its last 16 bytes, the
    ciphertext is empty and the tag follows the AD. 1348 B = outer header 16 + a 1332-B wire packet
    (16 + 1300 + 16). Per-key counters in emission order as in make_batch."""
    b = make_batch(alg, npkt, nkeys, sizes=(aad_len - 16,), seed=seed, name=name)
    stride = -(-(aad_len + 16) // 64) * 64
    arena = np.zeros(npkt * stride, np.uint8)
    slots = arena.reshape(npkt, stride)
    old = b.arena.reshape(npkt, b.stride)
    slots[:, :aad_len] = old[:, :aad_len]  # header.Encode + the inner packet's bytes
    desc = b.desc.copy()
    base = np.arange(npkt, dtype=np.uint64) * np.uint64(stride)
    desc["aad_off"] = base
    desc["src_off"] = base + np.uint64(aad_len)  # the tag, right after the AD
    desc["dst_off"] = base + np.uint64(aad_len)
    desc["len"] = 0
    desc["aad_len"] = aad_len
    return Batch(alg, b.keys, b.remote_index, desc, arena, stride, name)


# BASELINE.json configs
def config(idx: int, scale: float = 1.0) -> Batch:
    """configs[idx] of BASELINE.json. `scale` shrinks the packet count for quick tests."""
    def npk(n):
        return max(4, int(n * scale))
    if idx == 0:
        return make_batch(L.ALG_AESGCM, npk(1024), 1, name="C1 AES-256-GCM 1 key 1024x1300B")
    if idx == 1:
        return make_batch(L.ALG_AESGCM, npk(65536), 1, name="C2 AES-256-GCM 1 key 65536x1300B")
    if idx == 2:
        return make_batch(L.ALG_AESGCM, npk(65536), 4096, name="C3 AES-256-GCM 4096 keys 65536x1300B")
    if idx == 3:
        return make_batch(L.ALG_CHACHAPOLY, npk(65536), 4096, name="C4 ChaCha20-Poly1305 4096 keys 65536x1300B")
    if idx == 4:
        return make_batch(L.ALG_AESGCM, npk(1 << 20), 4096, sizes=(90, 576, 1300), ratio=(7, 4, 1),
                          name="C5 AES-256-GCM 4096 keys IMIX 1M")
    raise ValueError(idx)


def shard(b: Batch, rank: int, world: int) -> Batch:
    """Contiguous packet range for one GPU; offsets rebased to the shard's arena."""
    n = b.n
    lo, hi = n * rank // world, n * (rank + 1) // world
    d = b.desc[lo:hi].copy()
    base = np.uint64(lo * b.stride)
    for f in ("src_off", "dst_off", "aad_off"):
        d[f] -= base
    arena = b.arena[lo * b.stride:hi * b.stride].copy()
    return Batch(b.alg, b.keys, b.remote_index, d, arena, b.stride, f"{b.name} shard {rank}/{world}")


def shard_by_key(b: Batch, rank: int, world: int) -> Batch:
    """The packets of the tunnels with key_id mod world == rank (SURVEY.md §8e's partition by key):
    every tunnel's packets on one GPU, in their batch order. A tunnel's state — its replay window and
    message counter (connection_state.go:37-49) — then lives on one device, which a receive batch
    needs (its windows see every packet of their tunnel), and each GPU's batch keeps the whole batch's
    packets per tunnel. Offsets rebased to the shard's own arena (the selected slots, in order)."""
    idx = np.flatnonzero(b.desc["key_id"] % np.uint32(world) == rank)
    d = b.desc[idx].copy()
    slots = b.arena.reshape(b.n, b.stride)[idx]
    base = np.arange(len(idx), dtype=np.uint64) * np.uint64(b.stride)
    old = idx.astype(np.uint64) * np.uint64(b.stride)
    for f in ("src_off", "dst_off", "aad_off"):
        d[f] = d[f] - old + base
    return Batch(b.alg, b.keys, b.remote_index, d, slots.reshape(-1).copy(), b.stride,
                 f"{b.name} tunnels mod {world} = {rank}")

