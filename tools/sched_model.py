"""CPU model of the mixed-key scheduler (nebula_amd/csrc/sched.hpp, sched.hip): the (size class,
key) binning, the chunk plan of sched_alloc_kernel and the workspace bounds, rule for rule, so the
tests can check the plan's invariants and its lane utilisation on the BASELINE configs' shapes
without a GPU. The order of bins and of packets inside a bin is arbitrary on the device (atomics);
the model fixes one order, and no invariant checked depends on it."""
from dataclasses import dataclass
from typing import List

import numpy as np

CHUNK_PKTS = 16      # kChunkPkts: packets per group at 4 lanes per packet
SIZE_CLASSES = 8     # kSizeClasses
LPP = 4              # lanes per packet the size classes are counted at (neb_sched_build's lpp)
WAVE = 64


def size_class(aad_len: np.ndarray, length: np.ndarray, lpp: int = LPP) -> np.ndarray:
    """sched.hip size_class: ceil(log2(rounds at lpp lanes)), capped at SIZE_CLASSES - 1."""
    n = (aad_len.astype(np.int64) + 15) // 16 + (length.astype(np.int64) + 15) // 16 + 1
    r = (n + lpp - 1) // lpp
    # 32 - clz(R - 1) for R > 1, i.e. the bit length of R - 1
    c = np.array([0 if x <= 1 else int(x - 1).bit_length() for x in r], np.int64)
    return np.minimum(c, SIZE_CLASSES - 1)


def tail_lg(count: int, cls: int) -> int:
    """sched_tail_lg: 16 lanes for <= 4 packets, 8 for <= 8, else 4; capped for short classes."""
    fit = 4 if count <= 4 else (3 if count <= 8 else 2)
    size = 2 if cls == 0 else (3 if cls == 1 else 4)
    return min(fit, size)


SPLIT_TAIL_CLASS = 99  # the product never splits a tail (sched.hip)
# the round-4 experiment: from size class 4 a 9-12 packet tail = 8 packets at 8 lanes + the rest at
# 16. More lane-rounds busy in this model (C3 0.867 -> 0.894), slower on the GPU (each extra chunk
# pays its key staging and tree final: C3 469-472 -> 456-459 GiB/s, profiles/r4/split_tails.log)
EXPERIMENT_SPLIT_CLASS = 4


def groups(cls: int) -> int:
    """sched_groups: groups of 16 packets per front chunk."""
    return 1 if cls >= 3 else 8 >> cls


def tail_long(cls: int, lg: int) -> bool:
    return cls >= lg + 2


def nbins(max_keys: int) -> int:
    return SIZE_CLASSES * (max_keys + 1)


def max_chunks(n: int, max_keys: int) -> int:
    nb = nbins(max_keys)
    return (n + CHUNK_PKTS - 1) // CHUNK_PKTS + min(n, nb)


def max_short(n: int, max_keys: int) -> int:
    return min(n, nbins(max_keys))


@dataclass
class Chunk:
    kind: str          # "front", "long" or "short"
    packets: np.ndarray  # packet indices (a range of `sorted`)
    key: int
    cls: int
    lg: int            # lanes per packet = 2**lg


def plan(key_id: np.ndarray, aad_len: np.ndarray, length: np.ndarray, max_keys: int,
         split_cls: int = SPLIT_TAIL_CLASS) -> List[Chunk]:
    """The chunks sched_alloc_kernel writes for one batch (every bin, its front chunks and tail)."""
    key = np.where(key_id < max_keys, key_id, max_keys).astype(np.int64)
    cls = size_class(aad_len, length)
    b = cls * (max_keys + 1) + key
    order = np.argsort(b, kind="stable")
    sb = b[order]
    starts = np.r_[0, np.flatnonzero(np.diff(sb)) + 1]
    ends = np.r_[starts[1:], len(sb)]
    out: List[Chunk] = []
    for s, e in zip(starts, ends):
        if s == e:
            continue
        bin_ = int(sb[s])
        k, c = bin_ % (max_keys + 1), bin_ // (max_keys + 1)
        cnt = int(e - s)
        nfull, tail = divmod(cnt, CHUNK_PKTS)
        lg = tail_lg(tail, c) if tail else 2
        split = lg == 2 and 9 <= tail <= 12 and c >= split_cls
        fpk = nfull * CHUNK_PKTS + (tail if tail and lg == 2 and not split else 0)
        cpk = groups(c) * CHUNK_PKTS
        for j in range(0, fpk, cpk):
            out.append(Chunk("front", order[s + j:s + min(fpk, j + cpk)], k, c, 2))
        if split:
            out.append(Chunk("long" if tail_long(c, 3) else "short", order[s + fpk:s + fpk + 8], k, c, 3))
            out.append(Chunk("long" if tail_long(c, 4) else "short", order[s + fpk + 8:e], k, c, 4))
        elif tail and lg != 2:
            out.append(Chunk("long" if tail_long(c, lg) else "short", order[s + fpk:e], k, c, lg))
    return out


def blocks(aad_len: np.ndarray, length: np.ndarray) -> np.ndarray:
    """GHASH blocks of each packet: AAD blocks + ciphertext blocks + the length block."""
    return (aad_len.astype(np.int64) + 15) // 16 + (length.astype(np.int64) + 15) // 16 + 1


def lane_rounds(ch: Chunk, nblk: np.ndarray) -> int:
    """Lane-rounds the chunk's wave spends: its groups one after another, each as many rounds as
    its longest packet needs at 2**lg lanes, on all 64 lanes."""
    lpp = 1 << ch.lg
    per = WAVE // lpp  # packets per group
    total = 0
    for g in range(0, len(ch.packets), per):
        r = int(((nblk[ch.packets[g:g + per]] + lpp - 1) // lpp).max())
        total += r * WAVE
    return total
