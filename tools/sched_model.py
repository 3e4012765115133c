"""CPU model of the mixed-key scheduler (nebula_amd/csrc/sched.hpp, sched.hip): the (size class,
key) binning, the per-key chunk plan of sched_alloc_kernel (round 6: a key's leftovers planned
together, longest-first cost buckets) and the workspace bounds, rule for rule, so the
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


def groups(cls: int) -> int:
    """sched_groups: groups of 16 packets per front chunk."""
    return 1 if cls >= 3 else 8 >> cls


BUCKETS = 8


def bucket(cost: int) -> int:
    """sched_bucket: cost (rounds at the class's upper bound + finals) -> bucket, longest first."""
    for b, lo in enumerate((24, 16, 12, 9, 7, 5, 3)):
        if cost >= lo:
            return b
    return 7


def front_cost(ngroups: int, cls: int) -> int:
    return ngroups * ((1 << cls) + 1)


def tail_cost(cls: int, lg: int) -> int:
    r = ((1 << cls) * 4) >> lg
    return max(r, 1) + 2


def nbins(max_keys: int) -> int:
    return SIZE_CLASSES * (max_keys + 1)


def max_chunks(n: int, max_keys: int) -> int:
    nb = nbins(max_keys)
    return (n + CHUNK_PKTS - 1) // CHUNK_PKTS + min(n, nb)


@dataclass
class Chunk:
    kind: str            # "front" (4-lane groups) or "tail" (one group at 8 or 16 lanes)
    packets: np.ndarray  # packet indices: segment 0 (class cls), then segment 1 (a smaller class)
    key: int
    cls: int             # segment 0's size class
    lg: int              # lanes per packet = 2**lg
    count0: int          # packets in segment 0
    bucket: int


def key_chunks(key: int, counts, starts, max_groups: int = 8):
    """sched_alloc_block's chunks for one key: counts[cls] packets of class cls from starts[cls] in
    `sorted`, front chunks of at most min(groups(cls), max_groups) groups.
    Returns (kind, cls, lg, (start0, count0), (start1, count1), bucket) in emission order."""
    out = []
    left, lpos = [0] * SIZE_CLASSES, [0] * SIZE_CLASSES
    for c in range(SIZE_CLASSES):
        nf, g = counts[c] // CHUNK_PKTS, min(groups(c), max_groups)
        for j in range(0, nf, g):
            gc = min(g, nf - j)
            out.append(("front", c, 2, (starts[c] + j * CHUNK_PKTS, gc * CHUNK_PKTS), (0, 0), bucket(front_cost(gc, c))))
        left[c] = counts[c] % CHUNK_PKTS
        lpos[c] = starts[c] + nf * CHUNK_PKTS
    for i in range(SIZE_CLASSES - 1, -1, -1):
        L = left[i]
        if L == 0:
            continue
        lg = tail_lg(L, i)
        free = (64 >> lg) - L
        s1 = c1 = 0
        for j in range(i - 1, -1, -1):  # the next smaller class with a leftover fills the free slots
            if left[j]:
                c1 = min(free, left[j])
                s1 = lpos[j]
                lpos[j] += c1
                left[j] -= c1
                break
        front = lg == 2
        out.append(("front" if front else "tail", i, lg, (lpos[i], L), (s1, c1),
                    bucket(front_cost(1, i) if front else tail_cost(i, lg))))
    return out


def plan(key_id: np.ndarray, aad_len: np.ndarray, length: np.ndarray, max_keys: int,
         max_groups: int = 8) -> List[Chunk]:
    """The chunks sched_alloc_kernel writes for one batch: per key, its classes one after another in
    `sorted`, and sched_key_chunks' records."""
    key = np.where(key_id < max_keys, key_id, max_keys).astype(np.int64)
    cls = size_class(aad_len, length)
    order = np.lexsort((cls, key))  # sorted[]: key-major, classes in turn (any order inside a bin)
    out: List[Chunk] = []
    sk, sc = key[order], cls[order]
    kstarts = np.r_[0, np.flatnonzero(np.diff(sk)) + 1] if len(sk) else np.zeros(0, np.int64)
    kends = np.r_[kstarts[1:], len(sk)]
    for s, e in zip(kstarts, kends):
        k = int(sk[s])
        counts = [int((sc[s:e] == c).sum()) for c in range(SIZE_CLASSES)]
        starts = list(s + np.r_[0, np.cumsum(counts)[:-1]])
        for kind, c, lg, (s0, c0), (s1, c1), b in key_chunks(k, counts, starts, max_groups):
            pk = np.r_[order[s0:s0 + c0], order[s1:s1 + c1]].astype(np.int64)
            out.append(Chunk(kind, pk, k, c, lg, c0, b))
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
