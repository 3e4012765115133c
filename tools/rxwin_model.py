"""CPU model of the device batched receive's parallel form (nebula_amd/csrc/rxwin.hip), step for
step as the kernels compute it, for one window's run of packets whose tags all verify. Used by
tests/test_rxwin_model.py to check the formulas against the sequential oracle
(oracle/replay_oracle.py) before anything runs on a GPU.

admit(k)   = first occurrence of c_k in the run and (c_k > cur_(k-1) or (c_k strictly within the
             window of cur_(k-1) and not received before the batch)), cur_k = max(current_0, c_1..c_k)
final bits = per slot s: the counter c_s it holds after the batch, (c_s <= current_0 ? old bit : 0)
             | (c_s admitted); above current the slots stay as they were during warmup
lost      += counters e >= 1 that left the window and were received neither before nor during
"""
from __future__ import annotations

M64 = (1 << 64) - 1


def in_window(i: int, cur: int, length: int) -> bool:
    if i < length and cur < length:
        return True
    return i > ((cur - length) & M64)


def admit(run, cur0: int, bits: list, length: int):
    """run: counters in arrival order -> admitted flags (rx_first_kernel + rx_admit_kernel)."""
    mask = length - 1
    seen = set()
    out = []
    prev = cur0
    for c in run:
        first = c not in seen
        seen.add(c)
        ok = c > prev
        if not ok and in_window(c, prev, length):
            ok = not (c <= cur0 and bits[c & mask])
        out.append(ok and first)
        prev = max(prev, c)
    return out


def ring(start: int, count: int, length: int) -> set:
    """slots of the circular range [start, start + count) mod length (count <= length)."""
    return {(start + k) % length for k in range(min(count, length))}


def finish_ranges(run, adm, cur0: int, bits: list, lost0: int, length: int):
    """The same as finish(), in the range form the device computes per bitmap word
    (rx_final_word_kernel): the slots of the counters new in (cur0, cur] are cleared, the admitted
    ones ORed in; the counters leaving the old window are one circular slot range too."""
    mask = length - 1
    cur = max([cur0] + list(run))
    lo = cur0 - length + 1 if cur0 >= length else 1
    hi = cur - length if cur >= length else 0
    scratch = [False] * length
    recv = 0
    for c, a in zip(run, adm):
        if not a:
            continue
        if cur < length or c > cur - length:
            scratch[c & mask] = True
        if lo <= c <= hi:
            recv += 1
    base = cur - length if (cur >= length and cur - length > cur0) else cur0
    clear = ring((base + 1) & mask, cur - base, length)
    ehi = min(hi, cur0)
    leaving = ring(lo & mask, ehi - lo + 1, length) if ehi >= lo else set()
    out = [(bits[s] and s not in clear) or scratch[s] for s in range(length)]
    recv += sum(1 for s in leaving if bits[s])
    exits = hi - lo + 1 if hi >= lo else 0
    return cur, out, lost0 + exits - recv


def finish(run, adm, cur0: int, bits: list, lost0: int, length: int):
    """(current, bits, lost) after the batch (rx_final_* kernels)."""
    mask = length - 1
    cur = max([cur0] + list(run))
    lo = cur0 - length + 1 if cur0 >= length else 1
    hi = cur - length if cur >= length else 0
    scratch = [False] * length
    recv = 0
    for c, a in zip(run, adm):
        if not a:
            continue
        if cur < length or c > cur - length:
            scratch[c & mask] = True
        if lo <= c <= hi:
            recv += 1
    out = list(bits)
    for s in range(length):
        ob = bits[s]
        has_old = not (cur0 < length and s > cur0)
        e_old = cur0 - ((cur0 - s) & mask) if cur0 >= length else s
        has_new = not (cur < length and s > cur)
        c_new = cur - ((cur - s) & mask) if cur >= length else s
        if has_old and ob and lo <= e_old <= min(hi, cur0):
            recv += 1
        if has_new:
            out[s] = (ob if c_new <= cur0 else False) or scratch[s]
    exits = hi - lo + 1 if hi >= lo else 0
    return cur, out, lost0 + exits - recv
