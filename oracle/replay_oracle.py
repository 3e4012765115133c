"""replay_oracle.py — TEST INFRASTRUCTURE ONLY: a pure-Python restatement of Nebula's anti-replay
window and of the receive-side Check → DecryptDanger → Update sequence, used by tests/ as the
checker for the engine's C++ window (nebula_amd/csrc/window.cpp) and batched RX open. The
product never imports this module.

Restated from slackhq/nebula (read as text, not copied):
  Bits / NewBits        bits.go:18-50   (power-of-two length, bitmap of length bits, slot 0 seeded)
  get / set             bits.go:52-61
  clearRange            bits.go:63-118  (clear `count` circular slots from startPos, return how many were set)
  strictlyWithinWindow  bits.go:120-132 (warmup clause, then i > current - length in uint64 arithmetic)
  Check                 bits.go:134-150
  Update / updateSlow   bits.go:152-262 (fast path i == current+1, jump path with lost accounting,
                                         in-window backfill / duplicate, out of window)
  ConnectionState.Decrypt  connection_state.go:99-119 (Check under lock, DecryptDanger, Update)

Pinned by tests/golden/replay_window.json: the scenarios and expected values of the reference's
bits_test.go (TestBits, TestBitsLargeJumps, TestBitsDupeCounter, TestBitsOutOfWindowCounter,
TestBitsLostCounter, TestBitsLostCounterIssue1, TestBitsWarmupOvershoot,
TestBitsCheckAcrossWarmupBoundary, TestBitsMarkerInvariant), transcribed as data.
"""
from __future__ import annotations

M64 = (1 << 64) - 1


def _i64(x: int) -> int:
    """Go's int64(x) / int64 arithmetic: two's-complement wrap."""
    x &= M64
    return x - (1 << 64) if x >> 63 else x

# status codes of the batched RX open (include/nebula_aead.h)
OK, AUTH_FAILED, EXHAUSTED, BAD_KEY, REPLAY, INVALID, NOT_MESSAGE = 0, 1, 2, 3, 4, 5, 7


class Bits:
    def __init__(self, length: int):
        if length == 0 or length & (length - 1):
            raise ValueError(f"Bits length must be a power of two, got {length}")
        self.length = length
        self.mask = length - 1
        self.current = 0
        self.bits = [False] * length  # one flag per slot; the packing into words is irrelevant here
        self.bits[0] = True           # counter 0 never exists: seeded as received
        self.lost = self.dupe = self.out_of_window = 0

    def get(self, i: int) -> bool:
        return self.bits[i & self.mask]

    def set(self, i: int) -> None:
        self.bits[i & self.mask] = True

    def clear_range(self, start: int, count: int) -> int:
        if count >= self.length:
            was = sum(self.bits)
            self.bits = [False] * self.length
            return was
        was = 0
        for k in range(count):
            p = (start + k) & self.mask
            was += self.bits[p]
            self.bits[p] = False
        return was

    def strictly_within_window(self, i: int) -> bool:
        if i < self.length and self.current < self.length:
            return True
        return i > ((self.current - self.length) & M64)

    def check(self, i: int) -> bool:
        if i > self.current:
            return True
        if self.strictly_within_window(i):
            return not self.get(i)
        return False

    def update(self, i: int) -> bool:
        if i == ((self.current + 1) & M64):
            if i > self.length and not self.get(i):
                self.lost += 1
            self.set(i)
            self.current = i
            return True
        if i > self.current:
            top = (self.current + self.length) & M64  # uint64 arithmetic, as in Go
            end = top if i > top else i
            count = (end - self.current) & M64
            start = (self.current + 1) & self.mask
            if self.current >= self.length:
                lost = _i64(count - self.clear_range(start, count))
            else:
                lost = sum(1 for n in range(self.current + 1, end + 1) if not self.get(n) and n > self.length)
                self.clear_range(start, count)
            if i > top:
                lost = _i64(lost + _i64(i - self.current - self.length))
            self.lost = _i64(self.lost + lost)
            self.set(i)
            self.current = i
            return True
        if self.strictly_within_window(i):
            if self.current == i or self.get(i):
                self.dupe += 1
                return False
            self.set(i)
            return True
        self.out_of_window += 1
        return False

    def reset_counters(self) -> None:
        self.lost = self.dupe = self.out_of_window = 0

    def snapshot(self):
        return list(self.bits)


def rx_sequential(windows, keys, counters, verdicts):
    """Reference receive order (connection_state.go:99-119), one packet after another:
    Check → DecryptDanger (its verdict: True/OK, False/AUTH_FAILED, or BAD_KEY for a key the
    engine does not hold) → Update. Returns the per-packet statuses and, for each packet, whether
    DecryptDanger ran on it (a packet refused by Check is never decrypted).
    windows: dict key -> Bits (missing key → BAD_KEY, no window activity)."""
    status, decrypted = [], []
    for k, c, v in zip(keys, counters, verdicts):
        v = OK if v is True else AUTH_FAILED if v is False else v
        w = windows.get(k)
        if w is None:
            status.append(BAD_KEY)
            decrypted.append(False)
            continue
        if not w.check(c):
            status.append(REPLAY)
            decrypted.append(False)
            continue
        decrypted.append(True)
        if v != OK:
            status.append(v)
            continue
        status.append(OK if w.update(c) else REPLAY)
    return status, decrypted


def read_outside_gate(packet: bytes, has_tunnel: bool, own_source: bool = False):
    """readOutsidePackets (outside.go:30-114) up to the decrypt, restated: h.Parse
    (header.go:143-156), the version and IsValidSubType checks (header.go:192-205), the caller's
    double-encryption check (outside.go:66-74, `own_source`), the unencrypted
    types handed elsewhere (outside.go:83-89), the hostinfo lookup (outside.go:94-106) and the size
    check (outside.go:108-114). Returns (status, None) for a packet that stops here, or
    (None, (kind, counter)) with kind "decrypt" (Decrypt, header as AD, in place) or "relay"
    (VerifyRelay: AD = packet[:len-16], tag = the last 16 bytes)."""
    if len(packet) < 16:
        return INVALID, None
    ver, typ, sub = packet[0] >> 4, packet[0] & 15, packet[1]
    if ver != 1:
        return INVALID, None
    if typ in (1, 4):
        valid = sub in (0, 1)
    elif typ in (0, 2, 3, 5, 6):
        valid = sub == 0
    else:
        valid = False
    if not valid:
        return INVALID, None
    if own_source:  # outside.go:66-74: not relayed, UDP source inside the node's own VPN networks
        return INVALID, None
    if typ in (0, 2):
        return NOT_MESSAGE, None
    if not has_tunnel:
        return BAD_KEY, None
    if len(packet) < 32:
        return INVALID, None
    counter = int.from_bytes(packet[8:16], "big")
    return None, ("relay" if (typ == 1 and sub == 1) else "decrypt", counter)
