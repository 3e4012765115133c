"""CPU check of the bitsliced AES-256-CTR construction the single-key kernel uses for 8 of a
packet's rounds (tools/bs_model.py mirrors the device code step for step; the S-box network is
tools/gen_bs_sbox.py's output): its keystream must equal the oracle's AES on every counter."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_generated_sbox_matches_fips197():
    import bs_model as M
    for x in range(256):
        planes = [M.M32 if (x >> b) & 1 else 0 for b in range(8)]
        out = M.sbox_planes(planes)
        y = sum(1 << b for b in range(8) if out[b] & 1)
        assert y == M.G.SBOX[x]


def test_transposes():
    import bs_model as M
    rng = random.Random(5)
    a = [rng.getrandbits(32) for _ in range(32)]
    t = M.transpose32(a)
    for k in range(32):
        for r in range(32):
            assert (t[k] >> r) & 1 == (a[r] >> k) & 1
    Mx = [[rng.getrandbits(32) for _ in range(4)] for _ in range(4)]
    N = M.quad_transpose(Mx)
    assert all(N[l][c] == Mx[c][l] for l in range(4) for c in range(4))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bitsliced_keystream_matches_oracle(oracle_mod, seed):
    import bs_model as M
    rng = random.Random(seed)
    key = bytes(rng.getrandbits(8) for _ in range(32))
    n = rng.getrandbits(64)
    rk = M.key_schedule_words(key)
    c1 = int.from_bytes((n >> 32).to_bytes(4, "big"), "little")
    c2 = int.from_bytes((n & 0xFFFFFFFF).to_bytes(4, "big"), "little")
    base = rng.choice([2, 3, 18, 34, 50, 200])
    ks = M.bs_keystream(rk, c1, c2, base)
    for k in range(32):
        ctr = (base + k) & 0xFF
        blk = bytes(4) + n.to_bytes(8, "big") + ctr.to_bytes(4, "big")
        ref = oracle_mod.aes_block(key, blk)
        got = b"".join(w.to_bytes(4, "little") for w in ks[k])
        assert got == ref, (k, ctr)


def test_byte_window_ghash_model(oracle_mod):
    """The byte-window GHASH of the single-key kernel (gf_mul_byte, NEB_GHASH8): F8_P[b] built from
    the nibble table, each lane reading its 16 byte positions rotated by lane & 15 so that the 16
    lanes of a ds_read_b128 group hit 16 different bank groups; the product equals X·H^4."""
    rng = random.Random(11)
    H4 = bytes(rng.getrandbits(8) for _ in range(16))

    def elem(p, v):  # nibble v at nibble position p (GCM bit order, v's MSB -> x^(4p))
        bits = bytearray(16)
        for t in range(4):
            if (v >> (3 - t)) & 1:
                bit = 4 * p + t
                bits[bit // 8] |= 0x80 >> (bit % 8)
        return bytes(bits)

    def xor(a, b):
        return bytes(x ^ y for x, y in zip(a, b))

    F4 = [[oracle_mod.gf128_mul(elem(p, v), H4) for v in range(16)] for p in range(32)]
    F8 = [xor(F4[2 * (i & 15)][(i >> 4) >> 4], F4[2 * (i & 15) + 1][(i >> 4) & 15]) for i in range(4096)]
    M32 = 0xFFFFFFFF
    for _ in range(64):
        x = bytes(rng.getrandbits(8) for _ in range(16))
        lane = rng.randrange(64)
        f = lane & 15
        Z = [int.from_bytes(x[4 * q:4 * q + 4], "little") for q in range(4)]  # bswap of the BE words
        r1 = Z[1:] + Z[:1] if f & 4 else Z
        r2 = r1[2:] + r1[:2] if f & 8 else r1
        s = 8 * (f & 3)
        Y = [((r2[(m + 1) & 3] << 32 | r2[m]) >> s) & M32 for m in range(4)]
        acc = bytes(16)
        banks = set()
        for j in range(16):
            b = (Y[j >> 2] >> (8 * (j & 3))) & 0xFF
            P = (f + j) & 15
            banks.add(P)
            acc = xor(acc, F8[b * 16 + P])
        assert len(banks) == 16
        assert acc == oracle_mod.gf128_mul(x, H4)
