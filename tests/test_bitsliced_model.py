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
