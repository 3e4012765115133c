"""CPU model of the key-setup kernel's GF(2^128) word arithmetic (aes_gcm.hip): gf_mul_xpow (q·x^i as
a shifted 256-bit product, reduced by gf_reduce) builds every basis table of gcm_key_setup_kernel in
parallel, one lane per power. The model follows the device code word for word and is checked
against the bit-serial multiply by x (gf_mulx) it replaced, for every i < 128."""
import random

M = 0xFFFFFFFF


def mulx(v):
    x, y, z, w = v
    return [((x >> 1) ^ (0xE1000000 if w & 1 else 0)) & M, ((x << 31) | (y >> 1)) & M,
            ((y << 31) | (z >> 1)) & M, ((z << 31) | (w >> 1)) & M]


def shr64(hi, lo, s):  # v_alignbit_b32
    return (((hi << 32) | lo) >> s) & M


def gf_reduce(z):
    l0, l1, l2, l3 = z[4:8]
    t0 = l0 ^ (l0 >> 1) ^ (l0 >> 2) ^ (l0 >> 7)
    t1 = l1 ^ shr64(l0, l1, 1) ^ shr64(l0, l1, 2) ^ shr64(l0, l1, 7) ^ z[1]
    t2 = l2 ^ shr64(l1, l2, 1) ^ shr64(l1, l2, 2) ^ shr64(l1, l2, 7) ^ z[2]
    t3 = l3 ^ shr64(l2, l3, 1) ^ shr64(l2, l3, 2) ^ shr64(l2, l3, 7) ^ z[3]
    o = ((l3 << 31) ^ (l3 << 30) ^ (l3 << 25)) & M
    of = o ^ (o >> 1) ^ (o >> 2) ^ (o >> 7)
    return [z[0] ^ t0 ^ of, t1, t2, t3]


def gf_mul_xpow(q, i):
    w, b = i >> 5, i & 31
    y = [next((q[j] for j in range(4) if k - j == w), 0) for k in range(8)]
    z = [y[0] >> b] + [shr64(y[k - 1], y[k], b) for k in range(1, 8)]
    return gf_reduce(z)


def test_gf_mul_xpow_matches_repeated_mulx():
    rng = random.Random(2026)
    cases = [[0, 0, 0, 1], [0x80000000, 0, 0, 0], [M, M, M, M]] + \
            [[rng.getrandbits(32) for _ in range(4)] for _ in range(60)]
    for q in cases:
        v = list(q)
        for i in range(128):
            assert gf_mul_xpow(q, i) == v, (q, i)
            v = mulx(v)


def _gmul(a, b):
    """GF(2^128) product in GCM bit order (SP 800-38D, algorithm 1) on 128-bit ints."""
    R = 0xE1 << 120
    z, v = 0, a
    for i in range(127, -1, -1):
        if (b >> i) & 1:
            z ^= v
        v = (v >> 1) ^ (R if v & 1 else 0)
    return z


def _ghash_lanes(X, H, lpp, U):
    """The GHASH pass's lane layout (aes_gcm.hip ghash_packet_group): the n blocks front-padded to
    lpp·R, lane l owning padded blocks lpp·r + l; rounds aggregated U at a time (zero rounds in
    front), A <- A·H^(U·lpp) ⊕ Σ_i X_i·H^((U-1-i)·lpp); then Σ_l A_l·H^(lpp-l)."""
    n = len(X)
    R = -(-n // lpp)
    pad = lpp * R - n
    M = -(-R // U)
    front = U * M - R
    pw = [1 << 127]  # x^0: the most significant bit in GCM bit order
    for _ in range(U * lpp + 1):
        pw.append(_gmul(pw[-1], H))
    S = 0
    for l in range(lpp):
        def blk(r):
            if r < 0 or r >= R:
                return 0
            g = lpp * r + l - pad
            return X[g] if 0 <= g < n else 0
        A = 0
        for mr in range(M):
            acc = _gmul(A, pw[U * lpp]) if mr else 0
            for i in range(U - 1):
                acc ^= _gmul(blk(U * mr + i - front), pw[(U - 1 - i) * lpp])
            A = acc ^ blk(U * mr + U - 1 - front)
        S ^= _gmul(A, pw[lpp - l])
    return S


def test_aggregated_ghash_rounds_equal_ghash():
    """Aggregating U rounds (one reduction, zero rounds in front when U does not divide R) leaves
    GHASH unchanged: every block count 1..60, U = 1..3, 4 lanes per packet (and 8 / 16 at U = 1)."""
    rng = random.Random(7)
    H = rng.getrandbits(128) | 1
    for n in range(1, 61):
        X = [rng.getrandbits(128) for _ in range(n)]
        ref = 0
        for x in X:  # Y_i = (Y_(i-1) ⊕ X_i)·H
            ref = _gmul(ref ^ x, H)
        for U in (1, 2, 3):
            assert _ghash_lanes(X, H, 4, U) == ref, (n, U)
        for lpp in (8, 16):
            assert _ghash_lanes(X, H, lpp, 1) == ref, (n, lpp)
