"""Reference model of the single-key kernel's bitsliced AES-256-CTR pass (aes_gcm.hip, bs_pass),
step for step as the device code runs it on one quad of lanes (one packet): used by
tests/test_bitsliced_model.py to check the construction against the oracle's AES on the CPU.

Layout. Lane c (0..3) of the quad holds column c of the AES state of 32 counter blocks in 32
bit planes P[i][b] (row i = byte 4c + i of the block, bit b of that byte); bit k of a plane
belongs to block k, whose counter is base + k. The S-box is the generated bitop3 network
(tools/gen_bs_sbox.py), ShiftRows moves row i from lane (c + i) & 3 (a DPP quad_perm on the
device), MixColumns and AddRoundKey are plane XORs. After round 14 a 32x32 bit transpose gives
each lane D[k] = column word c of block k, and a 4x4 exchange across the quad gives lane l the
four column words of block 4j + l for consumption round j.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gen_bs_sbox as G  # noqa: E402

M32 = 0xFFFFFFFF
K_PLANES = [0xAAAAAAAA, 0xCCCCCCCC, 0xF0F0F0F0, 0xFF00FF00, 0xFFFF0000, 0, 0, 0]


def _network():
    gates = G.parse()
    nodes = G.to_nodes(gates)
    order = [g[0] for g in gates]
    nodes, order = G.fold(nodes, order)
    return [(n, *G.bitop3_code(*nodes[n])) for n in order]


NET = _network()


def bitop3(code, a, b, c):
    r = 0
    for idx in range(8):
        if (code >> idx) & 1:
            ma = a if idx & 4 else ~a
            mb = b if idx & 2 else ~b
            mc = c if idx & 1 else ~c
            r |= ma & mb & mc
    return r & M32


def sbox_planes(p):
    """p[7] = MSB plane ... p[0] = LSB plane -> S-box applied to all 32 bytes."""
    env = {f"x{i}": p[7 - i] for i in range(8)}
    for n, ops, code in NET:
        env[n] = bitop3(code, env[ops[0]], env[ops[1]], env[ops[2]])
    return [env[f"s{7 - b}"] for b in range(8)]


def mask(word, bit):
    return M32 if (word >> bit) & 1 else 0


def bs_keystream(rk_words, c1, c2, base):
    """Keystream of counters base..base+31 (low byte; bytes 12-14 zero) for one packet nonce.
    rk_words: the 60 little-endian round-key words. Returns ks[k] = 4 LE column words."""
    P = [[[0] * 8 for _ in range(4)] for _ in range(4)]  # P[lane][row][bit]
    for c in range(4):
        w = (0, c1, c2, 0)[c] ^ rk_words[c]
        for i in range(4):
            for b in range(8):
                P[c][i][b] = mask(w, 8 * i + b)
        # counter planes: bits of (base + k), bitsliced ripple add; only lane 3, row 3 (byte 15)
        carry, is3 = 0, M32 if c == 3 else 0
        for b in range(8):
            Bb = mask(base & 0xFF, b)
            s = K_PLANES[b] ^ Bb ^ carry
            carry = (K_PLANES[b] & Bb) | (K_PLANES[b] & carry) | (Bb & carry)
            P[c][3][b] ^= s & is3
    for r in range(1, 15):
        for c in range(4):
            for i in range(4):
                P[c][i] = sbox_planes(P[c][i])
        # ShiftRows: lane c, row i <- lane (c + i) & 3
        P = [[list(P[(c + i) & 3][i]) for i in range(4)] for c in range(4)]
        for c in range(4):
            kw = rk_words[4 * r + c]
            a = P[c]
            if r < 14:
                t = [[a[i][b] ^ a[(i + 1) & 3][b] for b in range(8)] for i in range(4)]
                u = [t[0][b] ^ a[2][b] ^ a[3][b] for b in range(8)]
                out = []
                for i in range(4):
                    ti = t[i]
                    X = [ti[7], ti[0] ^ ti[7], ti[1], ti[2] ^ ti[7], ti[3] ^ ti[7], ti[4], ti[5], ti[6]]
                    out.append([X[b] ^ u[b] ^ a[i][b] ^ mask(kw, 8 * i + b) for b in range(8)])
                P[c] = out
            else:
                P[c] = [[a[i][b] ^ mask(kw, 8 * i + b) for b in range(8)] for i in range(4)]
    # transpose: D[k] bit (8i + b) = bit k of P[i][b]
    D = []
    for c in range(4):
        rows = [P[c][r >> 3][r & 7] for r in range(32)]
        D.append(transpose32(rows))
    # quad exchange: lane l, round j <- (D[0][4j+l], D[1][4j+l], D[2][4j+l], D[3][4j+l])
    ks = []
    for j in range(8):
        M = [[D[c][4 * j + l] for l in range(4)] for c in range(4)]  # lane c, slot l
        N = quad_transpose(M)
        for l in range(4):
            ks.append(tuple(N[l]))
    return ks  # index 4j + l = block k


def transpose32(a):
    """a[r] bit k -> out[k] bit r, by the 5-stage swap network the device code uses."""
    a = list(a)
    masks = {16: 0x0000FFFF, 8: 0x00FF00FF, 4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}
    for w in (16, 8, 4, 2, 1):
        m = masks[w]
        for r in range(32):
            if r & w:
                continue
            x, y = a[r], a[r + w]
            # rows r (bit w clear) and r + w: swap x's high w-blocks with y's low w-blocks
            t = ((x >> w) ^ y) & m
            a[r + w] = y ^ t
            a[r] = x ^ ((t << w) & M32)
    return a


def quad_transpose(M):
    """The device's two-stage exchange: xor-2 partners then xor-1 partners, 4 slots per lane."""
    A = [[M[c ^ 2][l ^ 2] if ((c ^ l) & 2) else M[c][l] for l in range(4)] for c in range(4)]
    B = [[A[c ^ 1][l ^ 1] if ((c ^ l) & 1) else A[c][l] for l in range(4)] for c in range(4)]
    return B


def key_schedule_words(key: bytes):
    """FIPS-197 AES-256 key expansion as 60 little-endian words (the kernel's rk layout)."""
    sbox = G.SBOX
    w = [list(key[4 * i:4 * i + 4]) for i in range(8)]
    rcon = 1
    for i in range(8, 60):
        t = list(w[i - 1])
        if i % 8 == 0:
            t = [sbox[t[1]] ^ rcon, sbox[t[2]], sbox[t[3]], sbox[t[0]]]
            rcon = ((rcon << 1) ^ (0x1B if rcon & 0x80 else 0)) & 0xFF
        elif i % 8 == 4:
            t = [sbox[x] for x in t]
        w.append([a ^ b for a, b in zip(w[i - 8], t)])
    return [x[0] | x[1] << 8 | x[2] << 16 | x[3] << 24 for x in w]
