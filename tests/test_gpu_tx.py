"""GPU: the transmit batch (neb_tx_seal_batch[_host] — sendInsideMessage over a batch of TUN reads,
inside.go:154-240) against the oracle's packet-by-packet model (oracle/segment_oracle.py tx_batch:
decodeRead + SegmentSuperpacket + header.Encode + AEAD seal): every wire byte, counters, statuses."""
import random
import struct

import numpy as np
import pytest

from nebula_amd import _lib as L

pytestmark = pytest.mark.gpu

from test_segment_oracle import build_tcpv4_super, build_tcpv6_super, build_udpv4_super  # noqa: E402


def build_udpv6_super(pay_len):
    pkt = bytearray(48 + pay_len)
    pkt[0] = 0x60
    struct.pack_into(">H", pkt, 4, 8 + pay_len)
    pkt[6], pkt[7] = 17, 64
    pkt[8:24] = bytes(range(16, 32))
    pkt[24:40] = bytes(range(200, 216))
    struct.pack_into(">HH", pkt, 40, 4500, 4501)
    for i in range(pay_len):
        pkt[48 + i] = (i * 31 + 7) & 0xFF
    return bytes(pkt), 48, 40


def _pk(data, tunnel, flags=0, gso_type=0, gso_size=0, csum_start=0, csum_offset=0, hdr_len=0):
    return dict(data=bytes(data), tunnel=tunnel, flags=flags, gso_type=gso_type, hdr_len=hdr_len, gso_size=gso_size,
                csum_start=csum_start, csum_offset=csum_offset)


def _mixed_packets(S, rng):
    P = []
    tcp, _, cs = build_tcpv4_super(5000)
    P.append(_pk(tcp, 0, 1, S.GSO_TCPV4, 1448, cs, 16))                       # 4 TSO segments
    tcp6, _, cs6 = build_tcpv6_super(3001)
    P.append(_pk(tcp6, 1, 1, S.GSO_TCPV6 | S.GSO_ECN, 1000, cs6, 16))         # ECN-qualified, CWR/FIN
    udp, _, csu = build_udpv4_super(2500)
    P.append(_pk(udp, 0, 1, S.GSO_UDP_L4, 1200, csu, 6))                      # USO v4
    udp6, _, csu6 = build_udpv6_super(777)
    P.append(_pk(udp6, 2, 1, S.GSO_UDP_L4, 300, csu6, 6))                     # USO v6
    small, _, cs = build_tcpv4_super(44)
    P.append(_pk(small, 1, 1, S.GSO_TCPV4, 8, cs, 16))                        # gso < header length
    P.append(_pk(bytes(rng.getrandbits(8) for _ in range(1300)), 2))          # plain, no checksum work
    from test_segment_oracle import build_udpv4_single
    P.append(_pk(build_udpv4_single(S, b"finish me please" * 5), 0, S.F_NEEDS_CSUM, 0, 0, 20, 6))  # FinishChecksum
    P.append(_pk(tcp, 0, 1, S.GSO_TCPV4, 0, cs, 16))                          # gso_size 0: invalid
    P.append(_pk(udp, 1, 1, S.GSO_UDP_L4 | S.GSO_ECN, 1200, csu, 6))          # ECN on UDP: invalid
    P.append(_pk(tcp6, 0, 1, S.GSO_TCPV4, 1000, cs6, 16))                     # version mismatch
    P.append(_pk(tcp, 3, 1, S.GSO_TCPV4, 1448, cs, 16))                       # tunnel without a key
    P.append(_pk(tcp[:30], 0, 1, S.GSO_TCPV4, 1448, 20, 16))                  # too short for its TCP header
    P.append(_pk(b"", 0))                                                     # empty read
    P.append(_pk(tcp, 2, 1, S.GSO_TCPV4, 536, cs, 16))                        # many segments
    return P


def _to_arrays(packets, skew=None):
    from nebula_amd.inside import TX_PACKET_DTYPE

    offs, arena = [], bytearray()
    for p in packets:
        if skew is not None:  # read i starts skew[i % len(skew)] bytes past a 16-byte boundary
            off = ((len(arena) + 15) & ~15) + skew[len(offs) % len(skew)]
        else:
            off = (len(arena) + 15) & ~15 if len(offs) % 2 == 0 else len(arena) + 4  # 16- and 4-aligned inputs
        arena.extend(bytes(off - len(arena)))
        offs.append(off)
        arena.extend(p["data"])
    arena.extend(bytes(64))
    pk = np.zeros(len(packets), TX_PACKET_DTYPE)
    for i, (p, o) in enumerate(zip(packets, offs)):
        pk[i] = (o, len(p["data"]), p["tunnel"], p["flags"], p["gso_type"], p["hdr_len"], p["gso_size"],
                 p["csum_start"], p["csum_offset"], 0)
    return pk, np.frombuffer(bytes(arena), np.uint8).copy()


def _check(engine, oracle_mod, alg, packets, tun_spec, out_cap=1 << 20, max_wires=4096, device=False, key_hint=None,
           skew=None):
    import segment_oracle as S
    from nebula_amd.inside import TX_TUNNEL_DTYPE, DeviceTxBatch, tx_seal_batch_host
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly

    cf = CipherAESGCM if alg == L.ALG_AESGCM else CipherChaChaPoly
    ciphers = [cf.Cipher(engine, t["key"]) if t["key"] is not None else None for t in tun_spec]
    try:
        tun = np.zeros(len(tun_spec), TX_TUNNEL_DTYPE)
        for i, (t, c) in enumerate(zip(tun_spec, ciphers)):
            tun[i] = (t["counter"], c.key_id if c is not None else L.KEYS_MIXED, t["remote_index"])
        pk, arena = _to_arrays(packets, skew)

        def seal(a, key, ctr, hdr, seg):
            return oracle_mod.seal(a, key, oracle_mod.nonce(a, ctr), hdr, seg)

        exp_w, exp_pst, exp_ctr = S.tx_batch(alg, tun_spec, packets, out_cap, max_wires, seal,
                                             oracle_mod.header_encode)
        hint = L.KEYS_MIXED if key_hint is None else ciphers[key_hint].key_id
        if device:
            import torch
            db = DeviceTxBatch(engine, alg, tun, pk, arena, out_cap, max_wires, hint)
            db.seal()
            torch.cuda.synchronize()
            r = db.result()
        else:
            r = tx_seal_batch_host(engine, alg, tun, pk, arena, out_cap, max_wires, hint)
        assert r.packet_status.tolist() == exp_pst
        assert len(r.wires) == len(exp_w)
        for i, (off, c, ln, p, j, st, data) in enumerate(exp_w):
            w = r.wires[i]
            assert (int(w["out_off"]), int(w["counter"]), int(w["len"]), int(w["packet"]), int(w["segment"])) == \
                (off, c, ln, p, j), i
            assert int(r.wire_status[i]) == st, i
            if data is not None:
                assert r.wire_bytes(i) == data, (i, p, j)
        assert r.tunnels["message_counter"].tolist() == exp_ctr
        return r
    finally:
        for c in ciphers:
            if c is not None:
                c.destroy()


def _tunnels(rng, n=4, keyless=(3,)):
    return [dict(counter=2 + 1000 * t, remote_index=0xA000 + t,
                 key=None if t in keyless else bytes(rng.getrandbits(8) for _ in range(32))) for t in range(n)]


@pytest.mark.parametrize("alg", [L.ALG_AESGCM, L.ALG_CHACHAPOLY])
@pytest.mark.parametrize("device", [False, True])
def test_tx_batch_matches_sendinside(engine, oracle_mod, alg, device):
    import segment_oracle as S

    rng = random.Random(alg * 10 + device)
    _check(engine, oracle_mod, alg, _mixed_packets(S, rng), _tunnels(rng), device=device)


def test_tx_batch_exhaustion_and_single_key(engine, oracle_mod):
    """Counters crossing RejectAfterMessages mid-superpacket: the crossing segments are dropped
    (EXHAUSTED) with their counters used (inside.go:127-145); a one-tunnel batch on the single-key
    kernel."""
    import segment_oracle as S

    rng = random.Random(5)
    tun = _tunnels(rng, n=1, keyless=())
    tun[0]["counter"] = S.REJECT_AFTER - 3
    tcp, _, cs = build_tcpv4_super(6000)
    pk = [_pk(tcp, 0, 1, S.GSO_TCPV4, 1000, cs, 16), _pk(b"x" * 100, 0)]
    r = _check(engine, oracle_mod, L.ALG_AESGCM, pk, tun, key_hint=0)
    assert (r.wire_status == L.STATUS_EXHAUSTED).sum() == 5


def test_tx_batch_capacity_prefix(engine, oracle_mod):
    """An output too small for the batch keeps the longest fitting prefix of packets; the rest are
    NO_SPACE and use no counters."""
    import segment_oracle as S

    rng = random.Random(9)
    P = _mixed_packets(S, rng)
    _check(engine, oracle_mod, L.ALG_AESGCM, P, _tunnels(rng), out_cap=9000)
    _check(engine, oracle_mod, L.ALG_AESGCM, P, _tunnels(rng), max_wires=7)


def test_tx_batch_random_superpackets(engine, oracle_mod):
    """Random TSO/USO superpackets (v4/v6, header options, MSS, payload sizes up to 64 KiB) over 8
    tunnels."""
    import segment_oracle as S

    rng = random.Random(11)
    P = []
    for _ in range(60):
        kind = rng.randrange(4)
        pay = rng.choice([0, 1, 7, 100, 1447, 1448, 1449, 9000, 20000, 65000 - 120])
        if kind == 0:
            d, _, cs = build_tcpv4_super(pay)
            P.append(_pk(d, rng.randrange(8), 1, S.GSO_TCPV4, rng.choice([536, 1200, 1448, 8960]), cs, 16))
        elif kind == 1:
            d, _, cs = build_tcpv6_super(pay, tcp_opts=rng.choice([0, 12, 40]))
            P.append(_pk(d, rng.randrange(8), 1, S.GSO_TCPV6, rng.choice([1000, 1428]), cs, 16))
        elif kind == 2:
            d, _, cs = build_udpv4_super(pay)
            P.append(_pk(d, rng.randrange(8), 1, S.GSO_UDP_L4, rng.choice([512, 1472]), cs, 6))
        else:
            d, _, cs = build_udpv6_super(pay)
            P.append(_pk(d, rng.randrange(8), 1, S.GSO_UDP_L4, rng.choice([333, 1452]), cs, 6))
    _check(engine, oracle_mod, L.ALG_AESGCM, P, _tunnels(rng, n=8, keyless=()), out_cap=8 << 20, max_wires=8192)


@pytest.mark.parametrize("n", [1500, 3000])
def test_tx_batch_pre_parsed_plan(engine, oracle_mod, n):
    """1024 < reads <= 8192: parsed grid-wide first, then planned by one workgroup (2 and 8 reads
    per lane); keyless tunnels, invalid reads and an output that keeps only a prefix."""
    import segment_oracle as S

    rng = random.Random(n)
    P = []
    for i in range(n):
        if i % 211 == 3:
            d, _, cs = build_tcpv4_super(rng.choice([3000, 9000]))
            P.append(_pk(d, rng.randrange(8), 1, S.GSO_TCPV4, 1448, cs, 16))
        elif i % 97 == 5:
            P.append(_pk(b"", rng.randrange(8)))
        else:
            P.append(_pk(bytes(rng.getrandbits(8) for _ in range(rng.randrange(20, 120))), rng.randrange(9)))
    tun = _tunnels(rng, n=8, keyless=(2,))
    _check(engine, oracle_mod, L.ALG_AESGCM, P, tun, out_cap=n * 150, max_wires=16384)


@pytest.mark.parametrize("cut", [False, True])
def test_tx_batch_large_plan_path(engine, oracle_mod, cut):
    """More TUN reads than one workgroup plans (kTxPlanSmallMax = 8192): the device-wide planning
    path (hipCUB scan, radix sort, scan-by-key) and its counter update after the seal, with keyless
    tunnels, invalid reads and, with `cut`, an output that keeps only a prefix."""
    import segment_oracle as S

    rng = random.Random(21 + cut)
    P = []
    for i in range(8300):
        if i % 997 == 5:
            d, _, cs = build_tcpv4_super(rng.choice([3000, 9000]))
            P.append(_pk(d, rng.randrange(16), 1, S.GSO_TCPV4, 1448, cs, 16))
        elif i % 331 == 7:
            P.append(_pk(b"", rng.randrange(16)))  # short tun read
        else:
            P.append(_pk(bytes(rng.getrandbits(8) for _ in range(rng.randrange(20, 90))), rng.randrange(17)))
    tun = _tunnels(rng, n=16, keyless=(5,))
    _check(engine, oracle_mod, L.ALG_AESGCM, P, tun, out_cap=(600_000 if cut else 4 << 20), max_wires=16384)


@pytest.mark.parametrize("alg,single", [(L.ALG_AESGCM, True), (L.ALG_AESGCM, False), (L.ALG_CHACHAPOLY, False)])
def test_tx_batch_byte_skewed_reads(engine, oracle_mod, alg, single):
    """TUN reads at every byte skew from a 16-byte boundary: the seal reads each segment's payload
    from inside its read (sources 1-15 bytes off alignment, a header prefix from the slot), on the
    single-key kernel, the mixed-key chunk kernel and ChaCha20-Poly1305."""
    import segment_oracle as S

    rng = random.Random(31 + single + alg)
    P = []
    for i in range(32):
        d, _, cs = build_tcpv4_super(rng.choice([1447, 5000, 14000]))
        P.append(_pk(d, 0 if single else i % 3, 1, S.GSO_TCPV4, rng.choice([1448, 1200, 999]), cs, 16))
    P.append(_pk(bytes(rng.getrandbits(8) for _ in range(300)), 0))                      # plain
    tun = _tunnels(rng, n=1 if single else 3, keyless=())
    _check(engine, oracle_mod, alg, P, tun, out_cap=4 << 20, max_wires=4096, key_hint=0 if single else None,
           skew=list(range(16)))


@pytest.mark.parametrize("grid", [None, 1])
def test_tx_single_key_checksums_in_seal(engine, oracle_mod, grid, knobs):
    """One AES-GCM tunnel key: the seal sums the payloads into the L4 checksums itself (aes_gcm.hip
    gcm_csum_fix) — TSO v4/v6, USO v4/v6, FinishChecksum on TCP and UDP, an odd checksum start, and a
    field straddling two blocks (summed by the segment kernel instead). With `grid`, a 1-workgroup
    seal grid (NEB_KNOB_SINGLE_MAX_GRID) leaves a partial last pass to the tail kernel, whose segments
    the segment kernel sums."""
    import segment_oracle as S
    from test_segment_oracle import build_udpv4_single

    if grid is not None:
        knobs(L.KNOB_SINGLE_MAX_GRID, grid)
    rng = random.Random(77)
    P = []
    for i in range(24):
        d, _, cs = build_tcpv4_super(rng.choice([3000, 20000, 14477]))
        P.append(_pk(d, 0, 1, S.GSO_TCPV4, rng.choice([1448, 1200, 536]), cs, 16))
        if i % 4 == 0:
            d, _, cs = build_tcpv6_super(rng.choice([900, 9000]), tcp_opts=rng.choice([0, 12]))
            P.append(_pk(d, 0, 1, S.GSO_TCPV6, 1000, cs, 16))
            d, _, cs = build_udpv4_super(rng.choice([100, 5000]))
            P.append(_pk(d, 0, 1, S.GSO_UDP_L4, 1200, cs, 6))
            d, _, cs = build_udpv6_super(3000)
            P.append(_pk(d, 0, 1, S.GSO_UDP_L4, 333, cs, 6))
            P.append(_pk(build_udpv4_single(S, bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 300)))), 0,
                         S.F_NEEDS_CSUM, 0, 0, 20, 6))                                    # FinishChecksum, UDP
            d, _, cs = build_tcpv4_super(rng.randrange(1, 700))
            P.append(_pk(d, 0, S.F_NEEDS_CSUM, 0, 0, 20, 16))                             # FinishChecksum, TCP
            P.append(_pk(bytes(rng.getrandbits(8) for _ in range(200)), 0, S.F_NEEDS_CSUM, 0, 0, 21, 6))  # odd start
            P.append(_pk(bytes(rng.getrandbits(8) for _ in range(90)), 0, S.F_NEEDS_CSUM, 0, 0, 9, 6))    # straddles
            P.append(_pk(bytes(rng.getrandbits(8) for _ in range(777)), 0))                                # plain
    tun = _tunnels(rng, n=1, keyless=())
    r = _check(engine, oracle_mod, L.ALG_AESGCM, P, tun, out_cap=4 << 20, max_wires=4096, key_hint=0,
               skew=[0, 4, 8, 3])
    if grid is not None:
        assert len(r.wires) > 16 * 16 * grid  # past one full pass of the capped grid
