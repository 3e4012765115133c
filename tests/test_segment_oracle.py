"""CPU: the TX superpacket oracle (oracle/segment_oracle.py) pinned by the reference's own tests,
overlay/tio/virtio/segment_linux_test.go and overlay/checksum/checksum_test.go (same builders,
cases and assertions, restated), plus an independent from-scratch check of every checksum."""
import random
import struct

import pytest


@pytest.fixture(scope="module")
def S():
    import segment_oracle

    return segment_oracle


def build_tcpv4_super(pay_len):
    """segment_linux_test.go:36-67: 20 B IPv4 + 20 B TCP, ID 0x4242, seq 10000, ack 20000, ACK|PSH."""
    pkt = bytearray(40 + pay_len)
    pkt[0] = 0x45
    struct.pack_into(">H", pkt, 2, 40 + pay_len)
    struct.pack_into(">H", pkt, 4, 0x4242)
    pkt[8], pkt[9] = 64, 6
    pkt[12:16], pkt[16:20] = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    struct.pack_into(">HHII", pkt, 20, 12345, 80, 10000, 20000)
    pkt[32], pkt[33] = 0x50, 0x18
    struct.pack_into(">H", pkt, 34, 65535)
    for i in range(pay_len):
        pkt[40 + i] = i & 0xFF
    return bytes(pkt), 40, 20


def build_udpv4_super(pay_len):
    """segment_linux_test.go:69-90: 20 B IPv4 + 8 B UDP."""
    pkt = bytearray(28 + pay_len)
    pkt[0] = 0x45
    struct.pack_into(">H", pkt, 2, 28 + pay_len)
    struct.pack_into(">H", pkt, 4, 0x4242)
    pkt[8], pkt[9] = 64, 17
    pkt[12:16], pkt[16:20] = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    struct.pack_into(">HH", pkt, 20, 12345, 53)
    for i in range(pay_len):
        pkt[28 + i] = i & 0xFF
    return bytes(pkt), 28, 20


def pseudo_v4(S, src, dst, proto, l4len):
    s = S.checksum(src) + S.checksum(dst) + proto + l4len
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return s


def verify(S, b, pseudo):
    return S.checksum(b, pseudo) == 0xFFFF


@pytest.mark.parametrize("pay_len,gso", [(40, 8), (44, 8), (250, 100)])
def test_segment_tcp_header_not_corrupted(S, pay_len, gso):
    """segment_linux_test.go:127-218."""
    pkt, hl, cs = build_tcpv4_super(pay_len)
    segs = S.segment_tcp(pkt, hl, cs, gso)
    assert len(segs) == (pay_len + gso - 1) // gso
    off = 0
    for i, seg in enumerate(segs):
        assert seg[0] == 0x45 and seg[9] == 6
        assert seg[12:16] == bytes([10, 0, 0, 1]) and seg[16:20] == bytes([10, 0, 0, 2])
        assert struct.unpack_from(">HH", seg, 20) == (12345, 80)
        assert struct.unpack_from(">I", seg, 28)[0] == 20000 and seg[32] == 0x50
        assert struct.unpack_from(">I", seg, 24)[0] == 10000 + i * gso
        pl = len(seg) - hl
        assert seg[hl:] == bytes((off + k) & 0xFF for k in range(pl))
        off += pl
        assert verify(S, seg[:20], 0)
        assert verify(S, seg[20:], pseudo_v4(S, seg[12:16], seg[16:20], 6, len(seg) - 20))


@pytest.mark.parametrize("pay_len,gso", [(40, 8), (44, 8), (250, 100)])
def test_segment_udp_header_not_corrupted(S, pay_len, gso):
    """segment_linux_test.go:267-340."""
    pkt, hl, cs = build_udpv4_super(pay_len)
    segs = S.segment_udp(pkt, hl, cs, gso)
    assert len(segs) == (pay_len + gso - 1) // gso
    off = 0
    for i, seg in enumerate(segs):
        assert seg[0] == 0x45 and seg[9] == 17
        assert struct.unpack_from(">HH", seg, 20) == (12345, 53)
        assert struct.unpack_from(">H", seg, 4)[0] == 0x4242 + i
        pl = len(seg) - hl
        assert struct.unpack_from(">H", seg, 24)[0] == 8 + pl
        assert seg[hl:] == bytes((off + k) & 0xFF for k in range(pl))
        off += pl
        assert verify(S, seg[:20], 0)
        assert verify(S, seg[20:], pseudo_v4(S, seg[12:16], seg[16:20], 17, len(seg) - 20))


def test_correct_hdr_len_checksum_bound(S):
    """segment_linux_test.go:220-265."""
    pkt, _, cs = build_udpv4_super(12)
    assert S.correct_hdr_len(pkt, S.GSO_UDP_L4, cs, 6) == cs + 8
    short = bytes([0x45]) + bytes(24)
    with pytest.raises(S.SegmentError):
        S.correct_hdr_len(short, S.GSO_UDP_L4, 20, 6)


def build_udpv4_single(S, payload):
    """segment_linux_test.go:342-364: checksum field preloaded with the folded pseudo-header sum."""
    pkt = bytearray(28 + len(payload))
    pkt[0] = 0x45
    struct.pack_into(">H", pkt, 2, len(pkt))
    pkt[8], pkt[9] = 64, 17
    pkt[12:16], pkt[16:20] = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    struct.pack_into(">HHH", pkt, 20, 12345, 53, 8 + len(payload))
    pkt[28:] = payload
    struct.pack_into(">H", pkt, 26, pseudo_v4(S, pkt[12:16], pkt[16:20], 17, 8 + len(payload)))
    return bytes(pkt)


def test_finish_checksum_udp_zero_stores_all_ones(S):
    """segment_linux_test.go:366-393."""
    payload = None
    for i in range(0x10000):
        p = bytes([i >> 8, i & 0xFF])
        pkt = bytearray(build_udpv4_single(S, p))
        partial = struct.unpack_from(">H", pkt, 26)[0]
        pkt[26] = pkt[27] = 0
        if (~S.checksum(pkt[20:], partial)) & 0xFFFF == 0:
            payload = p
            break
    assert payload is not None
    out = S.finish_checksum(build_udpv4_single(S, payload), 20, 6)
    assert struct.unpack_from(">H", out, 26)[0] == 0xFFFF


def test_finish_checksum_tcp_zero_preserved(S):
    """segment_linux_test.go:395-423."""
    cs, co = 20, 16
    seg = bytearray(cs + co + 2)
    for i in range(len(seg) - cs):
        seg[cs + i] = (i * 7) & 0xFF
    partial = None
    for i in range(0x10000):
        struct.pack_into(">H", seg, cs + co, i)
        probe = bytearray(seg)
        probe[cs + co] = probe[cs + co + 1] = 0
        if (~S.checksum(probe[cs:], i)) & 0xFFFF == 0:
            partial = i
            break
    struct.pack_into(">H", seg, cs + co, partial)
    out = S.finish_checksum(bytes(seg), cs, co)
    assert struct.unpack_from(">H", out, cs + co)[0] == 0


def test_finish_checksum_udp_validates(S):
    """segment_linux_test.go:425-436."""
    payload = b"the definitive tun offloads branch"
    out = S.finish_checksum(build_udpv4_single(S, payload), 20, 6)
    assert verify(S, out[20:], pseudo_v4(S, out[12:16], out[16:20], 17, 8 + len(payload)))


@pytest.mark.parametrize("name,v6,gso_type,want_err", [
    ("tcpv4-ecn-v4", False, 1 | 0x80, False),
    ("tcpv4-ecn-v6-mismatch", True, 1 | 0x80, True),
    ("tcpv6-ecn-v4-mismatch", False, 4 | 0x80, True),
    ("udp-l4-ecn-rejected", False, 5 | 0x80, True),
    ("tcpv4-plain-v4", False, 1, False),
    ("tcpv4-plain-v6-mismatch", True, 1, True),
])
def test_check_valid_masks_gso_ecn(S, name, v6, gso_type, want_err):
    """segment_linux_test.go:442-475."""
    pkt, _, _ = build_tcpv4_super(100)
    if v6:
        pkt = bytes([0x60]) + pkt[1:]
    if want_err:
        with pytest.raises(S.SegmentError):
            S.check_valid(pkt, 0, gso_type, 100)
    else:
        S.check_valid(pkt, 0, gso_type, 100)


def test_check_valid_rejects_zero_gso_size(S):
    """segment_linux_test.go:477-485."""
    pkt, _, _ = build_tcpv4_super(100)
    with pytest.raises(S.SegmentError):
        S.check_valid(pkt, 0, S.GSO_TCPV4, 0)


@pytest.mark.parametrize("c", [0, 1, 0xFFFF, 0x10000, 0x1FFFE, 0xFFFF0000, 0xFFFEFFFF, 0xFFFFFFFF])
def test_fold_complement_matches_reference(S, c):
    """segment_linux_test.go:487-513."""
    s = c
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    assert S.fold_complement(c) == (~s) & 0xFFFF


def _lcg(state):
    state[0] = (state[0] * 1664525 + 1013904223) & 0xFFFFFFFF
    return state[0] >> 24


def test_base_sums_match_zeroing_reference(S):
    """segment_linux_test.go:542-602 (fewer iterations): the incremental base sums equal summing a
    copy with the rewritten fields zeroed, as seen on the wire."""
    st = [12345]
    for ihl in range(20, 61, 4):
        for _ in range(200):
            pkt = bytearray(_lcg(st) for _ in range(ihl))
            pkt[0] = 0x40 | (ihl // 4)
            tmp = bytearray(pkt)
            for o in (2, 3, 10, 11, 4, 5):
                tmp[o] = 0
            want = S.checksum(tmp)
            got = S.base_ipv4_hdr_sum(bytes(pkt), ihl)
            for tl in (20, 1500, 65535):
                for i in (0, 0x4242, 0xFFFF):
                    assert S.fold_complement(want + tl + i) == S.fold_complement(got + tl + i)
    for doff in range(5, 16):
        tl = doff * 4
        hl = 20 + tl
        for _ in range(100):
            pkt = bytearray(_lcg(st) for _ in range(hl + 64))
            pkt[0] = 0x45
            pkt[20 + 12] = doff << 4
            tmp = bytearray(pkt[20:hl])
            for o in (4, 5, 6, 7, 13, 16, 17):
                tmp[o] = 0
            want = S.checksum(tmp)
            got = S.base_tcp_hdr_sum(bytes(pkt), 20, hl)
            for seq in (0, 1, 0x42424242, 0xFFFFFFFF):
                for fl in (0x00, 0x10, 0x18, 0x19, 0xFF):
                    for l4 in (20, 1460, 65535):
                        assert S.fold_complement(want + seq + fl + l4) == S.fold_complement(got + seq + fl + l4)


def _gvisor_checksum_bytewise(buf, initial):
    """checksum_test.go's reference: plain 16-bit big-endian accumulation."""
    s = initial
    for i in range(0, len(buf) - 1, 2):
        s += (buf[i] << 8) | buf[i + 1]
    if len(buf) & 1:
        s += buf[-1] << 8
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


@pytest.mark.parametrize("n", [0, 1, 2, 3, 7, 31, 32, 33, 63, 64, 65, 127, 1300, 1501, 9001])
def test_checksum_matches_bytewise(S, n):
    """checksum_test.go:41-179: lengths across the tail paths, seeds 0 / 0xffff / random."""
    rng = random.Random(n)
    buf = bytes(rng.getrandbits(8) for _ in range(n))
    for init in (0, 0xFFFF, rng.getrandbits(16)):
        assert S.checksum(buf, init) == _gvisor_checksum_bytewise(buf, init)
    assert S.checksum(b"\xff" * n, 0) == _gvisor_checksum_bytewise(b"\xff" * n, 0)


def build_tcpv6_super(pay_len, tcp_opts=12):
    pkt = bytearray(40 + 20 + tcp_opts + pay_len)
    pkt[0] = 0x60
    struct.pack_into(">H", pkt, 4, 20 + tcp_opts + pay_len)
    pkt[6], pkt[7] = 6, 64
    pkt[8:24] = bytes(range(16))
    pkt[24:40] = bytes(range(100, 116))
    struct.pack_into(">HHII", pkt, 40, 443, 50000, 0xFFFFFF00, 7)
    pkt[52] = ((20 + tcp_opts) // 4) << 4
    pkt[53] = 0x80 | 0x18 | 0x01  # CWR | ACK | PSH | FIN
    for i in range(pay_len):
        pkt[60 + tcp_opts + i] = (i * 13) & 0xFF
    return bytes(pkt), 60 + tcp_opts, 40


def test_segment_tcp_v6_flags_seq_wrap(S):
    """IPv6 TSO with options: CWR only on the first segment, FIN|PSH only on the last, the sequence
    number wraps, payload length per segment, checksums verify from scratch."""
    pkt, hl, cs = build_tcpv6_super(5000)
    segs = S.segment_superpacket(pkt, S.F_NEEDS_CSUM, S.GSO_TCPV6, 0, 1400, cs, 16)
    assert len(segs) == 4
    for i, seg in enumerate(segs):
        fl = seg[cs + 13]
        assert bool(fl & 0x80) == (i == 0)
        assert bool(fl & 0x09) == (i == len(segs) - 1)
        assert struct.unpack_from(">I", seg, cs + 4)[0] == (0xFFFFFF00 + i * 1400) & 0xFFFFFFFF
        assert struct.unpack_from(">H", seg, 4)[0] == len(seg) - 40
        ps = S.checksum(seg[8:40]) + 6 + (len(seg) - 40)
        ps = (ps & 0xFFFF) + (ps >> 16)
        assert verify(S, seg[40:], ps)
