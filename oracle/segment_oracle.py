"""segment_oracle.py — TEST INFRASTRUCTURE ONLY: a numpy/Python restatement of Nebula's TX
superpacket path — TSO/USO segmentation with checksum completion, then the per-segment
header.Encode + EncryptDanger into send-batch slots — used by tests/ and bench.py's cpu_baseline
leg as the checker for the engine's fused segment+seal batch (nebula_amd/csrc/tx.hip, the TX
batch's plan, segment and seal kernels).
The product never imports this module.

Restated from slackhq/nebula (read as text, not copied):
  RFC 1071 sum               overlay/checksum/checksum_*.go (gvisor tcpip/checksum.Checksum [ext]:
                             big-endian 16-bit one's-complement sum, odd tail byte as the high
                             byte, seeded with `initial`, folded, not complemented)
  virtio_net_hdr             overlay/tio/virtio/header_linux.go:14-75 (GSOType masks GSO_ECN 0x80)
  CheckValid                 overlay/tio/virtio/segment_linux.go:74-120
  CorrectHdrLen              segment_linux.go:122-154
  segCount                   segment_linux.go:156-164
  basePseudoSum / baseIPv4HdrSum / baseTCPHdrSum   segment_linux.go:166-208
  SegmentTCP                 segment_linux.go:210-310 (seq += offset, CWR only on the first segment,
                             FIN|PSH only on the last, IPv4 ID += i, incremental checksums)
  SegmentUDP                 segment_linux.go:312-398 (UDP length, checksum over header+payload,
                             0 sent as 0xffff)
  FinishChecksum             segment_linux.go:400-423
  foldComplement             segment_linux.go:425-431
  decodeRead                 overlay/tio/tio_gso_linux.go:231-280 (GSO_NONE: FinishChecksum only)
  SegmentSuperpacket         overlay/tio/tun_linux_offload.go:46-60
  sendInsideMessage          inside.go:154-240 (each segment sealed into a Reserve(16+len+16) slot)
  sendInsideEncrypt          inside.go:123-146 (NextMessageCounter; on refusal the segment is dropped)
"""
from __future__ import annotations

import struct

import numpy as np

# linux/virtio_net.h
F_NEEDS_CSUM = 1
F_DATA_VALID = 2
F_RSC_INFO = 4
GSO_NONE = 0
GSO_TCPV4 = 1
GSO_UDP = 3
GSO_TCPV6 = 4
GSO_UDP_L4 = 5
GSO_ECN = 0x80
IPPROTO_TCP = 6
IPPROTO_UDP = 17

MAX_SEG_HDR = 120


class SegmentError(ValueError):
    pass


def checksum(buf, initial: int = 0) -> int:
    """RFC 1071 one's-complement sum of buf (big-endian words, odd tail byte high), seeded."""
    b = np.frombuffer(bytes(buf), np.uint8)
    s = int(initial)
    n2 = len(b) & ~1
    if n2:
        s += int(b[:n2].view(">u2").astype(np.uint64).sum())
    if len(b) & 1:
        s += int(b[-1]) << 8
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def fold_complement(s: int) -> int:
    s &= 0xFFFFFFFF
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def check_valid(pkt: bytes, flags: int, gso_type: int, gso_size: int) -> None:
    if flags & F_RSC_INFO:
        raise SegmentError("virtio RSC_INFO flag not supported on TUN reads")
    if len(pkt) < 20:
        raise SegmentError("packet too short")
    ver = pkt[0] >> 4
    if ver == 6 and len(pkt) < 40:
        raise SegmentError("packet too short")
    g = gso_type & ~GSO_ECN
    if g != GSO_NONE and gso_size == 0:
        raise SegmentError("GSO type with zero gso_size")
    if gso_type & GSO_ECN and g not in (GSO_TCPV4, GSO_TCPV6):
        raise SegmentError("GSO_ECN on non-TCP GSO type")
    if g == GSO_TCPV4 and ver != 4:
        raise SegmentError("IP version mismatch")
    if g == GSO_TCPV6 and ver != 6:
        raise SegmentError("IP version mismatch")
    if ver not in (4, 6):
        raise SegmentError("invalid IP version")


def correct_hdr_len(pkt: bytes, gso_type: int, csum_start: int, csum_offset: int) -> int:
    """Returns the corrected header length (CorrectHdrLen)."""
    if gso_type & ~GSO_ECN == GSO_UDP_L4:
        hdr_len = csum_start + 8
    else:
        if len(pkt) <= csum_start + 12:
            raise SegmentError("packet is too short")
        tl = (pkt[csum_start + 12] >> 4) * 4
        if tl < 20 or tl > 60:
            raise SegmentError(f"tcp header len is invalid: {tl}")
        hdr_len = csum_start + tl
    if len(pkt) < hdr_len:
        raise SegmentError("packet shorter than header")
    if hdr_len < csum_start:
        raise SegmentError("hdr_len < csum_start")
    if csum_start + csum_offset + 1 >= len(pkt):
        raise SegmentError("checksum offset beyond packet")
    return hdr_len


def seg_count(pay_len: int, gso_size: int) -> int:
    return max(1, (pay_len + gso_size - 1) // gso_size)


def _u16(b, o):
    return (b[o] << 8) | b[o + 1]


def base_pseudo_sum(pkt, v4: bool, proto: int) -> int:
    return checksum(pkt[12:20] if v4 else pkt[8:40]) + proto


def base_ipv4_hdr_sum(pkt, csum_start: int) -> int:
    ihl = (pkt[0] & 0x0F) * 4
    if ihl < 20 or ihl > csum_start:
        raise SegmentError(f"bad IPv4 IHL: {ihl}")
    s = checksum(pkt[:ihl])
    s += (~_u16(pkt, 2)) & 0xFFFF
    s += (~_u16(pkt, 10)) & 0xFFFF
    s += (~_u16(pkt, 4)) & 0xFFFF
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return s


def base_tcp_hdr_sum(pkt, cs: int, hdr_len: int) -> int:
    seq = struct.unpack_from(">I", pkt, cs + 4)[0]
    flags = pkt[cs + 13]
    s = checksum(pkt[cs:hdr_len])
    s += (~(seq >> 16)) & 0xFFFF
    s += (~seq) & 0xFFFF
    s += (~flags) & 0xFFFF
    s += (~_u16(pkt, cs + 16)) & 0xFFFF
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return s


def segment_tcp(pkt: bytes, hdr_len: int, cs: int, gso: int):
    """Yields the segments' plaintext bytes in order (SegmentTCP)."""
    if gso == 0:
        raise SegmentError("gso_size is zero")
    if cs == 0:
        raise SegmentError("csum_start is zero")
    if hdr_len > MAX_SEG_HDR:
        raise SegmentError("header too long")
    pkt = bytes(pkt)
    v4 = pkt[0] >> 4 == 4
    tcp_hl = (pkt[cs + 12] >> 4) * 4
    pay_len = len(pkt) - hdr_len
    nseg = seg_count(pay_len, gso)
    seq0 = struct.unpack_from(">I", pkt, cs + 4)[0]
    fl0 = pkt[cs + 13]
    proto_sum = base_pseudo_sum(pkt, v4, IPPROTO_TCP)
    tcp_sum = base_tcp_hdr_sum(pkt, cs, hdr_len)
    if v4:
        id0 = _u16(pkt, 4)
        ip_sum = base_ipv4_hdr_sum(pkt, cs)
    hdr = pkt[:hdr_len]
    out = []
    for i in range(nseg):
        a = i * gso
        e = min(a + gso, pay_len)
        pl = e - a
        seg = bytearray(hdr + pkt[hdr_len + a:hdr_len + e])
        seq = (seq0 + a) & 0xFFFFFFFF
        fl = fl0
        if i != 0:
            fl &= ~0x80 & 0xFF
        if i != nseg - 1:
            fl &= ~0x09 & 0xFF
        total = hdr_len + pl
        if v4:
            sid = (id0 + i) & 0xFFFF
            struct.pack_into(">H", seg, 2, total & 0xFFFF)
            struct.pack_into(">H", seg, 4, sid)
            struct.pack_into(">H", seg, 10, fold_complement(ip_sum + total + sid))
        else:
            struct.pack_into(">H", seg, 4, (hdr_len - 40 + pl) & 0xFFFF)
        struct.pack_into(">I", seg, cs + 4, seq)
        seg[cs + 13] = fl
        tcp_len = tcp_hl + pl
        wide = tcp_sum + checksum(pkt[hdr_len + a:hdr_len + e]) + proto_sum + seq + fl + tcp_len
        wide = (wide & 0xFFFFFFFF) + (wide >> 32)
        wide = (wide & 0xFFFFFFFF) + (wide >> 32)
        struct.pack_into(">H", seg, cs + 16, fold_complement(wide))
        out.append(bytes(seg))
    return out


def segment_udp(pkt: bytes, hdr_len: int, cs: int, gso: int):
    """Yields the segments' plaintext bytes in order (SegmentUDP)."""
    if gso == 0:
        raise SegmentError("gso_size is zero")
    if cs == 0:
        raise SegmentError("csum_start is zero")
    if hdr_len > MAX_SEG_HDR:
        raise SegmentError("header too long")
    if hdr_len - cs != 8:
        raise SegmentError("udp header len mismatch")
    pkt = bytes(pkt)
    v4 = pkt[0] >> 4 == 4
    pay_len = len(pkt) - hdr_len
    nseg = seg_count(pay_len, gso)
    proto_sum = base_pseudo_sum(pkt, v4, IPPROTO_UDP)
    if v4:
        id0 = _u16(pkt, 4)
        ip_sum = base_ipv4_hdr_sum(pkt, cs)
    hdr = pkt[:hdr_len]
    out = []
    for i in range(nseg):
        a = i * gso
        e = min(a + gso, pay_len)
        pl = e - a
        seg = bytearray(hdr + pkt[hdr_len + a:hdr_len + e])
        total = hdr_len + pl
        udp_len = 8 + pl
        if v4:
            sid = (id0 + i) & 0xFFFF
            struct.pack_into(">H", seg, 2, total & 0xFFFF)
            struct.pack_into(">H", seg, 4, sid)
            struct.pack_into(">H", seg, 10, fold_complement(ip_sum + total + sid))
        else:
            struct.pack_into(">H", seg, 4, (hdr_len - 40 + pl) & 0xFFFF)
        struct.pack_into(">H", seg, cs + 4, udp_len & 0xFFFF)
        seg[cs + 6] = seg[cs + 7] = 0
        ps = proto_sum + udp_len
        ps = (ps & 0xFFFF) + (ps >> 16)
        ps = (ps & 0xFFFF) + (ps >> 16)
        c = (~checksum(seg[cs:], ps)) & 0xFFFF
        if c == 0:
            c = 0xFFFF
        struct.pack_into(">H", seg, cs + 6, c)
        out.append(bytes(seg))
    return out


def finish_checksum(seg: bytes, csum_start: int, csum_offset: int) -> bytes:
    cs, co = csum_start, csum_offset
    if cs + co + 2 > len(seg):
        raise SegmentError("csum offsets out of range")
    seg = bytearray(seg)
    partial = _u16(seg, cs + co)
    seg[cs + co] = seg[cs + co + 1] = 0
    c = (~checksum(seg[cs:], partial)) & 0xFFFF
    if co == 6 and c == 0:
        c = 0xFFFF
    struct.pack_into(">H", seg, cs + co, c)
    return bytes(seg)


def segment_superpacket(pkt: bytes, flags: int, gso_type: int, hdr_len: int, gso_size: int, csum_start: int,
                        csum_offset: int):
    """The TUN read → plaintext segments path (decodeRead, overlay/tio/tio_gso_linux.go:236-280, then
    SegmentSuperpacket): GSO_NONE → FinishChecksum when NEEDS_CSUM, one segment; otherwise
    CheckValid, CorrectHdrLen, the protocol from the GSO type, SegmentTCP / SegmentUDP."""
    g = gso_type & ~GSO_ECN
    if g == GSO_NONE:
        if flags & F_NEEDS_CSUM:
            return [finish_checksum(pkt, csum_start, csum_offset)]
        return [bytes(pkt)]
    check_valid(pkt, flags, gso_type, gso_size)
    hl = correct_hdr_len(pkt, gso_type, csum_start, csum_offset)
    if g in (GSO_TCPV4, GSO_TCPV6):
        return segment_tcp(pkt, hl, csum_start, gso_size)
    if g == GSO_UDP_L4:
        return segment_udp(pkt, hl, csum_start, gso_size)
    raise SegmentError(f"unsupported virtio gso type: {gso_type}")


REJECT_AFTER = (1 << 64) - 1 - (1 << 40)
OK, BAD_KEY, EXHAUSTED, INVALID, NO_SPACE = 0, 3, 2, 5, 6


def slot_bytes(seg_len: int) -> int:
    return (seg_len + 32 + 15) & ~15


def tx_batch(alg, tunnels, packets, out_cap, max_wires, seal, header_encode):
    """The batch as sendInsideMessage would send it, packet by packet in order (inside.go:154-240),
    laid out as the engine's TX batch returns it: wires in order, each at a 16-byte aligned slot.
    tunnels: [dict(counter, remote_index, key or None)] (counter = messageCounter before the batch);
    packets: [dict(data, tunnel, flags, gso_type, hdr_len, gso_size, csum_start, csum_offset)].
    A packet refused at read time (decodeRead) is INVALID; one whose tunnel has no key BAD_KEY; then
    segment-time errors INVALID. The output keeps its longest fitting prefix of packets; the rest
    are NO_SPACE and use no counter. Returns (wires [(off, counter, len, packet, segment, status,
    bytes)], packet statuses, final counters)."""
    ctr = [t["counter"] for t in tunnels]
    pst, plans = [], []
    for p in packets:
        g = p["gso_type"] & ~GSO_ECN
        st, segs = OK, None
        try:  # read time
            if len(p["data"]) == 0:
                raise SegmentError("short read")
            if g == GSO_NONE:
                if p["flags"] & F_NEEDS_CSUM:
                    segs = [finish_checksum(p["data"], p["csum_start"], p["csum_offset"])]
                else:
                    segs = [bytes(p["data"])]
            else:
                check_valid(p["data"], p["flags"], p["gso_type"], p["gso_size"])
                hl = correct_hdr_len(p["data"], p["gso_type"], p["csum_start"], p["csum_offset"])
                if g not in (GSO_TCPV4, GSO_TCPV6, GSO_UDP_L4):
                    raise SegmentError("unsupported gso type")
        except SegmentError:
            st = INVALID
        if st == OK and (p["tunnel"] >= len(tunnels) or tunnels[p["tunnel"]]["key"] is None):
            st = BAD_KEY
        if st == OK and segs is None:
            try:
                fn = segment_tcp if g in (GSO_TCPV4, GSO_TCPV6) else segment_udp
                segs = fn(p["data"], hl, p["csum_start"], p["gso_size"])
            except SegmentError:
                st = INVALID
        pst.append(st)
        plans.append(segs if st == OK else [])
    # fitting prefix
    nw = nb = 0
    fit = len(packets)
    for i, segs in enumerate(plans):
        nw2 = nw + len(segs)
        nb2 = nb + sum(slot_bytes(len(s)) for s in segs)
        if nw2 > max_wires or nb2 > out_cap:
            fit = i
            break
        nw, nb = nw2, nb2
    wires, off = [], 0
    for i, (p, segs) in enumerate(zip(packets, plans)):
        if i >= fit:
            if pst[i] == OK:
                pst[i] = NO_SPACE
            continue
        t = p["tunnel"]
        for j, seg in enumerate(segs):
            ctr[t] = (ctr[t] + 1) & ((1 << 64) - 1)
            c = ctr[t]
            hdr = header_encode(1, 1, 0, tunnels[t]["remote_index"], c)
            if c >= REJECT_AFTER:
                wires.append((off, c, len(seg) + 32, i, j, EXHAUSTED, None))
            else:
                wires.append((off, c, len(seg) + 32, i, j, OK, hdr + seal(alg, tunnels[t]["key"], c, hdr, seg)))
            off += slot_bytes(len(seg))
    return wires, pst, ctr
