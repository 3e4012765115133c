// tx.hip — the transmit path on the device: a batch of TUN reads (IP packets and TSO/USO
// superpackets) becomes sealed wire packets, as sendInsideMessage does packet by packet
// (inside.go:154-240). Stages, all on the engine stream:
//
//   tx_parse_kernel    one thread per packet: decodeRead's checks (overlay/tio/tio_gso_linux.go:
//                      231-280: FinishChecksum bounds for plain packets; CheckValid, CorrectHdrLen,
//                      the GSO protocol for superpackets) plus the early errors of SegmentTCP/UDP
//                      (segment_linux.go:214-250, 316-345) → segment count, corrected header length
//                      and output bytes, or a drop status.
//   prefix sums        (segments, bytes) over the batch → each packet's first wire and slot offset;
//                      a stable sort by tunnel + a scan by key → each packet's first counter within its
//                      tunnel (counters follow batch order per tunnel, inside.go:127). A batch that
//                      overflows the output keeps its longest fitting prefix.
//   tx_segment_kernel  one wave per segment: the per-segment header (segment_linux.go:252-304 TCP,
//                      :347-393 UDP: lengths, IPv4 ID and checksum, seq, CWR/FIN/PSH, L4 checksum
//                      over the payload chunk) or FinishChecksum (:400-423) for a plain packet, copied
//                      with its payload into a 16-byte aligned slot behind header.Encode(Message,
//                      remote index, counter) (header/header.go:102-110); the seal descriptor.
//   seal               the AES-GCM / ChaCha20-Poly1305 batch kernels, in place, with the segment
//                      count read on the device.
//   tx_finish_kernel   tunnels' message counters advance by their segments in this batch.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "../../include/nebula_aead.h"
#include "device_common.hpp"
#include "layout.hpp"
#include "tx.hpp"

namespace neb {

__device__ __forceinline__ uint32_t rd8(const uint8_t* p) { return p[0]; }
__device__ __forceinline__ uint32_t rd16be(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

// ---- stage 1: per-packet checks and sizes ---------------------------------------------------

__global__ void tx_parse_kernel(const neb_tx_packet* __restrict__ pk, uint32_t n, const uint8_t* __restrict__ in,
                                const neb_tx_tunnel* __restrict__ tun, uint32_t ntun, const uint32_t* __restrict__ keys,
                                uint32_t max_keys, int alg, TxWs ws, int32_t* __restrict__ pk_status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const neb_tx_packet P = pk[i];
    TxPlan plan{};
    int32_t st = NEB_STATUS_OK;
    const uint8_t* b = in + P.in_off;
    const uint32_t len = P.len, cs = P.csum_start, co = P.csum_offset, gso = P.gso_size;
    const uint32_t g = P.gso_type & ~(uint32_t)NEB_GSO_ECN;
    uint32_t hl = 0, ver = 0;
    // 1. read time (decodeRead): the virtio header and what it points at
    if (len == 0) {
        st = NEB_STATUS_INVALID;  // "short tun read"
    } else if (g == NEB_GSO_NONE) {
        plan.kind = (P.vnet_flags & NEB_VNET_F_NEEDS_CSUM) ? kTxFinish : kTxPass;
        if (plan.kind == kTxFinish && cs + co + 2u > len) st = NEB_STATUS_INVALID;  // FinishChecksum
    } else {
        ver = rd8(b) >> 4;  // CheckValid
        if (P.vnet_flags & NEB_VNET_F_RSC_INFO) st = NEB_STATUS_INVALID;
        else if (len < 20u || (ver == 6u && len < 40u)) st = NEB_STATUS_INVALID;
        else if (gso == 0u) st = NEB_STATUS_INVALID;
        else if ((P.gso_type & NEB_GSO_ECN) && g != NEB_GSO_TCPV4 && g != NEB_GSO_TCPV6) st = NEB_STATUS_INVALID;
        else if (g == NEB_GSO_TCPV4 && ver != 4u) st = NEB_STATUS_INVALID;
        else if (g == NEB_GSO_TCPV6 && ver != 6u) st = NEB_STATUS_INVALID;
        else if (ver != 4u && ver != 6u) st = NEB_STATUS_INVALID;
        if (st == NEB_STATUS_OK) {  // CorrectHdrLen
            if (g == NEB_GSO_UDP_L4) {
                hl = cs + 8u;
            } else if (len <= cs + 12u) {
                st = NEB_STATUS_INVALID;
            } else {
                const uint32_t thl = (rd8(b + cs + 12u) >> 4) * 4u;
                if (thl < 20u || thl > 60u) st = NEB_STATUS_INVALID;
                hl = cs + thl;
            }
        }
        if (st == NEB_STATUS_OK && (len < hl || hl < cs || cs + co + 1u >= len)) st = NEB_STATUS_INVALID;
        if (st == NEB_STATUS_OK) {  // protoFromGSOType
            if (g == NEB_GSO_TCPV4 || g == NEB_GSO_TCPV6) plan.kind = kTxTcp;
            else if (g == NEB_GSO_UDP_L4) plan.kind = kTxUdp;
            else st = NEB_STATUS_INVALID;
        }
    }
    // 2. the tunnel has no eKey: sendInsideMessage returns before segmenting (inside.go:155-158)
    if (st == NEB_STATUS_OK) {
        if (P.tunnel >= ntun) {
            st = NEB_STATUS_BAD_KEY;
        } else {
            const uint32_t key = tun[P.tunnel].key_id;
            if (key >= max_keys || keys[(size_t)key * kKeyRecDwords + kRecAlg] != (uint32_t)alg) st = NEB_STATUS_BAD_KEY;
        }
    }
    // 3. segment time: SegmentTCP/UDP's early errors and baseIPv4HdrSum's IHL bound
    if (st == NEB_STATUS_OK) {
        if (plan.kind == kTxPass || plan.kind == kTxFinish) {
            plan.nseg = 1;
            plan.hdr_len = 0;
            plan.full_slot = align16(len + 32u);
        } else {
            const bool v4 = ver == 4u;
            if (cs == 0u || hl > kTxMaxHdr) st = NEB_STATUS_INVALID;
            if (st == NEB_STATUS_OK && v4) {
                const uint32_t ihl = (rd8(b) & 15u) * 4u;
                if (ihl < 20u || ihl > cs) st = NEB_STATUS_INVALID;
            }
            if (st == NEB_STATUS_OK) {
                const uint32_t pay = len - hl;
                plan.nseg = pay ? (pay + gso - 1u) / gso : 1u;
                plan.hdr_len = hl;
                plan.v4 = v4;
                plan.full_slot = align16(hl + gso + 32u);
            }
        }
    }
    uint64_t bytes = 0;
    if (st == NEB_STATUS_OK) {
        if (plan.kind == kTxPass || plan.kind == kTxFinish) {
            bytes = plan.full_slot;
        } else {
            const uint32_t pay = len - plan.hdr_len;
            const uint32_t last = pay - (plan.nseg - 1u) * gso;
            bytes = (uint64_t)(plan.nseg - 1u) * plan.full_slot + align16(plan.hdr_len + last + 32u);
        }
    } else {
        plan.nseg = 0;
    }
    ws.plan[i] = plan;
    ws.scan_in[i] = ((uint64_t)plan.nseg << 40) | bytes;
    ws.tun_key[i] = st == NEB_STATUS_OK ? P.tunnel : ntun;
    ws.idx[i] = i;
    pk_status[i] = st;
}

__global__ void tx_gather_kernel(uint32_t n, TxWs ws) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ws.nseg_sorted[i] = ws.plan[ws.idx_sorted[i]].nseg;
}

// Counter offsets back in batch order; the fitting prefix; per-tunnel totals; the batch totals.
__global__ void tx_scatter_kernel(uint32_t n, uint32_t ntun, uint64_t out_cap, uint32_t max_wires, TxWs ws,
                                  int32_t* __restrict__ pk_status, uint32_t* __restrict__ d_nwires) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = ws.idx_sorted[i];
    ws.ctr_off[p] = ws.ctr_sorted[i];
    const uint64_t pre = ws.scan_out[p], own = ws.scan_in[p];
    const uint64_t end_seg = (pre >> 40) + (own >> 40);
    const uint64_t end_bytes = (pre & kTxBytesMask) + (own & kTxBytesMask);
    const uint32_t t = ws.tun_key[p];
    if (t < ntun) {
        if (end_seg <= max_wires && end_bytes <= out_cap) {
            atomicAdd(&ws.tun_total[t], (unsigned long long)(own >> 40));
        } else {
            pk_status[p] = NEB_STATUS_NO_SPACE;  // outside the fitting prefix
        }
    }
    if (p == n - 1u) {
        // segments of the fitting prefix: the last packet whose end fits (prefixes are monotone)
        const uint64_t tot_seg = end_seg, tot_bytes = end_bytes;
        uint64_t seg = tot_seg, byt = tot_bytes;
        if (tot_seg > max_wires || tot_bytes > out_cap) {
            // binary search for the fitting prefix (packets are in batch order in scan_out)
            uint32_t lo = 0, hi = n;  // first packet that does not fit
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                const uint64_t e = ws.scan_out[m] + ws.scan_in[m];
                if ((e >> 40) <= max_wires && (e & kTxBytesMask) <= out_cap) lo = m + 1;
                else hi = m;
            }
            const uint64_t e = lo ? ws.scan_out[lo - 1] + ws.scan_in[lo - 1] : 0;
            seg = e >> 40;
            byt = e & kTxBytesMask;
        }
        *d_nwires = (uint32_t)seg;
        ws.totals[0] = seg;
        ws.totals[1] = byt;
    }
}

// ---- stage 3: one wave per segment ----------------------------------------------------------

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}
__device__ __forceinline__ uint32_t fold16(uint64_t s) {
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return (uint32_t)s;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
__device__ __forceinline__ uint32_t fold_complement(uint32_t s) {  // segment_linux.go:425-431
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return ~s & 0xFFFFu;
}

// Byte j (0..3) of a little-endian dword; set it.
__device__ __forceinline__ uint32_t byte_at(uint32_t w, uint32_t j) { return (w >> (8u * j)) & 0xFFu; }
__device__ __forceinline__ uint32_t set_byte(uint32_t w, uint32_t j, uint32_t v) {
    return (w & ~(0xFFu << (8u * j))) | ((v & 0xFFu) << (8u * j));
}

// This lane's dword of a header image covers bytes [4l, 4l+4): write the big-endian field
// [off, off+nbytes) = val where it overlaps.
__device__ __forceinline__ uint32_t put_be(uint32_t w, uint32_t lane, uint32_t off, uint32_t nbytes, uint32_t val) {
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t k = 4u * lane + j;
        if (k >= off && k < off + nbytes) w = set_byte(w, j, val >> (8u * (off + nbytes - 1u - k)));
    }
    return w;
}

// RFC 1071 contribution of this lane's 4 header bytes to checksum(hdr[lo:hi]) (pairing from lo).
__device__ __forceinline__ uint32_t lane_sum(uint32_t w, uint32_t lane, uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t k = 4u * lane + j;
        if (k >= lo && k < hi) s += ((k - lo) & 1u) ? byte_at(w, j) : byte_at(w, j) << 8;
    }
    return s;
}

// Σ of 16-bit little-endian words of a 16-byte unit (pairing from the unit start).
__device__ __forceinline__ uint32_t unit_le_sum(uint4 v) {
    return (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) + (v.z & 0xFFFFu) + (v.z >> 16) +
           (v.w & 0xFFFFu) + (v.w >> 16);
}
// zero bytes [lo, hi) of a unit whose first byte is at position `base`
__device__ __forceinline__ uint4 zero_range(uint4 v, uint32_t base, uint32_t lo, uint32_t hi) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
        const uint32_t k = base + j;
        if (k >= lo && k < hi) w[j >> 2] &= ~(0xFFu << (8u * (j & 3u)));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ uint4 put_be_unit(uint4 v, uint32_t base, uint32_t off, uint32_t val16) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
        const uint32_t k = base + j;
        if (k == off) w[j >> 2] = set_byte(w[j >> 2], j & 3u, val16 >> 8);
        if (k == off + 1u) w[j >> 2] = set_byte(w[j >> 2], j & 3u, val16);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

constexpr int kTxWaves = 4;

__global__ __launch_bounds__(kTxWaves * 64) void tx_segment_kernel(const neb_tx_packet* __restrict__ pk, uint32_t n,
                                                                     const uint8_t* __restrict__ in,
                                                                     const neb_tx_tunnel* __restrict__ tun,
                                                                     uint8_t* __restrict__ out, TxWs ws,
                                                                     neb_tx_wire* __restrict__ wires,
                                                                     const uint32_t* __restrict__ d_nwires) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = __builtin_amdgcn_readfirstlane(*d_nwires);
    for (uint32_t s = blockIdx.x * kTxWaves + (threadIdx.x >> 6); s < nw; s += gridDim.x * kTxWaves) {
        // packet of segment s: the last packet whose first segment index is <= s
        uint32_t lo = 0, hi = n;
        while (hi - lo > 1u) {
            const uint32_t m = (lo + hi) >> 1;
            if ((ws.scan_out[m] >> 40) <= s) lo = m;
            else hi = m;
        }
        const uint32_t p = lo;
        const uint64_t pre = ws.scan_out[p];
        const uint32_t j = s - (uint32_t)(pre >> 40);
        const TxPlan plan = ws.plan[p];
        const neb_tx_packet P = pk[p];
        const neb_tx_tunnel T = tun[P.tunnel];
        const uint64_t counter = T.message_counter + ws.ctr_off[p] + j + 1u;
        const uint64_t slot = (pre & kTxBytesMask) + (uint64_t)j * plan.full_slot;
        const uint8_t* src = in + P.in_off;
        const uint32_t hl = plan.hdr_len, cs = P.csum_start, co = P.csum_offset;
        const bool gsok = plan.kind == kTxTcp || plan.kind == kTxUdp;
        const uint32_t a = gsok ? j * P.gso_size : 0u;
        const uint32_t pl = gsok ? min((uint32_t)P.gso_size, P.len - hl - a) : P.len;
        const uint32_t seg_len = hl + pl;
        uint8_t* dst = out + slot;

        if (lane == 0) {
            wires[s] = neb_tx_wire{slot, counter, seg_len + 32u, p, j, 0u};
            ws.seal_desc[s] = neb_desc{slot + 16u, slot + 16u, slot, counter, seg_len, 16u, T.key_id, 0u};
            // header.Encode(Version 1, Message 1, subtype 0, remote index, counter)
            const uint32_t ri = T.remote_index;
            *reinterpret_cast<uint4*>(dst) = make_uint4(0x00000011u, bswap32(ri), bswap32((uint32_t)(counter >> 32)),
                                                        bswap32((uint32_t)counter));
        }
        if (counter >= kRejectAfterMessages) continue;  // sendInsideEncrypt drops it; nothing but the header

        // ---- header image (superpacket segments) ----
        uint32_t hw = 0;  // this lane's dword of the segment's L3+L4 header
        uint32_t l4_seed = 0;
        uint64_t tcp_wide = 0;
        if (gsok) {
            uint32_t h0 = 0;  // pristine header bytes [4 lane, 4 lane + 4)
            if (4u * lane < hl) {
#pragma unroll
                for (uint32_t k = 0; k < 4; k++)
                    if (4u * lane + k < hl) h0 |= (uint32_t)src[4u * lane + k] << (8u * k);
            }
            auto hb = [&](uint32_t pos) { return byte_at((uint32_t)__shfl((int)h0, (int)(pos >> 2)), pos & 3u); };
            const bool v4 = plan.v4;
            const bool tcp = plan.kind == kTxTcp;
            // base sums over the pristine header (segment_linux.go:166-208)
            const uint32_t pseudo =
                fold16(wave_sum(v4 ? lane_sum(h0, lane, 12, 20) : lane_sum(h0, lane, 8, 40))) + (tcp ? 6u : 17u);
            uint32_t ip_base = 0, id0 = 0;
            if (v4) {
                const uint32_t ihl = (hb(0) & 15u) * 4u;
                uint32_t sum = fold16(wave_sum(lane_sum(h0, lane, 0, ihl)));
                id0 = (hb(4) << 8) | hb(5);
                sum += (~((hb(2) << 8) | hb(3)) & 0xFFFFu) + (~((hb(10) << 8) | hb(11)) & 0xFFFFu) + (~id0 & 0xFFFFu);
                sum = (sum & 0xFFFFu) + (sum >> 16);
                sum = (sum & 0xFFFFu) + (sum >> 16);
                ip_base = sum;
            }
            uint32_t tcp_base = 0, seq0 = 0, fl0 = 0;
            if (tcp) {
                seq0 = (hb(cs + 4u) << 24) | (hb(cs + 5u) << 16) | (hb(cs + 6u) << 8) | hb(cs + 7u);
                fl0 = hb(cs + 13u);
                const uint32_t ck0 = (hb(cs + 16u) << 8) | hb(cs + 17u);
                uint32_t sum = fold16(wave_sum(lane_sum(h0, lane, cs, hl)));
                sum += (~(seq0 >> 16)) & 0xFFFFu;
                sum += (~seq0) & 0xFFFFu;
                sum += (~fl0) & 0xFFFFu;
                sum += (~ck0) & 0xFFFFu;
                sum = (sum & 0xFFFFu) + (sum >> 16);
                sum = (sum & 0xFFFFu) + (sum >> 16);
                tcp_base = sum;
            }
            // the per-segment fields, in the reference's write order
            hw = h0;
            if (v4) {
                const uint32_t total = seg_len, id = (id0 + j) & 0xFFFFu;
                hw = put_be(hw, lane, 2, 2, total);
                hw = put_be(hw, lane, 4, 2, id);
                hw = put_be(hw, lane, 10, 2, fold_complement(ip_base + total + id));
            } else {
                hw = put_be(hw, lane, 4, 2, hl - 40u + pl);
            }
            if (tcp) {
                const uint32_t seq = seq0 + a;
                uint32_t fl = fl0;
                if (j != 0) fl &= ~0x80u;               // CWR only on the first segment
                if (j != plan.nseg - 1u) fl &= ~0x09u;  // FIN|PSH only on the last
                hw = put_be(hw, lane, cs + 4u, 4, seq);
                hw = put_be(hw, lane, cs + 13u, 1, fl);
                tcp_wide = (uint64_t)tcp_base + pseudo + seq + fl + ((hl - cs) + pl);  // + the payload sum
            } else {  // UDP: length, checksum zeroed, then ~checksum(seg[cs:], pseudo + udp length)
                const uint32_t udp_len = 8u + pl;
                hw = put_be(hw, lane, cs + 4u, 2, udp_len);
                hw = put_be(hw, lane, cs + 6u, 2, 0u);
                uint32_t ps = pseudo + udp_len;
                ps = (ps & 0xFFFFu) + (ps >> 16);
                ps = (ps & 0xFFFFu) + (ps >> 16);
                l4_seed = ps + fold16(wave_sum(lane_sum(hw, lane, cs, hl)));
            }
        }

        // ---- pass 1: the checksum over the payload units ----
        // image positions hl + 16u; the sum runs over [sum_lo, seg_len) with bytes [zlo, zhi) as zero
        const bool need_sum = plan.kind != kTxPass;
        const uint32_t sum_lo = plan.kind == kTxFinish ? cs : hl;
        const uint32_t zlo = plan.kind == kTxFinish ? cs + co : 0u, zhi = plan.kind == kTxFinish ? cs + co + 2u : 0u;
        const uint8_t* psrc = src + hl + a;
        uint32_t partial = 0;
        if (plan.kind == kTxFinish) partial = rd16be(src + cs + co);
        uint32_t csum = 0;
        if (need_sum) {
            uint32_t acc = 0;
            for (uint32_t u = lane; 16u * u < pl; u += 64u) {
                const uint32_t base = hl + 16u * u;
                uint4 v = load_block(psrc + 16u * u, min(16u, pl - 16u * u));
                v = zero_range(v, base, 0u, sum_lo);
                if (zhi) v = zero_range(v, base, zlo, zhi);
                acc += unit_le_sum(v);
            }
            const uint32_t le = fold16(wave_sum(acc));
            // pairing from sum_lo: unit starts have the parity of hl
            const uint32_t rel = ((hl ^ sum_lo) & 1u) ? le : bswap16(le);
            if (plan.kind == kTxTcp) {
                uint64_t w = tcp_wide + rel;
                w = (w & 0xFFFFFFFFull) + (w >> 32);
                w = (w & 0xFFFFFFFFull) + (w >> 32);
                csum = fold_complement((uint32_t)w);
            } else if (plan.kind == kTxUdp) {
                csum = ~fold16((uint64_t)l4_seed + rel) & 0xFFFFu;
                if (csum == 0u) csum = 0xFFFFu;  // RFC 768: a computed zero goes out as all ones
            } else {  // FinishChecksum
                csum = ~fold16((uint64_t)partial + rel) & 0xFFFFu;
                if (co == 6u && csum == 0u) csum = 0xFFFFu;
            }
        }

        // ---- pass 2: store the image ----
        uint8_t* ddst = dst + 16u;
        if (gsok && 4u * lane < hl) {
            hw = put_be(hw, lane, plan.kind == kTxTcp ? cs + 16u : cs + 6u, 2, csum);
            const uint32_t nb = min(4u, hl - 4u * lane);
            if (nb == 4u) *reinterpret_cast<uint32_t*>(ddst + 4u * lane) = hw;
            else for (uint32_t k = 0; k < nb; k++) ddst[4u * lane + k] = (uint8_t)(hw >> (8u * k));
        }
        for (uint32_t u = lane; 16u * u < pl; u += 64u) {
            const uint32_t base = hl + 16u * u;
            const uint32_t nb = min(16u, pl - 16u * u);
            uint4 v = load_block(psrc + 16u * u, nb);
            if (plan.kind == kTxFinish) v = put_be_unit(v, base, cs + co, csum);
            store_block(ddst + base, v, nb);
        }
    }
}

__global__ void tx_finish_kernel(neb_tx_tunnel* __restrict__ tun, uint32_t ntun, TxWs ws) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ntun) tun[t].message_counter += ws.tun_total[t];
}

}  // namespace neb

// ------------------------------------------------------------------------------------------
// Host-side launchers (engine.cpp owns the workspace and the seal launch)

extern "C" size_t neb_tx_ws_bytes(uint32_t n, uint32_t ntun, uint32_t max_wires, size_t* cub_bytes) {
    size_t c1 = 0, c2 = 0, c3 = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, c1, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n);
    hipcub::DeviceRadixSort::SortPairs(nullptr, c2, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    hipcub::DeviceScan::ExclusiveSumByKey(nullptr, c3, (const uint32_t*)nullptr, (const uint32_t*)nullptr,
                                          (uint32_t*)nullptr, (int)n);
    *cub_bytes = std::max(c1, std::max(c2, c3));
    return neb::tx_ws_layout(n, ntun, max_wires, *cub_bytes, nullptr, nullptr);
}

extern "C" hipError_t neb_tx_plan(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                  const neb_tx_tunnel* d_tun, uint32_t ntun, const uint32_t* d_keys, uint32_t max_keys,
                                  int alg, const neb::TxWs* ws, uint64_t out_cap, uint32_t max_wires,
                                  int32_t* d_pk_status, uint32_t* d_nwires, hipStream_t s) {
    const uint32_t tpb = 256, grid = (n + tpb - 1) / tpb;
    hipError_t e = hipMemsetAsync(ws->tun_total, 0, (size_t)ntun * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_parse_kernel, dim3(grid), dim3(tpb), 0, s, d_pk, n, d_in, d_tun, ntun, d_keys,
                       max_keys, alg, *ws, d_pk_status);
    size_t cb = ws->cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(ws->cub_tmp, cb, ws->scan_in, ws->scan_out, (int)n, s);
    if (e != hipSuccess) return e;
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= ntun) bits++;
    cb = ws->cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(ws->cub_tmp, cb, ws->tun_key, ws->tun_key_sorted, ws->idx, ws->idx_sorted,
                                           (int)n, 0, bits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_gather_kernel, dim3(grid), dim3(tpb), 0, s, n, *ws);
    cb = ws->cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSumByKey(ws->cub_tmp, cb, ws->tun_key_sorted, ws->nseg_sorted, ws->ctr_sorted,
                                              (int)n, hipcub::Equality(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_scatter_kernel, dim3(grid), dim3(tpb), 0, s, n, ntun, out_cap, max_wires, *ws,
                       d_pk_status, d_nwires);
    return hipGetLastError();
}

extern "C" hipError_t neb_tx_segment(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                     const neb_tx_tunnel* d_tun, uint8_t* d_out, const neb::TxWs* ws,
                                     neb_tx_wire* d_wires, const uint32_t* d_nwires, uint32_t max_wires, int cu_count,
                                     hipStream_t s) {
    const uint32_t want = (max_wires + neb::kTxWaves - 1) / neb::kTxWaves;
    const uint32_t cap = (uint32_t)cu_count * 8u;
    const uint32_t grid = want < cap ? want : cap;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::tx_segment_kernel, dim3(grid), dim3(neb::kTxWaves * 64), 0, s, d_pk, n, d_in, d_tun, d_out,
                       *ws, d_wires, d_nwires);
    return hipGetLastError();
}

extern "C" hipError_t neb_tx_finish(neb_tx_tunnel* d_tun, uint32_t ntun, const neb::TxWs* ws, hipStream_t s) {
    if (ntun == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::tx_finish_kernel, dim3((ntun + 255) / 256), dim3(256), 0, s, d_tun, ntun, *ws);
    return hipGetLastError();
}
