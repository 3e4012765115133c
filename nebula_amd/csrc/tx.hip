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
// two end-around folds of a 32-bit partial sum (the reference's `s = s&0xffff + s>>16` twice)
__device__ __forceinline__ uint32_t fold2(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    return (s & 0xFFFFu) + (s >> 16);
}
// checksum.Checksum(p[lo:hi], 0): big-endian words paired from lo, odd tail byte high, folded
// (headers are at most 120 bytes: 8 loads in flight per step instead of one dependent load a byte)
__device__ uint32_t csum_range(const uint8_t* p, uint32_t lo, uint32_t hi) {
    uint32_t s = 0, k = lo;
    for (; k + 8u <= hi; k += 8u) {
        uint32_t b[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; q++) b[q] = p[k + q];
#pragma unroll
        for (uint32_t q = 0; q < 8; q += 2) s += (b[q] << 8) | b[q + 1];  // k - lo is even here
    }
    for (; k < hi; k++) s += ((k - lo) & 1u) ? (uint32_t)p[k] : (uint32_t)p[k] << 8;
    while (s >> 16) s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

// ---- stage 1: per-packet checks and sizes ---------------------------------------------------

struct TxParsed {
    TxPlan plan;
    int32_t st;
    uint64_t scan;  // nseg << 40 | output bytes
};

__device__ TxParsed tx_parse_one(const neb_tx_packet& P, const uint8_t* __restrict__ in,
                                 const neb_tx_tunnel* __restrict__ tun, uint32_t ntun,
                                 const uint32_t* __restrict__ keys, uint32_t max_keys, int alg) {
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
                // the constants of every segment header, from the pristine superpacket header
                const uint32_t pseudo = (v4 ? csum_range(b, 12, 20) : csum_range(b, 8, 40)) +
                                        (plan.kind == kTxTcp ? 6u : 17u);  // basePseudoSum
                if (v4) {  // baseIPv4HdrSum
                    plan.id0 = rd16be(b + 4);
                    uint32_t sum = csum_range(b, 0, (rd8(b) & 15u) * 4u);
                    sum += (~rd16be(b + 2) & 0xFFFFu) + (~rd16be(b + 10) & 0xFFFFu) + (~plan.id0 & 0xFFFFu);
                    plan.ip_base = fold2(sum);
                }
                if (plan.kind == kTxTcp) {  // baseTCPHdrSum
                    plan.seq0 = (rd16be(b + cs + 4u) << 16) | rd16be(b + cs + 6u);
                    plan.fl0 = (uint8_t)rd8(b + cs + 13u);
                    uint32_t sum = csum_range(b, cs, hl);
                    sum += (~(plan.seq0 >> 16)) & 0xFFFFu;
                    sum += (~plan.seq0) & 0xFFFFu;
                    sum += (~(uint32_t)plan.fl0) & 0xFFFFu;
                    sum += (~rd16be(b + cs + 16u)) & 0xFFFFu;
                    plan.l4_base = fold2(sum) + pseudo;
                } else {
                    plan.l4_base = pseudo;
                }
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
    return TxParsed{plan, st, ((uint64_t)plan.nseg << 40) | bytes};
}

__global__ void tx_parse_kernel(const neb_tx_packet* __restrict__ pk, uint32_t n, const uint8_t* __restrict__ in,
                                const neb_tx_tunnel* __restrict__ tun, uint32_t ntun, const uint32_t* __restrict__ keys,
                                uint32_t max_keys, int alg, TxWs ws, int32_t* __restrict__ pk_status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const neb_tx_packet P = pk[i];
    const TxParsed r = tx_parse_one(P, in, tun, ntun, keys, max_keys, alg);
    ws.plan[i] = r.plan;
    ws.scan_in[i] = r.scan;
    ws.tun_key[i] = r.st == NEB_STATUS_OK ? P.tunnel : ntun;
    ws.idx[i] = i;
    pk_status[i] = r.st;
}

// wire -> packet map of the fitting prefix, one wave per packet
__global__ void tx_segmap_kernel(uint32_t n, uint32_t max_wires, uint64_t out_cap, TxWs ws) {
    const uint32_t p = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (p >= n) return;
    const uint64_t pre = ws.scan_out[p], own = ws.scan_in[p];
    const uint64_t end_seg = (pre >> 40) + (own >> 40), end_bytes = (pre & kTxBytesMask) + (own & kTxBytesMask);
    if (end_seg > max_wires || end_bytes > out_cap) return;
    for (uint32_t k = (uint32_t)(pre >> 40) + (threadIdx.x & 63u); k < (uint32_t)end_seg; k += 64u) ws.seg_pkt[k] = p;
}

__global__ void tx_gather_kernel(uint32_t n, TxWs ws) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ws.nseg_sorted[i] = ws.plan[ws.idx_sorted[i]].nseg;
}

// Counter offsets back in batch order; the fitting prefix; per-tunnel totals; the batch totals.
__global__ void tx_scatter_kernel(uint32_t n, const neb_tx_tunnel* __restrict__ tun, uint32_t ntun, uint64_t out_cap,
                                  uint32_t max_wires, TxWs ws, int32_t* __restrict__ pk_status,
                                  uint32_t* __restrict__ d_nwires) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = ws.idx_sorted[i];
    const uint64_t pre = ws.scan_out[p], own = ws.scan_in[p];
    const uint64_t end_seg = (pre >> 40) + (own >> 40);
    const uint64_t end_bytes = (pre & kTxBytesMask) + (own & kTxBytesMask);
    const uint32_t t = ws.tun_key_sorted[i];
    // tx_finish_kernel advances the counters only after the segment kernel has run
    ws.ctr_base[p] = (t < ntun ? tun[t].message_counter : 0ull) + ws.ctr_sorted[i];
    const bool fits = end_seg <= max_wires && end_bytes <= out_cap;
    if (t < ntun) {
        if (fits) {
            // the last fitting packet of its tunnel's run (sorted by tunnel, then batch order) writes
            // the tunnel's segment total: its exclusive offset plus its own segments
            bool last = i + 1u == n || ws.tun_key_sorted[i + 1u] != t;
            if (!last) {
                const uint32_t q = ws.idx_sorted[i + 1u];
                const uint64_t e = ws.scan_out[q] + ws.scan_in[q];
                last = !((e >> 40) <= max_wires && (e & kTxBytesMask) <= out_cap);
            }
            if (last) ws.tun_total[t] = ws.ctr_sorted[i] + (own >> 40);
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

// ---- the whole plan in one workgroup (n <= kTxPlanSmallMax) ----------------------------------
//
// Same results as parse + scan + sort + scan-by-key + scatter + finish above, in one launch:
// at the batch sizes a TUN queue flush has (hundreds to a few thousand reads) those twelve launches
// cost ~60 us of which almost all is launch and drain. Thread t owns packets 8t..8t+7 (blocked, in
// batch order), so block-wide scans and a stable block radix sort by tunnel give batch-order
// prefixes and per-tunnel counters; the tunnels' counters advance here, after every read of them.
// The wire -> packet map stays a grid-wide launch (tx_segmap_kernel): 65 Ki uncoalesced 4-byte
// stores from one CU took 31 us (a merge-path split over the workgroup's threads, measured).

#ifdef NEB_TX_PLAN_PROF
#define TXPROF(x) __syncthreads(); const unsigned long long x = wall_clock64()
#else
#define TXPROF(x)
#endif

struct TxSegPair {  // segmented-sum element: head = a tunnel's run starts inside
    uint32_t head, sum;
};
struct TxSegOp {
    __device__ TxSegPair operator()(const TxSegPair& a, const TxSegPair& b) const {
        return TxSegPair{a.head | b.head, b.head ? b.sum : a.sum + b.sum};
    }
};

template <uint32_t IT, bool PARSED>
__global__ __launch_bounds__(kTxPlanThreads) void tx_plan_small_kernel(
    const neb_tx_packet* __restrict__ pk, uint32_t n, const uint8_t* __restrict__ in, neb_tx_tunnel* __restrict__ tun,
    uint32_t ntun, const uint32_t* __restrict__ keys, uint32_t max_keys, int alg, uint64_t out_cap, uint32_t max_wires,
    int key_bits, TxWs ws, int32_t* __restrict__ pk_status, uint32_t* __restrict__ d_nwires) {
    static_assert(IT <= kTxPlanItems, "the LDS arrays hold kTxPlanSmallMax reads");
    using Sort = hipcub::BlockRadixSort<uint32_t, kTxPlanThreads, IT, uint32_t>;
    using Scan64 = hipcub::BlockScan<uint64_t, kTxPlanThreads>;
    using ScanSeg = hipcub::BlockScan<TxSegPair, kTxPlanThreads>;
    using Reduce = hipcub::BlockReduce<uint32_t, kTxPlanThreads>;
    __shared__ union {
        typename Sort::TempStorage sort;
        typename Scan64::TempStorage scan;
        typename ScanSeg::TempStorage seg;
        typename Reduce::TempStorage red;
    } tmp;
    __shared__ uint32_t s_end[kTxPlanSmallMax];   // per packet: output bytes (parse -> blocked)
    __shared__ uint32_t s_nseg[kTxPlanSmallMax];  // per packet: its segments
    __shared__ uint32_t s_key[kTxPlanSmallMax];   // the sorted tunnel keys
    __shared__ uint32_t s_fit;

    const uint32_t t = threadIdx.x;
    uint64_t sc[IT];
    uint32_t key[IT], idx[IT];
    TXPROF(T0);
    // 1. parse (tx_parse_kernel), packets striped over the threads; then each thread takes its
    // blocked 8 through the LDS (the output bytes of one read fit 32 bits: at most 65535 segments of
    // at most 160 bytes)
    for (uint32_t i = t; i < n; i += kTxPlanThreads) {
        if constexpr (PARSED) {  // tx_parse_kernel ran first, grid-wide
            const uint64_t sc = ws.scan_in[i];
            s_nseg[i] = (uint32_t)(sc >> 40);
            s_end[i] = (uint32_t)(sc & kTxBytesMask);
            s_key[i] = ws.tun_key[i];
        } else {
            const neb_tx_packet P = pk[i];
            const TxParsed r = tx_parse_one(P, in, tun, ntun, keys, max_keys, alg);
            ws.plan[i] = r.plan;
            pk_status[i] = r.st;
            s_nseg[i] = r.plan.nseg;
            s_end[i] = (uint32_t)(r.scan & kTxBytesMask);
            s_key[i] = r.st == NEB_STATUS_OK ? P.tunnel : ntun;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
        const uint32_t i = t * IT + k;
        sc[k] = 0;
        key[k] = ntun;
        idx[k] = i;
        if (i < n) {
            sc[k] = ((uint64_t)s_nseg[i] << 40) | s_end[i];
            key[k] = s_key[i];
        }
    }
    __syncthreads();
    TXPROF(T1);
    // 2. batch-order exclusive prefix of (segments, bytes); the fitting prefix
    uint64_t tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) tot += sc[k];
    uint64_t pre;
    Scan64(tmp.scan).ExclusiveSum(tot, pre);
    uint32_t nfit = 0;
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
        const uint32_t i = t * IT + k;
        const uint64_t end = pre + sc[k];
        const bool fits = (end >> 40) <= max_wires && (end & kTxBytesMask) <= out_cap;
        if (i < n) {
            ws.scan_out[i] = pre;
            ws.scan_in[i] = sc[k];
            if (!fits && key[k] < ntun) pk_status[i] = NEB_STATUS_NO_SPACE;  // outside the fitting prefix
            nfit += fits;
        }
        if (!fits) key[k] = ntun;  // takes no counters
        pre = end;
    }
    __syncthreads();
    const uint32_t F = Reduce(tmp.red).Sum(nfit);  // prefixes are monotone: packets 0..F-1 fit
    if (t == 0) s_fit = F;
    __syncthreads();
    const uint32_t fit = s_fit;
    if (t == 0) {
        const uint64_t e = fit ? ws.scan_out[fit - 1u] + ws.scan_in[fit - 1u] : 0ull;
        *d_nwires = (uint32_t)(e >> 40);
        ws.totals[0] = e >> 40;
        ws.totals[1] = e & kTxBytesMask;
    }
    TXPROF(T2);
    // 3. counters: a stable sort by tunnel keeps batch order inside each tunnel's run
    __syncthreads();
    Sort(tmp.sort).Sort(key, idx, 0, key_bits);
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) s_key[t * IT + k] = key[k];
    __syncthreads();
    uint32_t val[IT], head[IT];
    TxSegPair agg{0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
        const uint32_t r = t * IT + k;
        val[k] = key[k] < ntun ? s_nseg[idx[k]] : 0u;
        head[k] = r == 0u || s_key[r - 1u] != key[k];
        agg = TxSegOp{}(agg, TxSegPair{head[k], val[k]});
    }
    TXPROF(T3);
    TxSegPair carry;
    ScanSeg(tmp.seg).ExclusiveScan(agg, carry, TxSegPair{0u, 0u}, TxSegOp{});
    uint32_t run = carry.sum;
    uint64_t newctr[IT];
    bool last[IT];
#pragma unroll
    for (uint32_t k = 0; k < IT; k++) {
        const uint32_t r = t * IT + k;
        if (head[k]) run = 0;
        last[k] = false;
        if (key[k] < ntun) {
            const uint64_t base = tun[key[k]].message_counter;
            ws.ctr_base[idx[k]] = base + run;
            last[k] = r + 1u == kTxPlanThreads * IT || s_key[r + 1u] != key[k];
            newctr[k] = base + run + val[k];
        }
        run += val[k];
    }
    TXPROF(T4);
    __syncthreads();  // every read of the old counters is done
#pragma unroll
    for (uint32_t k = 0; k < IT; k++)
        if (last[k]) tun[key[k]].message_counter = newctr[k];
    TXPROF(T5);
    TXPROF(T6);
#ifdef NEB_TX_PLAN_PROF
    __syncthreads();
    TXPROF(T7);
    if (t == 0)
        printf("txplan n=%u parse %llu prefix %llu sort %llu segscan %llu ctr %llu - %llu sync %llu (x10ns)\n", n,
               T1 - T0, T2 - T1, T3 - T2, T4 - T3, T5 - T4, T6 - T5, T7 - T6);
#endif
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
#ifndef NEB_TX_GROUP
#define NEB_TX_GROUP 16     // measured (64 KiB TSO batch): 16 lanes x 6 units 308 GiB/s, 32 x 3 303,
#define NEB_TX_REGUNITS 6  // 64 x 2 279; 6 blocks/CU (80 VGPRs) spills: 241
#define NEB_TX_MINBLOCKS 4
#endif
constexpr uint32_t kTxGroup = NEB_TX_GROUP;        // lanes per segment: 64 / kTxGroup segments per wave
constexpr uint32_t kTxRegUnits = NEB_TX_REGUNITS;  // payload units per lane kept in registers (16 x 6 x 16 B = 1.5 KiB)

__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
#pragma unroll
    for (int o = kTxGroup / 2; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, (int)kTxGroup);
    return v;
}

// CSM (the seal sums the payloads, cs_slots != 0): no payload registers, so more waves per CU
// (96 VGPRs, 5 blocks; 6 spills): the kernel is a chain of dependent loads per segment, bound by
// how many segments are in flight
#ifndef NEB_TX_CSM_BLOCKS
#define NEB_TX_CSM_BLOCKS 5
#endif
template <bool CSM>
__global__ __launch_bounds__(kTxWaves * 64, CSM ? NEB_TX_CSM_BLOCKS : NEB_TX_MINBLOCKS) void tx_segment_kernel(const neb_tx_packet* __restrict__ pk,
                                                                     const uint8_t* __restrict__ in,
                                                                     const neb_tx_tunnel* __restrict__ tun,
                                                                     uint8_t* __restrict__ out, TxWs ws,
                                                                     neb_tx_wire* __restrict__ wires,
                                                                     const uint32_t* __restrict__ d_nwires,
                                                                     uint32_t cs_slots) {
    const uint32_t g = threadIdx.x & (kTxGroup - 1u);  // lane within the segment's group
    const uint32_t nw = __builtin_amdgcn_readfirstlane(*d_nwires);
    // cs_slots != 0: the single-key seal sums the payload into the L4 checksums (aes_gcm.hip
    // gcm_csum_fix), except for the segments after its last full pass of cs_slots waves x 16
    // packets, which its tail kernel seals: those are summed here
    const uint32_t ngroups = (nw + 15u) / 16u;
    const uint32_t cs_p0 =
        cs_slots == 0u ? 0u : (ngroups > cs_slots && ngroups % cs_slots) ? ngroups / cs_slots * cs_slots * 16u : nw;
    const uint32_t groups_per_block = blockDim.x / kTxGroup;
    const uint32_t first = blockIdx.x * groups_per_block + threadIdx.x / kTxGroup;
    const uint32_t rounds = (nw + gridDim.x * groups_per_block - 1u) / (gridDim.x * groups_per_block);
    for (uint32_t r = 0; r < rounds; r++) {  // uniform trip count: every lane reaches the shuffles
        const uint32_t s = first + r * gridDim.x * groups_per_block;
        const bool live = s < nw;
        const uint32_t p = live ? ws.seg_pkt[s] : 0u;
        const uint64_t pre = live ? ws.scan_out[p] : 0u;
        const uint32_t j = s - (uint32_t)(pre >> 40);
        TxPlan plan{};
        neb_tx_packet P{};
        neb_tx_tunnel T{};
        uint64_t ctr_base = 0;
        if (live) {
            plan = ws.plan[p];
            P = pk[p];
            ctr_base = ws.ctr_base[p];
        }
        if (live) T = tun[P.tunnel];
        const uint64_t counter = ctr_base + j + 1u;
        const uint64_t slot = (pre & kTxBytesMask) + (uint64_t)j * plan.full_slot;
        const uint8_t* src = in + P.in_off;
        const uint32_t hl = plan.hdr_len, cs = P.csum_start, co = P.csum_offset;
        const bool gsok = plan.kind == kTxTcp || plan.kind == kTxUdp;
        const uint32_t a = gsok ? j * P.gso_size : 0u;
        const uint32_t pl = !live ? 0u : gsok ? min((uint32_t)P.gso_size, P.len - hl - a) : P.len;
        const uint32_t seg_len = hl + pl;
        uint8_t* dst = out + slot;
        const bool work = live && counter < kRejectAfterMessages;  // an exhausted one keeps only its header
        // the seal's checksum: the field inside one 16-B block and inside the prefix the seal reads
        // from the slot, the payload words paired like the checksum start's, e < 1024
        const uint32_t fld = gsok ? (plan.kind == kTxTcp ? cs + 16u : cs + 6u) : cs + co;
        const uint32_t hdr_b = gsok ? hl : plan.kind == kTxFinish ? cs + co + 2u : 0u;
        const bool seal_cs = work && s < cs_p0 && plan.kind != kTxPass && (fld & 15u) != 15u &&
                             ((hdr_b - cs) & 1u) == 0u && fld + 2u <= hdr_b && seg_len < 16384u;

        if (live && g == 0) {
            wires[s] = neb_tx_wire{slot, counter, seg_len + 32u, p, j, 0u};
            if constexpr (kTxSealFromInput) {
                // plaintext byte x of the segment image: x < hdr from the slot (the patched header, or
                // a plain packet up to its finished checksum), else the TUN read's byte in_off + a + x
                const uint32_t kind = (plan.kind == kTxUdp || (plan.kind == kTxFinish && co == 6u)) ? 2u : 1u;
                const uint32_t fl = seal_cs ? hdr_b | fld << 12 | kind << 24 | (cs & 1u) << 26 : hdr_b;
                const uint64_t src = (uint64_t)((uintptr_t)(in + P.in_off + a) - (uintptr_t)out);
                ws.seal_desc[s] = neb_desc{src, slot + 16u, slot, counter, seg_len, 16u, T.key_id, fl};
            } else {
                ws.seal_desc[s] = neb_desc{slot + 16u, slot + 16u, slot, counter, seg_len, 16u, T.key_id, 0u};
            }
            // header.Encode(Version 1, Message 1, subtype 0, remote index, counter)
            // store_block: `out` may start at any byte address
            store_block(dst, make_uint4(0x00000011u, bswap32(T.remote_index), bswap32((uint32_t)(counter >> 32)),
                                        bswap32((uint32_t)counter)), 16u);
        }

        // ---- the segment's L3+L4 header: dwords g and g + 16 of it (superpackets) ----
        uint32_t hw[2] = {0, 0};
        uint32_t le = 0;  // this lane's Σ of 16-bit words of the L4 checksum range, paired from its start, swapped
        uint64_t tcp_wide = 0;
        uint32_t udp_seed = 0;
        if (work && gsok) {
#pragma unroll
            for (uint32_t h = 0; h < 2; h++) {
                const uint32_t d = g + kTxGroup * h;
                if (4u * d < hl) {
                    const uint8_t* hp = src + 4u * d;
                    if (((P.in_off & 3u) == 0u) && 4u * d + 4u <= hl) {
                        hw[h] = *reinterpret_cast<const uint32_t*>(hp);
                    } else {
#pragma unroll
                        for (uint32_t k = 0; k < 4; k++)
                            if (4u * d + k < hl) hw[h] |= (uint32_t)hp[k] << (8u * k);
                    }
                }
            }
            const uint32_t total = seg_len, id = (plan.id0 + j) & 0xFFFFu;
            const uint32_t ipck = fold_complement(plan.ip_base + total + id);
            uint32_t seq = 0, fl = 0, udp_len = 8u + pl;
            if (plan.kind == kTxTcp) {
                seq = plan.seq0 + a;
                fl = plan.fl0;
                if (j != 0) fl &= ~0x80u;               // CWR only on the first segment
                if (j != plan.nseg - 1u) fl &= ~0x09u;  // FIN|PSH only on the last
                tcp_wide = (uint64_t)plan.l4_base + seq + fl + ((hl - cs) + pl);  // + the payload sum
            } else {
                udp_seed = fold2(plan.l4_base + udp_len);
            }
#pragma unroll
            for (uint32_t h = 0; h < 2; h++) {
                const uint32_t d = g + kTxGroup * h;
                uint32_t w = hw[h];
                if (plan.v4) {  // the reference's write order: total length, ID, checksum
                    w = put_be(w, d, 2, 2, total);
                    w = put_be(w, d, 4, 2, id);
                    w = put_be(w, d, 10, 2, ipck);
                } else {
                    w = put_be(w, d, 4, 2, hl - 40u + pl);
                }
                if (plan.kind == kTxTcp) {
                    w = put_be(w, d, cs + 4u, 4, seq);
                    w = put_be(w, d, cs + 13u, 1, fl);
                } else {  // UDP: length and a zeroed checksum enter the sum over seg[cs:]
                    w = put_be(w, d, cs + 4u, 2, udp_len);
                    w = put_be(w, d, cs + 6u, 2, 0u);
#pragma unroll
                    for (uint32_t k = 0; k < 4; k++) {
                        const uint32_t pos = 4u * d + k;
                        if (pos >= cs && pos < hl) le += ((pos - cs) & 1u) ? byte_at(w, k) << 8 : byte_at(w, k);
                    }
                }
                hw[h] = w;
            }
        }

        // ---- payload units: image positions hl + 16u; the L4 checksum covers [sum_lo, seg_len) ----
        // (seal_cs: a plain packet's prefix up to its checksum only; a segment's payload not at all)
        const bool need_sum = work && plan.kind != kTxPass && (!seal_cs || plan.kind == kTxFinish);
        const uint32_t sum_lo = plan.kind == kTxFinish ? cs : hl;
        const uint32_t zlo = plan.kind == kTxFinish ? cs + co : 0u, zhi = plan.kind == kTxFinish ? cs + co + 2u : 0u;
        const uint8_t* psrc = src + hl + a;
        const uint32_t nunits = !work ? 0u : seal_cs ? min((pl + 15u) >> 4, (hdr_b + 15u) >> 4) : (pl + 15u) >> 4;
        const bool in_regs = !kTxSealFromInput && nunits <= kTxGroup * kTxRegUnits;
        const bool flip = ((hl ^ sum_lo) & 1u) != 0u;  // units start at the parity of hl
        uint4 keep[kTxRegUnits];
        if (kTxSealFromInput && !CSM) {
            // the checksum only: kTxRegUnits loads in flight per lane, then their sums
            if (need_sum) {
                for (uint32_t u0 = 0; u0 < nunits; u0 += kTxGroup * kTxRegUnits) {
#pragma unroll
                    for (uint32_t k = 0; k < kTxRegUnits; k++) {
                        const uint32_t u = u0 + g + kTxGroup * k;
                        keep[k] = make_uint4(0, 0, 0, 0);
                        if (u < nunits) keep[k] = load_block(psrc + 16u * u, min(16u, pl - 16u * u));
                    }
#pragma unroll
                    for (uint32_t k = 0; k < kTxRegUnits; k++) {
                        const uint32_t u = u0 + g + kTxGroup * k;
                        if (u < nunits) {
                            uint4 v = keep[k];
                            if (plan.kind == kTxFinish) {
                                v = zero_range(v, hl + 16u * u, 0u, sum_lo);
                                v = zero_range(v, hl + 16u * u, zlo, zhi);
                                if (seal_cs) v = zero_range(v, hl + 16u * u, hdr_b, 0xFFFFFFFFu);
                            }
                            const uint32_t su = unit_le_sum(v);
                            le += flip ? bswap16(fold16(su)) : su;
                        }
                    }
                }
            }
        } else if (in_regs) {
#pragma unroll
            for (uint32_t k = 0; k < kTxRegUnits; k++) {
                const uint32_t u = g + kTxGroup * k;
                keep[k] = make_uint4(0, 0, 0, 0);
                if (u < nunits) keep[k] = load_block(psrc + 16u * u, min(16u, pl - 16u * u));
            }
            if (need_sum) {
#pragma unroll
                for (uint32_t k = 0; k < kTxRegUnits; k++) {
                    const uint32_t u = g + kTxGroup * k;
                    if (u < nunits) {
                        uint4 v = keep[k];
                        if (plan.kind == kTxFinish) {  // only FinishChecksum sums part of its units
                            v = zero_range(v, hl + 16u * u, 0u, sum_lo);
                            v = zero_range(v, hl + 16u * u, zlo, zhi);
                        }
                        const uint32_t su = unit_le_sum(v);
                        le += flip ? bswap16(fold16(su)) : su;
                    }
                }
            }
        } else if (need_sum) {
            for (uint32_t u = g; u < nunits; u += kTxGroup) {
                uint4 v = load_block(psrc + 16u * u, min(16u, pl - 16u * u));
                if (plan.kind == kTxFinish) {
                    v = zero_range(v, hl + 16u * u, 0u, sum_lo);
                    v = zero_range(v, hl + 16u * u, zlo, zhi);
                    if (seal_cs) v = zero_range(v, hl + 16u * u, hdr_b, 0xFFFFFFFFu);
                }
                const uint32_t su = unit_le_sum(v);
                le += flip ? bswap16(fold16(su)) : su;
            }
        }
        // the group total, folded and byte-swapped, is the big-endian RFC 1071 sum
        const uint32_t rel = bswap16(fold16(group_sum(le)));
        uint32_t csum = 0;
        // (seal_cs: the partial sum, not complemented, for the seal to finish)
        if (plan.kind == kTxTcp) {
            uint64_t w = tcp_wide + rel;
            w = (w & 0xFFFFFFFFull) + (w >> 32);
            w = (w & 0xFFFFFFFFull) + (w >> 32);
            csum = seal_cs ? fold16(w) : fold_complement((uint32_t)w);
        } else if (plan.kind == kTxUdp) {
            csum = seal_cs ? fold16((uint64_t)udp_seed + rel) : ~fold16((uint64_t)udp_seed + rel) & 0xFFFFu;
            if (!seal_cs && csum == 0u) csum = 0xFFFFu;  // RFC 768: a computed zero goes out as all ones
        } else if (plan.kind == kTxFinish && work) {  // seeded with the partial sum left in the field
            const uint64_t t = (uint64_t)rd16be(src + cs + co) + rel;
            csum = seal_cs ? fold16(t) : ~fold16(t) & 0xFFFFu;
            if (!seal_cs && co == 6u && csum == 0u) csum = 0xFFFFu;
        }

        // ---- store the image ----
        uint8_t* ddst = dst + 16u;
        if (work && gsok) {
#pragma unroll
            for (uint32_t h = 0; h < 2; h++) {
                const uint32_t d = g + kTxGroup * h;
                if (4u * d < hl) {
                    const uint32_t w = put_be(hw[h], d, plan.kind == kTxTcp ? cs + 16u : cs + 6u, 2, csum);
                    const uint32_t nb = min(4u, hl - 4u * d);
                    if (nb == 4u) *reinterpret_cast<uint32_t*>(ddst + 4u * d) = w;
                    else for (uint32_t k = 0; k < nb; k++) ddst[4u * d + k] = (uint8_t)(w >> (8u * k));
                }
            }
        }
        if (kTxSealFromInput) {
            // a plain packet's prefix up to its finished checksum; the seal reads the rest from the read
            if (work && plan.kind == kTxFinish) {
                const uint32_t hdr = cs + co + 2u;
                for (uint32_t u = g; 16u * u < hdr; u += kTxGroup) {
                    const uint32_t nb = min(16u, hdr - 16u * u);
                    const uint4 v = put_be_unit(load_block(psrc + 16u * u, nb), 16u * u, cs + co, csum);
                    store_block(ddst + 16u * u, v, nb);
                }
            }
        } else if (in_regs) {
#pragma unroll
            for (uint32_t k = 0; k < kTxRegUnits; k++) {
                const uint32_t u = g + kTxGroup * k;
                if (u < nunits) {
                    uint4 v = keep[k];
                    if (plan.kind == kTxFinish) v = put_be_unit(v, hl + 16u * u, cs + co, csum);
                    store_block(ddst + hl + 16u * u, v, min(16u, pl - 16u * u));
                }
            }
        } else {
            for (uint32_t u = g; u < nunits; u += kTxGroup) {
                const uint32_t nb = min(16u, pl - 16u * u);
                uint4 v = load_block(psrc + 16u * u, nb);
                if (plan.kind == kTxFinish) v = put_be_unit(v, hl + 16u * u, cs + co, csum);
                store_block(ddst + hl + 16u * u, v, nb);
            }
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

#ifndef NEB_TX_SMALL_PLAN
#define NEB_TX_SMALL_PLAN 1
#endif

extern "C" hipError_t neb_tx_plan(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                  neb_tx_tunnel* d_tun, uint32_t ntun, const uint32_t* d_keys, uint32_t max_keys,
                                  int alg, const neb::TxWs* ws, uint64_t out_cap, uint32_t max_wires,
                                  int32_t* d_pk_status, uint32_t* d_nwires, hipStream_t s) {
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= ntun) bits++;
    if (NEB_TX_SMALL_PLAN && n <= neb::kTxPlanSmallMax) {
        // Parsing is a chain of dependent header loads per read: past one read per lane of the one
        // workgroup it runs grid-wide first (1457 reads: plan 24.8 -> the two kernels below).
        const bool pre = n > neb::kTxPlanThreads;
        if (pre) {
            const uint32_t tpb = 256;
            hipLaunchKernelGGL(neb::tx_parse_kernel, dim3((n + tpb - 1) / tpb), dim3(tpb), 0, s, d_pk, n, d_in, d_tun,
                               ntun, d_keys, max_keys, alg, *ws, d_pk_status);
        }
        // the block sort and scans cost by items per thread: 2 up to 2048 reads
        auto plan = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(neb::kTxPlanThreads), 0, s, d_pk, n, d_in, d_tun, ntun, d_keys,
                               max_keys, alg, out_cap, max_wires, bits, *ws, d_pk_status, d_nwires);
        };
        if (n <= 2u * neb::kTxPlanThreads)
            pre ? plan(neb::tx_plan_small_kernel<2, true>) : plan(neb::tx_plan_small_kernel<2, false>);
        else
            plan(neb::tx_plan_small_kernel<neb::kTxPlanItems, true>);
        hipLaunchKernelGGL(neb::tx_segmap_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, max_wires, out_cap, *ws);
        return hipGetLastError();
    }
    const uint32_t tpb = 256, grid = (n + tpb - 1) / tpb;
    hipError_t e = hipMemsetAsync(ws->tun_total, 0, (size_t)ntun * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_parse_kernel, dim3(grid), dim3(tpb), 0, s, d_pk, n, d_in, d_tun, ntun, d_keys,
                       max_keys, alg, *ws, d_pk_status);
    size_t cb = ws->cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(ws->cub_tmp, cb, ws->scan_in, ws->scan_out, (int)n, s);
    if (e != hipSuccess) return e;
    cb = ws->cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(ws->cub_tmp, cb, ws->tun_key, ws->tun_key_sorted, ws->idx, ws->idx_sorted,
                                           (int)n, 0, bits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_gather_kernel, dim3(grid), dim3(tpb), 0, s, n, *ws);
    cb = ws->cub_bytes;
    e = hipcub::DeviceScan::ExclusiveSumByKey(ws->cub_tmp, cb, ws->tun_key_sorted, ws->nseg_sorted, ws->ctr_sorted,
                                              (int)n, hipcub::Equality(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::tx_scatter_kernel, dim3(grid), dim3(tpb), 0, s, n, d_tun, ntun, out_cap, max_wires, *ws,
                       d_pk_status, d_nwires);
    hipLaunchKernelGGL(neb::tx_segmap_kernel, dim3((n + 3) / 4), dim3(256), 0, s, n, max_wires, out_cap, *ws);
    return hipGetLastError();
}

extern "C" hipError_t neb_tx_segment(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                     const neb_tx_tunnel* d_tun, uint8_t* d_out, const neb::TxWs* ws,
                                     neb_tx_wire* d_wires, const uint32_t* d_nwires, uint32_t max_wires, int cu_count,
                                     uint32_t cs_slots, hipStream_t s) {
    (void)n;
    const uint32_t per_block = neb::kTxWaves * 64u / neb::kTxGroup;
    const uint32_t want = (max_wires + per_block - 1) / per_block;
#ifndef NEB_TX_SEG_CAP
#define NEB_TX_SEG_CAP 8
#endif
    const uint32_t cap = (uint32_t)cu_count * NEB_TX_SEG_CAP;
    const uint32_t grid = want < cap ? want : cap;
    if (grid == 0) return hipSuccess;
    if (cs_slots)
        hipLaunchKernelGGL(neb::tx_segment_kernel<true>, dim3(grid), dim3(neb::kTxWaves * 64), 0, s, d_pk, d_in, d_tun,
                           d_out, *ws, d_wires, d_nwires, cs_slots);
    else
        hipLaunchKernelGGL(neb::tx_segment_kernel<false>, dim3(grid), dim3(neb::kTxWaves * 64), 0, s, d_pk, d_in, d_tun,
                           d_out, *ws, d_wires, d_nwires, cs_slots);
    return hipGetLastError();
}

extern "C" hipError_t neb_tx_finish(neb_tx_tunnel* d_tun, uint32_t n, uint32_t ntun, const neb::TxWs* ws,
                                    hipStream_t s) {
    if (ntun == 0 || (NEB_TX_SMALL_PLAN && n <= neb::kTxPlanSmallMax)) return hipSuccess;  // done by the plan kernel
    hipLaunchKernelGGL(neb::tx_finish_kernel, dim3((ntun + 255) / 256), dim3(256), 0, s, d_tun, ntun, *ws);
    return hipGetLastError();
}
