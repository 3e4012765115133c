// tx.hpp — device workspace of the transmit batch (tx.hip), shared with engine.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"

namespace neb {

constexpr uint32_t kTxMaxHdr = 120;  // IPv4 max IHL 60 + TCP max data offset 60 (segment_linux.go:30-32)
constexpr uint64_t kTxBytesMask = (1ull << 40) - 1;  // scan word: segments << 40 | output bytes
// Batches of at most this many TUN reads are planned by one workgroup in one launch
// (tx_plan_small_kernel) instead of the 12-launch device-wide path.
constexpr uint32_t kTxPlanThreads = 1024, kTxPlanItems = 8;
constexpr uint32_t kTxPlanSmallMax = kTxPlanThreads * kTxPlanItems;

enum : uint8_t { kTxPass = 0, kTxFinish = 1, kTxTcp = 2, kTxUdp = 3 };

// The seal reads each segment's payload straight from its TUN read and only the patched header
// prefix from the output slot (neb_desc::flags = that prefix's length, GcmArgs::hdr_from_dst): the
// segment kernel writes headers and computes checksums but copies no payload. 0 = round-1 path
// (the segment kernel copies the whole segment image into the slot; the seal runs in place).
#ifndef NEB_TX_FUSED
#define NEB_TX_FUSED 1
#endif
constexpr int kTxSealFromInput = NEB_TX_FUSED;

struct TxPlan {          // per packet (tx_parse_kernel)
    uint32_t nseg;       // 0 = dropped
    uint32_t hdr_len;    // superpackets: the corrected L3+L4 header length
    uint32_t full_slot;  // output bytes of one full-size segment (16-aligned)
    uint8_t kind, v4, fl0, pad0;
    // per-superpacket constants of the segment headers (segment_linux.go:166-208), computed once
    uint32_t ip_base;    // baseIPv4HdrSum
    uint32_t l4_base;    // TCP: baseTCPHdrSum + basePseudoSum; UDP: basePseudoSum
    uint32_t seq0;       // TCP sequence number
    uint32_t id0;        // IPv4 ID
};

struct TxWs {
    TxPlan* plan;
    uint64_t* scan_in;   // per packet: nseg << 40 | bytes
    uint64_t* scan_out;  // exclusive prefix
    uint32_t* tun_key;   // tunnel (ntun for a dropped packet)
    uint32_t* tun_key_sorted;
    uint32_t* idx;
    uint32_t* idx_sorted;
    uint32_t* nseg_sorted;
    uint32_t* ctr_sorted;
    uint64_t* ctr_base;          // per packet: its tunnel's message counter + the segments of that tunnel
                                 // earlier in the batch (the counter of segment j is ctr_base + j + 1)
    uint32_t* seg_pkt;           // per wire: its packet
    unsigned long long* tun_total;  // per tunnel: segments in this batch
    unsigned long long* totals;     // [0] segments, [1] bytes of the fitting prefix
    neb_desc* seal_desc;         // per wire
    void* cub_tmp;
    size_t cub_bytes;
};

inline size_t tx_align(size_t x) { return (x + 255) & ~(size_t)255; }

// Carve a TxWs out of `base` (nullptr: only size it). Returns the bytes needed.
inline size_t tx_ws_layout(uint32_t n, uint32_t ntun, uint32_t max_wires, size_t cub_bytes, uint8_t* base, TxWs* ws) {
    size_t off = 0;
    auto take = [&](size_t bytes) {
        uint8_t* p = base ? base + off : nullptr;
        off += tx_align(bytes);
        return p;
    };
    TxWs w{};
    w.plan = (TxPlan*)take((size_t)n * sizeof(TxPlan));
    w.scan_in = (uint64_t*)take((size_t)n * 8);
    w.scan_out = (uint64_t*)take((size_t)n * 8);
    w.tun_key = (uint32_t*)take((size_t)n * 4);
    w.tun_key_sorted = (uint32_t*)take((size_t)n * 4);
    w.idx = (uint32_t*)take((size_t)n * 4);
    w.idx_sorted = (uint32_t*)take((size_t)n * 4);
    w.nseg_sorted = (uint32_t*)take((size_t)n * 4);
    w.ctr_sorted = (uint32_t*)take((size_t)n * 4);
    w.ctr_base = (uint64_t*)take((size_t)n * 8);
    w.tun_total = (unsigned long long*)take((size_t)(ntun ? ntun : 1) * 8);
    w.totals = (unsigned long long*)take(16);
    w.seal_desc = (neb_desc*)take((size_t)(max_wires ? max_wires : 1) * sizeof(neb_desc));
    w.seg_pkt = (uint32_t*)take((size_t)(max_wires ? max_wires : 1) * 4);
    w.cub_tmp = take(cub_bytes);
    w.cub_bytes = cub_bytes;
    if (ws) *ws = w;
    return off;
}

}  // namespace neb

extern "C" size_t neb_tx_ws_bytes(uint32_t n, uint32_t ntun, uint32_t max_wires, size_t* cub_bytes);
// Plans the batch; for n <= kTxPlanSmallMax it also advances the tunnels' message counters
// (neb_tx_finish is then a no-op to skip).
extern "C" hipError_t neb_tx_plan(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                  neb_tx_tunnel* d_tun, uint32_t ntun, const uint32_t* d_keys, uint32_t max_keys,
                                  int alg, const neb::TxWs* ws, uint64_t out_cap, uint32_t max_wires,
                                  int32_t* d_pk_status, uint32_t* d_nwires, hipStream_t s);
extern "C" hipError_t neb_tx_segment(const neb_tx_packet* d_pk, uint32_t n, const uint8_t* d_in,
                                     const neb_tx_tunnel* d_tun, uint8_t* d_out, const neb::TxWs* ws,
                                     neb_tx_wire* d_wires, const uint32_t* d_nwires, uint32_t max_wires, int cu_count,
                                     uint32_t cs_slots, hipStream_t s);
extern "C" hipError_t neb_tx_finish(neb_tx_tunnel* d_tun, uint32_t n, uint32_t ntun, const neb::TxWs* ws,
                                    hipStream_t s);
