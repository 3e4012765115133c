// sched.hpp — batch scheduling for mixed-key / mixed-size batches (shared by the AEAD kernels).
//
// A batch with many tunnel keys and mixed packet sizes is regrouped on the device before the
// crypto kernel runs: packets are binned by (size class, key) with global atomics, each key's bins
// are cut into chunks of groups of up to kChunkPkts packets, and one wavefront processes one chunk.
// Inside a chunk the key is wave-uniform (round keys in scalar registers, one set of GHASH tables)
// and the packets need a similar number of rounds, so lanes neither diverge on keys nor idle on
// sizes. No prefix scan over packets is needed: keys reserve their output ranges with an atomic
// cursor, so the order of keys (and of packets inside a bin) is arbitrary — every packet's result is
// independent of it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"

namespace neb {

constexpr uint32_t kChunkPkts = 16;   // packets per packet group at 4 lanes per packet
constexpr uint32_t kSizeClasses = 8;  // round-count classes at 4 lanes per packet: 1, 2, 3-4, 5-8, 9-16, 17-32, 33-64, 65+

// A bin of c packets becomes c / 16 full groups of 16 packets at 4 lanes per packet, packed into
// "front" chunks of up to sched_groups(cls) groups: one wave runs a chunk's groups one after another
// on one staging of the key's tables and round keys, so short packets (IMIX 90 B: 2 rounds per
// group) do not pay the staging per 16 packets. The c mod 16 others (the bin's leftover) form one
// group at 2^lg lanes per packet: lg 4 (16 lanes) for up to 4 packets, 3 for up to 8, else 2 —
// capped for short packets so that no lane idles on a block that does not exist (size class 0:
// <= 4 blocks, lg 2; class 1: <= 8 blocks, lg 3). A wave then runs a leftover of 1-4 packets in a
// quarter of the rounds instead of leaving 48-60 of its lanes idle.
// Round 6: the leftovers of one key are planned together (sched_key_chunks), largest class first,
// and a leftover group's free packet slots take the next smaller class's leftover packets: a smaller
// class needs no more rounds at the same lanes, so they ride along for free, and when a class's whole
// leftover is taken its own chunk (key staging, GHASH final, descriptor loads) is gone. A chunk is
// then up to two segments of `sorted` (its own class's, and the absorbed class's).
constexpr uint32_t kChunkLgShift = 16;  // chunk record .w: count0 | count1 << 8 | lg << 16 | front << 20 | cls << 24
__host__ __device__ inline uint32_t sched_tail_lg(uint32_t count, uint32_t cls) {
    const uint32_t fit = count <= 4u ? 4u : (count <= 8u ? 3u : 2u);
    const uint32_t size = cls == 0u ? 2u : (cls == 1u ? 3u : 4u);
    return fit < size ? fit : size;
}
// groups of 16 packets per front chunk: about 8 rounds of work per chunk for the short classes
__host__ __device__ inline uint32_t sched_groups(uint32_t cls) { return cls >= 3u ? 1u : 8u >> cls; }
constexpr uint32_t kMaxChunkPkts = 8u * kChunkPkts;
// chunk record {start of segment 0 in sorted, start of segment 1, key_id, w}
__host__ __device__ inline uint32_t chunk_w(uint32_t c0, uint32_t c1, uint32_t lg, bool front, uint32_t cls) {
    return c0 | c1 << 8 | lg << kChunkLgShift | (front ? 1u : 0u) << 20 | cls << 24;
}

// Chunks are ordered longest first (round 6): each is filed in one of kBuckets cost buckets, a
// bucket holding up to max_chunks records (the bound on the whole batch's chunks), and the crypto
// kernel enumerates bucket 0, then 1, ... Workgroup w owns chunks w, w + G, ... of that order, so
// every workgroup's waves start on the longest work and its last chunks are the shortest. The cost
// is in rounds at the class's upper bound (2^cls rounds at 4 lanes), plus one per group (its final)
// and two per leftover group at 8-16 lanes (its deeper final).
constexpr uint32_t kBuckets = 8;
__host__ __device__ inline uint32_t sched_bucket(uint32_t cost) {
    return cost >= 24u ? 0u : cost >= 16u ? 1u : cost >= 12u ? 2u : cost >= 9u ? 3u :
           cost >= 7u ? 4u : cost >= 5u ? 5u : cost >= 3u ? 6u : 7u;
}
__host__ __device__ inline uint32_t sched_front_cost(uint32_t groups, uint32_t cls) { return groups * ((1u << cls) + 1u); }
__host__ __device__ inline uint32_t sched_tail_cost(uint32_t cls, uint32_t lg) {
    const uint32_t r = (1u << cls) * 4u >> lg;
    return (r ? r : 1u) + 2u;
}

// A batch that gives each resident wave of the chunk kernel only one or two chunks balances badly
// (C5's 8-GPU shard by tunnel, 131 072 packets over 512 keys, 32 per wave: waves 0.69 busy over the
// span). Below kSmallBatchPerWave packets per wave the front chunks of the short classes hold
// kSmallBatchGroups groups at most (SchedWs::max_groups), so the waves draw smaller pieces. A/B
// (profiles/r6/ab/front_groups*.jsonl): that shard 377 -> 410 GiB/s at 1 group (402 at 2); at 64 and
// 128 packets per wave equal or slower, 1 Mi (256) 528 -> 512, so those keep sched_groups. Running
// the 576 B+ classes' full groups as two 8-lane halves as well was slower everywhere (C3 545 -> 512,
// the shard 410 -> 378).
#ifndef NEB_SMALL_BATCH_PER_WAVE
#define NEB_SMALL_BATCH_PER_WAVE 48
#endif
constexpr uint32_t kSmallBatchPerWave = NEB_SMALL_BATCH_PER_WAVE, kSmallBatchGroups = 1;

// counters[] slots
constexpr uint32_t kCntPackets = 0;  // cursor into sorted[]
constexpr uint32_t kCntBucket = 1;   // [kBuckets] chunks filed in each cost bucket
#ifndef NEB_CHUNK_STEAL  // gcm_chunk_kernel: the last 1/NEB_CHUNK_STEAL of a batch's chunks drawn per XCD (0: off)
#define NEB_CHUNK_STEAL 8
#endif
#if NEB_CHUNK_STEAL
// the chunk kernel's per-XCD cursors over the batch's last chunks, 128 B apart (gcm_chunk_kernel)
constexpr uint32_t kCntSteal = 32, kStealStride = 32;
constexpr uint32_t kSchedCounters = kCntSteal + 8 * kStealStride;
#else
constexpr uint32_t kSchedCounters = 16;
#endif
// sorted[] entry of a packet the crypto kernel must skip (the device receive's refused packets)
constexpr uint32_t kSortedSkip = 0xFFFFFFFFu;

// Each bin counts its packets in kSubBins sub-bins (sub-bin = the counting workgroup's index mod
// kSubBins), so the returning atomics of one bin's packets spread over kSubBins words: a 4096-key
// IMIX batch of 1 Mi packets put ≈ 85 adds on each word, and the memory-side atomics on one address
// run one after another (pass 1 took 56 µs).
#ifndef NEB_SUB_BINS
#define NEB_SUB_BINS 8
#endif
constexpr uint32_t kSubBins = NEB_SUB_BINS;
// batches of at least this many packets (the host's bound) count in kSubBins sub-bins, smaller ones in
// one: C3's 64 Ki packets put ≈ 16 adds on each of 4096 bins, and pass 2 then reads 1/8 of the words
#ifndef NEB_SUB_BINS_FROM
#define NEB_SUB_BINS_FROM (1u << 18)
#endif
constexpr uint32_t kSubBinsFrom = NEB_SUB_BINS_FROM;
static_assert(kSubBins == 1 || kSubBins == 2 || kSubBins == 4 || kSubBins == 8, "sub-bins: a power of two <= 8");

// Large batches bin without a global atomic per packet (round 5; the histogram pass was bound by
// the memory-side atomic rate, ≈ 23 G returning adds/s chip-wide whatever their scope or spread,
// tools/micro/xcd_atomic.hip): the batch is cut into T ≤ kTileMax tiles of ≤ 65535 packets, one
// 1024-thread workgroup per tile counts its packets per bin in LDS (two 16-bit counts per word,
// the LDS add's return is the packet's rank within the tile), a scan over the tiles gives each
// (tile, bin) its offset inside the bin and each bin its count, the allocation pass runs as for
// one sub-bin, and the scatter puts packet i at base[bin] + tile offset + rank.
constexpr uint32_t kTileMax = 128;       // tiles (workgroups of the counting pass)
constexpr uint32_t kTileMinPkts = 1024;  // packets per tile at least
constexpr uint32_t kTileThreads = 1024;
constexpr uint32_t kTileLdsMax = 152u * 1024u;  // the counting pass's LDS budget (160 KiB per CU)
#ifndef NEB_TILE_BINS_FROM
#define NEB_TILE_BINS_FROM (1u << 18)
#endif
constexpr uint32_t kTileBinsFrom = NEB_TILE_BINS_FROM;
// 16-bit counts, two per word; rows padded to 16 words (the scan takes 16 words per workgroup)
__host__ __device__ inline uint32_t sched_tile_words(uint32_t nbins) { return ((nbins + 1u) / 2u + 15u) & ~15u; }

struct SchedWs {          // device workspace, sized for n packets and nbins bins
    uint32_t* counters;   // [kSchedCounters] counters, then hist[nbins * kSubBins]
    uint32_t* hist;       // [bin * kSubBins + sub] packets counted
    uint32_t* base;       // [bin * kSubBins + sub] output offset of each non-empty sub-bin
    uint32_t* binof;      // [n] sub-bin (bin * kSubBins + sub) of each packet
    uint32_t* binpos;     // [n] rank of each packet within its bin (the histogram atomic's return)
    uint32_t* sorted;     // [n] packet indices, bin-contiguous
    uint4* chunks;        // [kBuckets][max_chunks] chunk records (chunk_w), bucket b's from b * max_chunks
    uint32_t max_chunks;  // the batch's chunks at most, and each bucket's capacity
    uint32_t max_groups = 8;  // cap on sched_groups (groups per front chunk) for this batch
    uint32_t* tcnt;       // [kTileMax][sched_tile_words] per-tile bin counts, 16 bits each (null: no tiles)
    uint32_t* tpre;       // [kTileMax][nbins] each (tile, bin)'s offset inside its bin
};

__host__ __device__ inline uint32_t sched_nbins(uint32_t max_keys) { return kSizeClasses * (max_keys + 1u); }
__host__ __device__ inline uint32_t sched_max_chunks(uint32_t n, uint32_t max_keys) {
    const uint32_t nb = sched_nbins(max_keys);
    return (n + kChunkPkts - 1u) / kChunkPkts + (n < nb ? n : nb);
}
}  // namespace neb

// Host launcher (sched.hip): the three binning passes on stream s. The workspace's counters and
// bin counts must be zero before the first batch (pass 1 clears the cursors and pass 2 the bin
// counts it reads, so a batch leaves them zero for the next).
extern "C" hipError_t neb_sched_build(const neb_desc* d_desc, uint32_t n, const uint32_t* d_n, uint32_t max_keys,
                                      uint32_t lpp, const neb::SchedWs* ws, hipStream_t s);
