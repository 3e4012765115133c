// sched_body.hpp — the device bodies of the mixed-key binning passes (sched.hpp): the stand-alone
// launches in sched.hip, and the device receive's plan (rxwin.hip), which runs them as extra
// workgroups of its own launches.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <hipcub/hipcub.hpp>

#include "sched.hpp"

namespace neb {

__device__ __forceinline__ uint32_t size_class(const neb_desc& d, uint32_t lpp) {
    const uint32_t n = ((d.aad_len + 15u) >> 4) + ((d.len + 15u) >> 4) + 1u;  // GHASH / Poly1305 blocks
    const uint32_t R = (n + lpp - 1u) / lpp;
    const uint32_t c = R <= 1u ? 0u : 32u - (uint32_t)__builtin_clz(R - 1u);
    return c < kSizeClasses ? c : kSizeClasses - 1u;
}

// pass 1: histogram of (size class, key) bins; keys outside the table go to key index max_keys.
// The returning add also ranks the packet inside its bin, so pass 3 needs no atomics: the adds
// execute at the memory side (MI355X_MICROARCH.md, global atomics), ≈55 µs per 1 Mi packets each.
// SUB: sub-bins per bin for this batch (kSubBins for large batches, 1 for small ones: the contention
// the sub-bins spread is a large batch's, and pass 2 reads SUB words per bin).
// One round of 256 packets from i0 (workgroup blk, 256 threads); every lane of a wave runs it (the
// shuffles), valid lanes are a prefix. Neighbouring lanes in the same bin (a batch already grouped
// by key, e.g. a receive batch in its windows' order) add their count once: the run's first lane
// adds the run's length and hands each lane its rank (one returning atomic per run instead of one
// per packet on the same word).
template <uint32_t SUB>
__device__ __forceinline__ void sched_hist_round(const neb_desc* __restrict__ desc, uint32_t n, uint32_t max_keys,
                                                 uint32_t lpp, const SchedWs& ws, uint32_t i0, uint32_t blk) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t upto = lane == 63u ? ~0ull : (2ull << lane) - 1u;  // lanes <= this one
    const uint32_t i = i0 + threadIdx.x;
    const bool valid = i < n;
    uint32_t b = 0xFFFFFFFFu;
    if (valid) {
        const neb_desc d = desc[i];
        const uint32_t key = d.key_id < max_keys ? d.key_id : max_keys;
        b = (size_class(d, lpp) * (max_keys + 1u) + key) * SUB + (blk & (SUB - 1u));
    }
    const uint32_t pb = (uint32_t)__shfl_up((int)b, 1);
    const bool head = valid && (lane == 0u || pb != b);
    const uint64_t hm = __ballot(head);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
    const uint32_t hl = 63u - (uint32_t)__builtin_clzll((hm & upto) | 1ull);  // this lane's run head
    const uint64_t after = hm & ~upto;
    const uint32_t next = after ? (uint32_t)__builtin_ctzll(after) : nvalid;  // the next run's head
    uint32_t base = 0;
    if (head) base = atomicAdd(&ws.hist[b], next - lane);
    base = (uint32_t)__shfl((int)base, (int)hl);
    if (valid) {
        ws.binof[i] = b;
        ws.binpos[i] = base + (lane - hl);
    }
}

// the cursors are cleared by the first workgroup of pass 1 (the previous batch's crypto kernel has
// finished with them); the bin counts were cleared by the previous batch's pass 2 as it read them
__device__ __forceinline__ void sched_clear_cursors(const SchedWs& ws) {
    for (uint32_t i = threadIdx.x; i < kSchedCounters; i += blockDim.x) ws.counters[i] = 0;
}

// pass 2: every non-empty bin reserves its range of `sorted` and its chunks. The reservations are
// aggregated per workgroup (block scans, then one atomic per counter and workgroup): one atomic per
// bin put ~4096 returning atomics on a single word for a 4096-tunnel batch. blk: this workgroup's
// index among the pass's (the grid covers the bins exactly once, kAllocThreads threads each).
constexpr int kAllocThreads = 256;
template <uint32_t SUB>
struct SchedAllocLds {
    typename hipcub::BlockScan<uint32_t, kAllocThreads>::TempStorage tmp;
    uint32_t wg_base[4];
};
template <uint32_t SUB>
__device__ __forceinline__ void sched_alloc_block(uint32_t max_keys, const SchedWs& ws, uint32_t blk,
                                                  SchedAllocLds<SUB>& sl) {
    using Scan = hipcub::BlockScan<uint32_t, kAllocThreads>;
    const uint32_t nb = sched_nbins(max_keys);
    const uint32_t b = blk * kAllocThreads + threadIdx.x;
    uint32_t sc[SUB], c = 0;
#pragma unroll
    for (uint32_t j = 0; j < SUB; j++) {
        sc[j] = b < nb ? ws.hist[b * SUB + j] : 0u;
        c += sc[j];
    }
    if (c)  // clear for the next batch
#pragma unroll
        for (uint32_t j = 0; j < SUB; j++) ws.hist[b * SUB + j] = 0u;
    const uint32_t key = b % (max_keys + 1u), cls = b / (max_keys + 1u);
    const uint32_t nfull = c / kChunkPkts, tail = c % kChunkPkts;
    const uint32_t lg = tail ? sched_tail_lg(tail, cls) : 2u;
    // the bin's first `fpk` packets run in groups at 4 lanes per packet (a 9-15 packet tail is a
    // partial group), packed sched_groups(cls) groups to a front chunk; a tail at 8 or 16 lanes is
    // one back chunk. The crypto kernels take the front chunks, then the back ones. Front <= n/16 +
    // bins, back <= bins and front + back <= n/16 + min(n, bins): the ranges never meet inside
    // max_chunks (sched_max_chunks).
    const uint32_t fpk = nfull * kChunkPkts + (tail && lg == 2u ? tail : 0u);
    const uint32_t cpk = sched_groups(cls) * kChunkPkts;  // packets per front chunk
    const uint32_t nfront = (fpk + cpk - 1u) / cpk;
    const bool back = tail && lg != 2u;
    const bool is_long = back && sched_tail_long(cls, lg);
    const uint32_t nlong = is_long ? 1u : 0u, nshort = back && !is_long ? 1u : 0u;
    uint32_t off_p, off_f, off_l, off_s, tot_p, tot_f, tot_l, tot_s;
    Scan(sl.tmp).ExclusiveSum(c, off_p, tot_p);
    __syncthreads();
    Scan(sl.tmp).ExclusiveSum(nfront, off_f, tot_f);
    __syncthreads();
    Scan(sl.tmp).ExclusiveSum(nlong, off_l, tot_l);
    __syncthreads();
    Scan(sl.tmp).ExclusiveSum(nshort, off_s, tot_s);
    if (threadIdx.x == 0) {
        sl.wg_base[0] = tot_p ? atomicAdd(&ws.counters[kCntPackets], tot_p) : 0u;
        sl.wg_base[1] = tot_f ? atomicAdd(&ws.counters[kCntFrontChunks], tot_f) : 0u;
        sl.wg_base[2] = tot_l ? atomicAdd(&ws.counters[kCntBackChunks], tot_l) : 0u;
        sl.wg_base[3] = tot_s ? atomicAdd(&ws.counters[kCntShortChunks], tot_s) : 0u;
    }
    __syncthreads();
    if (c == 0u) return;
    const uint32_t base = sl.wg_base[0] + off_p;
    uint32_t sb = base;
#pragma unroll
    for (uint32_t j = 0; j < SUB; j++) {
        ws.base[b * SUB + j] = sb;
        sb += sc[j];
    }
    const uint32_t cf = sl.wg_base[1] + off_f;
    for (uint32_t j = 0; j < nfront && cf + j < ws.max_chunks; j++)
        ws.chunks[cf + j] = make_uint4(base + j * cpk, min(cpk, fpk - j * cpk), key, cls | (2u << kChunkLgShift));
    if (back) {
        const uint4 ch = make_uint4(base + fpk, tail, key, cls | (lg << kChunkLgShift));
        const uint32_t tl = sl.wg_base[2] + off_l, ts = sl.wg_base[3] + off_s;
        if (is_long) {
            if (tl < ws.max_chunks) ws.chunks[ws.max_chunks - 1u - tl] = ch;
        } else if (ts < ws.max_short) {
            ws.chunks[ws.max_chunks + ts] = ch;
        }
    }
}

// pass 3: scatter packet i's index into its bin's range, at the rank pass 1 drew
__device__ __forceinline__ void sched_scatter_one(const SchedWs& ws, uint32_t i) {
    ws.sorted[ws.base[ws.binof[i]] + ws.binpos[i]] = i;
}

}  // namespace neb
