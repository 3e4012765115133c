// sched_body.hpp — the device bodies of the mixed-key binning passes (sched.hpp): the stand-alone
// launches in sched.hip, and the device receive's plan (rxwin.hip), which runs them as extra
// workgroups of its own launches.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// pass 2 (round 6: per key): every non-empty bin reserves its range of `sorted`, and each key's
// chunks are written into the cost buckets (sched_key_chunks). One thread per bin, the 8 bins
// (size classes) of a key on 8 neighbouring lanes, so a key's plan is computed beside its counts
// (shuffles within the 8 lanes) and every class emits its own chunks in parallel. Reservations go
// through LDS atomics per workgroup, then one global atomic per counter and workgroup (one atomic
// per bin put ~4096 returning atomics on a single word for a 4096-tunnel batch). blk: this
// workgroup's index among the pass's (the grid covers the 8 (max_keys + 1) bins once, kAllocThreads
// each).
constexpr int kAllocThreads = 256;
constexpr uint32_t kAllocCounts = 1u + kBuckets;  // packets, then chunks per bucket
struct SchedAllocLds {
    uint32_t cnt[kAllocCounts];
    uint32_t wg_base[kAllocCounts];
};

// The leftover group of class i of one key (counts c[cls], class cls's range of `sorted` from
// bstart[cls]): the key's leftovers (c mod 16 per class) are planned largest class first, each one
// group at sched_tail_lg lanes that also takes as many of the next smaller class's leftover packets as
// it has free slots (its second segment; a smaller class needs no more rounds at the same lanes).
// Returns false when class i has no group of its own (no leftover, or all of it rode along).
__device__ __forceinline__ bool sched_leftover_group(uint32_t i, uint32_t key, const uint32_t (&c)[kSizeClasses],
                                                     const uint32_t (&bstart)[kSizeClasses], uint32_t& bucket,
                                                     uint4& rec) {
    uint32_t left[kSizeClasses], lpos[kSizeClasses];
#pragma unroll
    for (uint32_t k = 0; k < kSizeClasses; k++) {
        left[k] = c[k] % kChunkPkts;
        lpos[k] = bstart[k] + c[k] / kChunkPkts * kChunkPkts;
    }
    bool mine = false;
#pragma unroll
    for (int g = (int)kSizeClasses - 1; g >= 0; g--) {
        const uint32_t L = left[g];
        if (L == 0u) continue;
        const uint32_t lg = sched_tail_lg(L, (uint32_t)g), free = (64u >> lg) - L;
        uint32_t s1 = 0, c1 = 0;
        bool found = false;
#pragma unroll
        for (int j = g - 1; j >= 0; j--) {  // the next smaller class with a leftover fills the free slots
            if (!found && left[j] != 0u) {
                found = true;
                c1 = min(free, left[j]);
                s1 = lpos[j];
                lpos[j] += c1;
                left[j] -= c1;
            }
        }
        if ((uint32_t)g == i) {
            const bool front = lg == 2u;
            bucket = sched_bucket(front ? sched_front_cost(1u, (uint32_t)g) : sched_tail_cost((uint32_t)g, lg));
            rec = make_uint4(lpos[g], s1, key, chunk_w(L, c1, lg, front, (uint32_t)g));
            mine = true;
        }
    }
    return mine;
}

// THREADS: the workgroup's size (the receive plan's launches run it in their 256-thread workgroups)
template <uint32_t SUB, uint32_t THREADS = kAllocThreads>
__device__ __forceinline__ void sched_alloc_block(uint32_t max_keys, const SchedWs& ws, uint32_t blk,
                                                  SchedAllocLds& sl) {
    const uint32_t K1 = max_keys + 1u;
    const uint32_t t = blk * THREADS + threadIdx.x, key = t / kSizeClasses, cls = t % kSizeClasses;
    const uint32_t lane = threadIdx.x & 63u, grp = lane & ~(kSizeClasses - 1u);
    const bool valid = key < K1;
    const uint32_t bin = cls * K1 + key;
    if (threadIdx.x < kAllocCounts) sl.cnt[threadIdx.x] = 0;
    uint32_t sc[SUB], c = 0;
#pragma unroll
    for (uint32_t j = 0; j < SUB; j++) {
        sc[j] = valid ? ws.hist[bin * SUB + j] : 0u;
        c += sc[j];
    }
    if (c)  // clear for the next batch
#pragma unroll
        for (uint32_t j = 0; j < SUB; j++) ws.hist[bin * SUB + j] = 0u;
    uint32_t cc[kSizeClasses];  // the key's counts
#pragma unroll
    for (uint32_t k = 0; k < kSizeClasses; k++) cc[k] = (uint32_t)__shfl((int)c, (int)(grp + k));
    // this class's front chunks: nfc of g groups, the last one of lastg; and the leftover group
    const uint32_t nf = c / kChunkPkts, g = min(sched_groups(cls), ws.max_groups);
    const uint32_t nfc = (nf + g - 1u) / g, lastg = nf - (nfc ? nfc - 1u : 0u) * g;
    const uint32_t bfull = sched_bucket(sched_front_cost(g, cls)), blast = sched_bucket(sched_front_cost(lastg, cls));
    uint32_t lb = 0;
    uint4 lrec;
    const uint32_t zero[kSizeClasses] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool has_left = c != 0u && sched_leftover_group(cls, key, cc, zero, lb, lrec);
    __syncthreads();
    // reservations inside the workgroup (LDS atomics), then the workgroup's totals globally
    uint32_t o_pk = 0, o_full = 0, o_last = 0, o_left = 0;
    {  // the packets' offset: a wave scan, then one LDS add per wave (not one per bin)
        uint32_t inc = c;
#pragma unroll
        for (uint32_t d = 1; d < 64u; d *= 2u) {
            const uint32_t v = (uint32_t)__shfl_up((int)inc, d);
            if (lane >= d) inc += v;
        }
        uint32_t wbase = 0;
        if (lane == 63u && inc) wbase = atomicAdd(&sl.cnt[0], inc);
        o_pk = (uint32_t)__shfl((int)wbase, 63) + inc - c;
    }
    if (nfc > 1u) o_full = atomicAdd(&sl.cnt[1u + bfull], nfc - 1u);
    if (nfc) o_last = atomicAdd(&sl.cnt[1u + blast], 1u);
    if (has_left) o_left = atomicAdd(&sl.cnt[1u + lb], 1u);
    __syncthreads();
    if (threadIdx.x < kAllocCounts) {
        const uint32_t all = sl.cnt[threadIdx.x];
        sl.wg_base[threadIdx.x] = all ? atomicAdd(&ws.counters[threadIdx.x == 0 ? kCntPackets : kCntBucket + threadIdx.x - 1u], all) : 0u;
    }
    __syncthreads();
    // the bin's range of sorted[] (its sub-bins in turn), and the key's other bins' starts
    const uint32_t base = sl.wg_base[0] + o_pk;
    uint32_t pos = base;
#pragma unroll
    for (uint32_t j = 0; j < SUB; j++) {
        if (c) ws.base[bin * SUB + j] = pos;
        pos += sc[j];
    }
    uint32_t bs[kSizeClasses];
#pragma unroll
    for (uint32_t k = 0; k < kSizeClasses; k++) bs[k] = (uint32_t)__shfl((int)base, (int)(grp + k));
    if (!c) return;
    auto put = [&](uint32_t b, uint32_t slot, uint4 rec) {
        if (slot < ws.max_chunks) ws.chunks[(size_t)b * ws.max_chunks + slot] = rec;
    };
    for (uint32_t j = 0; j < nfc; j++) {
        const bool last = j + 1u == nfc;
        const uint32_t gc = last ? lastg : g;
        put(last ? blast : bfull, last ? sl.wg_base[1u + blast] + o_last : sl.wg_base[1u + bfull] + o_full + j,
            make_uint4(base + j * g * kChunkPkts, 0u, key, chunk_w(gc * kChunkPkts, 0u, 2u, true, cls)));
    }
    if (has_left) {
        sched_leftover_group(cls, key, cc, bs, lb, lrec);
        put(lb, sl.wg_base[1u + lb] + o_left, lrec);
    }
}

// pass 3: scatter packet i's index into its bin's range, at the rank pass 1 drew
__device__ __forceinline__ void sched_scatter_one(const SchedWs& ws, uint32_t i) {
    ws.sorted[ws.base[ws.binof[i]] + ws.binpos[i]] = i;
}

}  // namespace neb
