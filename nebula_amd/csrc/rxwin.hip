// rxwin.hip — batched receive with the replay windows in device memory (neb_rx_open_batch,
// window.cpp): ConnectionState.Decrypt (connection_state.go:99-119) over a device-resident batch,
// with results identical to running it packet by packet in arrival order.
//
// The sequential Check → DecryptDanger → Update of one window (bits.go:134-262) has a parallel
// form when every packet's tag verifies and no counter is near 2^64 (no uint64 wrap in
// current + length). Within one window's run of packets, in arrival order:
//   cur_k   = max(current_0, c_1..c_k)                       (a segmented prefix max)
//   admit_k = c_k is the first occurrence of its value in the run, and
//             c_k > cur_(k-1), or c_k is strictly within the window of cur_(k-1) and was not
//             received before the batch (old bit, for c_k <= current_0)
// (an earlier equal counter was either admitted, making this one a duplicate, or refused for a
// reason that still holds, since cur only grows). After the batch:
//   current = cur_n; the slot of every counter c_s in the final window holds
//   (c_s <= current_0 ? its old bit : 0) | (c_s admitted in the batch); slots above current stay
//   as they were during warmup;
//   lost += the counters e >= 1 that left the window (old window's first .. current - length)
//           and were received neither before nor during the batch (the sum of the fast path's
//           and the jump path's lost accounting, bits.go:173-240);
//   dupe and out-of-window counters do not move (Update only runs after Check passed).
// Windows where a tag fails, or whose counters come within 2^62 of wrapping (those admit nothing
// here), are finished on the host with the sequential code in rounds (window.cpp exact_rounds).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/nebula_aead.h"
#include "rxwin.hpp"
#include "sched_body.hpp"

namespace neb {

__device__ __forceinline__ bool rx_in_window(uint64_t i, uint64_t cur, uint64_t len) {  // bits.go:120-132
    if (i < len && cur < len) return true;
    return i > cur - len;
}
__device__ __forceinline__ bool rx_bit(const uint64_t* bits, uint64_t mask, uint64_t i) {
    const uint64_t p = i & mask;
    return (bits[p >> 6] >> (p & 63)) & 1u;
}

__device__ __forceinline__ uint32_t rx_hash(uint32_t w, uint64_t c, uint32_t lg) {
    uint64_t h = (c ^ ((uint64_t)w << 40) ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    return (uint32_t)(h >> (64 - lg));
}

// The slot of packet i's (window, counter) key: claimed by the first to arrive at it, found by
// comparing the owner's key (exact, no hash comparison); the table has at least 4n slots. An
// entry whose generation is not this batch's is empty.
__device__ __forceinline__ uint32_t rx_slot(const RxDevWs& ws, uint32_t i, uint32_t w, uint64_t c, bool insert) {
    const uint32_t tmask = (1u << ws.tab_lg) - 1u;
    const uint64_t mine = ((uint64_t)ws.gen << 32) | (i + 1u);
    uint32_t h = rx_hash(w, c, ws.tab_lg);
    for (;;) {
        uint64_t o = ws.tab_owner[h];
        if (insert) {
            while ((uint32_t)(o >> 32) != ws.gen) {  // empty: claim it
                const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(ws.tab_owner + h), o, mine);
                if (seen == o) return h;
                o = seen;
            }
        }
        // (a lookup always finds its own key before an empty slot)
        const uint32_t oi = (uint32_t)o - 1u;
        if (o == mine || (ws.keyw[oi] == w && ws.ctr[oi] == c)) return h;
        h = (h + 1u) & tmask;
    }
}


// The first-occurrence table's insert, in the keys kernel: as rx_slot, but an owner's key comes
// from its descriptor (keyw / ctr of other workgroups are being written in the same launch).
__device__ __forceinline__ uint32_t rx_slot_insert(const RxDevWs& ws, const RxDevWin& win,
                                                   const neb_desc* __restrict__ desc, uint32_t i, uint32_t w,
                                                   uint64_t c) {
    const uint32_t tmask = (1u << ws.tab_lg) - 1u;
    const uint64_t mine = ((uint64_t)ws.gen << 32) | (i + 1u);
    uint32_t h = rx_hash(w, c, ws.tab_lg);
    for (;;) {
        uint64_t o = ws.tab_owner[h];  // may be stale: the CAS returns the slot's real owner
        while ((uint32_t)(o >> 32) != ws.gen) {  // empty: claim it
            const uint64_t seen = atomicCAS(reinterpret_cast<unsigned long long*>(ws.tab_owner + h), o, mine);
            if (seen == o) return h;
            o = seen;
        }
        if (o == mine) return h;
        const uint32_t oi = (uint32_t)o - 1u;
        const uint32_t ok = desc[oi].key_id;
        const uint32_t ow = ok < win.count && win.present[ok] ? ok : win.count;
        if (ow == w && desc[oi].counter == c) return h;
        h = (h + 1u) & tmask;
    }
}

// ---- the stable sort of the packets by window (LSD radix, arrival order kept) ----------------
// At most kRxSortBlocks workgroups of 256 x items packets each, so every workgroup of a pass can
// read all the workgroups' digit counts itself (no scan launch) and the next pass's counts are
// gathered per output workgroup in LDS. One pass is two launches (the first fused into the keys
// kernel), every further pass one more: 2 launches up to 256 windows, 3 up to 16 Ki.
struct RxSort {
    uint32_t n, items, per_blk, nblk;  // per_blk = 256 x items
    uint32_t passes;
    uint32_t shift[kRxSortMaxPasses];
    uint32_t bits[kRxSortMaxPasses];
};

// Per packet: its window (or count: none) and counter, and the first pass's digit counts per
// workgroup (packet e = b * per_blk + j * 256 + t). Also clears the window flags, the admitted
// count and the later passes' digit counts (the grid covers the packets and the windows).
// Workgroups from kgrid on insert the packets' (window, counter) keys into the first-occurrence table,
// one packet per thread, and mark a window whose counter is near the wrap for the host (the
// scan-admit reads both). Nothing else in the launch reads the table, so the inserts run beside the
// keys work instead of after it: inside the keys workgroups' loop (4 packets per thread on 64
// workgroups) they cost 33-35 µs on C3, as a launch of their own 14 after the keys' 8.
__global__ __launch_bounds__(256) void rx_keys_kernel(const neb_desc* __restrict__ desc, RxDevWin win, RxDevWs ws,
                                                      RxSort so, uint32_t kgrid, RxBin bin) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_mixed;
    if (blockIdx.x >= kgrid) {
        const uint32_t e = (blockIdx.x - kgrid) * 256u + threadIdx.x;
        // the open's binning, pass 1, over the same 256 packets (every lane: its shuffles)
        if (bin.on) sched_hist_round<1>(desc, so.n, bin.max_keys, 4u, bin.ws, e - threadIdx.x, blockIdx.x - kgrid);
        if (e >= so.n) return;
        const uint32_t k = desc[e].key_id;
        if (k >= win.count || !win.present[k]) return;
        const uint64_t c = desc[e].counter;
        const uint32_t h = rx_slot_insert(ws, win, desc, e, k, c);
        atomicMax(reinterpret_cast<unsigned long long*>(ws.tab_min + h), ((unsigned long long)ws.gen << 32) | (0xFFFFFFFFu - e));
        if (c >= kRxRiskyCounter) atomicMax(ws.wrisky + k, ws.gen);
        return;
    }
    const uint32_t t = threadIdx.x, b = blockIdx.x;
    hist[t] = 0;
    if (t == 0) s_mixed = 0;
    for (uint32_t x = t; x < so.per_blk; x += 256) {
        const size_t wi = (size_t)b * so.per_blk + x;
        if (wi < win.count) ws.wflag[wi] = 0;
    }
    if (b == 0 && t == 0) {
        *ws.ticket = 0;
        *ws.err = 0;
    }
    if (b == 0 && bin.on) sched_clear_cursors(bin.ws);
    if (b >= so.nblk) return;
    for (uint32_t p = 1; p < so.passes; p++) ws.sort_hist[((size_t)p * kRxSortBlocks + b) * 256 + t] = 0;
    __syncthreads();
    const uint32_t mask = (1u << so.bits[0]) - 1u;
    // the first packet's window: a batch whose packets all name it needs no sort
    uint32_t w0 = win.count;
    {
        const uint32_t k0 = desc[0].key_id;
        if (k0 < win.count && win.present[k0]) w0 = k0;
    }
    bool differs = false;
    constexpr uint32_t R = kRxSortLoad;
    for (uint32_t j0 = 0; j0 < so.items; j0 += R) {
        uint32_t kid[R], pres[R];
        uint64_t ctr[R];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = b * so.per_blk + (j0 + r) * 256u + t;
            kid[r] = win.count;
            ctr[r] = 0;
            if (j0 + r < so.items && e < so.n) {
                kid[r] = desc[e].key_id;
                ctr[r] = desc[e].counter;
            }
        }
#pragma unroll
        for (uint32_t r = 0; r < R; r++) pres[r] = kid[r] < win.count ? win.present[kid[r]] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = b * so.per_blk + (j0 + r) * 256u + t;
            if (j0 + r >= so.items || e >= so.n) break;
            const uint32_t w = pres[r] ? kid[r] : win.count;
            ws.keyw[e] = w;
            ws.ctr[e] = ctr[r];
            differs |= w != w0;
            atomicAdd(&hist[(w >> so.shift[0]) & mask], 1u);
        }
    }
    if (differs) s_mixed = 1u;
    __syncthreads();
    ws.sort_hist[(size_t)b * 256 + t] = hist[t];
    if (t == 0 && s_mixed) *ws.mixed = ws.gen;  // read by the sort passes (the next launches)
}

// One pass: every packet of the workgroup to base[digit] + (its digit's count in earlier
// workgroups) + (its rank among the workgroup's packets of that digit, in arrival order: a round
// of 256 at a time, ranks within a wave from ballots, waves in order through LDS). Unless this is
// the last pass, the next digit is counted per output workgroup in LDS and added to its counts.
// A batch whose packets all name one window (the keys kernel did not mark this generation mixed:
// one tunnel's flush) is already in run order: pass 0 writes the identity into the run arrays and
// the later passes do nothing.
template <bool FIRST>
__global__ __launch_bounds__(256) void rx_sort_pass_kernel(RxSort so, uint32_t p, uint32_t* hist_all,
                                                           const uint32_t* __restrict__ src_k,
                                                           const uint32_t* __restrict__ src_v, uint32_t* dst_k,
                                                           uint32_t* dst_v, const uint32_t* mixed, uint32_t gen,
                                                           uint32_t* run_w, uint32_t* run_i, RxBin bin) {
    __shared__ uint32_t gbase[256], run[256], wcnt[4][256], wtot[4];
    __shared__ uint32_t agg[kRxSortBlocks << kRxSortDigit];
    if (blockIdx.x >= so.nblk) {  // the open's binning: pass 2 beside the first sort pass, 3 beside the second
        const uint32_t r = blockIdx.x - so.nblk;
        if (FIRST) {
            __shared__ SchedAllocLds sl;
            sched_alloc_block<1>(bin.max_keys, bin.ws, r, sl);
        } else {
            const uint32_t i = r * 256u + threadIdx.x;
            if (i < so.n) sched_scatter_one(bin.ws, i);
        }
        return;
    }
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6, b = blockIdx.x;
    if (__builtin_amdgcn_readfirstlane(*mixed) != gen) {
        if (FIRST) {
            const uint32_t e1 = min(so.n, (b + 1u) * so.per_blk);
            for (uint32_t e = b * so.per_blk + t; e < e1; e += 256u) {
                run_w[e] = src_k[e];
                run_i[e] = e;
            }
        }
        return;
    }
    const uint32_t* hist = hist_all + (size_t)p * kRxSortBlocks * 256;
    const bool next = p + 1 < so.passes;
    const uint32_t nb2 = next ? 1u << so.bits[p + 1] : 0u;
    // digit t: the count in earlier workgroups, and the total (exclusive scan over digits below)
    uint32_t pre = 0, tot = 0;
    // every row loaded at once (rows from nblk on are allocated and masked): one memory latency
    // instead of nblk / 8 of them one after another (C3: the two passes 19.1 -> 17.9 us)
#pragma unroll
    for (uint32_t q = 0; q < kRxSortBlocks; q++) {
        const uint32_t h = hist[(size_t)q * 256 + t];
        const uint32_t hv = q < so.nblk ? h : 0u;
        tot += hv;
        pre += q < b ? hv : 0u;
    }
    uint32_t x = tot;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63u) wtot[wv] = x;
    run[t] = 0;
#pragma unroll
    for (uint32_t v = 0; v < 4; v++) wcnt[v][t] = 0;
    for (uint32_t i = t; i < so.nblk * nb2; i += 256) agg[i] = 0;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t v = 0; v < wv; v++) wbase += wtot[v];
    gbase[t] = wbase + x - tot + pre;
    __syncthreads();
    const uint32_t sh = so.shift[p], nbits = so.bits[p], mask = (1u << nbits) - 1u;
    const uint32_t sh2 = next ? so.shift[p + 1] : 0u, mask2 = nb2 - 1u;
    const uint64_t lt = (1ull << lane) - 1u;
    // rounds of 256 packets, keys loaded kRxSortLoad rounds ahead
    constexpr uint32_t R = kRxSortLoad;
    for (uint32_t j0 = 0; j0 < so.items; j0 += R) {
        uint32_t key[R], val[R];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = b * so.per_blk + (j0 + r) * 256u + t;
            const bool valid = j0 + r < so.items && e < so.n;
            key[r] = valid ? src_k[e] : 0u;
            val[r] = FIRST ? e : (valid ? src_v[e] : 0u);
        }
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            if (j0 + r >= so.items) break;  // uniform
            const uint32_t e = b * so.per_blk + (j0 + r) * 256u + t;
            const bool valid = e < so.n;
            const uint32_t dg = (key[r] >> sh) & mask;
            uint64_t eq = __ballot(valid);
            for (uint32_t bit = 0; bit < nbits; bit++) {
                const uint64_t bb = __ballot((dg >> bit) & 1u);
                eq &= ((dg >> bit) & 1u) ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(eq & lt);
            if (valid && rank == 0) wcnt[wv][dg] = (uint32_t)__popcll(eq);
            __syncthreads();
            if (valid) {
                uint32_t pos = gbase[dg] + run[dg] + rank;
                for (uint32_t v = 0; v < wv; v++) pos += wcnt[v][dg];
                dst_k[pos] = key[r];
                dst_v[pos] = val[r];
                if (next) atomicAdd(&agg[(pos / so.per_blk) * nb2 + ((key[r] >> sh2) & mask2)], 1u);
            }
            __syncthreads();
            run[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
#pragma unroll
            for (uint32_t v = 0; v < 4; v++) wcnt[v][t] = 0;
            __syncthreads();
        }
    }
    if (next) {
        uint32_t* h2 = hist_all + (size_t)(p + 1) * kRxSortBlocks * 256;
        for (uint32_t i = t; i < so.nblk * nb2; i += 256) {
            const uint32_t c = agg[i];
            if (c) atomicAdd(&h2[(i / nb2) * 256u + (i & (nb2 - 1u))], c);
        }
    }
}

// The open's binning, pass 3, as a launch of its own when the sort took one pass (the scan after it
// rewrites refused packets' places in sorted[], so the scatter cannot run beside it).
__global__ __launch_bounds__(256) void rx_bin_scatter_kernel(uint32_t n, RxBin bin) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n) sched_scatter_one(bin.ws, i);
}

// (head, max) pairs of the segmented max scan: a head starts a new run
struct RxSeg {
    uint32_t f;
    uint64_t v;
};
__device__ __forceinline__ RxSeg rx_seg(RxSeg a, RxSeg b) { return {a.f | b.f, b.f ? b.v : max(a.v, b.v)}; }

// R2 granules (cdna_hip_programming.md Guideline 16): {gen:32 | value:32}, one aligned 8-B
// agent-scope atomic store each, read back by agent-scope atomic loads until the tag matches
__device__ __forceinline__ void rx_pub(uint64_t* g, uint32_t gen, uint32_t v) {
    __hip_atomic_store(g, ((uint64_t)gen << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t rx_peek(const uint64_t* g) {
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// kRxSpinLimit (rxwin.hpp) polls, ≈ 0.1 s: then the batch fails (need_host bit 1)

// Scan and admission in one launch, kRxBlock run positions per workgroup, in the order the
// workgroups start (a ticket), so every block a workgroup waits for has started and waits only
// for blocks before it. Per workgroup:
//  1. its counters into run order, touched / risky flags of its runs' heads, and the segmented
//     inclusive max of the counters within the block; then its first head and the max at its last
//     position are published (rx_pub, tagged with the batch generation);
//  2. one wave looks back over the blocks before it, as far as (and including) the first that holds
//     a run head, and takes the max of their published values: the max over the part of the run
//     that continues into this block from before it;
//  3. which packets the sequential receive would decrypt, if every tag verified (safe windows):
//     c > the run's max so far, or inside the window, not received before and the first
//     occurrence of its (window, counter) (the table the keys kernel filled): the admission mask
//     adm, which the open reads (it runs over the whole batch and skips the rest: no compaction, so
//     the mixed-key binning can run beside this plan, window.cpp); the run's last packet sets its
//     window's final current and the range of counters that leave it.
// A window with a counter near the wrap (wrisky, from the keys kernel) or a current near it is
// decided on the host.
__global__ __launch_bounds__(kRxThreads) void rx_scan_admit_kernel(const neb_desc* __restrict__ desc, uint32_t n,
                                                                     RxDevWin win, RxDevWs ws,
                                                                     int32_t* __restrict__ status, RxBin bin) {
    __shared__ uint64_t s_v[kRxThreads / 64];
    __shared__ uint32_t s_f[kRxThreads / 64];
    __shared__ uint64_t s_incl[kRxBlock];
    __shared__ uint64_t s_pre;
    __shared__ uint32_t s_fh, s_b;
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    if (t == 0) {
        s_b = atomicAdd(ws.ticket, 1u);
        s_fh = kRxBlock;
    }
    __syncthreads();
    const uint32_t b = s_b, b0 = b * kRxBlock, k0 = b0 + t * kRxItems;
    const uint32_t gen = ws.gen;
    uint64_t c[kRxItems];
    uint32_t hd[kRxItems], wj[kRxItems], ij[kRxItems];
    RxSeg agg{0u, 0ull};
#pragma unroll
    for (uint32_t j = 0; j < kRxItems; j++) {
        const uint32_t k = k0 + j;
        c[j] = 0;
        hd[j] = 0;
        wj[j] = win.count;
        ij[j] = 0;
        if (k >= n) continue;
        const uint32_t w = ws.run_w[k];
        const uint32_t i = ws.run_i[k];
        wj[j] = w;
        ij[j] = i;
        c[j] = ws.ctr[i];
        ws.run_c[k] = c[j];
        hd[j] = k == 0u || ws.run_w[k - 1u] != w;
        agg = rx_seg(agg, {hd[j], c[j]});
        // flag words are written by the run's head only (one window's whole batch on one address
        // would serialise)
        if (w < win.count && hd[j]) {
            const bool risky = ws.wrisky[w] == gen || win.cur[w] >= kRxRiskyCounter;
            atomicOr(&ws.wflag[w], kRxTouched | (risky ? kRxRisky : 0u));
            if (risky) ws.need_host[0] = 1u;  // (pinned host word) the window finishes on the host
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < kRxItems; j++)
        if (hd[j]) {
            atomicMin(&s_fh, t * kRxItems + j);
            break;
        }
    // exclusive prefix of the thread aggregates: within the wave, then across the waves
    RxSeg x = agg;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t f = __shfl_up(x.f, o);
        const uint64_t v = __shfl_up(x.v, o);
        if (lane >= o) x = rx_seg({f, v}, x);
    }
    if (lane == 63u) {
        s_f[wv] = x.f;
        s_v[wv] = x.v;
    }
    RxSeg ex{__shfl_up(x.f, 1), __shfl_up(x.v, 1)};
    if (lane == 0) ex = {0u, 0ull};
    __syncthreads();
    RxSeg wp{0u, 0ull};
    for (uint32_t q = 0; q < wv; q++) wp = rx_seg(wp, {s_f[q], s_v[q]});
    RxSeg run = rx_seg(wp, ex);
    const uint32_t fh = s_fh;
#pragma unroll
    for (uint32_t j = 0; j < kRxItems; j++) {
        const uint32_t k = k0 + j;
        run = rx_seg(run, {hd[j], c[j]});
        s_incl[t * kRxItems + j] = run.v;
        if (k + 1u == n || k == b0 + kRxBlock - 1u) {  // the block's last position: publish
            rx_pub(ws.blk_pub + 3u * b, gen, fh);
            rx_pub(ws.blk_pub + 3u * b + 1u, gen, (uint32_t)run.v);
            rx_pub(ws.blk_pub + 3u * b + 2u, gen, (uint32_t)(run.v >> 32));
        }
    }
    // the max over the run that continues into this block: back over earlier blocks to (and
    // including) the first one holding a run head, 64 at a time, each lane polling one block's
    // granules until they carry this batch's generation
    if (wv == 0) {
        uint64_t pre = 0;
        bool timed_out = false;
        if (fh > 0u)
            for (int64_t base = (int64_t)b - 1; base >= 0 && !timed_out; base -= 64) {
                const int64_t bb = base - (int64_t)lane;
                const bool valid = bb >= 0;
                uint32_t g_fh = kRxBlock;
                uint64_t g_max = 0;
                bool got = !valid;
                uint32_t spins = 0;
                if (ws.spin_limit == 0u) {  // test hook: a lookback that has to wait fails at once
                    timed_out = true;
                    break;
                }
                for (;;) {
                    if (!got) {
                        const uint64_t* g = ws.blk_pub + 3u * (uint64_t)bb;
                        const uint64_t a0 = rx_peek(g), a1 = rx_peek(g + 1), a2 = rx_peek(g + 2);
                        if ((uint32_t)(a0 >> 32) == gen && (uint32_t)(a1 >> 32) == gen && (uint32_t)(a2 >> 32) == gen) {
                            got = true;
                            g_fh = (uint32_t)a0;
                            g_max = (uint64_t)(uint32_t)a1 | ((uint64_t)(uint32_t)a2 << 32);
                        }
                    }
                    // done once the blocks up to the nearest one with a head (or all 64) are in
                    const uint64_t in = __ballot(got), heads = __ballot(got && g_fh < kRxBlock);
                    const uint64_t need = heads ? ((heads & (~heads + 1u)) << 1) - 1u : ~0ull;  // lanes <= first head
                    if ((in & need) == need) break;
                    if (++spins > ws.spin_limit) {
                        timed_out = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (timed_out) break;
                const bool has = valid && g_fh < kRxBlock;
                const uint64_t stop = __ballot(has);
                const uint32_t last = stop ? (uint32_t)__builtin_ctzll(stop) : 63u;
                uint64_t m = (valid && lane <= last) ? g_max : 0ull;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) m = max(m, (uint64_t)__shfl_xor(m, o));
                pre = max(pre, m);
                if (stop) break;
            }
        if (lane == 0) {
            s_pre = pre;
            if (timed_out) {
                atomicOr(ws.err, 1u);
                ws.need_host[0] = 1u;
                ws.need_host[1] = 1u;  // the batch fails; no window moves (rx_final_window_kernel reads err)
                s_fh = 0xFFFFFFFFu;    // admit nothing here
            }
        }
    }
    __syncthreads();
    const uint64_t pre = s_pre;
    const bool failed = s_fh == 0xFFFFFFFFu;
    auto incl_at = [&](uint32_t k) -> uint64_t {  // the run's inclusive max at k (k >= b0 - 1)
        if (k < b0) return pre;
        const uint64_t v = s_incl[k - b0];
        return k - b0 >= fh ? v : max(pre, v);
    };
#pragma unroll
    for (uint32_t j = 0; j < kRxItems; j++) {
        const uint32_t k = k0 + j;
        if (k >= n) continue;
        const uint32_t w = wj[j];
        const uint32_t i = ij[j];
        ws.verdict[i] = NEB_STATUS_OK;
        ws.adm[i] = 0;
        // the open's binning (RxBin) placed every packet: a packet not admitted leaves its place
        // empty (kSortedSkip), so the plain chunk kernel skips it with no mask of its own
        if (bin.on) bin.ws.sorted[bin.ws.base[bin.ws.binof[i]] + bin.ws.binpos[i]] = kSortedSkip;
        if (w >= win.count) {
            status[i] = NEB_STATUS_BAD_KEY;  // no window: no ConnectionState for this index
            continue;
        }
        const uint64_t cur0 = win.cur[w];
        if (k + 1u == n || ws.run_w[k + 1u] != w) {  // the run's last packet: the window's finish
            const uint64_t len = win.length, cur = max(cur0, incl_at(k));
            ws.curnew[w] = cur;
            ws.exit_lo[w] = cur0 >= len ? cur0 - len + 1u : 1u;  // counter 0 is never lost
            ws.exit_hi[w] = cur >= len ? cur - len : 0u;          // lo > hi: none left
            ws.recv[w] = 0;
        }
        if (failed || ws.wrisky[w] == gen || cur0 >= kRxRiskyCounter) continue;  // decided on the host
        const bool head = hd[j] != 0u;
        const uint64_t prev = head ? cur0 : max(cur0, incl_at(k - 1u));
        const uint64_t cc = c[j];
        const uint64_t* bits = win.bits + ((size_t)w << win.words_lg);
        bool ok = cc > prev;  // above every earlier counter of the run: its first occurrence too
        if (!ok && rx_in_window(cc, prev, win.length)) {
            ok = !(cc <= cur0 && rx_bit(bits, win.length - 1u, cc));
            // the first occurrence of (window, counter)
            ok = ok && ws.tab_min[rx_slot(ws, i, w, cc, false)] == (((uint64_t)gen << 32) | (0xFFFFFFFFu - i));
        }
        if (ok) {
            ws.adm[i] = 1;  // the open runs it (the admission mask)
            if (bin.on) bin.ws.sorted[bin.ws.base[bin.ws.binof[i]] + bin.ws.binpos[i]] = i;
        } else {
            status[i] = NEB_STATUS_REPLAY;  // (a slow window's statuses are rewritten on the host)
        }
    }
}

__global__ void rx_gather_desc_kernel(const neb_desc* __restrict__ desc, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < *ws.nsub) ws.sub_desc[j] = desc[ws.sub_map[j]];
}

__global__ __launch_bounds__(256) void rx_span_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                      const neb_span* __restrict__ spans, uint32_t n) {
    const uint32_t j = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (j >= n) return;
    const neb_span sp = spans[j];
    for (uint32_t k = lane; k < sp.len; k += 64u) dst[sp.dst + k] = src ? src[sp.src + k] : (uint8_t)0;
}

__global__ __launch_bounds__(256) void rx_wire_kernel(const neb_rx_packet* __restrict__ pk, uint32_t n,
                                                      const uint8_t* __restrict__ arena, neb_desc* __restrict__ desc,
                                                      int32_t* __restrict__ gate) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const neb_rx_packet p = pk[i];
    uint8_t h[16];
    if (neb_rx_len(p) >= 16u)
        for (int k = 0; k < 16; k++) h[k] = arena[p.off + k];
    neb_desc d{p.off, p.off, p.off, 0, 0, 0, NEB_KEYS_MIXED, 0};
    const int32_t g = neb_rx_wire_gate(h, p, &d);
    if (g != NEB_STATUS_OK) d = neb_desc{p.off, p.off, p.off, 0, 0, 0, NEB_KEYS_MIXED, 0};
    desc[i] = d;
    gate[i] = g;
}

__global__ __launch_bounds__(256) void rx_wire_fix_kernel(const int32_t* __restrict__ gate, int32_t* __restrict__ status,
                                                          uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n && gate[i] != NEB_STATUS_OK) status[i] = gate[i];
}

__device__ __forceinline__ bool rx_fast(uint32_t fl) { return (fl & kRxTouched) && !(fl & (kRxRisky | kRxSlow)); }

// Per admitted packet, in run order (the windows' runs are contiguous there, so the atomics below
// aggregate): its tag verdict (the status the open wrote at its arrival index; a failure sends the
// window to the sequential host pass, which rewrites that window's statuses), its counter into the
// scratch bitmap when it stays in the final window, and into the received count when it leaves it.
// The window's fast / slow state is not known yet: the finish applies the scratch and the count to
// fast windows only and clears the scratch of the others. One atomic per (wave, window, word)
// instead of one per packet (a single tunnel's batch would otherwise serialise tens of thousands
// of atomics on one address); every lane runs to the end (the shuffles need the whole wave).
__global__ void rx_settle_kernel(uint32_t n, RxDevWin win, RxDevWs ws, const int32_t* __restrict__ status) {
    __shared__ unsigned long long s_recv;
    if (threadIdx.x == 0) s_recv = 0;
    __syncthreads();
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t w = win.count;
    uint64_t c = 0, cur = 0, lo = 1, hi = 0;
    bool ok = false;
    if (k < n) {
        const uint32_t i = ws.run_i[k];
        if (ws.adm[i]) {
            const int32_t st = status[i];
            w = ws.run_w[k];
            c = ws.run_c[k];
            ws.verdict[i] = st;
            ok = st == NEB_STATUS_OK;
            if (!ok) atomicOr(&ws.wflag[w], kRxSlow);
            cur = ws.curnew[w];
            lo = ws.exit_lo[w];
            hi = ws.exit_hi[w];
        }
    }
    const uint64_t len = win.length;
    const bool in_final = ok && (cur < len || c > cur - len);
    const bool leaves = ok && c >= lo && c <= hi;
    const uint64_t p = c & (len - 1u);
    // word key of this lane's bit; lanes of one (window, word) OR their bits into one atomic
    const uint64_t wkey = in_final ? (((uint64_t)w << 32) | (p >> 6)) : ~0ull;
    uint64_t pending = __ballot(in_final);
    while (pending) {
        const uint32_t leader = __builtin_ctzll(pending);
        const uint64_t lk = __shfl(wkey, (int)leader);
        const bool mine = in_final && wkey == lk;
        uint64_t bits = mine ? 1ull << (p & 63) : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bits |= __shfl_xor(bits, o);
        if (__lane_id() == leader)
            atomicOr(reinterpret_cast<unsigned long long*>(ws.scratch + ((size_t)w << win.words_lg) + (p >> 6)), bits);
        pending &= ~__ballot(mine);
    }
    // counters leaving the window: one atomic per (wave, window), through LDS for the window of
    // the workgroup's first run position
    const uint32_t k0 = blockIdx.x * blockDim.x;
    const uint32_t w0 = k0 < n ? ws.run_w[k0] : win.count;
    uint64_t pend2 = __ballot(leaves);
    while (pend2) {
        const uint32_t leader = __builtin_ctzll(pend2);
        const uint32_t lw = __shfl(w, (int)leader);
        const uint64_t same = __ballot(leaves && w == lw);
        if (__lane_id() == leader) {
            if (w == w0)
                atomicAdd(&s_recv, (unsigned long long)__popcll(same));
            else
                atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w), (unsigned long long)__popcll(same));
        }
        pend2 &= ~same;
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_recv) atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w0), s_recv);
}

// bits of the slots [a, b) within the word whose first slot is q0 (nb slots)
__device__ __forceinline__ uint64_t rx_seg_mask(uint64_t q0, uint32_t nb, uint64_t a, uint64_t b) {
    const uint64_t lo = max(a, q0), hi = min(b, q0 + nb);
    if (lo >= hi) return 0;
    const uint32_t m = (uint32_t)(hi - lo);
    return (m == 64u ? ~0ull : ((1ull << m) - 1u)) << (lo - q0);
}
// ... within the circular slot range [start, start + count) mod len (start < len)
__device__ __forceinline__ uint64_t rx_ring_mask(uint64_t q0, uint32_t nb, uint64_t start, uint64_t count,
                                                 uint64_t len) {
    if (count == 0) return 0;
    if (count >= len) return nb == 64u ? ~0ull : ((1ull << nb) - 1u);
    uint64_t m = rx_seg_mask(q0, nb, start, min(start + count, len));
    if (start + count > len) m |= rx_seg_mask(q0, nb, 0, start + count - len);
    return m;
}

// Per fast window, lanes over its bitmap words (min(words, 64) lanes a window, so a wave holds
// one or more whole windows): the slots of the counters new in (cur0, cur] are cleared and the
// admitted counters ORed in; the old window's counters that leave it are counted as received
// where their old bit is set (tools/rxwin_model.py finish_ranges, checked against the oracle);
// then the window's lost count and current.
__global__ void rx_final_window_kernel(RxDevWin win, RxDevWs ws) {
    const uint32_t lanes_lg = win.words_lg < 6u ? win.words_lg : 6u, L = 1u << lanes_lg;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t wl = t >> lanes_lg;
    const uint32_t sub = (uint32_t)t & (L - 1u);
    const uint32_t w = wl < win.count ? (uint32_t)wl : 0u;
    const uint32_t fl = wl < win.count ? ws.wflag[w] : 0u;
    // After a scan lookback timeout the batch fails and no window moves: the blocks that did finish
    // computed their windows' finals from a partial prefix, and the failed block's packets were never
    // opened, so their counters are unauthenticated (a forged high counter must not advance a window).
    const bool err = *ws.err != 0u;
    const bool fast = rx_fast(fl) && !err;
    // a touched window that is risky or slow goes to the host (pinned host word 0; word 1: the
    // timeout, set by the scan)
    if ((fl & kRxTouched) && (fl & (kRxRisky | kRxSlow)) && sub == 0) ws.need_host[0] = 1u;
    uint64_t r = 0;
    uint64_t cur = 0, lo = 1, hi = 0;
    if ((fl & kRxTouched) && !fast) {  // the settle may have set bits of a window finished on the host
        uint64_t* scr = ws.scratch + ((size_t)w << win.words_lg);
        for (uint32_t q = sub; q < win.words; q += L) scr[q] = 0;
    }
    if (fast) {
        const uint64_t len = win.length, mask = len - 1u, cur0 = win.cur[w];
        cur = ws.curnew[w];
        lo = ws.exit_lo[w];
        hi = ws.exit_hi[w];
        const uint32_t nb = len < 64u ? (uint32_t)len : 64u;
        const uint64_t base = (cur >= len && cur - len > cur0) ? cur - len : cur0;
        const uint64_t ehi = min(hi, cur0);
        uint64_t* bits = win.bits + ((size_t)w << win.words_lg);
        uint64_t* scr = ws.scratch + ((size_t)w << win.words_lg);
        for (uint32_t q = sub; q < win.words; q += L) {
            const uint64_t q0 = (uint64_t)q * 64u;
            const uint64_t clear = rx_ring_mask(q0, nb, (base + 1u) & mask, cur - base, len);
            const uint64_t leaving = ehi >= lo ? rx_ring_mask(q0, nb, lo & mask, ehi - lo + 1u, len) : 0ull;
            const uint64_t old = bits[q];
            bits[q] = (old & ~clear) | scr[q];
            scr[q] = 0;  // zero again for the next batch (zeroed once at allocation)
            r += (uint32_t)__popcll(old & leaving);
        }
    }
    for (uint32_t o = L >> 1; o > 0; o >>= 1) r += __shfl_xor(r, (int)o);  // within the window's lanes
    if (fast && sub == 0) {
        const uint64_t exits = hi >= lo ? hi - lo + 1u : 0u;
        win.lost[w] += (int64_t)(exits - ws.recv[w] - r);
        win.cur[w] = cur;
    }
}

}  // namespace neb

using neb::RxDevWin;
using neb::RxDevWs;

static inline dim3 rx_grid(size_t n) { return dim3((unsigned)((n + 255) / 256)); }

static int rx_bits_for(uint32_t v) {
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= v) bits++;
    return bits;
}

// Phase 1: group by window, prefix maxima, first occurrences, and the admission mask for the safe
// windows (ws->adm).
extern "C" hipError_t neb_rxdev_plan(const neb_desc* d_desc, uint32_t n, const RxDevWin* win, const RxDevWs* ws,
                                     int32_t* d_status, const neb::RxBin* binp, hipStream_t s) {
    neb::RxBin bin{};
    if (binp && binp->on) {
        bin = *binp;
        bin.hist_blocks = (n + 255u) / 256u;  // (the keys launch's insert workgroups: one packet per thread)
        bin.alloc_blocks = (neb::sched_nbins(bin.max_keys) + neb::kAllocThreads - 1) / neb::kAllocThreads;
        bin.scatter_blocks = (n + 255u) / 256u;
    }
    neb::RxSort so{};
    so.n = n;
    so.items = (n + 256u * neb::kRxSortBlocks - 1) / (256u * neb::kRxSortBlocks);
    so.per_blk = 256u * so.items;
    so.nblk = (n + so.per_blk - 1) / so.per_blk;
    const int bits = rx_bits_for(win->count);  // keys 0..count (count: no window)
    so.passes = bits <= 8 ? 1u : (uint32_t)(bits + neb::kRxSortDigit - 1) / neb::kRxSortDigit;
    for (uint32_t p = 0, sh = 0; p < so.passes; p++) {
        so.shift[p] = sh;
        so.bits[p] = (uint32_t)(bits - (int)sh + (int)(so.passes - p) - 1) / (so.passes - p);
        sh += so.bits[p];
    }
    const uint32_t kgrid = std::max<uint32_t>(so.nblk, (win->count + so.per_blk - 1) / so.per_blk);
    hipLaunchKernelGGL(neb::rx_keys_kernel, dim3(kgrid + (n + 255u) / 256u), dim3(256), 0, s, d_desc, *win, *ws, so, kgrid,
                       bin);
    // pass p writes the run arrays when (passes - 1 - p) is even, so the last pass ends there
    for (uint32_t p = 0; p < so.passes; p++) {
        const bool to_run = ((so.passes - 1 - p) & 1u) == 0;
        uint32_t* dk = to_run ? ws->run_w : ws->tmp_k;
        uint32_t* dv = to_run ? ws->run_i : ws->tmp_v;
        const uint32_t* sk = p == 0 ? ws->keyw : (to_run ? ws->tmp_k : ws->run_w);
        const uint32_t* sv = p == 0 ? nullptr : (to_run ? ws->tmp_v : ws->run_i);
        // extra workgroups: the binning's pass 2 beside pass 0, its pass 3 beside pass 1
        const uint32_t extra = !bin.on ? 0u : p == 0 ? bin.alloc_blocks : p == 1 ? bin.scatter_blocks : 0u;
        neb::RxBin b = bin;
        if (p > 1) b.on = 0;
        if (p == 0)
            hipLaunchKernelGGL(neb::rx_sort_pass_kernel<true>, dim3(so.nblk + extra), dim3(256), 0, s, so, p,
                               ws->sort_hist, sk, sv, dk, dv, ws->mixed, ws->gen, ws->run_w, ws->run_i, b);
        else
            hipLaunchKernelGGL(neb::rx_sort_pass_kernel<false>, dim3(so.nblk + extra), dim3(256), 0, s, so, p,
                               ws->sort_hist, sk, sv, dk, dv, ws->mixed, ws->gen, ws->run_w, ws->run_i, b);
    }
    if (bin.on && so.passes == 1)
        hipLaunchKernelGGL(neb::rx_bin_scatter_kernel, dim3(bin.scatter_blocks), dim3(256), 0, s, n, bin);
    const uint32_t nscan = (n + neb::kRxBlock - 1) / neb::kRxBlock;
    hipLaunchKernelGGL(neb::rx_scan_admit_kernel, dim3(nscan), dim3(neb::kRxThreads), 0, s, d_desc, n, *win, *ws,
                       d_status, bin);
    return hipGetLastError();
}

// The descriptors of the packets listed in ws->sub_map[0, *ws->nsub) (at most n), compacted.
extern "C" hipError_t neb_rxdev_gather(const neb_desc* d_desc, uint32_t n, const RxDevWs* ws, hipStream_t s) {
    hipLaunchKernelGGL(neb::rx_gather_desc_kernel, rx_grid(n), dim3(256), 0, s, d_desc, *ws);
    return hipGetLastError();
}

// Phase 3: verdicts and the admitted counters' bits, then the parallel finish of every window
// whose admitted packets all verified.
extern "C" hipError_t neb_rxdev_spans(const uint8_t* src, uint8_t* dst, const neb_span* d_spans, uint32_t n,
                                      hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::rx_span_kernel, dim3((n + 3u) / 4u), dim3(256), 0, s, src, dst, d_spans, n);
    return hipGetLastError();
}

extern "C" hipError_t neb_rxdev_wire(const neb_rx_packet* d_pk, uint32_t n, const uint8_t* d_arena, neb_desc* d_desc,
                                     int32_t* d_gate, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::rx_wire_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, d_pk, n, d_arena, d_desc, d_gate);
    return hipGetLastError();
}

extern "C" hipError_t neb_rxdev_wire_fix(const int32_t* d_gate, int32_t* d_status, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::rx_wire_fix_kernel, dim3((n + 255u) / 256u), dim3(256), 0, s, d_gate, d_status, n);
    return hipGetLastError();
}

extern "C" hipError_t neb_rxdev_finish(uint32_t n, const RxDevWin* win, const RxDevWs* ws, int32_t* d_status,
                                       hipStream_t s) {
    hipLaunchKernelGGL(neb::rx_settle_kernel, rx_grid(n), dim3(256), 0, s, n, *win, *ws, d_status);
    const uint32_t lanes_lg = win->words_lg < 6u ? win->words_lg : 6u;
    hipLaunchKernelGGL(neb::rx_final_window_kernel, rx_grid((size_t)win->count << lanes_lg), dim3(256), 0, s, *win,
                       *ws);
    return hipGetLastError();
}
