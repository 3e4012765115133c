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

#include <hipcub/hipcub.hpp>

#include "../../include/nebula_aead.h"
#include "rxwin.hpp"

namespace neb {

__device__ __forceinline__ bool rx_in_window(uint64_t i, uint64_t cur, uint64_t len) {  // bits.go:120-132
    if (i < len && cur < len) return true;
    return i > cur - len;
}
__device__ __forceinline__ bool rx_bit(const uint64_t* bits, uint64_t mask, uint64_t i) {
    const uint64_t p = i & mask;
    return (bits[p >> 6] >> (p & 63)) & 1u;
}

// per packet: its window (or W: none), arrival index, counter
__global__ void rx_keys_kernel(const neb_desc* __restrict__ desc, uint32_t n, RxDevWin win, RxDevWs ws) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const neb_desc d = desc[i];
    ws.keyw[i] = (d.key_id < win.count && win.present[d.key_id]) ? d.key_id : win.count;
    ws.idx[i] = i;
    ws.ctr[i] = d.counter;
    ws.adm[i] = 0;
    ws.verdict[i] = NEB_STATUS_OK;
}

// run order: counters, run bounds, touched / risky windows
__global__ void rx_runs_kernel(uint32_t n, RxDevWin win, RxDevWs ws) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t w = ws.run_w[k];
    const uint32_t i = ws.run_i[k];
    const uint64_t c = ws.ctr[i];
    ws.run_c[k] = c;
    if (w >= win.count) return;
    // flag words are written by the run's head and by risky packets only (one window's whole batch
    // on one address would serialise)
    uint32_t fl = c >= kRxRiskyCounter ? kRxRisky : 0u;
    if (k == 0u || ws.run_w[k - 1u] != w) {
        ws.rstart[w] = k;
        fl |= kRxTouched | (win.cur[w] >= kRxRiskyCounter ? kRxRisky : 0u);
    }
    if (k + 1u == n || ws.run_w[k + 1u] != w) ws.rend[w] = k + 1u;
    if (fl) atomicOr(&ws.wflag[w], fl);
}

__device__ __forceinline__ uint32_t rx_hash(uint32_t w, uint64_t c, uint32_t lg) {
    uint64_t h = (c ^ ((uint64_t)w << 40) ^ w) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    return (uint32_t)(h >> (64 - lg));
}

// the slot of packet i's (window, counter) key: claimed by the first to arrive at it, found by
// comparing the owner's key (exact, no hash comparison); the table has at least 2n slots
__device__ __forceinline__ uint32_t rx_slot(const RxDevWs& ws, uint32_t i, bool insert) {
    const uint32_t w = ws.keyw[i];
    const uint64_t c = ws.ctr[i];
    const uint32_t tmask = (1u << ws.tab_lg) - 1u;
    uint32_t h = rx_hash(w, c, ws.tab_lg);
    for (;;) {
        const uint32_t o = insert ? atomicCAS(&ws.tab_owner[h], 0u, i + 1u) : ws.tab_owner[h];
        if (o == 0u) return h;  // claimed (insert); a lookup always finds its own key first
        if (o == i + 1u || (ws.keyw[o - 1u] == w && ws.ctr[o - 1u] == c)) return h;
        h = (h + 1u) & tmask;
    }
}

__global__ void rx_first_insert_kernel(uint32_t n, RxDevWs ws) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicMin(&ws.tab_min[rx_slot(ws, i, true)], i);
}

// which packets the sequential receive would decrypt, if every tag verified (safe windows)
__global__ void rx_admit_kernel(uint32_t n, RxDevWin win, RxDevWs ws, int32_t* __restrict__ status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;  // (whole waves: the ballot below sees only live lanes)
    const uint32_t w = ws.run_w[k];
    const uint32_t i = ws.run_i[k];
    if (w >= win.count) {
        status[i] = NEB_STATUS_BAD_KEY;  // no window: no ConnectionState for this index
        return;
    }
    if (ws.wflag[w] & kRxRisky) return;  // decided on the host
    const uint64_t cur0 = win.cur[w];
    const uint64_t prev = k == ws.rstart[w] ? cur0 : max(cur0, ws.incl[k - 1u]);
    const uint64_t c = ws.run_c[k];
    const uint64_t* bits = win.bits + ((size_t)w << win.words_lg);
    bool ok = c > prev;
    if (!ok && rx_in_window(c, prev, win.length)) ok = !(c <= cur0 && rx_bit(bits, win.length - 1u, c));
    ok = ok && ws.tab_min[rx_slot(ws, i, false)] == i;  // the first occurrence of (window, counter)
    ws.adm[i] = ok;
    // admitted count (wflag[count]): every packet admitted lets the open skip the compaction
    const uint64_t ball = __ballot(ok);
    if (ok && __lane_id() == (uint32_t)__builtin_ctzll(ball)) atomicAdd(&ws.wflag[win.count], (uint32_t)__popcll(ball));
}

__global__ void rx_gather_desc_kernel(const neb_desc* __restrict__ desc, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < *ws.nsub) ws.sub_desc[j] = desc[ws.sub_map[j]];
}

// tag verdicts back per packet; a failed one sends its window to the sequential host pass
__global__ void rx_verdict_kernel(uint32_t n, RxDevWs ws, int all) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (all ? n : *ws.nsub)) return;
    const uint32_t i = all ? j : ws.sub_map[j];  // all: every packet was opened in arrival order
    const int32_t st = ws.sub_status[j];
    ws.verdict[i] = st;
    if (st != NEB_STATUS_OK) atomicOr(&ws.wflag[ws.keyw[i]], kRxSlow);
}

__device__ __forceinline__ bool rx_fast(uint32_t fl) { return (fl & kRxTouched) && !(fl & (kRxRisky | kRxSlow)); }

// per window: the final current and the range of counters that leave the window
__global__ void rx_final_window_kernel(RxDevWin win, RxDevWs ws) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= win.count || !rx_fast(ws.wflag[w])) return;
    const uint64_t cur0 = win.cur[w], len = win.length;
    const uint64_t cur = max(cur0, ws.incl[ws.rend[w] - 1u]);
    ws.curnew[w] = cur;
    ws.exit_lo[w] = cur0 >= len ? cur0 - len + 1u : 1u;  // counter 0 is never lost
    ws.exit_hi[w] = cur >= len ? cur - len : 0u;          // lo > hi: none left
    ws.recv[w] = 0;
}

// per packet of a fast window: its status; its counter into the scratch bitmap, and into the
// received count when it leaves the window — one atomic per (wave, window, word) instead of one per packet: a
// single tunnel's batch would otherwise serialise tens of thousands of atomics on one address.
// Every lane runs to the end (the shuffles need the whole wave).
__global__ void rx_final_packet_agg_kernel(uint32_t n, RxDevWin win, RxDevWs ws, int32_t* __restrict__ status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t w = win.count;
    uint64_t c = 0;
    bool adm = false;
    if (k < n) {
        w = ws.run_w[k];
        if (w < win.count && rx_fast(ws.wflag[w])) {
            const uint32_t i = ws.run_i[k];
            adm = ws.adm[i];
            status[i] = adm ? NEB_STATUS_OK : NEB_STATUS_REPLAY;
            c = ws.run_c[k];
        } else {
            w = win.count;
        }
    }
    uint64_t cur = 0, lo = 1, hi = 0;
    if (adm) {
        cur = ws.curnew[w];
        lo = ws.exit_lo[w];
        hi = ws.exit_hi[w];
    }
    const uint64_t len = win.length;
    const bool in_final = adm && (cur < len || c > cur - len);
    const bool leaves = adm && c >= lo && c <= hi;
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
    uint64_t pend2 = __ballot(leaves);
    while (pend2) {
        const uint32_t leader = __builtin_ctzll(pend2);
        const uint32_t lw = __shfl(w, (int)leader);
        const uint64_t same = __ballot(leaves && w == lw);
        if (__lane_id() == leader)
            atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w), (unsigned long long)__popcll(same));
        pend2 &= ~same;
    }
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

// per bitmap word of a fast window: the slots of the counters new in (cur0, cur] are cleared and
// the admitted counters ORed in; the old window's counters that leave it are counted as received
// where their old bit is set (tools/rxwin_model.py finish_ranges, checked against the oracle)
__global__ void rx_final_word_kernel(RxDevWin win, RxDevWs ws) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ((size_t)win.count << win.words_lg)) return;
    const uint32_t w = (uint32_t)(t >> win.words_lg), q = (uint32_t)(t & (win.words - 1u));
    if (!rx_fast(ws.wflag[w])) return;
    const uint64_t len = win.length, mask = len - 1u, cur0 = win.cur[w], cur = ws.curnew[w];
    const uint32_t nb = len < 64u ? (uint32_t)len : 64u;
    const uint64_t q0 = (uint64_t)q * 64u;
    const uint64_t base = (cur >= len && cur - len > cur0) ? cur - len : cur0;
    const uint64_t clear = rx_ring_mask(q0, nb, (base + 1u) & mask, cur - base, len);
    const uint64_t lo = ws.exit_lo[w], ehi = min(ws.exit_hi[w], cur0);
    const uint64_t leaving = ehi >= lo ? rx_ring_mask(q0, nb, lo & mask, ehi - lo + 1u, len) : 0ull;
    const uint64_t old = win.bits[t];
    win.bits[t] = (old & ~clear) | ws.scratch[t];
    ws.scratch[t] = 0;  // zero again for the next batch (zeroed once at allocation)
    const uint32_t r = (uint32_t)__popcll(old & leaving);
    if (r) atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w), (unsigned long long)r);
}

__global__ void rx_commit_window_kernel(RxDevWin win, RxDevWs ws) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= win.count || !rx_fast(ws.wflag[w])) return;
    const uint64_t lo = ws.exit_lo[w], hi = ws.exit_hi[w];
    const uint64_t exits = hi >= lo ? hi - lo + 1u : 0u;
    win.lost[w] += (int64_t)(exits - ws.recv[w]);
    win.cur[w] = ws.curnew[w];
}

}  // namespace neb

using neb::RxDevWin;
using neb::RxDevWs;

static inline dim3 rx_grid(size_t n) { return dim3((unsigned)((n + 255) / 256)); }

// Device-side bytes of the hipCUB passes for n packets.
extern "C" size_t neb_rxdev_cub_bytes(uint32_t n) {
    size_t a = 0, b = 0, c = 0, d = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    hipcub::DeviceScan::InclusiveScanByKey(nullptr, c, (const uint32_t*)nullptr, (const uint64_t*)nullptr,
                                           (uint64_t*)nullptr, hipcub::Max(), (int)n, hipcub::Equality());
    hipcub::DeviceSelect::Flagged(nullptr, d, (const uint32_t*)nullptr, (const uint8_t*)nullptr, (uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (int)n);
    return std::max(std::max(a, b), std::max(c, d));
}

static int rx_bits_for(uint32_t v) {
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= v) bits++;
    return bits;
}

// Phase 1: group by window, prefix maxima, first occurrences, admission for the safe windows.
extern "C" hipError_t neb_rxdev_plan(const neb_desc* d_desc, uint32_t n, const RxDevWin* win, const RxDevWs* ws,
                                     int32_t* d_status, hipStream_t s) {
    hipError_t e = hipMemsetAsync(ws->wflag, 0, ((size_t)win->count + 1u) * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_keys_kernel, rx_grid(n), dim3(256), 0, s, d_desc, n, *win, *ws);
    const int wbits = rx_bits_for(win->count);
    size_t cb = ws->cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(ws->cub_tmp, cb, ws->keyw, ws->run_w, ws->idx, ws->run_i, (int)n, 0, wbits,
                                           s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_runs_kernel, rx_grid(n), dim3(256), 0, s, n, *win, *ws);
    cb = ws->cub_bytes;
    e = hipcub::DeviceScan::InclusiveScanByKey(ws->cub_tmp, cb, ws->run_w, ws->run_c, ws->incl, hipcub::Max(), (int)n,
                                               hipcub::Equality(), s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(ws->tab_owner, 0, (size_t)4 << ws->tab_lg, s);
    if (e == hipSuccess) e = hipMemsetAsync(ws->tab_min, 0xFF, (size_t)4 << ws->tab_lg, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_first_insert_kernel, rx_grid(n), dim3(256), 0, s, n, *ws);
    hipLaunchKernelGGL(neb::rx_admit_kernel, rx_grid(n), dim3(256), 0, s, n, *win, *ws, d_status);
    return hipGetLastError();
}

// Phase 2: the admitted packets' descriptors, compacted in arrival order (count in *ws->nsub).
extern "C" hipError_t neb_rxdev_compact(const neb_desc* d_desc, uint32_t n, const RxDevWs* ws, hipStream_t s) {
    size_t cb = ws->cub_bytes;
    hipError_t e = hipcub::DeviceSelect::Flagged(ws->cub_tmp, cb, ws->idx, ws->adm, ws->sub_map, ws->nsub, (int)n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_gather_desc_kernel, rx_grid(n), dim3(256), 0, s, d_desc, *ws);
    return hipGetLastError();
}

// The descriptors of the packets listed in ws->sub_map[0, *ws->nsub) (at most n), compacted.
extern "C" hipError_t neb_rxdev_gather(const neb_desc* d_desc, uint32_t n, const RxDevWs* ws, hipStream_t s) {
    hipLaunchKernelGGL(neb::rx_gather_desc_kernel, rx_grid(n), dim3(256), 0, s, d_desc, *ws);
    return hipGetLastError();
}

// Phase 3: verdicts, then the parallel finish of every window whose admitted packets all verified.
extern "C" hipError_t neb_rxdev_finish(uint32_t n, const RxDevWin* win, const RxDevWs* ws, int32_t* d_status,
                                       int all, hipStream_t s) {
    hipLaunchKernelGGL(neb::rx_verdict_kernel, rx_grid(n), dim3(256), 0, s, n, *ws, all);
    hipLaunchKernelGGL(neb::rx_final_window_kernel, rx_grid(win->count), dim3(256), 0, s, *win, *ws);
    const size_t nw = (size_t)win->count << win->words_lg;
    hipLaunchKernelGGL(neb::rx_final_packet_agg_kernel, rx_grid(n), dim3(256), 0, s, n, *win, *ws, d_status);
    hipLaunchKernelGGL(neb::rx_final_word_kernel, rx_grid(nw), dim3(256), 0, s, *win, *ws);
    hipLaunchKernelGGL(neb::rx_commit_window_kernel, rx_grid(win->count), dim3(256), 0, s, *win, *ws);
    return hipGetLastError();
}
