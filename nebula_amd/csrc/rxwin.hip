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
// Windows where a tag fails, or whose counters come within 2^62 of wrapping, are finished on the
// host with the sequential code (window.cpp), exactly.
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
    uint32_t fl = kRxTouched;
    if (c >= kRxRiskyCounter) fl |= kRxRisky;
    if (k == 0u || ws.run_w[k - 1u] != w) {
        ws.rstart[w] = k;
        if (win.cur[w] >= kRxRiskyCounter) fl |= kRxRisky;
    }
    if (k + 1u == n || ws.run_w[k + 1u] != w) ws.rend[w] = k + 1u;
    atomicOr(&ws.wflag[w], fl);
}

__global__ void rx_gather_w_kernel(uint32_t n, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) ws.w_c[j] = ws.keyw[ws.i_c[j]];
}

// first occurrence of (window, counter) in arrival order: the batch sorted by counter, then
// stably by window, keeps arrival order among equal pairs
__global__ void rx_first_kernel(uint32_t n, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t i = ws.i_cw[j];
    bool first = true;
    if (j > 0u) {
        const uint32_t q = ws.i_cw[j - 1u];
        first = ws.w_cw[j - 1u] != ws.w_cw[j] || ws.ctr[q] != ws.ctr[i];
    }
    ws.first[i] = first;
}

// which packets the sequential receive would decrypt, if every tag verified (safe windows)
__global__ void rx_admit_kernel(uint32_t n, RxDevWin win, RxDevWs ws, int32_t* __restrict__ status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
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
    const uint64_t* bits = win.bits + (size_t)w * win.words;
    bool ok = c > prev;
    if (!ok && rx_in_window(c, prev, win.length)) ok = !(c <= cur0 && rx_bit(bits, win.length - 1u, c));
    ws.adm[i] = ok && ws.first[i];
}

__global__ void rx_gather_desc_kernel(const neb_desc* __restrict__ desc, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < *ws.nsub) ws.sub_desc[j] = desc[ws.sub_map[j]];
}

// tag verdicts back per packet; a failed one sends its window to the sequential host pass
__global__ void rx_verdict_kernel(uint32_t n, RxDevWs ws) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= *ws.nsub) return;
    const uint32_t i = ws.sub_map[j];
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

__global__ void rx_zero_scratch_kernel(RxDevWin win, RxDevWs ws) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)win.count * win.words) return;
    if (rx_fast(ws.wflag[t / win.words])) ws.scratch[t] = 0;
}

// per packet of a fast window: status, admitted counters into the scratch bitmap, received exits
__global__ void rx_final_packet_kernel(uint32_t n, RxDevWin win, RxDevWs ws, int32_t* __restrict__ status) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t w = ws.run_w[k];
    if (w >= win.count || !rx_fast(ws.wflag[w])) return;
    const uint32_t i = ws.run_i[k];
    if (!ws.adm[i]) {
        status[i] = NEB_STATUS_REPLAY;
        return;
    }
    status[i] = NEB_STATUS_OK;
    const uint64_t c = ws.run_c[k], cur = ws.curnew[w], len = win.length;
    if (cur < len || c > cur - len) {  // still inside the final window
        const uint64_t p = c & (len - 1u);
        atomicOr(reinterpret_cast<unsigned long long*>(ws.scratch + (size_t)w * win.words + (p >> 6)),
                 1ull << (p & 63));
    }
    if (c >= ws.exit_lo[w] && c <= ws.exit_hi[w]) atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w), 1ull);
}

// per bitmap word of a fast window: the final bits, and how many leaving counters were received
// before the batch
__global__ void rx_final_word_kernel(RxDevWin win, RxDevWs ws) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)win.count * win.words) return;
    const uint32_t w = (uint32_t)(t / win.words), q = (uint32_t)(t % win.words);
    if (!rx_fast(ws.wflag[w])) return;
    const uint64_t len = win.length, mask = len - 1u, cur0 = win.cur[w], cur = ws.curnew[w];
    const uint64_t lo = ws.exit_lo[w], hi = min(ws.exit_hi[w], cur0);
    const uint64_t old = win.bits[t], adm = ws.scratch[t];
    const uint32_t nb = len < 64u ? (uint32_t)len : 64u;
    uint64_t out = old;
    uint64_t recv_old = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint64_t s = (uint64_t)q * 64u + b;
        const uint64_t ob = (old >> b) & 1u;
        // the counter slot s held before the batch, and the one it holds after
        bool has_old = true, has_new = true;
        const uint64_t e_old = cur0 >= len ? cur0 - ((cur0 - s) & mask) : s;
        if (cur0 < len && s > cur0) has_old = false;
        const uint64_t c_new = cur >= len ? cur - ((cur - s) & mask) : s;
        if (cur < len && s > cur) has_new = false;  // warmup: untouched above current
        if (has_old && ob && e_old >= lo && e_old <= hi) recv_old++;
        if (has_new) {
            const uint64_t nbit = (c_new <= cur0 ? ob : 0u) | ((adm >> b) & 1u);
            out = (out & ~(1ull << b)) | (nbit << b);
        }
    }
    win.bits[t] = out;
    if (recv_old) atomicAdd(reinterpret_cast<unsigned long long*>(ws.recv + w), (unsigned long long)recv_old);
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
    hipcub::DeviceRadixSort::SortPairs(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr,
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
    hipError_t e = hipMemsetAsync(ws->wflag, 0, (size_t)win->count * sizeof(uint32_t), s);
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
    cb = ws->cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(ws->cub_tmp, cb, ws->ctr, ws->c_s, ws->idx, ws->i_c, (int)n, 0, 64, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_gather_w_kernel, rx_grid(n), dim3(256), 0, s, n, *ws);
    cb = ws->cub_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(ws->cub_tmp, cb, ws->w_c, ws->w_cw, ws->i_c, ws->i_cw, (int)n, 0, wbits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(neb::rx_first_kernel, rx_grid(n), dim3(256), 0, s, n, *ws);
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

// Phase 3: verdicts, then the parallel finish of every window whose admitted packets all verified.
extern "C" hipError_t neb_rxdev_finish(uint32_t n, const RxDevWin* win, const RxDevWs* ws, int32_t* d_status,
                                       hipStream_t s) {
    hipLaunchKernelGGL(neb::rx_verdict_kernel, rx_grid(n), dim3(256), 0, s, n, *ws);
    hipLaunchKernelGGL(neb::rx_final_window_kernel, rx_grid(win->count), dim3(256), 0, s, *win, *ws);
    const size_t nw = (size_t)win->count * win->words;
    hipLaunchKernelGGL(neb::rx_zero_scratch_kernel, rx_grid(nw), dim3(256), 0, s, *win, *ws);
    hipLaunchKernelGGL(neb::rx_final_packet_kernel, rx_grid(n), dim3(256), 0, s, n, *win, *ws, d_status);
    hipLaunchKernelGGL(neb::rx_final_word_kernel, rx_grid(nw), dim3(256), 0, s, *win, *ws);
    hipLaunchKernelGGL(neb::rx_commit_window_kernel, rx_grid(win->count), dim3(256), 0, s, *win, *ws);
    return hipGetLastError();
}
