// sched.hip — device-side binning of a batch into single-key, similar-size chunks (sched.hpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "knobs.hpp"
#include "sched_body.hpp"

namespace neb {

template <uint32_t SUB>
__global__ void sched_hist_kernel(const neb_desc* __restrict__ desc, uint32_t n, const uint32_t* dn,
                                  uint32_t max_keys, uint32_t lpp, SchedWs ws) {
    if (blockIdx.x == 0) sched_clear_cursors(ws);
    if (dn) n = min(n, *dn);
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n; i0 += gridDim.x * blockDim.x)
        sched_hist_round<SUB>(desc, n, max_keys, lpp, ws, i0, blockIdx.x);
}

// Workgroup size of the allocation pass (1024 threads, 4x fewer workgroups and so 4x fewer returning
// atomics on the bucket counters: C5 shard 400 against 408 GiB/s, profiles/r6/ab/alloc_threads.jsonl)
#ifndef NEB_SCHED_ALLOC_THREADS
#define NEB_SCHED_ALLOC_THREADS 256
#endif
constexpr uint32_t kAllocThreadsSched = NEB_SCHED_ALLOC_THREADS;
template <uint32_t SUB>
__global__ __launch_bounds__(kAllocThreadsSched) void sched_alloc_kernel(uint32_t max_keys, SchedWs ws) {
    __shared__ SchedAllocLds sl;
    sched_alloc_block<SUB, kAllocThreadsSched>(max_keys, ws, blockIdx.x, sl);
}

__global__ void sched_scatter_kernel(const neb_desc* __restrict__ desc, uint32_t n, const uint32_t* dn, SchedWs ws) {
    if (dn) n = min(n, *dn);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) sched_scatter_one(ws, i);
}

// ---- tile binning (sched.hpp: large batches, no global atomic per packet) ----------------------

// pass 1: tile blockIdx.x = packets [t·P, (t+1)·P): each packet's bin and its rank among the tile's
// packets of that bin (the LDS add's return), then the tile's counts as one row of tcnt. Runs of
// neighbouring lanes in one bin (a batch already grouped by key) add once, as sched_hist_round.
__global__ __launch_bounds__(kTileThreads) void sched_tile_hist_kernel(const neb_desc* __restrict__ desc, uint32_t n,
                                                                       const uint32_t* dn, uint32_t max_keys,
                                                                       uint32_t lpp, SchedWs ws, uint32_t P,
                                                                       uint32_t words) {
    extern __shared__ uint32_t cnt[];  // two 16-bit counts per word
    if (blockIdx.x == 0) sched_clear_cursors(ws);
    if (dn) n = min(n, *dn);
    for (uint32_t w = threadIdx.x; w < words; w += kTileThreads) cnt[w] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t upto = lane == 63u ? ~0ull : (2ull << lane) - 1u;  // lanes <= this one
    const uint32_t i0 = blockIdx.x * P, i1 = min(n, i0 + P);
    for (uint32_t r = i0; r < i1; r += kTileThreads) {  // (every lane of a wave: its shuffles)
        const uint32_t i = r + threadIdx.x;
        const bool valid = i < i1;
        uint32_t b = 0xFFFFFFFFu;
        if (valid) {
            const neb_desc d = desc[i];
            const uint32_t key = d.key_id < max_keys ? d.key_id : max_keys;
            b = size_class(d, lpp) * (max_keys + 1u) + key;
        }
        const uint32_t pb = (uint32_t)__shfl_up((int)b, 1);
        const bool head = valid && (lane == 0u || pb != b);
        const uint64_t hm = __ballot(head);
        const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
        const uint32_t hl = 63u - (uint32_t)__builtin_clzll((hm & upto) | 1ull);  // this lane's run head
        const uint64_t after = hm & ~upto;
        const uint32_t next = after ? (uint32_t)__builtin_ctzll(after) : nvalid;  // the next run's head
        uint32_t base = 0;
        if (head) {
            const uint32_t sh = (b & 1u) * 16u;
            base = (atomicAdd(&cnt[b >> 1], (next - lane) << sh) >> sh) & 0xFFFFu;
        }
        base = (uint32_t)__shfl((int)base, (int)hl);
        if (valid) {
            ws.binof[i] = b;
            ws.binpos[i] = base + (lane - hl);
        }
    }
    __syncthreads();
    uint32_t* row = ws.tcnt + (size_t)blockIdx.x * words;
    for (uint32_t w = threadIdx.x; w < words; w += kTileThreads) row[w] = cnt[w];
}

// pass 2: per bin, the exclusive sum over the tiles (tpre) and the total (hist[b], read by the
// allocation pass as one sub-bin). A workgroup takes 16 count words (32 bins) × 16 slices of the
// tiles; the slices' sums meet in LDS.
constexpr uint32_t kTileSlices = 16, kTileSliceMax = kTileMax / kTileSlices;
__global__ __launch_bounds__(256) void sched_tile_scan_kernel(SchedWs ws, uint32_t T, uint32_t words, uint32_t nb) {
    __shared__ uint32_t part[kTileSlices][16][2];
    const uint32_t wl = threadIdx.x & 15u, sl = threadIdx.x >> 4;
    const uint32_t w = blockIdx.x * 16u + wl;
    const uint32_t S = (T + kTileSlices - 1u) / kTileSlices, t0 = sl * S;
    uint32_t v[kTileSliceMax];
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (uint32_t k = 0; k < kTileSliceMax; k++) {
        v[k] = k < S && t0 + k < T ? ws.tcnt[(size_t)(t0 + k) * words + w] : 0u;
        lo += v[k] & 0xFFFFu;
        hi += v[k] >> 16;
    }
    part[sl][wl][0] = lo;
    part[sl][wl][1] = hi;
    __syncthreads();
    uint32_t plo = 0, phi = 0;
    for (uint32_t j = 0; j < sl; j++) {
        plo += part[j][wl][0];
        phi += part[j][wl][1];
    }
    const uint32_t b0 = 2u * w, b1 = b0 + 1u;
#pragma unroll
    for (uint32_t k = 0; k < kTileSliceMax; k++) {
        if (k < S && t0 + k < T) {
            uint32_t* pre = ws.tpre + (size_t)(t0 + k) * nb;
            if (b1 < nb)
                *reinterpret_cast<uint2*>(pre + b0) = make_uint2(plo, phi);  // (nb even: 8 (max_keys + 1))
            else if (b0 < nb)
                pre[b0] = plo;
        }
        plo += v[k] & 0xFFFFu;
        phi += v[k] >> 16;
    }
    if (sl == kTileSlices - 1u) {  // its running sums now hold every tile's
        if (b0 < nb) ws.hist[b0] = plo;
        if (b1 < nb) ws.hist[b1] = phi;
    }
}

// pass 4: packet i to its bin's range, after the earlier tiles' packets of that bin. The tile's
// offsets are read at random from its row of tpre, so the workgroups of one tile run on one XCD
// (blockIdx mod 8, a placement observed, not promised: it only decides which L2 caches the row):
// XCD slot x takes tiles x, x + 8, …, each row then pulled into one L2 instead of all eight (P is a
// multiple of 256, so a workgroup's 256 packets lie in one tile).
// With fewer than 8 tiles the XCD slots past T would get no work: the pieces are then dealt to the
// whole grid instead (every workgroup strides over all T · P / 256 of them).
__global__ void sched_tile_scatter_kernel(SchedWs ws, uint32_t n, const uint32_t* dn, uint32_t P, uint32_t nb, uint32_t T) {
    if (dn) n = min(n, *dn);
    const bool flat = T < 8u;
    const uint32_t x = flat ? 0u : blockIdx.x & 7u, per_tile = P >> 8;
    const uint32_t xs = flat ? 1u : 8u;  // tiles between one slot's consecutive tiles
    // workgroup-sized pieces of XCD slot x (flat: of every tile)
    const uint32_t mine = (flat ? T : (T > x ? (T - x + 7u) >> 3 : 0u)) * per_tile;
    for (uint32_t k = flat ? blockIdx.x : blockIdx.x >> 3; k < mine; k += flat ? gridDim.x : gridDim.x >> 3) {
        const uint32_t t = x + xs * (k / per_tile);
        const uint32_t i = t * P + (k % per_tile) * 256u + threadIdx.x;
        if (i < n) {
            const uint32_t b = ws.binof[i];
            ws.sorted[ws.base[b] + ws.tpre[(size_t)t * nb + b] + ws.binpos[i]] = i;
        }
    }
}

// Descriptors of a shard whose engine disagrees with engine 0 on some key slots (engine.cpp
// KeyFence): copied with those packets' key_id pointing past every key table, so the batch kernels
// give them NEB_STATUS_BAD_KEY instead of sealing with another tunnel's key.
__global__ void fence_keys_kernel(const neb_desc* __restrict__ in, neb_desc* __restrict__ out, uint32_t n,
                                  const uint8_t* __restrict__ bad, uint32_t nbad) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        neb_desc d = in[i];
        if (d.key_id < nbad && bad[d.key_id]) d.key_id = NEB_KEYS_MIXED - 1u;
        out[i] = d;
    }
}

}  // namespace neb

extern "C" hipError_t neb_fence_keys(const neb_desc* in, neb_desc* out, uint32_t n, const uint8_t* bad, uint32_t nbad,
                                     hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t g = (n + 255u) / 256u < 1024u ? (n + 255u) / 256u : 1024u;
    hipLaunchKernelGGL(neb::fence_keys_kernel, dim3(g), dim3(256), 0, s, in, out, n, bad, nbad);
    return hipGetLastError();
}

// The counting pass's LDS above the default 64 KiB, asked for once per device (an engine per GPU
// in one process); a device that refuses it bins through the atomic histogram.
static bool tile_lds_granted() {
    constexpr int kMaxDevices = 64;
    static std::atomic<int> state[kMaxDevices];  // 0 not asked, 1 granted, -1 refused
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return false;
    int st = state[dev].load(std::memory_order_relaxed);
    if (st == 0) {
        st = hipFuncSetAttribute((const void*)neb::sched_tile_hist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)neb::kTileLdsMax) == hipSuccess ? 1 : -1;
        if (st < 0) (void)hipGetLastError();  // (not the batch's error: it bins the other way)
        state[dev].store(st, std::memory_order_relaxed);
    }
    return st > 0;
}

extern "C" hipError_t neb_sched_build(const neb_desc* d_desc, uint32_t n, const uint32_t* d_n, uint32_t max_keys,
                                      uint32_t lpp, const neb::SchedWs* ws, hipStream_t s) {
    const uint32_t nb = neb::sched_nbins(max_keys);
    const uint32_t tpb = 256;
    const uint32_t gp = (n + tpb - 1) / tpb < 4096u ? (n + tpb - 1) / tpb : 4096u;
    const dim3 ga((nb + neb::kAllocThreadsSched - 1) / neb::kAllocThreadsSched), ta(neb::kAllocThreadsSched);
    // NEB_KNOB_SUB_BINS_FROM (per batch): the A/B of the threshold, and the tests' coverage of both
    // counting layouts
    const int64_t from = neb::knob(NEB_KNOB_SUB_BINS_FROM);
    const uint32_t words = neb::sched_tile_words(nb);
    const uint32_t T = std::min<uint32_t>(neb::kTileMax, (n + neb::kTileMinPkts - 1) / neb::kTileMinPkts);
    const uint32_t P = T ? ((n + T - 1) / T + 255u) & ~255u : 0u;  // (whole workgroups of the scatter)
    if (n && ws->tcnt && (int64_t)n >= neb::knob(NEB_KNOB_TILE_BINS_FROM) && words * 4u <= neb::kTileLdsMax &&
        P <= 0xFFFFu && tile_lds_granted()) {
        hipLaunchKernelGGL(neb::sched_tile_hist_kernel, dim3(T), dim3(neb::kTileThreads), words * 4u, s, d_desc, n, d_n,
                           max_keys, lpp, *ws, P, words);
        hipLaunchKernelGGL(neb::sched_tile_scan_kernel, dim3(words / 16u), dim3(256), 0, s, *ws, T, words, nb);
        hipLaunchKernelGGL(neb::sched_alloc_kernel<1>, ga, ta, 0, s, max_keys, *ws);
        hipLaunchKernelGGL(neb::sched_tile_scatter_kernel, dim3(std::max<uint32_t>(8u, gp & ~7u)), dim3(tpb), 0, s, *ws,
                           n, d_n, P, nb, T);
        return hipGetLastError();
    }
    if ((int64_t)n >= from) {
        hipLaunchKernelGGL(neb::sched_hist_kernel<neb::kSubBins>, dim3(gp), dim3(tpb), 0, s, d_desc, n, d_n, max_keys, lpp,
                           *ws);
        hipLaunchKernelGGL(neb::sched_alloc_kernel<neb::kSubBins>, ga, ta, 0, s, max_keys, *ws);
    } else {
        hipLaunchKernelGGL(neb::sched_hist_kernel<1>, dim3(gp), dim3(tpb), 0, s, d_desc, n, d_n, max_keys, lpp, *ws);
        hipLaunchKernelGGL(neb::sched_alloc_kernel<1>, ga, ta, 0, s, max_keys, *ws);
    }
    hipLaunchKernelGGL(neb::sched_scatter_kernel, dim3(gp), dim3(tpb), 0, s, d_desc, n, d_n, *ws);
    return hipGetLastError();
}
