// sched.hip — device-side binning of a batch into single-key, similar-size chunks (sched.hpp).
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

// pass 1: histogram of (size class, key) bins; keys outside the table go to key index max_keys
__global__ void sched_hist_kernel(const neb_desc* __restrict__ desc, uint32_t n, const uint32_t* dn,
                                  uint32_t max_keys, uint32_t lpp, SchedWs ws) {
    if (dn) n = min(n, *dn);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const neb_desc d = desc[i];
        const uint32_t key = d.key_id < max_keys ? d.key_id : max_keys;
        const uint32_t b = size_class(d, lpp) * (max_keys + 1u) + key;
        ws.binof[i] = b;
        atomicAdd(&ws.hist[b], 1u);
    }
}

// pass 2: every non-empty bin reserves its range of `sorted` and its chunks
__global__ void sched_alloc_kernel(uint32_t max_keys, SchedWs ws) {
    const uint32_t nb = sched_nbins(max_keys);
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x) {
        const uint32_t c = ws.hist[b];
        if (c == 0u) continue;
        const uint32_t base = atomicAdd(&ws.counters[kCntPackets], c);
        ws.base[b] = base;
        const uint32_t key = b % (max_keys + 1u), cls = b / (max_keys + 1u);
        const uint32_t nfull = c / kChunkPkts, tail = c % kChunkPkts;
        // chunks at 4 lanes per packet (the long ones) from the front, the short tails from the
        // back: the crypto kernel takes them in that order. Front <= n/16 + bins, back <= bins and
        // front + back <= n/16 + min(n, bins): the ranges never meet inside max_chunks
        // (sched_max_chunks).
        if (nfull) {
            const uint32_t cb = atomicAdd(&ws.counters[kCntFrontChunks], nfull);
            for (uint32_t j = 0; j < nfull && cb + j < ws.max_chunks; j++)
                ws.chunks[cb + j] = make_uint4(base + j * kChunkPkts, kChunkPkts, key, cls | (2u << kChunkLgShift));
        }
        if (tail) {
            const uint32_t lg = sched_tail_lg(tail, cls);
            const uint4 ch = make_uint4(base + nfull * kChunkPkts, tail, key, cls | (lg << kChunkLgShift));
            if (lg == 2u) {
                const uint32_t t = atomicAdd(&ws.counters[kCntFrontChunks], 1u);
                if (t < ws.max_chunks) ws.chunks[t] = ch;
            } else {
                const uint32_t t = atomicAdd(&ws.counters[kCntBackChunks], 1u);
                if (t < ws.max_chunks) ws.chunks[ws.max_chunks - 1u - t] = ch;
            }
        }
    }
}

// pass 3: scatter packet indices into their bin's range
__global__ void sched_scatter_kernel(uint32_t n, const uint32_t* dn, SchedWs ws) {
    if (dn) n = min(n, *dn);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t b = ws.binof[i];
        const uint32_t pos = atomicAdd(&ws.fill[b], 1u);
        ws.sorted[ws.base[b] + pos] = i;
    }
}

}  // namespace neb

extern "C" hipError_t neb_sched_build(const neb_desc* d_desc, uint32_t n, const uint32_t* d_n, uint32_t max_keys,
                                      uint32_t lpp, const neb::SchedWs* ws, hipStream_t s) {
    const uint32_t nb = neb::sched_nbins(max_keys);
    // counters, hist and fill are contiguous: one memset per batch
    hipError_t e = hipMemsetAsync(ws->counters, 0, (neb::kSchedCounters + 2u * nb) * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t tpb = 256;
    const uint32_t gp = (n + tpb - 1) / tpb < 4096u ? (n + tpb - 1) / tpb : 4096u;
    const uint32_t gb = (nb + tpb - 1) / tpb < 4096u ? (nb + tpb - 1) / tpb : 4096u;
    hipLaunchKernelGGL(neb::sched_hist_kernel, dim3(gp), dim3(tpb), 0, s, d_desc, n, d_n, max_keys, lpp, *ws);
    hipLaunchKernelGGL(neb::sched_alloc_kernel, dim3(gb), dim3(tpb), 0, s, max_keys, *ws);
    hipLaunchKernelGGL(neb::sched_scatter_kernel, dim3(gp), dim3(tpb), 0, s, n, d_n, *ws);
    return hipGetLastError();
}
