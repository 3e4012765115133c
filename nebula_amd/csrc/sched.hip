// sched.hip — device-side binning of a batch into single-key, similar-size chunks (sched.hpp).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

template <uint32_t SUB>
__global__ __launch_bounds__(kAllocThreads) void sched_alloc_kernel(uint32_t max_keys, SchedWs ws) {
    __shared__ SchedAllocLds<SUB> sl;
    sched_alloc_block<SUB>(max_keys, ws, blockIdx.x, sl);
}

__global__ void sched_scatter_kernel(const neb_desc* __restrict__ desc, uint32_t n, const uint32_t* dn, SchedWs ws) {
    if (dn) n = min(n, *dn);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) sched_scatter_one(ws, i);
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

extern "C" hipError_t neb_sched_build(const neb_desc* d_desc, uint32_t n, const uint32_t* d_n, uint32_t max_keys,
                                      uint32_t lpp, const neb::SchedWs* ws, hipStream_t s) {
    const uint32_t nb = neb::sched_nbins(max_keys);
    const uint32_t tpb = 256;
    const uint32_t gp = (n + tpb - 1) / tpb < 4096u ? (n + tpb - 1) / tpb : 4096u;
    const dim3 ga((nb + neb::kAllocThreads - 1) / neb::kAllocThreads), ta(neb::kAllocThreads);
    // NEB_KNOB_SUB_BINS_FROM (per batch): the A/B of the threshold, and the tests' coverage of both
    // counting layouts
    const int64_t from = neb::knob(NEB_KNOB_SUB_BINS_FROM);
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
