// timing.hpp — dispatch-bound kernel timing for the benchmark (neb_time_next_kernel).
//
// A timing event recorded on the stream around a kernel is a marker packet of its own, and its cost
// lands inside the bracket (≈ 3.5 µs per marker here) and between the batches. hipExtLaunchKernel
// instead binds a start and a stop event to one dispatch: they carry that kernel's own begin and end
// and add no packet. A caller arms one pair for the next batch its thread launches; the batch binds
// it to its dominant kernel (the single-key kernel, the mixed-key chunk kernel, the ChaCha kernel)
// and records a key-use event it would have bound there as a marker after it instead.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace neb {

struct KernelTiming {
    hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local KernelTiming g_kernel_timing;  // engine.cpp
extern thread_local const void* g_timed_kernel;    // engine.cpp: the kernel the last armed pair went to

// launch `kern` on s with the armed timing pair (consumed) or `stop` bound to it; with a timing pair
// armed, `stop` is recorded after the kernel
template <class K, class... A>
inline hipError_t launch_bound(K kern, dim3 grid, dim3 block, hipStream_t s, hipEvent_t stop, A... args) {
    const KernelTiming t = g_kernel_timing;
    if (t.start && t.stop) {
        g_kernel_timing = {};
        g_timed_kernel = reinterpret_cast<const void*>(kern);
        hipExtLaunchKernelGGL(kern, grid, block, 0, s, t.start, t.stop, 0, args...);
        hipError_t err = hipGetLastError();
        if (err == hipSuccess && stop) err = hipEventRecord(stop, s);
        return err;
    }
    if (stop) hipExtLaunchKernelGGL(kern, grid, block, 0, s, nullptr, stop, 0, args...);
    else hipLaunchKernelGGL(kern, grid, block, 0, s, args...);
    return hipGetLastError();
}

}  // namespace neb
