// sched.hpp — batch scheduling for mixed-key / mixed-size batches (shared by the AEAD kernels).
//
// A batch with many tunnel keys and mixed packet sizes is regrouped on the device before the
// crypto kernel runs: packets are binned by (size class, key) with global atomics, each bin is
// cut into chunks of at most kChunkPkts packets, and one wavefront processes one chunk. Inside a
// chunk the key is wave-uniform (round keys in scalar registers, one set of GHASH tables) and the
// packets need a similar number of rounds, so lanes neither diverge on keys nor idle on sizes.
// No prefix scan is needed: bins reserve their output ranges with an atomic cursor, so the order
// of bins (and of packets inside a bin) is arbitrary — every packet's result is independent of it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"

namespace neb {

constexpr uint32_t kChunkPkts = 16;   // packets per wavefront (4 lanes each)
constexpr uint32_t kSizeClasses = 8;  // round-count classes: 1, 2, 3-4, 5-8, 9-16, 17-32, 33-64, 65+

struct SchedWs {          // device workspace, sized for n packets and nbins bins
    uint32_t* counters;   // [0] packet cursor, [1] chunk count, then hist[nbins], fill[nbins]
    uint32_t* hist;
    uint32_t* fill;
    uint32_t* base;       // [nbins] output offset of each non-empty bin
    uint32_t* binof;      // [n] bin of each packet
    uint32_t* sorted;     // [n] packet indices, bin-contiguous
    uint4* chunks;        // [max_chunks] {start in sorted, count, key_id, size class}
    uint32_t max_chunks;
};

__host__ __device__ inline uint32_t sched_nbins(uint32_t max_keys) { return kSizeClasses * (max_keys + 1u); }
__host__ __device__ inline uint32_t sched_max_chunks(uint32_t n, uint32_t max_keys) {
    const uint32_t nb = sched_nbins(max_keys);
    return (n + kChunkPkts - 1u) / kChunkPkts + (n < nb ? n : nb);
}

}  // namespace neb

// Host launcher (sched.hip): zero the counters and run the three binning passes on stream s.
extern "C" hipError_t neb_sched_build(const neb_desc* d_desc, uint32_t n, const uint32_t* d_n, uint32_t max_keys,
                                      uint32_t lpp, const neb::SchedWs* ws, hipStream_t s);
