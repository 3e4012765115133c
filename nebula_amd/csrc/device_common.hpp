// device_common.hpp — byte/word helpers shared by the gfx950 AEAD kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace neb {

constexpr int kWave = 64;

// v_perm_b32: byte i of the result = selector byte i picking from {b bytes 0-3 (0..3), a bytes 0-3 (4..7)},
// 0x0C = 0x00.
__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
    return __builtin_amdgcn_perm(a, b, sel);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }
// rotate right by s (v_alignbit_b32)
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t s) { return __builtin_amdgcn_alignbit(x, x, s); }
// ({hi,lo} >> s)[31:0]
__device__ __forceinline__ uint32_t shr64(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }

// Load `n` (1..16) bytes at p as four little-endian dwords, zero-filling the rest.
__device__ __forceinline__ uint4 load_block(const uint8_t* p, uint32_t n) {
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (n == 16) {
        if ((a & 15) == 0) return *reinterpret_cast<const uint4*>(p);
        if ((a & 3) == 0) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
            return make_uint4(q[0], q[1], q[2], q[3]);
        }
    }
    uint32_t w[4] = {0, 0, 0, 0};
    if ((a & 3) == 0) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
        uint32_t full = n >> 2;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (i < full) w[i] = q[i];
        for (uint32_t i = full << 2; i < n; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    } else {
        for (uint32_t i = 0; i < n; i++) w[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Store the first `n` (1..16) bytes of four little-endian dwords at p.
__device__ __forceinline__ void store_block(uint8_t* p, uint4 v, uint32_t n) {
    uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (n == 16) {
        if ((a & 15) == 0) {
            *reinterpret_cast<uint4*>(p) = v;
            return;
        }
        if ((a & 3) == 0) {
            uint32_t* q = reinterpret_cast<uint32_t*>(p);
            q[0] = v.x; q[1] = v.y; q[2] = v.z; q[3] = v.w;
            return;
        }
    }
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if ((a & 3) == 0) {
        uint32_t* q = reinterpret_cast<uint32_t*>(p);
        uint32_t full = n >> 2;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (i < full) q[i] = w[i];
        for (uint32_t i = full << 2; i < n; i++) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    } else {
        for (uint32_t i = 0; i < n; i++) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// Keep the first n bytes (0..16) of a little-endian block, zero the rest.
__device__ __forceinline__ uint4 mask_block(uint4 v, uint32_t n) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        int32_t keep = (int32_t)n - (int32_t)(4 * i);
        uint32_t m = keep >= 4 ? 0xFFFFFFFFu : (keep <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * keep)));
        w[i] &= m;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace neb
