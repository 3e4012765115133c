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

// 16 bytes at a 4-byte aligned address: one global_load_dwordx4 (gfx950 needs dword alignment only)
struct alignas(4) U4a4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ uint4 load_u4_a4(const uint8_t* p) {
    const U4a4 v = *reinterpret_cast<const U4a4*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void store_u4_a4(uint8_t* p, uint4 v) {
    *reinterpret_cast<U4a4*>(p) = U4a4{v.x, v.y, v.z, v.w};
}

// 16 bytes at any byte address p from the two aligned 16-byte blocks that hold them (never beyond
// the aligned block of the last byte read, so never into another page).
__device__ __forceinline__ uint4 load_shifted16(const uint8_t* p) {
    const uint32_t s = (uint32_t)reinterpret_cast<uintptr_t>(p) & 15u;
    const uint4* a = reinterpret_cast<const uint4*>(p - s);
    const uint4 lo = a[0];
    uint4 hi = make_uint4(0, 0, 0, 0);
    if (s) hi = a[1];
    const uint32_t q = s >> 2, r = 8u * (s & 3u);
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    uint32_t t[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; k++)
        t[k] = q == 0u ? w[k] : q == 1u ? w[k + 1] : q == 2u ? w[k + 2] : w[k + 3];
    return make_uint4(__builtin_amdgcn_alignbit(t[1], t[0], r), __builtin_amdgcn_alignbit(t[2], t[1], r),
                      __builtin_amdgcn_alignbit(t[3], t[2], r), __builtin_amdgcn_alignbit(t[4], t[3], r));
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

// Block of n bytes (1..16) whose first h bytes come from hp and the rest from sp (the TX seal's
// plaintext: the patched L3/L4 header image in the output slot, the payload in the TUN read).
__device__ __forceinline__ uint4 load_block_hdr(const uint8_t* hp, const uint8_t* sp, uint32_t n, uint32_t h) {
    if (h >= n) return load_block(hp, n);
    const uint4 a = load_block(hp, h);
    const uint4 b = load_block(sp, n);
    const uint4 bh = mask_block(b, h);
    return make_uint4(a.x | (b.x ^ bh.x), a.y | (b.y ^ bh.y), a.z | (b.z ^ bh.z), a.w | (b.w ^ bh.w));
}

// The per-packet kernels' last step (aes_gcm.hip gcm_one_kernel, chacha_poly.hip chacha_one_kernel):
// every result store of the wave released at system scope (s_waitcnt + L2 write-back: the host
// reads the result straight from its pinned slot), then the status, staged in LDS by the packet's
// last lane, as one system-scope store. The host polls that word (engine.cpp one_packet).
__device__ __forceinline__ void one_publish_status(int32_t* host_status, const int32_t* staged) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the staging lane's LDS store, wave-wide
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int32_t st = *staged;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the result stores are visible first
    if (__lane_id() == 0) __hip_atomic_store(host_status, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace neb
