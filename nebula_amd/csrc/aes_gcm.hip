// aes_gcm.hip — AES-256-GCM seal/open of a packet batch on gfx950 (MI355X).
//
// Replaces the arithmetic behind noiseutil/aesgcm.go:24-49 (EncryptDanger/DecryptDanger = Go
// crypto/cipher GCM Seal/Open with nonce 00000000 || BE64(n)) for a whole batch of packets.
//
// Work decomposition:
//  * A "packet group" is 64 / LPP packets of one wave, LPP = 2^lg lanes each (4 in the single-key
//    kernel and in full mixed-key chunks; 8 or 16 for short tail chunks; 64 in the tail kernel).
//  * A packet's GHASH input is n = a + m + 1 blocks (a AAD blocks, m ciphertext blocks, 1 length
//    block), front-padded with zero blocks to n' = LPP·R. In round r lane l owns padded block
//    g' = LPP·r + l + 1: it runs the AES-CTR keystream for that block (if it is a ciphertext block),
//    loads / XORs / stores the 16 payload bytes, and folds the block into its Horner accumulator
//    A_l = A_l·H^LPP ⊕ X. The length block always lands on the packet's last lane; that lane also
//    computes E_K(J0) for the tag.
//  * After R rounds GHASH = Σ_l A_l·H^(LPP-l): one multiply per lane after a lane permutation
//    (LPP 4), or a pairwise tree (LPP 8-64).
//  * AES: T-tables in LDS, 32 swizzled copies so every ds_read_b32 is bank-conflict-free and its
//    address is one v_perm_b32 (four tables, 128 KiB, in the single-key kernel; two tables, 64 KiB,
//    T1/T3 by one rotate, elsewhere). Round keys are wave-uniform (scalar registers).
//  * GHASH tables (precomputed at key install): a reduction-free "full" nibble table of H^4, and
//    position / Shoup tables of the other powers, staged in LDS per workgroup (one key) or per
//    wave and chunk (mixed keys).
#include <hip/hip_runtime.h>

#include <atomic>
#include <hip/hip_ext.h>

#include <cstdlib>
#include <cstring>
#include <stdint.h>

#include <type_traits>

#include "../../include/nebula_aead.h"
#include "device_common.hpp"
#include "knobs.hpp"
#include "layout.hpp"
#include "rxwin.hpp"
#include "sched.hpp"
#include "timing.hpp"

// ISA region markers for tools/r6/isa_regions.py (an analysis build only: -DNEB_ISA_MARKS)
#ifdef NEB_ISA_MARKS
#define NEB_MARK(x) asm volatile(";NEBMARK " #x)
#else
#define NEB_MARK(x) ((void)0)
#endif

namespace neb {

// ------------------------------------------------------------------------------------------
// AES tables (FIPS-197 S-box) — T0 in little-endian column form: bytes [2S, S, S, 3S].

struct T0Table {
    uint32_t t[256];
};
constexpr uint8_t kSbox[256] = {
    0x63,0x7c,0x77,0x7b,0xf2,0x6b,0x6f,0xc5,0x30,0x01,0x67,0x2b,0xfe,0xd7,0xab,0x76,
    0xca,0x82,0xc9,0x7d,0xfa,0x59,0x47,0xf0,0xad,0xd4,0xa2,0xaf,0x9c,0xa4,0x72,0xc0,
    0xb7,0xfd,0x93,0x26,0x36,0x3f,0xf7,0xcc,0x34,0xa5,0xe5,0xf1,0x71,0xd8,0x31,0x15,
    0x04,0xc7,0x23,0xc3,0x18,0x96,0x05,0x9a,0x07,0x12,0x80,0xe2,0xeb,0x27,0xb2,0x75,
    0x09,0x83,0x2c,0x1a,0x1b,0x6e,0x5a,0xa0,0x52,0x3b,0xd6,0xb3,0x29,0xe3,0x2f,0x84,
    0x53,0xd1,0x00,0xed,0x20,0xfc,0xb1,0x5b,0x6a,0xcb,0xbe,0x39,0x4a,0x4c,0x58,0xcf,
    0xd0,0xef,0xaa,0xfb,0x43,0x4d,0x33,0x85,0x45,0xf9,0x02,0x7f,0x50,0x3c,0x9f,0xa8,
    0x51,0xa3,0x40,0x8f,0x92,0x9d,0x38,0xf5,0xbc,0xb6,0xda,0x21,0x10,0xff,0xf3,0xd2,
    0xcd,0x0c,0x13,0xec,0x5f,0x97,0x44,0x17,0xc4,0xa7,0x7e,0x3d,0x64,0x5d,0x19,0x73,
    0x60,0x81,0x4f,0xdc,0x22,0x2a,0x90,0x88,0x46,0xee,0xb8,0x14,0xde,0x5e,0x0b,0xdb,
    0xe0,0x32,0x3a,0x0a,0x49,0x06,0x24,0x5c,0xc2,0xd3,0xac,0x62,0x91,0x95,0xe4,0x79,
    0xe7,0xc8,0x37,0x6d,0x8d,0xd5,0x4e,0xa9,0x6c,0x56,0xf4,0xea,0x65,0x7a,0xae,0x08,
    0xba,0x78,0x25,0x2e,0x1c,0xa6,0xb4,0xc6,0xe8,0xdd,0x74,0x1f,0x4b,0xbd,0x8b,0x8a,
    0x70,0x3e,0xb5,0x66,0x48,0x03,0xf6,0x0e,0x61,0x35,0x57,0xb9,0x86,0xc1,0x1d,0x9e,
    0xe1,0xf8,0x98,0x11,0x69,0xd9,0x8e,0x94,0x9b,0x1e,0x87,0xe9,0xce,0x55,0x28,0xdf,
    0x8c,0xa1,0x89,0x0d,0xbf,0xe6,0x42,0x68,0x41,0x99,0x2d,0x0f,0xb0,0x54,0xbb,0x16};

constexpr uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
constexpr T0Table make_t0() {
    T0Table r{};
    for (int i = 0; i < 256; i++) {
        uint32_t s = kSbox[i], s2 = xt(kSbox[i]), s3 = s2 ^ s;
        r.t[i] = s2 | (s << 8) | (s << 16) | (s3 << 24);
    }
    return r;
}
__constant__ T0Table c_T0 = make_t0();

// ------------------------------------------------------------------------------------------
// Instruction helpers

// Three-input XOR in one VALU op. gfx950 has no v_xor3_b32; its v_bitop3_b32 evaluates any
// 3-input truth table (0x96 = a ^ b ^ c), but hipcc does not form it from a ^ b ^ c chains.
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// same, third operand wave-uniform (a round key in an SGPR)
__device__ __forceinline__ uint32_t x3s(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 x34(uint4 a, uint4 b, uint4 c) {
    return make_uint4(x3(a.x, b.x, c.x), x3(a.y, b.y, c.y), x3(a.z, b.z, c.z), x3(a.w, b.w, c.w));
}
__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
    return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
__device__ __forceinline__ uint4 bswap4(uint4 v) { return make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w)); }
__device__ __forceinline__ uint4 shfl_xor4(uint4 v, int m) {
    return make_uint4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}
// byte k of w, zero-extended (one VALU op)
__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) {
    return k == 0 ? (w & 0xFFu) : (k == 3 ? (w >> 24) : __builtin_amdgcn_ubfe(w, 8 * k, 8));
}

template <class T>
__device__ __forceinline__ T lds_at(const void* base, uint32_t byte_off) {
    // every table offset is a multiple of sizeof(T): say so, or 16-byte reads get split into
    // ds_read2/b96 pieces that conflict
    return *reinterpret_cast<const T*>(
        __builtin_assume_aligned(reinterpret_cast<const char*>(base) + byte_off, sizeof(T)));
}

// ------------------------------------------------------------------------------------------
// AES-256 encryption of one block per lane (little-endian column words in and out).
// ttab: LDS, 32 copies of 256 8-byte entries, entry x of copy c at byte x*256 + c*8 holding
// (T0[x], T2[x]) for c < 16 and (T2[x], T0[x]) for c >= 16, T2 = rotl16(T0). Lane l uses copy
// c = l mod 32 and reads single dwords: T0 at lb.x = 8c + 4(c >= 16), T2 at lb.y = 8c + 4(c < 16).
// A ds_read_b32 banks on (addr/4) mod 32, so the 32 lanes of a half-wave hit dwords 2c + {0,1}
// arranged to be 32 distinct banks: every lookup is conflict-free.
// high: added to both lane bases (bit 16 when the table sits at LDS byte 65536 + an offset-field
// constant, so every lookup address is still one v_perm: its byte 2 comes from the lane base)
__device__ __forceinline__ uint2 ttab_lane_base(uint32_t lane, uint32_t high = 0u) {
    const uint32_t c = lane & 31u, hi = c >> 4;
    return make_uint2((c << 3) | (hi << 2) | high, (c << 3) | ((hi ^ 1u) << 2) | high);
}
__device__ __forceinline__ uint2 ttab_entry(uint32_t i) {  // i = x*32 + c
    const uint32_t t = c_T0.t[i >> 5], t2 = __builtin_amdgcn_alignbit(t, t, 16);
    return (i & 16u) ? make_uint2(t2, t) : make_uint2(t, t2);
}

// Wave priority while a round's 16 lookups are issued (s_setprio): the SIMD arbiter then prefers
// the wave that feeds the LDS over waves busy with their XOR phase, which keeps the LDS queue
// full. Measured on C2: 0.150 -> 0.136 ms per seal launch (priority 1, 2 and 3 alike; raising it
// for the GHASH lookups as well was slower). NEB_PRIO=0 disables it.
#ifndef NEB_PRIO
#define NEB_PRIO 3
#endif
#ifndef NEB_PRIO_AGE  // gcm_single_kernel: the younger half of each SIMD's waves at 1 between lookups
#define NEB_PRIO_AGE 1
#endif

struct RkRegs {  // wave-uniform round keys (scalar registers)
    const uint32_t* k;
    static constexpr bool kUniform = true;
    // s_setprio levels around a round's lookups (kPrioHi) and after them (kPrioLo)
    static constexpr int kPrioHi = NEB_PRIO, kPrioLo = 0;
    __device__ __forceinline__ uint4 get(int r) const {
        return make_uint4(k[4 * r], k[4 * r + 1], k[4 * r + 2], k[4 * r + 3]);
    }
};
// The same keys with the priority levels of one age rank (gcm_single_kernel: the SIMD arbiter
// prefers a SIMD's older waves at equal priority, §3.1)
template <int HI, int LO>
struct RkRegsPrio : RkRegs {
    static constexpr int kPrioHi = HI, kPrioLo = LO;
};
struct RkLds {  // per-packet round keys staged in LDS
    const uint4* base;
    static constexpr bool kUniform = false;
    static constexpr int kPrioHi = NEB_PRIO, kPrioLo = 0;
    __device__ __forceinline__ uint4 get(int r) const { return base[r]; }
};

// T-table lookups: T0[byte k of s], T2[byte k of s] (T1 = rotl8 T0, T3 = rotl8 T2).
struct TLook {
    const uint2* ttab;
    uint2 lb;
    __device__ __forceinline__ uint32_t t0(uint32_t s, int k) const {
        return lds_at<uint32_t>(ttab, perm(s, lb.x, 0x0C020000u | ((4u + (uint32_t)k) << 8)));
    }
    __device__ __forceinline__ uint32_t t2(uint32_t s, int k) const {
        return lds_at<uint32_t>(ttab, perm(s, lb.y, 0x0C020000u | ((4u + (uint32_t)k) << 8)));
    }
    __device__ __forceinline__ uint32_t t1(uint32_t s, int k) const { return rotl8(t0(s, k)); }
    __device__ __forceinline__ uint32_t t3(uint32_t s, int k) const { return rotl8(t2(s, k)); }
    // the round's row-1/row-3 lookups before their rotation (one rotate per column, below)
    __device__ __forceinline__ uint32_t t1r(uint32_t s, int k) const { return t0(s, k); }
    __device__ __forceinline__ uint32_t t3r(uint32_t s, int k) const { return t2(s, k); }
    static constexpr bool kFour = false;
};

// Four T-tables (T0..T3) in LDS, 128 KiB: region A (byte offset 0) holds the pairs (T0[x], T1[x]),
// region B (offset 64 KiB) the pairs (T2[x], T3[x]), each laid out and swizzled like TLook's
// (32 copies, copy c of entry x at x*256 + c*8, the two dwords swapped for c >= 16). A round then
// combines each column with two XOR3s and no rotates (8 VALU per round fewer than TLook), at
// the price of one 1024-lane workgroup per CU. One lane base serves all four tables: byte 0 =
// the lane's row-0/row-2 dword offset in its 256-byte row, byte 3 = its row-1/row-3 dword offset,
// byte 2 = 1 (region B); each lookup's v_perm picks byte 0 or 3 and zero or byte 2.
__device__ __forceinline__ uint32_t ttab4_lane_base(uint32_t lane) {
    const uint32_t c = lane & 31u, hi = c >> 4;
    return ((c << 3) | (hi << 2)) | (1u << 16) | (((c << 3) | ((hi ^ 1u) << 2)) << 24);
}
__device__ __forceinline__ uint2 ttab4_entry(uint32_t i) {  // i = region*8192 + x*32 + c
    uint32_t t = c_T0.t[(i >> 5) & 255u];
    if (i & 8192u) t = __builtin_amdgcn_alignbit(t, t, 16);  // T2 = rotl16 T0
    const uint32_t t1 = rotl8(t);                            // T1 = rotl8 T0, T3 = rotl8 T2
    return (i & 16u) ? make_uint2(t1, t) : make_uint2(t, t1);
}
// Write N entries of an LDS T-table image with THREADS threads: every source word is loaded
// before any is stored, so the prologue pays one global-load latency instead of one per entry (a
// strided loop left a load + vmcnt(0) + store per iteration: 16 serialised L2 round trips).
template <uint32_t N, uint32_t THREADS, class F>
__device__ __forceinline__ void fill_ttab(uint2* dst, uint32_t tid, F entry) {
    constexpr uint32_t K = (N + THREADS - 1) / THREADS;
    constexpr bool kWhole = N % THREADS == 0;
    uint2 v[K];
#pragma unroll
    for (uint32_t j = 0; j < K; j++) v[j] = entry((tid + j * THREADS) % N);
#pragma unroll
    for (uint32_t j = 0; j < K; j++)
        if (kWhole || tid + j * THREADS < N) dst[tid + j * THREADS] = v[j];
}
struct TLook4 {
    const uint2* ttab;
    uint32_t lb;
    __device__ __forceinline__ uint32_t at(uint32_t s, int k, uint32_t sel) const {
        return lds_at<uint32_t>(ttab, perm(s, lb, sel | ((4u + (uint32_t)k) << 8)));
    }
    __device__ __forceinline__ uint32_t t0(uint32_t s, int k) const { return at(s, k, 0x0C0C0000u); }
    __device__ __forceinline__ uint32_t t1(uint32_t s, int k) const { return at(s, k, 0x0C0C0003u); }
    __device__ __forceinline__ uint32_t t2(uint32_t s, int k) const { return at(s, k, 0x0C020000u); }
    __device__ __forceinline__ uint32_t t3(uint32_t s, int k) const { return at(s, k, 0x0C020003u); }
    __device__ __forceinline__ uint32_t t1r(uint32_t s, int k) const { return t1(s, k); }
    __device__ __forceinline__ uint32_t t3r(uint32_t s, int k) const { return t3(s, k); }
    static constexpr bool kFour = true;
};

// AES-256 rounds FIRST..13 (full) and 14 (final) on the state s0..s3 (after round FIRST-1).
template <int FIRST, class TL, class RK>
__device__ __forceinline__ uint4 aes256_rounds(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, const TL& T,
                                               const RK& rk) {
    uint4 k;
#pragma unroll
    for (int r = FIRST; r < 14; r++) {
        k = rk.get(r);
#if NEB_PRIO
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(RK::kPrioHi);
#endif
        const uint32_t a0 = T.t0(s0, 0), a1 = T.t1r(s1, 1), a2 = T.t2(s2, 2), a3 = T.t3r(s3, 3);
        const uint32_t b0 = T.t0(s1, 0), b1 = T.t1r(s2, 1), b2 = T.t2(s3, 2), b3 = T.t3r(s0, 3);
        const uint32_t c0 = T.t0(s2, 0), c1 = T.t1r(s3, 1), c2 = T.t2(s0, 2), c3 = T.t3r(s1, 3);
        const uint32_t d0 = T.t0(s3, 0), d1 = T.t1r(s0, 1), d2 = T.t2(s1, 2), d3 = T.t3r(s2, 3);
#if NEB_PRIO
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(RK::kPrioLo);
#endif
        // T0[a] ^ T1[b] ^ T2[c] ^ T3[d] ^ k; with two tables T1 = rotl8 T0, T3 = rotl8 T2
        if constexpr (TL::kFour) {
            if constexpr (RK::kUniform) {
                s0 = x3s(x3(a0, a1, a2), a3, k.x);
                s1 = x3s(x3(b0, b1, b2), b3, k.y);
                s2 = x3s(x3(c0, c1, c2), c3, k.z);
                s3 = x3s(x3(d0, d1, d2), d3, k.w);
            } else {
                s0 = x3(x3(a0, a1, a2), a3, k.x);
                s1 = x3(x3(b0, b1, b2), b3, k.y);
                s2 = x3(x3(c0, c1, c2), c3, k.z);
                s3 = x3(x3(d0, d1, d2), d3, k.w);
            }
        } else if constexpr (RK::kUniform) {
            s0 = x3s(a0, a2, k.x) ^ rotl8(a1 ^ a3);
            s1 = x3s(b0, b2, k.y) ^ rotl8(b1 ^ b3);
            s2 = x3s(c0, c2, k.z) ^ rotl8(c1 ^ c3);
            s3 = x3s(d0, d2, k.w) ^ rotl8(d1 ^ d3);
        } else {
            s0 = x3(a0, a2, k.x) ^ rotl8(a1 ^ a3);
            s1 = x3(b0, b2, k.y) ^ rotl8(b1 ^ b3);
            s2 = x3(c0, c2, k.z) ^ rotl8(c1 ^ c3);
            s3 = x3(d0, d2, k.w) ^ rotl8(d1 ^ d3);
        }
    }
    k = rk.get(14);
    // last round: SubBytes+ShiftRows; S[x] is byte 1 of T0[x]
#if NEB_PRIO
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(RK::kPrioHi);
#endif
    const uint32_t a0 = T.t0(s0, 0), a1 = T.t0(s1, 1), a2 = T.t0(s2, 2), a3 = T.t0(s3, 3);
    const uint32_t b0 = T.t0(s1, 0), b1 = T.t0(s2, 1), b2 = T.t0(s3, 2), b3 = T.t0(s0, 3);
    const uint32_t c0 = T.t0(s2, 0), c1 = T.t0(s3, 1), c2 = T.t0(s0, 2), c3 = T.t0(s1, 3);
    const uint32_t d0 = T.t0(s3, 0), d1 = T.t0(s0, 1), d2 = T.t0(s1, 2), d3 = T.t0(s2, 3);
#if NEB_PRIO
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(RK::kPrioLo);
#endif
    uint4 o;
    if constexpr (RK::kUniform) {
        o.x = x3s(perm(a1, a0, 0x0C0C0501u), perm(a3, a2, 0x05010C0Cu), k.x);
        o.y = x3s(perm(b1, b0, 0x0C0C0501u), perm(b3, b2, 0x05010C0Cu), k.y);
        o.z = x3s(perm(c1, c0, 0x0C0C0501u), perm(c3, c2, 0x05010C0Cu), k.z);
        o.w = x3s(perm(d1, d0, 0x0C0C0501u), perm(d3, d2, 0x05010C0Cu), k.w);
    } else {
        o.x = x3(perm(a1, a0, 0x0C0C0501u), perm(a3, a2, 0x05010C0Cu), k.x);
        o.y = x3(perm(b1, b0, 0x0C0C0501u), perm(b3, b2, 0x05010C0Cu), k.y);
        o.z = x3(perm(c1, c0, 0x0C0C0501u), perm(c3, c2, 0x05010C0Cu), k.z);
        o.w = x3(perm(d1, d0, 0x0C0C0501u), perm(d3, d2, 0x05010C0Cu), k.w);
    }
    return o;
}

template <class TL, class RK>
__device__ __forceinline__ uint4 aes256_block(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, const TL& T,
                                              const RK& rk) {
    const uint4 k = rk.get(0);
    return aes256_rounds<1>(s0 ^ k.x, s1 ^ k.y, s2 ^ k.z, s3 ^ k.w, T, rk);
}

// Counter-mode caching. A packet's counter blocks are 00000000 || BE64(n) || BE32(ctr): with
// ctr < 2^16 they differ only in state bytes 14 and 15 (word 3, bytes 2 and 3). Round 1 then
// varies only through T2[byte 14] in column 1 and T3[byte 15] in column 0, and round 2 only
// through the two varying columns of round 1: per block 2 + 8 lookups instead of 32. K (round 1)
// and L (round 2) hold the packet-constant parts, round keys folded in.
struct CtrConst {
    uint4 K, L;
    uint32_t k0w;  // word 3 of round key 0
};

template <class TL, class RK>
__device__ __forceinline__ CtrConst aes_ctr_prep(uint32_t c1, uint32_t c2, const TL& T, const RK& rk) {
    const uint4 k0 = rk.get(0), k1 = rk.get(1), k2 = rk.get(2);
    const uint32_t s0 = k0.x, s1 = c1 ^ k0.y, s2 = c2 ^ k0.z, s3 = k0.w;  // counter bytes = 0
    CtrConst c;
    c.k0w = k0.w;
    c.K.x = T.t0(s0, 0) ^ rotl8(T.t0(s1, 1)) ^ T.t2(s2, 2) ^ k1.x;                      // minus T3[b3 s3]
    c.K.y = T.t0(s1, 0) ^ rotl8(T.t0(s2, 1)) ^ rotl8(T.t2(s0, 3)) ^ k1.y;               // minus T2[b2 s3]
    c.K.z = T.t0(s2, 0) ^ rotl8(T.t0(s3, 1) ^ T.t2(s1, 3)) ^ T.t2(s0, 2) ^ k1.z;
    c.K.w = T.t0(s3, 0) ^ rotl8(T.t0(s0, 1) ^ T.t2(s2, 3)) ^ T.t2(s1, 2) ^ k1.w;
    c.L.x = T.t2(c.K.z, 2) ^ rotl8(T.t2(c.K.w, 3)) ^ k2.x;
    c.L.y = rotl8(T.t0(c.K.z, 1)) ^ T.t2(c.K.w, 2) ^ k2.y;
    c.L.z = T.t0(c.K.z, 0) ^ rotl8(T.t0(c.K.w, 1)) ^ k2.z;
    c.L.w = T.t0(c.K.w, 0) ^ rotl8(T.t2(c.K.z, 3)) ^ k2.w;
    return c;
}

template <class TL, class RK>
__device__ __forceinline__ uint4 aes256_ctr_block(const CtrConst& c, uint32_t ctr, const TL& T, const RK& rk) {
    const uint32_t s3 = c.k0w ^ bswap32(ctr);
    const uint32_t t0 = c.K.x ^ T.t3(s3, 3);
    const uint32_t t1 = c.K.y ^ T.t2(s3, 2);
    const uint32_t u0 = x3(c.L.x, T.t0(t0, 0), T.t1(t1, 1));
    const uint32_t u1 = x3(c.L.y, T.t0(t1, 0), T.t3(t0, 3));
    const uint32_t u2 = x3(c.L.z, T.t2(t0, 2), T.t3(t1, 3));
    const uint32_t u3 = x3(c.L.w, T.t2(t1, 2), T.t1(t0, 1));
    return aes256_rounds<3>(u0, u1, u2, u3, T, rk);
}

// The same with every counter below 2^8 (packets under 4 KiB): byte 14 is zero too, so round 1
// varies only through T3[byte 15] in column 0, and round 2 through the 4 bytes of that column,
// one per output column: 1 + 4 lookups per block instead of 2 + 8.
template <class TL, class RK>
__device__ __forceinline__ CtrConst aes_ctr_prep8(uint32_t c1, uint32_t c2, const TL& T, const RK& rk) {
    CtrConst c = aes_ctr_prep(c1, c2, T, rk);
    const uint4 k2 = rk.get(2);
    c.K.y ^= T.t2(c.k0w, 2);  // round 1 column 1 is constant now
    c.L.x = rotl8(T.t0(c.K.y, 1)) ^ T.t2(c.K.z, 2) ^ rotl8(T.t2(c.K.w, 3)) ^ k2.x;
    c.L.y = T.t0(c.K.y, 0) ^ rotl8(T.t0(c.K.z, 1)) ^ T.t2(c.K.w, 2) ^ k2.y;
    c.L.z = T.t0(c.K.z, 0) ^ rotl8(T.t0(c.K.w, 1) ^ T.t2(c.K.y, 3)) ^ k2.z;
    c.L.w = T.t0(c.K.w, 0) ^ T.t2(c.K.y, 2) ^ rotl8(T.t2(c.K.z, 3)) ^ k2.w;
    return c;
}

template <class TL, class RK>
__device__ __forceinline__ uint4 aes256_ctr8_block(const CtrConst& c, uint32_t ctr, const TL& T, const RK& rk) {
    const uint32_t t0 = c.K.x ^ T.t3(c.k0w ^ (ctr << 24), 3);
    const uint32_t u0 = c.L.x ^ T.t0(t0, 0);
    const uint32_t u1 = c.L.y ^ T.t3(t0, 3);
    const uint32_t u2 = c.L.z ^ T.t2(t0, 2);
    const uint32_t u3 = c.L.w ^ T.t1(t0, 1);
    return aes256_rounds<3>(u0, u1, u2, u3, T, rk);
}

// ------------------------------------------------------------------------------------------
// GF(2^128), GCM bit order. An element is 4 big-endian words w0..w3; the coefficient of x^j is
// bit 31 - (j mod 32) of w[j / 32], so multiplying by x is a 128-bit logical right shift.
// Nibble p (p = 8q + r, 0..31) of x = bits 28-4r..31-4r of w[q]; its value v has MSB = x^(4p).

__device__ __forceinline__ uint4 gf_mulx(uint4 v) {
    uint32_t lsb = v.w & 1u;
    uint4 r;
    r.w = shr64(v.z, v.w, 1);
    r.z = shr64(v.y, v.z, 1);
    r.y = shr64(v.x, v.y, 1);
    r.x = (v.x >> 1) ^ (lsb ? 0xE1000000u : 0u);
    return r;
}

// 256-bit product z[0..7] (x^0..x^255) -> 128-bit, modulo x^128 + x^7 + x^2 + x + 1.
__device__ __forceinline__ uint4 gf_reduce(const uint32_t z[8]) {
    const uint32_t l0 = z[4], l1 = z[5], l2 = z[6], l3 = z[7];
    // L·(1 + x + x^2 + x^7), the bits shifted out (x^128..x^134) collected in o
    uint32_t t0 = x3(l0, l0 >> 1, l0 >> 2) ^ (l0 >> 7);
    uint32_t t1 = x3(x3(l1, shr64(l0, l1, 1), shr64(l0, l1, 2)), shr64(l0, l1, 7), z[1]);
    uint32_t t2 = x3(x3(l2, shr64(l1, l2, 1), shr64(l1, l2, 2)), shr64(l1, l2, 7), z[2]);
    uint32_t t3 = x3(x3(l3, shr64(l2, l3, 1), shr64(l2, l3, 2)), shr64(l2, l3, 7), z[3]);
    uint32_t o = x3(l3 << 31, l3 << 30, l3 << 25);
    uint32_t of = x3(o, o >> 1, o >> 2) ^ (o >> 7);
    return make_uint4(x3(z[0], t0, of), t1, t2, t3);
}

// q·x^i, i < 128: q shifted right by i bits as a 256-bit product, then reduced (any lane, no loop).
__device__ __forceinline__ uint4 gf_mul_xpow(uint4 q, uint32_t i) {
    const uint32_t w = i >> 5, b = i & 31u;
    const uint32_t src[4] = {q.x, q.y, q.z, q.w};
    uint32_t y[8], z[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) v = (uint32_t)(k - j) == w ? src[j] : v;
        y[k] = v;
    }
    z[0] = y[0] >> b;
#pragma unroll
    for (int k = 1; k < 8; k++) z[k] = shr64(y[k - 1], y[k], b);
    return gf_reduce(z);
}

// q·x^b, b < 32 (gf_mul_xpow with no whole-word shift): 128 + 32 bits, the top word reduced.
__device__ __forceinline__ uint4 gf_mul_xpow32(uint4 q, uint32_t b) {
    const uint32_t z[8] = {q.x >> b, shr64(q.x, q.y, b), shr64(q.y, q.z, b), shr64(q.z, q.w, b), shr64(q.w, 0u, b),
                           0u, 0u, 0u};
    return gf_reduce(z);
}

// (byte K of w) & 0xF0 in one VALU op (SDWA byte select); hipcc emits a shift + and for most K.
template <int K>
__device__ __forceinline__ uint32_t byte_hi_nibble(uint32_t w) {
    uint32_t r;
    if constexpr (K == 0) {
        r = w & 0xF0u;
    } else {
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_%c3 src1_sel:DWORD"
            : "=v"(r) : "v"(w), "s"(0xF0u), "i"(K));
    }
    return r;
}

// x · F where ftab (LDS) is a full table F_p[v] at byte p*256 + v*16; acc is XORed in.
// Table addresses: the high nibble of byte k as is, the low nibble after one shift of the word:
// 9 VALU per word for its 8 lookups.
__device__ __forceinline__ uint4 gf_mul_full(uint4 x, uint4 acc, const uint4* ftab) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t hi = xw[q];        // byte k: nibble r = 6-2k in bits 4-7
        const uint32_t lo = xw[q] << 4;   // byte k: nibble r = 7-2k in bits 4-7
        const uint32_t ah[4] = {byte_hi_nibble<0>(hi), byte_hi_nibble<1>(hi), byte_hi_nibble<2>(hi),
                                byte_hi_nibble<3>(hi)};
        const uint32_t al[4] = {byte_hi_nibble<0>(lo), byte_hi_nibble<1>(lo), byte_hi_nibble<2>(lo),
                                byte_hi_nibble<3>(lo)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 e1 = lds_at<uint4>(ftab, (uint32_t)(8 * q + 6 - 2 * k) * 256u + ah[k]);
            const uint4 e2 = lds_at<uint4>(ftab, (uint32_t)(8 * q + 7 - 2 * k) * 256u + al[k]);
            acc = x34(acc, e1, e2);
        }
    }
    return acc;
}

// x · P where ptab (LDS) holds the 8 position tables T_r[v] = v·x^(4r)·P (reduced) at byte
// r*256 + v*16: nibble r of word q contributes T_r[v]·x^(32q), a shift by whole words, so the 32
// lookups XOR straight into a 224-bit product that is reduced once. No shifts (the Shoup form
// shifts every lookup by 4r bits): ~125 VALU per multiply instead of ~240, at 2 KiB per power.
// For P = H^4 the tables are the first 8 positions of the single-key full table.
__device__ __forceinline__ uint4 gf_mul_pos(uint4 x, const uint4* ptab) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t hi = xw[q], lo = xw[q] << 4;
        const uint32_t ah[4] = {byte_hi_nibble<0>(hi), byte_hi_nibble<1>(hi), byte_hi_nibble<2>(hi),
                                byte_hi_nibble<3>(hi)};
        const uint32_t al[4] = {byte_hi_nibble<0>(lo), byte_hi_nibble<1>(lo), byte_hi_nibble<2>(lo),
                                byte_hi_nibble<3>(lo)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 e1 = lds_at<uint4>(ptab, (uint32_t)(6 - 2 * k) * 256u + ah[k]);
            const uint4 e2 = lds_at<uint4>(ptab, (uint32_t)(7 - 2 * k) * 256u + al[k]);
            z[q] = x3(z[q], e1.x, e2.x);
            z[q + 1] = x3(z[q + 1], e1.y, e2.y);
            z[q + 2] = x3(z[q + 2], e1.z, e2.z);
            z[q + 3] = x3(z[q + 3], e1.w, e2.w);
        }
    }
    return gf_reduce(z);
}

// z ^= x · P unreduced (the 256-bit product of gf_mul_pos, before gf_reduce): several products
// share one reduction (the GHASH pass's aggregated rounds).
__device__ __forceinline__ void gf_acc_pos(uint4 x, const uint4* ptab, uint32_t z[8]) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t hi = xw[q], lo = xw[q] << 4;
        const uint32_t ah[4] = {byte_hi_nibble<0>(hi), byte_hi_nibble<1>(hi), byte_hi_nibble<2>(hi),
                                byte_hi_nibble<3>(hi)};
        const uint32_t al[4] = {byte_hi_nibble<0>(lo), byte_hi_nibble<1>(lo), byte_hi_nibble<2>(lo),
                                byte_hi_nibble<3>(lo)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 e1 = lds_at<uint4>(ptab, (uint32_t)(6 - 2 * k) * 256u + ah[k]);
            const uint4 e2 = lds_at<uint4>(ptab, (uint32_t)(7 - 2 * k) * 256u + al[k]);
            z[q] = x3(z[q], e1.x, e2.x);
            z[q + 1] = x3(z[q + 1], e1.y, e2.y);
            z[q + 2] = x3(z[q + 2], e1.z, e2.z);
            z[q + 3] = x3(z[q + 3], e1.w, e2.w);
        }
    }
}

// gf_mul_pos with the tables at byte offset `off` (per lane, a multiple of 256) from `base`
__device__ __forceinline__ uint4 gf_mul_pos_off(uint4 x, const void* base, uint32_t off) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t hi = xw[q], lo = xw[q] << 4;
        const uint32_t ah[4] = {byte_hi_nibble<0>(hi), byte_hi_nibble<1>(hi), byte_hi_nibble<2>(hi),
                                byte_hi_nibble<3>(hi)};
        const uint32_t al[4] = {byte_hi_nibble<0>(lo), byte_hi_nibble<1>(lo), byte_hi_nibble<2>(lo),
                                byte_hi_nibble<3>(lo)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 e1 = lds_at<uint4>(base, (uint32_t)(6 - 2 * k) * 256u + (ah[k] | off));
            const uint4 e2 = lds_at<uint4>(base, (uint32_t)(7 - 2 * k) * 256u + (al[k] | off));
            z[q] = x3(z[q], e1.x, e2.x);
            z[q + 1] = x3(z[q + 1], e1.y, e2.y);
            z[q + 2] = x3(z[q + 2], e1.z, e2.z);
            z[q + 3] = x3(z[q + 3], e1.w, e2.w);
        }
    }
    return gf_reduce(z);
}

// x · H^k where `tab` is the LDS byte offset (multiple of 256, < 2^24, relative to `base`) of a
// Shoup table M[v] = v·H^k. 32 independent lookups grouped by shift residue, reduced once.
__device__ __forceinline__ uint4 gf_mul_shoup(uint4 x, uint32_t tab, const uint4* base) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    uint32_t hi[4], lo[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        hi[q] = xw[q] & 0xF0F0F0F0u;
        lo[q] = (xw[q] << 4) & 0xF0F0F0F0u;
    }
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 8; r++) {
        // nibble r of every word: byte (3 - r/2) of hi (even r) or lo (odd r)
        const int k = 3 - (r >> 1);
        uint4 m[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t src = (r & 1) ? lo[q] : hi[q];
            // address = tab | (nibble << 4): byte k of src into byte 0, tab's bytes 1..3 kept
            m[q] = lds_at<uint4>(base, perm(src, tab, 0x03020100u | (uint32_t)(4 + k)));
        }
        uint32_t a[7];
        a[0] = m[0].x;
        a[1] = m[0].y ^ m[1].x;
        a[2] = x3(m[0].z, m[1].y, m[2].x);
        a[3] = x3(m[0].w, m[1].z, m[2].y) ^ m[3].x;
        a[4] = x3(m[1].w, m[2].z, m[3].y);
        a[5] = m[2].w ^ m[3].z;
        a[6] = m[3].w;
        if (r == 0) {
#pragma unroll
            for (int i = 0; i < 7; i++) z[i] ^= a[i];
        } else {
            const uint32_t sh = 4 * r;
            z[0] ^= a[0] >> sh;
#pragma unroll
            for (int i = 1; i < 7; i++) z[i] ^= shr64(a[i - 1], a[i], sh);
            z[7] ^= a[6] << (32 - sh);
        }
        __builtin_amdgcn_sched_barrier(0);  // at most one residue's lookups in flight
    }
    return gf_reduce(z);
}

// Entry e (0..15) of the 4-bit Shoup table of P: XOR of P·x^j for the set bits (bit 3 ↔ x^0).
__device__ __forceinline__ uint4 gf_tab_entry(uint4 p, uint32_t e) {
    uint4 p1 = gf_mulx(p), p2 = gf_mulx(p1), p3 = gf_mulx(p2);
    uint32_t m8 = (e & 8) ? ~0u : 0u, m4 = (e & 4) ? ~0u : 0u, m2 = (e & 2) ? ~0u : 0u, m1 = (e & 1) ? ~0u : 0u;
    uint4 r;
    r.x = (p.x & m8) ^ (p1.x & m4) ^ (p2.x & m2) ^ (p3.x & m1);
    r.y = (p.y & m8) ^ (p1.y & m4) ^ (p2.y & m2) ^ (p3.y & m1);
    r.z = (p.z & m8) ^ (p1.z & m4) ^ (p2.z & m2) ^ (p3.z & m1);
    r.w = (p.w & m8) ^ (p1.w & m4) ^ (p2.w & m2) ^ (p3.w & m1);
    return r;
}

__device__ __forceinline__ uint4 ld_rec4(const uint32_t* rec, uint32_t i) {
    return *reinterpret_cast<const uint4*>(rec + i);
}

// ------------------------------------------------------------------------------------------
// Per-packet work shared by both kernels

struct GcmArgs {
    const neb_desc* desc;
    uint32_t npkt;
    uint8_t* arena;
    const uint32_t* keys;  // key table, kKeyRecDwords per key
    uint32_t max_keys;
    uint32_t key_hint;     // SINGLE: the one key_id
    int32_t* status;
    const uint32_t* npkt_dev;  // optional: the batch's packet count in device memory (min with npkt)
    // TX batches only (tx.hip): a descriptor's first `flags` plaintext bytes are read from its
    // destination (the patched header image), the rest from src (the TUN read itself)
    uint32_t hdr_from_dst;
    // single-key kernel: the waves of its grid (packets past its full passes are left to
    // gcm_single_tail_kernel), 0 = it takes every packet itself
    uint32_t tail_slots;
    // the device receive's admission mask (window.cpp): only packets with adm[p] != 0 are opened, the
    // others keep the status the receive's plan gave them (RX instantiations only)
    const uint8_t* adm;
};

struct PktShape {
    uint32_t na, m, n, R, pad;
};

__device__ __forceinline__ PktShape pkt_shape(const neb_desc& d, bool run) {
    PktShape s;
    s.na = (d.aad_len + 15u) >> 4;
    s.m = (d.len + 15u) >> 4;
    s.n = s.na + s.m + 1u;
    s.R = run ? (s.n + 15u) >> 4 : 0u;
    s.pad = 16u * s.R - s.n;
    return s;
}

// One round of one packet lane: keystream, payload XOR, GHASH input block. Returns X (BE words).
// Block roles of lane l in round r: 1-based GHASH index g and, for a ciphertext block, its counter.
struct LaneBlock {
    int32_t g;
    bool is_aad, is_ct, is_len;
    uint32_t k, ctr;
};
__device__ __forceinline__ LaneBlock lane_block(const PktShape& sh, uint32_t r, uint32_t l, uint32_t lg) {
    LaneBlock b;
    b.g = (int32_t)((r << lg) + l + 1u) - (int32_t)sh.pad;
    b.is_aad = b.g >= 1 && b.g <= (int32_t)sh.na;
    b.is_ct = b.g > (int32_t)sh.na && b.g <= (int32_t)(sh.na + sh.m);
    b.is_len = b.g == (int32_t)sh.n;
    b.k = (uint32_t)(b.g - (int32_t)sh.na);  // ciphertext block index (1-based)
    b.ctr = b.is_ct ? b.k + 1u : 1u;          // the length lane computes E_K(J0)
    return b;
}

// Input block of lane block b: the AAD block or the payload block (zero-padded), else zero.
// hdr: plaintext bytes [0, hdr) come from the destination (GcmArgs::hdr_from_dst).
__device__ __forceinline__ uint4 gcm_lane_load(const neb_desc& d, const LaneBlock& b, const uint8_t* arena,
                                               uint32_t hdr) {
    uint4 in = make_uint4(0, 0, 0, 0);
    if (b.is_aad) {
        const uint32_t off = 16u * (uint32_t)(b.g - 1);
        in = load_block(arena + d.aad_off + off, min(16u, d.aad_len - off));
    }
    if (b.is_ct) {
        const uint32_t off = 16u * (b.k - 1u);
        const uint32_t nb = min(16u, d.len - off);
        in = off < hdr ? load_block_hdr(arena + d.dst_off + off, arena + d.src_off + off, nb, hdr - off)
                       : load_block(arena + d.src_off + off, nb);
    }
    return in;
}

// Where the length lane keeps E_K(J0) from its round to the tag finish.
struct Ej0Reg {
    uint4 v = make_uint4(0, 0, 0, 0);
    __device__ __forceinline__ void set(uint4 k) { v = k; }
    __device__ __forceinline__ uint4 get() const { return v; }
};

// Payload XOR and GHASH input of one block given its input and keystream. Returns X (BE words).
template <bool OPEN, class EJ>
__device__ __forceinline__ uint4 gcm_lane_io(const neb_desc& d, const LaneBlock& b, uint4 in, uint4 ks,
                                             uint8_t* arena, EJ& ej0) {
    uint4 X = make_uint4(0, 0, 0, 0);
    if (b.is_aad) X = bswap4(in);
    if (b.is_ct) {
        const uint32_t off = 16u * (b.k - 1u);
        const uint32_t nb = min(16u, d.len - off);
        const uint4 out = xor4(in, mask_block(ks, nb));
        store_block(arena + d.dst_off + off, out, nb);
        X = bswap4(OPEN ? in : out);
    }
    if (b.is_len) {
        const uint64_t abits = (uint64_t)d.aad_len * 8u, cbits = (uint64_t)d.len * 8u;
        X = make_uint4((uint32_t)(abits >> 32), (uint32_t)abits, (uint32_t)(cbits >> 32), (uint32_t)cbits);
        ej0.set(ks);
    }
    return X;
}

// Keystream block of lane block b. CM: counter-mode caching level — 0 none, 1 every counter of
// the wave below 2^16, 2 below 2^8.
template <int CM, class TL, class RK>
__device__ __forceinline__ uint4 gcm_lane_ks(const LaneBlock& b, uint32_t c1, uint32_t c2, const CtrConst& cc,
                                             const TL& T, const RK& rk) {
    if constexpr (CM == 2) return aes256_ctr8_block(cc, b.ctr, T, rk);
    else if constexpr (CM == 1) return aes256_ctr_block(cc, b.ctr, T, rk);
    else return aes256_block(0u, c1, c2, bswap32(b.ctr), T, rk);
}

// Tag finish on the packet's last lane, which holds E_K(J0) (seal: store; open: compare, zero
// the payload on mismatch).
template <bool OPEN>
__device__ __forceinline__ uint32_t gcm_finish(const neb_desc& d, uint4 S, uint4 ej0, uint32_t lane, uint32_t l,
                                               uint32_t LPP, uint8_t* arena) {
    const uint4 tag = xor4(ej0, bswap4(S));  // valid on lane LPP-1
    uint32_t fail = 0;
    if (l == LPP - 1u) {
        if constexpr (!OPEN) {
            store_block(arena + d.dst_off + d.len, tag, 16);
        } else {
            const uint4 rt = load_block(arena + d.src_off + d.len, 16);
            const uint4 df = xor4(rt, tag);
            fail = (df.x | df.y | df.z | df.w) != 0u;
        }
    }
    if constexpr (OPEN) {
        fail = (uint32_t)__shfl((int)fail, (int)(lane | (LPP - 1u)));
        if (fail) {
            for (uint32_t off = 16u * l; off < d.len; off += 16u * LPP)
                store_block(arena + d.dst_off + off, make_uint4(0, 0, 0, 0), min(16u, d.len - off));
        }
    }
    return fail;
}

// ------------------------------------------------------------------------------------------
// Packet groups: LPP = 2^lg lanes per packet (4 in the single-key kernel; 4, 8 or 16 per chunk in
// the mixed-key kernel), 64 / LPP packets per wave.
//
// Lane l of a packet owns padded GHASH blocks g' = LPP·r + l + 1 (n' = LPP·ceil(n/LPP); a
// 1300-byte packet has n = 84, so at LPP 4 nothing is padded). Horner stride H^LPP. The final
// Σ_l A_l·H^(LPP-l) multiplies with one table shared by every lane of a ds_read_b128 group at a
// time: no bank conflicts (per-lane power tables conflicted on every lookup and cost 17%).
// The round keys are wave-uniform (scalar registers) in both kernels below: one key per batch, or
// one key per chunk of a regrouped mixed-key batch (sched.hpp).

constexpr uint32_t kLg = 2;             // single-key kernel: log2 lanes per packet
constexpr uint32_t kLpp = 1u << kLg;    // = kFullPow, the full table's power
constexpr uint32_t kPpw = 64u / kLpp;   // packets per wave
static_assert(kLpp == kFullPow, "the single-key Horner stride is the full table's power");

__device__ __forceinline__ uint4 shfl4(uint4 v, uint32_t src) {
    return make_uint4(__shfl(v.x, (int)src), __shfl(v.y, (int)src), __shfl(v.z, (int)src), __shfl(v.w, (int)src));
}
__device__ __forceinline__ uint4 shfl_down4(uint4 v, uint32_t d) {
    return make_uint4(__shfl_down(v.x, d), __shfl_down(v.y, d), __shfl_down(v.z, d), __shfl_down(v.w, d));
}

// GHASH tables a packet group multiplies with: horner(A) = A·H^LPP, and final(A) = the packet's
// Σ_l A_l·H^(LPP-l), valid at least on the packet's last lane (the one holding E_K(J0)).
//
// The final as one multiply per lane (LPP 4): lane l of a quad needs A_l·H^(4-l), and the quad
// XOR of those is the packet's Σ_l A_l·H^(4-l). A ds_read_b128 is served in four groups of 16 lanes
// (MI355X_MICROARCH.md, LDS); lanes of one group reading different tables at the same nibble would
// conflict, so the accumulators are first permuted (ds_bpermute) so that group g holds role g of
// all 16 packets and multiplies by H^(4-g) alone — conflict-free, as the Horner step — then pulled
// back and XORed over the quad. 8 bpermutes + 1 multiply instead of a quad Horner's 4 multiplies.
struct FinalPermLanes {
    uint32_t src1, src2, off;  // pull source (role g of packet idx), pull-back source, table offset
};
// tab_off[g]: byte offset from the LDS base of the tables of H^(4-g)
__device__ __forceinline__ FinalPermLanes final_perm_lanes(uint32_t lane, const uint32_t tab_off[4]) {
    // b128 lane groups: lanes 32h + 4·c + j with c = quad index mod 8, group 2h + parity(c), index
    // 4·(c >> 1) + j within it (groups {0-3,12-15,20-27}, {4-11,16-19,28-31} and the upper half)
    const uint32_t c = (lane >> 2) & 7u, h = lane >> 5;
    const uint32_t g = ((uint32_t)__popc(c) & 1u) + 2u * h;
    const uint32_t i = 4u * (c >> 1) + (lane & 3u);
    const uint32_t l = lane & 3u, q = lane >> 2, m = q >> 2;
    const uint32_t b = (l & 1u) ^ ((uint32_t)__popc(m) & 1u);
    FinalPermLanes f;
    f.src1 = 4u * i + g;
    f.src2 = 32u * (l >> 1) + 4u * (2u * m + b) + (q & 3u);
    f.off = g == 0u ? tab_off[0] : g == 1u ? tab_off[1] : g == 2u ? tab_off[2] : tab_off[3];
    return f;
}
template <int CTRL>
__device__ __forceinline__ uint4 dpp4(uint4 v) {
    return make_uint4((uint32_t)__builtin_amdgcn_mov_dpp((int)v.x, CTRL, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_mov_dpp((int)v.y, CTRL, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_mov_dpp((int)v.z, CTRL, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w, CTRL, 0xF, 0xF, false));
}
// pull role g of every packet into b128 group g, multiply, pull back, XOR over the quad
template <class MUL>
__device__ __forceinline__ uint4 final_perm(uint4 A, const FinalPermLanes& fp, MUL&& mul) {
    const uint4 a = shfl4(A, fp.src1);
    uint4 v = shfl4(mul(a, fp.off), fp.src2);
    v = xor4(v, dpp4<0xB1>(v));     // quad_perm [1,0,3,2]
    return xor4(v, dpp4<0x4E>(v));  // quad_perm [2,3,0,1]
}

// One key per batch, LPP 4 (gcm_single_kernel): reduction-free full table of H^4 for the Horner
// step, position tables of H, H^2, H^3, H^4 for the permuted final.
struct GhFullPerm {
    const uint4* full;
    const void* base;  // the LDS base of FinalPermLanes::off
    FinalPermLanes fp;
    __device__ __forceinline__ uint4 horner(uint4 a, uint32_t) const {
        return gf_mul_full(a, make_uint4(0, 0, 0, 0), full);
    }
    __device__ __forceinline__ uint4 final(uint4 A, uint32_t, uint32_t) const {
        return final_perm(A, fp, [&](uint4 a, uint32_t off) { return gf_mul_pos_off(a, base, off); });
    }
};

// Pairwise tree over the packet's lanes: level i folds V_l·H^(2^i) ⊕ V_(l+2^i) into the lanes
// l ≡ 0 mod 2^(i+1); after lg levels lane 0 holds Z with Σ_l A_l·H^(LPP-l) = Z·H: lg + 1 multiplies
// instead of a Horner's LPP. shoup_off(i): LDS byte offset (from base) of the Shoup table of H^(2^i).
template <class OFF>
__device__ __forceinline__ uint4 tree_final(uint4 A, uint32_t lane, uint32_t lg, const uint4* base, OFF&& shoup_off) {
    uint4 V = A;
    for (uint32_t i = 0; i < lg; i++) V = xor4(gf_mul_shoup(V, shoup_off(i), base), shfl_down4(V, 1u << i));
    V = gf_mul_shoup(V, shoup_off(0u), base);
    return shfl4(V, lane & ~((1u << lg) - 1u));
}

// 64 lanes per packet (the tail and per-packet kernels): lane l = 16a + b needs A_l·H^(64-l) =
// A_l·H^(16-b)·H^(16(3-a)). Each lane multiplies by its own M_(16-b) (the record's Shoup tables
// of H^1..H^16, m16), the 16 lanes of a quarter XOR their products (S_a), quarters 0 and 2 multiply
// by H^16 and then quarters 0 and 1 by H^32, and the quarters XOR: 3 dependent multiplies instead
// of the tree's 7 (GhShoup, kept for other lane counts). NEB_TAIL_TREE=1 keeps the tree (A/B).
#ifndef NEB_TAIL_TREE
#define NEB_TAIL_TREE 0
#endif
struct GhShoup64 {
    const uint4* m16;    // M_1..M_16, 256 B each
    const uint4* shoup;  // M of H^(2^j), j < 6: M_32 is j = 5 (the tree of the A/B build)
    const uint4* pos;    // position tables of H^64 (the Horner stride)
    const uint4* hi;     // M_16, M_32, M_48: the quarters' powers
    __device__ __forceinline__ uint4 horner(uint4 a, uint32_t) const { return gf_mul_pos(a, pos); }
    __device__ __forceinline__ uint4 final(uint4 A, uint32_t lane, uint32_t lg) const {
#if NEB_TAIL_TREE
        return tree_final(A, lane, lg, shoup, [](uint32_t i) { return i * 256u; });
#else
        const uint32_t b = lane & 15u, a = (lane >> 4) & 3u;
        uint4 V = gf_mul_shoup(A, (15u - b) * 256u, m16);
        V = xor4(V, shfl_xor4(V, 8));
        V = xor4(V, shfl_xor4(V, 4));
        V = xor4(V, shfl_xor4(V, 2));
        V = xor4(V, shfl_xor4(V, 1));
        const uint4 W = gf_mul_shoup(V, (a < 3u ? 2u - a : 0u) * 256u, hi);  // S_a·H^(16(3-a))
        V = a < 3u ? W : V;
        V = xor4(V, shfl_xor4(V, 16));
        return xor4(V, shfl_xor4(V, 32));
#endif
    }
};

// Mixed-key chunks (gcm_chunk_kernel), tables in the wave's LDS slice, restaged per chunk.
// Full chunks (16 packets at 4 lanes, the single-key kernel's layout): Horner on the position
// tables of H^4, the permuted final on the Shoup tables M_1..M_4 (b128 group g multiplies role g of
// every packet by M_(4-g)).
struct GhChunk4 {
    const uint4* shoup;  // M_1, M_2, M_3, M_4 (record Shoup tables 0-3)
    const uint4* pos;    // position tables of H^4
    __device__ __forceinline__ uint4 horner(uint4 a, uint32_t) const { return gf_mul_pos(a, pos); }
    __device__ __forceinline__ uint4 final(uint4 A, uint32_t lane, uint32_t) const {
        // the lane permutation is recomputed here rather than held across the chunk loop, where
        // its registers would be spilled (the compiler would hoist it: the opaque copy of `lane`
        // keeps it here)
        const uint32_t ln = lane;
        const uint32_t tab_off[4] = {3u * 256u, 2u * 256u, 256u, 0u};  // M_4, M_3, M_2, M_1
        return final_perm(A, final_perm_lanes(ln, tab_off),
                          [&](uint4 a, uint32_t off) { return gf_mul_shoup(a, off, shoup); });
    }
};
// Tail chunks (1-8 packets at 8 or 16 lanes): Horner on the position tables of H^(2^lg); the final
// as quads, then a short tree over the packet's quads (round 6). Lane l = 4a + b of a packet needs
// A_l·H^(LPP-l) = A_l·H^(4-b)·H^(4(LPP/4-1-a)): the permuted one-multiply final of the 4-lane chunks
// gives every quad Q_a = Σ_b A_(4a+b)·H^(4-b) (final_perm treats each quad as a packet), then
// LPP 8: Q_0·H^4 ⊕ Q_1; LPP 16: (Q_0·H^4 ⊕ Q_1)·H^8 ⊕ (Q_2·H^4 ⊕ Q_3). Every lane of a level multiplies
// by the same table (M_4, then M_8), so the lookups stay conflict-free: 2 or 3 dependent multiplies
// instead of the pairwise tree's 4 or 5 (that tree cost ≈ 2 rounds of VALU per tail chunk, and tail
// chunks are half of a C5 shard's chunks).
struct GhChunkTail {
    const uint4* shoup;  // M_1, M_2, M_3, M_4, M_8
    const uint4* pos;    // position tables of H^(2^lg)
    __device__ __forceinline__ uint4 horner(uint4 a, uint32_t) const { return gf_mul_pos(a, pos); }
    __device__ __forceinline__ uint4 final(uint4 A, uint32_t lane, uint32_t lg) const {
        const uint32_t ln = lane;
        const uint32_t tab_off[4] = {3u * 256u, 2u * 256u, 256u, 0u};  // M_4, M_3, M_2, M_1
        const uint4 Q = final_perm(A, final_perm_lanes(ln, tab_off),
                                   [&](uint4 a, uint32_t off) { return gf_mul_shoup(a, off, shoup); });
        const uint32_t a = (ln >> 2) & ((1u << (lg - 2u)) - 1u);  // the quad's index in its packet
        // (selects per component: a select of two uint4 values went through a scratch array)
        const uint4 W = sel4((a & 1u) != 0u, Q, gf_mul_shoup(Q, 3u * 256u, shoup));  // even quads: Q·H^4
        const uint4 P = xor4(W, shfl_xor4(W, 4));  // quads (0,1): Q_0·H^4 ⊕ Q_1, (2,3): Q_2·H^4 ⊕ Q_3
        if (lg == 3u) return P;
        const uint4 U = sel4((a & 2u) != 0u, P, gf_mul_shoup(P, 4u * 256u, shoup));  // quads 0, 1: ·H^8
        return xor4(U, shfl_xor4(U, 8));
    }
};

// ---- the TX checksum in the seal (CS; tx.hip kTxCsumFlag) ----------------------------------
// The TX segment kernel leaves in the L4 checksum field the partial sum of everything but the
// payload bytes the seal reads from the TUN read ([hdr, len)); the seal adds those bytes' 16-bit
// words as it encrypts them. The field's block was encrypted with the partial (round 0): the
// packet's last lane then stores the field's final ciphertext bytes and moves the tag by the
// change, S' = S ^ Δ·H^e (GHASH is linear; e = n + 1 - the field block's index), with the Shoup
// tables of H^(2^j), j < 10, in LDS (e < 1024: segments under 16 KB).
// desc.flags = hdr | field << 12 | kind << 24 | parity << 26 (kind 1: TCP or a plain packet, 2:
// UDP, whose computed zero goes out as 0xFFFF; parity: the checksum start's, for the word pairing).
constexpr uint32_t kCsHdrMask = 0xFFFu;
__device__ __forceinline__ uint32_t le16_sum(uint4 v) {
    return (v.x & 0xFFFFu) + (v.x >> 16) + (v.y & 0xFFFFu) + (v.y >> 16) + (v.z & 0xFFFFu) + (v.z >> 16) +
           (v.w & 0xFFFFu) + (v.w >> 16);
}
__device__ __forceinline__ uint32_t block_byte(uint4 v, uint32_t q) {
    const uint32_t w = q < 4u ? v.x : q < 8u ? v.y : q < 12u ? v.z : v.w;
    return (w >> (8u * (q & 3u))) & 0xFFu;
}
__device__ __forceinline__ uint32_t cs_fold16(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}
// The tag lane: the final checksum from the packet's payload sum `acc` (little-endian words) and
// the field word `fk` (partial << 16 | keystream bytes there); stores the field's ciphertext and
// returns Δ·H^e for the tag.
__device__ __forceinline__ uint4 gcm_csum_fix(const neb_desc& d, uint32_t n, uint32_t na, uint32_t acc, uint32_t fk,
                                              uint8_t* arena, const uint4* pow2) {
    const uint32_t kind = (d.flags >> 24) & 3u, f = (d.flags >> 12) & 0xFFFu;
    uint32_t sum = cs_fold16(acc);
    if (!((d.flags >> 26) & 1u)) sum = ((sum & 0xFFu) << 8) | (sum >> 8);  // big-endian words
    const uint32_t fval = fk >> 16, ks16 = fk & 0xFFFFu;
    uint32_t c = ~cs_fold16(sum + fval) & 0xFFFFu;
    if (kind == 2u && c == 0u) c = 0xFFFFu;
    const uint32_t delta = fval ^ c;
    __threadfence_block();  // the field's block was stored by a lane of this wave in an earlier round
    uint8_t* ct = arena + d.dst_off + f;
    ct[0] = (uint8_t)((ks16 ^ c) >> 8);
    ct[1] = (uint8_t)(ks16 ^ c);
    // Δ as a GHASH block (big-endian words): bytes q and q + 1 (q < 15: the segment kernel keeps
    // the field inside one block)
    const uint32_t q = f & 15u, q1 = q + 1u;
    const uint32_t hi = (delta >> 8) << (24u - 8u * (q & 3u)), lo = (delta & 0xFFu) << (24u - 8u * (q1 & 3u));
    uint4 corr = make_uint4(((q >> 2) == 0u ? hi : 0u) | ((q1 >> 2) == 0u ? lo : 0u),
                            ((q >> 2) == 1u ? hi : 0u) | ((q1 >> 2) == 1u ? lo : 0u),
                            ((q >> 2) == 2u ? hi : 0u) | ((q1 >> 2) == 2u ? lo : 0u),
                            ((q >> 2) == 3u ? hi : 0u) | ((q1 >> 2) == 3u ? lo : 0u));
    const uint32_t e = n - na - (f >> 4);  // n + 1 - (na + f / 16 + 1)
    for (uint32_t j = 0; j < 10u; j++)
        if ((e >> j) & 1u) corr = gf_mul_shoup(corr, j * 256u, pow2);
    return corr;
}

#ifdef NEB_WAVE_TRACE
// per-wave phase times of the packet groups (tools/wave_trace.py, trace build only): the chunk kernel
// clears them per chunk and records them; s_memrealtime ticks summed over the chunk's groups, each
// phase closed by a full s_waitcnt (so a phase's time includes the latency of its own accesses)
constexpr uint32_t kWavePhaseWaves = 8192;
__device__ uint32_t g_wphase[kWavePhaseWaves * 4];  // desc, rounds, final, finish
__device__ __forceinline__ uint32_t wave_gid() { return blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); }
__device__ __forceinline__ uint64_t phase_now() {
    __builtin_amdgcn_s_waitcnt(0);
    return __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void phase_add(uint32_t k, uint64_t t0, uint64_t t1) {
    const uint32_t w = wave_gid();
    if ((threadIdx.x & 63u) == 0u && w < kWavePhaseWaves) g_wphase[4u * w + k] += (uint32_t)(t1 - t0);
}
#endif

// Seal or open packet `p` (lanes (lane >> lg) << lg ... + LPP-1 of the wave). `expect_key`: the key
// this wave's round keys and tables belong to; key_ok: that key is installed with the right
// algorithm. lg is wave-uniform.
// own (optional): the packet's descriptor itself, not args.desc[p] (the per-packet kernel's, rebased).
// RX: the device receive's open (args.adm), an instantiation of its own so the plain opens keep their
// registers.
template <bool OPEN, bool CS = false, bool RX = false, class GH, class TL, class RK>
__device__ __forceinline__ void gcm_packet_group(const GcmArgs& args, uint32_t p, bool valid, uint32_t expect_key,
                                                 bool key_ok, const RK& rk, const GH& gh, const TL& T,
                                                 uint32_t lane, uint32_t lg, const uint4* cs_pow = nullptr,
                                                 const neb_desc* own = nullptr) {
    const uint32_t LPP = 1u << lg;
    const uint32_t l = lane & (LPP - 1u);
    NEB_MARK(grp_begin);
#ifdef NEB_WAVE_TRACE
    const uint64_t tq0 = phase_now();
#endif
    neb_desc d = {};
    uint32_t admit = 1u;
    if (valid) {
        d = own ? *own : args.desc[p];
        if constexpr (RX) admit = args.adm[p];  // (beside the descriptor's load, not behind it)
    }
#ifdef NEB_WAVE_TRACE
    const uint64_t tq1 = phase_now();
    phase_add(0, tq0, tq1);
#endif
    // the device receive opens only what its windows admitted (the rest keep the plan's status)
    if constexpr (RX) valid = valid && admit != 0u;
    uint32_t st = NEB_STATUS_OK;
    if (!key_ok || d.key_id != expect_key) st = NEB_STATUS_BAD_KEY;
    if (!OPEN && st == NEB_STATUS_OK && d.counter >= kRejectAfterMessages) st = NEB_STATUS_EXHAUSTED;
    const bool run = valid && st == NEB_STATUS_OK;
    const uint32_t hdr = args.hdr_from_dst ? d.flags & kCsHdrMask : 0u;
    // CS: this lane's payload word sum, and (the field's lane) partial << 16 | keystream bytes
    uint32_t cs_acc = 0, cs_fk = 0;
    const bool cs_on = CS && !OPEN && ((d.flags >> 24) & 3u) != 0u;
    const uint32_t cs_f = (d.flags >> 12) & 0xFFFu;
    PktShape sh;
    sh.na = (d.aad_len + 15u) >> 4;
    sh.m = (d.len + 15u) >> 4;
    sh.n = sh.na + sh.m + 1u;
    sh.R = run ? (sh.n + LPP - 1u) >> lg : 0u;
    sh.pad = (sh.R << lg) - sh.n;
    Ej0Reg ej0;

    // nonce 00000000 || BE64(n) as little-endian words; counter block word 3 = BE32(ctr)
    const uint32_t c1 = bswap32((uint32_t)(d.counter >> 32));
    const uint32_t c2 = bswap32((uint32_t)d.counter);
    uint4 A = make_uint4(0, 0, 0, 0);
    auto rounds = [&](auto cm) {
        constexpr int CM = decltype(cm)::value;
        CtrConst cc{};
        if constexpr (CM == 2) cc = aes_ctr_prep8(c1, c2, T, rk);
        else if constexpr (CM == 1) cc = aes_ctr_prep(c1, c2, T, rk);
        NEB_MARK(ctr_done);
        // The common round: every active lane holds a full payload block with a 16-B aligned
        // destination (the arena base counts too: a caller may pass an arena at any byte address);
        // a source off 16-B alignment (a TX segment inside its TUN read) is read as two aligned
        // blocks and shifted. Its block is loaded at the top of the round (fast_load), so the load's
        // latency overlaps the round's GHASH and AES instead of following them: a wave's round is
        // a chain of dependent LDS lookups, and the mixed-key kernel's last chunks run with few
        // waves per CU to hide it (C3 +2.7%, C2 equal; tools/wave_trace.py).
        auto fast_round = [&](const LaneBlock& b) {
            const uint32_t off = 16u * (b.k - 1u);
            return __all(b.is_ct && off + 16u <= d.len && off >= hdr &&
                         ((d.dst_off | (uint32_t)(uintptr_t)args.arena) & 15u) == 0u);
        };
        auto fast_load = [&](const LaneBlock& b) {
            const uint8_t* sp = args.arena + d.src_off + 16u * (b.k - 1u);
            return __all(((uint32_t)(uintptr_t)sp & 3u) == 0u) ? load_u4_a4(sp) : load_shifted16(sp);
        };
        // round r's payload XOR and GHASH fold, given G = A·H^LPP (the rounds before), the keystream
        // and (a common round) the block loaded at the round's top
        auto io = [&](const LaneBlock& b, uint4 G, uint4 ks, bool fast, uint4 pre) {
            const uint32_t off = 16u * (b.k - 1u);
            if (fast) {
                const uint4 in = pre;
                if constexpr (CS) {
                    if (cs_on) cs_acc += le16_sum(in);
                }
                const uint4 out = xor4(in, ks);
                *reinterpret_cast<uint4*>(args.arena + d.dst_off + off) = out;
                A = xor4(G, bswap4(OPEN ? in : out));
                return;
            }
            const uint4 in = gcm_lane_load(d, b, args.arena, hdr);
            if constexpr (CS) {
                if (cs_on && b.is_ct) {
                    const uint32_t off = 16u * (b.k - 1u);
                    const uint32_t hi = min(16u, d.len - off), lo = hdr > off ? min(hdr - off, 16u) : 0u;
                    if (lo < hi) {  // the bytes of [hdr, len) in this block
                        const uint4 v = mask_block(in, hi);
                        cs_acc += le16_sum(xor4(v, mask_block(v, lo)));
                    }
                    if (cs_f - off < 16u) {
                        const uint32_t q = cs_f - off;
                        cs_fk = (block_byte(in, q) << 24) | (block_byte(in, q + 1u) << 16) | (block_byte(ks, q) << 8) |
                                block_byte(ks, q + 1u);
                    }
                }
            }
            A = xor4(G, gcm_lane_io<OPEN>(d, b, in, ks, args.arena, ej0));
        };
        auto horner = [&](uint32_t r) -> uint4 { return r == 0 ? make_uint4(0, 0, 0, 0) : gh.horner(A, lg); };
        // one round on the LDS: GHASH of the previous rounds first, then this round's T-table AES
        // (one phase's registers at a time)
        auto tround = [&](uint32_t r) {
            NEB_MARK(round_begin);
            if (r < sh.R) {
                const LaneBlock b = lane_block(sh, r, l, lg);
                const bool fast = fast_round(b);
                uint4 pre = make_uint4(0, 0, 0, 0);
                if (fast) pre = fast_load(b);
                const uint4 G = horner(r);
                __builtin_amdgcn_sched_barrier(0);
                // a round with no ciphertext or length block in the wave needs no keystream: the
                // AAD-only rounds of GMAC (relay verify, connection_state.go:121-148) skip the AES
                uint4 ks = make_uint4(0, 0, 0, 0);
                if (__any(b.is_ct || b.is_len)) ks = gcm_lane_ks<CM>(b, c1, c2, cc, T, rk);
                io(b, G, ks, fast, pre);
            }
            NEB_MARK(round_end);
        };
        // rounds until no packet of the wave has one left (a ballot, no cross-lane reduction; a
        // shuffle max of the round counts first was 4-7% slower in the chunk kernel)
        for (uint32_t r = 0; __any(r < sh.R); r++) tround(r);
    };
#if NEB_ONE_TRACE
    const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
#endif
    // counter caching needs every block counter of every packet in the wave below 2^8 / 2^16
    if (__all(sh.m + 1u < 256u)) rounds(std::integral_constant<int, 2>{});
    else if (__all(sh.m + 1u < 65536u)) rounds(std::integral_constant<int, 1>{});
    else rounds(std::integral_constant<int, 0>{});
    if constexpr (CS) {
        for (uint32_t sft = 1; sft < LPP; sft <<= 1) {
            cs_acc += (uint32_t)__shfl_xor((int)cs_acc, (int)sft);
            cs_fk |= (uint32_t)__shfl_xor((int)cs_fk, (int)sft);
        }
    }
#if NEB_ONE_TRACE
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t tp1 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef NEB_WAVE_TRACE
    const uint64_t tq2 = phase_now();
    phase_add(1, tq1, tq2);
#endif
    NEB_MARK(rounds_done);
    uint4 V = gh.final(A, lane, lg);  // every lane: the tree shuffles across the packet's lanes
    NEB_MARK(final_done);
#ifdef NEB_WAVE_TRACE
    const uint64_t tq3 = phase_now();
    phase_add(2, tq2, tq3);
#endif
#if NEB_ONE_TRACE
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t tp2 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) printf("  rounds %u  final %u (x10 ns, R=%u)\n", (unsigned)(tp1 - tp0), (unsigned)(tp2 - tp1), sh.R);
#endif
    if constexpr (CS) {
        if (run && cs_on && l == LPP - 1u) V = xor4(V, gcm_csum_fix(d, sh.n, sh.na, cs_acc, cs_fk, args.arena, cs_pow));
    }
    if (run && gcm_finish<OPEN>(d, V, ej0.get(), lane, l, LPP, args.arena)) st = NEB_STATUS_AUTH_FAILED;
    if (valid && l == LPP - 1u) args.status[p] = (int32_t)st;
    NEB_MARK(grp_end);
#ifdef NEB_WAVE_TRACE
    phase_add(3, tq3, phase_now());
#endif
}

__device__ __forceinline__ void load_round_keys(const uint32_t* rec, uint32_t rks[60]) {
#pragma unroll
    for (int i = 0; i < 60; i++) rks[i] = __builtin_amdgcn_readfirstlane(rec[kRecRoundKeys + i]);
}

// Wave timeline of the single-key and chunk kernels, for tools/wave_trace.py only (a build with -DNEB_WAVE_TRACE=1;
// the product build has none of it): per chunk {workgroup << 20 | wave << 16 | count << 8 | lg << 4
// | full, chunk index, start, end} in s_memrealtime ticks (100 MHz), and per wave {…, ~0u, kernel
// start, tables filled}.
#ifdef NEB_WAVE_TRACE
// fixed slots per wave (no shared counter: one atomic word serialised the waves and skewed the
// timeline it was meant to record): slot 0 the wave's start, slot 1 + k its k-th chunk
constexpr uint32_t kWaveTraceSlots = 64, kWaveTraceWaves = 8192, kWaveTraceCap = kWaveTraceSlots * kWaveTraceWaves;
__device__ uint4 g_wtrace[kWaveTraceCap];
__device__ __forceinline__ void wave_trace(uint32_t lane, uint32_t slot, uint32_t a, uint32_t b, uint64_t t0,
                                           uint64_t t1) {
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (lane == 0u && w < kWaveTraceWaves && slot < kWaveTraceSlots)
        g_wtrace[w * kWaveTraceSlots + slot] = make_uint4(a | 0x80000000u, b, (uint32_t)t0, (uint32_t)t1);
}
#endif

// ---- one tunnel key for the whole batch -------------------------------------------------------

// Four-table AES (TLook4, 128 KiB) + the GHASH tables: one 1024-lane workgroup per CU, 4 waves per
// SIMD, at most 128 VGPRs.
constexpr int kSingleWaves = 16;
constexpr int kSingleWpe = 4;  // launch bound: waves per SIMD
constexpr int kSingleThreads = kSingleWaves * kWave;

struct SingleLds {
    uint4 full[32 * 16];       // 8 KiB   F_p[v] for H^4 (first: its offsets fit the ds_read offset field)
    uint4 pos1[8 * 16];        // 2 KiB   position tables of H
    uint2 ttab[2 * 256 * 32];  // 128 KiB (T0,T1) and (T2,T3) pairs, 32 copies each
    uint4 pos23[2][8 * 16];    // 4 KiB   position tables of H^2 and H^3 (the permuted final)
};
struct SingleLdsCs : SingleLds {
    uint4 pow2[10 * 16];  // 2.5 KiB  Shoup tables of H^(2^j), j < 10 (the TX checksum correction)
};

// CS: the TX seal with the L4 checksums (gcm_csum_fix); RX: the device receive's open (GcmArgs::adm)
template <bool OPEN, bool CS = false, bool RX = false>
__global__ __launch_bounds__(kSingleThreads, kSingleWpe) void gcm_single_kernel(GcmArgs args) {
    __shared__ std::conditional_t<CS, SingleLdsCs, SingleLds> lds;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    const uint32_t* srec = args.keys + (size_t)args.key_hint * kKeyRecDwords;
#ifdef NEB_WAVE_TRACE
    const uint64_t tk0 = __builtin_amdgcn_s_memrealtime();
#endif
    // the record's GHASH tables: loaded before the T-table fill and stored after it, so their
    // latency overlaps the fill's instead of following it
    static_assert(kSingleThreads >= 512, "one full-table entry per thread");
    uint4 r_full = make_uint4(0, 0, 0, 0), r_h = make_uint4(0, 0, 0, 0), r_p = make_uint4(0, 0, 0, 0);
    if (tid < 512u) r_full = ld_rec4(srec, kRecFull + 4u * tid);
    if (tid < 128u) r_h = ld_rec4(srec, kRecPos1 + 4u * tid);
    if (tid < 256u) r_p = ld_rec4(srec, (tid < 128u ? kRecPos2 : kRecPos3) + 4u * (tid & 127u));
    const TLook4 T{lds.ttab, ttab4_lane_base(lane)};
    fill_ttab<2u * 256u * 32u, kSingleThreads>(lds.ttab, tid, ttab4_entry);
    if (tid < 512u) lds.full[tid] = r_full;
    if (tid < 128u) lds.pos1[tid] = r_h;
    if (tid < 256u) lds.pos23[tid >> 7][tid & 127u] = r_p;

    const uint4* cs_pow = nullptr;
    if constexpr (CS) {
        if (tid < 160u) lds.pow2[tid] = ld_rec4(srec, rec_shoup_pow2(tid >> 4) + 4u * (tid & 15u));
        cs_pow = lds.pow2;
    }
    uint32_t rks[60];
    load_round_keys(srec, rks);
    __syncthreads();
    const RkRegs rk{rks};
    const uint32_t tab_off[4] = {(uint32_t)offsetof(SingleLds, full), (uint32_t)offsetof(SingleLds, pos23[1]),
                                 (uint32_t)offsetof(SingleLds, pos23[0]), (uint32_t)offsetof(SingleLds, pos1)};
    const GhFullPerm gh{lds.full, &lds, final_perm_lanes(lane, tab_off)};

    // The slot must still hold an AES-GCM key when the batch runs (a key destroyed, or its slot
    // reused by another algorithm, while the batch was queued): every packet gets BAD_KEY then.
    const bool key_ok = __builtin_amdgcn_readfirstlane(srec[kRecAlg]) == NEB_ALG_AESGCM;
    uint32_t npkt = args.npkt;
    if (args.npkt_dev) npkt = min(npkt, __builtin_amdgcn_readfirstlane(*args.npkt_dev));
    const uint32_t ngroups = (npkt + kPpw - 1u) / kPpw;
    const uint32_t slots = gridDim.x * kSingleWaves;  // waves of the grid
    uint32_t main_groups = ngroups;
    if (args.tail_slots && ngroups > slots && ngroups % slots)
        main_groups = ngroups / slots * slots;  // full passes only: the tail kernel takes the rest
    // groups go to workgroups first (group g: workgroup g mod G, wave g / G), so a batch of fewer
    // groups than waves spreads over as many CUs as it can instead of filling a few (a 2048-packet
    // batch on 8 CUs ran as long as a whole 64 Ki pass)
#ifdef NEB_WAVE_TRACE
    uint32_t trace_k = 1;
    wave_trace(lane, 0, blockIdx.x << 20 | wave << 16, ~0u, tk0, __builtin_amdgcn_s_memrealtime());
#endif
    auto groups = [&](const auto& rkp) {
        for (uint32_t grp = blockIdx.x + wave * gridDim.x; grp < main_groups; grp += slots) {
#ifdef NEB_WAVE_TRACE
            const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
#endif
            const uint32_t p = grp * kPpw + lane / kLpp;
            gcm_packet_group<OPEN, CS, RX>(args, p, p < npkt, args.key_hint, key_ok, rkp, gh, T, lane, kLg, cs_pow);
#ifdef NEB_WAVE_TRACE
            wave_trace(lane, trace_k++, blockIdx.x << 20 | wave << 16 | 16u << 8 | 2u << 4 | 1u, grp, tc0,
                       __builtin_amdgcn_s_memrealtime());
#endif
        }
    };
#if NEB_PRIO && NEB_PRIO_AGE
    // A workgroup's waves w, w+4, w+8, w+12 share a SIMD in that age order (wave >> 2 is the
    // rank), and the SIMD arbiter serves the older first at equal priority: ranks 0-3 finished
    // their groups in 74 / 78 / 84 / 88 µs (tools/wave_trace.py, C2 seal, settled clock). Ranks 2
    // and 3 keep priority 1 instead of 0 between their lookup phases, so they are not passed over
    // by the older pair there. Alternating A/B against the same code at 0 (tools/r5_prio_ab.sh,
    // profiles/r5/ab_balance): seal 96.5-98.7 -> 94.2-95.6 µs. Every other split tried — lookup levels by
    // rank, four distinct levels, 0/1/1/1, 0/0/2/2 — was equal or slower.
    if (__builtin_amdgcn_readfirstlane(wave) >> 3) groups(RkRegsPrio<NEB_PRIO, 1>{rk});
    else groups(rk);
#else
    groups(rk);
#endif
}

// The tail pass: the packets after gcm_single_kernel's full passes over args.tail_slots waves (the
// groups that would otherwise run alone after everything else: 65 565 packets = 4098 groups of 16
// on 4096 waves), 2^kTailLg lanes per packet: the two-table AES (64 KiB), Horner stride
// H^(2^kTailLg) on its position tables, the 3-deep final on the Shoup tables of H .. H^16 and H^32
// (GhShoup64). A tail is small and runs on few waves, so its time is one packet's latency: at 64
// lanes a 1300-B packet takes 2 rounds instead of 6 at 16 (bench.py --mode tx: 1457 vs 1456
// superpackets, 0.243 vs 0.207 ms before it).
constexpr uint32_t kTailLg = 6, kTailPpw = kWave >> kTailLg;
// GcmArgs::tail_slots value for a batch small enough to run entirely in the tail kernel: one packet
// per wave over 64 lanes is 2 rounds for 1300 B instead of 21, and a batch under a few thousand
// packets is bound by one wave's latency, not by throughput
constexpr uint32_t kTailAll = 0xFFFFFFFFu;
// packets (host-known count) up to which the tail kernel takes them all (A/B: 6144 55.8 vs 71.3 us
// per seal, 8192 equal, 12288 101 vs 75)
constexpr uint32_t kSmallBatch = 6144;
constexpr int kTailWaves = 8;
struct TailLds {
    uint2 ttab[256 * 32];       // 64 KiB T-table pairs, 32 copies
    uint4 shoup[kTailLg * 16];  // 1.5 KiB
    uint4 pos[8 * 16];          // 2 KiB
    uint4 m16[16 * 16];         // 4 KiB: M_1..M_16 (GhShoup64)
    uint4 hi[3 * 16];           // M_16, M_32, M_48 (GhShoup64)
};
static_assert(kTailLg == 6, "GhShoup64: 64 lanes per packet");
template <bool OPEN, bool RX = false>
__global__ __launch_bounds__(kTailWaves * kWave) void gcm_single_tail_kernel(GcmArgs args) {
    __shared__ TailLds lds;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t npkt = args.npkt;
    if (args.npkt_dev) npkt = min(npkt, __builtin_amdgcn_readfirstlane(*args.npkt_dev));
    const uint32_t ngroups = (npkt + kPpw - 1u) / kPpw, slots = args.tail_slots;
    uint32_t p0 = 0;  // kTailAll: a small batch, every packet here
    if (slots != kTailAll) {
        if (ngroups <= slots || ngroups % slots == 0u) return;  // no partial pass: nothing to do
        p0 = ngroups / slots * slots * kPpw;
    }
    const uint32_t tgroups = (npkt - p0 + kTailPpw - 1u) / kTailPpw;
    if (blockIdx.x * kTailWaves >= tgroups) return;
    const uint32_t* srec = args.keys + (size_t)args.key_hint * kKeyRecDwords;
    fill_ttab<256u * 32u, kTailWaves * kWave>(lds.ttab, tid, ttab_entry);
    if (tid < 16u * kTailLg) {  // M[v] of H^(2^j), j < kTailLg
        const uint32_t j = tid >> 4, v = tid & 15u;
        lds.shoup[tid] = ld_rec4(srec, rec_shoup_pow2(j) + 4u * v);
    }
    if (tid < 128u) lds.pos[tid] = ld_rec4(srec, kRecPos64 + 4u * tid);
    if (tid < 256u) lds.m16[tid] = ld_rec4(srec, kRecShoup + 4u * tid);
    if (tid < 48u) lds.hi[tid] = ld_rec4(srec, (tid < 16u ? kRecShoup + 15u * 64u : tid < 32u ? kRecShoup32 : kRecShoup48) + 4u * (tid & 15u));
    uint32_t rks[60];
    load_round_keys(srec, rks);
    __syncthreads();
    const TLook T{lds.ttab, ttab_lane_base(lane)};
    const GhShoup64 gh{lds.m16, lds.shoup, lds.pos, lds.hi};
    const bool key_ok = __builtin_amdgcn_readfirstlane(srec[kRecAlg]) == NEB_ALG_AESGCM;
    for (uint32_t t = blockIdx.x * kTailWaves + wave; t < tgroups; t += gridDim.x * kTailWaves) {
        const uint32_t p = p0 + kTailPpw * t + (lane >> kTailLg);
        gcm_packet_group<OPEN, false, RX>(args, p, p < npkt, args.key_hint, key_ok, RkRegs{rks}, gh, T, lane, kTailLg);
    }
}

// ---- one packet, its bytes in the kernel arguments (the per-packet CipherState calls) ---------
// A per-packet call through the tail kernel spent ≈ 18.6 µs on the device for one packet, mostly
// a chain of PCIe round trips to the caller's pinned staging: the descriptor, then each round's
// payload block, then (open) the received tag. Here the host puts the descriptor, the AAD and the
// payload (+ tag) into the kernel's argument block, which the runtime writes to device memory with
// the dispatch, so the kernel reads nothing over PCIe; it writes the result and the status into
// the caller's pinned staging (posted writes). One wave, 64 lanes per packet (2 rounds for 1300 B).
constexpr uint32_t kOneBytes = 2048;  // AAD (padded to 16) + payload (+ tag): larger packets take the batch path

// The status goes out last, behind a system-scope release of the wave's result stores, so the host
// may take the result as soon as it sees the status word change (engine.cpp one_packet) instead of
// waiting for the stream (hipStreamSynchronize: ≈ 26 µs of a ≈ 36 µs call, round 4).
struct OneArgs {
    neb_desc d;           // offsets from `in`; dst_off reaches the host output (a wrapping 64-bit offset)
    const uint32_t* keys;
    uint32_t max_keys, key;
    int32_t* status;      // host
    uint32_t pad_[2];
    uint8_t in[kOneBytes];  // 16-B aligned within the argument block
};
static_assert(offsetof(OneArgs, in) % 16 == 0, "the packet bytes are read as 16-B blocks");
// The 64 KiB T-table image is filled by NEB_ONE_FILL_WAVES waves (the packet's one wave alone spent
// most of the kernel on it); the others leave after the fill.
#ifndef NEB_ONE_FILL_WAVES
#define NEB_ONE_FILL_WAVES 4
#endif
constexpr uint32_t kOneFillThreads = NEB_ONE_FILL_WAVES * kWave;
template <bool OPEN>
__global__ __launch_bounds__(kOneFillThreads) void gcm_one_kernel(OneArgs a) {
    __shared__ TailLds lds;
    const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1u);
    // the argument block in place (a by-value struct indexed per lane would be copied to scratch)
    // the block's address as an opaque integer: derived from the constant-address kernarg pointer,
    // the output address (base + dst_off) would let the compiler treat the result stores as stores
    // to constant memory and drop them
#if NEB_ONE_TRACE  // phase stamps (100 MHz) printed by lane 0: an A/B build only
    const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint64_t kb = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kb));
    const uint8_t* ka = reinterpret_cast<const uint8_t*>(kb);
    const uint32_t key = a.key;
    const uint32_t* srec = a.keys + (size_t)(key < a.max_keys ? key : 0u) * kKeyRecDwords;
    // The packet's bytes (the argument block's 2 KiB, in device memory) are touched by the fill's
    // threads first, so the rounds' block loads after the fill hit the caches (0.4 µs of 12).
    uint4 warm = make_uint4(0, 0, 0, 0);
    if (tid < kOneBytes / 16u) warm = *reinterpret_cast<const uint4*>(ka + offsetof(OneArgs, in) + 16u * tid);
    // T-tables, 16 entries per thread at a time (loads before stores, as fill_ttab)
    for (uint32_t j0 = 0; j0 < 256u * 32u; j0 += 16u * kOneFillThreads) {
        uint2 v[16];
#pragma unroll
        for (uint32_t j = 0; j < 16u; j++) v[j] = ttab_entry(j0 + j * kOneFillThreads + tid);
#pragma unroll
        for (uint32_t j = 0; j < 16u; j++) lds.ttab[j0 + j * kOneFillThreads + tid] = v[j];
    }
    for (uint32_t tdx = tid; tdx < 16u * kTailLg; tdx += kOneFillThreads)  // M[v] of H^(2^j), j < kTailLg
        lds.shoup[tdx] = ld_rec4(srec, rec_shoup_pow2(tdx >> 4) + 4u * (tdx & 15u));
    for (uint32_t tdx = tid; tdx < 128u; tdx += kOneFillThreads) lds.pos[tdx] = ld_rec4(srec, kRecPos64 + 4u * tdx);
    for (uint32_t tdx = tid; tdx < 256u; tdx += kOneFillThreads) lds.m16[tdx] = ld_rec4(srec, kRecShoup + 4u * tdx);
    if (tid < 48u)
        lds.hi[tid] = ld_rec4(srec, (tid < 16u ? kRecShoup + 15u * 64u : tid < 32u ? kRecShoup32 : kRecShoup48) + 4u * (tid & 15u));
    asm volatile("" ::"v"(warm.x), "v"(warm.y), "v"(warm.z), "v"(warm.w));  // the loads complete
    __syncthreads();
    if (tid >= kWave) return;  // the packet is one wave's
#if NEB_ONE_TRACE
    const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t rks[60];
    load_round_keys(srec, rks);
    const TLook T{lds.ttab, ttab_lane_base(lane)};
    const GhShoup64 gh{lds.m16, lds.shoup, lds.pos, lds.hi};
    const bool key_ok = key < a.max_keys && __builtin_amdgcn_readfirstlane(srec[kRecAlg]) == NEB_ALG_AESGCM;
    uint8_t* base = const_cast<uint8_t*>(ka + offsetof(OneArgs, in));
    __shared__ int32_t s_status;
    GcmArgs ga{nullptr, 1u, base, a.keys, a.max_keys, key, &s_status, nullptr, 0u, 0u, nullptr};
    // the host passed the output's address in dst_off: rebase it on the argument block (wrapping)
    neb_desc d = a.d;
    d.dst_off = a.d.dst_off - (uint64_t)(uintptr_t)base;
#if NEB_ONE_TRACE
    const uint64_t ts2 = __builtin_amdgcn_s_memrealtime();
#endif
    gcm_packet_group<OPEN>(ga, 0u, true, key, key_ok, RkRegs{rks}, gh, T, lane, kTailLg, nullptr, &d);
    one_publish_status(a.status, &s_status);
#if NEB_ONE_TRACE
    __builtin_amdgcn_s_waitcnt(0);
    const uint64_t ts3 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0)
        printf("one %d: fill %u  keys %u  packet %u  (x10 ns)\n", (int)OPEN, (unsigned)(ts1 - ts0), (unsigned)(ts2 - ts1),
               (unsigned)(ts3 - ts2));
#endif
}

// ---- per-packet calls that arrive together, in one launch (engine.cpp's combiner) -------------
// Concurrent EncryptDanger / DecryptDanger calls (several threads, each its own tunnel) that arrive
// while another call's launch is being made are collected in a pinned batch buffer and launched
// together: one wave per request, four waves per workgroup. The waves fill the workgroup's T-table
// image together; each stages its own key's GHASH tables (the per-packet kernel's set, GhShoup64)
// in a slice of its own and copies its request's slot from host memory into LDS with one parallel
// load (under the fill), then seals or opens it at 64 lanes, writes the result back into its slot
// (in place, host memory) and publishes its status last (one_publish_status), as the per-packet
// kernel does. The buffer (engine.cpp PktComb): statuses and slots (request r's bytes in slot r,
// kCombSlot apart); the descriptors (offsets from the slots' base) travel in the kernel arguments,
// so the key record's loads do not wait for a PCIe round trip (17.5 µs per launch with the
// descriptors in the pinned buffer, round-6 trace).
constexpr int kOneBatchWaves = 4;
constexpr uint32_t kOneBatchMax = 32;  // engine.cpp kCombMax
struct OneBatchDescs {
    neb_desc d[kOneBatchMax];
};
constexpr uint32_t kCombSlot = kOneBytes + 64u;  // AAD | payload (+ tag), room for the tag a seal appends
struct OneBatchLds {
    uint2 ttab[256 * 32];  // 64 KiB T-table pairs, 32 copies
    struct KeyTabs {
        uint4 shoup[kTailLg * 16];
        uint4 pos[8 * 16];
        uint4 m16[16 * 16];
        uint4 hi[3 * 16];
    } k[kOneBatchWaves];                              // 8.25 KiB each
    uint4 data[kOneBatchWaves][kCombSlot / 16u];      // the request's slot
    int32_t st[kOneBatchWaves];
};
template <bool OPEN>
__global__ __launch_bounds__(kOneBatchWaves * kWave) void gcm_one_batch_kernel(const OneBatchDescs descs, int32_t* status,
                                                                                uint8_t* slots, uint32_t n,
                                                                                const uint32_t* keys,
                                                                                uint32_t max_keys) {
    __shared__ OneBatchLds lds;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t r = blockIdx.x * kOneBatchWaves + w;
    const bool have = r < n;
    // the request's descriptor and bytes first (host memory: one PCIe round trip, under the fill)
    constexpr uint32_t kSlotVecs = kCombSlot / 16u;
    neb_desc d = {};
    uint4 b[(kSlotVecs + kWave - 1) / kWave];
    if (have) {
        d = descs.d[r];
#pragma unroll
        for (uint32_t k = 0; k < (kSlotVecs + kWave - 1) / kWave; k++)
            if (k * kWave + lane < kSlotVecs)
                b[k] = *reinterpret_cast<const uint4*>(slots + (size_t)r * kCombSlot + 16u * (k * kWave + lane));
    }
    fill_ttab<256u * 32u, kOneBatchWaves * kWave>(lds.ttab, tid, ttab_entry);
    const uint32_t key = __builtin_amdgcn_readfirstlane(d.key_id);
    const uint32_t* srec = keys + (size_t)(key < max_keys ? key : 0u) * kKeyRecDwords;
    OneBatchLds::KeyTabs& kt = lds.k[w];
    if (have) {
        for (uint32_t t = lane; t < 16u * kTailLg; t += kWave) kt.shoup[t] = ld_rec4(srec, rec_shoup_pow2(t >> 4) + 4u * (t & 15u));
        for (uint32_t t = lane; t < 128u; t += kWave) kt.pos[t] = ld_rec4(srec, kRecPos64 + 4u * t);
        for (uint32_t t = lane; t < 256u; t += kWave) kt.m16[t] = ld_rec4(srec, kRecShoup + 4u * t);
        if (lane < 48u)
            kt.hi[lane] = ld_rec4(srec, (lane < 16u ? kRecShoup + 15u * 64u : lane < 32u ? kRecShoup32 : kRecShoup48) + 4u * (lane & 15u));
#pragma unroll
        for (uint32_t k = 0; k < (kSlotVecs + kWave - 1) / kWave; k++)
            if (k * kWave + lane < kSlotVecs) lds.data[w][k * kWave + lane] = b[k];
    }
    __syncthreads();
    if (!have) return;
    uint32_t rks[60];
    load_round_keys(srec, rks);
    const TLook T{lds.ttab, ttab_lane_base(lane)};
    const GhShoup64 gh{kt.m16, kt.shoup, kt.pos, kt.hi};
    const bool key_ok = key < max_keys && __builtin_amdgcn_readfirstlane(srec[kRecAlg]) == NEB_ALG_AESGCM;
    // the bytes in LDS, addressed through a generic pointer (flat loads): the descriptor's offsets are
    // from the slots' base, so the LDS copy stands at slot r's place; the output goes to the slot in
    // host memory (a wrapping offset from there)
    uint64_t lb = (uint64_t)(uintptr_t)(const void*)&lds.data[w][0] - (uint64_t)r * kCombSlot;
    asm volatile("" : "+s"(lb));
    uint8_t* base = reinterpret_cast<uint8_t*>(lb);
    d.dst_off = d.dst_off + (uint64_t)(uintptr_t)slots - lb;
    GcmArgs ga{nullptr, 1u, base, keys, max_keys, key, &lds.st[w], nullptr, 0u, 0u, nullptr};
    gcm_packet_group<OPEN>(ga, 0u, true, key, key_ok, RkRegs{rks}, gh, T, lane, kTailLg, nullptr, &d);
    one_publish_status(status + r, &lds.st[w]);
}

// ---- mixed keys: one key per chunk of the regrouped batch (sched.hpp) --------------------------


// One kernel, two code paths, each specialised for its chunk shape (one path with a run-time lanes
// per packet spilled 52-64 B per lane at 128 VGPRs, inside the chunk loop):
//  front chunks (chunks[0, F)): groups of 16 packets at 4 lanes each, the layout of the single-key
//               kernel (GhChunk4), one after another on one staging of the key;
//  back chunks (chunks[max - 1 - j], j < B): tails of 1-8 packets at 8 or 16 lanes (GhChunkTail).
// The two-table AES (64 KiB): 16 waves per workgroup, one workgroup per CU.
constexpr int kChunkWaves = 16;
constexpr int kChunkWpe = 4;  // launch bound: waves per SIMD (at most 128 VGPRs)
constexpr int kChunkThreads = kChunkWaves * kWave;

struct ChunkLds {
    uint4 shoup[kChunkWaves][5][16];  // per wave: Shoup tables (1.25 KiB): M_1..M_4, and M_8 (tails)
    uint4 pos[kChunkWaves][8 * 16];   // per wave: position tables of H^(2^lg) (2 KiB)
    uint2 ttab[256 * 32];             // 64 KiB T-table pairs, 32 copies
};

// Stage a chunk key's GHASH tables in the wave's LDS slice, computed from the record's raw powers
// H^1..H^16 (16 B each) rather than copied from its precomputed tables: 128 B of key material per
// chunk instead of 3 KiB, which for IMIX-sized chunks was a third of the kernel's memory traffic.
//   shoup[t][v] = v·H^(t+1), t < 4, and (tails) shoup[4][v] = v·H^8
//   pos[r][v]   = v·x^(4r)·P, r < 8, P = H^(2^lg): XOR of the basis P·x^(4r+j) over the set bits
//                 of v (bit 3 ↔ j = 0), the basis P·x^i (i < 32) one per lane and shuffled
template <bool FULL>
__device__ __forceinline__ void stage_chunk_tables(const uint32_t* rec, uint32_t lane, uint32_t lg, uint4* wtab,
                                                   uint4* wpos) {
    const uint32_t t = lane >> 4, v = lane & 15u;
    const uint4 he = ld_rec4(rec, kRecHPow + 4u * t);
    const uint4 P = ld_rec4(rec, kRecHPow + 4u * ((1u << lg) - 1u));
    wtab[lane] = gf_tab_entry(he, v);
    if constexpr (!FULL) {
        const uint4 h8 = ld_rec4(rec, kRecHPow + 4u * 7u);
        if (lane < 16u) wtab[64u + lane] = gf_tab_entry(h8, v);
    }
    const uint4 B = gf_mul_xpow32(P, lane & 31u);
    uint4 e0 = make_uint4(0, 0, 0, 0), e1 = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t j = 0; j < 4u; j++) {
        const uint4 b0 = shfl4(B, 4u * t + j), b1 = shfl4(B, 4u * t + 16u + j);
        const uint32_t m = (v >> (3u - j)) & 1u ? ~0u : 0u;
        e0 = xor4(e0, make_uint4(b0.x & m, b0.y & m, b0.z & m, b0.w & m));
        e1 = xor4(e1, make_uint4(b1.x & m, b1.y & m, b1.z & m, b1.w & m));
    }
    wpos[lane] = e0;
    wpos[64u + lane] = e1;
}

struct ChunkArgs {
    const uint32_t* sorted;
    const uint4* chunks;  // [kBuckets][max_chunks] (sched.hpp)
    uint32_t* counters;   // the scheduler's counters (sched.hpp kCnt*)
    uint32_t max_chunks;
};

// Chunk order: the cost buckets in turn, longest first (sched.hpp sched_bucket). Workgroup w owns
// chunks w, w + G, w + 2G, ... of that order (G workgroups) and its waves draw them from an LDS
// cursor as each finishes its chunk. Balance stays dynamic inside the workgroup and no wave touches a global atomic (a global work cursor: returning
// atomics on one word serialise across the chip; C3 step -8%, IMIX -27% against it, A/B,
// profiles/r2_micro/ab_chunk_order.log).
template <bool OPEN, bool RX = false>
__global__ __launch_bounds__(kChunkThreads, kChunkWpe) void gcm_chunk_kernel(GcmArgs args, ChunkArgs ca) {
    __shared__ ChunkLds lds;
    __shared__ uint32_t wg_cursor;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    // chunk index space: bucket 0's chunks, then bucket 1's, ... (bucket b's records from b * max_chunks);
    // the buckets' ends in LDS (read per chunk: held in registers they were spilled)
    __shared__ uint32_t s_bend[kBuckets];
    uint32_t nch = 0;
#pragma unroll
    for (uint32_t b = 0; b < kBuckets; b++) nch += min(__builtin_amdgcn_readfirstlane(ca.counters[kCntBucket + b]), ca.max_chunks);
    if (tid < kBuckets) {
        uint32_t e = 0;
        for (uint32_t b = 0; b <= tid; b++) e += min(ca.counters[kCntBucket + b], ca.max_chunks);
        s_bend[tid] = e;
    }
    const uint32_t c0 = 0u;
    if (c0 + blockIdx.x >= nch) return;  // owns no chunk (uniform over the workgroup)
#ifdef NEB_WAVE_TRACE
    const uint64_t tk0 = __builtin_amdgcn_s_memrealtime();
#endif
    fill_ttab<256u * 32u, kChunkThreads>(lds.ttab, tid, ttab_entry);
    if (tid == 0) wg_cursor = kChunkWaves;
    __syncthreads();
#ifdef NEB_WAVE_TRACE
    uint32_t trace_k = 1;
    wave_trace(lane, 0, blockIdx.x << 20 | wave << 16, ~0u, tk0, __builtin_amdgcn_s_memrealtime());
#endif
    uint4* wtab = &lds.shoup[wave][0][0];
    uint4* wpos = &lds.pos[wave][0];
    auto chunk_at = [&](uint32_t c) {
        uint32_t b = 0, lo = 0;
        for (uint32_t k = 0; k + 1u < kBuckets; k++) {
            const uint32_t e = __builtin_amdgcn_readfirstlane(s_bend[k]);
            if (c < e) break;
            b = k + 1u;
            lo = e;
        }
        return ca.chunks[(size_t)b * ca.max_chunks + (c - lo)];
    };
    // Workgroup w owns chunks w, w + G, w + 2G, ... (the longest first) and its waves
    // draw them from an LDS cursor as they finish. Drawing the last 10-50% from a global cursor
    // instead (dynamic balance across workgroups) made the C3 kernel 26-50% slower: the returning
    // atomics on one word serialise across the chip (A/B).
    auto chunk_of = [&](uint32_t k) -> uint32_t { return c0 + blockIdx.x + k * gridDim.x; };
    uint32_t c = 0;
    if (lane == 0u) c = chunk_of(wave);
    c = __builtin_amdgcn_readfirstlane(c);
    uint4 ch_next = make_uint4(0, 0, 0, 0);
    if (c < nch) ch_next = chunk_at(c);
#if NEB_CHUNK_STEAL
#ifndef NEB_STEAL_MIN_PER_WG
#define NEB_STEAL_MIN_PER_WG 32u
#endif
    // The batch's last 1/8 of chunks (the shortest) are not owned: a wave whose workgroup has run
    // out of its own draws them from its XCD's cursor (blockIdx mod 8, one word per XCD, 128 B
    // apart), so workgroups that drew lighter chunks take more of them. C5's workgroups carried
    // 3752-4426 packets and spanned 562-616 µs with every chunk owned (tools/wave_trace.py). A/B,
    // alternating (profiles/r5/ab_balance): C3 547-548 -> 553-555 GiB/s, C5 512-514 -> 518; the
    // last 1/4 or 1/16 the same within noise. Every partition has a drawer (at least 8 workgroups)
    // and every wave's first chunk is still owned (at least 32 chunks per workgroup).
    const uint32_t ndyn = (gridDim.x >= 8u && nch >= NEB_STEAL_MIN_PER_WG * gridDim.x) ? nch / NEB_CHUNK_STEAL : 0u;
    const uint32_t nstat = nch - ndyn;
    auto claim = [&]() -> uint32_t {
        uint32_t k = 0;
        if (lane == 0u) {
            k = chunk_of(atomicAdd(&wg_cursor, 1u));
            if (k >= nstat) {
                const uint32_t x = blockIdx.x & 7u;
                k = nstat + x + 8u * atomicAdd(&ca.counters[kCntSteal + kStealStride * x], 1u);
            }
        }
        return __builtin_amdgcn_readfirstlane(k);
    };
#else
    auto claim = [&]() -> uint32_t {
        uint32_t k = 0;
        if (lane == 0u) k = chunk_of(atomicAdd(&wg_cursor, 1u));
        return __builtin_amdgcn_readfirstlane(k);
    };
#endif
    while (c < nch) {
        const uint4 ch = ch_next;
        NEB_MARK(chunk_begin);
        const uint32_t cw = __builtin_amdgcn_readfirstlane(ch.w);
        const bool full = (cw >> 20) & 1u;  // 4-lane groups (front), or one group at 8 or 16 lanes
#ifdef NEB_WAVE_TRACE
        const uint64_t tc0 = __builtin_amdgcn_s_memrealtime();
#endif
        // Lane-derived constants (the T-table lane base, shuffle sources, the final's permutation)
        // are rebuilt per chunk from an opaque copy of the lane index: hoisted out of the chunk loop
        // they stay live across it and the compiler spills them (36-104 B of scratch per lane).
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        const TLook T{lds.ttab, ttab_lane_base(ln)};
#ifdef NEB_WAVE_TRACE
        if (lane == 0u && wave_gid() < kWavePhaseWaves)
            for (uint32_t k = 0; k < 4u; k++) g_wphase[4u * wave_gid() + k] = 0u;
        const uint64_t tcd = phase_now();  // the chunk's descriptor in
#endif
        // the chunk's packets: segment 0 (count0 from start0 in sorted), then segment 1 (a smaller
        // class's leftover packets riding in free slots, sched_key_chunks)
        const uint32_t start = __builtin_amdgcn_readfirstlane(ch.x);
        const uint32_t start1 = __builtin_amdgcn_readfirstlane(ch.y);
        const uint32_t count0 = cw & 0xFFu, count = count0 + ((cw >> 8) & 0xFFu);
        const uint32_t key = __builtin_amdgcn_readfirstlane(ch.z);
        auto sorted_at = [&](uint32_t q) { return ca.sorted[q < count0 ? start + q : start1 + (q - count0)]; };
        const uint32_t* rec = args.keys + (size_t)(key < args.max_keys ? key : 0u) * kKeyRecDwords;
        const bool key_ok = key < args.max_keys && rec[kRecAlg] == NEB_ALG_AESGCM;
        uint32_t rks[60];
        load_round_keys(rec, rks);
#ifdef NEB_WAVE_TRACE
        const uint64_t tck = phase_now();  // round keys in
        uint64_t tcs = tck;
#endif
        if (full) {
            NEB_MARK(stage_full);
            stage_chunk_tables<true>(rec, ln, 2u, wtab, wpos);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef NEB_WAVE_TRACE
            tcs = phase_now();
#endif
            // the chunk's groups of 16 packets at 4 lanes, one after another on the staged tables
            const GhChunk4 gh{wtab, wpos};
            for (uint32_t g0 = 0; g0 < count; g0 += kChunkPkts) {
                const uint32_t q = g0 + (ln >> 2);
                const uint32_t sp = q < count ? sorted_at(q) : kSortedSkip;
                const bool valid = sp != kSortedSkip;  // (a device receive's refused packet: skipped)
                const uint32_t p = valid ? sp : 0u;
                gcm_packet_group<OPEN, false, RX>(args, p, valid, key, key_ok, RkRegs{rks}, gh, T, ln, 2u);
            }
        } else {
            const uint32_t lg = (cw >> kChunkLgShift) & 15u;  // 3 or 4
            NEB_MARK(stage_tail);
            stage_chunk_tables<false>(rec, ln, lg, wtab, wpos);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef NEB_WAVE_TRACE
            tcs = phase_now();
#endif
            const uint32_t q = ln >> lg;
            const uint32_t sp = q < count ? sorted_at(q) : kSortedSkip;
            const bool valid = sp != kSortedSkip;
            const uint32_t p = valid ? sp : 0u;
            const GhChunkTail gh{wtab, wpos};
            gcm_packet_group<OPEN, false, RX>(args, p, valid, key, key_ok, RkRegs{rks}, gh, T, ln, lg);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the slice is rewritten next chunk
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the next chunk is claimed when this one is done, not when it starts: a claim at the start
        // handed the workgroup's second round of chunks to whichever waves reached the cursor first
        // at time 0 (the older ones), and C3's waves then finished 97-115 µs apart
        // (tools/wave_trace.py). A/B, alternating (profiles/r5/ab_balance): C3 526-527 -> 536-537 GiB/s,
        // C5 504-505 -> 515-516; claiming ahead only while more than a round of chunks is left:
        // C3 537-542, C5 506-508.
        NEB_MARK(chunk_claim);
        const uint32_t cn = claim();
        if (cn < nch) ch_next = chunk_at(cn);
        NEB_MARK(chunk_claimed);
#ifdef NEB_WAVE_TRACE
        wave_trace(lane, trace_k++,
                   blockIdx.x << 20 | wave << 16 | min(count, 255u) << 8 | ((cw >> kChunkLgShift) & 15u) << 4 |
                       (full ? 1u : 0u),
                   c, tc0, __builtin_amdgcn_s_memrealtime());
        if (trace_k <= 21u) {  // phases: {descriptor in, round keys in, tables staged} and the groups' sums
            const uint32_t w = wave_gid() < kWavePhaseWaves ? wave_gid() : 0u;
            const uint32_t* ph = &g_wphase[4u * w];
            const uint32_t tag = blockIdx.x << 20 | wave << 16;
            wave_trace(lane, 20u + 2u * (trace_k - 1u), tag, 0xFFFFFFFEu,
                       (uint32_t)(tcd - tc0) | (uint32_t)(tck - tcd) << 16, (uint32_t)(tcs - tck));
            wave_trace(lane, 21u + 2u * (trace_k - 1u), tag, 0xFFFFFFFDu, ph[0] | ph[1] << 16, ph[2] | ph[3] << 16);
        }
#endif
        c = cn;
    }
}

// ------------------------------------------------------------------------------------------
// Key install: AES-256 key expansion, H = E_K(0), H^1..H^16, and the GHASH tables.
// Runs once per tunnel key (one workgroup of 256 lanes).

__device__ uint8_t sbox_b(uint32_t x) { return (uint8_t)(c_T0.t[x & 255u] >> 8); }
__device__ uint8_t xtime_d(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// One workgroup per key of a batch install (neb_cipher_create_batch: n keys in one launch); the
// workgroup first clears its record (the slot may have held another key or algorithm).
__global__ __launch_bounds__(256) void gcm_key_setup_kernel(const uint8_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ slots,
                                                            uint32_t* __restrict__ table) {
    const uint8_t* key = keys + 32u * blockIdx.x;
    uint32_t* rec = table + (size_t)slots[blockIdx.x] * kKeyRecDwords;
    for (uint32_t j = threadIdx.x; j < kKeyRecDwords; j += blockDim.x) rec[j] = 0u;
    __shared__ uint4 hp[16];      // H^1..H^16
    __shared__ uint4 basis[128];  // x^i · H^kFullPow
    __shared__ uint4 basis8[32];  // x^i · H^8
    __shared__ uint4 basis16[32]; // x^i · H^16
    __shared__ uint4 basis23[2][32]; // x^i · H^2, x^i · H^3
    __shared__ uint4 basis12[32];    // x^i · H^12
    __shared__ uint4 basis_h[128];  // x^i · H
    __shared__ uint4 part[2];
    // the S-box in LDS for the key schedule and H = E_K(0) on lane 0: its ~330 dependent lookups
    // from global memory cost ~25 µs per key
    __shared__ uint8_t sb[256];
    __shared__ uint8_t rk[240];  // the key schedule (in LDS: as a lane array it lived in scratch)
    sb[threadIdx.x] = (uint8_t)(c_T0.t[threadIdx.x] >> 8);
    __syncthreads();
    if (threadIdx.x == 0) {
        auto sbox_b = [&](uint32_t x) { return sb[x & 255u]; };
        for (int i = 0; i < 32; i++) rk[i] = key[i];
        uint8_t rcon = 1;
        for (int i = 8; i < 60; i++) {
            uint8_t t0 = rk[4 * i - 4], t1 = rk[4 * i - 3], t2 = rk[4 * i - 2], t3 = rk[4 * i - 1];
            if (i % 8 == 0) {
                uint8_t u = t0;
                t0 = sbox_b(t1) ^ rcon; t1 = sbox_b(t2); t2 = sbox_b(t3); t3 = sbox_b(u);
                rcon = xtime_d(rcon);
            } else if (i % 8 == 4) {
                t0 = sbox_b(t0); t1 = sbox_b(t1); t2 = sbox_b(t2); t3 = sbox_b(t3);
            }
            rk[4 * i] = rk[4 * i - 32] ^ t0; rk[4 * i + 1] = rk[4 * i - 31] ^ t1;
            rk[4 * i + 2] = rk[4 * i - 30] ^ t2; rk[4 * i + 3] = rk[4 * i - 29] ^ t3;
        }
        for (int i = 0; i < 60; i++)
            rec[kRecRoundKeys + i] = (uint32_t)rk[4 * i] | (uint32_t)rk[4 * i + 1] << 8 |
                                     (uint32_t)rk[4 * i + 2] << 16 | (uint32_t)rk[4 * i + 3] << 24;
        // H = E_K(0^128), byte-oriented FIPS-197 cipher
        uint8_t s[16];
        for (int i = 0; i < 16; i++) s[i] = rk[i];
        for (int r = 1; r <= 14; r++) {
            uint8_t t[16];
            for (int c = 0; c < 4; c++)
                for (int j = 0; j < 4; j++) t[4 * c + j] = sbox_b(s[4 * ((c + j) & 3) + j]);
            if (r != 14) {
                for (int c = 0; c < 4; c++) {
                    uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                    uint8_t x = a0 ^ a1 ^ a2 ^ a3;
                    t[4 * c] = a0 ^ x ^ xtime_d(a0 ^ a1);
                    t[4 * c + 1] = a1 ^ x ^ xtime_d(a1 ^ a2);
                    t[4 * c + 2] = a2 ^ x ^ xtime_d(a2 ^ a3);
                    t[4 * c + 3] = a3 ^ x ^ xtime_d(a3 ^ a0);
                }
            }
            for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk[16 * r + i];
        }
        uint32_t h[4];
        for (int i = 0; i < 4; i++)
            h[i] = (uint32_t)s[4 * i] << 24 | (uint32_t)s[4 * i + 1] << 16 | (uint32_t)s[4 * i + 2] << 8 | s[4 * i + 3];
        hp[0] = make_uint4(h[0], h[1], h[2], h[3]);
    }
    __syncthreads();
    // basis_h[i] = x^i·H: a product P·H is the XOR of basis_h[i] over the set bits i of P
    if (threadIdx.x < 128u) basis_h[threadIdx.x] = gf_mul_xpow(hp[0], threadIdx.x);
    __syncthreads();
    // H^2..H^16: H^k = H^(k-1)·H with lane i < 128 contributing basis_h[i] if bit i of H^(k-1) is
    // set, XOR-reduced across the two waves (the bit-serial form on one lane took ~100 µs).
    for (uint32_t k = 1; k < kNumHPow; k++) {
        const uint32_t t = threadIdx.x;
        const uint4 P = hp[k - 1];
        uint4 c = make_uint4(0, 0, 0, 0);
        if (t < 128u) {
            const uint32_t w = t < 32u ? P.x : (t < 64u ? P.y : (t < 96u ? P.z : P.w));
            if ((w >> (31u - (t & 31u))) & 1u) c = basis_h[t];
        }
        for (int m = 32; m >= 1; m >>= 1) c = xor4(c, shfl_xor4(c, m));
        if (t == 0u || t == 64u) part[t >> 6] = c;
        __syncthreads();
        if (t == 0u) hp[k] = xor4(part[0], part[1]);
        __syncthreads();
    }
    if (threadIdx.x < 64u) {
        const uint4 v = hp[threadIdx.x >> 2];
        const uint32_t c = threadIdx.x & 3u;
        rec[kRecHPow + threadIdx.x] = c == 0u ? v.x : c == 1u ? v.y : c == 2u ? v.z : v.w;
    }
    if (threadIdx.x < 128u) basis[threadIdx.x] = gf_mul_xpow(hp[kFullPow - 1], threadIdx.x);
    if (threadIdx.x < 32u) {
        basis8[threadIdx.x] = gf_mul_xpow(hp[7], threadIdx.x);
        basis16[threadIdx.x] = gf_mul_xpow(hp[15], threadIdx.x);
        basis23[0][threadIdx.x] = gf_mul_xpow(hp[1], threadIdx.x);
        basis23[1][threadIdx.x] = gf_mul_xpow(hp[2], threadIdx.x);
        basis12[threadIdx.x] = gf_mul_xpow(hp[11], threadIdx.x);
    }
    if (threadIdx.x == 0) rec[kRecAlg] = NEB_ALG_AESGCM;
    __syncthreads();
    const uint32_t t = threadIdx.x;
    // Shoup tables: entry (k, v) for k = 1..16
    {
        const uint32_t k = t >> 4, v = t & 15u;
        const uint4 e = gf_tab_entry(hp[k], v);
        uint32_t* o = rec + kRecShoup + 64u * k + 4u * v;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    // full table of H^kFullPow: F_p[v] = XOR of basis[4p + j] for the set bits of v (bit 3 ↔ j = 0)
    for (uint32_t i = t; i < 512u; i += 256u) {
        const uint32_t p = i >> 4, v = i & 15u;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, basis[4 * p + j]);
        uint32_t* o = rec + kRecFull + 4u * i;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    // position tables of H^8 and H^16: T_r[v] = XOR of basis[4r + j] for the set bits of v
    {
        const uint32_t tab = t >> 7, i = t & 127u, r = i >> 4, v = i & 15u;
        const uint4* bs = tab ? basis16 : basis8;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, bs[4 * r + j]);
        uint32_t* o = rec + (tab ? kRecPos16 : kRecPos8) + 4u * i;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    if (t < 128u) {  // and of H
        const uint32_t r = t >> 4, v = t & 15u;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, basis_h[4 * r + j]);
        uint32_t* o = rec + kRecPos1 + 4u * t;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    if (t < 128u) {  // and of H^12
        const uint32_t r = t >> 4, v = t & 15u;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, basis12[4 * r + j]);
        uint32_t* o = rec + kRecPos12 + 4u * t;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    {  // and of H^2, H^3
        const uint32_t tab = t >> 7, i = t & 127u, r = i >> 4, v = i & 15u;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, basis23[tab][4 * r + j]);
        uint32_t* o = rec + (tab ? kRecPos3 : kRecPos2) + 4u * i;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    // H^32 .. H^512 by squaring (the tail kernel's 64-lane packets, the TX seal's checksum
    // correction): P·Q is the XOR of basis[i] = x^i·Q over the set bits i of P (lane i < 128), as
    // for H^2..H^16 above
    auto basis_of = [&](uint4 q, uint32_t cnt) {
        __syncthreads();  // basis[] is free again
        if (t < cnt) basis[t] = gf_mul_xpow(q, t);
        __syncthreads();
    };
    auto mul_by_basis = [&](uint4 P) -> uint4 {
        uint4 c = make_uint4(0, 0, 0, 0);
        if (t < 128u) {
            const uint32_t w = t < 32u ? P.x : (t < 64u ? P.y : (t < 96u ? P.z : P.w));
            if ((w >> (31u - (t & 31u))) & 1u) c = basis[t];
        }
        for (int m = 32; m >= 1; m >>= 1) c = xor4(c, shfl_xor4(c, m));
        if (t == 0u || t == 64u) part[t >> 6] = c;
        __syncthreads();
        const uint4 r = xor4(part[0], part[1]);
        __syncthreads();
        return r;
    };
    basis_of(hp[15], 128u);
    const uint4 h32 = mul_by_basis(hp[15]);
    const uint4 h48 = mul_by_basis(h32);  // (the basis is still H^16's)
    basis_of(h32, 128u);
    const uint4 h64 = mul_by_basis(h32);
    basis_of(h64, 128u);
    const uint4 h128 = mul_by_basis(h64);
    if (t < 128u) {  // the position tables of H^64 (basis[0, 32))
        const uint32_t r = t >> 4, v = t & 15u;
        uint4 e = make_uint4(0, 0, 0, 0);
        for (uint32_t j = 0; j < 4; j++)
            if ((v >> (3 - j)) & 1u) e = xor4(e, basis[4 * r + j]);
        uint32_t* o = rec + kRecPos64 + 4u * t;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
    basis_of(h128, 128u);
    const uint4 h256 = mul_by_basis(h128);
    basis_of(h256, 128u);
    const uint4 h512 = mul_by_basis(h256);
    if (t < 96u) {  // Shoup tables of H^32, H^64, H^128, H^256, H^512 and H^48
        const uint32_t k = t >> 4, v = t & 15u;
        const uint4 P = k == 0u ? h32 : k == 1u ? h64 : k == 2u ? h128 : k == 3u ? h256 : k == 4u ? h512 : h48;
        const uint4 e = gf_tab_entry(P, v);
        uint32_t* o = rec + (k < 5u ? rec_shoup_pow2(5u + k) : kRecShoup48) + 4u * v;
        o[0] = e.x; o[1] = e.y; o[2] = e.z; o[3] = e.w;
    }
}

}  // namespace neb

// ------------------------------------------------------------------------------------------
// Host-side launchers (called by engine.cpp)

extern "C" hipError_t neb_gcm_probe(void) {
    hipFuncAttributes attr;
    return hipFuncGetAttributes(&attr, (const void*)neb::gcm_single_kernel<false>);
}

extern "C" hipError_t neb_gcm_key_setup(const uint8_t* keys, const uint32_t* slots, uint32_t n, uint32_t* table,
                                        hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::gcm_key_setup_kernel, dim3(n), dim3(256), 0, s, keys, slots, table);
    return hipGetLastError();
}

template <class K, class... Extra>
static hipError_t launch_grid(K kern, int threads, uint32_t work_waves, int cu_count, hipStream_t s, Extra... args) {
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint32_t waves = (uint32_t)threads / 64u;
    const uint32_t want = (work_waves + waves - 1) / waves;
    const uint32_t cap = (uint32_t)(per_cu * cu_count);
    const uint32_t grid = want < cap ? want : cap;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, s, args...);
    return hipGetLastError();
}
// the same with `stop` (optional) bound to the dispatch (hipExtLaunchKernel): the event completes
// with the kernel, and no marker packet follows it on the stream
constexpr int kMaxDevices = 64;
template <class K, class... Extra>
static hipError_t launch_grid_stop(K kern, int threads, uint32_t work_waves, int cu_count, hipStream_t s,
                                   hipEvent_t stop, Extra... args) {
    // workgroups per CU, cached per instantiation and device (engines on GPUs of different
    // architectures in one process each get their own)
    static std::atomic<int> cache[kMaxDevices];
    int dev = 0;
    (void)hipGetDevice(&dev);
    int per_cu = dev >= 0 && dev < kMaxDevices ? cache[dev].load(std::memory_order_relaxed) : 0;
    if (per_cu < 1) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        if (dev >= 0 && dev < kMaxDevices) cache[dev].store(per_cu, std::memory_order_relaxed);
    }
    const uint32_t waves = (uint32_t)threads / 64u;
    const uint32_t want = (work_waves + waves - 1) / waves;
    const uint32_t cap = (uint32_t)(per_cu * cu_count);
    const uint32_t grid = want < cap ? want : cap;
    if (grid == 0) return stop ? hipEventRecord(stop, s) : hipSuccess;
    return neb::launch_bound(kern, dim3(grid), dim3(threads), s, stop, args...);
}

// Waves of gcm_single_kernel's grid for a batch of at most n packets (a full pass is that many
// groups of kPpw packets; the packets after the last full pass go to the tail kernel). The TX
// segment kernel uses it to know which segments the tail seals (without the checksum).
extern "C" uint32_t neb_gcm_single_slots(uint32_t n, int cu_count, int open, int hdr_from_dst) {
    const uint32_t groups = (n + neb::kPpw - 1u) / neb::kPpw;
    const void* kern = open ? (const void*)neb::gcm_single_kernel<true>
                            : hdr_from_dst == 2 ? (const void*)neb::gcm_single_kernel<false, true>
                                                : (const void*)neb::gcm_single_kernel<false>;
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, neb::kSingleThreads, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    uint32_t cap = (uint32_t)(per_cu * cu_count);
    // test hook: a smaller grid, so that small batches have a partial last pass (the tail kernel)
    if (const int64_t g = neb::knob(NEB_KNOB_SINGLE_MAX_GRID); g > 0) cap = std::max(1u, std::min<uint32_t>(cap, (uint32_t)g));
    // one workgroup per group up to the cap: a small batch runs one or a few groups per CU
    const uint32_t grid = std::min(groups, cap);
    return grid * neb::kSingleWaves;
}

// One tunnel key (key_hint) for every descriptor.
// Launch on s; `stop` (optional) completes with the kernel itself: an event bound to the dispatch
// (hipExtLaunchKernel) instead of a marker packet recorded after it (a barrier with an
// agent-scope release between two batches, ≈ 3.3 µs).
// (A timing pair armed by neb_time_next_kernel goes to the batch's first kernel: the main kernel, or
// the tail kernel of a small batch.)
template <class K>
static void launch_k(K kern, dim3 grid, dim3 block, hipStream_t s, hipEvent_t stop, const neb::GcmArgs& a) {
    (void)neb::launch_bound(kern, grid, block, s, stop, a);
}

extern "C" hipError_t neb_gcm_batch_single(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                           const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                           int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                           int hdr_from_dst, hipEvent_t stop, const uint8_t* rx) {
    neb::GcmArgs a{d_desc, n, d_arena, d_keys, max_keys, key_hint, d_status, d_n, (uint32_t)hdr_from_dst, 0u, rx};
    const uint32_t groups = (n + neb::kPpw - 1u) / neb::kPpw;
    const bool cs = !open && hdr_from_dst == 2;  // the TX seal with its checksums (tx.hip)
    if (!d_n && !cs && n <= neb::kSmallBatch) {
        a.tail_slots = neb::kTailAll;
        const uint32_t tgrid = std::min<uint32_t>(
            ((n + neb::kTailPpw - 1u) / neb::kTailPpw + neb::kTailWaves - 1u) / neb::kTailWaves,
            2u * (uint32_t)std::max(cu_count, 1));
        if (open && rx)
            launch_k(neb::gcm_single_tail_kernel<true, true>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
        else if (open)
            launch_k(neb::gcm_single_tail_kernel<true>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
        else
            launch_k(neb::gcm_single_tail_kernel<false>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
        return hipGetLastError();
    }
    const uint32_t slots = neb_gcm_single_slots(n, cu_count, open, hdr_from_dst);
    // a partial last pass (at most n packets; the real count may be on the device) goes to the
    // tail kernel, 16 lanes per packet
    const bool tail = groups > slots && (d_n || groups % slots);
    if (tail) a.tail_slots = slots;
    const dim3 grid(slots / neb::kSingleWaves);
    if (grid.x == 0) return hipSuccess;
    hipEvent_t main_stop = tail ? nullptr : stop;  // the stop event goes to the batch's last kernel
    if (open && rx)
        launch_k(neb::gcm_single_kernel<true, false, true>, grid, dim3(neb::kSingleThreads), s, main_stop, a);
    else if (open)
        launch_k(neb::gcm_single_kernel<true>, grid, dim3(neb::kSingleThreads), s, main_stop, a);
    else if (cs)
        launch_k(neb::gcm_single_kernel<false, true>, grid, dim3(neb::kSingleThreads), s, main_stop, a);
    else
        launch_k(neb::gcm_single_kernel<false>, grid, dim3(neb::kSingleThreads), s, main_stop, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !tail) return e;
    // the tail: exact for a host count; for a device count the largest one, under one pass and n
    // packets (a device count may leave a partial pass even when the bound n is a whole number of
    // passes). The grid is capped at two workgroups per CU (as many as fit; the kernel strides over
    // the rest): one workgroup per possible tail wave put 8 Ki mostly empty workgroups behind every
    // TX batch (a 29-packet tail took 20 µs, almost all of it dispatching workgroups that exit).
    const uint32_t tail_pkts = d_n ? std::min(n, slots * neb::kPpw) : n - groups / slots * slots * neb::kPpw;
    const uint32_t tgrid = std::min<uint32_t>(
        ((tail_pkts + neb::kTailPpw - 1u) / neb::kTailPpw + neb::kTailWaves - 1u) / neb::kTailWaves,
        2u * (uint32_t)std::max(cu_count, 1));
    if (open && rx)
        launch_k(neb::gcm_single_tail_kernel<true, true>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
    else if (open)
        launch_k(neb::gcm_single_tail_kernel<true>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
    else
        launch_k(neb::gcm_single_tail_kernel<false>, dim3(tgrid), dim3(neb::kTailWaves * neb::kWave), s, stop, a);
    return hipGetLastError();
}

// Mixed keys: the batch has been regrouped into chunks by neb_sched_build.

#ifdef NEB_WAVE_TRACE
// tools/wave_trace.py: copy out (at most max entries) and reset the chunk kernel's wave timeline
extern "C" NEB_API int neb_debug_wave_trace(void* out, uint32_t max) {
    void* d = nullptr;
    if (hipDeviceSynchronize() != hipSuccess || hipGetSymbolAddress(&d, HIP_SYMBOL(neb::g_wtrace)) != hipSuccess)
        return -1;
    const uint32_t n = std::min(neb::kWaveTraceCap, max);
    if (hipMemcpy(out, d, (size_t)n * 16u, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemset(d, 0, (size_t)neb::kWaveTraceCap * 16u) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return -1;
    return (int)n;
}
#endif

// One packet (the per-packet path): aad[aad_len] and in[in_len] (payload, + tag when opening) go
// in the kernel arguments; the kernel writes len payload bytes (+ the tag when sealing) to `out`
// and the status to *status (pinned host memory, or device memory). hipErrorInvalidValue when the
// packet does not fit kOneBytes (the caller takes the batch path).
extern "C" hipError_t neb_gcm_one(int open, const uint8_t* aad, uint32_t aad_len, const uint8_t* in, uint32_t in_len,
                                  uint32_t len, uint64_t counter, uint8_t* out, int32_t* status, const uint32_t* d_keys,
                                  uint32_t max_keys, uint32_t key, hipStream_t s) {
    const uint32_t pay = (aad_len + 15u) & ~15u;
    if ((uint64_t)pay + in_len > neb::kOneBytes) return hipErrorInvalidValue;
    neb::OneArgs a;
    std::memset(&a, 0, offsetof(neb::OneArgs, in));
    if (aad_len) std::memcpy(a.in, aad, aad_len);
    if (in_len) std::memcpy(a.in + pay, in, in_len);
    a.d.aad_off = 0;
    a.d.src_off = pay;
    a.d.len = len;
    a.d.aad_len = aad_len;
    a.d.counter = counter;
    a.d.key_id = key;
    a.keys = d_keys;
    a.max_keys = max_keys;
    a.key = key;
    a.status = status;
    a.d.dst_off = (uint64_t)(uintptr_t)out;  // the output's address: the kernel rebases it on its argument block
    if (open)
        hipLaunchKernelGGL(neb::gcm_one_kernel<true>, dim3(1), dim3(neb::kOneFillThreads), 0, s, a);
    else
        hipLaunchKernelGGL(neb::gcm_one_kernel<false>, dim3(1), dim3(neb::kOneFillThreads), 0, s, a);
    return hipGetLastError();
}

// A combined launch of n per-packet requests (engine.cpp PktComb): descriptors, statuses and slots
// (kCombSlot bytes each, the descriptors' offsets from `slots`) in pinned host memory.
namespace neb {
// A host-staged chunk's descriptors from pinned host memory into device memory (engine.cpp
// batch_host), many loads in flight at once: the batch kernels then read them from HBM. Read in
// place, each wave's descriptor loads waited behind the staging copies' PCIe traffic.
__global__ __launch_bounds__(256) void copy_desc_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                        uint32_t nvec) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nvec; i += gridDim.x * 256u) dst[i] = src[i];
}
// A host-staged chunk's span between pinned host memory and HBM (engine.cpp batch_host,
// NEB_PIPE_COPY): 16-byte vectors (both ends share their address mod 16), four in flight per lane,
// bytes at the ragged ends.
__global__ __launch_bounds__(256) void copy_span_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                                        size_t head, size_t nvec, size_t bytes) {
    const size_t tid = (size_t)blockIdx.x * 256u + threadIdx.x, nthr = (size_t)gridDim.x * 256u;
    uint4* d = reinterpret_cast<uint4*>(dst + head);
    const uint4* s = reinterpret_cast<const uint4*>(src + head);
    size_t i = tid;
    for (; i + 3u * nthr < nvec; i += 4u * nthr) {
        const uint4 a = s[i], b = s[i + nthr], c = s[i + 2u * nthr], e = s[i + 3u * nthr];
        d[i] = a;
        d[i + nthr] = b;
        d[i + 2u * nthr] = c;
        d[i + 3u * nthr] = e;
    }
    for (; i < nvec; i += nthr) d[i] = s[i];
    for (size_t j = tid; j < head; j += nthr) dst[j] = src[j];
    for (size_t j = head + nvec * 16u + tid; j < bytes; j += nthr) dst[j] = src[j];
}
}  // namespace neb

extern "C" hipError_t neb_copy_span(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    auto* d = static_cast<uint8_t*>(dst);
    auto* src8 = static_cast<const uint8_t*>(src);
    if (((uintptr_t)d & 15u) != ((uintptr_t)src8 & 15u)) return hipErrorInvalidValue;  // (the caller copies)
    const size_t head = std::min(bytes, (size_t)((16u - ((uintptr_t)d & 15u)) & 15u));
    const size_t nvec = (bytes - head) / 16u;
    const uint32_t grid = (uint32_t)std::min<size_t>((nvec + 255u) / 256u, 2048u);
    hipLaunchKernelGGL(neb::copy_span_kernel, dim3(std::max(grid, 1u)), dim3(256), 0, s, d, src8, head, nvec, bytes);
    return hipGetLastError();
}

extern "C" hipError_t neb_copy_desc(neb_desc* dst, const neb_desc* src, uint32_t n, hipStream_t s) {
    static_assert(sizeof(neb_desc) % 16 == 0, "descriptors copy as 16-byte vectors");
    const uint32_t nvec = n * (uint32_t)(sizeof(neb_desc) / 16);
    if (!nvec) return hipSuccess;
    const uint32_t grid = std::min((nvec + 255u) / 256u, 1024u);
    hipLaunchKernelGGL(neb::copy_desc_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<uint4*>(dst),
                       reinterpret_cast<const uint4*>(src), nvec);
    return hipGetLastError();
}

extern "C" hipError_t neb_gcm_one_batch(int open, const neb_desc* descs, int32_t* status, uint8_t* slots, uint32_t n,
                                        const uint32_t* d_keys, uint32_t max_keys, hipStream_t s) {
    if (n == 0 || n > neb::kOneBatchMax) return hipErrorInvalidValue;
    neb::OneBatchDescs a;
    std::memcpy(a.d, descs, n * sizeof(neb_desc));
    const dim3 grid((n + neb::kOneBatchWaves - 1) / neb::kOneBatchWaves), block(neb::kOneBatchWaves * neb::kWave);
    if (open)
        hipLaunchKernelGGL(neb::gcm_one_batch_kernel<true>, grid, block, 0, s, a, status, slots, n, d_keys, max_keys);
    else
        hipLaunchKernelGGL(neb::gcm_one_batch_kernel<false>, grid, block, 0, s, a, status, slots, n, d_keys, max_keys);
    return hipGetLastError();
}

extern "C" hipError_t neb_gcm_batch_chunked(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                            const uint32_t* d_keys, uint32_t max_keys, int32_t* d_status,
                                            const uint32_t* d_sorted, const uint4* d_chunks,
                                            uint32_t* d_counters, uint32_t max_chunks,
                                            int cu_count, hipStream_t s, int hdr_from_dst,
                                            hipEvent_t stop, const uint8_t* rx) {
    neb::GcmArgs a{d_desc, n, d_arena, d_keys, max_keys, NEB_KEYS_MIXED, d_status, nullptr, (uint32_t)hdr_from_dst, 0u, rx};
    neb::ChunkArgs ca{d_sorted, d_chunks, d_counters, max_chunks};
    // one workgroup per chunk up to the occupancy cap (tails make chunks outnumber n / 16), so a
    // small batch's chunks spread over the CUs; the chunk counts are only known on the device:
    // workgroups past them exit before filling their tables. Full chunks first, then the tails.
    const uint32_t bound = max_chunks * (uint32_t)neb::kChunkWaves;
    // stop (optional): an event bound to the kernel's dispatch (no marker packet after it)
    if (open && rx)
        return launch_grid_stop(neb::gcm_chunk_kernel<true, true>, neb::kChunkThreads, bound, cu_count, s, stop, a, ca);
    return open ? launch_grid_stop(neb::gcm_chunk_kernel<true>, neb::kChunkThreads, bound, cu_count, s, stop, a, ca)
                : launch_grid_stop(neb::gcm_chunk_kernel<false>, neb::kChunkThreads, bound, cu_count, s, stop, a, ca);
}
