// aes_gcm.hip — AES-256-GCM seal/open of a packet batch on gfx950 (MI355X).
//
// Replaces the arithmetic behind noiseutil/aesgcm.go:24-49 (EncryptDanger/DecryptDanger = Go
// crypto/cipher GCM Seal/Open with nonce 00000000 || BE64(n)) for a whole batch of packets.
//
// Work decomposition:
//  * One wavefront holds 4 packets at a time, 16 lanes per packet ("packet group").
//  * A packet's GHASH input is n = a + m + 1 blocks (a AAD blocks, m ciphertext blocks, 1 length
//    block), front-padded with zero blocks to n' = 16·R. In round r lane l owns padded block
//    g' = 16r + l + 1: it runs the AES-CTR keystream for that block (if it is a ciphertext block),
//    loads / XORs / stores the 16 payload bytes (coalesced: 16 lanes × 16 B contiguous per packet),
//    and folds the block into its Horner accumulator A_l = A_l·H^16 ⊕ X.
//  * After R rounds GHASH = Σ_l A_l·H^(16-l): lane l multiplies by H^(NLP - l mod NLP) from a
//    per-lane table, the NLP-lane groups XOR-reduce, and a log-tree over the 16/NLP groups with
//    multipliers H^NLP, H^2NLP, … finishes. The length block always lands on lane 15 of the last
//    round; that lane also computes E_K(J0) for the tag.
//  * AES: T-table in LDS with one copy per lane (64 copies × 1 KiB): lookups are bank-conflict-free
//    and the address is one v_perm_b32. GF(2^128) multiply: 4-bit tables M[v] = v·H^k in LDS
//    (16 × 16 B = 256 B: the 16 entries cover all 64 banks, so a ds_read_b128 of one table never
//    conflicts), 32 independent lookups with deferred reduction (no serial dependency).
//  * SINGLE (one tunnel key for the whole batch, NEB_KEYS_MIXED not set): round keys are
//    wave-uniform (SGPRs), H^1..H^16 tables are built once per workgroup, NLP = 16.
//    MIXED keys: each packet's round keys and 5 tables (H, H^2, H^4, H^8, H^16; NLP = 2) are
//    staged in the wave's LDS slice per packet group.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"
#include "device_common.hpp"
#include "layout.hpp"

#ifndef NEB_WAVES_PER_WG
#define NEB_WAVES_PER_WG 8
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
// LDS

extern __shared__ __attribute__((aligned(16))) char g_lds[];

constexpr uint32_t kTTabBytes = 256 * 64 * 4;  // 64 KiB: entry x at x*256 + lane*4
constexpr uint32_t kGhTabBytes = 256;          // one 4-bit GHASH table
constexpr int kWavesPerWG = NEB_WAVES_PER_WG;
constexpr int kThreads = kWavesPerWG * kWave;

template <int NLP>
struct GhCfg {
    static constexpr int kLevels = NLP == 16 ? 0 : (NLP == 8 ? 1 : (NLP == 4 ? 2 : 3));
    static constexpr int NT = NLP + kLevels;  // tables per key
    static constexpr int kHorner = NT - 1;    // index of H^16
    // power of table t
    __host__ __device__ static constexpr int pw(int t) { return t < NLP ? t + 1 : (NLP << (t - NLP + 1)); }
    // table index of H^s for s = NLP, 2NLP, ..., 8 (tree levels)
    __host__ __device__ static constexpr int tree_tab(int s) {
        return s == NLP ? NLP - 1 : NLP + (s == 2 * NLP ? 0 : (s == 4 * NLP ? 1 : 2));
    }
};

// Multi-key wave slice: per packet [NT tables][round keys 240 B].
constexpr int kMultiNLP = 2;
constexpr uint32_t kMultiPktBytes = GhCfg<kMultiNLP>::NT * kGhTabBytes + 240;
constexpr uint32_t kMultiWaveBytes = 4 * kMultiPktBytes;
constexpr uint32_t kLdsSingle = kTTabBytes + GhCfg<16>::NT * kGhTabBytes;
constexpr uint32_t kLdsMulti = kTTabBytes + kWavesPerWG * kMultiWaveBytes;
static_assert(kLdsMulti <= 163840, "LDS budget");

__device__ __forceinline__ uint32_t lds_u32(uint32_t addr) { return *reinterpret_cast<const uint32_t*>(g_lds + addr); }
__device__ __forceinline__ uint4 lds_u128(uint32_t addr) { return *reinterpret_cast<const uint4*>(g_lds + addr); }
__device__ __forceinline__ void lds_st128(uint32_t addr, uint4 v) { *reinterpret_cast<uint4*>(g_lds + addr) = v; }

// ------------------------------------------------------------------------------------------
// AES-256 encryption of one block per lane (little-endian column words in and out).

// T0[byte k of s] — address = (byte << 8) | lane*4 built with one v_perm_b32.
__device__ __forceinline__ uint32_t tlook(uint32_t s, uint32_t lb, int k) {
    return lds_u32(perm(s, lb, 0x0C0C0000u | ((4u + (uint32_t)k) << 8)));
}

struct RkRegs {  // wave-uniform round keys (scalar registers)
    const uint32_t* k;
    __device__ __forceinline__ uint4 get(int r) const {
        return make_uint4(k[4 * r], k[4 * r + 1], k[4 * r + 2], k[4 * r + 3]);
    }
};
struct RkLds {  // per-packet round keys staged in LDS
    uint32_t base;
    __device__ __forceinline__ uint4 get(int r) const { return lds_u128(base + 16 * r); }
};

template <class RK>
__device__ __forceinline__ uint4 aes256_block(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t lb,
                                              const RK& rk) {
    uint4 k = rk.get(0);
    s0 ^= k.x; s1 ^= k.y; s2 ^= k.z; s3 ^= k.w;
#pragma unroll
    for (int r = 1; r < 14; r++) {
        k = rk.get(r);
        uint32_t t0 = xor3(tlook(s0, lb, 0), rotr(tlook(s1, lb, 1), 24), rotr(tlook(s2, lb, 2), 16)) ^ rotr(tlook(s3, lb, 3), 8) ^ k.x;
        uint32_t t1 = xor3(tlook(s1, lb, 0), rotr(tlook(s2, lb, 1), 24), rotr(tlook(s3, lb, 2), 16)) ^ rotr(tlook(s0, lb, 3), 8) ^ k.y;
        uint32_t t2 = xor3(tlook(s2, lb, 0), rotr(tlook(s3, lb, 1), 24), rotr(tlook(s0, lb, 2), 16)) ^ rotr(tlook(s1, lb, 3), 8) ^ k.z;
        uint32_t t3 = xor3(tlook(s3, lb, 0), rotr(tlook(s0, lb, 1), 24), rotr(tlook(s1, lb, 2), 16)) ^ rotr(tlook(s2, lb, 3), 8) ^ k.w;
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    k = rk.get(14);
    // last round: SubBytes+ShiftRows; S[x] is byte 1 of T0[x]
    uint32_t o0 = xor3(perm(tlook(s1, lb, 1), tlook(s0, lb, 0), 0x0C0C0501u), perm(tlook(s3, lb, 3), tlook(s2, lb, 2), 0x05010C0Cu), k.x);
    uint32_t o1 = xor3(perm(tlook(s2, lb, 1), tlook(s1, lb, 0), 0x0C0C0501u), perm(tlook(s0, lb, 3), tlook(s3, lb, 2), 0x05010C0Cu), k.y);
    uint32_t o2 = xor3(perm(tlook(s3, lb, 1), tlook(s2, lb, 0), 0x0C0C0501u), perm(tlook(s1, lb, 3), tlook(s0, lb, 2), 0x05010C0Cu), k.z);
    uint32_t o3 = xor3(perm(tlook(s0, lb, 1), tlook(s3, lb, 0), 0x0C0C0501u), perm(tlook(s2, lb, 3), tlook(s1, lb, 2), 0x05010C0Cu), k.w);
    return make_uint4(o0, o1, o2, o3);
}

// ------------------------------------------------------------------------------------------
// GF(2^128), GCM bit order. An element is 4 big-endian words w0..w3; the coefficient of x^j is
// bit 31 - (j mod 32) of w[j / 32], so multiplying by x is a 128-bit logical right shift.

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
    // L·(1 + x + x^2 + x^7) with the shifted-out bits (x^128..x^134) collected in o
    uint32_t t0 = l0 ^ (l0 >> 1) ^ (l0 >> 2) ^ (l0 >> 7);
    uint32_t t1 = xor3(l1, shr64(l0, l1, 1), shr64(l0, l1, 2)) ^ shr64(l0, l1, 7);
    uint32_t t2 = xor3(l2, shr64(l1, l2, 1), shr64(l1, l2, 2)) ^ shr64(l1, l2, 7);
    uint32_t t3 = xor3(l3, shr64(l2, l3, 1), shr64(l2, l3, 2)) ^ shr64(l2, l3, 7);
    uint32_t o = xor3(l3 << 31, l3 << 30, l3 << 25);
    uint32_t of = xor3(o, o >> 1, o >> 2) ^ (o >> 7);
    return make_uint4(xor3(z[0], t0, of), z[1] ^ t1, z[2] ^ t2, z[3] ^ t3);
}

// x · H^k where `tab` is the LDS byte address of M[v] = v·H^k (v's MSB = coefficient x^0).
// 32 independent 16-B lookups; partial products grouped by shift residue and reduced once.
__device__ __forceinline__ uint4 gf_mul_tab(uint4 x, uint32_t tab) {
    const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
    uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 8; r++) {
        uint32_t a[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t v = (xw[q] >> (28 - 4 * r)) & 15u;
            uint4 m = lds_u128(tab + (v << 4));
            a[q] ^= m.x; a[q + 1] ^= m.y; a[q + 2] ^= m.z; a[q + 3] ^= m.w;
        }
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
        // keep at most one residue's 4 lookups (16 VGPRs) in flight per wave
        __builtin_amdgcn_sched_barrier(0);
    }
    return gf_reduce(z);
}

// Entry e (0..15) of the 4-bit table of P: XOR of P·x^j for the set bits (bit 3 ↔ x^0).
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

__device__ __forceinline__ uint4 bswap4(uint4 v) { return make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w)); }
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }
__device__ __forceinline__ uint4 shfl_xor4(uint4 v, int m) {
    return make_uint4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}
__device__ __forceinline__ uint32_t ld_rec(const uint32_t* rec, uint32_t i) { return rec[i]; }
__device__ __forceinline__ uint4 ld_rec4(const uint32_t* rec, uint32_t i) {
    return *reinterpret_cast<const uint4*>(rec + i);
}

// ------------------------------------------------------------------------------------------
// The batch kernel.

struct GcmArgs {
    const neb_desc* desc;
    uint32_t npkt;
    uint8_t* arena;
    const uint32_t* keys;  // key table, kKeyRecDwords per key
    uint32_t max_keys;
    uint32_t key_hint;     // SINGLE: the one key_id
    int32_t* status;
};

template <bool OPEN, bool SINGLE>
__global__ __launch_bounds__(kThreads) void gcm_batch_kernel(GcmArgs args) {
    constexpr int NLP = SINGLE ? 16 : kMultiNLP;
    using G = GhCfg<NLP>;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave = tid >> 6;
    const uint32_t q = lane >> 4;   // packet slot in the wave
    const uint32_t l = lane & 15u;  // lane within the packet
    const uint32_t lb = lane << 2;  // T-table lane column

    // T-table: 64 copies, entry x at x*256 + lane*4
    for (uint32_t i = tid; i < 256u * 64u; i += kThreads)
        reinterpret_cast<uint32_t*>(g_lds)[i] = c_T0.t[i >> 6];

    const uint32_t* srec = args.keys + (size_t)args.key_hint * kKeyRecDwords;
    uint32_t rks[60];
    if constexpr (SINGLE) {
        // one key for the whole batch: tables H^1..H^16 once per workgroup, round keys uniform
        if (tid < 16u * 16u) {
            uint32_t t = tid >> 4, e = tid & 15u;
            uint4 p = ld_rec4(srec, kRecHPow + 4 * t);
            lds_st128(kTTabBytes + t * kGhTabBytes + e * 16u, gf_tab_entry(p, e));
        }
#pragma unroll
        for (int i = 0; i < 60; i++) rks[i] = __builtin_amdgcn_readfirstlane(ld_rec(srec, kRecRoundKeys + i));
    }
    __syncthreads();

    const uint32_t ngroups = (args.npkt + 3u) >> 2;
    const uint32_t wslice = kTTabBytes + wave * kMultiWaveBytes + q * kMultiPktBytes;  // MIXED only
    const uint32_t tabbase = SINGLE ? kTTabBytes : wslice;
    const uint32_t rkbase = wslice + G::NT * kGhTabBytes;

    for (uint32_t grp = blockIdx.x * kWavesPerWG + wave; grp < ngroups; grp += gridDim.x * kWavesPerWG) {
        const uint32_t p = grp * 4u + q;
        const bool valid = p < args.npkt;
        neb_desc d = {};
        if (valid) d = args.desc[p];
        const uint32_t* rec = args.keys + (size_t)d.key_id * kKeyRecDwords;
        uint32_t st = NEB_STATUS_OK;
        if (SINGLE) {
            if (d.key_id != args.key_hint) st = NEB_STATUS_BAD_KEY;
        } else {
            if (d.key_id >= args.max_keys || ld_rec(rec, kRecAlg) != NEB_ALG_AESGCM) st = NEB_STATUS_BAD_KEY;
        }
        if (!OPEN && st == NEB_STATUS_OK && d.counter >= kRejectAfterMessages) st = NEB_STATUS_EXHAUSTED;
        const bool run = valid && st == NEB_STATUS_OK;

        const uint32_t na = (d.aad_len + 15u) >> 4;
        const uint32_t m = (d.len + 15u) >> 4;
        const uint32_t n = na + m + 1u;
        const uint32_t R = run ? (n + 15u) >> 4 : 0u;
        const uint32_t pad = 16u * R - n;
        uint32_t Rmax = R;
        Rmax = max(Rmax, (uint32_t)__shfl_xor((int)Rmax, 16));
        Rmax = max(Rmax, (uint32_t)__shfl_xor((int)Rmax, 32));

        if constexpr (!SINGLE) {
            // stage this packet's round keys and GHASH tables in the wave's LDS slice
            if (run) {
                if (l < 15u) lds_st128(rkbase + 16u * l, ld_rec4(rec, kRecRoundKeys + 4u * l));
#pragma unroll
                for (int t = 0; t < G::NT; t++) {
                    uint4 pw = ld_rec4(rec, kRecHPow + 4u * (uint32_t)(G::pw(t) - 1));
                    lds_st128(tabbase + (uint32_t)t * kGhTabBytes + 16u * l, gf_tab_entry(pw, l));
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }

        // nonce 00000000 || BE64(n) as little-endian words; counter block word 3 = BE32(ctr)
        const uint32_t c1 = bswap32((uint32_t)(d.counter >> 32));
        const uint32_t c2 = bswap32((uint32_t)d.counter);
        uint8_t* arena = args.arena;

        uint4 A = make_uint4(0, 0, 0, 0);
        uint4 ej0 = make_uint4(0, 0, 0, 0);
        for (uint32_t r = 0; r < Rmax; r++) {
            if (r < R) {
                const int32_t g = (int32_t)(16u * r + l + 1u) - (int32_t)pad;  // 1-based GHASH index
                const bool is_aad = g >= 1 && g <= (int32_t)na;
                const bool is_ct = g > (int32_t)na && g <= (int32_t)(na + m);
                const bool is_len = g == (int32_t)n;
                const uint32_t k = (uint32_t)(g - (int32_t)na);  // ciphertext block index (1-based)
                const uint32_t ctr = is_ct ? k + 1u : 1u;
                uint4 ks;
                if constexpr (SINGLE) ks = aes256_block(0u, c1, c2, bswap32(ctr), lb, RkRegs{rks});
                else ks = aes256_block(0u, c1, c2, bswap32(ctr), lb, RkLds{rkbase});
                uint4 X = make_uint4(0, 0, 0, 0);
                if (is_aad) {
                    uint32_t off = 16u * (uint32_t)(g - 1);
                    X = bswap4(load_block(arena + d.aad_off + off, min(16u, d.aad_len - off)));
                }
                if (is_ct) {
                    uint32_t off = 16u * (k - 1u);
                    uint32_t nb = min(16u, d.len - off);
                    uint4 in = load_block(arena + d.src_off + off, nb);
                    uint4 out = xor4(in, mask_block(ks, nb));
                    store_block(arena + d.dst_off + off, out, nb);
                    X = bswap4(OPEN ? in : out);
                }
                if (is_len) {
                    uint64_t abits = (uint64_t)d.aad_len * 8u, cbits = (uint64_t)d.len * 8u;
                    X = make_uint4((uint32_t)(abits >> 32), (uint32_t)abits, (uint32_t)(cbits >> 32), (uint32_t)cbits);
                    ej0 = ks;
                }
                A = (r == 0) ? X : xor4(gf_mul_tab(A, tabbase + G::kHorner * kGhTabBytes), X);
            }
        }

        if (run) {
            // Σ_l A_l·H^(16-l): per-lane powers inside NLP-lane groups, then a tree over the groups
            uint4 V = gf_mul_tab(A, tabbase + (uint32_t)(NLP - 1 - (int)(l % NLP)) * kGhTabBytes);
#pragma unroll
            for (int s = 1; s < NLP; s <<= 1) V = xor4(V, shfl_xor4(V, s));
#pragma unroll
            for (int s = NLP; s < 16; s <<= 1) {
                uint4 mv = gf_mul_tab(V, tabbase + (uint32_t)G::tree_tab(s) * kGhTabBytes);
                uint4 pv = shfl_xor4(V, s), pm = shfl_xor4(mv, s);
                V = ((l / (uint32_t)s) & 1u) ? xor4(pm, V) : xor4(mv, pv);
            }
            uint4 tag = xor4(ej0, bswap4(V));  // valid on lane 15
            uint32_t fail = 0;
            if (l == 15u) {
                if constexpr (!OPEN) {
                    store_block(arena + d.dst_off + d.len, tag, 16);
                } else {
                    uint4 rt = load_block(arena + d.src_off + d.len, 16);
                    uint4 df = xor4(rt, tag);
                    fail = (df.x | df.y | df.z | df.w) != 0u;
                }
            }
            if constexpr (OPEN) {
                fail = (uint32_t)__shfl((int)fail, (int)(lane | 15u));
                if (fail) {
                    for (uint32_t off = 16u * l; off < d.len; off += 256u)
                        store_block(arena + d.dst_off + off, make_uint4(0, 0, 0, 0), min(16u, d.len - off));
                }
                if (fail) st = NEB_STATUS_AUTH_FAILED;
            }
        }
        if (valid && l == 15u) args.status[p] = (int32_t)st;
        if constexpr (!SINGLE) {
            // the next group overwrites this wave's LDS slice
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// ------------------------------------------------------------------------------------------
// Key install: AES-256 key expansion, H = E_K(0), H^1..H^16. One lane; runs once per tunnel key.

__device__ uint8_t sbox_b(uint32_t x) { return (uint8_t)(c_T0.t[x & 255u] >> 8); }
__device__ uint8_t xtime_d(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

__global__ void gcm_key_setup_kernel(const uint8_t* __restrict__ key, uint32_t* __restrict__ rec) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint8_t rk[240];
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
        rec[kRecRoundKeys + i] = (uint32_t)rk[4 * i] | (uint32_t)rk[4 * i + 1] << 8 | (uint32_t)rk[4 * i + 2] << 16 |
                                 (uint32_t)rk[4 * i + 3] << 24;
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
    // powers by bit-serial multiply (SP 800-38D Algorithm 1)
    uint32_t pw[4] = {h[0], h[1], h[2], h[3]};
    for (int k = 0; k < (int)kNumHPow; k++) {
        for (int i = 0; i < 4; i++) rec[kRecHPow + 4 * k + i] = pw[i];
        uint32_t z[4] = {0, 0, 0, 0}, v[4] = {h[0], h[1], h[2], h[3]};
        for (int b = 0; b < 128; b++) {
            if ((pw[b >> 5] >> (31 - (b & 31))) & 1u)
                for (int i = 0; i < 4; i++) z[i] ^= v[i];
            uint32_t lsb = v[3] & 1u;
            v[3] = (v[3] >> 1) | (v[2] << 31); v[2] = (v[2] >> 1) | (v[1] << 31);
            v[1] = (v[1] >> 1) | (v[0] << 31); v[0] = (v[0] >> 1) ^ (lsb ? 0xE1000000u : 0u);
        }
        for (int i = 0; i < 4; i++) pw[i] = z[i];
    }
    rec[kRecAlg] = NEB_ALG_AESGCM;
}

}  // namespace neb

// ------------------------------------------------------------------------------------------
// Host-side launchers (called by engine.cpp)

extern "C" hipError_t neb_gcm_key_setup(const uint8_t* d_key, uint32_t* d_rec, hipStream_t s) {
    hipLaunchKernelGGL(neb::gcm_key_setup_kernel, dim3(1), dim3(64), 0, s, d_key, d_rec);
    return hipGetLastError();
}

template <bool OPEN, bool SINGLE>
static hipError_t launch_gcm(const neb::GcmArgs& a, int cu_count, hipStream_t s) {
    auto kern = neb::gcm_batch_kernel<OPEN, SINGLE>;
    const uint32_t lds = SINGLE ? neb::kLdsSingle : neb::kLdsMulti;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    int per_cu = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, neb::kThreads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint32_t groups = (a.npkt + 3u) / 4u;
    uint32_t want = (groups + neb::kWavesPerWG - 1) / neb::kWavesPerWG;
    uint32_t cap = (uint32_t)(per_cu * cu_count);
    uint32_t grid = want < cap ? want : cap;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(neb::kThreads), lds, s, a);
    return hipGetLastError();
}

extern "C" hipError_t neb_gcm_batch(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                    const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint, int32_t* d_status,
                                    int cu_count, hipStream_t s) {
    neb::GcmArgs a{d_desc, n, d_arena, d_keys, max_keys, key_hint, d_status};
    const bool single = key_hint != NEB_KEYS_MIXED;
    if (open) return single ? launch_gcm<true, true>(a, cu_count, s) : launch_gcm<true, false>(a, cu_count, s);
    return single ? launch_gcm<false, true>(a, cu_count, s) : launch_gcm<false, false>(a, cu_count, s);
}
