// chacha_poly.hip — ChaCha20-Poly1305 (RFC 8439) seal/open of a packet batch on gfx950 (MI355X).
//
// Replaces the arithmetic behind noiseutil/chachapoly.go:23-48 (x/crypto chacha20poly1305 with
// nonce 00000000 || LE64(n)) for a whole batch.
//
// Work decomposition:
//  * One wavefront holds 4 packets at a time, 16 lanes per packet; each quad of lanes computes one
//    64-byte ChaCha20 block with one column (then one diagonal) quarter-round per lane, the
//    diagonal rotation done by quad permutes, and a 4×4 in-quad transpose hands every lane the 16
//    keystream bytes of "its" payload block.
//  * Poly1305 over AAD‖pad‖CT‖pad‖lengths (n 16-byte blocks) is evaluated as 16 interleaved Horner
//    chains: poly block i goes to lane (i + φ) mod 16, round ⌊(i + φ)/16⌋, with φ chosen so that
//    ciphertext block c sits on lane (c + 4) mod 16 — the lane that holds its keystream. Each
//    lane folds A = A·r^16 + m_i; at the end lane l multiplies by r^(e_l) (e_l = distance of its
//    last block from the end) and the 16 lanes add. r^1..r^16 come from a 4-step parallel prefix
//    product across the lanes (the one-time key r is per packet).
//  * Field arithmetic: 5 × 26-bit limbs, 64-bit partial products.
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstring>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"
#include "device_common.hpp"
#include "layout.hpp"
#include "rxwin.hpp"
#include "timing.hpp"

namespace neb {

constexpr int kChWavesPerWG = 4;  // 1, 2 and 4 measured equal on the uncapped grid, 8 -3%, 16 -13%
constexpr int kChThreads = kChWavesPerWG * kWave;

// ---- ChaCha20 quad ---------------------------------------------------------------------------

// quad_perm DPP: lane w of each quad receives the value of lane sel[w].
template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    constexpr int ctrl = S0 | (S1 << 2) | (S2 << 4) | (S3 << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
// (lane-permuted v) + o and (lane-permuted v) ^ o in one DPP VALU op, quad_perm control Q. The
// s_nop 1 covers the 2 wait states a DPP read needs after a VALU write of its source (inline asm
// is opaque to the hazard recognizer).
template <int Q>
__device__ __forceinline__ uint32_t dpp_add(uint32_t v, uint32_t o) {
    uint32_t r;
    asm("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[%c3,%c4,%c5,%c6] row_mask:0xf bank_mask:0xf"
        : "=v"(r) : "v"(v), "v"(o), "i"(Q & 3), "i"((Q >> 2) & 3), "i"((Q >> 4) & 3), "i"((Q >> 6) & 3));
    return r;
}
template <int Q>
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v, uint32_t o) {
    uint32_t r;
    asm("s_nop 1\n\tv_xor_b32_dpp %0, %1, %2 quad_perm:[%c3,%c4,%c5,%c6] row_mask:0xf bank_mask:0xf"
        : "=v"(r) : "v"(v), "v"(o), "i"(Q & 3), "i"((Q >> 2) & 3), "i"((Q >> 4) & 3), "i"((Q >> 6) & 3));
    return r;
}

#define NEB_QR(a, b, c, d)                \
    a += b; d ^= a; d = rotl(d, 16);      \
    c += d; b ^= c; b = rotl(b, 12);      \
    a += b; d ^= a; d = rotl(d, 8);       \
    c += d; b ^= c; b = rotl(b, 7);

// Lane w of a quad holds state column w: a = x[w], b = x[4+w], c = x[8+w], d = x[12+w].
// Returns the keystream words 4w..4w+3 of the block (bytes 16w..16w+15) as little-endian words.
__device__ __forceinline__ uint4 chacha_quad(uint32_t a0, uint32_t b0, uint32_t c0, uint32_t d0, uint32_t w) {
    uint32_t a = a0, b = b0, c = c0, d = d0;
    // The diagonal round needs b, c, d from lanes w+1, w+2, w+3 and the next column round needs
    // them back. No separate moves: each quarter-round reads the shifted operands through the DPP
    // of its first adds/XORs (v_add_u32_dpp / v_xor_b32_dpp), so b, c, d simply stay in the frame
    // of the round that wrote them — 24 VALU per double round instead of 30.
#define NEB_QR_DPP(P1, P2, P3)                                                          \
    a = dpp_add<P1>(b, a); d = rotl(dpp_xor<P3>(d, a), 16);                              \
    c = dpp_add<P2>(c, d); b = rotl(dpp_xor<P1>(b, c), 12);                              \
    a += b; d ^= a; d = rotl(d, 8);                                                     \
    c += d; b ^= c; b = rotl(b, 7);
#ifndef NEB_CHACHA_DPP
#define NEB_CHACHA_DPP 1
#endif
#if NEB_CHACHA_DPP
    constexpr int kL1 = 0x39, kL2 = 0x4E, kL3 = 0x93;  // quad_perm [1,2,3,0], [2,3,0,1], [3,0,1,2]
    NEB_QR(a, b, c, d)
    NEB_QR_DPP(kL1, kL2, kL3)  // diagonal round: lane w takes b from w+1, c from w+2, d from w+3
#pragma unroll 3
    for (int i = 1; i < 10; i++) {
        NEB_QR_DPP(kL3, kL2, kL1)  // column round, back from the diagonal frame
        NEB_QR_DPP(kL1, kL2, kL3)
    }
    b = qperm<3, 0, 1, 2>(b);
    c = qperm<2, 3, 0, 1>(c);
    d = qperm<1, 2, 3, 0>(d);
#else  // separate quad_perm moves before and after each diagonal round
#pragma unroll 2
    for (int i = 0; i < 10; i++) {
        NEB_QR(a, b, c, d)
        b = qperm<1, 2, 3, 0>(b);
        c = qperm<2, 3, 0, 1>(c);
        d = qperm<3, 0, 1, 2>(d);
        NEB_QR(a, b, c, d)
        b = qperm<3, 0, 1, 2>(b);
        c = qperm<2, 3, 0, 1>(c);
        d = qperm<1, 2, 3, 0>(d);
    }
#endif
#undef NEB_QR_DPP
    a += a0; b += b0; c += c0; d += d0;
    // 4x4 transpose inside the quad: lane w holds row elements (word 4e + w, e = 0..3) and needs
    // words 4w..4w+3, i.e. element w of every lane.
    // stage 1: exchange 2x2 blocks between lanes w and w^2
    const bool hi2 = (w & 2u) != 0;
    uint32_t sa = hi2 ? a : c, sb = hi2 ? b : d;     // values to send
    sa = qperm<2, 3, 0, 1>(sa);
    sb = qperm<2, 3, 0, 1>(sb);
    if (hi2) { a = sa; b = sb; } else { c = sa; d = sb; }
    // stage 2: exchange between lanes w and w^1
    const bool hi1 = (w & 1u) != 0;
    uint32_t sx = hi1 ? a : b, sy = hi1 ? c : d;
    sx = qperm<1, 0, 3, 2>(sx);
    sy = qperm<1, 0, 3, 2>(sy);
    if (hi1) { a = sx; c = sy; } else { b = sx; d = sy; }
    return make_uint4(a, b, c, d);
}

// ---- Poly1305 (mod 2^130 - 5), 5 x 26-bit limbs ------------------------------------------------

struct P5 {
    uint32_t v[5];
};

__device__ __forceinline__ P5 p5_from_words(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3, uint32_t hibit) {
    P5 r;
    r.v[0] = t0 & 0x3ffffffu;
    r.v[1] = ((t0 >> 26) | (t1 << 6)) & 0x3ffffffu;
    r.v[2] = ((t1 >> 20) | (t2 << 12)) & 0x3ffffffu;
    r.v[3] = ((t2 >> 14) | (t3 << 18)) & 0x3ffffffu;
    r.v[4] = (t3 >> 8) | (hibit << 24);
    return r;
}

// a·b mod p (partially reduced: limbs < 2^26 + small)
__device__ __forceinline__ P5 p5_mul(const P5& a, const P5& b) {
    const uint32_t s1 = b.v[1] * 5u, s2 = b.v[2] * 5u, s3 = b.v[3] * 5u, s4 = b.v[4] * 5u;
    uint64_t d0 = (uint64_t)a.v[0] * b.v[0] + (uint64_t)a.v[1] * s4 + (uint64_t)a.v[2] * s3 + (uint64_t)a.v[3] * s2 + (uint64_t)a.v[4] * s1;
    uint64_t d1 = (uint64_t)a.v[0] * b.v[1] + (uint64_t)a.v[1] * b.v[0] + (uint64_t)a.v[2] * s4 + (uint64_t)a.v[3] * s3 + (uint64_t)a.v[4] * s2;
    uint64_t d2 = (uint64_t)a.v[0] * b.v[2] + (uint64_t)a.v[1] * b.v[1] + (uint64_t)a.v[2] * b.v[0] + (uint64_t)a.v[3] * s4 + (uint64_t)a.v[4] * s3;
    uint64_t d3 = (uint64_t)a.v[0] * b.v[3] + (uint64_t)a.v[1] * b.v[2] + (uint64_t)a.v[2] * b.v[1] + (uint64_t)a.v[3] * b.v[0] + (uint64_t)a.v[4] * s4;
    uint64_t d4 = (uint64_t)a.v[0] * b.v[4] + (uint64_t)a.v[1] * b.v[3] + (uint64_t)a.v[2] * b.v[2] + (uint64_t)a.v[3] * b.v[1] + (uint64_t)a.v[4] * b.v[0];
    P5 r;
    uint64_t c;
    c = d0 >> 26; r.v[0] = (uint32_t)d0 & 0x3ffffffu; d1 += c;
    c = d1 >> 26; r.v[1] = (uint32_t)d1 & 0x3ffffffu; d2 += c;
    c = d2 >> 26; r.v[2] = (uint32_t)d2 & 0x3ffffffu; d3 += c;
    c = d3 >> 26; r.v[3] = (uint32_t)d3 & 0x3ffffffu; d4 += c;
    c = d4 >> 26; r.v[4] = (uint32_t)d4 & 0x3ffffffu;
    uint64_t t0 = (uint64_t)r.v[0] + c * 5u;
    r.v[0] = (uint32_t)t0 & 0x3ffffffu;
    r.v[1] += (uint32_t)(t0 >> 26);
    return r;
}

__device__ __forceinline__ P5 p5_add(const P5& a, const P5& b) {
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = a.v[i] + b.v[i];
    return r;
}

__device__ __forceinline__ P5 p5_shfl(const P5& a, int src) {
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = (uint32_t)__shfl((int)a.v[i], src);
    return r;
}
__device__ __forceinline__ P5 p5_shfl_xor(const P5& a, int m) {
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], m);
    return r;
}

// Final: full reduction mod p, then (h + s) mod 2^128 as four little-endian words.
__device__ __forceinline__ uint4 p5_finish(P5 h, uint4 s) {
    uint32_t c;
    // carry-propagate (limbs may be up to ~2^31 after the lane sum)
    c = h.v[0] >> 26; h.v[0] &= 0x3ffffffu; h.v[1] += c;
    c = h.v[1] >> 26; h.v[1] &= 0x3ffffffu; h.v[2] += c;
    c = h.v[2] >> 26; h.v[2] &= 0x3ffffffu; h.v[3] += c;
    c = h.v[3] >> 26; h.v[3] &= 0x3ffffffu; h.v[4] += c;
    c = h.v[4] >> 26; h.v[4] &= 0x3ffffffu; h.v[0] += c * 5u;
    c = h.v[0] >> 26; h.v[0] &= 0x3ffffffu; h.v[1] += c;
    c = h.v[1] >> 26; h.v[1] &= 0x3ffffffu; h.v[2] += c;
    c = h.v[2] >> 26; h.v[2] &= 0x3ffffffu; h.v[3] += c;
    c = h.v[3] >> 26; h.v[3] &= 0x3ffffffu; h.v[4] += c;
    c = h.v[4] >> 26; h.v[4] &= 0x3ffffffu; h.v[0] += c * 5u;
    c = h.v[0] >> 26; h.v[0] &= 0x3ffffffu; h.v[1] += c;
    // g = h + 5 - 2^130; pick g if it did not borrow
    uint32_t g0 = h.v[0] + 5u; c = g0 >> 26; g0 &= 0x3ffffffu;
    uint32_t g1 = h.v[1] + c; c = g1 >> 26; g1 &= 0x3ffffffu;
    uint32_t g2 = h.v[2] + c; c = g2 >> 26; g2 &= 0x3ffffffu;
    uint32_t g3 = h.v[3] + c; c = g3 >> 26; g3 &= 0x3ffffffu;
    uint32_t g4 = h.v[4] + c - (1u << 26);
    uint32_t mask = (g4 >> 31) - 1u;  // all ones if g4 did not go negative
    h.v[0] = (h.v[0] & ~mask) | (g0 & mask);
    h.v[1] = (h.v[1] & ~mask) | (g1 & mask);
    h.v[2] = (h.v[2] & ~mask) | (g2 & mask);
    h.v[3] = (h.v[3] & ~mask) | (g3 & mask);
    h.v[4] = (h.v[4] & ~mask) | (g4 & mask);
    uint32_t w0 = h.v[0] | (h.v[1] << 26);
    uint32_t w1 = (h.v[1] >> 6) | (h.v[2] << 20);
    uint32_t w2 = (h.v[2] >> 12) | (h.v[3] << 14);
    uint32_t w3 = (h.v[3] >> 18) | (h.v[4] << 8);
    uint64_t t = (uint64_t)w0 + s.x;
    w0 = (uint32_t)t;
    t = (uint64_t)w1 + s.y + (t >> 32);
    w1 = (uint32_t)t;
    t = (uint64_t)w2 + s.z + (t >> 32);
    w2 = (uint32_t)t;
    w3 = w3 + s.w + (uint32_t)(t >> 32);
    return make_uint4(w0, w1, w2, w3);
}

__device__ __forceinline__ uint4 xor4c(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

// ---- batch kernel ----------------------------------------------------------------------------

struct ChachaArgs {
    const neb_desc* desc;
    uint32_t npkt;
    uint8_t* arena;
    const uint32_t* keys;
    uint32_t max_keys;
    uint32_t key_hint;
    int32_t* status;
    const uint32_t* npkt_dev;  // optional: the batch's packet count in device memory (min with npkt)
    uint32_t hdr_from_dst;     // TX batches: the first `flags` plaintext bytes from dst (GcmArgs)
    const uint8_t* adm;        // the device receive's admission mask (GcmArgs::adm; RX instantiations)
};

// Payload and AAD blocks loaded one round ahead of their use (1) or in their round (0). Off: a
// round ahead measured 2-3% slower on C4 (110.0 vs 107.1 µs per seal launch, rocprof A/B,
// profiles/r2_s3/ab_chacha_prefetch): the kernel is bound by VALU issue, not by load latency.
// One wave's group of 4 packets (16 lanes each): packets 4·grp .. 4·grp + 3 of the batch, the
// descriptor of packet p from desc_of(p).
template <bool OPEN, bool RX = false, class DF>
__device__ __forceinline__ void chacha_group(const ChachaArgs& args, uint32_t grp, uint32_t npkt, DF&& desc_of) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l = lane & 15u;
    const uint32_t w = l & 3u;      // column within the quad
    const uint32_t j = l >> 2;      // quad within the packet
    const uint32_t q = lane >> 4;   // packet slot within the wave
    const uint32_t pbase = lane & ~15u;  // first lane of this packet
    constexpr uint32_t kConst[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    {
        const uint32_t p = grp * 4u + q;
        // the device receive opens only what its windows admitted (the rest keep the plan's status)
        const bool valid = p < npkt && !(RX && !args.adm[p]);
        neb_desc d = {};
        if (valid) d = desc_of(p);
        uint32_t st = NEB_STATUS_OK;
        if (args.key_hint != NEB_KEYS_MIXED && d.key_id != args.key_hint) st = NEB_STATUS_BAD_KEY;
        const uint32_t* rec = args.keys + (size_t)d.key_id * kKeyRecDwords;
        if (st == NEB_STATUS_OK && (d.key_id >= args.max_keys || rec[kRecAlg] != NEB_ALG_CHACHAPOLY))
            st = NEB_STATUS_BAD_KEY;
        if (!OPEN && st == NEB_STATUS_OK && d.counter >= kRejectAfterMessages) st = NEB_STATUS_EXHAUSTED;
        const bool run = valid && st == NEB_STATUS_OK;

        const uint32_t na = (d.aad_len + 15u) >> 4;
        const uint32_t m = (d.len + 15u) >> 4;
        const uint32_t n = na + m + 1u;
        const uint32_t phi = (4u - (na & 15u)) & 15u;
        const uint32_t kappa = (na + phi - 4u) >> 4;
        const uint32_t last = n - 1u + phi;
        const uint32_t nrounds = run ? (last >> 4) + 1u : 0u;
        const uint32_t t = (last & 15u) + 1u;
        uint32_t rmax = nrounds;
        rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, 16));
        rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, 32));
        if (rmax == 0u) {  // (wave-uniform)
            if (valid && l == 15u) args.status[p] = (int32_t)st;
            return;
        }

        // state column w: a = constant, b = key word w, c = key word 4+w, d = counter / nonce
        const uint32_t ka = run ? rec[kRecChaKey + w] : 0u;
        const uint32_t kc = run ? rec[kRecChaKey + 4u + w] : 0u;
        // nonce = 00000000 || LE64(n): state words 13,14,15 = 0, lo32(n), hi32(n) (chachapoly.go:30-34)
        const uint32_t dn = w == 2u ? (uint32_t)d.counter : (w == 3u ? (uint32_t)(d.counter >> 32) : 0u);
        // pre-pass: quads compute blocks 0..3; block 0 -> one-time Poly1305 key (lanes 0,1)
        uint4 ks = chacha_quad(kConst[w], ka, kc, w == 0u ? j : dn, w);
        const uint32_t src_r = pbase, src_s = pbase | 1u;
        uint4 rk = make_uint4(__shfl((int)ks.x, src_r), __shfl((int)ks.y, src_r), __shfl((int)ks.z, src_r), __shfl((int)ks.w, src_r));
        uint4 sk = make_uint4(__shfl((int)ks.x, src_s), __shfl((int)ks.y, src_s), __shfl((int)ks.z, src_s), __shfl((int)ks.w, src_s));
        rk.x &= 0x0fffffffu; rk.y &= 0x0ffffffcu; rk.z &= 0x0ffffffcu; rk.w &= 0x0ffffffcu;
        const P5 r1 = p5_from_words(rk.x, rk.y, rk.z, rk.w, 0u);
        // r^(l+1) by a Hillis-Steele prefix product over the 16 lanes
        P5 pw = r1;
#pragma unroll
        for (uint32_t s = 1; s < 16; s <<= 1) {
            P5 o = p5_shfl(pw, (int)(lane - s));
            P5 prod = p5_mul(pw, o);
            if (l >= s) pw = prod;
        }
        const P5 r16 = p5_shfl(pw, (int)(pbase | 15u));

        uint8_t* arena = args.arena;
        P5 A = {{0, 0, 0, 0, 0}};
        // the lane's input block of round rho (AAD or payload; zero for the length block and
        // outside the packet), loaded one round ahead so its latency overlaps a round of ChaCha
        const uint32_t hdr = args.hdr_from_dst ? d.flags : 0u;
        auto fetch = [&](uint32_t rho) -> uint4 {
            uint4 b = make_uint4(0, 0, 0, 0);
            const int32_t i = (int32_t)(16u * rho + l) - (int32_t)phi;
            if (rho < nrounds && i >= 0 && i < (int32_t)(na + m)) {
                if (i < (int32_t)na) {
                    const uint32_t off = 16u * (uint32_t)i;
                    b = load_block(arena + d.aad_off + off, min(16u, d.aad_len - off));
                } else {
                    const uint32_t off = 16u * ((uint32_t)i - na);
                    const uint32_t nb = min(16u, d.len - off);
                    b = off < hdr ? load_block_hdr(arena + d.dst_off + off, arena + d.src_off + off, nb, hdr - off)
                                  : load_block(arena + d.src_off + off, nb);
                }
            }
            return b;
        };
        // whole-block rounds need dword-aligned AAD, source and destination (load_u4_a4 / store_u4_a4)
        const bool a4 =
            (((uintptr_t)(arena + d.src_off) | (uintptr_t)(arena + d.dst_off) | (uintptr_t)(arena + d.aad_off)) & 3u) == 0u;
        // (loading each round's block one round ahead measured 2-3% slower: DESIGN.md §3.3)
        for (uint32_t rho = 0; rho < rmax; rho++) {
            {
                // A round in which every lane of the wave holds a whole block — AAD or payload —
                // or lies before the packet's first block (round 0's lanes below φ): one straight
                // path, without the length-block, partial-block and header-from-dst cases below.
                // At 1300 B that is every round but a packet's last.
                const int32_t i = (int32_t)(16u * rho + l) - (int32_t)phi;
                const bool is_data = i >= (int32_t)na;
                const uint32_t off = 16u * ((uint32_t)i - na);
                const bool ok = rho < nrounds && a4 &&
                                (i < 0 || (is_data ? off + 16u <= d.len && off >= hdr : 16u * (uint32_t)i + 16u <= d.aad_len));
                if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) {  // (wave-uniform)
                    uint4 in = make_uint4(0, 0, 0, 0);
                    if (i >= 0) in = load_u4_a4(is_data ? arena + d.src_off + off : arena + d.aad_off + 16u * (uint32_t)i);
                    if (rho > kappa) ks = chacha_quad(kConst[w], ka, kc, w == 0u ? 4u * (rho - kappa) + j : dn, w);
                    uint4 c = in;
                    if (is_data) {
                        const uint4 out = xor4c(in, ks);
                        store_u4_a4(arena + d.dst_off + off, out);
                        if (!OPEN) c = out;
                    }
                    // lanes before the first block: zero words and no 2^128 bit, so A stays 0
                    A = p5_add(p5_mul(A, r16), p5_from_words(c.x, c.y, c.z, c.w, i >= 0 ? 1u : 0u));
                    continue;
                }
            }
            if (rho >= nrounds) continue;
            const uint4 blk = fetch(rho);
            if (rho > kappa) ks = chacha_quad(kConst[w], ka, kc, w == 0u ? 4u * (rho - kappa) + j : dn, w);
            const int32_t i = (int32_t)(16u * rho + l) - (int32_t)phi;  // poly block index
            if (i < 0 || i >= (int32_t)n) continue;
            P5 mi;
            if (i < (int32_t)na) {
                mi = p5_from_words(blk.x, blk.y, blk.z, blk.w, 1u);
            } else if (i < (int32_t)(na + m)) {
                uint32_t off = 16u * ((uint32_t)i - na);
                uint32_t nb = min(16u, d.len - off);
                const uint4 in = blk;
                uint4 out = xor4c(in, mask_block(ks, nb));
                store_block(arena + d.dst_off + off, out, nb);
                uint4 c = OPEN ? in : out;
                mi = p5_from_words(c.x, c.y, c.z, c.w, 1u);
            } else {
                mi = p5_from_words(d.aad_len, 0u, d.len, 0u, 1u);
            }
            A = p5_add(p5_mul(A, r16), mi);
        }
        if (run) {  // (the packet's 16 lanes alike: the shuffles stay within the packet)
            // lane l's last block is e_l = ((t - l - 1) mod 16) + 1 blocks from the end
            const uint32_t e = ((t - l - 1u) & 15u) + 1u;
            P5 re = p5_shfl(pw, (int)(pbase | (e - 1u)));
            P5 h = p5_mul(A, re);
#pragma unroll
            for (int s = 1; s < 16; s <<= 1) h = p5_add(h, p5_shfl_xor(h, s));
            uint4 tag = p5_finish(h, sk);
            uint32_t fail = 0;
            if (l == 15u) {
                if constexpr (!OPEN) {
                    store_block(arena + d.dst_off + d.len, tag, 16);
                } else {
                    uint4 rt = load_block(arena + d.src_off + d.len, 16);
                    uint4 df = xor4c(rt, tag);
                    fail = (df.x | df.y | df.z | df.w) != 0u;
                }
            }
            if constexpr (OPEN) {
                fail = (uint32_t)__shfl((int)fail, (int)(pbase | 15u));
                if (fail) {
                    for (uint32_t off = 16u * l; off < d.len; off += 256u)
                        store_block(arena + d.dst_off + off, make_uint4(0, 0, 0, 0), min(16u, d.len - off));
                    st = NEB_STATUS_AUTH_FAILED;
                }
            }
        }
        if (valid && l == 15u) args.status[p] = (int32_t)st;
    }
}

template <bool OPEN, bool RX = false>
__global__ __launch_bounds__(kChThreads) void chacha_batch_kernel(ChachaArgs args) {
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t npkt = args.npkt;
    if (args.npkt_dev) npkt = min(npkt, __builtin_amdgcn_readfirstlane(*args.npkt_dev));
    const uint32_t ngroups = (npkt + 3u) >> 2;
    for (uint32_t grp = blockIdx.x * kChWavesPerWG + wave; grp < ngroups; grp += gridDim.x * kChWavesPerWG)
        chacha_group<OPEN, RX>(args, grp, npkt, [&](uint32_t p) { return args.desc[p]; });
}

// One packet, its bytes in the kernel arguments (the per-packet path; aes_gcm.hip gcm_one_kernel
// has the why): lanes 0-15 of one wave.
constexpr uint32_t kChOneBytes = 2048;
struct ChOneArgs {
    neb_desc d;  // offsets from `in`; dst_off = the output's address (rebased in the kernel)
    const uint32_t* keys;
    uint32_t max_keys, key;
    int32_t* status;
    uint32_t pad_[2];
    uint8_t in[kChOneBytes];
};
static_assert(offsetof(ChOneArgs, in) % 16 == 0, "the packet bytes are read as 16-B blocks");
template <bool OPEN>
__global__ __launch_bounds__(kWave) void chacha_one_kernel(ChOneArgs a) {
    // the block's address as an opaque integer: derived from the constant-address kernarg pointer,
    // the output address (base + dst_off) would let the compiler treat the result stores as stores
    // to constant memory and drop them
    uint64_t kb = (uint64_t)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(ChOneArgs, in);
    asm volatile("" : "+s"(kb));
    uint8_t* base = reinterpret_cast<uint8_t*>(kb);
    neb_desc d = a.d;
    d.dst_off = a.d.dst_off - (uint64_t)(uintptr_t)base;
    __shared__ int32_t s_status;
    const ChachaArgs ca{nullptr, 1u, base, a.keys, a.max_keys, a.key, &s_status, nullptr, 0u, nullptr};
    chacha_group<OPEN>(ca, 0u, 1u, [&](uint32_t) { return d; });
    one_publish_status(a.status, &s_status);
}

// Key install of a batch of keys, one workgroup per key: the record is cleared (it may have held
// another algorithm's key) and the raw key written, its algorithm tag last.
__global__ __launch_bounds__(256) void chacha_key_setup_kernel(const uint8_t* __restrict__ keys,
                                                               const uint32_t* __restrict__ slots,
                                                               uint32_t* __restrict__ table) {
    const uint8_t* key = keys + 32u * blockIdx.x;
    uint32_t* rec = table + (size_t)slots[blockIdx.x] * kKeyRecDwords;
    for (uint32_t j = threadIdx.x; j < kKeyRecDwords; j += blockDim.x) rec[j] = 0u;
    __syncthreads();
    const uint32_t i = threadIdx.x;
    if (i < 8u)
        rec[kRecChaKey + i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 | (uint32_t)key[4 * i + 2] << 16 |
                              (uint32_t)key[4 * i + 3] << 24;
    __syncthreads();
    if (i == 0) rec[kRecAlg] = NEB_ALG_CHACHAPOLY;
}

}  // namespace neb

extern "C" hipError_t neb_chacha_key_setup(const uint8_t* keys, const uint32_t* slots, uint32_t n, uint32_t* table,
                                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(neb::chacha_key_setup_kernel, dim3(n), dim3(256), 0, s, keys, slots, table);
    return hipGetLastError();
}

template <bool OPEN, bool RX = false>
static hipError_t launch_chacha(const neb::ChachaArgs& a, int cu_count, hipStream_t s, hipEvent_t stop) {
    (void)cu_count;
    auto kern = neb::chacha_batch_kernel<OPEN, RX>;
    // One workgroup per 4 groups of the batch, not a grid capped at what is resident with the waves
    // striding over the rest: the dispatcher then hands a freed slot the next workgroup, so the
    // waves a SIMD's arbiter serves first (the older) take more of the work instead of idling
    // while the younger finish a fixed share. A/B, alternating (profiles/r5/ab_balance): C4
    // 891-894 -> 981-984 GiB/s, seal 86.0 -> 77.7 µs.
    const uint32_t groups = (a.npkt + 3u) / 4u;
    const uint32_t grid = (groups + neb::kChWavesPerWG - 1) / neb::kChWavesPerWG;
    if (grid == 0) return stop ? hipEventRecord(stop, s) : hipSuccess;
    // stop (optional): bound to the dispatch, so no marker packet follows the batch (hipExtLaunchKernel)
    return neb::launch_bound(kern, dim3(grid), dim3(neb::kChThreads), s, stop, a);
}

// One packet (the per-packet path), as neb_gcm_one.
extern "C" hipError_t neb_chacha_one(int open, const uint8_t* aad, uint32_t aad_len, const uint8_t* in,
                                     uint32_t in_len, uint32_t len, uint64_t counter, uint8_t* out, int32_t* status,
                                     const uint32_t* d_keys, uint32_t max_keys, uint32_t key, hipStream_t s) {
    const uint32_t pay = (aad_len + 15u) & ~15u;
    if ((uint64_t)pay + in_len > neb::kChOneBytes) return hipErrorInvalidValue;
    neb::ChOneArgs a;
    std::memset(&a, 0, offsetof(neb::ChOneArgs, in));
    if (aad_len) std::memcpy(a.in, aad, aad_len);
    if (in_len) std::memcpy(a.in + pay, in, in_len);
    a.d.aad_off = 0;
    a.d.src_off = pay;
    a.d.dst_off = (uint64_t)(uintptr_t)out;
    a.d.len = len;
    a.d.aad_len = aad_len;
    a.d.counter = counter;
    a.d.key_id = key;
    a.keys = d_keys;
    a.max_keys = max_keys;
    a.key = key;
    a.status = status;
    if (open)
        hipLaunchKernelGGL(neb::chacha_one_kernel<true>, dim3(1), dim3(neb::kWave), 0, s, a);
    else
        hipLaunchKernelGGL(neb::chacha_one_kernel<false>, dim3(1), dim3(neb::kWave), 0, s, a);
    return hipGetLastError();
}

extern "C" hipError_t neb_chacha_batch(int open, const neb_desc* d_desc, uint32_t n, uint8_t* d_arena,
                                       const uint32_t* d_keys, uint32_t max_keys, uint32_t key_hint,
                                       int32_t* d_status, const uint32_t* d_n, int cu_count, hipStream_t s,
                                       int hdr_from_dst, hipEvent_t stop, const uint8_t* rx) {
    neb::ChachaArgs a{d_desc, n, d_arena, d_keys, max_keys, key_hint, d_status, d_n, (uint32_t)hdr_from_dst, rx};
    if (open && rx) return launch_chacha<true, true>(a, cu_count, s, stop);
    return open ? launch_chacha<true>(a, cu_count, s, stop) : launch_chacha<false>(a, cu_count, s, stop);
}
