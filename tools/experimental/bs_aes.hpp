// bs_aes.hpp — bitsliced AES-256-CTR on the VALU for the single-key GCM kernel (aes_gcm.hip).
//
// Why: the T-table AES + table GHASH of gcm_single_kernel saturate the LDS (one ds_read_b32 per
// 2 LDS cycles per wave; 83% of peak is what a pure lookup stream reaches, tools/micro) while the
// VALU issues only about half as fast as it could. This pass computes the CTR keystream of 8 of a
// packet's rounds with no LDS access at all, so each wave runs 8 rounds on the VALU and the rest on
// the LDS, and waves on one SIMD take their VALU pass at different rounds.
//
// Layout (tools/bs_model.py is the step-for-step CPU model, checked against the oracle by
// tests/test_bitsliced_model.py). Lane c = lane & 3 of a packet's quad holds column c of the AES
// state of 32 counter blocks as 32 bit planes P[i][b] (row i = byte 4c + i of the block, bit b);
// bit k of a plane belongs to block k, whose counter is base + k (counters < 256: bytes 12-14 of
// the counter block are zero).
//  * SubBytes: the generated Boyar-Peralta network (bs_sbox.inc, 84 bitop3/logic ops per row).
//  * ShiftRows: row i of lane c comes from lane (c + i) & 3 — one DPP quad_perm per plane.
//  * MixColumns + AddRoundKey: plane XORs; the round-key bits are sign-extended into plane masks
//    (v_bfe_i32) from the lane's column word of the round key.
//  * Out: a 32x32 bit transpose gives D[k] = column word c of block k; a two-stage DPP exchange
//    across the quad gives lane l the four column words of block 4j + l (consumption round j).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../nebula_amd/csrc/layout.hpp"

namespace neb {

template <int TT>
__device__ __forceinline__ uint32_t bs_op3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(TT));
    return r;
}

#include "bs_sbox.inc"

// value of lane (c + I) & 3 of the quad, for lane c
template <int I>
__device__ __forceinline__ uint32_t quad_rot(uint32_t v) {
    constexpr int ctrl = ((0 + I) & 3) | (((1 + I) & 3) << 2) | (((2 + I) & 3) << 4) | (((3 + I) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}
// quad partner lane c ^ X (X = 1 or 2)
template <int X>
__device__ __forceinline__ uint32_t quad_xor(uint32_t v) {
    constexpr int ctrl = (0 ^ X) | ((1 ^ X) << 2) | ((2 ^ X) << 4) | ((3 ^ X) << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, false);
}

// plane mask of bit `bit` of w: all ones or zero (v_bfe_i32)
__device__ __forceinline__ uint32_t bit_mask(uint32_t w, uint32_t bit) {
    return (uint32_t)__builtin_amdgcn_sbfe((int)w, bit, 1);
}

// the lane's column word (c = lane & 3) of round key r
template <class RK>
__device__ __forceinline__ uint32_t bs_rk_col(const RK& rk, int r, uint32_t c) {
    const uint4 k = rk.get(r);
    const uint32_t lo = (c & 1u) ? k.y : k.x, hi = (c & 1u) ? k.w : k.z;
    return (c & 2u) ? hi : lo;
}

// the same for a round index known only at run time: the round key from the key record in
// global memory (rec and r are wave-uniform: scalar loads)
__device__ __forceinline__ uint32_t bs_rk_col_mem(const uint32_t* rec, int r, uint32_t c) {
    const uint4 k = *reinterpret_cast<const uint4*>(rec + kRecRoundKeys + 4 * r);
    const uint32_t lo = (c & 1u) ? k.y : k.x, hi = (c & 1u) ? k.w : k.z;
    return (c & 2u) ? hi : lo;
}

// MixColumns + AddRoundKey on the shifted rows a[i][b] of this lane's column, round key word kw.
// out_i = xtime(a_i ^ a_(i+1)) ^ u ^ a_i ^ k_i with u = a_0 ^ a_1 ^ a_2 ^ a_3.
__device__ __forceinline__ void bs_mix_ark(uint32_t (&a)[4][8], uint32_t kw) {
    uint32_t u[8], a0[8];
#pragma unroll
    for (int b = 0; b < 8; b++) {
        u[b] = bs_op3<0x96>(a[0][b], a[1][b], a[2][b]) ^ a[3][b];
        a0[b] = a[0][b];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t t[8];
#pragma unroll
        for (int b = 0; b < 8; b++) t[b] = a[i][b] ^ (i == 3 ? a0[b] : a[i + 1][b]);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t v = bs_op3<0x96>(u[b], a[i][b], bit_mask(kw, 8 * i + b));
            // xtime: bit 0 <- t7; bits 1, 3, 4 <- t(b-1) ^ t7; others <- t(b-1)
            if (b == 0) a[i][b] = t[7] ^ v;
            else if (b == 1 || b == 3 || b == 4) a[i][b] = bs_op3<0x96>(t[b - 1], t[7], v);
            else a[i][b] = t[b - 1] ^ v;
        }
    }
}

// 32x32 bit transpose: x[r] bit k -> x[k] bit r (rows r = 8i + b of the planes).
__device__ __forceinline__ void bs_transpose32(uint32_t (&x)[32]) {
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const uint32_t m = w == 16 ? 0x0000FFFFu : w == 8 ? 0x00FF00FFu : w == 4 ? 0x0F0F0F0Fu
                         : w == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int r = 0; r < 32; r++) {
            if (r & w) continue;
            const uint32_t t = ((x[r] >> w) ^ x[r + w]) & m;
            x[r + w] ^= t;
            x[r] ^= t << w;
        }
    }
}

// AES-256-CTR keystream of counters base + k (k = 0..31, low byte; bytes 12-14 zero) under the
// nonce words (c1, c2), for the quad this lane belongs to. ks[j] = the 4 column words of block
// 4j + (lane & 3): the keystream this lane needs in consumption round j.
// rec: the key record; every round key is a scalar load from it (rounds 1-13 run in a loop that is
// not unrolled, and loads keep the compiler from hoisting round 0's and 14's 32 plane masks out of
// the packet loop into spilled registers).
// jmask: slots k whose counter is 1 instead (the quad's length block, which takes E_K(J0)).
__device__ __forceinline__ void bs_ctr_pass(uint32_t c1, uint32_t c2, uint32_t base, uint32_t jmask,
                                            const uint32_t* rec, uint32_t lane, uint4 (&ks)[8]) {
    const uint32_t c = lane & 3u;
    uint32_t P[4][8];
    {
        const uint32_t nw = c == 1u ? c1 : (c == 2u ? c2 : 0u);
        const uint32_t w = nw ^ bs_rk_col_mem(rec, 0, c);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int b = 0; b < 8; b++) P[i][b] = bit_mask(w, 8 * i + b);
        // byte 15 (lane 3, row 3): planes of base + k, a bitsliced ripple add of the constant
        // planes of k and the (uniform) bits of base
        const uint32_t is3 = c == 3u ? 0xFFFFFFFFu : 0u;
        constexpr uint32_t kK[8] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u, 0u, 0u, 0u};
        uint32_t carry = 0;
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t bb = bit_mask(base, b);
            uint32_t s = bs_op3<0x96>(kK[b], bb, carry);
            carry = bs_op3<0xE8>(kK[b], bb, carry);  // majority
            s = b == 0 ? (s | jmask) : (s & ~jmask);  // counter 1 in the jmask slots
            P[3][b] = bs_op3<0x78>(P[3][b], s, is3);  // P ^ (s & is3)
        }
    }
#pragma unroll 1
    for (int r = 1; r < 14; r++) {
        // one row's S-box network at a time: interleaving rows multiplies the live temporaries
#pragma unroll
        for (int i = 0; i < 4; i++) {
            bs_sbox(P[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int b = 0; b < 8; b++) {
            P[1][b] = quad_rot<1>(P[1][b]);
            P[2][b] = quad_rot<2>(P[2][b]);
            P[3][b] = quad_rot<3>(P[3][b]);
        }
        bs_mix_ark(P, bs_rk_col_mem(rec, r, c));
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        bs_sbox(P[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
    {
        const uint32_t kw = bs_rk_col_mem(rec, 14, c);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            P[0][b] ^= bit_mask(kw, b);
            P[1][b] = quad_rot<1>(P[1][b]) ^ bit_mask(kw, 8 + b);
            P[2][b] = quad_rot<2>(P[2][b]) ^ bit_mask(kw, 16 + b);
            P[3][b] = quad_rot<3>(P[3][b]) ^ bit_mask(kw, 24 + b);
        }
    }
    uint32_t D[32];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int b = 0; b < 8; b++) D[8 * i + b] = P[i][b];
    bs_transpose32(D);
    // 4x4 exchange per round j: lane c holds column c of blocks 4j..4j+3; lane l wants the four
    // columns of block 4j + l. Stage A swaps with the xor-2 partner, stage B with the xor-1 one.
    const bool hi = (c & 2u) != 0u, odd = (c & 1u) != 0u;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        // every lane runs every DPP move (a DPP source lane must be active); selects come after
        const uint32_t m0 = D[4 * j], m1 = D[4 * j + 1], m2 = D[4 * j + 2], m3 = D[4 * j + 3];
        const uint32_t x0 = quad_xor<2>(m0), x1 = quad_xor<2>(m1), x2 = quad_xor<2>(m2), x3 = quad_xor<2>(m3);
        const uint32_t a0 = hi ? x2 : m0, a1 = hi ? x3 : m1, a2 = hi ? m2 : x0, a3 = hi ? m3 : x1;
        const uint32_t y0 = quad_xor<1>(a0), y1 = quad_xor<1>(a1), y2 = quad_xor<1>(a2), y3 = quad_xor<1>(a3);
        ks[j].x = odd ? y1 : a0;
        ks[j].y = odd ? a1 : y0;
        ks[j].z = odd ? y3 : a2;
        ks[j].w = odd ? a3 : y2;
    }
}

}  // namespace neb
