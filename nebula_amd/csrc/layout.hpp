// layout.hpp — device key-table record layout shared by the host engine and the kernels.
#pragma once
#include <stdint.h>

namespace neb {

// One key record per installed tunnel key (28 KiB): the first 512 B hold the key schedule and
// raw H powers; the rest holds GHASH lookup tables precomputed at install time (AES-GCM only).
constexpr uint32_t kKeyRecDwords = 7168;
constexpr uint32_t kKeyRecBytes = kKeyRecDwords * 4;

// AES-256-GCM record
constexpr uint32_t kRecRoundKeys = 0;   // dwords [0,60): 15 round keys, little-endian column words
constexpr uint32_t kRecAlg = 60;        // algorithm tag (NEB_ALG_*); 0 = empty slot
constexpr uint32_t kRecHPow = 64;       // dwords [64,128): H^1..H^16, 4 big-endian words each (GCM bit order)
constexpr uint32_t kNumHPow = 16;
// 4-bit tables M_k[v] = v·H^k for k = 1..16: 16 tables × 16 entries × 4 BE words (Shoup layout)
constexpr uint32_t kRecShoup = 128;
// full 4-bit table of H^kFullPow over all 32 nibble positions: F_p[v] = (v·x^4p)·H^kFullPow
// (reduced), 32 × 16 entries × 4 BE words — a multiply by it is 32 lookups and XORs, no shifts.
// kFullPow = lanes per packet of the single-key kernel (its Horner stride).
constexpr uint32_t kFullPow = 4;
constexpr uint32_t kRecFull = kRecShoup + 16 * 16 * 4;
// position tables T_r[v] = (v·x^4r)·P (reduced), r = 0..7, of P = H^8 and H^16: the Horner
// multiplies of the mixed-key kernel's 8- and 16-lane chunks (its 4-lane chunks use positions 0-7
// of the full H^4 table). 8 × 16 entries × 4 BE words each.
constexpr uint32_t kRecPos8 = kRecFull + 32 * 16 * 4;
constexpr uint32_t kRecPos16 = kRecPos8 + 8 * 16 * 4;
// position tables of H itself: the single-key kernel's final quad Horner (4 multiplies by H)
constexpr uint32_t kRecPos1 = kRecPos16 + 8 * 16 * 4;
// the Shoup table of H^32 and the position tables of H^64: the single-key tail kernel's packets of
// 64 lanes (Horner stride H^64, final tree up to H^32)
constexpr uint32_t kRecShoup32 = kRecPos1 + 8 * 16 * 4;
constexpr uint32_t kRecPos64 = kRecShoup32 + 16 * 4;
// Shoup tables of H^64, H^128, H^256, H^512: with M_1, M_2, M_4, M_8, M_16 and M_32 above, the
// binary powers that take a block to any H^e, e < 1024 (the TX seal's checksum correction)
constexpr uint32_t kRecShoupHi = kRecPos64 + 8 * 16 * 4;
// position tables of H^2 and H^3: with those of H and H^4 above, the single-key kernel's final
// multiplies each lane's accumulator by its own power (one multiply per lane, not four per quad)
constexpr uint32_t kRecPos2 = kRecShoupHi + 4 * 16 * 4;
constexpr uint32_t kRecPos3 = kRecPos2 + 8 * 16 * 4;
// position tables of H^12: with those of H^4 (kRecFull) and H^8, the mixed-key GHASH pass's
// aggregated rounds (gcm_ghash_kernel: A·H^12 ⊕ X_0·H^8 ⊕ X_1·H^4 ⊕ X_2, one reduction)
constexpr uint32_t kRecPos12 = kRecPos3 + 8 * 16 * 4;
// the Shoup table of H^48: with M_16 and M_32, the 64-lane final's quarter powers (GhShoup64)
constexpr uint32_t kRecShoup48 = kRecPos12 + 8 * 16 * 4;
static_assert(kRecShoup48 + 16 * 4 == kKeyRecDwords, "record layout");
// record offset of the Shoup table of H^(2^j), j = 0..9
__host__ __device__ constexpr uint32_t rec_shoup_pow2(uint32_t j) {
    return j < 5u ? kRecShoup + 64u * ((1u << j) - 1u) : (j == 5u ? kRecShoup32 : kRecShoupHi + 64u * (j - 6u));
}
// position tables of H^(2^lg), lg = 0, 2, 3, 4 (lg 0: the mixed-key kernel's one-lane chunks)
__host__ __device__ constexpr uint32_t rec_pos_table(uint32_t lg) {
    return lg == 0u ? kRecPos1 : (lg == 2u ? kRecFull : (lg == 3u ? kRecPos8 : kRecPos16));
}

// ChaCha20-Poly1305 record
constexpr uint32_t kRecChaKey = 0;      // dwords [0,8): the 256-bit key as 8 little-endian words

constexpr uint64_t kRejectAfterMessages = ~0ULL - (1ULL << 40);

}  // namespace neb
