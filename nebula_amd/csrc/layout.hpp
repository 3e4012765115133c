// layout.hpp — device key-table record layout shared by the host engine and the kernels.
#pragma once
#include <stdint.h>

namespace neb {

// One key record per installed tunnel key (12.5 KiB): the first 512 B hold the key schedule and raw
// H powers; the rest holds GHASH lookup tables precomputed at install time (AES-GCM only).
constexpr uint32_t kKeyRecDwords = 3200;
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
static_assert(kRecFull + 32 * 16 * 4 == kKeyRecDwords, "record layout");

// ChaCha20-Poly1305 record
constexpr uint32_t kRecChaKey = 0;      // dwords [0,8): the 256-bit key as 8 little-endian words

constexpr uint64_t kRejectAfterMessages = ~0ULL - (1ULL << 40);

}  // namespace neb
