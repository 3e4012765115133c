// layout.hpp — device key-table record layout shared by the host engine and the kernels.
#pragma once
#include <stdint.h>

namespace neb {

// One key record per installed tunnel key: 128 dwords = 512 B (two 256-B lines).
constexpr uint32_t kKeyRecDwords = 128;
constexpr uint32_t kKeyRecBytes = kKeyRecDwords * 4;

// AES-256-GCM record
constexpr uint32_t kRecRoundKeys = 0;   // dwords [0,60): 15 round keys, little-endian column words
constexpr uint32_t kRecAlg = 60;        // algorithm tag (NEB_ALG_*); 0 = empty slot
constexpr uint32_t kRecHPow = 64;       // dwords [64,128): H^1..H^16, 4 big-endian words each (GCM bit order)
constexpr uint32_t kNumHPow = 16;

// ChaCha20-Poly1305 record
constexpr uint32_t kRecChaKey = 0;      // dwords [0,8): the 256-bit key as 8 little-endian words

constexpr uint64_t kRejectAfterMessages = ~0ULL - (1ULL << 40);

}  // namespace neb
