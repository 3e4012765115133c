// host_common.hpp — host-side checks shared by the engine (engine.cpp), the batched receive
// (window.cpp) and the submission queue (queue_core.hpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/nebula_aead.h"

// [off, off + len) lies inside [0, cap), written so that no sum can wrap around 2^64.
inline bool span_in(uint64_t off, uint64_t len, uint64_t cap) { return off <= cap && len <= cap - off; }

// Every region a descriptor touches lies inside a host arena of arena_len bytes: the AAD, the
// source (payload, plus the tag when opening) and the destination (payload, plus the tag when
// sealing). Every host-memory batch is checked this way before anything is copied, launched or any
// replay window moves (a kernel access outside a mapped arena would fault the GPU).
inline bool neb_desc_in_arena(const neb_desc& d, int open, size_t arena_len) {
    const uint64_t pay = (uint64_t)d.len + (open ? 16u : 0u), outl = (uint64_t)d.len + (open ? 0u : 16u);
    return span_in(d.src_off, pay, arena_len) && span_in(d.dst_off, outl, arena_len) &&
           span_in(d.aad_off, d.aad_len, arena_len);
}
