// knobs.hpp — process-wide A/B and test knobs (neb_set_knob / neb_get_knob, engine.cpp). Each
// starts from its environment variable, read once; the batch paths read them with one relaxed
// atomic load, so no getenv runs per batch (getenv is not safe beside another thread's setenv).
#pragma once
#include <stdint.h>

#include "../../include/nebula_aead.h"

namespace neb {
int64_t knob(int k);  // engine.cpp
}  // namespace neb
