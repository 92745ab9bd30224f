// Internal host-side declarations shared by the libdppo translation units.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>

#include "dppo.h"

namespace dppo {

void set_error(const char* fmt, ...);

// Device-side view of the flat parameter layout (offsets in floats; -1 = absent).
struct ParamOffsets {
  int64_t W1, b1, W2, b2, Wa, ba, Wo, bo, Wc, bc, Wv, bv, ls;
};

ParamOffsets offsets_from_layout(const dppo_dims& d, const dppo_layout& L);

}  // namespace dppo
