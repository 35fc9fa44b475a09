// progops.hpp — operations of the class atom programs (encoder and K0).
#pragma once

#include <cstdint>

namespace sr {

// op = atom << 2 | kind:  acc &= atom | acc &= ~atom | open an ORed term | AND into the open term
enum : int32_t { PROG_AND = 0, PROG_ANDNOT = 1, PROG_TERM_START = 2, PROG_TERM_AND = 3 };

}  // namespace sr
