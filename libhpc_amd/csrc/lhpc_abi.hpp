// lhpc_abi.hpp — the C ABI's exception boundary (no HIP dependency, so the
// host-only translation units include it too).  Every int-returning
// extern "C" entry point wraps its body in try { … } LHPC_ABI_CATCH: no C++
// exception — a host std::vector that cannot allocate, say — crosses the
// boundary (SURVEY §8b error convention: int status, no exceptions).
#pragma once

#include <new>

#include "../../include/lhpc.h"

#define LHPC_ABI_CATCH                     \
  catch (const std::bad_alloc &) {         \
    return LHPC_ERR_ALLOC;                 \
  }                                        \
  catch (...) {                            \
    return LHPC_ERR_INTERNAL;              \
  }
