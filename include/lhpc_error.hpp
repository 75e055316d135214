// lhpc_error.hpp — C++ side of the C-ABI status convention.
//
// Mirrors the reference's CUDA error idiom (lib/gpu/util/include/cudaHelper.cuh:10-27:
// a std::error_category named "CUDA", makeCudaError, throwCudaError(e, file, line)
// → std::system_error) for the lhpc status space of include/lhpc.h.
#pragma once
#ifndef LHPC_ERROR_HPP_
#define LHPC_ERROR_HPP_

#include <string>
#include <system_error>

#include "lhpc.h"

namespace lhpc {

inline const std::error_category &lhpcErrorCategory() noexcept {
  struct Category final : std::error_category {
    const char *name() const noexcept override { return "lhpc"; }
    std::string message(int v) const override { return lhpc_strerror(v); }
  };
  static const Category instance;
  return instance;
}

inline std::error_code makeLhpcError(int status) noexcept { return {status, lhpcErrorCategory()}; }

[[noreturn]] inline void throwLhpcError(int status, const char *file, int line) {
  throw std::system_error(makeLhpcError(status),
                          std::string(file ? file : "[??]") + ":" + std::to_string(line));
}

inline int checkLhpc(int status, const char *file = __builtin_FILE(), int line = __builtin_LINE()) {
  if (status != LHPC_OK) throwLhpcError(status, file, line);
  return status;
}

}  // namespace lhpc
#endif  // LHPC_ERROR_HPP_
