// hpc/HPCHighDimensionFlatArray.hpp — drop-in for the reference's
// lib/hpc/include/HPCHighDimensionFlatArray.hpp (the host layout contract of
// the stencil buffers and the host x/y vectors of SpMV).
//
// Contract kept bit-for-bit (pinned by tests/test_layout.py against the
// reference header itself via oracle/_ref/ref_probe):
//   * row-major over the PADDED extents e[d] = dim[d] + Low + High, last
//     index fastest: stride[D-1] = 1, stride[d] = stride[d+1]·e[d+1]
//     (reference :161-171);
//   * logical index i[d] ∈ [-Low, dim[d] + High) lives at
//     Σ_d stride[d]·(i[d] + Low) (reference :151-153, :180-187);
//   * every cell, ghosts included, is value-initialised (zero) on
//     construction (reference :135-144);
//   * at() bounds-checks and throws std::out_of_range (reference :107-109,
//     :197-208); operator() does not check (:123-125);
//   * default Alignment 16, default allocator hpc::AlignedAllocator<T, 16>.
// Additions: const overloads of operator()/at(), and dims()/strides()/size()
// accessors so device mirrors (include/hpc/Stencil.hpp) can size HBM copies.
#pragma once
#ifndef LHPC_HPC_HIGH_DIMENSION_FLAT_ARRAY_HPP_
#define LHPC_HPC_HIGH_DIMENSION_FLAT_ARRAY_HPP_

#include <array>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <type_traits>
#include <utility>
#include <vector>

#include "AlignedAlloc.hpp"

namespace hpc {

template <std::size_t Dimension, typename _Ty, std::size_t Low_Bound = 0,
          std::size_t High_Bound = Low_Bound, std::size_t Alignment = 16,
          class Alloc = AlignedAllocator<_Ty, Alignment>>
class HPCHighDimensionFlatArray {
  static_assert(Dimension > 0, "Dimension must larger than zero");
  static_assert(std::is_same_v<std::remove_cv_t<std::remove_reference_t<_Ty>>, _Ty>,
                "_Ty must not be cvref");

  using Extents = std::array<std::size_t, Dimension>;
  using Index = std::array<std::intptr_t, Dimension>;
  static constexpr std::intptr_t kLow = static_cast<std::intptr_t>(Low_Bound);
  static constexpr std::intptr_t kHigh = static_cast<std::intptr_t>(High_Bound);

 public:
  using value_type = _Ty;
  static constexpr std::size_t dimension = Dimension;
  static constexpr std::size_t low_bound = Low_Bound;
  static constexpr std::size_t high_bound = High_Bound;

  template <typename... DimForEachLayer,
            std::enable_if_t<(sizeof...(DimForEachLayer) == Dimension &&
                              std::conjunction_v<std::is_integral<DimForEachLayer>...>),
                             int> = 0>
  explicit HPCHighDimensionFlatArray(const DimForEachLayer &...dims)
      : HPCHighDimensionFlatArray(Extents{static_cast<std::size_t>(dims)...}) {}

  void shrink_to_fit() { _flat.shrink_to_fit(); }

  constexpr _Ty *data() noexcept { return _flat.data(); }
  constexpr const _Ty *data() const noexcept { return _flat.data(); }

  _Ty &at(const Index &indices) { return _flat[static_cast<std::size_t>(safe_linearize(indices))]; }
  const _Ty &at(const Index &indices) const {
    return _flat[static_cast<std::size_t>(safe_linearize(indices))];
  }

  template <typename... Indicies,
            std::enable_if_t<(sizeof...(Indicies) == Dimension &&
                              std::conjunction_v<std::is_integral<Indicies>...>),
                             int> = 0>
  _Ty &operator()(const Indicies &...idxs) noexcept {
    return data()[unsafe_linearize(Index{static_cast<std::intptr_t>(idxs)...})];
  }
  template <typename... Indicies,
            std::enable_if_t<(sizeof...(Indicies) == Dimension &&
                              std::conjunction_v<std::is_integral<Indicies>...>),
                             int> = 0>
  const _Ty &operator()(const Indicies &...idxs) const noexcept {
    return data()[unsafe_linearize(Index{static_cast<std::intptr_t>(idxs)...})];
  }

  // -- additions (not in the reference) --
  const Extents &dims() const noexcept { return _dim; }          // logical extents
  const Extents &strides() const noexcept { return _stride; }    // padded strides
  std::size_t size() const noexcept { return _flat.size(); }     // padded cell count
  std::size_t padded_extent(std::size_t d) const noexcept { return _dim[d] + Low_Bound + High_Bound; }

 protected:
  void resize(const Extents &dim, const _Ty &value = _Ty{}) {
    const auto st = compute_stride_and_total(dim);
    assert(st.second > 0 && "resize() attempted to create zero-sized flat array!");
    _dim = dim;
    _stride = st.first;
    _flat.assign(st.second, value);
  }

  std::intptr_t padded_index(std::intptr_t val) const noexcept { return val + kLow; }

  static constexpr std::pair<Extents, std::size_t> compute_stride_and_total(
      const Extents &dims) noexcept {
    Extents stride{};
    std::size_t running = 1;
    for (std::size_t k = 0; k < Dimension; ++k) {
      const std::size_t d = Dimension - 1 - k;  // innermost first
      stride[d] = running;
      running *= dims[d] + Low_Bound + High_Bound;
    }
    return {stride, running};
  }

  std::intptr_t unsafe_linearize(const Index &idx) const noexcept {
    std::intptr_t off = 0;
    for (std::size_t d = 0; d < Dimension; ++d)
      off += static_cast<std::intptr_t>(_stride[d]) * padded_index(idx[d]);
    return off;
  }

  std::intptr_t safe_linearize(const Index &idx) const {
    for (std::size_t d = 0; d < Dimension; ++d) {
      const std::intptr_t hi = static_cast<std::intptr_t>(_dim[d]) + kHigh;
      if (idx[d] < -kLow || idx[d] >= hi) throw std::out_of_range("invalid index, out of boundary");
    }
    return unsafe_linearize(idx);
  }

 private:
  std::vector<_Ty, Alloc> _flat;
  Extents _dim{};
  Extents _stride{};

  explicit HPCHighDimensionFlatArray(const Extents &extents) { resize(extents); }
};

}  // namespace hpc

#endif  // LHPC_HPC_HIGH_DIMENSION_FLAT_ARRAY_HPP_
