// sparse/BaseBlock.hpp — block traits / virtual block interface of the
// sparse grid, drop-in for reference lib/sparse/include/BaseBlock.hpp.
//
// Same names and interface as the reference (BlockTraits, BlockInfo,
// SubBlockInfo, details::constexpr_log2 / has_bshift / get_bshift), with two
// corrections:
//  * self-contained: <cstdint> is included (§2c-2: the reference header is
//    not, `std::intptr_t` fails standalone);
//  * SubBlockInfo<Sub>::offset_bits is the child's TOTAL coordinate span
//    (its own BShift plus everything below it), not just its own BShift
//    (reference BaseBlock.hpp:36-37).  With ≥ 2 levels under a Hash/Pointer
//    block the reference indexes overlapping coordinate bits and its
//    RootGrid::foreach reports wrong global coordinates (§2c-5: (-5,7) came
//    back as (235,7)); here every level owns a disjoint bit range.
#pragma once
#ifndef LHPC_SPARSE_BASEBLOCK_HPP_
#define LHPC_SPARSE_BASEBLOCK_HPP_

#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <type_traits>

namespace sparse {
namespace details {
static constexpr inline std::intptr_t constexpr_log2(std::intptr_t n) {
  return (n < 2) ? 0 : 1 + constexpr_log2(n >> 1);
}

template <typename _Ty, typename = void>
struct has_bshift : std::false_type {};
template <typename _Ty>
struct has_bshift<_Ty, std::void_t<decltype(_Ty::BShift)>> : std::is_integral<decltype(_Ty::BShift)> {};

template <typename _Ty, typename = void>
struct get_bshift;
template <typename _Ty>
struct get_bshift<_Ty, std::enable_if_t<has_bshift<_Ty>::value, void>> {
  static constexpr std::intptr_t value = _Ty::BShift;
};

// total coordinate bits a block covers: its own BShift + its child's span
template <typename _Ty, typename = void>
struct span_bits {
  static constexpr std::intptr_t value = get_bshift<_Ty>::value;
};
template <typename _Ty>
struct span_bits<_Ty, std::void_t<decltype(_Ty::span_bits)>> {
  static constexpr std::intptr_t value = _Ty::span_bits;
};

// floor(v / 2^s) and v·2^s for signed coordinates (no UB on negatives)
constexpr std::intptr_t shr_floor(std::intptr_t v, std::intptr_t s) { return v >> s; }
constexpr std::intptr_t shl(std::intptr_t v, std::intptr_t s) {
  return static_cast<std::intptr_t>(static_cast<std::uintptr_t>(v) << s);
}
}  // namespace details

template <typename SubBlock>
struct SubBlockInfo {
  static_assert(details::has_bshift<SubBlock>::value, "SubBlockInfo: SubBlock must define static constexpr BShift");
  static_assert(!SubBlock::is_unbounded, "SubBlockInfo: an unbounded (hash) block can only be the root");
  // total span of the child (corrected; see the header comment)
  static constexpr std::intptr_t offset_bits = details::span_bits<SubBlock>::value;
};

template <std::intptr_t BlockSize, bool IsLeaf>
struct BlockTraits {
  static_assert(BlockSize > 0 && ((BlockSize & (BlockSize - 1)) == 0), "BlockSize must be a power of 2 and > 0");
  static constexpr std::intptr_t B = BlockSize;
  static constexpr std::intptr_t BShift = details::constexpr_log2(B);
  static constexpr std::intptr_t BMask = B - 1;
  static constexpr bool is_leaf = IsLeaf;
  static constexpr bool is_unbounded = false;
};

template <std::intptr_t BlockSize, bool IsLeaf, typename _Ty>
struct BlockInfo : BlockTraits<BlockSize, IsLeaf> {
  using value_type = _Ty;
  using reference = _Ty &;
  using const_value = const _Ty;

  virtual ~BlockInfo() = default;

  virtual std::optional<std::reference_wrapper<value_type>> operator()(const std::intptr_t x,
                                                                       const std::intptr_t y) = 0;
  virtual std::optional<std::reference_wrapper<const_value>> operator()(const std::intptr_t x,
                                                                        const std::intptr_t y) const = 0;
  virtual std::optional<std::reference_wrapper<const_value>> read(const std::intptr_t x,
                                                                  const std::intptr_t y) const = 0;
  virtual void write(const std::intptr_t x, const std::intptr_t y, const _Ty &value) = 0;
  virtual void write(const std::intptr_t x, const std::intptr_t y, _Ty &&value) = 0;
  virtual std::optional<std::reference_wrapper<value_type>> fetch_pointer(const std::intptr_t x,
                                                                          const std::intptr_t y) = 0;
  virtual std::reference_wrapper<value_type> touch_pointer(const std::intptr_t x, const std::intptr_t y) = 0;
};
}  // namespace sparse

#endif  // LHPC_SPARSE_BASEBLOCK_HPP_
