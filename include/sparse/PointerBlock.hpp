// sparse/PointerBlock.hpp — fixed N×N grid of lazily created children,
// drop-in for reference lib/sparse/include/PointerBlock.hpp:13-161.
//
// Same interface (has, operator(), read, write, fetch_pointer, touch_pointer,
// access() → WriteAccessor with a per-accessor child cache, foreach, copy
// assignment, m_data of std::atomic<pointer>), and the same lock-free child
// creation: compare-exchange of a freshly allocated child into the null slot,
// the loser deletes its copy (reference :99-125).
//
// Indexing (corrected): the slot of global coordinate (x, y) is
// ((x >> child_span) & BMask, (y >> child_span) & BMask), where child_span is
// the child's TOTAL coordinate span, so stacked levels use disjoint bits.  As
// in the reference (:157-160), coordinates outside the block's range wrap
// (& BMask): a PointerBlock root covers [0, N·2^child_span) per axis and
// foreach reports coordinates in that range.
#pragma once
#ifndef LHPC_SPARSE_POINTERBLOCK_HPP_
#define LHPC_SPARSE_POINTERBLOCK_HPP_

#include <atomic>
#include <map>

#include "BaseBlock.hpp"

namespace sparse {
namespace details {
using Coord2D = std::pair<std::intptr_t, std::intptr_t>;
}  // namespace details

template <std::intptr_t PointerGridSize, typename OtherBlock>
struct PointerBlock : BlockInfo<PointerGridSize, false, OtherBlock> {
  static_assert((PointerGridSize & (PointerGridSize - 1)) == 0, "PointerGridSize must be a power of 2");
  using Base = BlockInfo<PointerGridSize, false, OtherBlock>;

  static constexpr std::intptr_t subblock_shift_bits = SubBlockInfo<OtherBlock>::offset_bits;
  static constexpr std::intptr_t span_bits = Base::BShift + subblock_shift_bits;

  using value_type = OtherBlock;
  using pointer = OtherBlock *;
  using reference = OtherBlock &;
  using const_value = const OtherBlock;

  PointerBlock() {
    for (std::intptr_t i = 0; i < PointerGridSize; ++i)
      for (std::intptr_t j = 0; j < PointerGridSize; ++j) m_data[i][j].store(nullptr, std::memory_order_relaxed);
  }
  PointerBlock(const PointerBlock &o) : PointerBlock() { *this = o; }
  ~PointerBlock() override {
    for (std::intptr_t x = 0; x < PointerGridSize; ++x)
      for (std::intptr_t y = 0; y < PointerGridSize; ++y) delete m_data[x][y].load(std::memory_order_relaxed);
  }

  struct WriteAccessor {
    explicit WriteAccessor(PointerBlock &grid) : m_global(grid) {}
    void write(const std::intptr_t x, const std::intptr_t y, const OtherBlock &value) {
      const auto key = slot(x, y);
      auto it = m_cache.find(key);
      if (it != m_cache.end()) {
        it->second.get() = value;
        return;
      }
      auto ref = m_global.touch_pointer(x, y);
      ref.get() = value;
      m_cache.try_emplace(key, ref);
    }
    PointerBlock &m_global;
    std::map<details::Coord2D, std::reference_wrapper<value_type>> m_cache;
  };

  bool has(std::intptr_t x, std::intptr_t y) const {
    const auto [i, j] = slot(x, y);
    return m_data[i][j].load(std::memory_order_acquire) != nullptr;
  }

  std::optional<std::reference_wrapper<value_type>> operator()(const std::intptr_t x,
                                                               const std::intptr_t y) override {
    const auto [i, j] = slot(x, y);
    pointer b = m_data[i][j].load(std::memory_order_acquire);
    return b ? std::make_optional(std::ref(*b)) : std::nullopt;
  }
  std::optional<std::reference_wrapper<const_value>> operator()(const std::intptr_t x,
                                                                const std::intptr_t y) const override {
    const auto [i, j] = slot(x, y);
    pointer b = m_data[i][j].load(std::memory_order_acquire);
    return b ? std::make_optional(std::cref(*b)) : std::nullopt;
  }
  std::optional<std::reference_wrapper<const_value>> read(const std::intptr_t x,
                                                          const std::intptr_t y) const override {
    return operator()(x, y);
  }
  void write(const std::intptr_t x, const std::intptr_t y, const OtherBlock &value) override {
    touch_pointer(x, y).get() = value;
  }
  void write(const std::intptr_t x, const std::intptr_t y, OtherBlock &&value) override {
    touch_pointer(x, y).get() = std::move(value);
  }
  std::optional<std::reference_wrapper<value_type>> fetch_pointer(const std::intptr_t x,
                                                                  const std::intptr_t y) override {
    return operator()(x, y);
  }
  std::reference_wrapper<value_type> touch_pointer(const std::intptr_t x, const std::intptr_t y) override {
    const auto [i, j] = slot(x, y);
    pointer b = m_data[i][j].load(std::memory_order_acquire);
    if (!b) {
      pointer desired = new OtherBlock;
      pointer expected = nullptr;
      if (m_data[i][j].compare_exchange_strong(expected, desired, std::memory_order_acq_rel,
                                               std::memory_order_acquire)) {
        b = desired;
      } else {
        delete desired;  // another thread published first
        b = expected;
      }
    }
    return std::ref(*b);
  }

  WriteAccessor access() { return WriteAccessor{*this}; }

  // func(slot_x, slot_y, child&) over the populated slots, x-major
  template <typename Func>
  void foreach (Func &&func) {
    for (std::intptr_t x = 0; x < PointerGridSize; ++x)
      for (std::intptr_t y = 0; y < PointerGridSize; ++y)
        if (pointer b = m_data[x][y].load(std::memory_order_acquire)) func(x, y, *b);
  }
  template <typename Func>
  void foreach (Func &&func) const {
    for (std::intptr_t x = 0; x < PointerGridSize; ++x)
      for (std::intptr_t y = 0; y < PointerGridSize; ++y)
        if (pointer b = m_data[x][y].load(std::memory_order_acquire)) func(x, y, static_cast<const OtherBlock &>(*b));
  }

  PointerBlock &operator=(const PointerBlock &other) {
    if (this == &other) return *this;
    for (std::intptr_t x = 0; x < PointerGridSize; ++x)
      for (std::intptr_t y = 0; y < PointerGridSize; ++y) {
        pointer src = other.m_data[x][y].load(std::memory_order_relaxed);
        delete m_data[x][y].exchange(src ? new OtherBlock(*src) : nullptr, std::memory_order_relaxed);
      }
    return *this;
  }

  std::atomic<pointer> m_data[PointerGridSize][PointerGridSize];

 private:
  static details::Coord2D slot(const std::intptr_t x, const std::intptr_t y) {
    return {details::shr_floor(x, subblock_shift_bits) & Base::BMask,
            details::shr_floor(y, subblock_shift_bits) & Base::BMask};
  }
};
}  // namespace sparse

#endif  // LHPC_SPARSE_POINTERBLOCK_HPP_
