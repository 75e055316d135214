// sparse/DenseBlock.hpp — leaf B×B tile, drop-in for reference
// lib/sparse/include/DenseBlock.hpp:12-79.
//
// Same layout: m_block[(x & BMask)·B + (y & BMask)] (row-major with x as the
// major index, reference :22, :27, :75-78), value-initialised on construction;
// foreach visits every cell of the tile with its local (x, y) (:63-70).
// Storage is a plain owning array (the reference's tbb::concurrent_vector is
// only resized at construction; concurrent writes to distinct cells are safe
// with either) — not std::vector, whose bool specialisation has no real
// references (the reference benchmarks use DenseBlock<16, bool>).
#pragma once
#ifndef LHPC_SPARSE_DENSEBLOCK_HPP_
#define LHPC_SPARSE_DENSEBLOCK_HPP_

#include <algorithm>
#include <cassert>
#include <cstddef>
#include <memory>

#include "BaseBlock.hpp"

namespace sparse {
namespace details {
using Coord2D = std::pair<std::intptr_t, std::intptr_t>;

// fixed-size, value-initialised, copyable array with real element references
template <typename _Ty>
struct DenseStorage {
  explicit DenseStorage(std::size_t n) : n_(n), p_(new _Ty[n]()) {}
  DenseStorage(const DenseStorage &o) : n_(o.n_), p_(new _Ty[o.n_]) { std::copy(o.p_.get(), o.p_.get() + n_, p_.get()); }
  DenseStorage &operator=(const DenseStorage &o) {
    if (this != &o) {
      DenseStorage t(o);
      std::swap(n_, t.n_);
      std::swap(p_, t.p_);
    }
    return *this;
  }
  DenseStorage(DenseStorage &&) noexcept = default;
  DenseStorage &operator=(DenseStorage &&) noexcept = default;
  _Ty &operator[](std::size_t i) { return p_[i]; }
  const _Ty &operator[](std::size_t i) const { return p_[i]; }
  std::size_t size() const noexcept { return n_; }
  _Ty *begin() { return p_.get(); }
  _Ty *end() { return p_.get() + n_; }
  const _Ty *begin() const { return p_.get(); }
  const _Ty *end() const { return p_.get() + n_; }

 private:
  std::size_t n_;
  std::unique_ptr<_Ty[]> p_;
};
}  // namespace details

template <std::intptr_t BlockSize, typename _Ty>
struct DenseBlock : BlockInfo<BlockSize, true, _Ty> {
  static_assert((BlockSize & (BlockSize - 1)) == 0, "BlockSize must be a power of 2");
  using value_type = _Ty;
  using reference = _Ty &;
  using const_value = const _Ty;
  static constexpr std::intptr_t span_bits = BlockInfo<BlockSize, true, _Ty>::BShift;

  DenseBlock() : m_block(static_cast<std::size_t>(BlockSize * BlockSize)) {}

  std::optional<std::reference_wrapper<value_type>> operator()(const std::intptr_t x,
                                                               const std::intptr_t y) override {
    return std::make_optional(std::ref(m_block[index(x, y)]));
  }
  std::optional<std::reference_wrapper<const_value>> operator()(const std::intptr_t x,
                                                                const std::intptr_t y) const override {
    return std::make_optional(std::cref(m_block[index(x, y)]));
  }
  std::optional<std::reference_wrapper<const_value>> read(const std::intptr_t x,
                                                          const std::intptr_t y) const override {
    return operator()(x, y);
  }
  void write(const std::intptr_t x, const std::intptr_t y, const _Ty &value) override {
    touch_pointer(x, y).get() = value;
  }
  void write(const std::intptr_t x, const std::intptr_t y, _Ty &&value) override {
    touch_pointer(x, y).get() = std::move(value);
  }
  std::optional<std::reference_wrapper<value_type>> fetch_pointer(const std::intptr_t x,
                                                                  const std::intptr_t y) override {
    return operator()(x, y);
  }
  std::reference_wrapper<value_type> touch_pointer(const std::intptr_t x, const std::intptr_t y) override {
    return std::ref(m_block[index(x, y)]);
  }

  // func(local_x, local_y, value&) for every cell, x-major
  template <typename Func>
  void foreach (Func &&func) {
    for (std::intptr_t x = 0; x < BlockSize; ++x)
      for (std::intptr_t y = 0; y < BlockSize; ++y) func(x, y, m_block[static_cast<std::size_t>(x * BlockSize + y)]);
  }
  template <typename Func>
  void foreach (Func &&func) const {
    for (std::intptr_t x = 0; x < BlockSize; ++x)
      for (std::intptr_t y = 0; y < BlockSize; ++y) func(x, y, m_block[static_cast<std::size_t>(x * BlockSize + y)]);
  }

  details::DenseStorage<_Ty> m_block;

 private:
  static std::size_t index(const std::intptr_t x, const std::intptr_t y) {
    constexpr std::intptr_t M = BlockSize - 1;
    return static_cast<std::size_t>((x & M) * BlockSize + (y & M));
  }
};
}  // namespace sparse

#endif  // LHPC_SPARSE_DENSEBLOCK_HPP_
