// sparse/HashBlock.hpp — unbounded root level of the sparse grid, drop-in
// for reference lib/sparse/include/HashBlock.hpp:33-126.
//
// Same interface (operator(), read, write, fetch_pointer, touch_pointer,
// foreach(func(key_x, key_y, child&))) and the same key hash
// (hash_combine of the two coordinates, reference :12-29).  The reference
// keeps the children in a tbb::concurrent_hash_map (TBB is not available
// here); this one is lock-striped: 64 shards, each an
// unordered_map guarded by its own mutex, so concurrent touch_pointer from
// many threads (the reference benchmarks write from `omp parallel for`,
// test_hpc_benchmark.cpp:866-870) creates each child exactly once.  Children
// are heap-allocated and never move, so returned references stay valid.
//
// Coordinates: every block method here takes GLOBAL (x, y); this level's key
// is (floor(x / 2^child_span), floor(y / 2^child_span)) — negative
// coordinates included — and foreach reports keys.
#pragma once
#ifndef LHPC_SPARSE_HASHBLOCK_HPP_
#define LHPC_SPARSE_HASHBLOCK_HPP_

#include <array>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "BaseBlock.hpp"

namespace sparse {
namespace details {
using Coord2D = std::pair<std::intptr_t, std::intptr_t>;

template <typename SizeT>
static void hash_combine_impl(SizeT &seed, SizeT value) {
  seed ^= value + 0x9e3779b9 + (seed << 6) + (seed >> 2);
}

struct Coord2D_HashCompare {
  static size_t hash(const Coord2D &key) {
    std::size_t seed = 0;
    hash_combine_impl(seed, static_cast<std::size_t>(key.first));
    hash_combine_impl(seed, static_cast<std::size_t>(key.second));
    return seed;
  }
  static bool equal(const Coord2D &a, const Coord2D &b) { return a == b; }
  std::size_t operator()(const Coord2D &k) const { return hash(k); }
};
}  // namespace details

template <typename OtherBlock>
struct HashBlock : public BlockInfo<1, false, OtherBlock> {
  using value_type = OtherBlock;
  using reference = OtherBlock &;
  using const_value = const OtherBlock;
  using CurrBlockType = BlockInfo<1, false, OtherBlock>;
  static constexpr bool is_unbounded = true;

  // child span (corrected: see BaseBlock.hpp)
  static constexpr std::intptr_t subblock_shift_bits = SubBlockInfo<OtherBlock>::offset_bits;

  static constexpr int kShards = 64;
  using Shard = std::unordered_map<details::Coord2D, std::unique_ptr<OtherBlock>, details::Coord2D_HashCompare>;

  HashBlock() = default;
  HashBlock(const HashBlock &o) { *this = o; }
  HashBlock &operator=(const HashBlock &o) {
    if (this == &o) return *this;
    for (int i = 0; i < kShards; ++i) {
      std::scoped_lock lk(m_lock[i], o.m_lock[i]);
      m_shard[i].clear();
      for (const auto &kv : o.m_shard[i]) m_shard[i].emplace(kv.first, std::make_unique<OtherBlock>(*kv.second));
    }
    return *this;
  }

  std::optional<std::reference_wrapper<value_type>> operator()(const std::intptr_t x,
                                                               const std::intptr_t y) override {
    OtherBlock *b = find(x, y);
    return b ? std::make_optional(std::ref(*b)) : std::nullopt;
  }
  std::optional<std::reference_wrapper<const_value>> operator()(const std::intptr_t x,
                                                                const std::intptr_t y) const override {
    const OtherBlock *b = find(x, y);
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
    const details::Coord2D key = key_of(x, y);
    const int s = shard_of(key);
    std::lock_guard<std::mutex> lk(m_lock[s]);
    auto &slot = m_shard[s][key];
    if (!slot) slot = std::make_unique<OtherBlock>();
    return std::ref(*slot);
  }

  std::size_t size() const {
    std::size_t n = 0;
    for (int i = 0; i < kShards; ++i) {
      std::lock_guard<std::mutex> lk(m_lock[i]);
      n += m_shard[i].size();
    }
    return n;
  }

  // func(key_x, key_y, child&) over a snapshot of the keys (reference :104-118)
  template <typename Func>
  void foreach (Func &&func) {
    for (auto &[k, b] : snapshot()) func(k.first, k.second, *b);
  }
  template <typename Func>
  void foreach (Func &&func) const {
    for (auto &[k, b] : snapshot()) func(k.first, k.second, static_cast<const OtherBlock &>(*b));
  }

 private:
  static int shard_of(const details::Coord2D &k) {
    return static_cast<int>((details::Coord2D_HashCompare::hash(k) >> 7) % kShards);
  }
  static details::Coord2D key_of(const std::intptr_t x, const std::intptr_t y) {
    return {details::shr_floor(x, subblock_shift_bits), details::shr_floor(y, subblock_shift_bits)};
  }
  OtherBlock *find(const std::intptr_t x, const std::intptr_t y) const {
    const details::Coord2D key = key_of(x, y);
    const int s = shard_of(key);
    std::lock_guard<std::mutex> lk(m_lock[s]);
    auto it = m_shard[s].find(key);
    return it == m_shard[s].end() ? nullptr : it->second.get();
  }
  std::vector<std::pair<details::Coord2D, OtherBlock *>> snapshot() const {
    std::vector<std::pair<details::Coord2D, OtherBlock *>> v;
    for (int i = 0; i < kShards; ++i) {
      std::lock_guard<std::mutex> lk(m_lock[i]);
      for (const auto &kv : m_shard[i]) v.emplace_back(kv.first, kv.second.get());
    }
    return v;
  }

  std::array<Shard, kShards> m_shard;
  mutable std::array<std::mutex, kShards> m_lock;
};
}  // namespace sparse

#endif  // LHPC_SPARSE_HASHBLOCK_HPP_
