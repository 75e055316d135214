// sparse/RootGrid.hpp — sparse (x, y) → T map over a block hierarchy,
// drop-in for reference lib/sparse/include/RootGrid.hpp:12-85.
//
// Same API: read(x, y) → std::optional<T>, write(x, y, value),
// foreach(func(x, y, value&)), over a layout such as
// HashBlock<DenseBlock<16,T>>, PointerBlock<N, PointerBlock<M, DenseBlock<B,T>>>
// or HashBlock<PointerBlock<N, DenseBlock<B,T>>> (the reference benchmarks'
// three layouts, test_hpc_benchmark.cpp:859-925).
//
// Corrected semantics: every level receives the global
// coordinates and takes its own disjoint bit range (BaseBlock.hpp), and
// foreach rebuilds the global coordinate as Σ level_index · 2^(span below) —
// the reference shifted by the child's own BShift only, so with ≥ 2 levels
// under the root it reported e.g. (235, 7) for a cell written at (-5, 7).
// As in the reference, a leaf's foreach visits every cell of an allocated
// tile (default-valued ones included), and PointerBlock levels wrap
// coordinates outside their range.
//
// Also here: const read/foreach, and sparse::to_csr / sparse::bounds
// (sparse/ToCSR.hpp) for assembling a CSRMatrix from a grid.
#pragma once
#ifndef LHPC_SPARSE_ROOTGRID_HPP_
#define LHPC_SPARSE_ROOTGRID_HPP_

#include <optional>

#include "BaseBlock.hpp"

namespace sparse {
namespace details {
using Coord2D = std::pair<std::intptr_t, std::intptr_t>;
}  // namespace details

template <typename _Ty, typename _Layout>
struct RootGrid {
  using value_type = _Ty;
  using layout_type = _Layout;

  std::optional<_Ty> read(std::intptr_t x, std::intptr_t y) const { return _read(m_root, x, y); }
  void write(std::intptr_t x, std::intptr_t y, const _Ty &value) { _write(m_root, x, y, value); }
  template <typename Func>
  void foreach (const Func &func) {
    _foreach(m_root, 0, 0, func);
  }
  template <typename Func>
  void foreach (const Func &func) const {
    _foreach(m_root, 0, 0, func);
  }

  _Layout &root() noexcept { return m_root; }
  const _Layout &root() const noexcept { return m_root; }

 private:
  template <typename Node>
  static std::optional<_Ty> _read(const Node &node, std::intptr_t x, std::intptr_t y) {
    if constexpr (Node::is_leaf) {
      auto opt = node.read(x, y);
      if (!opt.has_value()) return std::nullopt;
      return opt->get();
    } else {
      auto next = node.read(x, y);  // global coordinates at every level
      if (!next.has_value()) return std::nullopt;
      return _read(next->get(), x, y);
    }
  }

  template <typename Node>
  static void _write(Node &node, std::intptr_t x, std::intptr_t y, const _Ty &value) {
    if constexpr (Node::is_leaf) {
      node.write(x, y, value);
    } else {
      _write(node.touch_pointer(x, y).get(), x, y, value);
    }
  }

  template <typename Node, typename Func>
  static void _foreach(Node &node, std::intptr_t xBase, std::intptr_t yBase, const Func &func) {
    if constexpr (Node::is_leaf) {
      node.foreach ([&](auto x, auto y, auto &value) { func(xBase + x, yBase + y, value); });
    } else {
      node.foreach ([&](auto x, auto y, auto &child) {
        _foreach(child, xBase + details::shl(x, Node::subblock_shift_bits),
                 yBase + details::shl(y, Node::subblock_shift_bits), func);
      });
    }
  }

  _Layout m_root;
};
}  // namespace sparse

#endif  // LHPC_SPARSE_ROOTGRID_HPP_
