// hpc/AlignedAlloc.hpp — drop-in for the reference's lib/hpc/include/AlignedAlloc.hpp.
//
// Same names and semantics: hpc::AlignedAllocator<T, Align = 64> is an STL
// allocator returning Align-aligned storage from std::aligned_alloc and
// throwing std::bad_alloc on failure (reference AlignedAlloc.hpp:29, 42-94);
// hpc::detail::allocate_aligned_memory / deallocate_aligned_memory keep their
// signatures (:13-26).  Differences, both deliberate:
//   * the detail:: functions are `inline`, so the header can be included from
//     more than one translation unit (the reference's are not and fail to
//     link — SURVEY §2c-1);
//   * the request is rounded up to a multiple of Align, which
//     std::aligned_alloc requires (C11 7.22.3.1) and glibc tolerates anyway.
#pragma once
#ifndef LHPC_HPC_ALIGNED_ALLOC_HPP_
#define LHPC_HPC_ALIGNED_ALLOC_HPP_

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <new>
#include <type_traits>
#include <utility>

namespace hpc {
namespace detail {

inline void *allocate_aligned_memory(std::size_t align, std::size_t size) {
  if (size == 0) size = align;
  const std::size_t rounded = (size + align - 1) / align * align;
  return std::aligned_alloc(align, rounded);
}

inline void deallocate_aligned_memory(void *ptr) noexcept { std::free(ptr); }

}  // namespace detail

template <typename T, std::size_t Align = 64>
class AlignedAllocator;

template <std::size_t Align>
class AlignedAllocator<void, Align> {
 public:
  using value_type = void;
  using pointer = void *;
  using const_pointer = const void *;
  template <class U>
  struct rebind {
    using other = AlignedAllocator<U, Align>;
  };
};

template <typename T, std::size_t Align>
class AlignedAllocator {
  static_assert(Align >= alignof(T) && (Align & (Align - 1)) == 0,
                "alignment must be a power of two covering alignof(T)");

 public:
  using value_type = T;
  using pointer = T *;
  using const_pointer = const T *;
  using reference = T &;
  using const_reference = const T &;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using propagate_on_container_move_assignment = std::true_type;
  template <class U>
  struct rebind {
    using other = AlignedAllocator<U, Align>;
  };

  AlignedAllocator() noexcept = default;
  template <class U>
  AlignedAllocator(const AlignedAllocator<U, Align> &) noexcept {}

  size_type max_size() const noexcept { return (~size_type(0) - Align) / sizeof(T); }
  pointer address(reference r) const noexcept { return std::addressof(r); }
  const_pointer address(const_reference r) const noexcept { return std::addressof(r); }

  pointer allocate(size_type n, const void * = nullptr) {
    if (n > max_size()) throw std::bad_alloc();
    void *p = detail::allocate_aligned_memory(Align, n * sizeof(T));
    if (!p) throw std::bad_alloc();
    return static_cast<pointer>(p);
  }
  void deallocate(pointer p, size_type) noexcept { detail::deallocate_aligned_memory(p); }

  template <class U, class... Args>
  void construct(U *p, Args &&...args) {
    ::new (static_cast<void *>(p)) U(std::forward<Args>(args)...);
  }
  template <class U>
  void destroy(U *p) {
    p->~U();
  }
};

template <typename T, std::size_t TA, typename U, std::size_t UA>
inline bool operator==(const AlignedAllocator<T, TA> &, const AlignedAllocator<U, UA> &) noexcept {
  return TA == UA;
}
template <typename T, std::size_t TA, typename U, std::size_t UA>
inline bool operator!=(const AlignedAllocator<T, TA> &, const AlignedAllocator<U, UA> &) noexcept {
  return TA != UA;
}

}  // namespace hpc
#endif  // LHPC_HPC_ALIGNED_ALLOC_HPP_
