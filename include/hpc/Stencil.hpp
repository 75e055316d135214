// hpc/Stencil.hpp — ghost-cell stencils on MI355X over the reference's
// hpc::HPCHighDimensionFlatArray buffers.
//
//   hpc::blur_x<nblur>(a, b) / hpc::blur_y<nblur>(a, b)
//       a: HPCHighDimensionFlatArray<2,float,G> (G >= nblur), b: <2,float>
//       b(y,x) = Σ_{k=-nblur..nblur} a(y,x+k)  (resp. a(y+k,x)), ascending k,
//       bit-identical to the reference's BM_x_blur / BM_y_blur
//       (tests/test_hpc_benchmark/test_hpc_benchmark.cpp:354-368, :444-457).
//   hpc::stencil7(u, out, c0, c1)   <3,float,1> buffers (BASELINE config C5).
// Host arrays are staged through HBM and the call is synchronous; the raw
// device-pointer forms are in include/lhpc.h.
#pragma once
#ifndef LHPC_HPC_STENCIL_HPP_
#define LHPC_HPC_STENCIL_HPP_

#include <cstdint>

#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "HPCHighDimensionFlatArray.hpp"

namespace hpc {

template <int nblur, std::size_t G, std::size_t AA, class AlA, std::size_t AB, class AlB>
void blur_x(const HPCHighDimensionFlatArray<2, float, G, G, AA, AlA> &a,
            HPCHighDimensionFlatArray<2, float, 0, 0, AB, AlB> &b) {
  static_assert(G >= static_cast<std::size_t>(nblur), "ghost width must cover the blur radius");
  lhpc::checkLhpc(lhpc_blur_x_f32(a.data(), b.data(), static_cast<int64_t>(a.dims()[0]),
                                  static_cast<int64_t>(a.dims()[1]), static_cast<int64_t>(G), nblur, 0,
                                  nullptr));
}

template <int nblur, std::size_t G, std::size_t AA, class AlA, std::size_t AB, class AlB>
void blur_y(const HPCHighDimensionFlatArray<2, float, G, G, AA, AlA> &a,
            HPCHighDimensionFlatArray<2, float, 0, 0, AB, AlB> &b) {
  static_assert(G >= static_cast<std::size_t>(nblur), "ghost width must cover the blur radius");
  lhpc::checkLhpc(lhpc_blur_y_f32(a.data(), b.data(), static_cast<int64_t>(a.dims()[0]),
                                  static_cast<int64_t>(a.dims()[1]), static_cast<int64_t>(G), nblur, 0,
                                  nullptr));
}

template <std::size_t G, std::size_t A1, class Al1, std::size_t A2, class Al2>
void stencil7(const HPCHighDimensionFlatArray<3, float, G, G, A1, Al1> &u,
              HPCHighDimensionFlatArray<3, float, G, G, A2, Al2> &out, float c0, float c1) {
  static_assert(G >= 1, "7-point stencil needs one ghost layer");
  lhpc::checkLhpc(lhpc_stencil7_f32(u.data(), out.data(), static_cast<int64_t>(u.dims()[0]),
                                    static_cast<int64_t>(u.dims()[1]), static_cast<int64_t>(u.dims()[2]),
                                    static_cast<int64_t>(G), c0, c1, 0, nullptr));
}

}  // namespace hpc
#endif  // LHPC_HPC_STENCIL_HPP_
