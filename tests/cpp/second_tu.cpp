// second translation unit including the drop-in headers (ODR check)
#include <AlignedAlloc.hpp>
#include <HPCHighDimensionFlatArray.hpp>

int second_tu_sum(int n) {
  hpc::HPCHighDimensionFlatArray<1, int, 1> v(n);
  int s = 0;
  for (int i = 0; i < n; ++i) v(i) = i;
  for (int i = 0; i < n; ++i) s += v(i);
  return s;
}
