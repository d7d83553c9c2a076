// OpenMP parallel sort for host-side metric evaluation (reference analogue:
// include/LightGBM/utils/common.h ParallelSort, used by binary_metric.hpp:200,311).
// Chunks are sorted concurrently, then merged pairwise; each pairwise merge is itself cut
// into independent sub-merges at co-ranked split points, so every round keeps all threads
// busy (the last round merges two halves of the whole array).
#pragma once

#include <omp.h>

#include <algorithm>
#include <vector>

namespace lgap {
namespace common {

template <typename T, typename Cmp>
void ParallelSort(std::vector<T>* v, Cmp cmp) {
  const size_t n = v->size();
  const int nt = std::max(1, omp_get_max_threads());
  if (n < (size_t(1) << 15) || nt == 1) {
    std::sort(v->begin(), v->end(), cmp);
    return;
  }
  int chunks = 1;
  while (chunks < nt) chunks <<= 1;
  std::vector<size_t> bound(chunks + 1);
  for (int c = 0; c <= chunks; ++c) bound[c] = n * static_cast<size_t>(c) / chunks;
  T* src = v->data();
#pragma omp parallel for schedule(static, 1)
  for (int c = 0; c < chunks; ++c) std::sort(src + bound[c], src + bound[c + 1], cmp);
  std::vector<T> buf(n);
  T* dst = buf.data();
  for (int width = 1; width < chunks; width <<= 1) {
    const int merges = chunks / (2 * width);
    const int parts = std::max(1, nt / merges);  // sub-merges per pairwise merge
#pragma omp parallel for schedule(dynamic, 1)
    for (int job = 0; job < merges * parts; ++job) {
      const int m = job / parts, s = job - m * parts;
      const size_t lo = bound[2 * m * width], mid = bound[2 * m * width + width], hi = bound[2 * (m + 1) * width];
      const T* a = src + lo;
      const T* b = src + mid;
      const size_t na = mid - lo, nb = hi - mid;
      if (na == 0) {
        if (s == 0) std::copy(b, b + nb, dst + lo);
        continue;
      }
      // sub-merge s covers a[ia0, ia1) and the b elements ordered before a[ia1] (std::merge
      // order: on ties the a element first)
      const size_t ia0 = na * s / parts, ia1 = na * (s + 1) / parts;
      const size_t ib0 = s == 0 ? 0 : static_cast<size_t>(std::lower_bound(b, b + nb, a[ia0], cmp) - b);
      const size_t ib1 = s + 1 == parts ? nb : static_cast<size_t>(std::lower_bound(b, b + nb, a[ia1], cmp) - b);
      std::merge(a + ia0, a + ia1, b + ib0, b + ib1, dst + lo + ia0 + ib0, cmp);
    }
    std::swap(src, dst);
  }
  if (src != v->data()) std::copy(src, src + n, v->data());
}

}  // namespace common
}  // namespace lgap
