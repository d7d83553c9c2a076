// The per-leaf ridge-regularised Newton step of linear trees (reference linear_tree_learner.cpp
// CalculateLinear :191-356; Eq. 3 of arXiv:1802.05640), shared by the host linear learner and
// the device learner (whose Gram systems come from the fp64 MFMA kernel, linear_kernels.hip).
#pragma once

#include <cmath>
#include <cstdint>
#include <vector>

namespace lgap {

// A: m x m (row-major, lower triangle read) = sum h x x^T over the usable rows; b: m = -sum g x.
// Adds lambda to the first k = m - 1 diagonal entries (not the constant's), then solves by
// Cholesky. False when fewer usable values than unknowns or A is not positive definite.
inline bool SolveLinearLeaf(std::vector<double> A, const std::vector<double>& b, int64_t usable, int m, double lambda,
                            std::vector<double>* out) {
  if (usable < m) return false;
  for (int j = 0; j + 1 < m; ++j) A[static_cast<size_t>(j) * m + j] += lambda;
  std::vector<double> L(A.size(), 0.0);
  for (int i = 0; i < m; ++i) {
    for (int j = 0; j <= i; ++j) {
      double s = A[static_cast<size_t>(i) * m + j];
      for (int t = 0; t < j; ++t) s -= L[static_cast<size_t>(i) * m + t] * L[static_cast<size_t>(j) * m + t];
      if (i == j) {
        if (!(s > 1e-12)) return false;
        L[static_cast<size_t>(i) * m + i] = std::sqrt(s);
      } else {
        L[static_cast<size_t>(i) * m + j] = s / L[static_cast<size_t>(j) * m + j];
      }
    }
  }
  std::vector<double> y(m);
  out->assign(m, 0.0);
  for (int i = 0; i < m; ++i) {
    double s = b[i];
    for (int t = 0; t < i; ++t) s -= L[static_cast<size_t>(i) * m + t] * y[t];
    y[i] = s / L[static_cast<size_t>(i) * m + i];
  }
  for (int i = m - 1; i >= 0; --i) {
    double s = y[i];
    for (int t = i + 1; t < m; ++t) s -= L[static_cast<size_t>(t) * m + i] * (*out)[t];
    (*out)[i] = s / L[static_cast<size_t>(i) * m + i];
  }
  return true;
}

}  // namespace lgap
