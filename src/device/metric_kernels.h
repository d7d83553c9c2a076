// Ranking / AUC metrics on the device-resident score (no N-double download per evaluation):
//  * AUC / average precision (reference binary_metric.hpp:159-268): rows sorted by score
//    descending (rocPRIM radix sort, 64-bit keys), tied scores reduced into groups of
//    (positive, negative) weight (deterministic reduce-by-key), an exclusive scan over the
//    groups, and one term per group -- the host's tie-aware loop, group for group;
//  * NDCG@k / MAP@k / precision@k (rank_metric.hpp:86-165, map_metric.hpp:107-160, the fork's
//    precision_metric.hpp:16-141): each query's rows sorted by score descending (rocPRIM
//    segmented radix sort, stable like the host's std::stable_sort), one wave per query walks
//    the eval_at cut-offs with the host's cursor semantics.
// Every reduction runs over a fixed grid in a fixed order: results are run-to-run identical.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace lgap {
namespace device {

// Scratch of an AUC / average-precision evaluation over n rows.
size_t AucScratchBytes(int n);
// out (device, 2 doubles) = {accumulator, positive weight}; the host finishes the value.
void LaunchAucMetric(bool average_precision, const double* score, const float* label, const float* weight, int n,
                     void* scratch, size_t scratch_bytes, double* out, hipStream_t s);

// auc_mu: one class pair's rows (classes i and j, from the class-ordered row index) scored by
// t1 * sum_m v_m score[m][row] in the host's order and without contraction; labels 1 for class
// i rows (the AUC's positives), 0 for class j rows.
constexpr int kAucMuMaxClass = 64;
struct AucMuPairArgs {
  const double* score;  // [K][n] class-major
  int n, K;
  const int* idx;       // rows ordered by class
  int istart, ni, jstart, nj;
  double t1;
  double v[kAucMuMaxClass];
  const float* weight;  // nullptr: 1
  double* out_score;
  float* out_label;
  float* out_w;
};
void LaunchAucMuPair(const AucMuPairArgs& a, hipStream_t s);

struct QueryMetricArgs {
  int kind;               // RankMetricSpec::Kind (kNDCG, kMAP, kPrecision)
  const int* qb;          // [nq + 1] query boundaries
  int nq;
  const float* qw;        // [nq] query weights, nullptr: 1
  const double* inv_max;  // NDCG [nq][ne]
  const int* npos;        // MAP [nq]
  const int* ks;          // [ne] eval_at
  int ne;
  const double* gain;     // NDCG label gains [ngain]
  int ngain;
  const double* disc;     // [max query rows] 1 / log2(2 + position)
};

size_t QueryMetricScratchBytes(int n, int nq, int ne);
// out (device, ne doubles) = query-weighted sums of the metric at each eval_at position
void LaunchQueryMetric(const QueryMetricArgs& a, const double* score, const float* label, int n, void* scratch,
                       size_t scratch_bytes, double* out, hipStream_t s);

}  // namespace device
}  // namespace lgap
