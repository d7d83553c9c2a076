// Device gradient kernels. Gradients live interleaved as float2 (g, h),
// class-major: gh[k * num_data + i].
#pragma once

#include <hip/hip_runtime.h>

#include "lgap/pointwise.h"
#include "lgap/pointwise_metric.h"

namespace lgap {
namespace device {

void LaunchPointwiseGrad(const PointwiseParams& p, const double* score, const float* label, const float* weight,
                         const float* aux, int n, float2* gh, hipStream_t s);

void LaunchSoftmaxGrad(int num_class, double factor, const double* score, const float* label, const float* weight,
                       int n, float2* gh, hipStream_t s);

// multiclassova: one binary objective per class over the one-hot labels (label == k);
// params[k] carries class k's label weights (is_unbalance / scale_pos_weight)
void LaunchOvaGrad(int num_class, const PointwiseParams* params_dev, const double* score, const float* label,
                   const float* weight, int n, float2* gh, hipStream_t s);

constexpr int kMaxDeviceQueryDecl = 2048;
struct RankKernelArgs {
  int target = 0;
  int k = 30;
  int norm = 1;
  double sigmoid = 1.0;
  double gap_weight = 1.0;
  double tmin = -50.0, tmax = 50.0, tfactor = 1.0;
  int table_size = 0;  // bins of the host sigmoid table (tmin / tmax / tfactor: its range)
  const double* label_gain = nullptr;
  const double* disc = nullptr;        // 1 / log2(2 + r), r <= max_query
  int num_label_gain = 0;
  const double* inv_max_dcg = nullptr;  // per query
  const double* inv_max_bdcg = nullptr;
  const int* qb = nullptr;              // query boundaries (num_queries + 1)
  int num_queries = 0;
  int max_query = kMaxDeviceQueryDecl;  // largest query (documents): sizes the LDS
  const float* label = nullptr;
  const float* weight = nullptr;
  const double* score = nullptr;
  float2* gh = nullptr;
  // unbiased LambdaRank (rank_objective.hpp:554-591): score + bias[position] ranks the documents
  const int* positions = nullptr;  // per row, nullptr: no position bias
  const double* pos_bias = nullptr;  // learned position biases (fp64, as the reference's pos_biases_)
  // queries longer than kMaxDeviceQuery: their block works in global scratch
  int num_large = 0;
  const int* large_q = nullptr;          // the long queries
  const long long* large_off = nullptr;  // byte offset of each one's scratch
  char* large_scratch = nullptr;
};
// Largest query whose sort / accumulators live in LDS (longer ones use global scratch).
constexpr int kMaxDeviceQuery = 2048;
// global scratch bytes of one long query of `cnt` documents (lambdarank / xendcg)
size_t RankGlobalBytes(int cnt);
size_t XendcgGlobalBytes(int cnt);
void LaunchLambdarankGrad(const RankKernelArgs& a, hipStream_t s);

// Position-bias Newton step after the lambdas (rank_objective.hpp UpdatePositionBias):
// per position d1 -= g, d2 -= h, cnt += 1, then bias += lr * (d1 - bias * reg * cnt) /
// (|d2 - reg * cnt| + 0.001). `acc` holds 3 * num_pos int64 fixed-point sums.
void LaunchPositionBiasUpdate(const float2* gh, const int* positions, int n, int num_pos, double lr, double reg,
                              long long* acc, double* bias, hipStream_t s);

struct XendcgArgs {
  const int* qb = nullptr;  // query boundaries (num_queries + 1)
  int num_queries = 0;
  const float* label = nullptr;
  const float* weight = nullptr;
  const double* score = nullptr;
  unsigned* state = nullptr;  // per-query LCG state (Random(objective_seed + q))
  float2* gh = nullptr;
  int num_large = 0;  // queries longer than kMaxDeviceQuery (global scratch, as RankKernelArgs)
  const int* large_q = nullptr;
  const long long* large_off = nullptr;
  char* large_scratch = nullptr;
};
void LaunchXendcgGrad(const XendcgArgs& a, hipStream_t s);

void LaunchAddConstant(double* score, int n, double v, hipStream_t s);

// sum over rows of the pointwise metric's weighted row loss (PmRowTerm) -> *out (device);
// `partial` holds max_blocks doubles
void LaunchPointwiseMetric(const PwMetricParams& p, const double* score, const float* label, const float* weight, int n,
                           double* partial, int max_blocks, double* out, hipStream_t s);
// sum over rows of the multiclass metric's weighted row loss (MultiRowLoss) over a class-major
// score [num_class][n] -> *out (device)
void LaunchMultiMetric(const MultiMetricParams& p, const double* score, const float* label, const float* weight, int n,
                       double* partial, int max_blocks, double* out, hipStream_t s);

}  // namespace device
}  // namespace lgap
