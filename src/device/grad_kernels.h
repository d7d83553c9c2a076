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

constexpr int kMaxDeviceQueryDecl = 2048;
struct RankKernelArgs {
  int target = 0;
  int k = 30;
  int norm = 1;
  double sigmoid = 1.0;
  double gap_weight = 1.0;
  double tmin = -50.0, tmax = 50.0, tfactor = 1.0;
  int table_size = 0;
  const double* table = nullptr;        // sigmoid lookup table
  const double* label_gain = nullptr;
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
};
// Largest query the block-per-query kernel handles (LDS-resident sort).
constexpr int kMaxDeviceQuery = 2048;
void LaunchLambdarankGrad(const RankKernelArgs& a, hipStream_t s);

struct XendcgArgs {
  const int* qb = nullptr;  // query boundaries (num_queries + 1)
  int num_queries = 0;
  const float* label = nullptr;
  const float* weight = nullptr;
  const double* score = nullptr;
  unsigned* state = nullptr;  // per-query LCG state (Random(objective_seed + q))
  float2* gh = nullptr;
};
void LaunchXendcgGrad(const XendcgArgs& a, hipStream_t s);

void LaunchAddConstant(double* score, int n, double v, hipStream_t s);

// sum over rows of the pointwise metric's weighted row loss (PmRowTerm) -> *out (device);
// `partial` holds max_blocks doubles
void LaunchPointwiseMetric(const PwMetricParams& p, const double* score, const float* label, const float* weight, int n,
                           double* partial, int max_blocks, double* out, hipStream_t s);

}  // namespace device
}  // namespace lgap
