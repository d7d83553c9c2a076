// Ranking / AUC metric kernels (see metric_kernels.h).
#include "device/metric_kernels.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>

#include "device/hip_common.h"
#include "lgap/rank_metric_spec.h"

namespace lgap {
namespace device {
namespace {

constexpr int kMThreads = 256;
constexpr int kMBlocks = 512;  // fixed partial-sum grid (run-to-run identical reductions)
constexpr int kMaxE = RankMetricSpec::kMaxEvalAt;

// (positive, negative) weight of a group of tied scores
struct PN {
  double p, n;
};
struct PNPlus {
  __host__ __device__ PN operator()(const PN& a, const PN& b) const { return PN{a.p + b.p, a.n + b.n}; }
};
struct ToPN {
  __host__ __device__ PN operator()(const float2& v) const { return PN{static_cast<double>(v.x), static_cast<double>(v.y)}; }
};

// -0.0 and +0.0 compare equal but are distinct radix keys: one canonical zero
__device__ __forceinline__ double CanonKey(double s) { return s == 0.0 ? 0.0 : s; }

// block sum over 4 waves in a fixed order (the same value in every thread)
__device__ __forceinline__ double BlockSum256(double v) {
  __shared__ double s_w[4];
  v = WaveSum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s_w[w] = v;
  __syncthreads();
  return ((s_w[0] + s_w[1]) + s_w[2]) + s_w[3];
}

// keys = score (canonical zero), values = (w if label > 0, w if label <= 0): the host's
// cur_pos += (y > 0) * w, cur_neg += (y <= 0) * w
__global__ __launch_bounds__(kMThreads) void k_auc_prep(const double* __restrict__ score, const float* __restrict__ label,
                                                        const float* __restrict__ weight, int n, double* __restrict__ keys,
                                                        float2* __restrict__ vals) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float y = label[i];
    const float w = weight != nullptr ? weight[i] : 1.f;
    keys[i] = CanonKey(score[i]);
    vals[i] = make_float2(y > 0.f ? w : 0.f, y <= 0.f ? w : 0.f);
  }
}

// one term per group g (groups in descending score order; pref = exclusive prefix):
//   AUC  neg_g * (pos before g + pos_g / 2)
//   AP   pos_g * (pos through g / rows through g)
template <bool AP>
__global__ __launch_bounds__(kMThreads) void k_auc_terms(const PN* __restrict__ agg, const PN* __restrict__ pref,
                                                         const int* __restrict__ count, double* __restrict__ partial) {
  const int U = *count;
  double acc = 0.0;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < U; g += gridDim.x * blockDim.x) {
    const PN a = agg[g], b = pref[g];
    if (AP) {
      const double sp = b.p + a.p, st = (b.p + b.n) + (a.p + a.n);
      acc += a.p * (sp / st);
    } else {
      acc += a.n * (a.p * 0.5 + b.p);
    }
  }
  const double s = BlockSum256(acc);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kMThreads) void k_auc_fold(const double* __restrict__ partial, int nb,
                                                        const PN* __restrict__ agg, const PN* __restrict__ pref,
                                                        const int* __restrict__ count, double* __restrict__ out) {
  double acc = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) acc += partial[b];
  const double s = BlockSum256(acc);
  if (threadIdx.x == 0) {
    const int U = *count;
    out[0] = s;
    out[1] = U > 0 ? pref[U - 1].p + agg[U - 1].p : 0.0;
  }
}

__global__ __launch_bounds__(kMThreads) void k_rank_keys(const double* __restrict__ score, int n, double* __restrict__ keys) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) keys[i] = CanonKey(score[i]);
}

// One wave per query (grid-stride by wave), labels sorted by score descending within each
// query; every wave adds its queries' terms into its own LDS row (lane 0, in query order),
// the block's four rows are added in a fixed order.
template <int KIND>
__global__ __launch_bounds__(kMThreads) void k_query_metric(QueryMetricArgs a, const float* __restrict__ lab,
                                                            double* __restrict__ partial) {
  __shared__ double s_acc[4][kMaxE];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, ne = a.ne;
  if (lane < ne) s_acc[w][lane] = 0.0;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const int nw = gridDim.x * 4;
  for (int q = blockIdx.x * 4 + w; q < a.nq; q += nw) {
    const int b = a.qb[q], n = a.qb[q + 1] - b;
    const double qw = a.qw != nullptr ? static_cast<double>(a.qw[q]) : 1.0;
    const float* L = lab + b;
    if (KIND == RankMetricSpec::kNDCG) {
      const double* im = a.inv_max + static_cast<size_t>(q) * ne;
      if (im[0] <= 0.0) {
        if (lane < ne) s_acc[w][lane] += qw;
        continue;
      }
      double cur = 0.0;
      int left = 0;
      for (int e = 0; e < ne; ++e) {
        const int k = min(a.ks[e], n);
        double part = 0.0;
        for (int j = left + lane; j < k; j += 64) {
          const int li = min(max(static_cast<int>(L[j]), 0), a.ngain - 1);
          part += a.gain[li] * a.disc[j];
        }
        cur += WaveSum(part);
        if (lane == 0) s_acc[w][e] += cur * im[e] * qw;
        left = k;
      }
    } else if (KIND == RankMetricSpec::kMAP) {
      int hit = 0, left = 0;
      double sum_ap = 0.0;
      const int np = a.npos[q];
      for (int e = 0; e < ne; ++e) {
        const int k = min(a.ks[e], n);
        for (int j0 = left; j0 < k; j0 += 64) {
          const int j = j0 + lane;
          const bool rel = j < k && L[j] > 0.5f;
          const unsigned long long m = __ballot(rel);
          const int before = __popcll(m & lt);
          const double term =
              rel ? static_cast<double>(hit + before + 1) / static_cast<double>(static_cast<float>(j) + 1.0f) : 0.0;
          sum_ap += WaveSum(term);
          hit += __popcll(m);
        }
        const double v = np > 0 ? sum_ap / static_cast<double>(min(np, k)) : 1.0;
        if (lane == 0) s_acc[w][e] += v * qw;
        left = k;
      }
    } else {  // precision@k: the reference's denominator min(k, n - prev_k), else min(k, n)
      int hit = 0, left = 0;
      for (int e = 0; e < ne; ++e) {
        const int k = a.ks[e];
        for (int j0 = left; j0 < k && j0 < n; j0 += 64) {
          const int j = j0 + lane;
          hit += __popcll(__ballot(j < k && j < n && L[j] > 0.5f));
        }
        int den = min(k, n - left);
        if (den <= 0) den = min(k, n);
        const double v = den > 0 ? static_cast<double>(hit) / den : 0.0;
        if (lane == 0) s_acc[w][e] += v * qw;
        left = k;
      }
    }
  }
  __syncthreads();
  if (t < ne) partial[static_cast<size_t>(blockIdx.x) * ne + t] = ((s_acc[0][t] + s_acc[1][t]) + s_acc[2][t]) + s_acc[3][t];
}

__global__ __launch_bounds__(kMThreads) void k_query_fold(const double* __restrict__ partial, int nb, int ne,
                                                          double* __restrict__ out) {
  const int e = blockIdx.x;
  double acc = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) acc += partial[static_cast<size_t>(b) * ne + e];
  const double s = BlockSum256(acc);
  if (threadIdx.x == 0) out[e] = s;
}

size_t Align256(size_t x) { return (x + 255) & ~size_t(255); }

int StreamGrid(int n) { return std::max(1, std::min(4096, DivUp(n, kMThreads))); }

// temp bytes of the rocPRIM calls of an AUC evaluation over n rows
size_t AucTempBytes(int n) {
  const size_t m = static_cast<size_t>(std::max(n, 1));
  size_t a = 0, b = 0, c = 0;
  HIP_CHECK(rocprim::radix_sort_pairs_desc(nullptr, a, static_cast<double*>(nullptr), static_cast<double*>(nullptr),
                                           static_cast<float2*>(nullptr), static_cast<float2*>(nullptr), m, 0, 64));
  auto vin = rocprim::make_transform_iterator(static_cast<const float2*>(nullptr), ToPN());
  HIP_CHECK(rocprim::deterministic_reduce_by_key(nullptr, b, static_cast<const double*>(nullptr), vin, m,
                                                 static_cast<double*>(nullptr), static_cast<PN*>(nullptr),
                                                 static_cast<int*>(nullptr), PNPlus(), rocprim::equal_to<double>()));
  HIP_CHECK(rocprim::deterministic_exclusive_scan(nullptr, c, static_cast<const PN*>(nullptr), static_cast<PN*>(nullptr),
                                                  PN{0.0, 0.0}, m, PNPlus()));
  return std::max(a, std::max(b, c));
}

}  // namespace

size_t AucScratchBytes(int n) {
  const size_t m = static_cast<size_t>(std::max(n, 1));
  return Align256(AucTempBytes(n)) + 2 * Align256(m * sizeof(double)) + 2 * Align256(m * sizeof(float2)) +
         2 * Align256(m * sizeof(PN)) + Align256(sizeof(int)) + Align256(kMBlocks * sizeof(double));
}

void LaunchAucMetric(bool average_precision, const double* score, const float* label, const float* weight, int n,
                     void* scratch, size_t scratch_bytes, double* out, hipStream_t s) {
  if (scratch_bytes < AucScratchBytes(n)) Log::Fatal("LaunchAucMetric: scratch too small");
  const size_t m = static_cast<size_t>(std::max(n, 1));
  size_t temp_bytes = AucTempBytes(n);
  char* p = static_cast<char*>(scratch);
  void* temp = p;
  p += Align256(temp_bytes);
  double* k0 = reinterpret_cast<double*>(p);
  p += Align256(m * sizeof(double));
  double* k1 = reinterpret_cast<double*>(p);
  p += Align256(m * sizeof(double));
  float2* v0 = reinterpret_cast<float2*>(p);
  p += Align256(m * sizeof(float2));
  float2* v1 = reinterpret_cast<float2*>(p);
  p += Align256(m * sizeof(float2));
  PN* agg = reinterpret_cast<PN*>(p);
  p += Align256(m * sizeof(PN));
  PN* pref = reinterpret_cast<PN*>(p);
  p += Align256(m * sizeof(PN));
  int* count = reinterpret_cast<int*>(p);
  p += Align256(sizeof(int));
  double* partial = reinterpret_cast<double*>(p);
  if (n <= 0) {
    HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(double), s));
    return;
  }
  k_auc_prep<<<StreamGrid(n), kMThreads, 0, s>>>(score, label, weight, n, k0, v0);
  HIP_CHECK(hipGetLastError());
  size_t tb = temp_bytes;
  HIP_CHECK(rocprim::radix_sort_pairs_desc(temp, tb, k0, k1, v0, v1, m, 0, 64, s));
  auto vin = rocprim::make_transform_iterator(static_cast<const float2*>(v1), ToPN());
  tb = temp_bytes;
  HIP_CHECK(rocprim::deterministic_reduce_by_key(temp, tb, static_cast<const double*>(k1), vin, m, k0, agg, count,
                                                 PNPlus(), rocprim::equal_to<double>(), s));
  // (groups past the unique count are scanned too and ignored: their prefix never reaches a
  // group below the count)
  tb = temp_bytes;
  HIP_CHECK(rocprim::deterministic_exclusive_scan(temp, tb, static_cast<const PN*>(agg), pref, PN{0.0, 0.0}, m,
                                                  PNPlus(), s));
  const int nb = std::min(kMBlocks, StreamGrid(n));
  if (average_precision) k_auc_terms<true><<<nb, kMThreads, 0, s>>>(agg, pref, count, partial);
  else k_auc_terms<false><<<nb, kMThreads, 0, s>>>(agg, pref, count, partial);
  HIP_CHECK(hipGetLastError());
  k_auc_fold<<<1, kMThreads, 0, s>>>(partial, nb, agg, pref, count, out);
  HIP_CHECK(hipGetLastError());
}

// auc_mu pair scores (t1 * v . score of each row of classes i and j), ranked by the AUC kernels
// above. Ties: the AUC kernels group EXACTLY equal scores (reduce-by-key on equal_to<double>);
// the host AucMu (metrics.cpp, reference multiclass_metric.hpp AucMuMetric) counts two pair
// scores closer than kEpsilon (1e-15) as a tie. Scores a few ulps apart are therefore half-ties
// on the host and ordered here: a documented divergence below 1e-15 of the score scale, pinned
// by tests only for exact ties (test_device_metrics.py).
__global__ __launch_bounds__(kMThreads) void k_aucmu_pair(AucMuPairArgs a) {
  const int m = a.ni + a.nj;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < m; q += gridDim.x * blockDim.x) {
    const int row = q < a.ni ? a.idx[a.istart + q] : a.idx[a.jstart + q - a.ni];
    double va = 0.0;
    for (int c = 0; c < a.K; ++c) va = __dadd_rn(va, __dmul_rn(a.v[c], a.score[static_cast<size_t>(c) * a.n + row]));
    a.out_score[q] = __dmul_rn(a.t1, va);
    a.out_label[q] = q < a.ni ? 1.f : 0.f;
    a.out_w[q] = a.weight != nullptr ? a.weight[row] : 1.f;
  }
}

void LaunchAucMuPair(const AucMuPairArgs& a, hipStream_t s) {
  const int m = a.ni + a.nj;
  if (m <= 0) return;
  k_aucmu_pair<<<StreamGrid(m), kMThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

size_t QueryMetricScratchBytes(int n, int nq, int ne) {
  const size_t m = static_cast<size_t>(std::max(n, 1));
  size_t tmp = 0;
  HIP_CHECK(rocprim::segmented_radix_sort_pairs_desc(
      nullptr, tmp, static_cast<double*>(nullptr), static_cast<double*>(nullptr), static_cast<const float*>(nullptr),
      static_cast<float*>(nullptr), m, std::max(nq, 1), static_cast<const int*>(nullptr),
      static_cast<const int*>(nullptr), 0, 64));
  return Align256(tmp) + 2 * Align256(m * sizeof(double)) + Align256(m * sizeof(float)) +
         Align256(static_cast<size_t>(kMBlocks) * std::max(ne, 1) * sizeof(double));
}

void LaunchQueryMetric(const QueryMetricArgs& a, const double* score, const float* label, int n, void* scratch,
                       size_t scratch_bytes, double* out, hipStream_t s) {
  if (a.ne <= 0 || a.ne > kMaxE) Log::Fatal("LaunchQueryMetric: %d eval_at positions (1..%d)", a.ne, kMaxE);
  if (scratch_bytes < QueryMetricScratchBytes(n, a.nq, a.ne)) Log::Fatal("LaunchQueryMetric: scratch too small");
  const size_t m = static_cast<size_t>(std::max(n, 1));
  size_t tmp = 0;
  HIP_CHECK(rocprim::segmented_radix_sort_pairs_desc(
      nullptr, tmp, static_cast<double*>(nullptr), static_cast<double*>(nullptr), static_cast<const float*>(nullptr),
      static_cast<float*>(nullptr), m, std::max(a.nq, 1), static_cast<const int*>(nullptr),
      static_cast<const int*>(nullptr), 0, 64));
  char* p = static_cast<char*>(scratch);
  void* temp = p;
  p += Align256(tmp);
  double* k0 = reinterpret_cast<double*>(p);
  p += Align256(m * sizeof(double));
  double* k1 = reinterpret_cast<double*>(p);
  p += Align256(m * sizeof(double));
  float* lab = reinterpret_cast<float*>(p);
  p += Align256(m * sizeof(float));
  double* partial = reinterpret_cast<double*>(p);
  if (n > 0 && a.nq > 0) {
    k_rank_keys<<<StreamGrid(n), kMThreads, 0, s>>>(score, n, k0);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(rocprim::segmented_radix_sort_pairs_desc(temp, tmp, k0, k1, label, lab, m, a.nq, a.qb, a.qb + 1, 0, 64, s));
  }
  const int nb = std::max(1, std::min(kMBlocks, DivUp(std::max(a.nq, 1), 4)));
  if (a.kind == RankMetricSpec::kNDCG) k_query_metric<RankMetricSpec::kNDCG><<<nb, kMThreads, 0, s>>>(a, lab, partial);
  else if (a.kind == RankMetricSpec::kMAP) k_query_metric<RankMetricSpec::kMAP><<<nb, kMThreads, 0, s>>>(a, lab, partial);
  else k_query_metric<RankMetricSpec::kPrecision><<<nb, kMThreads, 0, s>>>(a, lab, partial);
  HIP_CHECK(hipGetLastError());
  k_query_fold<<<a.ne, kMThreads, 0, s>>>(partial, nb, a.ne, out);
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
