// Gradient / hessian kernels for the device-resident boosting loop.
//  * pointwise objectives: one thread per row, formulas shared with the host
//    objectives through lgap/pointwise.h (so both paths give the same numbers);
//  * multiclass softmax: one thread per row over the K class scores;
//  * multiclassova: one binary objective per class over one-hot labels;
//  * lambdarank (all 18 `lambdarank_target`s, position-biased scores for unbiased
//    LTR): one 256-thread workgroup per query (queries beyond kMaxDeviceQuery
//    documents in global scratch). The query's scores are bitonic-sorted in LDS (score desc, index
//    asc == std::stable_sort), the (i, j) pair space of the target is
//    flattened with an LDS prefix sum so every lane gets equal work, and the
//    per-document lambdas/hessians accumulate with LDS float atomics.
// Reference semantics: rank_objective.hpp:182-560 (targets, pair ranges,
// delta_pair, normalisation), multiclass_objective.hpp:120-150.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "device/grad_kernels.h"
#include "device/hip_common.h"
#include "lgap/pointwise_metric.h"
#include "lgap/rank_math.h"

namespace lgap {
namespace device {

namespace {

__global__ __launch_bounds__(256) void k_pointwise(PointwiseParams p, const double* __restrict__ score,
                                                   const float* __restrict__ label, const float* __restrict__ weight,
                                                   const float* __restrict__ aux, int n, float2* __restrict__ gh) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double w = weight ? static_cast<double>(weight[i]) : 1.0;
    const double ax = aux ? static_cast<double>(aux[i]) : 0.0;
    score_t g, h;
    PointwiseGradient(p, score[i], static_cast<double>(label[i]), w, weight != nullptr, ax, &g, &h);
    gh[i] = make_float2(g, h);
  }
}

// Two rows per thread with 16-byte score / gh and 8-byte label (weight, aux) accesses: the
// one-row kernel moved ~3.4 TB/s in 4- and 8-byte lane accesses (58 us at 10M rows).
__global__ __launch_bounds__(256) void k_pointwise2(PointwiseParams p, const double* __restrict__ score,
                                                    const float* __restrict__ label, const float* __restrict__ weight,
                                                    const float* __restrict__ aux, int n, float2* __restrict__ gh) {
  const int pairs = n >> 1;
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += stride) {
    const double2 sc = reinterpret_cast<const double2*>(score)[i];
    const float2 lb = reinterpret_cast<const float2*>(label)[i];
    const float2 w = weight ? reinterpret_cast<const float2*>(weight)[i] : make_float2(1.f, 1.f);
    const float2 ax = aux ? reinterpret_cast<const float2*>(aux)[i] : make_float2(0.f, 0.f);
    score_t g0, h0, g1, h1;
    PointwiseGradient(p, sc.x, static_cast<double>(lb.x), weight ? static_cast<double>(w.x) : 1.0, weight != nullptr,
                      aux ? static_cast<double>(ax.x) : 0.0, &g0, &h0);
    PointwiseGradient(p, sc.y, static_cast<double>(lb.y), weight ? static_cast<double>(w.y) : 1.0, weight != nullptr,
                      aux ? static_cast<double>(ax.y) : 0.0, &g1, &h1);
    reinterpret_cast<float4*>(gh)[i] = make_float4(g0, h0, g1, h1);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int i = n - 1;
    score_t g, h;
    PointwiseGradient(p, score[i], static_cast<double>(label[i]), weight ? static_cast<double>(weight[i]) : 1.0,
                      weight != nullptr, aux ? static_cast<double>(aux[i]) : 0.0, &g, &h);
    gh[i] = make_float2(g, h);
  }
}

__global__ __launch_bounds__(256) void k_softmax(int K, double factor, const double* __restrict__ score,
                                                 const float* __restrict__ label, const float* __restrict__ weight,
                                                 int n, float2* __restrict__ gh) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double mx = score[i];
    for (int k = 1; k < K; ++k) mx = fmax(mx, score[static_cast<size_t>(k) * n + i]);
    double den = 0.0;
    for (int k = 0; k < K; ++k) den += exp(score[static_cast<size_t>(k) * n + i] - mx);
    const int y = static_cast<int>(label[i]);
    const double w = weight ? static_cast<double>(weight[i]) : 1.0;
    for (int k = 0; k < K; ++k) {
      const double pk = exp(score[static_cast<size_t>(k) * n + i] - mx) / den;
      float g, h;
      if (weight) {
        g = static_cast<float>((y == k ? pk - 1.0f : pk) * w);
        h = static_cast<float>(factor * pk * (1.0f - pk) * w);
      } else {
        g = static_cast<float>(y == k ? pk - 1.0f : pk);
        h = static_cast<float>(factor * pk * (1.0f - pk));
      }
      gh[static_cast<size_t>(k) * n + i] = make_float2(g, h);
    }
  }
}

__global__ __launch_bounds__(256) void k_ova(int K, const PointwiseParams* __restrict__ params,
                                             const double* __restrict__ score, const float* __restrict__ label,
                                             const float* __restrict__ weight, int n, float2* __restrict__ gh) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int y = static_cast<int>(label[i]);
    const double w = weight ? static_cast<double>(weight[i]) : 1.0;
    for (int k = 0; k < K; ++k) {
      score_t g, h;
      PointwiseGradient(params[k], score[static_cast<size_t>(k) * n + i], y == k ? 1.0 : 0.0, w, weight != nullptr,
                        0.0, &g, &h);
      gh[static_cast<size_t>(k) * n + i] = make_float2(g, h);
    }
  }
}

__global__ void k_add_constant(double* score, int n, double v) {
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) score[i] += v;
}

constexpr int kRankThreads = 256;
constexpr int kNdcgMaxI = 32;  // NDCG register path: truncation levels up to this
constexpr int kRankLdsGains = 64;  // label gains staged in LDS

__device__ __forceinline__ bool RankBefore(double sa, int ia, double sb, int ib, int cnt) {
  const bool va = ia < cnt, vb = ib < cnt;
  if (va != vb) return va;
  if (sa != sb) return sa > sb;
  return ia < ib;
}


// Wave sums of 16 per-lane values at once (reduce-scatter butterfly: xor 32 / 16 / 8 / 4 halve
// the values each lane carries, xor 2 / 1 finish): returns the total of value index
// 8 b5 + 4 b4 + 2 b3 + b2 (lane bits), the same in the 4 lanes of a group.
__device__ __forceinline__ float WaveSum16(const float (&v)[16], int lane) {
  float a8[8], a4[4], a2[2];
  const bool h5 = lane & 32, h4 = lane & 16, h3 = lane & 8, h2 = lane & 4;
#pragma unroll
  for (int q = 0; q < 8; ++q) a8[q] = (h5 ? v[q + 8] : v[q]) + __shfl_xor(h5 ? v[q] : v[q + 8], 32, kWave);
#pragma unroll
  for (int q = 0; q < 4; ++q) a4[q] = (h4 ? a8[q + 4] : a8[q]) + __shfl_xor(h4 ? a8[q] : a8[q + 4], 16, kWave);
#pragma unroll
  for (int q = 0; q < 2; ++q) a2[q] = (h3 ? a4[q + 2] : a4[q]) + __shfl_xor(h3 ? a4[q] : a4[q + 2], 8, kWave);
  float a1 = (h2 ? a2[1] : a2[0]) + __shfl_xor(h2 ? a2[0] : a2[1], 4, kWave);
  a1 += __shfl_xor(a1, 2, kWave);
  a1 += __shfl_xor(a1, 1, kWave);
  return a1;
}

// The host objective's sigmoid table entry for a score difference (rank_objective.cpp
// BuildSigmoidTable / GetSigmoid): the same clamps and bin index in double, then the bin's
// value 1 / (1 + exp(s_bin * sigmoid)) evaluated in fp32 instead of read from the 8 MiB table
// (a dependent global load per pair).
// (bin_step / bin_base: the bin's sigmoid * score as step * idx + base, in fp32)
__device__ __forceinline__ float TableSigmoidF(const RankKernelArgs& a, double s, float bin_step, float bin_base) {
  int idx;
  if (s <= a.tmin) idx = 0;
  else if (s >= a.tmax) idx = a.table_size - 1;
  else idx = static_cast<int>((s - a.tmin) * a.tfactor);
  const float e = __expf(static_cast<float>(idx) * bin_step + bin_base);
  return __builtin_amdgcn_rcpf(1.0f + e);
}

struct LdsDiscount {
  const double* tab;
  __device__ double operator()(int r) const { return tab[r]; }
};

// Block bytes (LDS, or global scratch for a long query) for queries of up to `max_cnt`
// documents (P = pow2 >= max_cnt): scores, label gains, per-wave lambda / hessian sums,
// discounts, ranking, labels
inline size_t RankLdsBytes(int max_cnt) {
  int P = 1;
  while (P < max_cnt) P <<= 1;
  return static_cast<size_t>(P) * (2 * sizeof(double) + 2 * (kRankThreads / kWave) * sizeof(float) + sizeof(int) +
                                   sizeof(float)) +
         static_cast<size_t>(P + 1) * sizeof(double);
}

// kGlobal = false: one block per query, arrays in LDS sized by the dataset's largest query up
// to kMaxDeviceQuery (short queries then fit many blocks per CU); longer queries are skipped
// and handled by the kGlobal = true launch (one block per long query, the same arrays in its
// own slice of global scratch).
//
// Pairs: ONE WAVE per rank i (round robin over the waves), its lanes over the j range of
// TargetJRange. The pair math runs in fp32 (the score difference and the sigmoid bin index in
// fp64, as the host). Each wave accumulates into its OWN per-document lambda / hessian arrays
// (distinct lanes: distinct documents; the wave's ranks in program order), the rank-i side
// summed over the lanes first; the per-document totals add the four waves' arrays in wave
// order. Every sum runs in a fixed order: deterministic without atomics.
template <bool kGlobal, int TGT>
__global__ __launch_bounds__(kRankThreads) void k_lambdarank(RankKernelArgs a, int Pmax) {
  const int target = TGT >= 0 ? TGT : a.target;  // (TGT >= 0: the target's switch folded away)
  constexpr int kWaves = kRankThreads / kWave;
  extern __shared__ __align__(8) unsigned char s_dyn[];
  __shared__ double s_red[kWaves];
  __shared__ double s_lg[kRankLdsGains];   // label_gain (the first kRankLdsGains)
  __shared__ int s_pos2[kRankThreads / 2];  // rank sort: the second half's counts

  const int q = kGlobal ? a.large_q[blockIdx.x] : static_cast<int>(blockIdx.x);
  const int t = threadIdx.x;
  const int start = a.qb[q];
  const int cnt = a.qb[q + 1] - start;
  if (!kGlobal && cnt > kMaxDeviceQuery) return;
  float2* out = a.gh + start;
  if (cnt <= 1) {
    for (int i = t; i < cnt; i += blockDim.x) out[i] = make_float2(0.f, 0.f);
    return;
  }
  int P = 1;
  while (P < cnt) P <<= 1;
  const int Pa = kGlobal ? P : Pmax;  // array length
  unsigned char* base = kGlobal ? reinterpret_cast<unsigned char*>(a.large_scratch + a.large_off[blockIdx.x]) : s_dyn;
  double* s_score = reinterpret_cast<double*>(base);
  double* s_gain = s_score + Pa;                           // label_gain[label]
  float* s_acc = reinterpret_cast<float*>(s_gain + Pa);    // [wave][lambda | hessian][Pa], by rank
  double* s_disc = reinterpret_cast<double*>(s_acc + 2 * kWaves * Pa);  // 1 / log2(2 + r), r <= cnt
  int* s_idx = reinterpret_cast<int*>(s_disc + Pa + 1);
  float* s_lab = reinterpret_cast<float*>(s_idx + Pa);
  const bool full_sort = TargetNeedsFullSort(target) || target == kTgtPrecision;
  for (int i = t; i < P; i += blockDim.x) {
    if (i < cnt) {
      // unbiased LTR ranks by score + the position's learned bias (host: adj[j])
      s_score[i] = a.positions ? a.score[start + i] + a.pos_bias[a.positions[start + i]] : a.score[start + i];
      s_lab[i] = a.label[start + i];
#pragma unroll
      for (int w = 0; w < 2 * kWaves; ++w) s_acc[w * Pa + i] = 0.f;
    }
    s_idx[i] = i;
  }
  for (int r = t; r <= cnt; r += blockDim.x) s_disc[r] = a.disc[r];
  if (t < min(a.num_label_gain, kRankLdsGains)) s_lg[t] = a.label_gain[t];
  // (gains from the label once the LDS table is in: no dependent global load per document)
  auto gain_of = [&](float lb) {
    const int li = static_cast<int>(lb);
    return li < a.num_label_gain ? (li < kRankLdsGains ? s_lg[li] : a.label_gain[li]) : 0.0;
  };
  __syncthreads();
  // scores by original position; s_idx holds the ranking permutation (score desc, index asc:
  // RankBefore's keys are unique). Up to one document per thread: a rank sort (each thread counts
  // the documents before its own, one barrier); longer queries: the bitonic network.
  if (full_sort && cnt <= kRankThreads / 2) {
    // two threads per document, each counting the documents before it in one half
    const int d = t % (kRankThreads / 2), h = t / (kRankThreads / 2);
    const int half = (cnt + 1) >> 1, j0 = h * half, j1 = min(cnt, j0 + half);
    int pos = 0;
    if (d < cnt) {
      const double si = s_score[d];
      int j = j0;
      for (; j + 8 <= j1; j += 8) {
        double s8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) s8[u] = s_score[j + u];
        // (bitwise, not short-circuit: no branch per comparison)
#pragma unroll
        for (int u = 0; u < 8; ++u) pos += static_cast<int>((s8[u] > si) | ((s8[u] == si) & (j + u < d)));
      }
      for (; j < j1; ++j) {
        const double sj = s_score[j];
        pos += static_cast<int>((sj > si) | ((sj == si) & (j < d)));
      }
      if (h == 1) s_pos2[d] = pos;
    }
    __syncthreads();
    if (h == 0 && d < cnt) s_idx[pos + s_pos2[d]] = d;
    __syncthreads();
  } else if (full_sort && cnt <= kRankThreads) {
    int pos = 0;
    const double si = t < cnt ? s_score[t] : 0.0;
    if (t < cnt) {
      int j = 0;
      for (; j + 8 <= cnt; j += 8) {
        double s8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) s8[u] = s_score[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) pos += static_cast<int>((s8[u] > si) | ((s8[u] == si) & (j + u < t)));
      }
      for (; j < cnt; ++j) {
        const double sj = s_score[j];
        pos += static_cast<int>((sj > si) | ((sj == si) & (j < t)));
      }
    }
    __syncthreads();  // (every thread read the identity order's s_idx before it is overwritten)
    if (t < cnt) s_idx[pos] = t;
    __syncthreads();
  } else if (full_sort) {
    for (int k = 2; k <= P; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = t; i < P; i += blockDim.x) {
          const int l = i ^ j;
          if (l > i) {
            const int ai = s_idx[i], al = s_idx[l];
            const double sa = ai < cnt ? s_score[ai] : 0.0, sl = al < cnt ? s_score[al] : 0.0;
            const bool asc = (i & k) == 0;
            // asc segment: keep "before" order at i; desc segment: reversed
            const bool swap = asc ? RankBefore(sl, al, sa, ai, cnt) : RankBefore(sa, ai, sl, al, cnt);
            if (swap) {
              s_idx[i] = al;
              s_idx[l] = ai;
            }
          }
        }
        __syncthreads();
      }
    }
  }
  // best / worst scores
  double best, worst;
  if (TargetNeedsFullSort(target)) {
    best = s_score[s_idx[0]];
    int wi = cnt - 1;
    if (wi > 0 && s_score[s_idx[wi]] == kMinScore) wi -= 1;
    worst = s_score[s_idx[wi]];
  } else {
    double mx = -INFINITY, mn = INFINITY;
    for (int i = t; i < cnt; i += blockDim.x) {
      mx = fmax(mx, s_score[i]);
      mn = fmin(mn, s_score[i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      mx = fmax(mx, __shfl_xor(mx, o, kWave));
      mn = fmin(mn, __shfl_xor(mn, o, kWave));
    }
    if ((t & 63) == 0) s_red[t >> 6] = mx;
    __syncthreads();
    mx = s_red[0];
    for (int w = 1; w < kWaves; ++w) mx = fmax(mx, s_red[w]);
    __syncthreads();
    if ((t & 63) == 0) s_red[t >> 6] = mn;
    __syncthreads();
    mn = s_red[0];
    for (int w = 1; w < kWaves; ++w) mn = fmin(mn, s_red[w]);
    __syncthreads();
    best = mx;
    worst = mn;
  }
  // identity order for the order-free targets (the host iterates idx = 0..cnt-1); ranked
  // targets: scores / labels / gains permuted into rank order (s_idx: rank -> document)
  if (!full_sort) {
    for (int i = t; i < cnt; i += blockDim.x) s_idx[i] = i;
    __syncthreads();
  } else if (!kGlobal && cnt <= kRankThreads) {
    const int d = t < cnt ? s_idx[t] : 0;
    double sc = 0.0;
    float lb = 0.f;
    if (t < cnt) {
      sc = s_score[d];
      lb = s_lab[d];
    }
    __syncthreads();
    if (t < cnt) {
      s_score[t] = sc;
      s_lab[t] = lb;
      s_gain[t] = gain_of(lb);
    }
    __syncthreads();
  } else if (!kGlobal) {
    // (a long query in global scratch keeps document order and reads through s_idx)
    constexpr int kPer = kMaxDeviceQuery / kRankThreads;
    double sc[kPer], gn[kPer];
    float lb[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int r = u * kRankThreads + t;
      if (r < cnt) {
        const int d = s_idx[r];
        sc[u] = s_score[d];
        lb[u] = s_lab[d];
        gn[u] = gain_of(lb[u]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int r = u * kRankThreads + t;
      if (r < cnt) {
        s_score[r] = sc[u];
        s_gain[r] = gn[u];
        s_lab[r] = lb[u];
      }
    }
    __syncthreads();
  }
  if (kGlobal || !full_sort) {
    for (int i = t; i < cnt; i += blockDim.x) s_gain[i] = gain_of(s_lab[i]);
    __syncthreads();
  }
  // document of rank r in the score / label / gain arrays
  auto at = [&](int r) { return kGlobal && full_sort ? s_idx[r] : r; };
  const int i_end = TargetIEnd(target, cnt, a.k);
  const bool binary = TargetIsBinary(target);
  const bool norm = a.norm && best != worst;
  const double inv_dcg = a.inv_max_dcg ? a.inv_max_dcg[q] : 0.0;
  const double inv_bdcg = a.inv_max_bdcg ? a.inv_max_bdcg[q] : 0.0;
  const float sig = static_cast<float>(a.sigmoid), sig2 = sig * sig;
  const float bin_step = static_cast<float>(a.sigmoid / a.tfactor), bin_base = static_cast<float>(a.tmin * a.sigmoid);
  float sum_lambdas = 0.f;  // (this lane's pairs; the block total in fp64)
  const int lane = t & (kWave - 1), wave = t / kWave;
  float* w_lam = s_acc + 2 * wave * Pa;
  float* w_hes = w_lam + Pa;
  if (TGT == kTgtNdcg && !kGlobal && i_end <= kNdcgMaxI) {
    // NDCG, truncation <= 32: each lane keeps ONE rank j per 64-rank chunk (its score / label /
    // gain / discount in registers) and the wave's ranks i = wave + 4m as a register array, so
    // the pair loop touches no LDS: the j side sums in registers across the wave's ranks, the
    // i side in ilam[m] across the chunks (one wave sum per rank at the end)
    constexpr int kM = kNdcgMaxI / kWaves;
    float ilam[kM], ihes[kM];
#pragma unroll
    for (int m = 0; m < kM; ++m) ilam[m] = ihes[m] = 0.f;
    for (int c = 0; c < cnt; c += kWave) {
      const int j = c + lane;
      const bool inb = j < cnt;
      const double sdj = inb ? s_score[j] : kMinScore, gj = inb ? s_gain[j] : 0.0, dj = s_disc[inb ? j : 0];
      const float lj = inb ? s_lab[j] : 0.f;
      float jlam = 0.f, jhes = 0.f;
#pragma unroll
      for (int m = 0; m < kM; ++m) {
        const int i = wave + kWaves * m;
        if (i >= i_end) break;
        const double sdi = s_score[i], gi = s_gain[i], di = s_disc[i];
        const float li = s_lab[i];
        const bool live = j > i && sdj != kMinScore && sdi != kMinScore && li != lj;
        const bool i_high = li > lj;
        const double ds = i_high ? sdi - sdj : sdj - sdi;
        // (hg - lg) * |D(high rank) - D(low rank)| / maxDCG: the pair is symmetric in the ranks
        const double dp = (i_high ? gi - gj : gj - gi) * fabs(di - dj) * inv_dcg;
        float dpf = live ? static_cast<float>(dp) : 0.0f;
        if (norm) dpf *= __builtin_amdgcn_rcpf(0.01f + static_cast<float>(fabs(ds)));
        float pl = TableSigmoidF(a, live ? ds : 0.0, bin_step, bin_base);
        float ph = pl * (1.0f - pl);
        pl *= -sig * dpf;
        ph *= sig2 * dpf;
        ilam[m] += i_high ? pl : -pl;
        ihes[m] += ph;
        jlam += i_high ? -pl : pl;
        jhes += ph;
        sum_lambdas -= 2.0f * pl;
      }
      if (inb) {
        w_lam[j] = jlam;
        w_hes[j] = jhes;
      }
    }
    static_assert(kM == 8, "WaveSum16 reduces 8 ranks' lambda + hessian");
    float v16[16];
#pragma unroll
    for (int m = 0; m < kM; ++m) {
      v16[m] = ilam[m];
      v16[m + kM] = ihes[m];
    }
    const float tot = WaveSum16(v16, lane);
    const int vi = lane >> 2, m = vi & (kM - 1), i = wave + kWaves * m;
    if ((lane & 3) == 0 && i < i_end) (vi < kM ? w_lam : w_hes)[i] += tot;
  } else {
    for (int i = wave; i < i_end; i += kWaves) {
      int js, je;
      TargetJRange(target, i, cnt, a.k, &js, &je);
      const int di = at(i);
      const double sdi = s_score[di], gi = s_gain[di];
      const float li = s_lab[di];
      float li_lam = 0.f, li_hes = 0.f;
      if (sdi != kMinScore) {
        // branch-free body (a skipped pair's terms are masked to zero): nearly every wave has a
        // live pair, so the branches only cost
        for (int j = js + lane; j < je; j += kWave) {
          const int dj = at(j);
          const double sdj = s_score[dj];
          const float lj = s_lab[dj];
          const bool live = sdj != kMinScore && li != lj && !(binary && li > 0 && lj > 0);
          const bool i_high = li > lj;
          const int hr = i_high ? i : j, lr = i_high ? j : i;
          const float lh = i_high ? li : lj, ll = i_high ? lj : li;
          const double ds = i_high ? sdi - sdj : sdj - sdi;
          const double gj = s_gain[dj], hg = i_high ? gi : gj, lg = i_high ? gj : gi;
          const double dp = TargetDeltaPairD(target, i, j, hr, lr, hg, lg, lh, ll, inv_dcg, inv_bdcg, a.k, a.gap_weight,
                                             LdsDiscount{s_disc});
          float dpf = live ? static_cast<float>(dp) : 0.0f;
          if (norm) dpf *= __builtin_amdgcn_rcpf(0.01f + static_cast<float>(fabs(ds)));
          float pl = TableSigmoidF(a, live ? ds : 0.0, bin_step, bin_base);
          float ph = pl * (1.0f - pl);
          pl *= -sig * dpf;
          ph *= sig2 * dpf;
          // high doc: +pl, low doc: -pl (pl <= 0); both take ph
          li_lam += i_high ? pl : -pl;
          li_hes += ph;
          w_lam[j] += i_high ? -pl : pl;
          w_hes[j] += ph;
          sum_lambdas -= 2.0f * pl;
        }
      }
      li_lam = WaveSum(li_lam);
      li_hes = WaveSum(li_hes);
      if (lane == 0) {
        w_lam[i] += li_lam;
        w_hes[i] += li_hes;
      }
    }
  }
  const double wsum = WaveSum(static_cast<double>(sum_lambdas));
  if ((t & 63) == 0) s_red[t >> 6] = wsum;
  __syncthreads();
  double sl = 0.0;
  for (int w = 0; w < kWaves; ++w) sl += s_red[w];
  // (one lane evaluates the fp64 log2; the others read it)
  __shared__ double s_f;
  if (t == 0) s_f = a.norm && sl > 0 ? log2(1 + sl) / sl : 1.0;
  __syncthreads();
  const double f = s_f;
  for (int i = t; i < cnt; i += blockDim.x) {  // i: rank
    double lam = 0.0, hes = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      lam += s_acc[2 * w * Pa + i];
      hes += s_acc[(2 * w + 1) * Pa + i];
    }
    const int d = s_idx[i];
    float g = static_cast<float>(lam), h = static_cast<float>(hes);
    if (a.norm && sl > 0) {
      g = static_cast<float>(g * f);
      h = static_cast<float>(h * f);
    }
    if (a.weight) {
      const float w = a.weight[start + d];
      g = static_cast<float>(g * w);
      h = static_cast<float>(h * w);
    }
    out[d] = make_float2(g, h);
  }
}

int GridFor(int n) {
  int g = DivUp(n, 256);
  return g < 1 ? 1 : (g > 65536 ? 65536 : g);
}

// rank_xendcg (rank_objective.hpp:620-700; host twin RankXENDCG::OneQuery): one
// workgroup per query. The order-dependent parts (softmax max / denominator,
// the query's LCG draws, the three sums) run on lane 0 in document order so
// the lambdas match the host objective's sequential sums; the per-document
// terms run on all lanes from LDS. state[q] is the query's Random, advanced by
// cnt draws per call exactly like the host's rands_[q].
template <bool kGlobal>
__global__ __launch_bounds__(kRankThreads) void k_xendcg(XendcgArgs a) {
  __shared__ double l_rho[kGlobal ? 1 : kMaxDeviceQuery];
  __shared__ double l_p[kGlobal ? 1 : kMaxDeviceQuery];
  __shared__ float l_lam[kGlobal ? 1 : kMaxDeviceQuery];
  __shared__ double s_v[3];
  const int q = kGlobal ? a.large_q[blockIdx.x] : static_cast<int>(blockIdx.x);
  const int t = threadIdx.x;
  const int start = a.qb[q];
  const int cnt = a.qb[q + 1] - start;
  if (!kGlobal && cnt > kMaxDeviceQuery) return;  // the long-query launch handles it
  double* s_rho = l_rho;
  double* s_p = l_p;
  float* s_lam = l_lam;
  if (kGlobal) {
    s_rho = reinterpret_cast<double*>(a.large_scratch + a.large_off[blockIdx.x]);
    s_p = s_rho + cnt;
    s_lam = reinterpret_cast<float*>(s_p + cnt);
  }
  float2* out = a.gh + start;
  const double* score = a.score + start;
  const float* label = a.label + start;
  if (cnt <= 1) {  // the host returns before drawing
    for (int i = t; i < cnt; i += blockDim.x) out[i] = make_float2(0.f, 0.f);
    return;
  }
  if (t == 0) {
    double wmax = score[0];
    for (int i = 1; i < cnt; ++i) wmax = fmax(wmax, score[i]);
    s_v[0] = wmax;
  }
  __syncthreads();
  for (int i = t; i < cnt; i += blockDim.x) s_rho[i] = exp(score[i] - s_v[0]);
  __syncthreads();
  if (t == 0) {
    double den = 0.0;
    for (int i = 0; i < cnt; ++i) den += s_rho[i];
    unsigned x = a.state[q];
    double sp = 0.0;
    for (int i = 0; i < cnt; ++i) {
      x = 214013u * x + 2531011u;
      const float r = static_cast<float>(static_cast<int>((x >> 16) & 0x7FFF)) / 32768.0f;
      const double pi = pow(2.0, static_cast<int>(label[i])) - r;
      s_p[i] = pi;
      sp += pi;
    }
    a.state[q] = x;
    s_v[1] = den;
    s_v[2] = 1.0 / fmax(kEpsilon, sp);
  }
  __syncthreads();
  const double den = s_v[1], inv_den = s_v[2];
  for (int i = t; i < cnt; i += blockDim.x) {
    const double rho = s_rho[i] / den;
    s_rho[i] = rho;
    const double term = -s_p[i] * inv_den + rho;
    s_lam[i] = static_cast<float>(term);
    s_p[i] = term / (1. - rho);
  }
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {
    if (t == 0) {
      double sum = 0.0;
      for (int i = 0; i < cnt; ++i) sum += s_p[i];
      s_v[0] = sum;
    }
    __syncthreads();
    const double sum = s_v[0];
    for (int i = t; i < cnt; i += blockDim.x) {
      const double term = s_rho[i] * (sum - s_p[i]);
      s_lam[i] += static_cast<float>(term);
      if (pass == 0) s_p[i] = term / (1. - s_rho[i]);
    }
    __syncthreads();
  }
  for (int i = t; i < cnt; i += blockDim.x) {
    float g = s_lam[i];
    float h = static_cast<float>(s_rho[i] * (1.0 - s_rho[i]));
    if (a.weight) {
      g = static_cast<float>(g * a.weight[start + i]);
      h = static_cast<float>(h * a.weight[start + i]);
    }
    out[i] = make_float2(g, h);
  }
}

// Pointwise training metric from the device-resident score (reference CUDA
// EvalKernel, cuda_pointwise_metric.cu:20): per-block fp64 partial sums of
// PmRowTerm (the host metric's row term), then one wave folds the partials in
// a fixed order, so the value is run-to-run deterministic.
constexpr int kMetricThreads = 256;

__global__ __launch_bounds__(kMetricThreads) void k_metric_partial(PwMetricParams p, const double* __restrict__ score,
                                                                   const float* __restrict__ label,
                                                                   const float* __restrict__ weight, int n,
                                                                   double* __restrict__ partial) {
  __shared__ double s_w[kMetricThreads / kWave];
  double acc = 0.0;
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    acc += PmRowTerm(p, static_cast<double>(label[i]), score[i], weight != nullptr,
                     weight ? static_cast<double>(weight[i]) : 1.0);
  }
  acc = WaveSum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kMetricThreads / kWave; ++w) t += s_w[w];
    partial[blockIdx.x] = t;
  }
}

// multiclass metric rows (MultiRowLoss: the host MulticlassMetric's term), same partials / fold
__global__ __launch_bounds__(kMetricThreads) void k_multi_metric_partial(MultiMetricParams p, const double* __restrict__ score,
                                                                         const float* __restrict__ label,
                                                                         const float* __restrict__ weight, int n,
                                                                         double* __restrict__ partial) {
  __shared__ double s_w[kMetricThreads / kWave];
  double acc = 0.0;
  const int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double l = MultiRowLoss(p, score + i, static_cast<size_t>(n), static_cast<int>(label[i]));
    acc += weight != nullptr ? l * static_cast<double>(weight[i]) : l;
  }
  acc = WaveSum(acc);
  if ((threadIdx.x & (kWave - 1)) == 0) s_w[threadIdx.x / kWave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kMetricThreads / kWave; ++w) t += s_w[w];
    partial[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kWave) void k_metric_fold(const double* __restrict__ partial, int nb, double* out) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += kWave) acc += partial[i];
  acc = WaveSum(acc);
  if (threadIdx.x == 0) *out = acc;
}

// Position-bias statistics: per-position (-sum g, -sum h, count) as int64 fixed point
// (order independent), then one block applies the Newton step.
// 2^24: a position's |sum| up to ~5e11 stays inside int64 (at 2^32 unnormalised lambdas of a
// large dataset could approach the 2.1e9 limit)
constexpr double kPosScale = 16777216.0;
constexpr int kPosLds = 1024;

__global__ __launch_bounds__(256) void k_pos_accum(const float2* __restrict__ gh, const int* __restrict__ positions, int n,
                                                   int num_pos, long long* __restrict__ acc) {
  __shared__ unsigned long long s[3 * kPosLds];
  const bool lds = num_pos <= kPosLds;
  if (lds) {
    for (int i = threadIdx.x; i < 3 * num_pos; i += blockDim.x) s[i] = 0ull;
    __syncthreads();
  }
  unsigned long long* dst = lds ? s : reinterpret_cast<unsigned long long*>(acc);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int p = positions[i];
    const float2 v = gh[i];
    atomicAdd(&dst[3 * p], static_cast<unsigned long long>(__double2ll_rn(-static_cast<double>(v.x) * kPosScale)));
    atomicAdd(&dst[3 * p + 1], static_cast<unsigned long long>(__double2ll_rn(-static_cast<double>(v.y) * kPosScale)));
    atomicAdd(&dst[3 * p + 2], 1ull);
  }
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * num_pos; i += blockDim.x) {
      if (s[i]) atomicAdd(reinterpret_cast<unsigned long long*>(&acc[i]), s[i]);
    }
  }
}

__global__ __launch_bounds__(256) void k_pos_update(long long* __restrict__ acc, int num_pos, double lr, double reg,
                                                    double* __restrict__ bias) {
  for (int p = threadIdx.x; p < num_pos; p += blockDim.x) {
    const double d1 = static_cast<double>(acc[3 * p]) / kPosScale;
    const double d2 = static_cast<double>(acc[3 * p + 1]) / kPosScale;
    const double cnt = static_cast<double>(acc[3 * p + 2]);
    const double av = d1 - bias[p] * reg * cnt;
    const double bv = d2 - reg * cnt;
    bias[p] += lr * av / (fabs(bv) + 0.001);
    acc[3 * p] = acc[3 * p + 1] = acc[3 * p + 2] = 0;
  }
}

}  // namespace

size_t RankGlobalBytes(int cnt) {
  int P = 1;
  while (P < cnt) P <<= 1;
  return (RankLdsBytes(P) + 255) & ~static_cast<size_t>(255);
}

size_t XendcgGlobalBytes(int cnt) {
  return (static_cast<size_t>(cnt) * (2 * sizeof(double) + sizeof(float)) + 255) & ~static_cast<size_t>(255);
}

void LaunchOvaGrad(int num_class, const PointwiseParams* params_dev, const double* score, const float* label,
                   const float* weight, int n, float2* gh, hipStream_t s) {
  if (n <= 0) return;
  k_ova<<<GridFor(n), 256, 0, s>>>(num_class, params_dev, score, label, weight, n, gh);
  HIP_CHECK(hipGetLastError());
}

void LaunchPositionBiasUpdate(const float2* gh, const int* positions, int n, int num_pos, double lr, double reg,
                              long long* acc, double* bias, hipStream_t s) {
  if (n <= 0 || num_pos <= 0) return;
  k_pos_accum<<<std::min(GridFor(n), 1024), 256, 0, s>>>(gh, positions, n, num_pos, acc);
  HIP_CHECK(hipGetLastError());
  k_pos_update<<<1, 256, 0, s>>>(acc, num_pos, lr, reg, bias);
  HIP_CHECK(hipGetLastError());
}

void LaunchPointwiseGrad(const PointwiseParams& p, const double* score, const float* label, const float* weight,
                         const float* aux, int n, float2* gh, hipStream_t s) {
  if (n <= 0) return;
  auto al = [](const void* q, uintptr_t b) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & (b - 1)) == 0; };
  if (n >= 2 && al(score, 16) && al(gh, 16) && al(label, 8) && al(weight, 8) && al(aux, 8)) {
    k_pointwise2<<<GridFor((n + 1) / 2), 256, 0, s>>>(p, score, label, weight, aux, n, gh);
  } else {
    k_pointwise<<<GridFor(n), 256, 0, s>>>(p, score, label, weight, aux, n, gh);
  }
  HIP_CHECK(hipGetLastError());
}

void LaunchSoftmaxGrad(int num_class, double factor, const double* score, const float* label, const float* weight,
                       int n, float2* gh, hipStream_t s) {
  if (n <= 0) return;
  k_softmax<<<GridFor(n), 256, 0, s>>>(num_class, factor, score, label, weight, n, gh);
  HIP_CHECK(hipGetLastError());
}

void LaunchLambdarankGrad(const RankKernelArgs& a, hipStream_t s) {
  if (a.num_queries <= 0) return;
  int Pmax = 1;
  while (Pmax < std::max(2, std::min(a.max_query, kMaxDeviceQuery))) Pmax <<= 1;
  const size_t lds = RankLdsBytes(Pmax);
  if (lds > 64 * 1024) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_lambdarank<false, kTgtNdcg>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_lambdarank<false, -1>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  }
  // NDCG (the default target) gets its own instantiation: the per-pair target switch of the
  // generic one was most of the pair loop's branches
  if (a.target == kTgtNdcg) k_lambdarank<false, kTgtNdcg><<<a.num_queries, kRankThreads, lds, s>>>(a, Pmax);
  else k_lambdarank<false, -1><<<a.num_queries, kRankThreads, lds, s>>>(a, Pmax);
  HIP_CHECK(hipGetLastError());
  if (a.num_large > 0) {
    k_lambdarank<true, -1><<<a.num_large, kRankThreads, 0, s>>>(a, 0);
    HIP_CHECK(hipGetLastError());
  }
}

void LaunchXendcgGrad(const XendcgArgs& a, hipStream_t s) {
  if (a.num_queries <= 0) return;
  k_xendcg<false><<<a.num_queries, kRankThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
  if (a.num_large > 0) {
    k_xendcg<true><<<a.num_large, kRankThreads, 0, s>>>(a);
    HIP_CHECK(hipGetLastError());
  }
}

void LaunchPointwiseMetric(const PwMetricParams& p, const double* score, const float* label, const float* weight, int n,
                           double* partial, int max_blocks, double* out, hipStream_t s) {
  const int nb = std::max(1, std::min(max_blocks, (n + kMetricThreads - 1) / kMetricThreads));
  k_metric_partial<<<nb, kMetricThreads, 0, s>>>(p, score, label, weight, n, partial);
  HIP_CHECK(hipGetLastError());
  k_metric_fold<<<1, kWave, 0, s>>>(partial, nb, out);
  HIP_CHECK(hipGetLastError());
}

void LaunchMultiMetric(const MultiMetricParams& p, const double* score, const float* label, const float* weight, int n,
                       double* partial, int max_blocks, double* out, hipStream_t s) {
  const int nb = std::max(1, std::min(max_blocks, (n + kMetricThreads - 1) / kMetricThreads));
  k_multi_metric_partial<<<nb, kMetricThreads, 0, s>>>(p, score, label, weight, n, partial);
  HIP_CHECK(hipGetLastError());
  k_metric_fold<<<1, kWave, 0, s>>>(partial, nb, out);
  HIP_CHECK(hipGetLastError());
}

void LaunchAddConstant(double* score, int n, double v, hipStream_t s) {
  if (n <= 0) return;
  k_add_constant<<<GridFor(n), 256, 0, s>>>(score, n, v);
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
