// Linear-leaf Gram systems with fp64 MFMA (see linear_kernels.h).
#include "device/linear_kernels.h"

#include <algorithm>

#include "device/hip_common.h"

namespace lgap {
namespace device {
namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kLinThreads = 256;
constexpr int kLinSlot = kLinDim * kLinDim + 1;  // [A | c] and the usable count

// Block (chunk, leaf): each wave takes groups of four rows of the chunk; lane l holds row
// l >> 4 of the group and column l & 15 of a 16-wide tile, which is both its A element
// (A[i = column][k = row], i.e. X^T) and its B element (B[k = row][j = column], i.e. [HX | g]),
// so v_mfma_f64_16x16x4f64 adds the four rows' outer products to the accumulator tile
// (C/D on gfx950 f64: col = l & 15, row = (l >> 4) + 4 reg).
template <int T>
__global__ __launch_bounds__(kLinThreads) void k_linear_gram(LinearGramArgs a, double* __restrict__ partial) {
  constexpr int D = 16 * T;  // the tiles' dimension
  __shared__ double s_g[D * D];
  __shared__ long long s_use[4];
  const int leaf = blockIdx.y, chunk = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, rr = lane >> 4, cc = lane & 15;
  const LeafSeg seg = a.segs[leaf];
  const int f0 = a.feat_off[leaf], k = a.feat_off[leaf + 1] - f0, m = k + 1;
  const int rb = static_cast<int>(static_cast<long long>(seg.count) * chunk / gridDim.x);
  const int re = static_cast<int>(static_cast<long long>(seg.count) * (chunk + 1) / gridDim.x);
  const int* idx = seg.buf < 0 ? nullptr : a.idx[seg.buf] + seg.start;
  // this lane's feature columns (one per tile), fixed for the leaf
  int col_feat[T];
#pragma unroll
  for (int ti = 0; ti < T; ++ti) {
    const int j = 16 * ti + cc;
    col_feat[ti] = j < k ? a.feats[f0 + j] : (j == k ? -1 : -2);  // -1: the constant, -2: padding
  }
  d4 acc[T][T];
#pragma unroll
  for (int ti = 0; ti < T; ++ti) {
#pragma unroll
    for (int tj = 0; tj < T; ++tj) acc[ti][tj] = d4{0.0, 0.0, 0.0, 0.0};
  }
  long long usable = 0;
  for (int p0 = rb + 4 * w; p0 < re; p0 += 16) {
    const int p = p0 + rr;
    const bool valid = p < re;
    const int row = valid ? (idx ? idx[p] : seg.start + p) : 0;
    const float2 v = valid ? a.gh[row] : make_float2(0.f, 0.f);
    double x[T];
    int first_nan = k;  // (lowest NaN column of the row over its 16 lanes)
#pragma unroll
    for (int ti = 0; ti < T; ++ti) {
      const int cf = col_feat[ti];
      const float rv = (valid && cf >= 0) ? a.raw[static_cast<size_t>(row) * a.F + cf] : 0.f;
      const bool nan = valid && cf >= 0 && __builtin_isnan(rv);
      x[ti] = cf == -1 ? 1.0 : static_cast<double>(rv);
      const unsigned long long nm = __ballot(nan);
      const unsigned rowbits = static_cast<unsigned>(nm >> (16 * rr)) & 0xFFFFu;
      if (rowbits != 0u) first_nan = min(first_nan, 16 * ti + __ffs(rowbits) - 1);
    }
    const bool drop = !valid || first_nan < k;
    if (valid && cc == 0) usable += first_nan;
#pragma unroll
    for (int ti = 0; ti < T; ++ti) {
      const double av = drop ? 0.0 : x[ti];
#pragma unroll
      for (int tj = 0; tj < T; ++tj) {
        const int j = 16 * tj + cc;
        const double bv = drop ? 0.0 : (j < m ? static_cast<double>(v.y) * x[tj] : (j == m ? static_cast<double>(v.x) : 0.0));
        acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[ti][tj], 0, 0, 0);
      }
    }
  }
  // the block's four waves summed into one LDS image in a fixed order (wave 0 stores, waves 1-3
  // add in turn): ((w0 + w1) + w2) + w3 for every element, one wave's image of LDS (32 KB at T = 4)
  usable = static_cast<long long>(WaveSum(static_cast<double>(usable)));
  if (lane == 0) s_use[w] = usable;
  for (int ws = 0; ws < 4; ++ws) {
    if (w == ws) {
#pragma unroll
      for (int ti = 0; ti < T; ++ti) {
#pragma unroll
        for (int tj = 0; tj < T; ++tj) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double& g = s_g[(16 * ti + rr + 4 * r) * D + 16 * tj + cc];
            g = ws == 0 ? acc[ti][tj][r] : g + acc[ti][tj][r];
          }
        }
      }
    }
    __syncthreads();
  }
  double* out = partial + (static_cast<size_t>(chunk) * a.num_leaves + leaf) * kLinSlot;
  for (int i = t; i < kLinDim * kLinDim; i += kLinThreads) {
    const int row = i / kLinDim, col = i - row * kLinDim;
    out[i] = row < D && col < D ? s_g[row * D + col] : 0.0;
  }
  if (t == 0) out[kLinDim * kLinDim] = static_cast<double>(((s_use[0] + s_use[1]) + s_use[2]) + s_use[3]);
}

__global__ __launch_bounds__(kLinThreads) void k_linear_fold(const double* __restrict__ partial, int chunks,
                                                             int num_leaves, double* __restrict__ out,
                                                             long long* __restrict__ usable) {
  const int leaf = blockIdx.x;
  for (int i = threadIdx.x; i < kLinSlot; i += blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < chunks; ++c) s += partial[(static_cast<size_t>(c) * num_leaves + leaf) * kLinSlot + i];
    if (i < kLinDim * kLinDim) out[static_cast<size_t>(leaf) * kLinDim * kLinDim + i] = s;
    else usable[leaf] = static_cast<long long>(s + 0.5);
  }
}

}  // namespace

size_t LinearGramPartialDoubles(int num_leaves, int chunks) {
  return static_cast<size_t>(std::max(1, num_leaves)) * std::max(1, chunks) * kLinSlot;
}

void LaunchLinearGram(const LinearGramArgs& a, int max_m, double* partial, double* out, long long* usable,
                      hipStream_t s) {
  if (a.num_leaves <= 0) return;
  if (max_m > kLinMaxM) Log::Fatal("LaunchLinearGram: %d unknowns per leaf (at most %d)", max_m, kLinMaxM);
  const dim3 grid(std::max(1, a.chunks), a.num_leaves);
  // one 16x16 tile per dimension while [A | c] fits it (m + 1 <= 16), two up to 32, four beyond
  if (max_m + 1 <= 16) k_linear_gram<1><<<grid, kLinThreads, 0, s>>>(a, partial);
  else if (max_m + 1 <= 32) k_linear_gram<2><<<grid, kLinThreads, 0, s>>>(a, partial);
  else k_linear_gram<4><<<grid, kLinThreads, 0, s>>>(a, partial);
  HIP_CHECK(hipGetLastError());
  k_linear_fold<<<a.num_leaves, kLinThreads, 0, s>>>(partial, std::max(1, a.chunks), a.num_leaves, out, usable);
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
