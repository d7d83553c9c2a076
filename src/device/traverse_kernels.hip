// Tree traversal score update (see traverse_kernels.h).
//
// One block stages kRows contiguous packed rows in LDS with coalesced dword loads, then each
// thread walks kRows / 256 rows through the LDS-resident nodes; the walks of a thread's rows
// are interleaved level by level so their LDS reads overlap. Leaf values live in LDS too.
#include "device/traverse_kernels.h"

#include <algorithm>
#include <cstdlib>

#include "device/hip_common.h"
#include "device/linear_kernels.h"
#include "lgap/pointwise.h"

namespace lgap {
namespace device {
namespace {

constexpr int kTThreads = 256;
constexpr int kTRowsPerThread = 2;
constexpr int kTRows = kTThreads * kTRowsPerThread;
constexpr int kTMaxDw = 16;  // wider rows read global memory directly

// Row-walk grid: LGAP_TRAVERSE_BLOCKS_PER_CU blocks per CU, grid-stride over the chunks (0: one
// chunk per block, the hardware overlapping one block's loads with another's walk)
int TraverseGrid(long long n, int num_cu) {
  const char* e = std::getenv("LGAP_TRAVERSE_BLOCKS_PER_CU");
  const int per = e != nullptr ? std::atoi(e) : 8;
  const long long chunks = (n + kTRows - 1) / kTRows;
  if (per <= 0) return static_cast<int>(std::max<long long>(1, std::min<long long>(chunks, 1 << 30)));
  return static_cast<int>(std::max<long long>(1, std::min<long long>(chunks, static_cast<long long>(num_cu) * per)));
}

template <int W>
__device__ __forceinline__ uint32_t GroupBin(const uint8_t* row, int g) {
  if (W == 0) return (row[g >> 1] >> ((g & 1) * 4)) & 0xFu;  // 4-bit rows
  return W == 1 ? row[g] : reinterpret_cast<const uint16_t*>(row)[g];
}

__device__ __forceinline__ bool CatLeft(const TCat& c, const uint32_t* bits, uint32_t gb) {
  const int local = static_cast<int>(gb) - c.offset;
  uint32_t b;
  if (local < 0 || local >= c.num_bin - 1) b = static_cast<uint32_t>(c.mfb);
  else b = static_cast<uint32_t>(local < c.mfb ? local : local + 1);
  const uint32_t w = b >> 5;
  return static_cast<int>(w) < c.nwords && ((bits[c.begin + w] >> (b & 31u)) & 1u);
}

// a linear leaf's value for row `row` (reference linear tree Predict: the leaf's constant output
// when any of the model's features is NaN)
__device__ __forceinline__ double LinearValue(const LinearLeaves& lin, int leaf, long long row, double leaf_out) {
  double v = lin.cnst[leaf];
  for (int q = lin.off[leaf]; q < lin.off[leaf + 1]; ++q) {
    const float x = lin.raw[row * lin.F + lin.feat[q]];
    if (__builtin_isnan(x)) return leaf_out;
    v += lin.coef[q] * static_cast<double>(x);
  }
  return v;
}

// the next iteration's pointwise gradients from the updated score (GRAD instantiation of
// k_traverse: the score update of the last tree deferred into the gradient pass)
struct GradEpilogue {
  PointwiseParams p;
  const float* label;
  const float* weight;  // nullptr: unweighted
  const float* aux;     // MAPE label weights, nullptr: none
  float2* gh;
};

template <int W, bool LIN, bool GRAD = false>
__global__ __launch_bounds__(kTThreads) void k_traverse(const uint32_t* __restrict__ rowbins, int stride_dw, int n,
                                                        const TNode* __restrict__ nodes, int num_nodes,
                                                        const TCat* __restrict__ cats, const uint32_t* __restrict__ cat_bits,
                                                        const double* __restrict__ leaf_value, int num_leaves,
                                                        double* __restrict__ score, LinearLeaves lin,
                                                        GradEpilogue ge = GradEpilogue{}) {
  extern __shared__ __align__(16) unsigned char lds[];
  TNode* s_nodes = reinterpret_cast<TNode*>(lds);
  double* s_leaf = reinterpret_cast<double*>(lds + ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)));
  // 16-byte aligned row staging (uint4 stores)
  uint32_t* s_rows = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(s_leaf) +
                                                 ((sizeof(double) * num_leaves + 15) & ~size_t(15)));
  const int t = threadIdx.x;
  for (int i = t; i < num_nodes * static_cast<int>(sizeof(TNode) / 4); i += kTThreads) {
    reinterpret_cast<uint32_t*>(s_nodes)[i] = reinterpret_cast<const uint32_t*>(nodes)[i];
  }
  for (int i = t; i < num_leaves; i += kTThreads) s_leaf[i] = leaf_value[i];
  const bool staged = stride_dw <= kTMaxDw;
  for (long long base = static_cast<long long>(blockIdx.x) * kTRows; base < n;
       base += static_cast<long long>(gridDim.x) * kTRows) {
    const int rows = static_cast<int>(min(static_cast<long long>(kTRows), n - base));
    // this chunk's scores (and, for the gradient epilogue, labels / weights), loaded before the
    // walk so their latency hides behind it
    double sc[kTRowsPerThread];
    float lb[kTRowsPerThread], wt[kTRowsPerThread], ax[kTRowsPerThread];
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      const int r = t + j * kTThreads;
      sc[j] = r < rows ? score[base + r] : 0.0;
      if (GRAD) {
        lb[j] = r < rows ? ge.label[base + r] : 0.f;
        wt[j] = r < rows && ge.weight ? ge.weight[base + r] : 1.f;
        ax[j] = r < rows && ge.aux ? ge.aux[base + r] : 0.f;
      }
    }
    if (staged) {
      __syncthreads();  // the previous chunk's walks are done (first pass: nodes / leaves in place)
      const uint32_t* src = rowbins + base * stride_dw;
      const int ndw = rows * stride_dw;
      // 16-byte loads where the chunk is 16-byte aligned (kTRows * stride_dw dwords per chunk:
      // always, for rows from a 16-byte aligned buffer), dword loads for the tail
      const int nq = (reinterpret_cast<uintptr_t>(src) & 15u) == 0 ? ndw >> 2 : 0;
      const uint4* src4 = reinterpret_cast<const uint4*>(src);
      uint4* dst4 = reinterpret_cast<uint4*>(s_rows);
      for (int k = t; k < nq; k += kTThreads) dst4[k] = src4[k];
      for (int k = 4 * nq + t; k < ndw; k += kTThreads) s_rows[k] = src[k];
      __syncthreads();
    } else if (base == static_cast<long long>(blockIdx.x) * kTRows) {
      __syncthreads();
    }
    const uint8_t* row[kTRowsPerThread];
    int node[kTRowsPerThread];
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      const int r = t + j * kTThreads;
      node[j] = r < rows ? 0 : ~0;
      row[j] = staged ? reinterpret_cast<const uint8_t*>(s_rows + static_cast<size_t>(r) * stride_dw)
                      : reinterpret_cast<const uint8_t*>(rowbins + static_cast<size_t>(base + r) * stride_dw);
    }
    bool live = true;
    while (live) {
      live = false;
#pragma unroll
      for (int j = 0; j < kTRowsPerThread; ++j) {
        if (node[j] < 0) continue;
        const TNode nd = s_nodes[node[j]];
        const uint32_t gb = GroupBin<W>(row[j], nd.group);
        bool left;
        if (nd.flags & kTCat) {
          left = CatLeft(cats[node[j]], cat_bits, gb);
        } else if (gb < nd.lo || gb > nd.hi) {
          left = (nd.flags & kTOutLeft) != 0;
        } else if (static_cast<int>(gb) == nd.gmiss) {
          left = (nd.flags & kTDefaultLeft) != 0;
        } else {
          left = gb <= nd.tg;
        }
        node[j] = left ? nd.left : nd.right;
        live |= node[j] >= 0;
      }
    }
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      const int r = t + j * kTThreads;
      if (r < rows) {
        const double lv = LIN ? LinearValue(lin, ~node[j], base + r, s_leaf[~node[j]]) : s_leaf[~node[j]];
        const double ns = sc[j] + lv;
        score[base + r] = ns;
        if (GRAD) {
          score_t g, h;
          PointwiseGradient(ge.p, ns, static_cast<double>(lb[j]), static_cast<double>(wt[j]), ge.weight != nullptr,
                            static_cast<double>(ax[j]), &g, &h);
          ge.gh[base + r] = make_float2(g, h);
        }
      }
    }
  }
}

// Wide rows of the TRAINING set: walk over the group-major copy (colbins[g * n + row]), so lanes
// at the same node read one contiguous run of a column instead of one cache line per row.
template <int W>
__global__ __launch_bounds__(kTThreads) void k_traverse_col(const uint8_t* __restrict__ colbins, int n,
                                                            const TNode* __restrict__ nodes, int num_nodes,
                                                            const TCat* __restrict__ cats, const uint32_t* __restrict__ cat_bits,
                                                            const double* __restrict__ leaf_value, int num_leaves,
                                                            double* __restrict__ score) {
  extern __shared__ __align__(16) unsigned char lds[];
  TNode* s_nodes = reinterpret_cast<TNode*>(lds);
  double* s_leaf = reinterpret_cast<double*>(lds + ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)));
  const int t = threadIdx.x;
  for (int i = t; i < num_nodes * static_cast<int>(sizeof(TNode) / 4); i += kTThreads) {
    reinterpret_cast<uint32_t*>(s_nodes)[i] = reinterpret_cast<const uint32_t*>(nodes)[i];
  }
  for (int i = t; i < num_leaves; i += kTThreads) s_leaf[i] = leaf_value[i];
  __syncthreads();
  for (long long base = static_cast<long long>(blockIdx.x) * kTRows; base < n;
       base += static_cast<long long>(gridDim.x) * kTRows) {
    long long row[kTRowsPerThread];
    int node[kTRowsPerThread];
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      row[j] = base + t + j * kTThreads;
      node[j] = row[j] < n ? 0 : ~0;
    }
    bool live = true;
    while (live) {
      live = false;
#pragma unroll
      for (int j = 0; j < kTRowsPerThread; ++j) {
        if (node[j] < 0) continue;
        const TNode nd = s_nodes[node[j]];
        const size_t o = static_cast<size_t>(nd.group) * n + row[j];
        const uint32_t gb = W == 1 ? colbins[o] : reinterpret_cast<const uint16_t*>(colbins)[o];
        bool left;
        if (nd.flags & kTCat) {
          left = CatLeft(cats[node[j]], cat_bits, gb);
        } else if (gb < nd.lo || gb > nd.hi) {
          left = (nd.flags & kTOutLeft) != 0;
        } else if (static_cast<int>(gb) == nd.gmiss) {
          left = (nd.flags & kTDefaultLeft) != 0;
        } else {
          left = gb <= nd.tg;
        }
        node[j] = left ? nd.left : nd.right;
        live |= node[j] >= 0;
      }
    }
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      if (row[j] < n) score[row[j]] += s_leaf[~node[j]];
    }
  }
}

__global__ __launch_bounds__(256) void k_pack_nibbles(const uint32_t* __restrict__ rowbins, int stride_dw, int n,
                                                      int groups, uint32_t* __restrict__ out, int stride4) {
  const long long total = static_cast<long long>(n) * stride4;
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<long long>(gridDim.x) * blockDim.x) {
    const long long row = i / stride4;
    const int d = static_cast<int>(i - row * stride4);
    const uint32_t* r = rowbins + row * stride_dw;
    uint32_t v = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int g = 8 * d + k;
      if (g < groups) v |= ((r[g >> 2] >> (8 * (g & 3))) & 0xFu) << (4 * k);
    }
    out[i] = v;
  }
}

}  // namespace

void LaunchPackNibbles(const uint32_t* rowbins, int stride_dw, int n, int groups, uint32_t* out, int stride4,
                       hipStream_t s) {
  if (n <= 0) return;
  const long long total = static_cast<long long>(n) * stride4;
  const int grid = static_cast<int>(std::max<long long>(1, std::min<long long>((total + 255) / 256, 8192)));
  k_pack_nibbles<<<grid, 256, 0, s>>>(rowbins, stride_dw, n, groups, out, stride4);
  HIP_CHECK(hipGetLastError());
}

void LaunchTraverseCols(const uint8_t* colbins, int width, int n, const TNode* nodes, int num_nodes, const TCat* cats,
                        const uint32_t* cat_bits, const double* leaf_value, int num_leaves, double* score, int num_cu,
                        hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)) + sizeof(double) * num_leaves;
  const int grid = std::max(1, std::min(DivUp(n, kTRows), num_cu * 8));
  if (width == 1) {
    k_traverse_col<1><<<grid, kTThreads, lds, s>>>(colbins, n, nodes, num_nodes, cats, cat_bits, leaf_value, num_leaves,
                                                  score);
  } else {
    k_traverse_col<2><<<grid, kTThreads, lds, s>>>(colbins, n, nodes, num_nodes, cats, cat_bits, leaf_value, num_leaves,
                                                  score);
  }
  HIP_CHECK(hipGetLastError());
}

void LaunchTraverse(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                    const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves, double* score,
                    int num_cu, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)) + ((sizeof(double) * num_leaves + 15) & ~size_t(15)) +
                     (stride_dw <= kTMaxDw ? sizeof(uint32_t) * kTRows * stride_dw : 0);
  const int grid = TraverseGrid(n, num_cu);
  LinearLeaves none{};
  if (width == 0) {
    k_traverse<0, false><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits, leaf_value,
                                                     num_leaves, score, none);
  } else if (width == 1) {
    k_traverse<1, false><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits, leaf_value,
                                                     num_leaves, score, none);
  } else {
    k_traverse<2, false><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits, leaf_value,
                                                     num_leaves, score, none);
  }
  HIP_CHECK(hipGetLastError());
}

void LaunchTraverseGrad(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                        const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves,
                        double* score, const PointwiseParams& p, const float* label, const float* weight,
                        const float* aux, float2* gh, int num_cu, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)) + ((sizeof(double) * num_leaves + 15) & ~size_t(15)) +
                     (stride_dw <= kTMaxDw ? sizeof(uint32_t) * kTRows * stride_dw : 0);
  const int grid = TraverseGrid(n, num_cu);
  LinearLeaves none{};
  GradEpilogue ge;
  ge.p = p;
  ge.label = label;
  ge.weight = weight;
  ge.aux = aux;
  ge.gh = gh;
  if (width == 0) {
    k_traverse<0, false, true><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits,
                                                           leaf_value, num_leaves, score, none, ge);
  } else if (width == 1) {
    k_traverse<1, false, true><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits,
                                                           leaf_value, num_leaves, score, none, ge);
  } else {
    k_traverse<2, false, true><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits,
                                                           leaf_value, num_leaves, score, none, ge);
  }
  HIP_CHECK(hipGetLastError());
}

void LaunchTraverseLinear(const uint32_t* rowbins, int stride_dw, int width, int n, const TNode* nodes, int num_nodes,
                          const TCat* cats, const uint32_t* cat_bits, const double* leaf_value, int num_leaves,
                          const LinearLeaves& lin, double* score, int num_cu, hipStream_t s) {
  if (n <= 0) return;
  const size_t lds = ((sizeof(TNode) * num_nodes + 15) & ~size_t(15)) + ((sizeof(double) * num_leaves + 15) & ~size_t(15)) +
                     (stride_dw <= kTMaxDw ? sizeof(uint32_t) * kTRows * stride_dw : 0);
  const int grid = std::max(1, std::min(DivUp(n, kTRows), num_cu * 8));
  if (width == 1) {
    k_traverse<1, true><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits, leaf_value,
                                                    num_leaves, score, lin);
  } else {
    k_traverse<2, true><<<grid, kTThreads, lds, s>>>(rowbins, stride_dw, n, nodes, num_nodes, cats, cat_bits, leaf_value,
                                                    num_leaves, score, lin);
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace device
}  // namespace lgap
