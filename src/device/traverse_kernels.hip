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
#include "lgap/log.h"
#include "lgap/pointwise.h"

namespace lgap {
namespace device {
namespace {

constexpr int kTThreads = 256;
constexpr int kTRowsPerThread = 2;
constexpr int kTRows = kTThreads * kTRowsPerThread;
constexpr int kTMaxDw = 16;  // wider rows read global memory directly

// Row-walk grid: 8 blocks per CU, grid-stride over the chunks
int TraverseGrid(long long n, int num_cu) {
  const long long chunks = (n + kTRows - 1) / kTRows;
  return static_cast<int>(std::max<long long>(1, std::min<long long>(chunks, static_cast<long long>(num_cu) * 8)));
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

template <int W, bool LIN>
__global__ __launch_bounds__(kTThreads) void k_traverse(const uint32_t* __restrict__ rowbins, int stride_dw, int n,
                                                        const TNode* __restrict__ nodes, int num_nodes,
                                                        const TCat* __restrict__ cats, const uint32_t* __restrict__ cat_bits,
                                                        const double* __restrict__ leaf_value, int num_leaves,
                                                        double* __restrict__ score, LinearLeaves lin) {
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
    // this chunk's scores, loaded before the walk so their latency hides behind it
    double sc[kTRowsPerThread];
#pragma unroll
    for (int j = 0; j < kTRowsPerThread; ++j) {
      const int r = t + j * kTThreads;
      sc[j] = r < rows ? score[base + r] : 0.0;
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
        score[base + r] = sc[j] + lv;
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

// The out-of-bag rows of a bagged tree (LaunchLeafMapList): list[i] -> its leaf in map[row].
// List positions are ascending rows, so a wave's row loads and map writes stay local; the walk
// is k_traverse_col's (COL: group-major bins) or the packed rows' (W = 1 / 2 byte group bins).
template <bool COL, int W, typename T, int R>
__global__ __launch_bounds__(kTThreads) void k_traverse_list(const uint8_t* __restrict__ bins, long long stride, int n,
                                                             const int* __restrict__ list, int count,
                                                             const TNode* __restrict__ nodes, int num_nodes,
                                                             const TCat* __restrict__ cats,
                                                             const uint32_t* __restrict__ cat_bits, T* __restrict__ map) {
  extern __shared__ __align__(16) unsigned char lds[];
  TNode* s_nodes = reinterpret_cast<TNode*>(lds);
  const int t = threadIdx.x;
  for (int i = t; i < num_nodes * static_cast<int>(sizeof(TNode) / 4); i += kTThreads) {
    reinterpret_cast<uint32_t*>(s_nodes)[i] = reinterpret_cast<const uint32_t*>(nodes)[i];
  }
  __syncthreads();
  for (int base = blockIdx.x * kTThreads * R; base < count; base += gridDim.x * kTThreads * R) {
    int row[R], node[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int p = base + t + j * kTThreads;
      row[j] = p < count ? list[p] : 0;
      node[j] = p < count ? 0 : ~0;
    }
    // one level of all R walks per pass: the R node reads, then the R gathers issued together
    // (finished walks re-read the root's node and skip their gather), then the R decisions
    bool live = true;
    while (live) {
      live = false;
      TNode nd[R];
      uint32_t gb[R];
#pragma unroll
      for (int j = 0; j < R; ++j) nd[j] = s_nodes[node[j] < 0 ? 0 : node[j]];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        gb[j] = 0;
        if (node[j] >= 0) {
          if (COL) {
            const size_t o = static_cast<size_t>(nd[j].group) * n + row[j];
            gb[j] = W == 1 ? bins[o] : reinterpret_cast<const uint16_t*>(bins)[o];
          } else {
            gb[j] = GroupBin<W>(bins + static_cast<size_t>(row[j]) * stride, nd[j].group);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (node[j] < 0) continue;
        bool left;
        if (nd[j].flags & kTCat) {
          left = CatLeft(cats[node[j]], cat_bits, gb[j]);
        } else if (gb[j] < nd[j].lo || gb[j] > nd[j].hi) {
          left = (nd[j].flags & kTOutLeft) != 0;
        } else if (static_cast<int>(gb[j]) == nd[j].gmiss) {
          left = (nd[j].flags & kTDefaultLeft) != 0;
        } else {
          left = gb[j] <= nd[j].tg;
        }
        node[j] = left ? nd[j].left : nd[j].right;
        live |= node[j] >= 0;
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (base + t + j * kTThreads < count) map[row[j]] = static_cast<T>(~node[j]);
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

template <typename T, int R>
void LaunchListT(const uint8_t* colbins, const uint32_t* rowbins, int stride_dw, int width, int n, const int* list,
                 int count, const TNode* nodes, int num_nodes, const TCat* cats, const uint32_t* cat_bits, T* map,
                 int num_cu, hipStream_t s) {
  const size_t lds = sizeof(TNode) * static_cast<size_t>(std::max(num_nodes, 1));
  const int grid = std::max(1, std::min(DivUp(count, kTThreads * R), num_cu * 8));
  const long long stride = 4LL * stride_dw;
  if (colbins != nullptr) {
    if (width == 1) k_traverse_list<true, 1, T, R><<<grid, kTThreads, lds, s>>>(colbins, 0, n, list, count, nodes, num_nodes, cats, cat_bits, map);
    else k_traverse_list<true, 2, T, R><<<grid, kTThreads, lds, s>>>(colbins, 0, n, list, count, nodes, num_nodes, cats, cat_bits, map);
  } else {
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rowbins);
    if (width == 1) k_traverse_list<false, 1, T, R><<<grid, kTThreads, lds, s>>>(rb, stride, n, list, count, nodes, num_nodes, cats, cat_bits, map);
    else k_traverse_list<false, 2, T, R><<<grid, kTThreads, lds, s>>>(rb, stride, n, list, count, nodes, num_nodes, cats, cat_bits, map);
  }
}

template <typename T>
void LaunchListR(const uint8_t* colbins, const uint32_t* rowbins, int stride_dw, int width, int n, const int* list,
                 int count, const TNode* nodes, int num_nodes, const TCat* cats, const uint32_t* cat_bits, T* map,
                 int rows_per_thread, int num_cu, hipStream_t s) {
  if (rows_per_thread <= 2) LaunchListT<T, 2>(colbins, rowbins, stride_dw, width, n, list, count, nodes, num_nodes, cats, cat_bits, map, num_cu, s);
  else if (rows_per_thread <= 4) LaunchListT<T, 4>(colbins, rowbins, stride_dw, width, n, list, count, nodes, num_nodes, cats, cat_bits, map, num_cu, s);
  else LaunchListT<T, 8>(colbins, rowbins, stride_dw, width, n, list, count, nodes, num_nodes, cats, cat_bits, map, num_cu, s);
}

void LaunchLeafMapList(const uint8_t* colbins, const uint32_t* rowbins, int stride_dw, int width, int n,
                       const int* list, int count, const TNode* nodes, int num_nodes, const TCat* cats,
                       const uint32_t* cat_bits, int map_leaves, void* map, int rows_per_thread, int num_cu,
                       hipStream_t s) {
  if (count <= 0) return;
  if (width != 1 && width != 2) Log::Fatal("LaunchLeafMapList: group-bin width %d (8- / 16-bit rows)", width);
  if (map_leaves <= 256) {
    LaunchListR(colbins, rowbins, stride_dw, width, n, list, count, nodes, num_nodes, cats, cat_bits,
                static_cast<uint8_t*>(map), rows_per_thread, num_cu, s);
  } else {
    LaunchListR(colbins, rowbins, stride_dw, width, n, list, count, nodes, num_nodes, cats, cat_bits,
                static_cast<uint16_t*>(map), rows_per_thread, num_cu, s);
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

namespace {

constexpr int kLMThreads = 256;
constexpr int kLBItems = 8;                        // positions per lane in k_leaf_bounds
constexpr int kLTItems = kLTRows / kLMThreads;     // rows per lane in k_leaf_tile_map
static_assert(kLTRows % (4 * kLMThreads) == 0, "tile rows");

__device__ __forceinline__ const int* IdxBuf(const LeafMapArgs& a, int b) {
  const int* p = nullptr;  // selects, not a dynamically indexed kernel-argument array
#pragma unroll
  for (int q = 0; q < kLeafIdxBufs; ++q) p = q == b ? a.idx[q] : p;
  return p;
}

// largest power of two <= max(n - 1, 1): the first step of a uniform binary search over n
// sorted entries
__device__ __forceinline__ int SearchTop(int n) {
  int top = 1;
  while (2 * top <= n - 1) top *= 2;
  return top;
}

// A leaf's segment is monotone: the frontier partition keeps the parent's order for the left
// child and writes the right child's rows from the range's end, so a leaf's rows descend when
// it lies right of an odd number of its ancestors' splits (LeafSeg::pad bit 0, set by the
// host from the tree). A descending segment is read back to front: v = 0 .. count - 1 walks
// every leaf's rows in ascending order.
//
// bounds[l * (ntiles + 1) + t] = first (ascending-order) position of leaf l whose row is >=
// t * kLTRows. Position p writes the tiles its row opens after the previous position's row;
// the segment's last position closes the tiles past its row. Empty leaves write nothing (the
// tile kernel skips them). kLBItems positions per lane, each phase's loads issued together.
template <int MAXL>
__global__ __launch_bounds__(kLMThreads) void k_leaf_bounds(LeafMapArgs a, int ntiles, int* __restrict__ bounds) {
  __shared__ int s_off[MAXL + 1];
  __shared__ const int* s_first[MAXL];  // leaf l's ascending-order row v: s_first[l][s_step[l] * v]
  __shared__ int s_step[MAXL];
  const int nl = a.num_leaves, t = threadIdx.x;
  for (int i = t; i <= nl; i += kLMThreads) {
    s_off[i] = a.seg_off[i];
    if (i < nl) {
      const LeafSeg sg = a.segs[i];
      const bool desc = sg.pad & 1;
      s_first[i] = IdxBuf(a, sg.buf) + (desc ? sg.start + sg.count - 1 : sg.start);
      s_step[i] = desc ? -1 : 1;
    }
  }
  __syncthreads();
  // the leaf of the lane's first position by binary search; the later ones (256 positions on
  // each) almost always sit in the same leaf: a forward walk
  const int p0 = blockIdx.x * kLMThreads * kLBItems + t;
  int lo[kLBItems];
  lo[0] = 0;
  for (int st = SearchTop(nl); st > 0; st >>= 1) {
    const int c = lo[0] + st;
    if (c < nl && s_off[c] <= p0) lo[0] = c;
  }
#pragma unroll
  for (int k = 1; k < kLBItems; ++k) {
    int l = lo[k - 1];
    while (l + 1 < nl && s_off[l + 1] <= p0 + k * kLMThreads) ++l;
    lo[k] = l;
  }
  int r[kLBItems], rp[kLBItems];
#pragma unroll
  for (int k = 0; k < kLBItems; ++k) {
    const int p = p0 + k * kLMThreads;
    r[k] = rp[k] = -1;
    if (p < a.n) {
      const int l = lo[k], v = p - s_off[l], st = s_step[l];
      const int* f = s_first[l];
      r[k] = f[st * v];
      if (v > 0) rp[k] = f[st * (v - 1)];
    }
  }
#pragma unroll
  for (int k = 0; k < kLBItems; ++k) {
    const int p = p0 + k * kLMThreads;
    if (p >= a.n) continue;
    const int l = lo[k], tr = r[k] >> kLTShift, tp = rp[k] < 0 ? -1 : rp[k] >> kLTShift;
    int* bl = bounds + static_cast<size_t>(l) * (ntiles + 1);
    for (int tt = tp + 1; tt <= tr; ++tt) bl[tt] = p;
    if (p == s_off[l + 1] - 1) {
      for (int tt = tr + 1; tt <= ntiles; ++tt) bl[tt] = p + 1;
    }
  }
}

// One tile of kLTRows rows per block: the tile's run of every leaf (from the bounds), the
// row -> leaf map of the tile gathered into LDS from the runs' row indices, then written out
// coalesced (map[row], T = uint8 / uint16). Two rounds of global loads: the leaves' bounds /
// segments, then the runs' row indices. The leaf of each tile-local slot j is filled run by
// run (a wave per leaf) instead of searched per row. Block 0 also copies the leaf values
// (lv_out: the deferred score add reads them after the staging buffer has been reused).
template <int MAXL, typename T>
__global__ __launch_bounds__(kLMThreads) void k_leaf_tile_map(LeafMapArgs a, int ntiles, const int* __restrict__ bounds,
                                                              T* __restrict__ map, double* __restrict__ lv_out) {
  constexpr int kPer = MAXL / kLMThreads;  // leaves per lane
  __shared__ const int* s_ptr[MAXL];  // row of tile-local j in leaf l's run: s_ptr[l][s_step[l] * j]
  __shared__ int s_step[MAXL];
  __shared__ int s_pre[MAXL + 1];     // tile-local start of each leaf's run
  __shared__ __align__(16) uint16_t s_leaf[kLTRows];
  __shared__ __align__(16) T s_map[kLTRows];
  __shared__ int s_wsum[kLMThreads / kWave];
  const int tid = threadIdx.x, nl = a.num_leaves, t = blockIdx.x;
  const int r0 = t * kLTRows, rows = min(kLTRows, a.n - r0);
  // leaves l0 + i of this lane (i < kPer): loads, run lengths, block exclusive scan, descriptors
  const int l0 = tid * kPer;
  int o0[kPer], o1[kPer], b0[kPer], b1[kPer];
  LeafSeg sg[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int l = l0 + i;
    o0[i] = o1[i] = b0[i] = b1[i] = 0;
    if (l < nl) {
      const int* bl = bounds + static_cast<size_t>(l) * (ntiles + 1) + t;
      o0[i] = a.seg_off[l];
      o1[i] = a.seg_off[l + 1];
      b0[i] = bl[0];  // (unwritten for an empty leaf: not used)
      b1[i] = bl[1];
      sg[i] = a.segs[l];
      if (t == 0) lv_out[l] = a.leaf_value[l];
    }
  }
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) cnt += l0 + i < nl && o1[i] > o0[i] ? b1[i] - b0[i] : 0;
  const int incl = WaveInclusiveScan(cnt);
  const int w = tid / kWave, lane = tid % kWave;
  if (lane == kWave - 1) s_wsum[w] = incl;
  __syncthreads();
  int base = incl - cnt;
  for (int q = 0; q < w; ++q) base += s_wsum[q];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int l = l0 + i;
    if (l >= nl) continue;
    const bool nonempty = o1[i] > o0[i];
    const int c = nonempty ? b1[i] - b0[i] : 0, v0 = (nonempty ? b0[i] : o0[i]) - o0[i];
    const bool desc = sg[i].pad & 1;
    const int st = desc ? -1 : 1;
    // ascending-order row v of the leaf: first[st * v]; slot j of the run holds v = v0 + j - base
    const int* first = IdxBuf(a, sg[i].buf) + (desc ? sg[i].start + sg[i].count - 1 : sg[i].start);
    s_pre[l] = base;
    s_ptr[l] = first + st * (v0 - base);
    s_step[l] = st;
    base += c;
  }
  if (tid == 0) s_pre[nl] = rows;
  __syncthreads();
  for (int l = w; l < nl; l += kLMThreads / kWave) {
    const int j1 = s_pre[l + 1];
    for (int j = s_pre[l] + lane; j < j1; j += kWave) s_leaf[j] = static_cast<uint16_t>(l);
  }
  __syncthreads();
  int rr[kLTItems], ll[kLTItems];
#pragma unroll
  for (int k = 0; k < kLTItems; ++k) {
    const int j = tid + k * kLMThreads;
    if (j < rows) {
      const int l = s_leaf[j];
      ll[k] = l;
      rr[k] = s_ptr[l][s_step[l] * j];
    }
  }
#pragma unroll
  for (int k = 0; k < kLTItems; ++k) {
    if (tid + k * kLMThreads < rows) s_map[rr[k] - r0] = static_cast<T>(ll[k]);
  }
  __syncthreads();
  // out: 16 bytes per lane (the tile is 16-byte aligned in the map; a partial last tile by element)
  constexpr int kVec = 16 / sizeof(T);
  if (rows == kLTRows) {
    for (int q = tid; q < kLTRows / kVec; q += kLMThreads) {
      reinterpret_cast<uint4*>(map + r0)[q] = reinterpret_cast<const uint4*>(s_map)[q];
    }
  } else {
    for (int i = tid; i < rows; i += kLMThreads) map[r0 + i] = s_map[i];
  }
}

// The deferred score add: score[i] += lv[map[i]] over four rows per lane (GRAD: then the
// pointwise gradients at the new score, the next iteration's gradient pass folded in: the
// same PointwiseGradient on the same score value as k_pointwise2). Leaf values in LDS.
struct AddGradArgs {
  PointwiseParams p;
  const float* label;
  const float* weight;  // nullptr: unweighted
  const float* aux;     // MAPE label weights, nullptr: none
  float2* gh;
};

template <typename T, bool GRAD>
__device__ __forceinline__ void LeafAddRow(const double* s_lv, const T* map, double* score, const AddGradArgs& g, int i) {
  const double ns = score[i] + s_lv[map[i]];
  score[i] = ns;
  if (GRAD) {
    score_t gg, hh;
    PointwiseGradient(g.p, ns, static_cast<double>(g.label[i]), g.weight ? static_cast<double>(g.weight[i]) : 1.0,
                      g.weight != nullptr, g.aux ? static_cast<double>(g.aux[i]) : 0.0, &gg, &hh);
    g.gh[i] = make_float2(gg, hh);
  }
}

template <typename T, bool GRAD>
__global__ __launch_bounds__(kLMThreads) void k_leaf_add(const T* __restrict__ map, const double* __restrict__ leaf_value,
                                                         int nl, int n, bool vec, double* __restrict__ score,
                                                         AddGradArgs g) {
  __shared__ double s_lv[kLMMaxLeaves];
  for (int i = threadIdx.x; i < nl; i += kLMThreads) s_lv[i] = leaf_value[i];
  __syncthreads();
  const int stride = gridDim.x * kLMThreads;
  const int quads = vec ? n >> 2 : 0;
  for (int q = blockIdx.x * kLMThreads + threadIdx.x; q < quads; q += stride) {
    uint32_t l[4];
    if (sizeof(T) == 1) {
      const uint32_t m = reinterpret_cast<const uint32_t*>(map)[q];
      l[0] = m & 0xFFu, l[1] = (m >> 8) & 0xFFu, l[2] = (m >> 16) & 0xFFu, l[3] = m >> 24;
    } else {
      const uint2 m = reinterpret_cast<const uint2*>(map)[q];
      l[0] = m.x & 0xFFFFu, l[1] = m.x >> 16, l[2] = m.y & 0xFFFFu, l[3] = m.y >> 16;
    }
    double2* s2 = reinterpret_cast<double2*>(score) + 2 * q;
    double2 x = s2[0], y = s2[1];
    float4 lb, wt = make_float4(1.f, 1.f, 1.f, 1.f), ax = make_float4(0.f, 0.f, 0.f, 0.f);
    if (GRAD) {
      lb = reinterpret_cast<const float4*>(g.label)[q];
      if (g.weight) wt = reinterpret_cast<const float4*>(g.weight)[q];
      if (g.aux) ax = reinterpret_cast<const float4*>(g.aux)[q];
    }
    x.x += s_lv[l[0]];
    x.y += s_lv[l[1]];
    y.x += s_lv[l[2]];
    y.y += s_lv[l[3]];
    s2[0] = x;
    s2[1] = y;
    if (GRAD) {
      const double ns[4] = {x.x, x.y, y.x, y.y};
      const float lbs[4] = {lb.x, lb.y, lb.z, lb.w}, wts[4] = {wt.x, wt.y, wt.z, wt.w}, axs[4] = {ax.x, ax.y, ax.z, ax.w};
      score_t gg[4], hh[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        PointwiseGradient(g.p, ns[u], static_cast<double>(lbs[u]), g.weight ? static_cast<double>(wts[u]) : 1.0,
                          g.weight != nullptr, g.aux ? static_cast<double>(axs[u]) : 0.0, &gg[u], &hh[u]);
      }
      float4* o = reinterpret_cast<float4*>(g.gh) + 2 * q;
      o[0] = make_float4(gg[0], hh[0], gg[1], hh[1]);
      o[1] = make_float4(gg[2], hh[2], gg[3], hh[3]);
    }
  }
  for (int i = 4 * quads + blockIdx.x * kLMThreads + threadIdx.x; i < n; i += stride) {
    LeafAddRow<T, GRAD>(s_lv, map, score, g, i);
  }
}

template <int MAXL>
void LaunchLeafTile(const LeafMapArgs& a, int* bounds, void* map, double* lv_out, hipStream_t s) {
  const int ntiles = DivUp(a.n, kLTRows);
  k_leaf_bounds<MAXL><<<DivUp(a.n, kLMThreads * kLBItems), kLMThreads, 0, s>>>(a, ntiles, bounds);
  HIP_CHECK(hipGetLastError());
  if (a.num_leaves <= 256) {
    k_leaf_tile_map<MAXL, uint8_t><<<ntiles, kLMThreads, 0, s>>>(a, ntiles, bounds, static_cast<uint8_t*>(map), lv_out);
  } else {
    k_leaf_tile_map<MAXL, uint16_t><<<ntiles, kLMThreads, 0, s>>>(a, ntiles, bounds, static_cast<uint16_t*>(map), lv_out);
  }
  HIP_CHECK(hipGetLastError());
}

template <bool GRAD>
void LaunchAdd(const void* map, const double* lv, int nl, int n, double* score, const AddGradArgs& g, int num_cu,
               hipStream_t s) {
  if (n <= 0) return;
  // 16-byte score / gh accesses need 16-byte aligned slices (class k of K starts at k * n rows)
  const bool vec = (reinterpret_cast<uintptr_t>(score) & 15u) == 0;
  const int grid = std::max(1, std::min(DivUp(vec ? DivUp(n, 4) : n, kLMThreads), num_cu * 16));
  if (nl <= 256) {
    k_leaf_add<uint8_t, GRAD><<<grid, kLMThreads, 0, s>>>(static_cast<const uint8_t*>(map), lv, nl, n, vec, score, g);
  } else {
    k_leaf_add<uint16_t, GRAD><<<grid, kLMThreads, 0, s>>>(static_cast<const uint16_t*>(map), lv, nl, n, vec, score, g);
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace

size_t LeafTileBoundsInts(int n, int num_leaves) {
  return static_cast<size_t>(num_leaves) * ((n + kLTRows - 1) / kLTRows + 1);
}

void LaunchLeafMap(const LeafMapArgs& a, int* bounds, void* map, double* lv_out, hipStream_t s) {
  if (a.n <= 0 || a.num_leaves <= 0) return;
  if (a.num_leaves > kLMMaxLeaves) Log::Fatal("LaunchLeafMap: %d leaves > %d", a.num_leaves, kLMMaxLeaves);
  if (a.num_leaves <= 256) LaunchLeafTile<256>(a, bounds, map, lv_out, s);
  else LaunchLeafTile<kLMMaxLeaves>(a, bounds, map, lv_out, s);
}

void LaunchLeafMapAdd(const void* map, const double* lv, int num_leaves, int n, double* score, int num_cu,
                      hipStream_t s) {
  LaunchAdd<false>(map, lv, num_leaves, n, score, AddGradArgs{}, num_cu, s);
}

void LaunchLeafMapAddGrad(const void* map, const double* lv, int num_leaves, int n, double* score,
                          const PointwiseParams& p, const float* label, const float* weight, const float* aux, float2* gh,
                          int num_cu, hipStream_t s) {
  AddGradArgs g;
  g.p = p;
  g.label = label;
  g.weight = weight;
  g.aux = aux;
  g.gh = gh;
  LaunchAdd<true>(map, lv, num_leaves, n, score, g, num_cu, s);
}

}  // namespace device
}  // namespace lgap
