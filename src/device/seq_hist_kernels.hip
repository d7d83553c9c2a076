// Sequential chain: gradient quantizer, root sums, LDS fixed-point histograms (k_hist),
// slab reduce, owner push and the in-kernel xGMI exchange (declarations: seq_kernels.h).
#include "device/seq_kernels.h"

namespace lgap {
namespace device {
namespace seq {

// ---------------------------------------------------------------------------
// quantized-gradient training (reference gradient_discretizer.cpp:66-160):
// max |g|, |h| over the rows, then integer levels with stochastic rounding,
// stored de-scaled in place so the fixed-point histograms sum exact integers.

__device__ __forceinline__ float HashUniform(uint32_t seed, uint32_t i) {
  uint32_t x = i * 0x9E3779B1u + seed * 0x85EBCA77u;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return static_cast<float>(x >> 8) * (1.0f / 16777216.0f);
}

// 16-byte loads (two rows per float4), four in flight per thread, one atomic pair per block
// (the per-wave atomics and 8-byte loads ran at ~0.75 TB/s: 106 us at 10M rows)
__global__ __launch_bounds__(256) void k_qmax(const float2* gh, int n, unsigned* qmax) {
  __shared__ float s_m[2][4];
  float mg = 0.f, mh = 0.f;
  if ((reinterpret_cast<uintptr_t>(gh) & 15u) != 0 && n > 0) {  // class slice at an odd row offset
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      mg = fabsf(gh[0].x);
      mh = fabsf(gh[0].y);
    }
    ++gh;
    --n;
  }
  const float4* g4 = reinterpret_cast<const float4*>(gh);
  const int n4 = n / 2;
  const int stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = g4[i + j * stride];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mg = fmaxf(mg, fmaxf(fabsf(v[j].x), fabsf(v[j].z)));
      mh = fmaxf(mh, fmaxf(fabsf(v[j].y), fabsf(v[j].w)));
    }
  }
  for (; i < n4; i += stride) {
    const float4 v = g4[i];
    mg = fmaxf(mg, fmaxf(fabsf(v.x), fabsf(v.z)));
    mh = fmaxf(mh, fmaxf(fabsf(v.y), fabsf(v.w)));
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const float2 v = gh[n - 1];  // (n, gh: after the alignment step)
    mg = fmaxf(mg, fabsf(v.x));
    mh = fmaxf(mh, fabsf(v.y));
  }
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o, kWave));
    mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_m[0][w] = mg;
    s_m[1][w] = mh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) {
      mg = fmaxf(mg, s_m[0][k]);
      mh = fmaxf(mh, s_m[1][k]);
    }
    atomicMax(&qmax[0], __float_as_uint(mg));  // non-negative floats order as their bits
    atomicMax(&qmax[1], __float_as_uint(mh));
  }
}

// ghq (frontier engine, hist MODE 2): the same levels as int8 g << 8 | uint8 h
__global__ __launch_bounds__(256) void k_quantize(float2* gh, float2* gh_true, uint16_t* ghq, int n, const unsigned* qmax,
                                                  int bins, int const_hess, uint32_t seed, int stochastic) {
  const double mg = __uint_as_float(qmax[0]), mh = __uint_as_float(qmax[1]);
  const double gs = mg / (bins / 2), hs = const_hess ? mh : mh / bins;
  const double ig = gs > 0 ? 1.0 / gs : 0.0, ih = hs > 0 ? 1.0 / hs : 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 v = gh[i];
    if (gh_true) gh_true[i] = v;
    const double rg = stochastic ? HashUniform(seed, 2u * i) : 0.5;
    const double rh = stochastic ? HashUniform(seed, 2u * i + 1u) : 0.5;
    const double x = v.x * ig;
    const int q = static_cast<int>(v.x >= 0.f ? x + rg : x - rg);  // truncation toward zero
    const int qh = const_hess ? 1 : static_cast<int>(v.y * ih + rh);
    float2 o;
    o.x = static_cast<float>(q * gs);
    o.y = static_cast<float>(qh * hs);
    gh[i] = o;
    if (ghq) ghq[i] = static_cast<uint16_t>((static_cast<uint32_t>(static_cast<uint8_t>(static_cast<int8_t>(q))) << 8) |
                                            static_cast<uint32_t>(qh & 0xFF));
  }
}

// ---------------------------------------------------------------------------
// tree setup

__global__ __launch_bounds__(kNodeThreads) void k_init_tree(Args a) {
  const TreeParams tp = *a.tp;
  const int t = threadIdx.x;
  if (t == 0) {
    Ctl c;
    c.num_leaves = 1;
    c.done = 0;
    c.smaller = 0;
    c.larger = -1;
    c.skip = 0;
    c.num_splits = 0;
    c.split_leaf = -1;
    c.new_leaf = -1;
    c.parent_buf = tp.root_buf;
    c.parent_start = 0;
    c.parent_count = tp.root_count;
    c.target_buf = 0;
    c.left_count = 0;
    c.cls = tp.cls;
    c.scan_round = 0;
    c.max_count = tp.root_count;
    c.hist_nb = 0;
    // the split epoch keeps increasing across trees (tile_pub tags must never repeat)
    const unsigned e0 = a.ctl->epoch, e1 = a.ctl_next ? a.ctl_next->epoch : 0u;
    c.epoch = (e0 > e1 ? e0 : e1) + 1u;
    c.pad1 = c.pad2 = 0;
    c.plg = c.plh = 0.0;
    *a.ctl = c;
    LeafRange r;
    r.buf = tp.root_buf;
    r.start = 0;
    r.count = tp.root_count;
    r.pad = 0;
    a.range[0] = r;
    a.lsum[0] = make_double2(0.0, 0.0);
    for (int j = 0; j < 4; ++j) a.ghmax[j] = 0u;
    a.gcount[0] = tp.root_gcount;
    a.depth[0] = 0;
    a.lout[0] = 0.0;
    if (a.ic_leaf) a.ic_leaf[0] = ~0ull;
  }
  for (int i = t; i < a.L; i += blockDim.x) {
    a.slot[i] = i;
    a.bounds[i] = LeafBounds();
    a.best[i].Reset();
    a.leaf_key[i].feature = -1;
    a.leaf_key[i].gain = kMinScore;
  }
  for (int f = t; f < a.F; f += blockDim.x) a.splittable[f] = 1;
  if (a.fold_cnt) {
    for (int f = t; f < a.F; f += blockDim.x) a.fold_cnt[f] = 0u;
  }
}

// Root statistics in two steps: per-block partials (no atomics: 1024 blocks x
// device-scope fp64 atomics on one address serialised to ~97 us), then one block
// folds them and writes lsum[0] and the histogram scale bounds (max|g|, max|h|, and
// sum|g|, sum|h| rounded up: frontier.h FixedPointExp).
constexpr int kRootStats = 6;  // sum g, sum h, max|g|, max|h|, sum|g|, sum|h|

__device__ __forceinline__ double RootFold(int i, double x, double y) { return i == 2 || i == 3 ? fmax(x, y) : x + y; }
__device__ __forceinline__ void RootWaveFold(double* v) {
#pragma unroll
  for (int j = 0; j < kRootStats; ++j) {
    if (j == 2 || j == 3) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[j] = fmax(v[j], __shfl_xor(v[j], o, kWave));
    } else {
      v[j] = WaveSum(v[j]);
    }
  }
}

__global__ __launch_bounds__(kRootThreads) void k_root_sums(Args a) {
  __shared__ double sh[kRootStats][kRootThreads / 64];
  const TreeParams tp = *a.tp;
  const float2* gh = a.gh + static_cast<size_t>(tp.cls) * a.N;
  double v[kRootStats] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const int stride = gridDim.x * blockDim.x;
  // (unrolled: four rows' loads in flight per thread; the per-thread sums keep their order)
#pragma unroll 4
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tp.root_count; i += stride) {
    const float2 x = gh[RowAt(a, tp.root_buf, i)];
    v[0] += x.x;
    v[1] += x.y;
    v[2] = fmax(v[2], fabs(static_cast<double>(x.x)));
    v[3] = fmax(v[3], fabs(static_cast<double>(x.y)));
    v[4] += fabs(static_cast<double>(x.x));
    v[5] += fabs(static_cast<double>(x.y));
  }
  RootWaveFold(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int j = 0; j < kRootStats; ++j) sh[j][w] = v[j];
  }
  __syncthreads();
  if (threadIdx.x < kRootStats) {
    const int j = threadIdx.x;
    double x = sh[j][0];
    for (int i = 1; i < kRootThreads / 64; ++i) x = RootFold(j, x, sh[j][i]);
    a.root_part[kRootStats * blockIdx.x + j] = x;
  }
}

__global__ __launch_bounds__(kRootThreads) void k_root_final(Args a, int nblocks) {
  __shared__ double sh[kRootStats][kRootThreads / 64];
  double v[kRootStats] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
    for (int j = 0; j < kRootStats; ++j) v[j] = RootFold(j, v[j], a.root_part[kRootStats * b + j]);
  }
  RootWaveFold(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int j = 0; j < kRootStats; ++j) sh[j][w] = v[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kRootThreads / 64; ++i) {
#pragma unroll
      for (int j = 0; j < kRootStats; ++j) v[j] = RootFold(j, v[j], sh[j][i]);
    }
    a.lsum[0] = make_double2(v[0], v[1]);
    a.ghmax[0] = __float_as_uint(static_cast<float>(v[2]));
    a.ghmax[1] = __float_as_uint(static_cast<float>(v[3]));
    // (the fp64 sums of |value| are exact to ~1e-9 relative: a 2^-20 margin, rounded up)
    a.ghmax[2] = __float_as_uint(__double2float_ru(v[4] * (1.0 + 0x1p-20)));
    a.ghmax[3] = __float_as_uint(__double2float_ru(v[5] * (1.0 + 0x1p-20)));
  }
}

// ---------------------------------------------------------------------------
// histogram of the smaller leaf.
//
// gfx950 executes LDS float atomics (ds_add_f32/f64) at a small fraction of the
// integer rate (measured, scripts/hist_micro.hip: 10M x 28 root histogram 2.06 ms
// with ds_add_f32 vs 0.195 ms with ds_add_u64), so the per-block histogram is
// accumulated in FIXED POINT:
//   default    one ds_add_u64 per (row, group): signed g in the high 32 bits,
//              signed h in the low 32 bits, each scaled by the largest power of two
//              <= 2^30 / (rows_in_block * max|.|) so no partial sum can overflow (and
//              constant hessians are exact); low-part borrows are undone
//              when unpacking. Per-value resolution ~2^-30 * rows * max|g|, below
//              the error of fp32 accumulation for any bin with more than a few
//              hundred rows.
//   gpu_use_dp two ds_add_u64 (g, h) at scale ~2^62 / (rows * max|.|): ~2^-47
//              relative, indistinguishable from the CPU's double sums.
// Each active block unpacks its LDS histogram to real values and stores it into
// its own slab row (plain coalesced stores); k_hist_reduce sums the rows into
// `staging` (fp64). No float atomics anywhere on the hot path.


// MODE 0: packed (g32|h32) in one u64; MODE 1: two u64 (gpu_use_dp)
template <int W, int MODE>
__device__ __forceinline__ void HistRowsFixed(const Args& a, const HistTile& tile, const LeafRange& r, int cls, int rb,
                                              int re, const int* gst, unsigned long long* hist, float sg, float sh,
                                              double dsg, double dsh, double* rsum_g, double* rsum_h) {
  const int tpr = tile.d1 - tile.d0;
  const int rpi = blockDim.x / tpr;
  const int myr = threadIdx.x / tpr;
  const int myd = threadIdx.x - myr * tpr;
  *rsum_g = 0.0;
  *rsum_h = 0.0;
  if (myr >= rpi) return;
  constexpr int per = 4 / W;
  constexpr int R = LGAP_HIST_R;  // rows in flight per thread
  const int dw = tile.d0 + myd;
  const int gfirst = dw * per;
  int go[per];
#pragma unroll
  for (int k = 0; k < per; ++k) go[k] = gfirst + k < tile.g1 ? gst[gfirst + k - tile.g0] : -1;
  const float2* gh = a.gh + static_cast<size_t>(cls) * a.N;
  const int* idx = r.buf < 0 ? nullptr : a.idx[r.buf] + r.start;
  const int base = r.buf < 0 ? r.start : 0;
  // voting: the first dword's thread of each row also sums the row's (g, h) (local leaf sums)
  const bool sums = a.hsum_part != nullptr && myd == 0;
  double tg = 0.0, th = 0.0;
  for (int p0 = rb + myr; p0 < re; p0 += rpi * R) {
    int rows[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int p = p0 + j * rpi;
      rows[j] = p < re ? (idx ? idx[p] : base + p) : -1;
    }
    uint32_t word[R];
    float2 v[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      word[j] = rows[j] >= 0 ? a.rowbins[static_cast<size_t>(rows[j]) * a.stride_dw + dw] : 0u;
      v[j] = rows[j] >= 0 ? gh[rows[j]] : make_float2(0.f, 0.f);
    }
    if (sums) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        tg += v[j].x;
        th += v[j].y;
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      unsigned long long pg, ph = 0ull;
      if (MODE == 0) {
        const long long ig = __float2int_rn(v[j].x * sg);
        const long long ih = __float2int_rn(v[j].y * sh);
        pg = (static_cast<unsigned long long>(ig) << 32) + static_cast<unsigned long long>(ih);
      } else {
        pg = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v[j].x) * dsg));
        ph = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v[j].y) * dsh));
      }
#pragma unroll
      for (int k = 0; k < per; ++k) {
        const uint32_t b = W == 1 ? ((word[j] >> (8 * k)) & 0xFFu) : ((word[j] >> (16 * k)) & 0xFFFFu);
        if (b != 0u && go[k] >= 0) {
          const int o = go[k] + static_cast<int>(b);
          if (MODE == 0) {
            atomicAdd(&hist[o], pg);
          } else {
            atomicAdd(&hist[2 * o], pg);
            atomicAdd(&hist[2 * o + 1], ph);
          }
        }
      }
    }
  }
  *rsum_g = tg;
  *rsum_h = th;
}

// Rows of the (rare) tiles whose bins exceed the LDS budget: fp64 atomics into
// the block's own slab row (global memory, no cross-block contention).
template <int W, typename Acc>
__device__ void HistRowsDirect(const Args& a, const HistTile& tile, const LeafRange& r, int cls, int rb, int re,
                               const int* gst, Acc* hist, double* rsum_g, double* rsum_h) {
  const int tpr = tile.d1 - tile.d0;
  const int rpi = blockDim.x / tpr;
  const int myr = threadIdx.x / tpr;
  const int myd = threadIdx.x - myr * tpr;
  *rsum_g = 0.0;
  *rsum_h = 0.0;
  if (myr >= rpi) return;
  constexpr int per = 4 / W;
  const int dw = tile.d0 + myd;
  const float2* gh = a.gh + static_cast<size_t>(cls) * a.N;
  const int* idx = r.buf < 0 ? nullptr : a.idx[r.buf] + r.start;
  const int base = r.buf < 0 ? r.start : 0;
  const bool sums = a.hsum_part != nullptr && myd == 0;
  double tg = 0.0, th = 0.0;
  for (int p = rb + myr; p < re; p += rpi) {
    const int row = idx ? idx[p] : base + p;
    const uint32_t word = a.rowbins[static_cast<size_t>(row) * a.stride_dw + dw];
    const float2 v = gh[row];
    if (sums) {
      tg += v.x;
      th += v.y;
    }
#pragma unroll
    for (int k = 0; k < per; ++k) {
      const uint32_t b = W == 1 ? ((word >> (8 * k)) & 0xFFu) : ((word >> (16 * k)) & 0xFFFFu);
      const int g = dw * per + k;
      if (b != 0u && g < tile.g1) {
        const int o = gst[g - tile.g0] + static_cast<int>(b);
        atomicAdd(&hist[2 * o], static_cast<Acc>(v.x));
        atomicAdd(&hist[2 * o + 1], static_cast<Acc>(v.y));
      }
    }
  }
  *rsum_g = tg;
  *rsum_h = th;
}

// voting: block sum of the per-thread row sums -> hsum_part[blockIdx.x] (first tile's blocks)
__device__ void PublishRowSums(const Args& a, double tg, double th) {
  if (a.hsum_part == nullptr || blockIdx.y != 0) return;
  __shared__ double s_rs[2][kHistThreads / 64];
  tg = WaveSum(tg);
  th = WaveSum(th);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_rs[0][w] = tg;
    s_rs[1][w] = th;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double g = 0.0, h = 0.0;
    for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) g += s_rs[0][i], h += s_rs[1][i];
    a.hsum_part[blockIdx.x] = make_double2(g, h);
  }
}

template <int W, int MODE>
__global__ __launch_bounds__(kHistThreads) void k_hist(Args a) {
  extern __shared__ __align__(8) unsigned char lds_raw[];
  const Ctl* cp = a.ctl;
  if (cp->done || cp->skip) return;
  const int leaf = cp->smaller;
  const int cls = cp->cls;
  const HistTile tile = a.tiles[blockIdx.y];
  const LeafRange r = a.range[leaf];
  const int n = r.count;
  const int nb = HistActiveBlocks(n, gridDim.x, a.hist_min_rows);
  if (static_cast<int>(blockIdx.x) >= nb) return;
  const int chunk = (n + nb - 1) / nb;
  const int rb = blockIdx.x * chunk;
  const int re = min(n, rb + chunk);
  Stamp(a, 2, 0);
  double* slab = reinterpret_cast<double*>(a.hist_slab) + (static_cast<size_t>(blockIdx.x) * a.TB + tile.bin0) * 2;
  float* slabf = reinterpret_cast<float*>(a.hist_slab) + (static_cast<size_t>(blockIdx.x) * a.TB + tile.bin0) * 2;
  if (tile.direct) {
    int* gst = reinterpret_cast<int*>(lds_raw);
    for (int i = threadIdx.x; i < 2 * tile.nbins; i += blockDim.x) {
      if (MODE == 0) slabf[i] = 0.f;
      else slab[i] = 0.0;
    }
    for (int g = tile.g0 + threadIdx.x; g < tile.g1; g += blockDim.x) gst[g - tile.g0] = a.gstart[g] - tile.bin0;
    __threadfence_block();
    __syncthreads();
    double tg, th;
    if (MODE == 0) HistRowsDirect<W, float>(a, tile, r, cls, rb, re, gst, slabf, &tg, &th);
    else HistRowsDirect<W, double>(a, tile, r, cls, rb, re, gst, slab, &tg, &th);
    PublishRowSums(a, tg, th);
    return;
  }
  const float gmax = __uint_as_float(a.ghmax[0]), hmax = __uint_as_float(a.ghmax[1]);
  const double rows_in_block = static_cast<double>(re - rb > 0 ? re - rb : 1);
  const double kPk = 1073741824.0;            // 2^30
  const double kDp = 4611686018427387904.0;   // 2^62
  // Scales are POWERS OF TWO (the largest not above the overflow bound): scaling is then an
  // exponent shift, de-scaling is exact, and a value with few significant bits (a constant
  // hessian: l2, quantile, ...) is quantized exactly. A non-power-of-two scale rounded every
  // h = 1 the same way: a systematic relative bias of up to 0.5 / scale that the
  // parent - smaller subtraction carried, as an absolute error of the root-size bins, into
  // small deep leaves (near-zero or negative hessian sums, exploding outputs at ~8M rows).
  const double sgd = gmax > 0.f ? Pow2AtMost(kPk / (rows_in_block * gmax)) : 1.0;
  const double shd = hmax > 0.f ? Pow2AtMost(kPk / (rows_in_block * hmax)) : 1.0;
  const double dsg = gmax > 0.f ? Pow2AtMost(kDp / (rows_in_block * gmax)) : 1.0;
  const double dsh = hmax > 0.f ? Pow2AtMost(kDp / (rows_in_block * hmax)) : 1.0;
  const float sg = static_cast<float>(sgd), sh = static_cast<float>(shd);
  const int words = MODE == 0 ? tile.nbins : 2 * tile.nbins;
  unsigned long long* hist = reinterpret_cast<unsigned long long*>(lds_raw);
  int* gst = reinterpret_cast<int*>(hist + words);
  for (int i = threadIdx.x; i < words; i += blockDim.x) hist[i] = 0ull;
  for (int g = tile.g0 + threadIdx.x; g < tile.g1; g += blockDim.x) gst[g - tile.g0] = a.gstart[g] - tile.bin0;
  __syncthreads();
  Stamp(a, 2, 1);
  double tg, th;
  HistRowsFixed<W, MODE>(a, tile, r, cls, rb, re, gst, hist, sg, sh, dsg, dsh, &tg, &th);
  __syncthreads();
  PublishRowSums(a, tg, th);
  Stamp(a, 2, 2);
  if (MODE == 0) {
    const double ig = 1.0 / (static_cast<double>(sg)), ih = 1.0 / (static_cast<double>(sh));
    for (int i = threadIdx.x; i < tile.nbins; i += blockDim.x) {
      const unsigned long long x = hist[i];
      const int hs = static_cast<int>(static_cast<unsigned int>(x & 0xFFFFFFFFull));
      const long long gs = static_cast<long long>(x - static_cast<unsigned long long>(static_cast<long long>(hs))) >> 32;
      slabf[2 * i] = static_cast<float>(static_cast<double>(gs) * ig);
      slabf[2 * i + 1] = static_cast<float>(static_cast<double>(hs) * ih);
    }
  } else {
    const double ig = 1.0 / dsg, ih = 1.0 / dsh;
    for (int i = threadIdx.x; i < tile.nbins; i += blockDim.x) {
      slab[2 * i] = static_cast<double>(static_cast<long long>(hist[2 * i])) * ig;
      slab[2 * i + 1] = static_cast<double>(static_cast<long long>(hist[2 * i + 1])) * ih;
    }
  }
  StampEnd(a, 2);
}

// out[v] = sum over the active blocks' slab rows (v over 2 * TB values), folded
// in fp64. Used where the full histogram must exist in one place: data-parallel
// training (all-reduced over RCCL before the scan; fp32 rows unless gpu_use_dp,
// half the bytes on the wire) and the kernel tests (fp64 staging).
template <typename Acc, typename Out>
__global__ __launch_bounds__(1024) void k_hist_reduce(Args a, int hist_grid, Out* __restrict__ out) {
  __shared__ double part[16][64];
  const Ctl* cp = a.ctl;
  if (cp->done || cp->skip) return;
  const int n = a.range[cp->smaller].count;
  const int nb = cp->hist_nb > 0 ? cp->hist_nb : HistActiveBlocks(n, hist_grid, a.hist_min_rows);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t V = 2 * static_cast<size_t>(a.TB);
  const size_t v = static_cast<size_t>(blockIdx.x) * 64 + lane;
  const Acc* slab = reinterpret_cast<const Acc*>(a.hist_slab);
  double s = 0.0;
  if (v < V) {
    for (int p = w; p < nb; p += 16) s += static_cast<double>(slab[static_cast<size_t>(p) * V + v]);
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && v < V) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][lane];
    out[v] = static_cast<Out>(t);
  }
}

// ---------------------------------------------------------------------------
// Owner-computes data parallelism on the sequential chain (reference
// data_parallel_tree_learner.cpp:225-302, 305-450 and parallel_tree_learner.h:209-232): ranks own
// contiguous, bin-balanced ranges of feature groups; per split the smaller child's histogram is
// reduce-scattered by ownership (ncclReduceScatter, or the host-staged rehearsal collectives), each
// rank scans only the features it owns, and the per-feature candidates are all-gathered into the
// candidate table every rank's select reads. (The chain serves configurations the frontier engine
// does not hold; the frontier's exchanges run in-kernel over xGMI, frontier_kernels.hip.)

// Fold the smaller child's slab rows into the owner-permuted layout: destination q of
// [P][2 * bbin] takes value 2 * bin_lo[r] + l of the local histogram (r = q / (2 bbin),
// l = q % (2 bbin)); padding positions carry zeros. The row goes to `stage` (then
// ncclReduceScatter).
template <typename Acc>
__global__ __launch_bounds__(1024) void k_hist_owner(Args a, int hist_grid, Acc* __restrict__ stage) {
  __shared__ double part[16][64];
  const Ctl* cp = a.ctl;
  if (cp->done || cp->skip) return;
  const int n = a.range[cp->smaller].count;
  const int nb = cp->hist_nb > 0 ? cp->hist_nb : HistActiveBlocks(n, hist_grid, a.hist_min_rows);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int V2 = 2 * a.bbin;
  const int q = blockIdx.x * 64 + lane;
  const int r = q / V2;
  const int l = q - r * V2;
  const bool valid = r < a.P && l < 2 * (a.bin_lo[r + 1] - a.bin_lo[r]);
  const size_t V = 2 * static_cast<size_t>(a.TB);
  const size_t v = valid ? 2 * static_cast<size_t>(a.bin_lo[r]) + l : 0;
  const Acc* slab = reinterpret_cast<const Acc*>(a.hist_slab);
  double s = 0.0;
  if (valid) {
    for (int p = w; p < nb; p += 16) s += static_cast<double>(slab[static_cast<size_t>(p) * V + v]);
  }
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && r < a.P) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][lane];
    stage[q] = valid ? static_cast<Acc>(t) : static_cast<Acc>(0);
  }
}

// One workgroup (16 waves) per feature this rank owns (every feature on one GPU):
//  1. the smaller child's histogram of the feature into LDS: the sum of the active
//     histogram blocks' slab rows (single GPU / feature parallel), or of the owner rows
//     the data-parallel exchange delivered (scan_src 1)
//  2. smaller child's histogram -> its slot; larger child = parent - smaller
//     (the parent histogram lives in the larger child's slot)
//  3. reconstruct the most-frequent bin of each child, then wave 0 scans the
//     smaller child and wave 1 the larger one concurrently, from LDS
//  4. the block writes both candidates into this rank's block of the candidate table
// kGlobal: the block's scratch (histograms, partials, categorical sort) lives in its slice of
// global memory instead of LDS — features wider than the LDS budget (max_bin in the thousands;
// reference cuda_best_split_finder.cu:1561 global-memory variant).

// instantiations launched by the DeviceTreeLearner
template __global__ void k_hist<1, 0>(Args);
template __global__ void k_hist<1, 1>(Args);
template __global__ void k_hist<2, 0>(Args);
template __global__ void k_hist<2, 1>(Args);
template __global__ void k_hist_owner<double>(Args, int, double*);
template __global__ void k_hist_owner<float>(Args, int, float*);
template __global__ void k_hist_reduce<double, double>(Args, int, double*);
template __global__ void k_hist_reduce<float, double>(Args, int, double*);

}  // namespace seq
}  // namespace device
}  // namespace lgap
