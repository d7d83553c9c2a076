// Frontier tree-growth kernels for MI355X (gfx950): see frontier.h for the algorithm.
//
// Launch shapes (fixed per learner; the work of a round is read on the device):
//   k_f_init        1 x 256
//   k_f_partition   grid x 256 (contiguous tiles in block order: no co-residency needed)
//   k_f_hist        max(hist_grid, ceil(hist_grid / 2) + kmax) x LDS tiles, 512 or 1024 threads
//                   (1024 for single-tile rows at >= 4M rows: the 10M headline)
//   k_f_reduce      (2 or 4) x CUs x 256 (grid-stride over (expansion, bin chunk, row group))
//   k_f_scan        min(kmax * F, cap) x 256 (grid-stride over (expansion, feature)); k_f_scan_w
//                   one wave per item for wide numerical data
//   k_f_select      1 x 1024 (instantiations: CEGB / by-node raw candidates, wide phase A, xGMI
//                   exchange, intermediate monotone walk + rescans)
//   k_fx_root       1 x 64 (xGMI transport: once per tree)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "device/frontier.h"
#include "device/hip_common.h"
#include "device/split_scan.h"
#include "lgap/split_math.h"

namespace lgap {
namespace device {
namespace {

constexpr int kFPartThreads = 256;
constexpr int kFScanThreads = 256;
constexpr int kFSelThreads = 1024;
#ifndef LGAP_FHIST_R
#define LGAP_FHIST_R 16
#endif

__device__ __forceinline__ int FRowAt(const FArgs& a, int buf, int pos) { return buf < 0 ? pos : a.idx[buf][pos]; }

__device__ __forceinline__ uint32_t FColBin(const FArgs& a, int g, int row) {
  const size_t o = static_cast<size_t>(g) * a.N + row;
  return a.width == 1 ? a.colbins[o] : reinterpret_cast<const uint16_t*>(a.colbins)[o];
}

// Diagnostic phase stamps (100 MHz wall clock): block 0 / thread 0 records slot i of kernel
// `kern` in round `r`; FStampEnd keeps the latest exit over all blocks in slot 7.
__device__ __forceinline__ void FStamp(const FArgs& a, int r, int kern, int i) {
  if (a.stamps != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    a.stamps[((static_cast<size_t>(r & 255) * 4 + kern) * kFStampSlots) + i] = wall_clock64();
  }
}
// latest time over ALL blocks that reached point `i` (slots 4-6: the spread behind block 0's)
__device__ __forceinline__ void FStampMax(const FArgs& a, int r, int kern, int i) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    atomicMax(&a.stamps[((static_cast<size_t>(r & 255) * 4 + kern) * kFStampSlots) + i], wall_clock64());
  }
}
__device__ __forceinline__ void FStampEnd(const FArgs& a, int r, int kern) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    atomicMax(&a.stamps[((static_cast<size_t>(r & 255) * 4 + kern) * kFStampSlots) + 7], wall_clock64());
  }
}

// exponent k of the largest power of two <= x (x > 0): 2^k <= x < 2^(k+1)
__device__ __forceinline__ int Pow2Exp(double x) {
  int e;
  (void)frexp(x, &e);
  return e - 1;
}

// Global fixed-point exponents of the tree: every accumulator holds value * 2^E with
// 2^E <= 2^62 / min(root rows * max|value|, sum|value|), so no sum over any subset of the
// root's rows can overflow an int64 and every partial of every block, expansion and rank is
// EXACT integer arithmetic at one shared scale (deterministic and order free). Row-sharded
// ranks max-reduce their local sums: the global sum is at most sum_mult times that.
__device__ __forceinline__ void GlobalScaleExp(const FArgs& a, int* eg, int* eh) {
  const double n = static_cast<double>(a.tp->root_gcount > 0 ? a.tp->root_gcount : 1);
  constexpr double k62 = 4611686018427387904.0;
  const float m = a.sum_bound ? static_cast<float>(a.sum_mult > 1 ? a.sum_mult : 1) : INFINITY;
  *eg = FixedPointExp(k62, n, __uint_as_float(a.ghmax[0]), __uint_as_float(a.ghmax[2]) * m);
  *eh = FixedPointExp(k62, n, __uint_as_float(a.ghmax[1]), __uint_as_float(a.ghmax[3]) * m);
}

// Quantized training: the value of one g / h level (must match k_quantize in
// device_learner.hip, which stores float(level * scale) in gh for everything else).
__device__ __forceinline__ void QuantScales(const FArgs& a, double* gs, double* hs) {
  const double mg = __uint_as_float(a.qmax[0]), mh = __uint_as_float(a.qmax[1]);
  *gs = mg / (a.qbins / 2);
  *hs = a.qconst ? mh : mh / a.qbins;
}

// Word offset of (expansion e, bin b) in the round's accumulators: [e][TB] x pw words, or --
// data-parallel owner-computes -- [owner rank][xkb][own_w] x pw words, the layout the
// reduce-scatter splits by rank (rank r owns the groups of bins [own_b0[r], own_b0[r + 1]))
__device__ __forceinline__ size_t FAccAt(const FArgs& a, int e, int b, int pw) {
  if (!a.own) return (static_cast<size_t>(e) * a.TB + b) * pw;
  int r = 0;
  while (r + 1 < a.own_P && a.own_b0[r + 1] <= b) ++r;
  return ((static_cast<size_t>(r) * a.xkb + e) * a.own_w + (b - a.own_b0[r])) * pw;
}

// Accumulator words of (expansion e, bin b): the local round accumulators, or -- owner-computes
// over the xGMI transport -- the receive chunk [kmax][own_w] x pw of b's OWNER rank, in that rank's
// exchange buffer (feature parallel exchanges only its per-child bests: local accumulators)
__device__ __forceinline__ unsigned long long* FAccPtr(const FArgs& a, int e, int b, int pw) {
  if (!a.xg || !a.own) return a.acc + FAccAt(a, e, b, pw);
  int r = 0;
  while (r + 1 < a.own_P && a.own_b0[r + 1] <= b) ++r;
  return reinterpret_cast<unsigned long long*>(a.xc->peer[r] + a.xc->o_recv) +
         (static_cast<size_t>(e) * a.own_w + (b - a.own_b0[r])) * pw;
}

// Interaction constraints: feature f may split node c when some set allowed on c's path holds f
// (reference col_sampler.hpp GetByNode's allowed features), as 64-set words.
__device__ __forceinline__ bool FIcAllows(const FArgs& a, int c, int f) {
  unsigned long long any = 0ull;
  for (int w = 0; w < a.ic_words; ++w) {
    any |= a.ic[static_cast<size_t>(c) * a.ic_words + w] & a.ic_feat[static_cast<size_t>(f) * a.ic_words + w];
  }
  return any != 0ull;
}

// ---- xGMI transport handshake (FArgs::xg). Tags are (session << 32) | round: strictly
// increasing for the life of the exchange buffer, so a flag is only compared for "reached".
__device__ __forceinline__ unsigned long long FXTag(const FArgs& a, unsigned ep) {
  return (static_cast<unsigned long long>(a.xsession) << 32) | ep;
}
__device__ __forceinline__ unsigned long long* FXFlag(const FArgs& a, int owner, int kind, int src) {
  return reinterpret_cast<unsigned long long*>(a.xc->peer[owner] + a.xc->o_flag) + kind * kMaxXRanks + src;
}
// one lane: spin (bounded by xtimeout; then bar[3] = 1 + kind) until every rank tagged this rank's
// flag row `kind` with at least `tag`
__device__ inline bool FXWaitAll(const FArgs& a, int kind, unsigned long long tag) {
  const unsigned long long t0 = wall_clock64();
  for (int q = 0; q < a.xc->P; ++q) {
    unsigned long long* f = FXFlag(a, a.xc->rank, kind, q);
    unsigned spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < tag) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255u) == 0u &&
          (wall_clock64() - t0 > a.xc->timeout || __hip_atomic_load(&a.bar[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
        __hip_atomic_store(&a.bar[3], 1u + kind, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}
// Pushes into exchange buffers are SYSTEM-scope operations (atomics carry sc1, stores sc0 sc1): a
// peer's IPC mapping of a buffer need not be uncached in the pushing process, so a plain store or
// device-scope atomic could sit in the pusher's L2; at system scope the acknowledgement means the
// value reached memory, so a wave's s_waitcnt before it arrives is enough -- no L2 write-back.
__device__ __forceinline__ void FXAdd(unsigned long long* p, unsigned long long v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void FXStore(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void FXStoreRec(T* dst, const T& v) {
  static_assert(sizeof(T) % 4 == 0, "word records");
  for (int i = 0; i < static_cast<int>(sizeof(T) / 4); ++i) {
    FXStore(reinterpret_cast<uint32_t*>(dst) + i, reinterpret_cast<const uint32_t*>(&v)[i]);
  }
}

// Reads of what peers pushed are system-scope too (sc0 sc1: past every cache), whatever the
// mapping's cache policy: a line read in an earlier round must never be served stale.
__device__ __forceinline__ uint32_t FXLoad(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long FXLoad64(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void FXStore64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T FXLoadRec(const T* src) {
  T v;
  for (int i = 0; i < static_cast<int>(sizeof(T) / 4); ++i) {
    reinterpret_cast<uint32_t*>(&v)[i] = FXLoad(reinterpret_cast<const uint32_t*>(src) + i);
  }
  return v;
}
// (feature, gain) of a candidate key; `sys`: a record pushed by a peer (system-scope loads)
__device__ __forceinline__ void FKeyFG(const SplitKey& kk, bool sys, int* f, double* g) {
  if (!sys) {
    *f = kk.feature;
    *g = kk.gain;
    return;
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&kk);
  *f = static_cast<int>(FXLoad(w + offsetof(SplitKey, feature) / 4));
  const unsigned long long lo = FXLoad(w + offsetof(SplitKey, gain) / 4), hi = FXLoad(w + offsetof(SplitKey, gain) / 4 + 1);
  *g = __longlong_as_double(static_cast<long long>((hi << 32) | lo));
}

// Whether a producing launch has peers to signal: one rank has none (its pushes are ordered for
// the consumer by the kernel boundary), except under the fault-injection hook, which must wait.
__device__ __forceinline__ bool FXPeers(const FArgs& a) { return a.xc->P > 1 || a.xc->fault; }

// Every thread of every block of a producing launch calls this after its pushes: each wave waits
// until its stores / atomics are acknowledged (they target uncached memory, so no cache needs a
// write-back: a per-wave fence would write back the XCD's L2 once per wave, measured at ~40% of a
// 1.25M-row iteration), the block arrives on the launch's counter, and the LAST block to arrive
// releases system-wide, tags flag[kind][this rank] in every peer and waits until all P ranks
// tagged its own row. Only that one block spins, so the peers' producers always find CUs.
__device__ inline void FXArrive(const FArgs& a, int kind, unsigned long long tag) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x * gridDim.y;
    if (atomicAdd(&a.xc->cnt[kind], 1u) == nb - 1u) {
      atomicExch(&a.xc->cnt[kind], 0u);  // every block of this launch has arrived
      __threadfence_system();
      for (int q = 0; q < a.xc->P && !(a.xc->fault && a.xsession > 0); ++q) {
        __hip_atomic_store(FXFlag(a, q, kind, a.xc->rank), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      FXWaitAll(a, kind, tag);
    }
  }
}

// ---------------------------------------------------------------------------
// tree setup: the root node, the root "round" (one pseudo-expansion whose smaller child
// is the root), the committed-leaf table and the node states.
__device__ __forceinline__ void FInitTree(const FArgs& a) {
  const TreeParams tp = *a.tp;
  const int t = threadIdx.x;
  if (t == 0) {
    FState s;
    s.round = 0;
    s.k = 1;
    s.kx = 1;
    s.total_tiles = 0;
    s.done = 0;
    s.epoch = a.st->epoch + 1u;
    s.num_leaves = 1;
    s.num_splits = 0;
    s.cid_next = 1;
    s.blocked = -1;
    s.spec = 0;
    s.used_rows = s.waste_rows = 0;
    s.forced_next = a.num_forced > 0 ? 0 : -1;
    s.byn = a.bynode != nullptr ? 1 : 0;  // (the root's mask: row 0)
    s.byn_rng = tp.byn_rng;
    s.nsal = 0;
    *a.st = s;
    FNode r;
    r.buf = tp.root_buf;
    r.start = 0;
    r.count = tp.root_count;
    r.gcount = tp.root_gcount;
    r.depth = 0;
    r.parent = -1;
    r.left = -1;
    r.fidx = a.num_forced > 0 ? 0 : -1;
    a.nodes[0] = r;
    FExp x;
    x.parent = -1;
    x.left = -1;
    x.depth = -1;
    x.tile0 = x.ntiles = 0;
    x.src_buf = tp.root_buf;
    x.start = 0;
    x.count = tp.root_count;
    x.dst_buf = 0;
    x.group = x.offset = x.num_bin = x.mfb = x.default_bin = x.missing = x.thr = x.default_left = x.is_cat = 0;
    x.skip = 0;
    x.smaller = 0;
    x.larger = -1;
    x.h_buf = tp.root_buf;
    x.h_start = 0;
    x.h_count = tp.root_count;
    x.forced = -1;
    x.feature = -1;
    x.last = 0;
    x.rescan = 0;
    a.exps[0] = x;
    a.bounds[0] = LeafBounds();
    if (a.cbnd) a.cbnd[0] = LeafBounds();
    if (a.ic) {
      for (int w = 0; w < a.ic_words; ++w) a.ic[w] = ~0ull;
    }
    a.leaf_cid[0] = 0;
    a.lout[0] = 0.0;
  }
  for (int i = t; i < a.C; i += blockDim.x) a.nstate[i] = 0;
  for (int f = t; f < a.F; f += blockDim.x) a.spl[f] = 1;
}

__global__ __launch_bounds__(256) void k_f_init(FArgs a) { FInitTree(a); }

// The tree setup fused with the root statistics' final fold (one launch less per tree): the
// per-block partials of seq::k_root_sums (sum g, sum h, max|g|, max|h|, sum|g|, sum|h|) folded in
// exactly k_root_final's order -> the root's sums and the fixed-point scale bounds.
constexpr int kRootStatsF = 6;
__device__ __forceinline__ double FRootFold(int i, double x, double y) { return i == 2 || i == 3 ? fmax(x, y) : x + y; }
__global__ __launch_bounds__(256) void k_f_init_root(FArgs a, const double* __restrict__ root_part, int nblocks,
                                                     unsigned* __restrict__ ghmax) {
  __shared__ double sh[kRootStatsF][256 / 64];
  double v[kRootStatsF] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
    for (int j = 0; j < kRootStatsF; ++j) v[j] = FRootFold(j, v[j], root_part[kRootStatsF * b + j]);
  }
  FInitTree(a);
#pragma unroll
  for (int j = 0; j < kRootStatsF; ++j) {
    if (j == 2 || j == 3) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v[j] = fmax(v[j], __shfl_xor(v[j], o, kWave));
    } else {
      v[j] = WaveSum(v[j]);
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int j = 0; j < kRootStatsF; ++j) sh[j][w] = v[j];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < static_cast<int>(blockDim.x / 64); ++i) {
#pragma unroll
      for (int j = 0; j < kRootStatsF; ++j) v[j] = FRootFold(j, v[j], sh[j][i]);
    }
    a.lsum[0] = make_double2(v[0], v[1]);
    ghmax[0] = __float_as_uint(static_cast<float>(v[2]));
    ghmax[1] = __float_as_uint(static_cast<float>(v[3]));
    // (the fp64 sums of |value| are exact to ~1e-9 relative: a 2^-20 margin, rounded up)
    ghmax[2] = __float_as_uint(__double2float_ru(v[4] * (1.0 + 0x1p-20)));
    ghmax[3] = __float_as_uint(__double2float_ru(v[5] * (1.0 + 0x1p-20)));
  }
}

// ---------------------------------------------------------------------------
// k_f_hist: histograms of every expansion's smaller child.
//
// The round's smaller-child rows are cut into chunks of >= hist_min_rows rows, at most
// ~hist_grid chunks in all; block (b, tile) builds the histogram of its chunk for the LDS
// tile's feature groups and flushes it into the expansion's accumulator with 64-bit
// integer atomics at the tree's global scale. LDS accumulation:
//   MODE 0  one ds_add_u64 per (row, group): signed g in the high 32 bits, signed h in the
//           low 32 bits, at a per-block power-of-two scale (2^30 / (block rows * max));
//           the flush shifts each block sum up to the global scale (an exact shift);
//   MODE 1  (gpu_use_dp) two ds_add_u64 per (row, group) at the global scale itself.
//   MODE 2  (use_quantized_grad) the row's int8 g / uint8 h levels (2 bytes per row instead
//           of 8) packed g32|h32 into one ds_add_u64; integer sums need no scale, and the
//           flush adds each bin as ONE packed 64-bit word when the whole expansion's sums
//           fit 32 bits (qpack: root rows x max level < 2^31), halving the global atomics.
//           Reference: cuda_histogram_constructor.cu:251-450 (int16 / int32 packed bins).
//   MODE 3  MODE 2 with 32-bit LDS atomics: g16|h16 packed into one ds_add_u32 per (row,
//           group); the block walks its rows in sub-chunks small enough that no 16-bit
//           field can overflow (a.qsub rows) and folds the narrow bins into the 64-bit
//           LDS histogram after each one.
// Zero bins are skipped by the flush (most of a small leaf's histogram).
// Bank-interleaved LDS layout (il_gp > 0, MODE 0 / 2): bin b of the tile's local group g at slot
// b * il_gp + g (il_gp = group count rounded up to 16), so a ds_add_u64 of group g always hits
// bank pair g mod 16 whatever the bin. A lane adds its dword's groups in an order rotated by its
// row (row r starts at group r mod per): the 16 lanes of a bank group (two or three rows of the
// dword-per-lane mapping) then hit different bank pairs, instead of colliding on random bins
// ~3-4 ways (the row phase of a histogram is bound by these conflicts).
// the first pipeline chunk's row indices of this thread (FHistRows' load_rows of its first chunk),
// issued by k_f_hist before it zeroes its LDS histogram so the index round trip overlaps that
constexpr int kFHistR2 = LGAP_FHIST_R / 2;
__device__ __forceinline__ void FHistFirstRows(const FArgs& a, const HistTile& tile, int buf, int start, int rb, int re,
                                               int* rn) {
  const int tpr = tile.d1 - tile.d0;
  const int rpi = blockDim.x / tpr;
  const int myr = threadIdx.x / tpr;
  const int* idx = buf < 0 ? nullptr : a.idx[buf] + start;
  const int base = buf < 0 ? start : 0;
#pragma unroll
  for (int j = 0; j < kFHistR2; ++j) {
    const int p = rb + myr + j * rpi;
    rn[j] = myr < rpi && p < re ? (idx ? idx[p] : base + p) : -1;
  }
}

template <int W, int MODE>
__device__ __forceinline__ void FHistRows(const FArgs& a, const HistTile& tile, int buf, int start, int rb, int re,
                                          const int* gst, unsigned long long* hist, float sg, float sh, double dsg,
                                          double dsh, uint32_t* hist32 = nullptr, int il_gp = 0,
                                          const int* first_rows = nullptr) {
  const int tpr = tile.d1 - tile.d0;
  const int rpi = blockDim.x / tpr;
  const int myr = threadIdx.x / tpr;
  const int myd = threadIdx.x - myr * tpr;
  if (myr >= rpi) return;
  constexpr int per = W == 0 ? 8 : 4 / W;  // W = 0: 4-bit rows (8 groups per dword)
  constexpr int R = LGAP_FHIST_R;
  const int dw = tile.d0 + myd;
  const int gfirst = dw * per;
  // per k (the k-th add of a row): the group's LDS base (interleaved: its local index) and its
  // bit shift in the dword, rotated by the row when interleaved
  int go[per], gsh[per];
  const int rot = (MODE == 0 || MODE == 2) && il_gp > 0 ? (myr & (per - 1)) : 0;
#pragma unroll
  for (int kk = 0; kk < per; ++kk) {
    int gv = -1, sv = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
      if (k == ((kk + rot) & (per - 1))) {
        const int gl = gfirst + k - tile.g0;
        gv = gfirst + k < tile.g1 ? (il_gp > 0 ? gl : gst[gl]) : -1;
        sv = (W == 0 ? 4 : W == 1 ? 8 : 16) * k;
      }
    }
    go[kk] = gv;
    gsh[kk] = sv;
  }
  const float2* gh = a.gh + static_cast<size_t>(a.tp->cls) * a.N;
  const uint16_t* ghq = MODE >= 2 ? a.ghq + static_cast<size_t>(a.tp->cls) * a.N : nullptr;
  const int* idx = buf < 0 ? nullptr : a.idx[buf] + start;
  const int base = buf < 0 ? start : 0;
  // Two-stage software pipeline over chunks of R/2 rows per thread: while chunk i's LDS adds run,
  // chunk i+1's row words / gradients and chunk i+2's row indices are already in flight (the
  // waves of a block otherwise wait on their index -> row round trips in step with each other).
  // Rows past the range load nothing (row -1: word 0, no add).
  constexpr int R2 = R / 2;
  static_assert(R2 == kFHistR2, "first-chunk prefetch width");
  const int step = rpi * R2;
  auto load_rows = [&](int p0, int* rows) {
#pragma unroll
    for (int j = 0; j < R2; ++j) {
      const int p = p0 + j * rpi;
      rows[j] = p < re ? (idx ? idx[p] : base + p) : -1;
    }
  };
  auto load_data = [&](const int* rows, uint32_t* word, float2* v, uint32_t* q) {
#pragma unroll
    for (int j = 0; j < R2; ++j) {
      word[j] = rows[j] >= 0 ? a.rowbins[static_cast<size_t>(rows[j]) * a.stride_dw + dw] : 0u;
      if (MODE >= 2) q[j] = rows[j] >= 0 ? ghq[rows[j]] : 0u;
      else v[j] = rows[j] >= 0 ? gh[rows[j]] : make_float2(0.f, 0.f);
    }
  };
  int rn[R2];
  uint32_t word[R2], q[R2];
  float2 v[R2];
  if (first_rows != nullptr) {
#pragma unroll
    for (int j = 0; j < R2; ++j) rn[j] = first_rows[j];
  } else {
    load_rows(rb + myr, rn);
  }
  load_data(rn, word, v, q);
  load_rows(rb + myr + step, rn);
  for (int p0 = rb + myr; p0 < re; p0 += step) {
    uint32_t wn[R2], qn[R2];
    float2 vn[R2];
    load_data(rn, wn, vn, qn);
    load_rows(p0 + 2 * step, rn);
#pragma unroll
    for (int j = 0; j < R2; ++j) {
      unsigned long long pg = 0ull, ph = 0ull;
      uint32_t p32 = 0u;
      if (MODE == 3) {
        p32 = (static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(q[j] >> 8))) << 16) + (q[j] & 0xFFu);
      } else if (MODE == 2) {
        const long long ig = static_cast<int8_t>(q[j] >> 8);
        pg = (static_cast<unsigned long long>(ig) << 32) + (q[j] & 0xFFu);
      } else if (MODE == 0) {
        const long long ig = __float2int_rn(v[j].x * sg);
        const long long ih = __float2int_rn(v[j].y * sh);
        pg = (static_cast<unsigned long long>(ig) << 32) + static_cast<unsigned long long>(ih);
      } else {
        pg = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v[j].x) * dsg));
        ph = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v[j].y) * dsh));
      }
#pragma unroll
      for (int k = 0; k < per; ++k) {
        const uint32_t b = (word[j] >> gsh[k]) & (W == 0 ? 0xFu : W == 1 ? 0xFFu : 0xFFFFu);
        if (b != 0u && go[k] >= 0) {
          const int o = il_gp > 0 ? static_cast<int>(b) * il_gp + go[k] : go[k] + static_cast<int>(b);
          if (MODE == 3) {
            atomicAdd(&hist32[o], p32);
          } else if (MODE != 1) {
            atomicAdd(&hist[o], pg);
          } else {
            atomicAdd(&hist[2 * o], pg);
            atomicAdd(&hist[2 * o + 1], ph);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < R2; ++j) {
      word[j] = wn[j];
      q[j] = qn[j];
      v[j] = vn[j];
    }
  }
}

// Row chunking of a round's histograms (wave 0, lane = expansion; identical in k_f_hist, which
// assigns the chunks to blocks, and k_f_reduce, which sums each expansion's blocks): chunk rows c
// for the whole round, nb chunks of expansion `lane` in blocks [inc - nb, inc).
// sum over e of ceil(cnt_e / c) <= total / c + ke <= hist_grid while ke <= hist_grid / 2: with
// hist_grid below the CU count every working block gets a CU of its own (256 + k blocks doubled
// some CUs' work and the round waited on them: A/B at 10M, 330 it/s vs 363 it/s). Many expansions
// over a small grid (wide data, many LDS tiles) still get >= hist_grid / 2 row-balanced chunks.
// (the record fields are loaded by FHistChunkLoad before the round state is known: one round of
// independent loads, then FHistChunks masks them by the round's expansion count)
struct FChunkSrc {
  int cnt, buf, start;
};
__device__ __forceinline__ FChunkSrc FHistChunkLoad(const FArgs& a) {
  FChunkSrc c{0, -1, 0};
  const int t = threadIdx.x;
  if (t < kFrontierKmax) {
    const FExp& x = a.exps[t];
    c.cnt = x.skip ? 0 : x.h_count;
    c.buf = x.h_buf;
    c.start = x.h_start;
  }
  return c;
}
__device__ __forceinline__ void FHistChunks(const FArgs& a, int k, const FChunkSrc& src, int* cnt, int* nb, int* inc) {
  const int t = threadIdx.x;
  *cnt = t < k && t >= a.e_lo && t < a.e_hi ? src.cnt : 0;
  const int total = WaveSum(*cnt);
  const int ke = WaveSum(*cnt > 0 ? 1 : 0);
  const int slots = max(max(1, a.hist_grid / 2), a.hist_grid - ke);
  const int c = max(a.hist_min_rows, (total + slots - 1) / slots);
  *nb = (*cnt + c - 1) / c;
  *inc = WaveInclusiveScan(*nb);
}

template <int W, int MODE, int THREADS>
__global__ __launch_bounds__(THREADS) void k_f_hist(FArgs a) {
  extern __shared__ __align__(8) unsigned char lds_raw[];
  __shared__ int s_e, s_rb, s_re, s_buf, s_start;
  const FState* sp = a.st;
  const int t = threadIdx.x;
  // one round of independent loads before the first wait: the round state, every expansion's
  // chunking fields, the tile, the first group starts, the fixed-point scale inputs
  const FChunkSrc csrc = FHistChunkLoad(a);
  const HistTile tile = a.tiles[blockIdx.y];
  const int ng0 = tile.g1 - tile.g0;
  const int gst0 = t < ng0 ? a.gstart[tile.g0 + t] : 0;
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  if (sp->done) return;
  const int k = sp->k;
  const int rnd = sp->round;
  FStamp(a, rnd, kFStampHist, 0);
  if (t < 64) {
    int cnt, nb, inc;
    FHistChunks(a, k, csrc, &cnt, &nb, &inc);
    const int bx = static_cast<int>(blockIdx.x);
    const bool mine = nb > 0 && bx >= inc - nb && bx < inc;
    const unsigned long long m = __ballot(mine);
    if (mine) {
      const int j = bx - (inc - nb);
      const int chunk = (cnt + nb - 1) / nb;
      s_e = t;
      s_rb = j * chunk;
      s_re = min(cnt, (j + 1) * chunk);
      s_buf = csrc.buf;
      s_start = csrc.start;
    }
    if (t == 0 && m == 0ull) s_e = -1;
  }
  __syncthreads();
  const int e = s_e;
  if (e < 0) return;
  FStampMax(a, rnd, kFStampHist, 4);  // (latest start of a working block)
  const int rb = s_rb, re = s_re, buf = s_buf, start = s_start;
  // accumulator words per bin: 1 when quantized level sums are packed g32|h32 (qpack: the
  // expansion's rows are compact, so a data-parallel all-reduce moves half the bytes), else 2
  const int pw = a.quant && a.qpack ? 1 : 2;
  const double dsg = ldexp(1.0, EG), dsh = ldexp(1.0, EH);
  if (a.ltot != nullptr && blockIdx.y == 0) {
    // voting: the smaller child's LOCAL (sum g, sum h) at the global fixed-point scale (integer
    // levels when quantized), exact and order free; the first tile's blocks count each row once
    __shared__ unsigned long long s_tot[2];
    if (t < 2) s_tot[t] = 0ull;
    __syncthreads();
    long long sg = 0, sh = 0;
    for (int p = rb + t; p < re; p += blockDim.x) {
      const int row = FRowAt(a, buf, start + p);
      if (a.quant) {
        const uint32_t qv = a.ghq[static_cast<size_t>(a.tp->cls) * a.N + row];
        sg += static_cast<int8_t>(qv >> 8);
        sh += static_cast<long long>(qv & 0xFFu);
      } else {
        const float2 v = a.gh[static_cast<size_t>(a.tp->cls) * a.N + row];
        sg += __double2ll_rn(static_cast<double>(v.x) * dsg);
        sh += __double2ll_rn(static_cast<double>(v.y) * dsh);
      }
    }
    if (sg) atomicAdd(&s_tot[0], static_cast<unsigned long long>(sg));
    if (sh) atomicAdd(&s_tot[1], static_cast<unsigned long long>(sh));
    __syncthreads();
    if (t < 2 && s_tot[t]) atomicAdd(&a.ltot[2 * e + t], s_tot[t]);
  }
  if (tile.direct) {
    // groups too wide for LDS: each row's fixed-point value straight into the accumulator
    if (a.own && e >= a.xkb) return;  // (never: the round's bound covers its expansions)
    // (xGMI: every add lands in the owner's receive chunk; k_f_reduce, next on the stream,
    // signals the round once all of this launch's adds are visible)
    int* gst = reinterpret_cast<int*>(lds_raw);
    for (int g = t; g < ng0; g += blockDim.x) gst[g] = g == t ? gst0 : a.gstart[tile.g0 + g];
    __syncthreads();
    const int tpr = tile.d1 - tile.d0;
    const int rpi = blockDim.x / tpr;
    const int myr = t / tpr, myd = t - myr * tpr;
    if (myr >= rpi) return;
    constexpr int per = W == 0 ? 8 : 4 / W;
    const int dw = tile.d0 + myd;
    const float2* gh = a.gh + static_cast<size_t>(a.tp->cls) * a.N;
    for (int p = rb + myr; p < re; p += rpi) {
      const int row = FRowAt(a, buf, start + p);
      const uint32_t word = a.rowbins[static_cast<size_t>(row) * a.stride_dw + dw];
      unsigned long long qg, qh;
      if (MODE >= 2) {
        const uint32_t qv = a.ghq[static_cast<size_t>(a.tp->cls) * a.N + row];
        qg = static_cast<unsigned long long>(static_cast<long long>(static_cast<int8_t>(qv >> 8)));
        qh = qv & 0xFFu;
        if (a.qpack) qg = (qg << 32) + qh, qh = 0ull;
      } else {
        const float2 v = gh[row];
        qg = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v.x) * dsg));
        qh = static_cast<unsigned long long>(__double2ll_rn(static_cast<double>(v.y) * dsh));
      }
#pragma unroll
      for (int kk = 0; kk < per; ++kk) {
        const uint32_t b = W == 0   ? ((word >> (4 * kk)) & 0xFu)
                           : W == 1 ? ((word >> (8 * kk)) & 0xFFu)
                                    : ((word >> (16 * kk)) & 0xFFFFu);
        const int g = dw * per + kk;
        if (b != 0u && g < tile.g1) {
          unsigned long long* o = FAccPtr(a, e, gst[g - tile.g0] + static_cast<int>(b), pw);
          if (a.xg && a.own) {
            if (qg) FXAdd(o, qg);
            if (qh) FXAdd(o + 1, qh);
          } else {
            if (qg) atomicAdd(o, qg);
            if (qh) atomicAdd(o + 1, qh);
          }
        }
      }
    }
    if (a.xg && a.own) __builtin_amdgcn_s_waitcnt(0);  // (adds acknowledged before the launch ends)
    return;
  }
  // block scale: 2^30 / min(block rows * max, this rank's sum of |value| over all its rows)
  const double rows_in_block = static_cast<double>(re - rb > 0 ? re - rb : 1);
  constexpr double k30 = 1073741824.0;
  const float sbg = a.sum_bound ? __uint_as_float(a.ghmax[2]) : INFINITY;
  const float sbh = a.sum_bound ? __uint_as_float(a.ghmax[3]) : INFINITY;
  const int bg = FixedPointExp(k30, rows_in_block, __uint_as_float(a.ghmax[0]), sbg);
  const int bh = FixedPointExp(k30, rows_in_block, __uint_as_float(a.ghmax[1]), sbh);
  const float sg = ldexpf(1.f, bg), sh = ldexpf(1.f, bh);
  // bank-interleaved slots (FHistRows): tile.pad = the tile's largest group bin count, 0 = off
  const int ng = tile.g1 - tile.g0;
  // (only over contiguous rows -- the root without a bag -- where the adds, not the row gathers,
  // bound the pass: A/B at 10M, root round 184 -> 161 us; deeper rounds lose on the flush, whose
  // per-group reads of interleaved slots conflict)
  const int il_gp = (MODE == 0 || MODE == 2) && a.hist_il && tile.pad > 0 && (buf < 0 || a.hist_il > 1) ? ((ng + 15) & ~15) : 0;
  const int words = il_gp > 0 ? tile.pad * il_gp : (MODE != 1 ? tile.nbins : 2 * tile.nbins);
  unsigned long long* hist = reinterpret_cast<unsigned long long*>(lds_raw);
  uint32_t* hist32 = reinterpret_cast<uint32_t*>(hist + words);
  int* gst = reinterpret_cast<int*>(MODE == 3 ? reinterpret_cast<unsigned long long*>(hist32 + ((tile.nbins + 1) & ~1))
                                              : hist + words);
  // (interleaved: the packed image the partial store reads, after gst)
  unsigned long long* packed = il_gp > 0 ? reinterpret_cast<unsigned long long*>(gst + ((ng + 1) & ~1)) : nullptr;
  int first_rows[kFHistR2];
  if (MODE != 3) FHistFirstRows(a, tile, buf, start, rb, re, first_rows);
  for (int i = t; i < words; i += blockDim.x) hist[i] = 0ull;
  if (MODE == 3) {
    for (int i = t; i < tile.nbins; i += blockDim.x) hist32[i] = 0u;
  }
  for (int g = t; g < ng0; g += blockDim.x) gst[g] = (g == t ? gst0 : a.gstart[tile.g0 + g]) - tile.bin0;
  __syncthreads();
  FStamp(a, rnd, kFStampHist, 1);
  if (MODE == 3) {
    for (int sb = rb; sb < re; sb += a.qsub) {
      const int se = min(re, sb + a.qsub);
      FHistRows<W, MODE>(a, tile, buf, start, sb, se, gst, hist, sg, sh, dsg, dsh, hist32);
      __syncthreads();
      for (int i = t; i < tile.nbins; i += blockDim.x) {
        const uint32_t x = hist32[i];
        if (x == 0u) continue;
        hist32[i] = 0u;
        const uint32_t hs = x & 0xFFFFu;
        const long long gs = static_cast<int32_t>(x - hs) >> 16;
        hist[i] += (static_cast<unsigned long long>(gs) << 32) + hs;
      }
      __syncthreads();
    }
  } else {
    FHistRows<W, MODE>(a, tile, buf, start, rb, re, gst, hist, sg, sh, dsg, dsh, nullptr, il_gp, first_rows);
    __syncthreads();
  }
  if (il_gp > 0) {
    // interleaved slots -> the packed image (conflict-free reads in slot order), so the partial
    // store below writes consecutive bins of a group to consecutive words
    for (int sl = t; sl < words; sl += blockDim.x) {
      const int b = sl / il_gp, gl = sl - b * il_gp;
      if (gl >= ng) continue;
      const int nb = (gl + 1 < ng ? gst[gl + 1] : tile.nbins) - gst[gl];
      if (b < nb) packed[gst[gl] + b] = hist[sl];
    }
    __syncthreads();
  }
  FStamp(a, rnd, kFStampHist, 2);
  FStampMax(a, rnd, kFStampHist, 5);  // (latest block done with its rows)
  // The block's histogram -> its row of the partial slab with plain coalesced stores, raw (block
  // scale for MODE 0, its exponents in hmeta); k_f_reduce sums each expansion's rows at the
  // global scale. (A per-block flush of every bin with 64-bit global atomics executes at the
  // memory side at ~1.3 TB/s of added bytes: at 224 blocks x 7,140 bins x 2 words that was the
  // 13-18 us tail of every histogram launch.)
  const int sw = MODE == 1 ? 2 : 1;  // slab words per bin
  unsigned long long* prow = a.hslab + static_cast<size_t>(blockIdx.x) * a.hslab_stride + static_cast<size_t>(sw) * tile.bin0;
  const unsigned long long* src = il_gp > 0 ? packed : hist;
  for (int j = t; j < sw * tile.nbins; j += blockDim.x) prow[j] = src[j];
  if (MODE == 0 && t == 0) {
    a.hmeta[blockIdx.x] = static_cast<long long>((static_cast<unsigned long long>(static_cast<unsigned>(bh)) << 32) |
                                                 static_cast<unsigned>(bg));  // (every tile's block: the same value)
  }
  FStamp(a, rnd, kFStampHist, 3);
  FStampMax(a, rnd, kFStampHist, 6);  // (latest block done issuing its partial)
  FStampEnd(a, rnd, kFStampHist);
}

// ---------------------------------------------------------------------------
// k_f_reduce: the round's partial histograms (k_f_hist's slab rows) summed per expansion into
// its accumulator at the tree's global fixed-point scale (exact integer sums, order free).
// Work item = (expansion e, LDS tile, 256-bin chunk of the tile, group of kRedRows of e's row
// blocks): one thread per bin issues its kRedRows partial loads together; an expansion whose
// rows span one group stores its sums, more groups add theirs with 64-bit atomics (at most
// ceil(blocks / kRedRows) per bin instead of one per block). Reference counterpart: the
// per-block histogram merge of cuda_histogram_constructor.cu:20-70 (CUDA: block atomics into
// global memory).
constexpr int kRedThreads = 256;
constexpr int kRedRows = 16;
constexpr int kRedMaxTiles = 256;

// XG: the owner-computes xGMI exchange (its own instantiation: the single-GPU reduce compiles none
// of it)
template <int MODE, bool XG>
__global__ __launch_bounds__(kRedThreads) void k_f_reduce(FArgs a) {
  __shared__ int s_nb[kFrontierKmax], s_b0[kFrontierKmax], s_w0[kFrontierKmax + 1];
  __shared__ int s_tc[kRedMaxTiles + 1];  // chunk prefix over the LDS tiles (direct tiles: none)
  __shared__ int s_wc[kRedThreads / 64];
  __shared__ int s_tb0[kRedMaxTiles], s_tnb[kRedMaxTiles];  // tiles' first bin / bin count
  const FState* sp = a.st;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // one round of independent loads: state, expansion chunking fields, this thread's tile
  const FChunkSrc csrc = FHistChunkLoad(a);
  int tch = 0;  // bin chunks of tile t
  if (t < a.num_tiles) {
    const HistTile ty = a.tiles[t];
    tch = ty.direct ? 0 : (ty.nbins + kRedThreads - 1) / kRedThreads;
    // (kept in LDS: a work item's tile record is then no dependent global load of its own --
    // wide data runs many items per block, LambdaRank 5M x 300 ~12, each paying it)
    s_tb0[t] = ty.bin0;
    s_tnb[t] = ty.nbins;
  }
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  const bool xhist = XG && a.xg && a.own;  // (xGMI owner-computes: the histogram exchange ends here)
  const unsigned xep = xhist ? *a.xc->ep : 0u;  // (this round's tag is xep + 1)
  if (sp->done) return;
  const int k = sp->k;
  // chunk prefix over the tiles (block scan; num_tiles <= kRedThreads)
  const int tinc = WaveInclusiveScan(tch);
  if (lane == 63) s_wc[wv] = tinc;
  __syncthreads();
  int woff = 0;
  for (int q = 0; q < wv; ++q) woff += s_wc[q];
  if (t < a.num_tiles) s_tc[t] = woff + tinc - tch;
  if (t == 0) {
    int tot = 0;
    for (int q = 0; q < kRedThreads / 64; ++q) tot += s_wc[q];
    s_tc[a.num_tiles] = tot;
  }
  if (t < 64) {
    int cnt, nb, inc;
    FHistChunks(a, k, csrc, &cnt, &nb, &inc);
    if (t < kFrontierKmax) {
      s_nb[t] = nb;
      s_b0[t] = inc - nb;
    }
    // work items per expansion: bin chunks x row groups (prefix over the expansions)
    const int nch = s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3];
    const int items = ((nb + kRedRows - 1) / kRedRows) * nch;
    const int winc = WaveInclusiveScan(items);
    if (t < kFrontierKmax) s_w0[t + 1] = winc;
    if (t == 0) s_w0[0] = 0;
  }
  __syncthreads();
  const int nch = s_tc[a.num_tiles];
  const int W = nch > 0 ? s_w0[k] : 0;
  if (W == 0 && !xhist) return;  // (xGMI: a rank with no rows this round still signals it)
  // xGMI with several ranks: every rank adds into the owner's chunk, so no plain first store
  const bool shared_out = xhist && a.xc->P > 1;
  const int pw = a.quant && a.qpack ? 1 : 2;  // accumulator words per bin (see k_f_hist)
  constexpr int sw = MODE == 1 ? 2 : 1;       // slab words per bin
  for (int w = blockIdx.x; w < W; w += gridDim.x) {
    int e = 0;
    while (e + 1 < k && s_w0[e + 1] <= w) ++e;
    if (a.own && e >= a.xkb) continue;  // (never: the round's bound covers its expansions)
    const int r = w - s_w0[e];
    const int grp = r / nch, ch = r - grp * nch;
    int y = 0;
    while (y + 1 < a.num_tiles && s_tc[y + 1] <= ch) ++y;
    const int tbin0 = s_tb0[y];
    const int i = (ch - s_tc[y]) * kRedThreads + t;  // bin of the tile
    if (i >= s_tnb[y]) continue;
    const int nb = s_nb[e];
    const int r0 = s_b0[e] + grp * kRedRows, r1 = min(s_b0[e] + nb, r0 + kRedRows);
    const size_t col = static_cast<size_t>(sw) * (tbin0 + i);
    long long g = 0, h = 0;
    unsigned long long x0[kRedRows], x1[kRedRows];
#pragma unroll
    for (int j = 0; j < kRedRows; ++j) {
      const int row = r0 + j;
      x0[j] = row < r1 ? a.hslab[static_cast<size_t>(row) * a.hslab_stride + col] : 0ull;
      x1[j] = MODE == 1 && row < r1 ? a.hslab[static_cast<size_t>(row) * a.hslab_stride + col + 1] : 0ull;
    }
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < kRedRows; ++j) {
        if (r0 + j >= r1) continue;
        const long long mm = a.hmeta[r0 + j];  // (uniform: scalar loads; bh << 32 | bg)
        const int2 m = make_int2(static_cast<int>(mm & 0xFFFFFFFFll), static_cast<int>(mm >> 32));
        const int hv = static_cast<int>(static_cast<unsigned int>(x0[j] & 0xFFFFFFFFull));
        const long long gv = static_cast<long long>(x0[j] - static_cast<unsigned long long>(static_cast<long long>(hv))) >> 32;
        // exact shift of the block's fixed-point sums to the global scale (2^EG >= 2^bg: see
        // GlobalScaleExp; the guard keeps a degenerate max of 0 harmless)
        g += gv * (1ll << max(0, EG - m.x));
        h += static_cast<long long>(hv) * (1ll << max(0, EH - m.y));
      }
    } else if (MODE == 1) {
#pragma unroll
      for (int j = 0; j < kRedRows; ++j) {
        g += static_cast<long long>(x0[j]);
        h += static_cast<long long>(x1[j]);
      }
    } else if (pw == 1) {
      // packed g32|h32 level sums: the packed words add exactly (qpack bounds every field)
#pragma unroll
      for (int j = 0; j < kRedRows; ++j) g += static_cast<long long>(x0[j]);
    } else {
#pragma unroll
      for (int j = 0; j < kRedRows; ++j) {
        const unsigned long long hv = x0[j] & 0xFFFFFFFFull;
        g += static_cast<long long>(x0[j] - hv) >> 32;
        h += static_cast<long long>(hv);
      }
    }
    unsigned long long* out = XG ? FAccPtr(a, e, tbin0 + i, pw) : a.acc + FAccAt(a, e, tbin0 + i, pw);
    if (xhist) {
      // (xGMI: into the owner's receive chunk at system scope; one rank with one row group stores)
      if (nb <= kRedRows && !shared_out) {
        if (g) __hip_atomic_store(&out[0], static_cast<unsigned long long>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (pw == 2 && h) __hip_atomic_store(&out[1], static_cast<unsigned long long>(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        if (g) FXAdd(&out[0], static_cast<unsigned long long>(g));
        if (pw == 2 && h) FXAdd(&out[1], static_cast<unsigned long long>(h));
      }
    } else if (nb <= kRedRows && !shared_out) {
      // the expansion's only row group: the accumulator is zero here (the scan re-zeroes it)
      if (g) out[0] = static_cast<unsigned long long>(g);
      if (pw == 2 && h) out[1] = static_cast<unsigned long long>(h);
    } else {
      if (g) atomicAdd(&out[0], static_cast<unsigned long long>(g));
      if (pw == 2 && h) atomicAdd(&out[1], static_cast<unsigned long long>(h));
    }
  }
  // xGMI: the round's histogram exchange completes here (the owner's scan runs next)
  // (one rank: no peer to signal or wait for; the kernel boundary orders the chunk for the scan)
  if (xhist && FXPeers(a)) FXArrive(a, kFXHist, FXTag(a, xep + 1u));
}

// ---------------------------------------------------------------------------
// k_f_scan: one workgroup per (expansion, feature), grid-stride.
//  1. accumulator -> the smaller child's histogram (fp64, LDS + its node slot), the
//     accumulator words re-zeroed for the next round; larger = parent - smaller
//  2. most-frequent bins from the leaf sums; wave 0 scans the smaller child, wave 1 the
//     larger one (split_scan.h), both from LDS
//  3. the two candidates -> the round's candidate table [e][sel][f]
// EXT: the voting local pass, extra-trees draws, feature-parallel ownership and the scan-side
// best; the plain instantiation (serial / data-parallel) compiles none of it
template <bool EXT>
__global__ __launch_bounds__(kFScanThreads) void k_f_scan(FArgs a) {
  const bool voting = EXT && a.voting != 0;
  const bool xtrees = EXT && a.xrng != nullptr;
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ int s_skip, s_splp, s_rand[2], s_xn[2];
  __shared__ double s_xh[2];
  __shared__ __align__(8) unsigned char s_out_raw[2 * sizeof(SplitInfo)];
  __shared__ SplitKey s_key[2];
  SplitInfo* s_out = reinterpret_cast<SplitInfo*>(s_out_raw);
  const FState* stp = a.st;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int e0 = a.e_lo, F = a.F;
  // the first item's expansion and feature records load with the round state (one round of
  // independent loads before the first wait; later items load their own)
  // items: (expansion, feature) over every feature, or (owner-computes / feature parallel) over
  // this rank's owned features only (fown_list)
  const int NF = a.fown_list != nullptr ? a.fown_n : F;
  const int e_pre = min(e0 + static_cast<int>(blockIdx.x) / max(NF, 1), kFrontierKmax - 1);
  const int f_pre = a.fown_list != nullptr ? (NF > 0 ? a.fown_list[static_cast<int>(blockIdx.x) % NF] : 0)
                                           : static_cast<int>(blockIdx.x) % F;
  const int pre_skip = a.exps[e_pre].skip, pre_cs = a.exps[e_pre].smaller, pre_cl = a.exps[e_pre].larger,
            pre_p = a.exps[e_pre].parent, pre_rs = EXT ? a.exps[e_pre].rescan : 0;
  const DevFeature fi_pre = a.feat[f_pre];
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  if (stp->done) return;
  const int e1 = min(stp->k, a.e_hi);
  const int total = max(0, e1 - e0) * NF;
  const int rnd = stp->round;
  FStamp(a, rnd, kFStampScan, 0);
  if (!voting && blockIdx.x == 0 && t == 0 && e0 == 0 && pre_p < 0) {
    // the root round: the root's output (whatever features this rank scans: owner-computes and
    // feature-parallel ranks scan only their own; voting: k_f_elect writes the global one)
    const double2 rs = a.lsum[0];
    SplitParams p0 = a.sp;
    p0.path_smooth = 0.0;
    a.lout[0] = LeafOutputRaw(rs.x, rs.y, p0, a.nodes[0].gcount, 0.0);
  }
  if (a.own && !a.xg) {
    // the reduce-scatter consumed the send layout: zero it for the next round's k_f_reduce
    // (xGMI: no send layout; the owner re-zeroes its receive chunk as it reads it, below)
    const size_t nz = static_cast<size_t>(a.own_P) * a.xkb * a.own_w * (a.quant && a.qpack ? 1 : 2);
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nz; i += static_cast<size_t>(gridDim.x) * blockDim.x) {
      a.acc[i] = 0ull;
    }
  }
  double inv_g = ldexp(1.0, -EG), inv_h = ldexp(1.0, -EH);
  if (a.quant) QuantScales(a, &inv_g, &inv_h);
  const bool qpack = a.quant && a.qpack;
  const size_t TB2 = 2 * static_cast<size_t>(a.TB);
  double* hs_full = reinterpret_cast<double*>(smem);
  double* hl_full = hs_full + 2 * a.max_bin;
  int* order = reinterpret_cast<int*>(hl_full + 2 * a.max_bin);
  double* ckey = reinterpret_cast<double*>(order + 2 * a.cat_p2);
  __shared__ int s_last;
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    const int e = e0 + item / NF, fi_ = item - (e - e0) * NF;
    const int f = a.fown_list != nullptr ? a.fown_list[fi_] : fi_;
    const bool first = item == static_cast<int>(blockIdx.x);
    const int x_skip = first ? pre_skip : a.exps[e].skip;
    const int x_cs = first ? pre_cs : a.exps[e].smaller, x_cl = first ? pre_cl : a.exps[e].larger;
    const int x_p = first ? pre_p : a.exps[e].parent;
    // (intermediate monotone: a re-scan of node x_cs from its slot, no accumulator)
    const bool rescan = EXT && (first ? pre_rs : a.exps[e].rescan) != 0;
    if (x_skip) {
      continue;
    }
    const int cs = x_cs, cl = x_cl, p = x_p;
    const DevFeature fi = first ? fi_pre : a.feat[f];
    const int nbin = fi.num_bin;
    const size_t v0 = 2 * static_cast<size_t>(fi.hist_offset);
    const size_t pw = qpack ? 1 : 2;  // accumulator words per bin (see k_f_hist)
    // (owner-computes: this rank's summed chunk of the reduce-scatter)
    unsigned long long* acc =
        a.own ? a.acc_recv + (static_cast<size_t>(e) * a.own_w + (fi.hist_offset - a.own_b0[a.own_rank])) * pw
              : a.acc + static_cast<size_t>(e) * pw * a.TB + pw * static_cast<size_t>(fi.hist_offset);
    const double* gp = (p >= 0 && cl >= 0) ? a.slots + static_cast<size_t>(p) * TB2 + v0 : nullptr;
    double* gs = a.slots + static_cast<size_t>(cs) * TB2 + v0;
    double* gl = cl >= 0 ? a.slots + static_cast<size_t>(cl) * TB2 + v0 : nullptr;
    // leaf statistics the scanning waves use (lane 0 of waves 0 / 1)
    const int my = w == 0 ? cs : (w == 1 ? cl : -1);
    double2 pre_sum = make_double2(0.0, 0.0);
    int pre_n = 0, pre_depth = 0;
    double pre_out = 0.0;
    int pre_fidx = -1;
    LeafBounds pre_bounds;
    if (lane == 0 && my >= 0 && rescan) {
      // host RecomputeBestSplit (reference serial_tree_learner.cpp RecomputeBestSplitForLeaf):
      // the leaf's statistics from its pending best split, parent output 0 unless path smoothing
      const SplitInfo& bi = a.best[my];
      pre_sum = make_double2(bi.left_sum_gradient + bi.right_sum_gradient, bi.left_sum_hessian + bi.right_sum_hessian);
      pre_n = bi.left_count + bi.right_count;
      pre_depth = a.nodes[my].depth;
      SplitParams p0 = a.sp;
      p0.path_smooth = 0.0;
      pre_out = a.sp.path_smooth > kEpsilon ? LeafOutputRaw(pre_sum.x, pre_sum.y, p0, pre_n, 0.0) : 0.0;
      pre_bounds = a.bounds[my];
    } else if (lane == 0 && my >= 0) {
      pre_sum = a.lsum[my];
      pre_n = a.nodes[my].gcount;
      pre_depth = a.nodes[my].depth;
      pre_fidx = a.num_forced > 0 ? a.nodes[my].fidx : -1;
      pre_out = a.lout[my];
      pre_bounds = a.bounds[my];
      if (voting) {
        // voting's LOCAL pass: this rank's rows and sums (the smaller child's from the round's
        // exact local totals, the larger's as the parent's local sums minus them)
        pre_n = a.nodes[my].count;
        const double2 sm = make_double2(static_cast<double>(static_cast<long long>(a.ltot[2 * e])) * inv_g,
                                        static_cast<double>(static_cast<long long>(a.ltot[2 * e + 1])) * inv_h);
        if (my == cs) {
          pre_sum = sm;
        } else {
          const double2 ps = a.lsum_loc[p];
          pre_sum = make_double2(ps.x - sm.x, ps.y - sm.y);
        }
        if (f == 0) a.lsum_loc[my] = pre_sum;
      }
    }
    // Every global load of the item is issued before the first store that needs a wait: thread
    // 0's flags (stored to LDS after the bin loop) and, per bin, the accumulator words and the
    // parent's bins (read before the re-zeroing / slot stores, which the compiler must otherwise
    // assume alias them): one memory round trip instead of three or four.
    int skip_v = 0, splp_v = 1;
    if (t == 0) {
      // (feature parallel: only the features this rank owns)
      skip_v = !a.used_bytree[f] || (EXT && a.fowned != nullptr && !a.fowned[f]);
      splp_v = p >= 0 && !voting ? a.spl[static_cast<size_t>(p) * F + f] : 1;
    }
    for (int kk = t; kk < nbin - 1; kk += blockDim.x) {
      if (rescan) {
        // (the node's stored bins, as its first scan left them)
        const int b = kk < fi.mfb ? kk : kk + 1;
        hs_full[2 * b] = gs[2 * kk];
        hs_full[2 * b + 1] = gs[2 * kk + 1];
        continue;
      }
      const bool sys = EXT && a.xg && a.own;  // (the receive chunk the ranks pushed into)
      const unsigned long long x0 = sys ? FXLoad64(acc + pw * kk) : acc[pw * kk];
      const unsigned long long x1 = qpack ? 0ull : (sys ? FXLoad64(acc + 2 * kk + 1) : acc[2 * kk + 1]);
      const double gp0 = gl ? gp[2 * kk] : 0.0, gp1 = gl ? gp[2 * kk + 1] : 0.0;
      if (sys) {
        FXStore64(acc + pw * kk, 0ull);
        if (!qpack) FXStore64(acc + 2 * kk + 1, 0ull);
      } else {
        acc[pw * kk] = 0ull;
        if (!qpack) acc[2 * kk + 1] = 0ull;
      }
      long long q0 = static_cast<long long>(x0), q1 = static_cast<long long>(x1);
      if (qpack) {
        // packed g32|h32, one word per bin
        const unsigned long long hs = x0 & 0xFFFFFFFFull;
        q0 = static_cast<long long>(x0 - hs) >> 32;
        q1 = static_cast<long long>(hs);
      }
      const double sv0 = static_cast<double>(q0) * inv_g, sv1 = static_cast<double>(q1) * inv_h;
      const int b = kk < fi.mfb ? kk : kk + 1;
      hs_full[2 * b] = sv0;
      hs_full[2 * b + 1] = sv1;
      gs[2 * kk] = sv0;
      gs[2 * kk + 1] = sv1;
      if (gl) {
        const double l0 = gp0 - sv0, l1 = gp1 - sv1;
        hl_full[2 * b] = l0;
        hl_full[2 * b + 1] = l1;
        gl[2 * kk] = l0;
        gl[2 * kk + 1] = l1;
      }
    }
    if (t == 0) {
      s_skip = skip_v;
      s_splp = splp_v;
    }
    if (t < 2) {
      s_out[t].Reset();
      SplitKey kz;
      kz.gain = kMinScore;
      kz.feature = -1;
      kz.threshold = 0;
      kz.group = kz.offset = kz.num_bin = kz.mfb = kz.default_bin = 0;
      kz.missing = kz.default_left = kz.is_cat = kz.pad0 = 0;
      kz.pos = f;
      kz.pad2 = 0;
      s_key[t] = kz;
    }
    __syncthreads();
    if (item == static_cast<int>(blockIdx.x)) FStamp(a, rnd, kFStampScan, 1);  // (loads + histograms in LDS)
    const bool skip_both = s_skip || !s_splp;
    // most-frequent bin = leaf total - stored bins
    if (w < 2 && my >= 0) {
      double* H = w == 0 ? hs_full : hl_full;
      double sgs = 0.0, shs = 0.0;
      for (int b = lane; b < nbin; b += 64) {
        if (b == fi.mfb) continue;
        sgs += H[2 * b];
        shs += H[2 * b + 1];
      }
      sgs = WaveSum(sgs);
      shs = WaveSum(shs);
      if (lane == 0) {
        H[2 * fi.mfb] = pre_sum.x - sgs;
        H[2 * fi.mfb + 1] = pre_sum.y - shs;
        s_xn[w] = pre_n;
        s_xh[w] = pre_sum.y;
      }
    }
    __syncthreads();
    if (xtrees && t == 0) {
      // extra-trees thresholds, drawn in the host learner's order: the smaller child, then the
      // larger one (one expansion per round here: no other item advances this feature's stream)
      s_rand[0] = s_rand[1] = 0;
      if (!skip_both) {
        for (int sel = 0; sel < 2; ++sel) {
          if ((sel == 0 ? cs : cl) < 0) continue;
          unsigned* r = &a.xrng[f];
          if (fi.bin_type == 0) {
            if (fi.num_bin - 2 > 0) s_rand[sel] = RandNextInt(r, 0, fi.num_bin - 2);
          } else if (fi.num_bin <= a.sp.max_cat_to_onehot) {
            if (fi.num_bin - 1 > 0) s_rand[sel] = RandNextInt(r, 1, fi.num_bin);
          } else {
            const double* H = sel == 0 ? hs_full : hl_full;
            const double cf = s_xn[sel] / (s_xh[sel] + 2 * kEpsilon);
            int used = 0;
            for (int b = 1; b < fi.num_bin; ++b) used += RoundCount(H[2 * b + 1] * cf) >= a.sp.cat_smooth;
            const int max_num_cat = min(a.sp.max_cat_threshold, (used + 1) / 2);
            const int max_thr = max(min(max_num_cat, used) - 1, 0);
            if (max_thr > 0) s_rand[sel] = RandNextInt(r, 0, max_thr);
          }
        }
      }
    }
    if (xtrees) __syncthreads();
    if (w < 2 && my >= 0) {
      SplitInfo* out = &s_out[w];
      const double sg = __shfl(pre_sum.x, 0, kWave), sh = __shfl(pre_sum.y, 0, kWave);
      const int n = __shfl(pre_n, 0, kWave);
      const int depth = __shfl(pre_depth, 0, kWave);
      const SplitParams spp = voting ? *a.sp_local : a.sp;
      if (!skip_both) {
        const double* H = w ? hl_full : hs_full;
        double po;
        if (p < 0) {
          SplitParams p0 = spp;
          p0.path_smooth = 0.0;
          po = LeafOutputRaw(sg, sh, p0, n, 0.0);
        } else {
          po = __shfl(pre_out, 0, kWave);
        }
        LeafBounds bounds;
        bounds.min = __shfl(pre_bounds.min, 0, kWave);
        bounds.max = __shfl(pre_bounds.max, 0, kWave);
        bool spl;
        const int rt = xtrees ? s_rand[w] : 0;
        if (fi.bin_type == 0) {
          spl = ScanNumericalWave(spp, fi, H, sg, sh, n, po, bounds, rt, out);
        } else {
          FeatureScanMeta m;
          m.num_bin = fi.num_bin;
          m.default_bin = static_cast<uint32_t>(fi.default_bin);
          m.missing_type = fi.missing;
          m.bin_type = fi.bin_type;
          m.monotone = fi.monotone;
          m.penalty = fi.penalty;
          m.rand_threshold = rt;
          if (lane == 0) out->Reset();
          spl = ScanCategoricalWave(spp, m, H, sg, sh, n, po, bounds, a.cat_p2, order + w * a.cat_p2,
                                    ckey + w * a.cat_p2, out);
        }
        if (lane == 0) {
          if (!rescan) a.spl[static_cast<size_t>(my) * F + f] = spl ? 1 : 0;  // (a re-scan keeps the flags)
          // (children of forced splits are scanned past max_depth: no regular split there)
          if (!spl || (a.max_depth > 0 && depth >= a.max_depth)) {
            out->Reset();
          } else {
            out->feature = f;
            // cost-effective gradient boosting, split penalty (host CegbPenalty::DeltaGain:
            // subtracted before the monotone penalty multiplies the gain). With coupled
            // penalties the candidate stays raw: the select applies every penalty (CegbAdjust)
            // (voting's local pass ranks raw gains: penalties belong to the global pass)
            if (!a.cegb_raw && !voting) {
              if (a.cegb_split > 0.0) out->gain -= a.cegb_split * n;
              if (out->monotone_type != 0) out->gain *= MonotonePenaltyAt(a.monotone_penalty, depth);
            }
            if (a.ic && !voting && !FIcAllows(a, my, f)) out->Reset();
          }
        }
      } else if (lane == 0 && !rescan) {
        // feature not tried: the children inherit the parent's flag
        a.spl[static_cast<size_t>(my) * F + f] = static_cast<uint8_t>(s_splp);
      }
      if (lane == 0 && pre_fidx >= 0 && a.forced[pre_fidx].feature == f) {
        // the node's forced split at its threshold (host ForceSplits / reference
        // GatherInfoForThresholdNumerical: bins above the threshold go right, skipping the
        // zero bin (MissingType::Zero) and the NaN bin; missing values go left)
        const double pof = p < 0 ? LeafOutputRaw(sg, sh, [&] { SplitParams q = a.sp; q.path_smooth = 0.0; return q; }(), n, 0.0)
                                 : pre_out;
        const double* H = w ? hl_full : hs_full;
        const int thr = a.forced[pre_fidx].threshold;
        const bool na = fi.missing == 2, zero = fi.missing == 1;
        const double cf = static_cast<double>(n) / sh;
        double rg = 0.0, rh = 0.0;
        int rc = 0;
        for (int b = nbin - 1 - (na ? 1 : 0); b >= 1; --b) {
          if (b <= thr) break;
          if (zero && b == fi.default_bin) continue;
          rg += H[2 * b];
          rh += H[2 * b + 1];
          rc += RoundCount(H[2 * b + 1] * cf);
        }
        const double lg = sg - rg, lh = sh - rh;
        const int lc = n - rc;
        SplitInfo fin;
        fin.Reset();
        fin.feature = f;
        fin.threshold = static_cast<uint32_t>(thr);
        fin.default_left = 1;
        fin.left_sum_gradient = lg;
        fin.left_sum_hessian = lh;
        fin.right_sum_gradient = rg;
        fin.right_sum_hessian = rh;
        fin.left_count = lc;
        fin.right_count = rc;
        fin.left_output = LeafOutputRaw(lg, lh, a.sp, lc, pof);
        fin.right_output = LeafOutputRaw(rg, rh, a.sp, rc, pof);
        fin.gain = SplitGain(lg, lh, rg, rh, a.sp, 0, lc, rc, pof, LeafBounds()) - LeafGain(sg, sh, a.sp, n, pof) -
                   a.sp.min_gain_to_split;
        a.fbest[my] = fin;
        SplitKey fk;
        fk.gain = fin.gain;
        fk.feature = f;
        fk.threshold = static_cast<uint32_t>(thr);
        fk.group = fi.group;
        fk.offset = fi.offset;
        fk.num_bin = fi.num_bin;
        fk.mfb = fi.mfb;
        fk.default_bin = fi.default_bin;
        fk.missing = fi.missing;
        fk.default_left = 1;
        fk.is_cat = 0;
        fk.pad0 = 0;
        fk.pos = f;
        fk.pad2 = 0;
        a.fkey[my] = fk;
      }
      if (lane == 0) {
        SplitKey& kk = s_key[w];
        kk.feature = out->feature;
        kk.gain = SafeGain(*out);
        kk.threshold = out->threshold;
        kk.group = fi.group;
        kk.offset = fi.offset;
        kk.num_bin = fi.num_bin;
        kk.mfb = fi.mfb;
        kk.default_bin = fi.default_bin;
        kk.missing = fi.missing;
        kk.default_left = out->default_left;
        kk.is_cat = fi.bin_type != 0 ? 1 : 0;
        kk.pad0 = a.cegb_raw && out->feature >= 0 ? out->monotone_type : 0;
      }
    }
    __syncthreads();
    if (item == static_cast<int>(blockIdx.x)) FStamp(a, rnd, kFStampScan, 2);  // (scans done)
    // publish the candidates (dword-parallel copies of the LDS records)
    constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
    constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
    const int nsel = cl >= 0 ? 2 : 1;
    for (int i = t; i < nsel * (kKeyWords + kInfoWords); i += blockDim.x) {
      const int sel = i / (kKeyWords + kInfoWords);
      const int o = i - sel * (kKeyWords + kInfoWords);
      const size_t q = (static_cast<size_t>(e) * 2 + sel) * F + f;
      if (o < kKeyWords) {
        reinterpret_cast<uint32_t*>(a.ckey + q)[o] = reinterpret_cast<const uint32_t*>(&s_key[sel])[o];
      } else {
        reinterpret_cast<uint32_t*>(a.cinfo + q)[o - kKeyWords] = reinterpret_cast<const uint32_t*>(&s_out[sel])[o - kKeyWords];
      }
    }
    __syncthreads();  // LDS reused by the next item
    if (item == static_cast<int>(blockIdx.x)) FStamp(a, rnd, kFStampScan, 3);
  }
  FStampEnd(a, rnd, kFStampScan);
}

// ---------------------------------------------------------------------------
// k_f_scan_w: k_f_scan with ONE WAVE per (expansion, feature) item, the smaller child scanned
// before the larger one by the same wave. For wide data a round holds thousands of items and
// the block kernel (two of its four waves scanning, 183 VGPRs: two resident blocks per CU)
// is bound by how many items run at once; here four items share a block and nothing waits
// on a block barrier. The same records as k_f_scan's plain instantiation for numerical
// features without forced splits (LaunchFrontierScan routes everything else to k_f_scan).
__device__ __forceinline__ void FWaveSync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__global__ __launch_bounds__(kFScanWaves * 64) void k_f_scan_w(FArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ __align__(8) unsigned char s_out_raw[kFScanWaves * sizeof(SplitInfo)];
  __shared__ SplitKey s_key[kFScanWaves];
  const FState* stp = a.st;
  if (stp->done) return;
  const int e0 = a.e_lo, e1 = min(stp->k, a.e_hi), F = a.F;
  const int total = max(0, e1 - e0) * F;
  const int rnd = stp->round;
  FStamp(a, rnd, kFStampScan, 0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  double inv_g = ldexp(1.0, -EG), inv_h = ldexp(1.0, -EH);
  if (a.quant) QuantScales(a, &inv_g, &inv_h);
  const bool qpack = a.quant && a.qpack;
  const size_t TB2 = 2 * static_cast<size_t>(a.TB);
  double* hs_full = reinterpret_cast<double*>(smem + w * FrontierScanWaveBytes(a.max_bin, a.cat_p2));
  double* hl_full = hs_full + 2 * a.max_bin;
  SplitInfo* out = reinterpret_cast<SplitInfo*>(s_out_raw) + w;
  SplitKey* key = &s_key[w];
  constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  for (int item = static_cast<int>(blockIdx.x) * kFScanWaves + w; item < total;
       item += static_cast<int>(gridDim.x) * kFScanWaves) {
    const int e = e0 + item / F, f = item - (e - e0) * F;
    const FExp& xr = a.exps[e];
    if (xr.skip) continue;
    const int cs = xr.smaller, cl = xr.larger, p = xr.parent;
    const DevFeature fi = a.feat[f];
    const int nbin = fi.num_bin;
    const size_t v0 = 2 * static_cast<size_t>(fi.hist_offset);
    const size_t pw = qpack ? 1 : 2;
    unsigned long long* acc = a.acc + static_cast<size_t>(e) * pw * a.TB + pw * static_cast<size_t>(fi.hist_offset);
    const double* gp = (p >= 0 && cl >= 0) ? a.slots + static_cast<size_t>(p) * TB2 + v0 : nullptr;
    double* gs = a.slots + static_cast<size_t>(cs) * TB2 + v0;
    double* gl = cl >= 0 ? a.slots + static_cast<size_t>(cl) * TB2 + v0 : nullptr;
    // One round of loads for the item: the flags, both children's statistics (uniform) and up to
    // 64 x kScanWU bins of accumulator words and parent bins, all issued before the first store
    // (the re-zeroing and slot stores may alias the parent's bins for the compiler: loading in
    // the same iteration as the stores serialised one round trip per 64 bins, twice)
    const bool skip_both = !a.used_bytree[f] || !(p >= 0 ? a.spl[static_cast<size_t>(p) * F + f] : 1);
    const int splp = p >= 0 ? a.spl[static_cast<size_t>(p) * F + f] : 1;
    double2 cls0 = a.lsum[cs];
    double2 cls1 = cl >= 0 ? a.lsum[cl] : cls0;
    FNode cnd0 = a.nodes[cs];
    FNode cnd1 = cl >= 0 ? a.nodes[cl] : cnd0;
    if (a.voting) {
      // voting's LOCAL pass (as k_f_scan): this rank's rows and sums -- the smaller child's from the
      // round's exact local totals, the larger's as the parent's local sums minus them
      cls0 = make_double2(static_cast<double>(static_cast<long long>(a.ltot[2 * e])) * inv_g,
                          static_cast<double>(static_cast<long long>(a.ltot[2 * e + 1])) * inv_h);
      if (cl >= 0) {
        const double2 ps = a.lsum_loc[p];
        cls1 = make_double2(ps.x - cls0.x, ps.y - cls0.y);
      }
      cnd0.gcount = cnd0.count;
      cnd1.gcount = cnd1.count;
      if (f == 0 && lane == 0) {
        a.lsum_loc[cs] = cls0;
        if (cl >= 0) a.lsum_loc[cl] = cls1;
      }
    }
    const double cpo0 = a.lout[cs], cpo1 = cl >= 0 ? a.lout[cl] : cpo0;
    const LeafBounds cbd0 = a.bounds[cs], cbd1 = cl >= 0 ? a.bounds[cl] : cbd0;
    constexpr int kScanWU = 4;
#pragma unroll 1
    for (int k0 = lane; k0 < nbin - 1; k0 += 64 * kScanWU) {
      unsigned long long x0[kScanWU], x1[kScanWU];
      double pg0[kScanWU], pg1[kScanWU];
#pragma unroll
      for (int u = 0; u < kScanWU; ++u) {
        const int kk = k0 + 64 * u;
        const bool ok = kk < nbin - 1;
        x0[u] = ok ? acc[pw * kk] : 0ull;
        x1[u] = ok && !qpack ? acc[2 * kk + 1] : 0ull;
        pg0[u] = ok && gl ? gp[2 * kk] : 0.0;
        pg1[u] = ok && gl ? gp[2 * kk + 1] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < kScanWU; ++u) {
        const int kk = k0 + 64 * u;
        if (kk >= nbin - 1) continue;
        acc[pw * kk] = 0ull;
        if (!qpack) acc[2 * kk + 1] = 0ull;
        long long q0 = static_cast<long long>(x0[u]), q1 = static_cast<long long>(x1[u]);
        if (qpack) {
          const unsigned long long hs = x0[u] & 0xFFFFFFFFull;
          q0 = static_cast<long long>(x0[u] - hs) >> 32;
          q1 = static_cast<long long>(hs);
        }
        const double sv0 = static_cast<double>(q0) * inv_g, sv1 = static_cast<double>(q1) * inv_h;
        const int b = kk < fi.mfb ? kk : kk + 1;
        hs_full[2 * b] = sv0;
        hs_full[2 * b + 1] = sv1;
        gs[2 * kk] = sv0;
        gs[2 * kk + 1] = sv1;
        if (gl) {
          const double l0 = pg0[u] - sv0, l1 = pg1[u] - sv1;
          hl_full[2 * b] = l0;
          hl_full[2 * b + 1] = l1;
          gl[2 * kk] = l0;
          gl[2 * kk + 1] = l1;
        }
      }
    }
    FWaveSync();
    // most-frequent bins = leaf totals - stored bins
    const int nsel = cl >= 0 ? 2 : 1;
#pragma unroll 1
    for (int sel = 0; sel < nsel; ++sel) {
      double* H = sel ? hl_full : hs_full;
      const double2 lsum = sel ? cls1 : cls0;
      double sgs = 0.0, shs = 0.0;
#pragma unroll 1
      for (int b = lane; b < nbin; b += 64) {
        if (b == fi.mfb) continue;
        sgs += H[2 * b];
        shs += H[2 * b + 1];
      }
      sgs = WaveSum(sgs);
      shs = WaveSum(shs);
      if (lane == 0) {
        H[2 * fi.mfb] = lsum.x - sgs;
        H[2 * fi.mfb + 1] = lsum.y - shs;
      }
    }
    FWaveSync();
#pragma unroll 1
    for (int sel = 0; sel < nsel; ++sel) {
      const int my = sel ? cl : cs;
      const double* H = sel ? hl_full : hs_full;
      // the child's statistics (loaded with the item's bins)
      const double2 lsum = sel ? cls1 : cls0;
      const FNode nd = sel ? cnd1 : cnd0;
      const double pre_out = sel ? cpo1 : cpo0;
      const LeafBounds bnd = sel ? cbd1 : cbd0;
      if (lane == 0) {
        out->Reset();
        SplitKey kz;
        kz.gain = kMinScore;
        kz.feature = -1;
        kz.threshold = 0;
        kz.group = kz.offset = kz.num_bin = kz.mfb = kz.default_bin = 0;
        kz.missing = kz.default_left = kz.is_cat = kz.pad0 = 0;
        kz.pos = f;
        kz.pad2 = 0;
        *key = kz;
      }
      FWaveSync();
      const double sg = lsum.x, sh = lsum.y;
      const int n = nd.gcount;
      const int depth = nd.depth;
      const SplitParams spp = a.voting ? *a.sp_local : a.sp;
      if (!skip_both) {
        double po;
        if (p < 0) {
          SplitParams p0 = spp;
          p0.path_smooth = 0.0;
          po = LeafOutputRaw(sg, sh, p0, n, 0.0);
          if (f == 0 && lane == 0 && !a.voting) a.lout[0] = po;  // (voting: k_f_elect writes the global one)
        } else {
          po = pre_out;
        }
        const LeafBounds bounds = bnd;
        // (numerical features only: LaunchFrontierScan routes categorical data to k_f_scan)
        const bool spl = ScanNumericalWave(spp, fi, H, sg, sh, n, po, bounds, 0, out);
        if (lane == 0) {
          a.spl[static_cast<size_t>(my) * F + f] = spl ? 1 : 0;
          if (!spl || (a.max_depth > 0 && depth >= a.max_depth)) {
            out->Reset();
          } else {
            out->feature = f;
            // (voting's local pass ranks raw gains: penalties and masks belong to the global pass)
            if (!a.cegb_raw && !a.voting) {
              if (a.cegb_split > 0.0) out->gain -= a.cegb_split * n;
              if (out->monotone_type != 0) out->gain *= MonotonePenaltyAt(a.monotone_penalty, depth);
            }
            if (a.ic && !a.voting && !FIcAllows(a, my, f)) out->Reset();
          }
        }
      } else if (lane == 0) {
        a.spl[static_cast<size_t>(my) * F + f] = static_cast<uint8_t>(splp);
        if (p < 0 && f == 0 && !a.voting) {
          SplitParams p0 = a.sp;
          p0.path_smooth = 0.0;
          a.lout[0] = LeafOutputRaw(sg, sh, p0, n, 0.0);
        }
      }
      if (lane == 0) {
        key->feature = out->feature;
        key->gain = SafeGain(*out);
        key->threshold = out->threshold;
        key->group = fi.group;
        key->offset = fi.offset;
        key->num_bin = fi.num_bin;
        key->mfb = fi.mfb;
        key->default_bin = fi.default_bin;
        key->missing = fi.missing;
        key->default_left = out->default_left;
        key->is_cat = fi.bin_type != 0 ? 1 : 0;
        key->pad0 = a.cegb_raw && out->feature >= 0 ? out->monotone_type : 0;
      }
      FWaveSync();
      // publish (dword-parallel copy of the LDS records)
      const size_t q = (static_cast<size_t>(e) * 2 + sel) * F + f;
      for (int i = lane; i < kKeyWords + kInfoWords; i += 64) {
        if (i < kKeyWords) {
          reinterpret_cast<uint32_t*>(a.ckey + q)[i] = reinterpret_cast<const uint32_t*>(key)[i];
        } else {
          reinterpret_cast<uint32_t*>(a.cinfo + q)[i - kKeyWords] = reinterpret_cast<const uint32_t*>(out)[i - kKeyWords];
        }
      }
      FWaveSync();  // (out / key reused by the next child)
    }
    FWaveSync();  // (the histograms in LDS reused by the next item)
  }
  FStampEnd(a, rnd, kFStampScan);
}

// ---------------------------------------------------------------------------
// k_f_partition: stable 2-way partition of every expanded parent (reference
// data_partition.hpp:101 / cuda_data_partition.cu:290-937, as one launch).
// Tiles of all expansions are numbered globally ([tile0_e, tile0_e + ntiles_e) for expansion e);
// block b owns the MAXT contiguous tiles [b MAXT, b MAXT + MAXT). A block counts its tiles,
// publishes each count, finds the exclusive left-count prefix of its first tile by a decoupled
// look-back over the earlier tiles OF ITS EXPANSION, publishes its tiles' inclusive prefixes and
// scatters: lefts go to the front of the parent's range in order, rights fill it from the end.
// The block that scatters an expansion's last tile knows its total left count and writes the two
// children (post-split bookkeeping of serial_tree_learner.cpp:766-922).

// tile granule {epoch:32 | inclusive:1 | value:31}: a tile's left count, or (inclusive) the left
// count of its expansion's tiles up to and including it
__device__ __forceinline__ void FPublish(unsigned long long* p, unsigned epoch, int v, bool incl) {
  const unsigned long long w = (static_cast<unsigned long long>(epoch) << 32) | (incl ? 0x80000000ull : 0ull) |
                               static_cast<unsigned>(v);
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// split predicate of expansion x on group bin gb (GoLeft of split_scan.h, categorical set in `bits`)
__device__ __forceinline__ bool FGoLeft(const FExp& x, const uint32_t* bits, uint32_t gb) {
  const uint32_t b = DecodeBin(x.offset, x.num_bin, x.mfb, gb);
  if (x.is_cat) {
    const uint32_t wd = b >> 5;
    return wd < static_cast<uint32_t>(kMaxCatWords) && ((bits[wd] >> (b & 31u)) & 1u);
  }
  if ((x.missing == 1 && b == static_cast<uint32_t>(x.default_bin)) ||
      (x.missing == 2 && b == static_cast<uint32_t>(x.num_bin - 1))) {
    return x.default_left != 0;
  }
  return b <= static_cast<uint32_t>(x.thr);
}

constexpr unsigned kLookbackSpins = 2048;  // s_sleep(1) polls (~100 us) before a tile is counted here

constexpr int kLookbackPer = 4;  // predecessors per thread and window (1,024 per window)

struct FLookbackLds {
  int near, nmiss, list[256 * kLookbackPer], val[256 * kLookbackPer], red[4];
};

// Exclusive left-count prefix of tile i of expansion x (block-cooperative): windows of
// kLookbackPer x blockDim predecessors, nearest first, their granules loaded in one round; a window
// holding an inclusive granule ends the walk. Blocks own contiguous tiles, so a block only waits on
// LOWER blocks. A predecessor still unpublished after the poll bound (its block not running:
// nothing here assumes co-residency or dispatch order) is counted by this block -- the same pure
// function of the tile's rows its owner evaluates -- and published (the identical value). The
// part_selfcount test hook counts every predecessor here.
__device__ int FLookback(const FArgs& a, const FExp& x, const uint32_t* bits, int i, unsigned epoch, FLookbackLds* L) {
  const int t = threadIdx.x;
  const int nt = static_cast<int>(blockDim.x);
  constexpr int kInf = 0x7fffffff;
  int excl = 0;
  for (int hi = i; hi > x.tile0;) {
    const int lo = max(x.tile0, hi - kLookbackPer * nt);
    // predecessor d = u * nt + t (0 = the nearest) is tile hi - 1 - d
    unsigned long long v[kLookbackPer];
    bool have[kLookbackPer];
    if (t == 0) {
      L->near = kInf;
      L->nmiss = 0;
    }
#pragma unroll
    for (int u = 0; u < kLookbackPer; ++u) {
      const int j = hi - 1 - (u * nt + t);
      v[u] = j >= lo ? __hip_atomic_load(&a.tile_pub[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kLookbackPer; ++u) {
      const int j = hi - 1 - (u * nt + t);
      have[u] = false;
      if (j < lo) continue;
      for (unsigned spins = 0; static_cast<unsigned>(v[u] >> 32) != epoch && spins < kLookbackSpins; ++spins) {
        __builtin_amdgcn_s_sleep(1);
        v[u] = __hip_atomic_load(&a.tile_pub[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      have[u] = static_cast<unsigned>(v[u] >> 32) == epoch && !a.part_selfcount;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kLookbackPer; ++u) {
      const int j = hi - 1 - (u * nt + t);
      if (j >= lo && !have[u]) L->list[atomicAdd(&L->nmiss, 1)] = j;
    }
    __syncthreads();
    const int nm = L->nmiss;
    if (nm > 0) {
      // rare: count the unpublished predecessors with the whole block, one tile at a time
      for (int m = 0; m < nm; ++m) {
        const int tile = L->list[m];
        const int p0 = (tile - x.tile0) * a.part_tile, p1 = min(x.count, p0 + a.part_tile);
        int cc = 0;
        for (int p = p0 + t; p < p1; p += nt) {
          const int row = FRowAt(a, x.src_buf, x.start + p);
          cc += FGoLeft(x, bits, FColBin(a, x.group, row)) ? 1 : 0;
        }
        cc = BlockSumInt(cc, L->red);
        if (t == 0) {
          L->val[hi - 1 - tile] = cc;
          FPublish(&a.tile_pub[tile], epoch, cc, false);
        }
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < kLookbackPer; ++u) {
        const int j = hi - 1 - (u * nt + t);
        if (j >= lo && !have[u]) {
          v[u] = static_cast<unsigned long long>(static_cast<unsigned>(L->val[u * nt + t]));  // (an aggregate)
          have[u] = true;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < kLookbackPer; ++u) {
      if (have[u] && (v[u] & 0x80000000ull) != 0ull) atomicMin(&L->near, u * nt + t);
    }
    __syncthreads();
    const int near = L->near;
    int c = 0;
#pragma unroll
    for (int u = 0; u < kLookbackPer; ++u) {
      const int j = hi - 1 - (u * nt + t);
      if (j >= lo && u * nt + t <= near) c += static_cast<int>(v[u] & 0x7fffffffull);
    }
    excl += BlockSumInt(c, L->red);
    if (near != kInf) break;
    hi = lo;
  }
  return excl;
}

// children of expansion x (one thread)
__device__ void FPostSplit(const FArgs& a, int e, const FExp& x, int lc) {
  const SplitInfo& bi = x.forced >= 0 ? a.fbest[x.parent] : a.best[x.parent];
  const double lsg = bi.left_sum_gradient, lsh = bi.left_sum_hessian;
  const double rsg = bi.right_sum_gradient, rsh = bi.right_sum_hessian;
  const double lo = bi.left_output, ro = bi.right_output;
  const int ilc = bi.left_count, irc = bi.right_count;
  const int8_t mono = bi.monotone_type;
  const int16_t ncat = bi.num_cat_threshold;
  const int feature = bi.feature;
  LeafBounds bl = a.bounds[x.parent];
  const int rc = x.count - lc;
  const int glc = a.distributed ? ilc : lc;
  const int grc = a.distributed ? irc : rc;
  const int l = x.left, r = x.left + 1;
  const int dep = x.depth + 1;
  FNode nl, nr;
  nl.buf = nr.buf = x.dst_buf;
  nl.start = x.start;
  nl.count = lc;
  nl.gcount = glc;
  nr.start = x.start + lc;
  nr.count = rc;
  nr.gcount = grc;
  nl.depth = nr.depth = dep;
  nl.parent = nr.parent = x.parent;
  nl.left = nr.left = -1;
  nl.fidx = x.forced >= 0 ? a.forced[x.forced].left : -1;
  nr.fidx = x.forced >= 0 ? a.forced[x.forced].right : -1;
  a.nodes[l] = nl;
  a.nodes[r] = nr;
  a.lsum[l] = make_double2(lsg, lsh);
  a.lsum[r] = make_double2(rsg, rsh);
  a.lout[l] = lo;
  a.lout[r] = ro;
  LeafBounds br = bl;
  if (a.use_monotone && ncat == 0 && a.mono_inter) {
    // intermediate: the siblings bound each other by their actual outputs (host
    // MonotoneLeafConstraints::AfterSplit; reference monotone_constraints.hpp:560-574)
    if (mono < 0) {
      bl.min = fmax(bl.min, ro);
      br.max = fmin(br.max, lo);
    } else if (mono > 0) {
      bl.max = fmin(bl.max, ro);
      br.min = fmax(br.min, lo);
    }
  } else if (a.use_monotone && ncat == 0) {
    const double mid = (lo + ro) / 2.0f;
    if (mono < 0) {
      bl.min = fmax(bl.min, mid);
      br.max = fmin(br.max, mid);
    } else if (mono > 0) {
      bl.max = fmin(bl.max, mid);
      br.min = fmax(br.min, mid);
    }
  }
  a.bounds[l] = bl;
  a.bounds[r] = br;
  if (a.ic) {
    // the children's sets: the parent's that also hold the split feature
    for (int w = 0; w < a.ic_words; ++w) {
      const unsigned long long icm = a.ic[static_cast<size_t>(x.parent) * a.ic_words + w] &
                                     a.ic_feat[static_cast<size_t>(feature) * a.ic_words + w];
      a.ic[static_cast<size_t>(l) * a.ic_words + w] = icm;
      a.ic[static_cast<size_t>(r) * a.ic_words + w] = icm;
    }
  }
  const int md = a.sp.min_data_in_leaf;
  // children with forced splits of their own always get histograms (the forced split ignores
  // min_data / max_depth, as the host learner's ForceSplits does); the scan keeps their
  // regular candidates within max_depth
  const bool forced_child = nl.fidx >= 0 || nr.fidx >= 0;
  const bool skip = x.last || (!forced_child && ((a.max_depth > 0 && dep >= a.max_depth) || (grc < md * 2 && glc < md * 2)));
  const bool left_smaller = glc < grc;
  FExp* xo = a.exps + e;
  xo->skip = skip ? 1 : 0;
  xo->smaller = left_smaller ? l : r;
  xo->larger = left_smaller ? r : l;
  xo->h_buf = x.dst_buf;
  xo->h_start = left_smaller ? x.start : x.start + lc;
  xo->h_count = left_smaller ? lc : rc;
}

// block sums of M values at once (one barrier pair for all of them)
template <int M>
__device__ __forceinline__ void BlockSumMulti(int* v, int* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int m = 0; m < M; ++m) v[m] = WaveSum(v[m]);
  __syncthreads();  // sh is reused
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m) sh[m * 4 + w] = v[m];
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < M; ++m) v[m] = sh[m * 4] + sh[m * 4 + 1] + sh[m * 4 + 2] + sh[m * 4 + 3];
}

template <int ITERS, int MAXT>
__global__ __launch_bounds__(kFPartThreads) __attribute__((amdgpu_waves_per_eu(ITERS == 8 ? 5 : 1))) void k_f_partition(FArgs a) {
  static_assert(kFPartThreads == 256, "4 waves per block");
  static_assert(MAXT * ITERS <= 32, "left / valid bits of a thread fit one word");
  constexpr int kTile = kFPartThreads * ITERS;
  __shared__ int s_t0[kFrontierKmax + 1];
  __shared__ FExp s_x[kFrontierKmax];
  __shared__ uint32_t s_bits[kFrontierKmax][kMaxCatWords];
  __shared__ int sh[MAXT * 4];
  __shared__ int s_wl[MAXT][ITERS][kFPartThreads / 64];
  __shared__ int s_wv[MAXT][ITERS][kFPartThreads / 64];
  __shared__ FLookbackLds s_lb;
  const FState* stp = a.st;
  if (stp->done) return;
  const int k = stp->k, T = stp->total_tiles;
  const unsigned epoch = stp->epoch;
  const int rnd = stp->round;
  FStamp(a, rnd, kFStampPart, 0);
  const int G = static_cast<int>(gridDim.x);
  const int t = threadIdx.x;
  if (static_cast<int>(blockIdx.x) * MAXT >= T) return;
  // the round's expansions (dword-parallel copy) and their categorical sets
  constexpr int kXWords = static_cast<int>(sizeof(FExp) / 4);
  for (int i = t; i < k * kXWords; i += blockDim.x) {
    reinterpret_cast<uint32_t*>(s_x)[i] = reinterpret_cast<const uint32_t*>(a.exps)[i];
  }
  for (int i = t; i < k * kMaxCatWords; i += blockDim.x) s_bits[i / kMaxCatWords][i % kMaxCatWords] = a.exp_bits[i];
  __syncthreads();
  if (t <= k) s_t0[t] = t < k ? s_x[t].tile0 : T;
  __syncthreads();
  auto find = [&](int tile) {
    int lo = 0, hi = k - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_t0[mid] <= tile) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  auto go_left = [&](int e, uint32_t gb) { return FGoLeft(s_x[e], s_bits[e], gb); };
  FStamp(a, rnd, kFStampPart, 1);
  const int lane = t & 63, w = t >> 6;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // passes of G * MAXT tiles (one pass whenever the grid covers the tile capacity, as the learner
  // sizes it)
  for (int bid = static_cast<int>(blockIdx.x) * MAXT; bid < T; bid += G * MAXT) {
    // ---- counts of the block's tiles (loads issued together: row ids, then bins)
    int ex[MAXT], rows[MAXT][ITERS];
    unsigned lbits = 0u, vbits = 0u;  // bit j * ITERS + i: row valid / goes left
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int tile = bid + j;
      ex[j] = tile < T ? find(tile) : -1;
      const int e = ex[j] < 0 ? 0 : ex[j];
      const FExp& x = s_x[e];
      const int pos0 = (tile - x.tile0) * kTile + t;
#pragma unroll
      for (int i = 0; i < ITERS; ++i) {
        const int pos = pos0 + i * kFPartThreads;
        rows[j][i] = (ex[j] >= 0 && pos < x.count) ? FRowAt(a, x.src_buf, x.start + pos) : -1;
      }
    }
    int cnt[MAXT];
    {
      uint32_t gb[MAXT][ITERS];
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const int g = s_x[ex[j] < 0 ? 0 : ex[j]].group;
#pragma unroll
        for (int i = 0; i < ITERS; ++i) gb[j][i] = rows[j][i] >= 0 ? FColBin(a, g, rows[j][i]) : 0u;
      }
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        cnt[j] = 0;
#pragma unroll
        for (int i = 0; i < ITERS; ++i) {
          const bool valid = rows[j][i] >= 0;
          const bool left = valid && go_left(ex[j], gb[j][i]);
          vbits |= (valid ? 1u : 0u) << (j * ITERS + i);
          lbits |= (left ? 1u : 0u) << (j * ITERS + i);
          cnt[j] += left ? 1 : 0;
        }
      }
    }
    BlockSumMulti<MAXT>(cnt, sh);
    // aggregates first (a tile that starts its expansion publishes its count as inclusive)
    if (t == 0) {
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        if (ex[j] >= 0) FPublish(&a.tile_pub[bid + j], epoch, cnt[j], bid + j == s_x[ex[j]].tile0);
      }
    }
    FStamp(a, rnd, kFStampPart, 2);
    // ---- exclusive prefixes: a look-back for the block's first tile only (a later tile of the
    // block continues its predecessor's expansion, or is the first tile of the next one)
    int lb[MAXT];
    lb[0] = ex[0] >= 0 && bid > s_x[ex[0]].tile0 ? FLookback(a, s_x[ex[0]], s_bits[ex[0]], bid, epoch, &s_lb) : 0;
#pragma unroll
    for (int j = 1; j < MAXT; ++j) lb[j] = ex[j] >= 0 && ex[j] == ex[j - 1] ? lb[j - 1] + cnt[j - 1] : 0;
    if (t == 0) {
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        if (ex[j] >= 0 && bid + j > s_x[ex[j]].tile0) FPublish(&a.tile_pub[bid + j], epoch, lb[j] + cnt[j], true);
      }
    }
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
#pragma unroll
      for (int i = 0; i < ITERS; ++i) {
        const unsigned long long ml = __ballot((lbits >> (j * ITERS + i)) & 1u);
        const unsigned long long mv = __ballot((vbits >> (j * ITERS + i)) & 1u);
        if (lane == 0) {
          s_wl[j][i][w] = __popcll(ml);
          s_wv[j][i][w] = __popcll(mv);
        }
      }
    }
    __syncthreads();
    // ---- scatter
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      if (ex[j] < 0) continue;
      const int e = ex[j];
      const FExp& x = s_x[e];
      const int tile = bid + j;
      const int tt = tile - x.tile0;
      int lbase = lb[j];
      int rbase = tt * kTile - lbase;
      int* out = a.idx[x.dst_buf] + x.start;
#pragma unroll
      for (int i = 0; i < ITERS; ++i) {
        const bool valid = (vbits >> (j * ITERS + i)) & 1u;
        const bool left = (lbits >> (j * ITERS + i)) & 1u;
        const unsigned long long ml = __ballot(left);
        const unsigned long long mv = __ballot(valid);
        int pl = 0, pv = 0, tl = 0, tv = 0;
#pragma unroll
        for (int q = 0; q < kFPartThreads / 64; ++q) {
          if (q < w) {
            pl += s_wl[j][i][q];
            pv += s_wv[j][i][q];
          }
          tl += s_wl[j][i][q];
          tv += s_wv[j][i][q];
        }
        if (valid) {
          const int rl = pl + __popcll(ml & lt_mask);
          const int rv = pv + __popcll(mv & lt_mask);
          int* dst = left ? out + lbase + rl : out + (x.count - 1 - (rbase + (rv - rl)));
          *dst = rows[j][i];
        }
        lbase += tl;
        rbase += tv - tl;
      }
      if (tt == x.ntiles - 1 && t == 0) FPostSplit(a, e, x, lbase);
    }
    __syncthreads();  // (LDS ballot counts reused by the next pass)
  }
  FStamp(a, rnd, kFStampPart, 3);
  FStampEnd(a, rnd, kFStampPart);
}

// ---------------------------------------------------------------------------
// k_f_select: one workgroup. Every phase is ONE round of independent global loads (the
// select sits on the critical path of every round: its latency, not its work, matters).
//  A. per-child best split of the last round's children: arg-max over the features'
//     candidates (gain desc, feature asc: SplitInfo::BetterThan), full record -> best[c]
//  B. replay of best-first order over the committed leaves (wave 0, all in LDS): the leaf
//     with the largest gain (ties: smaller feature, then smaller leaf, as the sequential
//     select) is split if its node has been expanded, else the replay stops there
//  C. the committed splits -> SplitRec[] (tree order), leaf -> node table
//  D. the next round's expansions: the blocked node first, then the open nodes by gain,
//     as many as the remaining split budget can still use (+ spec_cap), under the
//     row-list rule (the list a child overwrites belongs to a committed split)
__device__ __forceinline__ bool FBetter(double ga, int fa, int la, double gb, int fb, int lb) {
  if (ga != gb) return ga > gb;
  if (fa != fb) return fa < fb;
  return la < lb;
}

// CEGB with coupled penalties: the penalised gain of a RAW candidate key at the current
// used-feature flags (host SerialTreeLearner::ScoreFeature: gain -= CegbPenalty::DeltaGain,
// then the monotone penalty multiplies a monotone split; key.pad0 = its monotone type)
__device__ __forceinline__ double CegbAdjust(const FArgs& a, const SplitKey& k, int n, int depth, const uint8_t* used,
                                             int node) {
  if (k.feature < 0) return kMinScore;
  double delta = a.cegb_split * n;
  if (a.cegb_coupled != nullptr && !used[k.feature]) delta += a.cegb_coupled[k.feature];
  if (a.cegb_lazy != nullptr) delta += a.cegb_lazy[k.feature] * a.nlazy[static_cast<size_t>(node) * a.F + k.feature];
  double g = k.gain - delta;
  if (k.pad0 != 0) g *= MonotonePenaltyAt(a.monotone_penalty, depth);
  return g;
}

// copy the stored raw candidate (node x, feature slot f) into node c's best / key with gain g
// (one lane: the CEGB refund / re-score paths are rare)
__device__ __forceinline__ void CegbSetBest(const FArgs& a, int c, size_t src, double g) {
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
  for (int i = 0; i < kInfoWords; ++i) reinterpret_cast<uint32_t*>(a.best + c)[i] = reinterpret_cast<const uint32_t*>(a.ninfo + src)[i];
  for (int i = 0; i < kKeyWords; ++i) reinterpret_cast<uint32_t*>(a.key + c)[i] = reinterpret_cast<const uint32_t*>(a.nkey + src)[i];
  a.best[c].gain = g;
  a.key[c].gain = g;
}

// By-node mask of node c under interaction constraints (FArgs::byn_draw; host ColSampler::GetByNode,
// reference col_sampler.hpp:91-150): the pool is the features in ascending order that the by-tree
// sample keeps and c's constraint sets allow; Random::Sample(N, K = min(byn_cnt, N)) picks pool
// indices with the sampler's LCG. One lane draws (each step depends on the last), the wave counts
// the pool and maps the picks back to features. s_pick: LDS scratch of F bytes. Called by a whole
// wave; rng is wave-uniform.
__device__ void FByNodeDraw(const FArgs& a, int c, uint8_t* mask, uint8_t* s_pick, unsigned* rng) {
  const int lane = threadIdx.x & 63, F = a.F;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int N = 0;
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int f = f0 + lane;
    const bool in = f < F && (!a.byn_reset || a.used_bytree[f]) && FIcAllows(a, c, f);
    N += __popcll(__ballot(in));
  }
  const int K = min(a.byn_cnt, N);
  const int mode = a.byn_mode[N];
  for (int i = lane; i < N; i += 64) s_pick[i] = mode == 1 ? 1 : 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  unsigned x = *rng;
  if (lane == 0 && mode >= 2) {
    if (mode == 2) {
      // Bernoulli scan: row i kept with probability (K - kept so far) / (N - i)
      int got = 0;
      for (int i = 0; i < N; ++i) {
        x = 214013u * x + 2531011u;
        const float r = static_cast<float>(static_cast<int>((x >> 16) & 0x7FFFu)) / 32768.0f;
        if (r < static_cast<double>(K - got) / static_cast<double>(N - i)) {
          s_pick[i] = 1;
          ++got;
        }
      }
    } else {
      // Floyd: v uniform in [0, r]; r itself when v was already taken
      for (int r = N - K; r < N; ++r) {
        x = 214013u * x + 2531011u;
        const int v = static_cast<int>(x & 0x7FFFFFFFu) % (r + 1);
        if (s_pick[v]) s_pick[r] = 1;
        else s_pick[v] = 1;
      }
    }
  }
  *rng = static_cast<unsigned>(ReadLane(static_cast<int>(x), 0));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  int base = 0;
  for (int f0 = 0; f0 < F; f0 += 64) {
    const int f = f0 + lane;
    const bool in = f < F && (!a.byn_reset || a.used_bytree[f]) && FIcAllows(a, c, f);
    const unsigned long long b = __ballot(in);
    if (f < F) mask[f] = in && s_pick[base + __popcll(b & lt)] ? 1 : 0;
    base += __popcll(b);
  }
  // (the re-score's lanes read the mask back through the same cache)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------------
// Intermediate monotone constraints in the select (host MonotoneLeafConstraints, reference
// monotone_constraints.hpp:516-857 IntermediateLeafConstraints). Each leaf of the committed tree
// carries its CURRENT bounds (cb) and the bounds its best split was scanned with (sb). A commit
// bounds the two children by each other's outputs and walks the committed tree: climbing from the
// split node, every numerical monotone ancestor that borders it (the first of its (feature, side)
// on the way up) bounds the leaves on its far side that can touch the new leaves. Bounds only
// tighten, and a tighter bound never raises a split's gain (the clamped outputs move away from
// the optimum; the order check cannot newly pass: both children clamp into one interval), so a
// STALE leaf's recorded gain is an upper bound of its re-scan: the replay commits a clean leaf
// only when no stale leaf's bound reaches its gain, otherwise it stops and the stale leaves are
// re-scanned from their slots (FExp::rescan) in the next round. 1M x 28 with 4 constrained
// features: 63 leaves 1.29x, 255 leaves 1.69x the unconstrained iteration time.
struct FMonoLds {
  double2* cb = nullptr;   // [L] current bounds (min, max) of each leaf
  double2* sb = nullptr;   // [L] the bounds its record was scanned with
  int* thr = nullptr;      // [C] split threshold bin | is_cat << 31
  int* ancd = nullptr;     // [L] ancestors of the committed node, by depth
  int* lvf = nullptr;      // [L] climb level: split feature (-1: categorical)
  int* lvt = nullptr;      // [L] climb level: threshold | 1 << 28 borders | 1 << 29 monotone | 1 << 30 decreasing
  uint8_t* lvs = nullptr;  // [L] climb level: 1 = reached from the right child
  int8_t* mono = nullptr;  // [F] monotone type of each feature
  int* cl = nullptr;       // [C] leaf index of each cid that is a leaf of the committed tree
  int* qa = nullptr;       // descent queues; these three live in the alive-sort area, unused
  int* qb = nullptr;       // during the replay
};
constexpr int kMonoBorder = 1 << 28, kMonoMono = 1 << 29, kMonoDec = 1 << 30, kMonoThr = (1 << 28) - 1;

__device__ __forceinline__ bool FMonoStale(const FMonoLds& mo, int l) {
  const double2 cb = mo.cb[l], sb = mo.sb[l];
  return cb.x > sb.x || cb.y < sb.y;
}

// Wave 0 after committing node c's split (leaf bl keeps the left child `left`, the right child is
// the new leaf nl - 1): host MonotoneLeafConstraints::AfterSplit (Climb / Descend)
__device__ void FMonoCommit(const FArgs& a, const FMonoLds& mo, const int* s_par, const int* s_left, const int* s_feat,
                            const int* s_dep, const uint8_t* s_st, const double* s_lg, int c, int left, int bl, int nl) {
  const int lane = threadIdx.x & 63;
  const SplitInfo& bi = a.best[c];
  const double lo = bi.left_output, ro = bi.right_output;
  const int mt = bi.monotone_type;
  const LeafBounds sbl = a.bounds[left], sbr = a.bounds[left + 1];
  const int cthr = mo.thr[c];
  const int sf = s_feat[c];
  const uint32_t sthr = static_cast<uint32_t>(cthr & 0x7fffffff);
  const int D = s_dep[c];
  const int nr = nl - 1;
  {
    // the children: the parent's current bounds, the siblings bounding each other by their outputs
    const double2 pb = mo.cb[bl];
    double2 lc = pb, rc = pb;
    if (cthr >= 0 && mt != 0) {
      if (mt < 0) {
        lc.x = fmax(lc.x, ro);
        rc.y = fmin(rc.y, lo);
      } else {
        lc.y = fmin(lc.y, ro);
        rc.x = fmax(rc.x, lo);
      }
    }
    FWaveSync();
    if (lane == 0) {
      mo.cb[bl] = lc;
      mo.cb[nr] = rc;
      mo.sb[bl] = make_double2(sbl.min, sbl.max);
      mo.sb[nr] = make_double2(sbr.min, sbr.max);
      int x = c;
      for (int d = D - 1; d >= 0; --d) {  // the ancestors by depth
        x = s_par[x];
        mo.ancd[d] = x;
      }
    }
  }
  FWaveSync();
  if (D == 0) return;
  // climb level i: ancestor ancd[D - 1 - i], reached from ancd[D - i] (level 0: from c)
  for (int i = lane; i < D; i += 64) {
    const int P = mo.ancd[D - 1 - i];
    const int node = i == 0 ? c : mo.ancd[D - i];
    const int th = mo.thr[P];
    mo.lvf[i] = th >= 0 ? s_feat[P] : -1;
    mo.lvt[i] = th & kMonoThr;
    mo.lvs[i] = s_left[P] + 1 == node ? 1 : 0;
  }
  FWaveSync();
  // a level borders the new leaves when no lower level split on the same feature from the same
  // side (those are the path entries the host pushes); bordering numerical monotone ones descend
  bool any = false;
  for (int i = lane; i < D; i += 64) {
    const int f = mo.lvf[i];
    const uint8_t side = mo.lvs[i];
    bool border = f >= 0;
    for (int j = 0; j < i && border; ++j) border = !(mo.lvf[j] == f && mo.lvs[j] == side);
    if (border) {
      int v = kMonoBorder;
      const int m = mo.mono[f];
      if (m != 0) {
        v |= kMonoMono | (m < 0 ? kMonoDec : 0);
        any = true;
      }
      mo.lvt[i] |= v;
    }
  }
  if (__ballot(any) == 0ull) return;
  FWaveSync();
  // Descend (host MonotoneLeafConstraints::Descend), top-down and pruned: a breadth-first walk of
  // the far subtrees of the bordering monotone levels, one lane per queued node. An entry packs
  // (node, level, use_left, use_right); a node lets the walk through a side unless a bordering
  // split below its level, on the same feature, separates that side from the new leaves, and a
  // split on the new split's own feature decides which new output each side borders. Every leaf
  // lies in one far subtree (that of its lowest common ancestor with c): no two lanes write one
  // leaf's bounds.
  const unsigned long long ltm = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int nq = 0;
  for (int i0 = 0; i0 < D; i0 += 64) {
    const int i = i0 + lane;
    bool push = false;
    int ent = 0;
    if (i < D && (mo.lvt[i] & kMonoMono)) {
      const int P = mo.ancd[D - 1 - i];
      const int node = i == 0 ? c : mo.ancd[D - i];
      const int far = s_left[P] == node ? s_left[P] + 1 : s_left[P];
      ent = far | (i << 16) | (3 << 28);
      push = true;
    }
    const unsigned long long m = __ballot(push);
    if (push) mo.qa[nq + __popcll(m & ltm)] = ent;
    nq += __popcll(m);
  }
  int* qcur = mo.qa;
  int* qnext = mo.qb;
  while (nq > 0) {
    FWaveSync();
    int nn = 0;
    for (int e0 = 0; e0 < nq; e0 += 64) {
      const int e = e0 + lane;
      int o0 = -1, o1 = -1;
      if (e < nq) {
        const int ent = qcur[e];
        const int x = ent & 0xFFFF, lam = (ent >> 16) & 0xFFF;
        const bool ul = (ent >> 28) & 1, ur = (ent >> 29) & 1;
        if (!(s_st[x] & kNodeCommitted)) {
          // a leaf of the committed tree
          const int l = mo.cl[x];
          if (l != bl && l != nr && s_lg[l] > kMinScore) {  // (host: best gain kMinScore, no update)
            const int lt = mo.lvt[lam];
            const bool from_right = mo.lvs[lam] != 0;
            const bool tmax = (lt & kMonoDec) ? !from_right : from_right;
            double vlo, vhi;
            if (ul && ur) {
              vlo = fmin(lo, ro);
              vhi = fmax(lo, ro);
            } else if (ur) {
              vlo = vhi = ro;
            } else {
              vlo = vhi = lo;
            }
            double2 cb = mo.cb[l];
            if (tmax) {
              if (vlo < cb.y) cb.y = vlo;
            } else {
              if (vhi > cb.x) cb.x = vhi;
            }
            mo.cb[l] = cb;
          }
        } else {
          const int th = mo.thr[x];
          bool gl = true, gr = true, lsr = true, rsl = true;
          if (th >= 0) {
            const int fx = s_feat[x];
            const uint32_t tx = static_cast<uint32_t>(th);
            for (int j = 0; j < lam; ++j) {
              const int tj = mo.lvt[j];
              if (mo.lvf[j] != fx || !(tj & kMonoBorder)) continue;
              const uint32_t tv = static_cast<uint32_t>(tj & kMonoThr);
              const bool sj = mo.lvs[j] != 0;
              if (tx >= tv && !sj) gr = false;
              if (tx <= tv && sj) gl = false;
            }
            if (fx == sf) {
              if (tx <= sthr) lsr = false;
              if (tx >= sthr) rsl = false;
            }
          }
          const int lx = s_left[x];
          if (gl) o0 = lx | (lam << 16) | ((ul ? 1 : 0) << 28) | ((lsr && ur ? 1 : 0) << 29);
          if (gr) o1 = (lx + 1) | (lam << 16) | ((rsl && ul ? 1 : 0) << 28) | ((ur ? 1 : 0) << 29);
        }
      }
      const int cnt = (o0 >= 0 ? 1 : 0) + (o1 >= 0 ? 1 : 0);
      const int inc = WaveInclusiveScan(cnt);
      int pos = nn + inc - cnt;
      if (o0 >= 0) qnext[pos++] = o0;
      if (o1 >= 0) qnext[pos] = o1;
      nn += ReadLane(inc, 63);
    }
    int* tq = qcur;
    qcur = qnext;
    qnext = tq;
    nq = nn;
  }
  FWaveSync();
}

constexpr int kSelWaves = kFSelThreads / 64;
constexpr int kSelPairs = 2 * kFrontierKmax / kSelWaves;  // (expansion, child) pairs per wave
constexpr int kSelRankMax = 256;  // alive nodes up to which the select ranks instead of sorting
constexpr int kSelLPer = 4;       // leaves per lane of the register replay (L <= 256)

// kWide: more than 64 features (phase A loads two feature chunks per round of loads: its own
// instantiation, so the headline's select keeps its register allocation)
// kXg: the xGMI transport's push / handshake / system-scope merge (its own instantiations)
// kMono: intermediate monotone constraints (FArgs::mono_inter; FMonoCommit below)
template <bool kCegb, bool kWide, bool kXg, bool kMono>
__global__ __launch_bounds__(kFSelThreads) void k_f_select(FArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int C = a.C, L = a.L, F = a.F;
  double* s_gain = reinterpret_cast<double*>(smem);          // [C]
  int* s_feat = reinterpret_cast<int*>(s_gain + C);          // [C]
  int* s_left = s_feat + C;                                  // [C]
  int* s_par = s_left + C;                                   // [C]
  int* s_dep = s_par + C;                                    // [C]
  int* s_rank = s_dep + C;                                   // [C] eligible: rank, else -1
  int* s_fidx = s_rank + C;                                  // [C] forced split index, -1: none
  int* s_lcid = s_fidx + C;                                  // [L]
  int* s_c0 = s_lcid + L;                                    // [L] committed leaves of this launch
  int* s_c1 = s_c0 + L;                                      // [L] their cids (~cid: a forced split)
  uint8_t* s_st = reinterpret_cast<uint8_t*>(s_c1 + L);      // [C]
  // intermediate monotone (kMono): after the common image (FrontierSelectMonoLds)
  FMonoLds mo;
  if (kMono) {
    const size_t o = (FrontierSelectLds(C, L) + 15) & ~static_cast<size_t>(15);
    mo.cb = reinterpret_cast<double2*>(smem + o);
    mo.sb = mo.cb + L;
    mo.thr = reinterpret_cast<int*>(mo.sb + L);
    mo.ancd = mo.thr + C;
    mo.lvf = mo.ancd + L;
    mo.lvt = mo.lvf + L;
    mo.lvs = reinterpret_cast<uint8_t*>(mo.lvt + L);
    mo.mono = reinterpret_cast<int8_t*>(mo.lvs + L);
  }
  __shared__ int s_cpos[2 * kFrontierKmax];  // this round's children: winning candidate position
  __shared__ int s_pc[2 * kFrontierKmax];    // pair -> child cid (-1: none / skipped)
  __shared__ int s_nl, s_ns, s_done, s_blocked, s_ncommit, s_k, s_tiles, s_fnext, s_bforced;
  __shared__ int s_exp[kFrontierKmax];       // chosen expansions (cids) by order
  __shared__ int s_rsc[kMono ? kFrontierKmax : 1], s_rsl[kMono ? kFrontierKmax : 1];  // (kMono) stale leaves: cid, leaf
  __shared__ int s_nrs, s_nr;  // (kMono) stale leaves listed, rescans taken
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const FState st = *a.st;
  const unsigned xep = kXg ? *a.xc->ep : 0u;  // (xGMI: this round's tag is xep + 1)
  // keys final once computed (no CEGB re-scoring; a monotone rescan's node re-enters as new): the
  // alive order carries over
  constexpr bool kIncr = !kCegb;
  __shared__ int s_rscan[kMono ? kFrontierKmax : 1], s_nrsc;  // (kMono) the last round's rescanned cids
  if (kMono && t == 0) s_nrsc = 0;
  if (st.done) return;
  const int kprev = st.k;
  const int cid_next = st.cid_next;
  const int np = 2 * kprev;
  const int rnd = st.round;
  FStamp(a, rnd, kFStampSel, 0);
  // this round's children are cids [base, base + 2 kx) (the root round: cid 0); pairs of the
  // intermediate-monotone rescans after them name older cids
  const int base = cid_next - 2 * st.kx;
  // ---- image of the computed nodes + the pairs of the last round (one load round)
  for (int c = t; c < cid_next; c += blockDim.x) {
    const SplitKey& kk = a.key[c];
    const FNode& nd = a.nodes[c];
    const int kf = kk.feature;
    const double kg = kk.gain;
    s_left[c] = nd.left;
    s_par[c] = nd.parent;
    s_dep[c] = nd.depth;
    s_st[c] = a.nstate[c];
    s_gain[c] = kf < 0 ? kMinScore : kg;
    s_feat[c] = kf;
    s_rank[c] = -1;
    s_fidx[c] = nd.fidx;
    if (kMono) mo.thr[c] = static_cast<int>(kk.threshold & 0x7fffffffu) | (kk.is_cat ? static_cast<int>(0x80000000u) : 0);
  }
  if (kMono) {
    for (int f = t; f < F; f += blockDim.x) mo.mono[f] = a.feat[f].monotone;
  }
  for (int l = t; l < st.num_leaves; l += blockDim.x) s_lcid[l] = a.leaf_cid[l];
  // CEGB coupled penalties: used-feature flags (after the sort scratch) and the event count
  constexpr bool cegb = kCegb;  // CEGB coupled penalties: its own instantiation (registers)
  uint8_t* s_used = reinterpret_cast<uint8_t*>(smem + FrontierSelectLds(C, L));
  const unsigned epoch0 = cegb && a.cegb_coupled != nullptr ? *a.cegb_epoch : 0u;
  if (cegb && a.cegb_coupled != nullptr) {
    for (int f = t; f < F; f += blockDim.x) s_used[f] = a.cegb_used[f];
  }
  if (t < 2 * kFrontierKmax) {
    int c = -1;
    if (t < np) {
      const FExp& x = a.exps[t >> 1];
      c = x.skip ? -1 : ((t & 1) ? x.larger : x.smaller);
      if (x.skip && !(t & 1)) c = -2 - x.smaller;  // skipped: children get empty records
      if (x.skip && (t & 1)) c = -2 - x.larger;
    }
    s_pc[t] = c;
    s_cpos[t] = -1;
  }
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
  static_assert(kInfoWords + kKeyWords <= 64, "one record word per lane");
  const float spec_alpha = a.tp->spec_alpha;  // (phase D; loaded here, off its critical path)
  __syncthreads();
  FStamp(a, rnd, kFStampSel, 1);
  if (cegb && a.cegb_lazy != nullptr) {
    // CEGB lazy penalties: unmarked-row counts of this round's children, the smaller's from
    // the round's counts (k_f_lazy), the larger's as parent - smaller (the split feature is on
    // both children's paths: zero)
    for (int i = t; i < np * F; i += blockDim.x) {
      const int q = i / F, f = i - q * F;
      const int c = s_pc[q];
      if (c < 0) continue;
      const FExp& x = a.exps[q >> 1];
      const int cnt = a.lazy_acc[static_cast<size_t>(q >> 1) * F + f];
      const int v = c == x.smaller ? cnt : (f == x.feature ? 0 : a.nlazy[static_cast<size_t>(x.parent) * F + f] - cnt);
      a.nlazy[static_cast<size_t>(c) * F + f] = v;
    }
    __syncthreads();
    for (int i = t; i < kprev * F; i += blockDim.x) a.lazy_acc[i] = 0;
    __syncthreads();
  }
  // ---- A. children of the last round: best over features (all pairs' keys in flight). Feature-
  // parallel and owner-computes data-parallel rounds: best over the RANKS' per-child records
  // (fpb, all-gathered after k_f_pair_best; gain desc, then feature asc -- the order of the
  // sequential select), the record copied from the winning rank's fpb entry
  const bool merge = a.fpb != nullptr;
  const int nsrc = merge ? a.vote_P : F;
  if (kXg && merge) {
    // ---- A0 (xGMI transport): this rank's best per child over the features it owns -> fpb[rank]
    // of every rank's exchange buffer, then the handshake (k_f_pair_best's job, folded into the
    // one-block select: no launch of its own); phase A then merges the P ranks' records
    constexpr int kKw = static_cast<int>(sizeof(SplitKey) / 4), kIw = static_cast<int>(sizeof(SplitInfo) / 4);
    for (int q = w; q < np; q += kSelWaves) {
      if (s_pc[q] < 0) continue;  // (no child, or a skipped expansion's: never merged)
      double bg = kMinScore;
      int bf = 0x7fffffff, bp = -1;
      for (int i = lane; i < a.fown_n; i += 64) {
        const int f = a.fown_list[i];
        const SplitKey& kk = a.ckey[static_cast<size_t>(q) * F + f];
        if (kk.feature >= 0 && FBetter(kk.gain, kk.feature, 0, bg, bf, 0)) {
          bg = kk.gain;
          bf = kk.feature;
          bp = f;
        }
      }
      bp = ReadLane(bp, WaveArgBestLane(bg, bf, 0));
      const uint32_t* sk = reinterpret_cast<const uint32_t*>(a.ckey + static_cast<size_t>(q) * F + max(bp, 0));
      const uint32_t* si = reinterpret_cast<const uint32_t*>(a.cinfo + static_cast<size_t>(q) * F + max(bp, 0));
      const uint32_t v = lane < kKw ? sk[lane] : (lane < kKw + kIw ? si[lane - kKw] : 0u);
      for (int r = 0; r < a.xc->P; ++r) {
        FPairBest* out = reinterpret_cast<FPairBest*>(a.xc->peer[r] + a.xc->o_fpb) + static_cast<size_t>(a.xc->rank) * 2 * a.kmax + q;
        if (bp < 0) {
          // (an empty record: feature -1, gain kMinScore)
          if (lane == 0) FXStore(reinterpret_cast<uint32_t*>(&out->key.feature), static_cast<uint32_t>(-1));
          if (lane < 2) FXStore(reinterpret_cast<uint32_t*>(&out->key.gain) + lane,
                                static_cast<uint32_t>(static_cast<unsigned long long>(__double_as_longlong(kMinScore)) >> (32 * lane)));
        } else if (lane < kKw) {
          FXStore(reinterpret_cast<uint32_t*>(&out->key) + lane, v);
        } else if (lane < kKw + kIw) {
          FXStore(reinterpret_cast<uint32_t*>(&out->info) + (lane - kKw), v);
        }
      }
    }
    if (FXPeers(a)) {
      FXArrive(a, kFXCand, FXTag(a, xep + 1u));  // (one block: it is the last to arrive, and waits)
    } else {
      __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
  }
  if (kXg && t == 0) *a.xc->ep = xep + 1u;  // this round's exchanges are complete: the next round's tag
  {
    double bg[kSelPairs];
    int bf[kSelPairs], bp[kSelPairs], pn[kSelPairs], pd[kSelPairs];
#pragma unroll
    for (int j = 0; j < kSelPairs; ++j) {
      bg[j] = kMinScore;
      bf[j] = 0x7fffffff;
      bp[j] = -1;
      pn[j] = pd[j] = 0;
      const int q = w + j * kSelWaves;
      if (cegb && q < np && s_pc[q] >= 0) {
        pn[j] = a.nodes[s_pc[q]].gcount;
        pd[j] = s_dep[s_pc[q]];
      }
    }
    if (!cegb && kWide) {
      // wide data: the keys of two 64-feature chunks of every pair are loaded before any compare
      // (one memory round trip per 128 features instead of per 64; F = 500: 4 instead of 8)
      bool pv[kSelPairs];
#pragma unroll
      for (int j = 0; j < kSelPairs; ++j) {
        const int q = w + j * kSelWaves;
        pv[j] = q < np && s_pc[q] >= 0;
      }
      for (int f0 = 0; f0 < nsrc; f0 += 128) {
        int kf[2][kSelPairs];
        double kg[2][kSelPairs];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int f = f0 + 64 * u + lane;
#pragma unroll
          for (int j = 0; j < kSelPairs; ++j) {
            const int q = w + j * kSelWaves;
            kf[u][j] = -1;
            kg[u][j] = kMinScore;
            if (pv[j] && f < nsrc) {
              const SplitKey& kk = merge ? a.fpb[static_cast<size_t>(f) * 2 * a.kmax + q].key : a.ckey[static_cast<size_t>(q) * F + f];
              FKeyFG(kk, kXg && merge, &kf[u][j], &kg[u][j]);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int f = f0 + 64 * u + lane;
#pragma unroll
          for (int j = 0; j < kSelPairs; ++j) {
            if (kf[u][j] < 0) continue;
            const int ff = kf[u][j];
            if (FBetter(kg[u][j], ff, 0, bg[j], bf[j], 0)) {
              bg[j] = kg[u][j];
              bf[j] = ff;
              bp[j] = f;
            }
          }
        }
      }
    } else
    for (int f0 = 0; f0 < nsrc; f0 += 64) {
      const int f = f0 + lane;
#pragma unroll
      for (int j = 0; j < kSelPairs; ++j) {
        const int q = w + j * kSelWaves;
        // (bynode: the root is scored at its mask, row 0; other children when their parent commits)
        if (q < np && f < nsrc && s_pc[q] >= 0 && !(cegb && a.bynode != nullptr && s_pc[q] == 0 && !a.bynode[f])) {
          const SplitKey& kk = merge ? a.fpb[static_cast<size_t>(f) * 2 * a.kmax + q].key : a.ckey[static_cast<size_t>(q) * F + f];
          int kf;
          double kgain;
          FKeyFG(kk, kXg && merge, &kf, &kgain);
          const double g = kf < 0 ? kMinScore : (cegb ? CegbAdjust(a, kk, pn[j], pd[j], s_used, s_pc[q]) : kgain);
          const int ff = kf < 0 ? 0x7fffffff : kf;
          if (FBetter(g, ff, 0, bg[j], bf[j], 0)) {
            bg[j] = g;
            bf[j] = ff;
            bp[j] = f;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kSelPairs; ++j) {
      const int q = w + j * kSelWaves;
      if (q >= np) continue;
      const int pc = s_pc[q];
      if (pc == -1) continue;  // no child (root round's second pair)
      const int c = pc >= 0 ? pc : -2 - pc;
      const int src = WaveArgBestLane(bg[j], bf[j], 0);
      const double g = ReadLane(bg[j], src);
      const int ff = ReadLane(bf[j], src);
      const int fpos = ReadLane(bp[j], src);
      const bool valid = pc >= 0 && ff != 0x7fffffff && fpos >= 0;
      // (keys / records written here are read back by LATER launches only; this launch
      // reads the candidate table, which an earlier launch wrote)
      if (valid) {
        const size_t pos = static_cast<size_t>(q) * F + fpos;
        const FPairBest* pb = merge ? a.fpb + static_cast<size_t>(fpos) * 2 * a.kmax + q : nullptr;
        const uint32_t* si = reinterpret_cast<const uint32_t*>(merge ? &pb->info : a.cinfo + pos);
        const uint32_t* sk = reinterpret_cast<const uint32_t*>(merge ? &pb->key : a.ckey + pos);
        const bool sys = kXg && merge;  // (a record a peer pushed)
        for (int i = lane; i < kInfoWords + kKeyWords; i += 64) {
          if (i < kInfoWords) {
            reinterpret_cast<uint32_t*>(a.best + c)[i] = sys ? FXLoad(si + i) : si[i];
          } else {
            reinterpret_cast<uint32_t*>(a.key + c)[i - kInfoWords] = sys ? FXLoad(sk + i - kInfoWords) : sk[i - kInfoWords];
          }
        }
      } else if (lane == 0) {
        a.best[c].Reset();
        SplitKey kz;
        kz.gain = kMinScore;
        kz.feature = -1;
        kz.threshold = 0;
        kz.group = kz.offset = kz.num_bin = kz.mfb = kz.default_bin = 0;
        kz.missing = kz.default_left = kz.is_cat = kz.pad0 = 0;
        kz.pos = -1;
        kz.pad2 = 0;
        a.key[c] = kz;
      }
      if (cegb) {
        // the child's raw candidates of every feature, kept for refunds / re-scoring (skipped
        // expansions' children: none); its best carries the penalised gain
        constexpr int kRow = kKeyWords + kInfoWords;
        const size_t dst = static_cast<size_t>(c) * F;
        for (int i = lane; i < F * kRow; i += 64) {
          const int f = i / kRow, o = i - f * kRow;
          const size_t src = static_cast<size_t>(q) * F + f;
          if (pc < 0) {
            if (o == 0) a.nkey[dst + f].feature = -1;
          } else if (o < kKeyWords) {
            reinterpret_cast<uint32_t*>(a.nkey + dst + f)[o] = reinterpret_cast<const uint32_t*>(a.ckey + src)[o];
          } else {
            reinterpret_cast<uint32_t*>(a.ninfo + dst + f)[o - kKeyWords] = reinterpret_cast<const uint32_t*>(a.cinfo + src)[o - kKeyWords];
          }
        }
        if (lane == 0) a.nuep[c] = static_cast<int>(epoch0);
      }
      if (lane == 0) {
        s_gain[c] = valid ? g : kMinScore;
        s_feat[c] = valid ? ff : -1;
        if (kMono && (q >> 1) >= st.kx && pc >= 0) {
          // (a rescan: its key changed; the merged alive order takes it as a new node)
          s_st[c] = static_cast<uint8_t>(s_st[c] | kNodeRescanTmp);
          s_rscan[atomicAdd(&s_nrsc, 1)] = c;
        }
        // (CEGB: the penalised best lives in best / key only)
        // (merged ranks' records: the next expansions read best / key, written above)
        // (a rescan's pair names an older cid: its record is read back from best / key)
        if (!kMono || (c >= base && c - base < 2 * kFrontierKmax)) {
          s_cpos[c - base] = valid && !cegb && !merge ? static_cast<int>(static_cast<size_t>(q) * F + fpos) : -1;
        }
      }
    }
  }
  __syncthreads();
  if (cegb) {
    // penalised gains into the best / key records phase A copied (raw) above
    for (int q = t; q < np; q += blockDim.x) {
      const int c = s_pc[q];
      if (c >= 0 && s_feat[c] >= 0) {
        a.best[c].gain = s_gain[c];
        a.key[c].gain = s_gain[c];
      }
    }
  }
  __syncthreads();
  FStamp(a, rnd, kFStampSel, 2);
  // ---- B. replay (wave 0): per-leaf (gain, feature) cached in LDS, one max scan per step
  // (the full three-key tie-break only when two leaves share the best gain)
  double* s_lg = reinterpret_cast<double*>(smem + ((reinterpret_cast<uintptr_t>(s_st + C) -
                                                     reinterpret_cast<uintptr_t>(smem) + 15) & ~uintptr_t(15)));  // [L]
  int* s_lf = reinterpret_cast<int*>(s_lg + L);                        // [L]
  double* s_sg = reinterpret_cast<double*>(smem + ((reinterpret_cast<uintptr_t>(s_lf + L) -
                                                    reinterpret_cast<uintptr_t>(smem) + 15) & ~uintptr_t(15)));  // [P2max]
  int* s_sc = reinterpret_cast<int*>(s_sg + FrontierSortCap(C));      // [P2max]
  if (kMono) {
    // (FMonoCommit's descent queues and cid -> leaf map: the sort area is unused until phase D)
    mo.qa = reinterpret_cast<int*>(s_sg);
    mo.qb = mo.qa + FrontierSortCap(C);
    mo.cl = s_sc;
  }
  // (the register replay below reads the leaves' keys itself: no LDS image, no barrier)
  const bool reg_replay = !cegb && !kMono && st.forced_next < 0 && L <= 64 * kSelLPer;
  if (!reg_replay) {
    for (int l = t; l < st.num_leaves; l += blockDim.x) {
      const int c = s_lcid[l];
      const int f = s_feat[c];
      s_lg[l] = f < 0 ? kMinScore : s_gain[c];
      s_lf[l] = f < 0 ? 0x7fffffff : f;
      if (kMono) {
        const LeafBounds cb = a.cbnd[c], sb = a.bounds[c];
        mo.cb[l] = make_double2(cb.min, cb.max);
        mo.sb[l] = make_double2(sb.min, sb.max);
        mo.cl[c] = l;
      }
    }
    __syncthreads();
  }
  __shared__ int s_byn;
  __shared__ unsigned s_brng;
  if (w == 0) {
    int nl = st.num_leaves, ns = st.num_splits, done = 0, blocked = -1, nc = 0;
    int fnext = st.forced_next, bforced = 0;
    int byn = st.byn;  // bynode masks drawn (wave-uniform)
    unsigned brng = st.byn_rng;  // (by-node draws in the select: the sampler's state, wave-uniform)
    unsigned epoch = epoch0;  // CEGB first-use events (wave-uniform)
    if (reg_replay) {
      // leaf l's (gain, feature, cid) in registers of lane l % 64, slot l / 64: per committed
      // split one wave max and two dependent LDS reads (the winner's left child, then its two
      // children's keys)
      const int nslot = (L + 63) >> 6;
      int lc[kSelLPer];
      double lg[kSelLPer];
      int lf[kSelLPer];
#pragma unroll
      for (int j = 0; j < kSelLPer; ++j) {
        const int l = lane + 64 * j;
        lc[j] = j < nslot && l < nl ? s_lcid[l] : -1;
        lg[j] = kMinScore;
        lf[j] = 0x7fffffff;
        if (lc[j] >= 0) {
          const int f = s_feat[lc[j]];
          lg[j] = f < 0 ? kMinScore : s_gain[lc[j]];
          lf[j] = f < 0 ? 0x7fffffff : f;
        }
      }
      for (;;) {
        if (nl >= L) {
          done = 1;
          break;
        }
        // the lane's best slot (slots in leaf order: FBetter's leaf tie-break holds)
        double pg = lg[0];
        int pf = lf[0], pl = lane;
#pragma unroll
        for (int j = 1; j < kSelLPer; ++j) {
          if (j < nslot && FBetter(lg[j], lf[j], lane + 64 * j, pg, pf, pl)) {
            pg = lg[j];
            pf = lf[j];
            pl = lane + 64 * j;
          }
        }
        const double mg = WaveMaxDpp(pg);
        const unsigned long long tie = __ballot(pg == mg);
        const int src = __popcll(tie) == 1 ? __ffsll(static_cast<long long>(tie)) - 1 : WaveArgBestLane(pg, pf, pl);
        const double bg = ReadLane(pg, src);
        const int bf = ReadLane(pf, src);
        const int bl = ReadLane(pl, src);
        if (bf == 0x7fffffff || !(bg > 0.0)) {
          done = 1;
          break;
        }
        int cl = -1;
#pragma unroll
        for (int j = 0; j < kSelLPer; ++j) cl = (bl >> 6) == j ? lc[j] : cl;
        const int c = ReadLane(cl, src);
        const int left = s_left[c];
        if (left < 0) {
          blocked = c;
          break;
        }
        const int fa = s_feat[left], fb = s_feat[left + 1];
        const double ga = s_gain[left], gb = s_gain[left + 1];
#pragma unroll
        for (int j = 0; j < kSelLPer; ++j) {
          if (lane + 64 * j == bl) {
            lc[j] = left;
            lg[j] = fa < 0 ? kMinScore : ga;
            lf[j] = fa < 0 ? 0x7fffffff : fa;
          }
          if (lane + 64 * j == nl) {
            lc[j] = left + 1;
            lg[j] = fb < 0 ? kMinScore : gb;
            lf[j] = fb < 0 ? 0x7fffffff : fb;
          }
        }
        if (lane == 0) {
          s_c0[nc] = bl;
          s_c1[nc] = c;
          s_st[c] |= kNodeCommitted;
        }
        ++nc;
        ++nl;
        ++ns;
      }
#pragma unroll
      for (int j = 0; j < kSelLPer; ++j) {
        if (lane + 64 * j < nl) s_lcid[lane + 64 * j] = lc[j];
      }
    } else
    for (;;) {
      if (nl >= L) {
        done = 1;
        break;
      }
      if (fnext >= 0) {
        // forced splits first, in the host learner's order (learner/forced_splits.h): the
        // leaf holding forced split `fnext`; a non-positive forced gain ends forced splitting
        int fl = -1;
        for (int l = lane; l < nl; l += 64) {
          if (s_fidx[s_lcid[l]] == fnext) fl = l;
        }
        const unsigned long long hit = __ballot(fl >= 0);
        if (hit == 0ull) {
          fnext = -1;
        } else {
          fl = __shfl(fl, __ffsll(static_cast<long long>(hit)) - 1, kWave);
          const int c = s_lcid[fl];
          const double fg = a.fbest[c].gain;  // (an earlier launch's scan wrote it)
          if (!(fg > 0.0)) {
            fnext = -1;
          } else if (s_left[c] < 0) {
            blocked = c;
            bforced = 1;
            break;
          } else {
            const int left = s_left[c];
            if (lane == 0) {
              s_c0[nc] = fl;
              s_c1[nc] = ~c;
              s_lcid[fl] = left;
              s_lcid[nl] = left + 1;
              s_st[c] |= kNodeCommitted;
              const int fa = s_feat[left], fb = s_feat[left + 1];
              s_lg[fl] = fa < 0 ? kMinScore : s_gain[left];
              s_lf[fl] = fa < 0 ? 0x7fffffff : fa;
              s_lg[nl] = fb < 0 ? kMinScore : s_gain[left + 1];
              s_lf[nl] = fb < 0 ? 0x7fffffff : fb;
            }
            ++nc;
            ++nl;
            ++ns;
            fnext = fnext + 1 < a.num_forced ? fnext + 1 : -1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            continue;
          }
        }
      }
      double bg = kMinScore;
      int bf = 0x7fffffff, bl = 0x7fffffff;
      double sgm = -INFINITY;  // (kMono) the largest gain bound among stale leaves
      for (int l = lane; l < nl; l += 64) {
        const double g = s_lg[l];
        const int ff = s_lf[l];
        if (FBetter(g, ff, l, bg, bf, bl)) {
          bg = g;
          bf = ff;
          bl = l;
        }
        if (kMono && g > 0.0 && FMonoStale(mo, l)) sgm = fmax(sgm, g);
      }
      const double mg = WaveMaxDpp(bg);
      const unsigned long long tie = __ballot(bg == mg);
      int src;
      if (__popcll(tie) == 1) src = __ffsll(static_cast<long long>(tie)) - 1;
      else src = WaveArgBestLane(bg, bf, bl);
      bg = ReadLane(bg, src);
      bf = ReadLane(bf, src);
      bl = ReadLane(bl, src);
      if (bl == 0x7fffffff || bf == 0x7fffffff || !(bg > 0.0)) {
        done = 1;
        break;
      }
      // (kMono: a stale leaf may still beat the best: its re-scan decides; ties included, as the
      // re-scanned record may win the feature / leaf tie-break. With max_delta_step or path
      // smoothing the raw output can sit beyond a bound on the optimum's side, a tighter bound
      // may then RAISE the gain: every stale leaf is re-scanned before the next commit)
      if (kMono) {
        const double sm = WaveMaxDpp(sgm);
        const bool ub = !(a.sp.max_delta_step > 0.0) && !(a.sp.path_smooth > kEpsilon);
        if (ub ? sm >= bg : sm > -INFINITY) break;
      }
      const int c = s_lcid[bl];
      const int left = s_left[c];
      if (left < 0) {
        blocked = c;
        break;
      }
      if (cegb) {
        if (a.cegb_coupled != nullptr && !s_used[bf]) {
          // first use of feature bf (host CegbPenalty::OnSplit): every other leaf's stored
          // candidate on bf -- the last valid one along its leaf index's chain of left
          // children, as the host's per-leaf table -- is refunded and may become its best
          const double refund = a.cegb_coupled[bf];
          for (int l = lane; l < nl; l += 64) {
            if (l == bl || !(s_lg[l] > kMinScore)) continue;
            int x = s_lcid[l], found = -1;
            for (;;) {
              if (a.nkey[static_cast<size_t>(x) * F + bf].feature >= 0) {
                found = x;
                break;
              }
              const int px = s_par[x];
              if (px < 0 || s_left[px] != x) break;
              x = px;
            }
            if (found < 0) continue;
            const size_t src = static_cast<size_t>(found) * F + bf;
            const double rg = a.nkey[src].gain + refund;
            if (!FBetter(rg, bf, 0, s_lg[l], s_lf[l], 0)) continue;
            const int cl = s_lcid[l];
            s_lg[l] = rg;
            s_lf[l] = bf;
            s_gain[cl] = rg;
            s_feat[cl] = bf;
            CegbSetBest(a, cl, src, rg);
            if (cl >= base && cl - base < 2 * kFrontierKmax) s_cpos[cl - base] = -1;
          }
          // speculation grown under the old gains is void: uncommitted expansions become
          // unexpanded again, everything below them dead
          for (int x = lane; x < cid_next; x += 64) {
            const uint8_t sx = s_st[x];
            if ((sx & kNodeExpanded) && !(sx & kNodeCommitted) && x != c) {
              s_st[x] = static_cast<uint8_t>((sx & ~kNodeExpanded) | 0x80);  // 0x80: children to kill
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          for (bool more = true; more;) {  // parents precede children (cids grow with depth)
            bool ch = false;
            for (int x = lane; x < cid_next; x += 64) {
              const int px = s_par[x];
              if (px < 0 || (s_st[x] & kNodeDead)) continue;
              if ((s_st[px] & 0x80) || (s_st[px] & kNodeDead)) {
                s_st[x] = static_cast<uint8_t>(s_st[x] | kNodeDead);
                ch = true;
              }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            more = __ballot(ch) != 0ull;
          }
          for (int x = lane; x < cid_next; x += 64) {
            const uint8_t sx = s_st[x];
            if (sx & 0x80) {
              s_left[x] = -1;
              a.nodes[x].left = -1;
            }
            const uint8_t nsx = static_cast<uint8_t>(sx & ~0x80);
            s_st[x] = nsx;
            if (nsx != sx || (nsx & kNodeDead)) a.nstate[x] = nsx;
          }
          if (lane == 0) {
            s_used[bf] = 1;
            a.cegb_used[bf] = 1;
            *a.cegb_epoch = epoch + 1u;
          }
          ++epoch;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        // the children are scored at the flags after this split (the host evaluates them
        // after OnSplit): re-score from their raw candidates when an event came since. With
        // by-node sampling always: the children's masks are the next two draws (smaller child
        // first, as the host's FindBestSplits), unless they are not scanned at all (max_depth /
        // min_data, or the tree's last split: the host's loop ends before scanning them and
        // draws nothing for them either)
        const uint8_t* cmask[2] = {nullptr, nullptr};
        if (a.bynode != nullptr) {
          const int gl = a.nodes[left].gcount, gr = a.nodes[left + 1].gcount, md = a.sp.min_data_in_leaf;
          const bool skip = nl + 1 >= L || (a.max_depth > 0 && s_dep[left] >= a.max_depth) ||
                            (gl < 2 * md && gr < 2 * md);
          if (!skip) {
            const bool left_smaller = gl < gr;
            if (a.byn_draw != nullptr) {
              // (interaction constraints: drawn here, over each child's own pool)
              FByNodeDraw(a, left_smaller ? left : left + 1, a.byn_draw + static_cast<size_t>(byn) * F, s_used + F + 16, &brng);
              FByNodeDraw(a, left_smaller ? left + 1 : left, a.byn_draw + static_cast<size_t>(byn + 1) * F, s_used + F + 16, &brng);
            }
            cmask[left_smaller ? 0 : 1] = a.bynode + static_cast<size_t>(byn) * F;
            cmask[left_smaller ? 1 : 0] = a.bynode + static_cast<size_t>(byn + 1) * F;
            byn += 2;
          }
        }
#pragma unroll 1
        for (int ch = left; ch <= left + 1; ++ch) {
          const uint8_t* mk = cmask[ch - left];
          if (a.bynode == nullptr && static_cast<unsigned>(a.nuep[ch]) == epoch) continue;
          const int n = a.nodes[ch].gcount, d = s_dep[ch];
          double cg = kMinScore;
          int cf = 0x7fffffff, cp = -1;
          for (int f = lane; f < F; f += 64) {
            const SplitKey& kk = a.nkey[static_cast<size_t>(ch) * F + f];
            if (kk.feature < 0 || (a.bynode != nullptr && (mk == nullptr || !mk[f]))) continue;
            const double g = CegbAdjust(a, kk, n, d, s_used, ch);
            if (FBetter(g, kk.feature, 0, cg, cf, 0)) {
              cg = g;
              cf = kk.feature;
              cp = f;
            }
          }
          const int src = WaveArgBestLane(cg, cf, 0);
          cg = ReadLane(cg, src);
          cf = ReadLane(cf, src);
          cp = ReadLane(cp, src);
          if (lane == 0) {
            if (cp >= 0) {
              CegbSetBest(a, ch, static_cast<size_t>(ch) * F + cp, cg);
            } else {
              a.best[ch].Reset();
              a.key[ch].feature = -1;
              a.key[ch].gain = kMinScore;
            }
            s_gain[ch] = cp >= 0 ? cg : kMinScore;
            s_feat[ch] = cp >= 0 ? cf : -1;
            a.nuep[ch] = static_cast<int>(epoch);
            if (ch >= base && ch - base < 2 * kFrontierKmax) s_cpos[ch - base] = -1;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
      }
      if (lane == 0) {
        s_c0[nc] = bl;
        s_c1[nc] = c;
        s_lcid[bl] = left;
        s_lcid[nl] = left + 1;
        if (kMono) {
          mo.cl[left] = bl;
          mo.cl[left + 1] = nl;
        }
        s_st[c] |= kNodeCommitted;
        const int fl = s_feat[left], fr = s_feat[left + 1];
        s_lg[bl] = fl < 0 ? kMinScore : s_gain[left];
        s_lf[bl] = fl < 0 ? 0x7fffffff : fl;
        s_lg[nl] = fr < 0 ? kMinScore : s_gain[left + 1];
        s_lf[nl] = fr < 0 ? 0x7fffffff : fr;
      }
      ++nc;
      ++nl;
      ++ns;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (kMono) FMonoCommit(a, mo, s_par, s_left, s_feat, s_dep, s_st, s_lg, c, left, bl, nl);
    }
    if (kMono) {
      // stale leaves -> this round's rescans (phase D), marked ineligible for expansion; every
      // leaf's current bounds back to the node table for the next select
      const unsigned long long ltm = lane == 0 ? 0ull : (~0ull >> (64 - lane));
      int cnt = 0;
      for (int l0 = 0; l0 < nl; l0 += 64) {
        const int l = l0 + lane;
        bool stl = false;
        int x = -1;
        if (l < nl) {
          x = s_lcid[l];
          const double2 cb = mo.cb[l];
          LeafBounds lb;
          lb.min = cb.x;
          lb.max = cb.y;
          a.cbnd[x] = lb;
          stl = s_lg[l] > 0.0 && FMonoStale(mo, l);
          if (stl) s_st[x] = static_cast<uint8_t>(s_st[x] | kNodeStale);
        }
        const unsigned long long m = __ballot(stl);
        const int pos = cnt + __popcll(m & ltm);
        if (stl && pos < kFrontierKmax) {
          s_rsc[pos] = x;
          s_rsl[pos] = l;
        }
        cnt += __popcll(m);
      }
      if (lane == 0) s_nrs = min(cnt, kFrontierKmax);
    }
    if (lane == 0) {
      s_nl = nl;
      s_ns = ns;
      s_done = done;
      s_blocked = blocked;
      s_ncommit = nc;
      s_fnext = fnext;
      s_bforced = bforced;
      s_byn = byn;
      s_brng = brng;
    }
  }
  __syncthreads();
  FStamp(a, rnd, kFStampSel, 3);
  const int nl = s_nl, ns = s_ns, ncommit = s_ncommit;
  int done = s_done;
  __shared__ int s_nsal;  // alive nodes ordered this round (FState::nsal)
  if (t == 0) s_nsal = 0;
  // ---- C. committed splits -> (leaf, cid) records, leaf table, states. The full records
  // (SplitInfo, children counts) are gathered once per tree by k_f_results: a committed
  // node's best never changes, and the copy no longer sits on every round's critical path
  for (int k = t; k < ncommit; k += blockDim.x) {
    const int c = s_c1[k] >= 0 ? s_c1[k] : ~s_c1[k];
    SplitRec* r = a.rec + st.num_splits + k;
    r->leaf = s_c0[k];
    r->pad = s_c1[k];  // committed cid (~cid: a forced split); k_f_results resolves it
    a.nstate[c] = static_cast<uint8_t>(s_st[c] & ~kNodeLocal);
  }
  for (int l = t; l < nl; l += blockDim.x) a.leaf_cid[l] = s_lcid[l];
  FStamp(a, rnd, kFStampSel, 4);
  // ---- D. next round
  if (!done) {
    // ALIVE uncommitted nodes (a positive-gain split, not part of the tree yet) are compacted
    // into a list; ELIGIBLE ones among them are unexpanded and the row list their children
    // overwrite (the ancestor kFrontierBufs - 1 levels up) belongs to a committed split
    __shared__ int s_na, s_ne, s_eu;
    if (t == 0) {
      s_na = 0;
      s_ne = 0;
      s_eu = 0;
    }
    if (kMono) {
      // intermediate monotone: an expansion grown from a stale leaf's record is void -- its
      // subtree dies (cids grow with depth: passes until no parent is newly dead), the leaf is
      // unexpanded and waits for its rescan (0x80: select-local "state changed")
      for (int i = t; i < s_nrs; i += blockDim.x) {
        const int c = s_rsc[i], lf = s_left[c];
        if (lf < 0) continue;
        s_st[lf] = static_cast<uint8_t>(s_st[lf] | kNodeDead | 0x80);
        s_st[lf + 1] = static_cast<uint8_t>(s_st[lf + 1] | kNodeDead | 0x80);
        s_st[c] = static_cast<uint8_t>((s_st[c] & ~kNodeExpanded) | 0x80);
        s_left[c] = -1;
        a.nodes[c].left = -1;
      }
      __syncthreads();
      for (;;) {
        bool ch = false;
        for (int x = t; x < cid_next; x += blockDim.x) {
          const int px = s_par[x];
          if (px >= 0 && (s_st[px] & kNodeDead) && !(s_st[x] & kNodeDead)) {
            s_st[x] = static_cast<uint8_t>(s_st[x] | kNodeDead | 0x80);
            ch = true;
          }
        }
        if (!__syncthreads_or(ch)) break;
      }
      for (int x = t; x < cid_next; x += blockDim.x) {
        const uint8_t sx = s_st[x];
        if (sx & 0x80) {
          s_st[x] = static_cast<uint8_t>(sx & ~0x80);
          a.nstate[x] = static_cast<uint8_t>(sx & ~kNodeLocal);
        }
      }
    }
    __syncthreads();
    int* s_ac = s_rank;  // [C] compacted alive cids, ~cid when not eligible (reuses s_rank)
    const int cap_list = C;
    for (int c0 = 0; c0 < cid_next; c0 += blockDim.x) {
      const int c = c0 + t;
      bool alive = false, elig = false, unc = false;
      if (c < cid_next) {
        const uint8_t sc = s_st[c];
        alive = !(sc & (kNodeCommitted | kNodeDead)) && s_feat[c] >= 0 && s_gain[c] > 0.0;
        elig = alive && !(sc & kNodeExpanded);
        // while forced splits are pending, their nodes are expanded only by them (the blocked one)
        if (elig && s_fnext >= 0 && s_fidx[c] >= 0 && c != s_blocked) elig = false;
        // by-node sampling: a node's split is known once its mask is, i.e. once it is a leaf of
        // the committed tree (its parent committed)
        if (elig && a.bynode != nullptr && s_par[c] >= 0 && !(s_st[s_par[c]] & kNodeCommitted)) elig = false;
        // extra trees: only the node the replay waits for (its children's random thresholds are
        // drawn when every earlier split of the sequential order has been scanned)
        if (elig && a.xrng != nullptr && c != s_blocked) elig = false;
        // intermediate monotone: not while its record is stale (it is re-scanned instead). A node
        // below an uncommitted one is speculated on its provisional bounds (the parent's scanned
        // ones, the sibling rule): they can only tighten by its commit, which the stale check
        // and the subtree kill above catch
        if (kMono && elig && (sc & kNodeStale)) elig = false;
        if (elig) {
          const int target = s_dep[c] + 1 - kFrontierBufs;
          if (target >= 1) {
            int an = c;
            for (int i = 0; i < kFrontierBufs - 1; ++i) an = s_par[an];
            elig = (s_st[an] & kNodeCommitted) != 0;
          }
        }
        unc = (sc & kNodeExpanded) && !(sc & kNodeCommitted);
        if (kIncr && elig) s_st[c] = static_cast<uint8_t>(sc | kNodeEligTmp);  // (the merged order's flags)
      }
      const unsigned long long ma = __ballot(alive);
      const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
      int basea = 0;
      if (lane == 0 && ma) basea = atomicAdd(&s_na, __popcll(ma));
      basea = __shfl(basea, 0, kWave);
      const int ne = __popcll(__ballot(elig)), eu = __popcll(__ballot(unc));
      if (lane == 0) {
        if (ne) atomicAdd(&s_ne, ne);
        if (eu) atomicAdd(&s_eu, eu);
      }
      if (alive) {
        const int pos = basea + __popcll(ma & lt);
        if (pos < cap_list) s_ac[pos] = elig ? c : ~c;
      }
    }
    __syncthreads();
    const int na = min(s_na, cap_list);
    if (t == 0) s_nsal = na;
    const int blocked = s_blocked;
    const int R = L - 1 - ns;  // splits the tree may still make
    // Order of the alive list by (gain desc, cid asc): a bitonic sort in LDS. Position p in the
    // sorted list = alive nodes with a better key; the eligible rank = eligible nodes (other
    // than the blocked one) before p. Policy 1 (default) takes an eligible node when its
    // position is within the speculation budget: best-first order commits at most R more
    // splits and takes them roughly by gain. Policy 0 budgets R minus every expanded but
    // uncommitted node. The blocked node always goes first.
    if (na <= 64) {
      // one wave ranks, scans and takes (no block barriers): each lane one alive node, its
      // position = alive nodes with a better key (gain desc, cid asc; keys are unique)
      if (w == 0) {
        int r = -1, ci = 0x7fffffff;
        double gi = -INFINITY;
        if (lane < na) {
          r = s_ac[lane];
          ci = r >= 0 ? r : ~r;
          gi = s_gain[ci];
        }
        int pos = 0;
#pragma unroll 8
        for (int j = 0; j < na; ++j) {  // (uniform j: scalar lane reads, no LDS permutes)
          const double gj = ReadLane(gi, j);
          const int cj = ReadLane(ci, j);
          pos += (gj > gi || (gj == gi && cj < ci)) ? 1 : 0;
        }
        if (lane < na) s_sc[pos] = r;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int rc = lane < na ? s_sc[lane] : -1;  // lane = sorted position
        const bool fl = rc >= 0 && rc != blocked;
        const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const int ex = __popcll(__ballot(fl) & lt);
        const int cap_nodes = (C - cid_next) / 2 - (R - 1);
        const float alpha = spec_alpha > 0.f ? spec_alpha : 1.f;
        const int budget = static_cast<int>(alpha * static_cast<float>(R)) + a.spec_cap;
        int lim = a.policy == 0 ? min(min(a.kmax, max(1, R - s_eu + a.spec_cap)), min(max(1, cap_nodes), s_ne))
                                : min(a.kmax, max(1, cap_nodes));
        if (a.kcap != nullptr && rnd + 1 < kFrontierRoundCap) lim = min(lim, max(1, a.kcap[rnd + 1]));
        if (kMono) lim = min(lim, max(1, a.kmax - min(s_nrs, a.kmax / 2)));  // (room for the rescans)
        int kk = 0;
        if (rc >= 0) {
          const int rr = rc == blocked ? 0 : ex + (blocked >= 0 ? 1 : 0);
          const bool take = a.policy == 0 || rc == blocked || lane < budget;
          if (take && rr < lim) {
            s_exp[rr] = rc;
            kk = rr + 1;
          }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) kk = max(kk, __shfl_xor(kk, o, kWave));
        if (lane == 0) s_k = kk;
      }
      __syncthreads();
    } else {
    int P2 = 64;
    while (P2 < na) P2 <<= 1;
    if (na <= kSelRankMax) {
      // rank sort (two barriers instead of the bitonic network's log2(P2)(log2(P2)+1)/2):
      // thread i's position = alive nodes ordered before it; keys are unique (cids), so the
      // ranks are a permutation and the order is the bitonic sort's. O(na) broadcast LDS reads
      // per thread: beyond kSelRankMax nodes the network is cheaper (255-leaf trees)
      for (int i = t; i < na; i += blockDim.x) s_sg[i] = s_gain[s_ac[i] >= 0 ? s_ac[i] : ~s_ac[i]];
      __syncthreads();
      int ri = 0, pos = 0;
      if (t < na) {
        ri = s_ac[t];
        const int ci = ri >= 0 ? ri : ~ri;
        const double gi = s_sg[t];
        // eight keys per step: their (broadcast) LDS reads issue together instead of one LDS
        // round trip per key (~7 us per round for ~100 alive nodes before)
        int j = 0;
        for (; j + 8 <= na; j += 8) {
          double g8[8];
          int c8[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int rj = s_ac[j + u];
            c8[u] = rj >= 0 ? rj : ~rj;
            g8[u] = s_sg[j + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) pos += (g8[u] > gi || (g8[u] == gi && c8[u] < ci)) ? 1 : 0;
        }
        for (; j < na; ++j) {
          const int rj = s_ac[j];
          const int cj = rj >= 0 ? rj : ~rj;
          const double gj = s_sg[j];
          pos += (gj > gi || (gj == gi && cj < ci)) ? 1 : 0;
        }
      }
      if (t < na) s_sc[pos] = ri;
      __syncthreads();
    } else {
    // Beyond kSelRankMax alive nodes (255-leaf trees): the previous select's order, filtered to the
    // nodes still alive, merged with the last round's children (rank-sorted among themselves).
    // Outside CEGB / intermediate-monotone rescans a computed node's key never changes, so the
    // merge is the full sort's order; if the counts disagree (they cannot) the network runs.
    bool merged = false;
    if (kIncr && a.salive != nullptr && st.nsal > 0) {
      constexpr int kNewMax = 3 * kFrontierKmax + 1;  // children + (kMono) rescanned nodes
      int* s_oc = reinterpret_cast<int*>(s_sg);  // [C] previous order, still alive
      int* s_nw = s_oc + C;                      // [kNewMax] the new ones, ordered
      int* s_nf = s_nw + kNewMax;                // [kNewMax] alive flags of the new ones
      __shared__ int s_nk, s_nn;
      const int nold = min(st.nsal, C);
      const int lo = max(base, 0), nch = min(cid_next - lo, 2 * kFrontierKmax + 1);
      const int nn = nch + (kMono ? s_nrsc : 0);
      auto live = [&](int c) {
        return !(s_st[c] & (kNodeCommitted | kNodeDead)) && s_feat[c] >= 0 && s_gain[c] > 0.0;
      };
      auto newc = [&](int i) { return kMono && i >= nch ? s_rscan[i - nch] : lo + i; };
      for (int i = t; i < nold; i += blockDim.x) s_sc[i] = a.salive[i];
      for (int i = t; i < nn; i += blockDim.x) s_nf[i] = live(newc(i)) ? 1 : 0;
      if (t == 0) s_nn = 0;
      __syncthreads();
      constexpr int kPm = kFrontierMaxNodes / kFSelThreads;
      int keep[kPm], kloc = 0;
#pragma unroll
      for (int q = 0; q < kPm; ++q) {
        const int p = t * kPm + q;
        keep[q] = p < nold && s_sc[p] < lo && !(kMono && (s_st[s_sc[p]] & kNodeRescanTmp)) && live(s_sc[p]) ? 1 : 0;
        kloc += keep[q];
      }
      const int kinc = WaveInclusiveScan(kloc);
      __shared__ int s_kw[kFSelThreads / 64];
      if (lane == 63) s_kw[w] = kinc;
      // the new ones' ranks among themselves (<= 129: broadcast reads)
      int nr = -1;
      if (t < nn && s_nf[t]) {
        const int ci = newc(t);
        const double gi = s_gain[ci];
        nr = 0;
        for (int j = 0; j < nn; ++j) {
          if (!s_nf[j]) continue;
          const int cj = newc(j);
          const double gj = s_gain[cj];
          nr += (gj > gi || (gj == gi && cj < ci)) ? 1 : 0;
        }
        atomicAdd(&s_nn, 1);
      }
      __syncthreads();
      int koff = 0;
      for (int q = 0; q < w; ++q) koff += s_kw[q];
      koff += kinc - kloc;
      if (t == kFSelThreads - 1) s_nk = koff + kloc;
#pragma unroll
      for (int q = 0; q < kPm; ++q) {
        if (keep[q]) s_oc[koff++] = s_sc[t * kPm + q];
      }
      if (nr >= 0) s_nw[nr] = newc(t);
      __syncthreads();
      const int nk = s_nk, nw = s_nn;
      if (nk + nw == na) {
        merged = true;
        auto better = [&](int c1, int c2) {  // c1 before c2 (gain desc, cid asc)
          const double g1 = s_gain[c1], g2 = s_gain[c2];
          return g1 > g2 || (g1 == g2 && c1 < c2);
        };
        auto enc = [&](int c) { return (s_st[c] & kNodeEligTmp) ? c : ~c; };
        for (int i = t; i < nk + nw; i += blockDim.x) {
          if (i < nk) {
            const int c = s_oc[i];
            int l = 0, h = nw;  // new ones before c
            while (l < h) {
              const int m = (l + h) >> 1;
              if (better(s_nw[m], c)) l = m + 1;
              else h = m;
            }
            s_sc[i + l] = enc(c);
          } else {
            const int j = i - nk, c = s_nw[j];
            int l = 0, h = nk;  // old ones before c
            while (l < h) {
              const int m = (l + h) >> 1;
              if (better(s_oc[m], c)) l = m + 1;
              else h = m;
            }
            s_sc[j + l] = enc(c);
          }
        }
      }
      __syncthreads();
    }
    if (!merged) {
    for (int i = t; i < P2; i += blockDim.x) {
      if (i < na) {
        const int c = s_ac[i] >= 0 ? s_ac[i] : ~s_ac[i];
        s_sg[i] = s_gain[c];
        s_sc[i] = s_ac[i];
      } else {
        s_sg[i] = -INFINITY;  // padding sorts last
        s_sc[i] = 0x7fffffff;
      }
    }
    __syncthreads();
    for (int kk = 2; kk <= P2; kk <<= 1) {
      for (int jj = kk >> 1; jj > 0; jj >>= 1) {
        for (int i = t; i < P2; i += blockDim.x) {
          const int l = i ^ jj;
          if (l <= i) continue;
          const double gi = s_sg[i], gl = s_sg[l];
          const int ri = s_sc[i], rl = s_sc[l];
          const int ci = ri >= 0 ? ri : ~ri, cl = rl >= 0 ? rl : ~rl;
          // does l belong before i (gain desc, cid asc; padding cid INT_MAX)
          const bool l_first = gl > gi || (gl == gi && cl < ci);
          if (l_first == ((i & kk) == 0)) {
            s_sg[i] = gl;
            s_sg[l] = gi;
            s_sc[i] = rl;
            s_sc[l] = ri;
          }
        }
        __syncthreads();
      }
    }
    }
    }
    // eligible ranks: exclusive scan of the eligible (non-blocked) flags in sorted order
    constexpr int kPer = kFrontierMaxNodes / kFSelThreads;  // <= 4 positions per thread
    int fl[kPer], loc = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int p = t * kPer + q;
      const int r = p < na ? s_sc[p] : -1;
      fl[q] = (r >= 0 && r != blocked) ? 1 : 0;
      loc += fl[q];
    }
    const int incl = WaveInclusiveScan(loc);
    __shared__ int s_wsum[kFSelThreads / 64];
    if (lane == 63) s_wsum[w] = incl;
    if (t == 0) s_k = 0;
    __syncthreads();
    int woff = 0;
    for (int q = 0; q < w; ++q) woff += s_wsum[q];
    int ex = woff + incl - loc;
    const int cap_nodes = (C - cid_next) / 2 - (R - 1);
    // policy 1 budget: the best `alpha` fraction of the remaining splits (alpha tuned per tree by
    // the host from the rows the previous trees' uncommitted expansions cost)
    const float alpha = spec_alpha > 0.f ? spec_alpha : 1.f;
    const int budget = static_cast<int>(alpha * static_cast<float>(R)) + a.spec_cap;
    int lim = a.policy == 0 ? min(min(a.kmax, max(1, R - s_eu + a.spec_cap)), min(max(1, cap_nodes), s_ne))
                            : min(a.kmax, max(1, cap_nodes));
    // data-parallel: the round's all-reduce covers only kcap[round] expansions
    if (a.kcap != nullptr && rnd + 1 < kFrontierRoundCap) lim = min(lim, max(1, a.kcap[rnd + 1]));
    if (kMono) lim = min(lim, max(1, a.kmax - min(s_nrs, a.kmax / 2)));  // (room for the rescans)
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int p = t * kPer + q;
      const int rc = p < na ? s_sc[p] : -1;
      if (rc >= 0) {  // eligible
        const int r = rc == blocked ? 0 : ex + (blocked >= 0 ? 1 : 0);
        const bool take = a.policy == 0 || rc == blocked || p < budget;
        if (take && r < lim) {
          s_exp[r] = rc;
          atomicMax(&s_k, r + 1);
        }
      }
      ex += fl[q];
    }
    __syncthreads();
    }
    FStamp(a, rnd, kFStampSel, 5);
    // this round's order of the alive nodes, for the next select's merge
    if (kIncr && a.salive != nullptr) {
      for (int i = t; i < na; i += blockDim.x) a.salive[i] = s_sc[i] >= 0 ? s_sc[i] : ~s_sc[i];
    }
    // (the node capacity bounds the round: expansions voided by CEGB first-use events leave
    // dead cids behind, so the reserve for the remaining splits is not a guarantee then)
    int K = min(s_k, (C - cid_next) / 2);
    // (kMono: the stale leaves' rescans fill the slots the expansions leave)
    const int NR = kMono ? max(0, min(s_nrs, a.kmax - max(K, 0))) : 0;
    if (K <= 0 && NR == 0) done = 1;  // nothing can be expanded: (only reachable without a blocked node)
    K = max(K, 0);
    __syncthreads();
    if (t == 0) {
      s_k = K;
      s_nr = NR;
    }
    if (a.kused != nullptr && t == 0 && rnd + 1 < kFrontierRoundCap) a.kused[rnd + 1] = done ? 0 : K;
    if (!done && w == 0) {
      // expansion records, tiles prefix (wave 0; K <= 64)
      const int kTile = a.part_tile;
      int ntiles = 0;
      FNode nd;
      int p = -1;
      SplitKey kk;
      if (lane < K) {
        p = s_exp[lane];
        const int cpos = (p >= base && p - base < 2 * kFrontierKmax) ? s_cpos[p - base] : -1;
        nd = a.nodes[p];
        kk = p == s_blocked && s_bforced ? a.fkey[p] : (cpos >= 0 ? a.ckey[cpos] : a.key[p]);
        ntiles = max(1, (nd.count + kTile - 1) / kTile);
      }
      const int inc = WaveInclusiveScan(ntiles);
      if (lane < K) {
        FExp x;
        x.parent = p;
        x.left = cid_next + 2 * lane;
        x.depth = nd.depth;
        x.tile0 = inc - ntiles;
        x.ntiles = ntiles;
        x.src_buf = nd.buf;
        x.start = nd.start;
        x.count = nd.count;
        x.dst_buf = FrontierDepthBuf(nd.depth % kFrontierBufs);
        x.group = kk.group;
        x.offset = kk.offset;
        x.num_bin = kk.num_bin;
        x.mfb = kk.mfb;
        x.default_bin = kk.default_bin;
        x.missing = kk.missing;
        x.thr = static_cast<int>(kk.threshold);
        x.default_left = kk.default_left;
        x.is_cat = kk.is_cat;
        x.skip = 0;
        x.smaller = x.larger = -1;
        x.h_buf = x.h_start = x.h_count = 0;
        x.forced = p == s_blocked && s_bforced ? s_fidx[p] : -1;
        x.feature = kk.feature;
        x.last = p == s_blocked && nl + 1 >= L ? 1 : 0;
        x.rescan = 0;
        a.exps[lane] = x;
        a.nodes[p].left = cid_next + 2 * lane;
        a.nstate[p] = static_cast<uint8_t>((s_st[p] & ~kNodeLocal) | kNodeExpanded);
      }
      if (kMono && lane >= K && lane < K + NR) {
        // a rescan: node c's record again from its slot under its current bounds; an expansion
        // grown from its stale record is void (children dead, the node unexpanded)
        const int c = s_rsc[lane - K], l = s_rsl[lane - K];
        FExp x;
        x.parent = c;
        x.left = -1;
        x.depth = s_dep[c];
        x.tile0 = inc;
        x.ntiles = 0;
        x.src_buf = x.start = x.count = x.dst_buf = 0;
        x.group = x.offset = x.num_bin = x.mfb = x.default_bin = x.missing = x.thr = x.default_left = x.is_cat = 0;
        x.skip = 0;
        x.smaller = c;
        x.larger = -1;
        x.h_buf = x.h_start = x.h_count = 0;
        x.forced = -1;
        x.feature = -1;
        x.last = 0;
        x.rescan = 1;
        a.exps[lane] = x;
        const double2 cb = mo.cb[l];
        LeafBounds lb;
        lb.min = cb.x;
        lb.max = cb.y;
        a.bounds[c] = lb;
        // (its expansion, if any, was voided at the start of phase D)
        a.nstate[c] = static_cast<uint8_t>(s_st[c] & ~(kNodeExpanded | kNodeLocal));
      }
      if (lane == 63) s_tiles = inc;
    } else if (!done) {
      // categorical left sets of the expansions (the other waves, concurrently)
      for (int i = t - 64; i < K * kMaxCatWords; i += blockDim.x - 64) {
        const int e = i / kMaxCatWords, wd = i - e * kMaxCatWords;
        const int p = s_exp[e];
        const int cpos = (p >= base && p - base < 2 * kFrontierKmax) ? s_cpos[p - base] : -1;
        a.exp_bits[i] = cpos >= 0 ? a.cinfo[cpos].cat_bitset[wd] : a.best[p].cat_bitset[wd];
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    FState ns_ = st;
    ns_.round = st.round + 1;
    ns_.num_leaves = nl;
    ns_.num_splits = ns;
    ns_.done = done;
    ns_.blocked = s_blocked;
    ns_.forced_next = s_fnext;
    ns_.byn = s_byn;
    ns_.byn_rng = s_brng;
    ns_.nsal = done ? 0 : s_nsal;
    if (!done) {
      ns_.k = s_k + (kMono ? s_nr : 0);
      ns_.kx = s_k;
      ns_.total_tiles = s_tiles;
      ns_.epoch = st.epoch + 1u;
      ns_.cid_next = cid_next + 2 * s_k;
      ns_.spec = st.spec + s_k;
    } else {
      ns_.k = 0;
      ns_.kx = 0;
      ns_.total_tiles = 0;
    }
    *a.st = ns_;
  }
  FStamp(a, rnd, kFStampSel, 6);
  FStampEnd(a, rnd, kFStampSel);
  if (done) {
    // rows partitioned by committed vs uncommitted expansions (the host's speculation feedback)
    __shared__ unsigned long long s_used, s_waste;
    if (t == 0) {
      s_used = 0ull;
      s_waste = 0ull;
    }
    __syncthreads();
    unsigned long long u = 0ull, wst = 0ull;
    for (int c = t; c < cid_next; c += blockDim.x) {
      const uint8_t sc = s_st[c];
      if (!(sc & kNodeExpanded)) continue;
      // data-parallel: the global count, so every rank steers its speculation the same way
      const unsigned long long cnt = static_cast<unsigned long long>(a.distributed ? a.nodes[c].gcount : a.nodes[c].count);
      if (sc & kNodeCommitted) u += cnt;
      else wst += cnt;
    }
    if (u) atomicAdd(&s_used, u);
    if (wst) atomicAdd(&s_waste, wst);
    __syncthreads();
    if (t == 0) {
      a.st->used_rows = static_cast<long long>(s_used);
      a.st->waste_rows = static_cast<long long>(s_waste);
    }
    for (int l = t; l < nl; l += blockDim.x) {
      const FNode nd = a.nodes[s_lcid[l]];
      LeafRange r;
      r.buf = nd.buf;
      r.start = nd.start;
      r.count = nd.count;
      r.pad = 0;
      a.range_out[l] = r;
    }
  }
}

// ---------------------------------------------------------------------------
// Voting parallel (PV-Tree) on the frontier: after the LOCAL pass of k_f_scan every rank
//  k_f_vote        ranks each child's local candidates (gain desc, feature asc) and writes its
//                  top-k (gain, feature, local rows) records; the candidate table is cleared
//  (all-gather of the records)
//  k_f_elect       GlobalVoting per child (the best record of each feature weighted by its local
//                  rows over the mean rows per rank, top-k of those), then this rank's local
//                  fixed-point rows of the elected features
//  (sum all-reduce of the rows: exact integers, identical on every rank)
//  k_f_vote_scan   the GLOBAL pass: each elected feature scanned from the summed rows with the
//                  global leaf statistics and penalties, into the candidate table the select reads
// Reference: voting_parallel_tree_learner.cpp:243-399 (FindBestSplits, GlobalVoting :150-181).
constexpr int kVoteThreads = 256;

__device__ __forceinline__ bool FVoteBetter(double ga, int fa, double gb, int fb) {
  return ga != gb ? ga > gb : fa < fb;
}

// the child cid of candidate pair q (2 e + sel) of the current round, -1: none / skipped
__device__ __forceinline__ int FPairChild(const FArgs& a, int k, int q) {
  const int e = q >> 1;
  if (e >= k) return -1;
  const FExp& x = a.exps[e];
  if (x.skip) return -1;
  return (q & 1) ? x.larger : x.smaller;
}

__device__ void FVoteBody(const FArgs& a, int k, int q);

__global__ __launch_bounds__(kVoteThreads) void k_f_vote(FArgs a) {
  const FState* stp = a.st;
  const unsigned xep = a.xg ? *a.xc->ep : 0u;
  if (stp->done) return;
  const int k = stp->k, q = blockIdx.x;
  if ((q >> 1) < k) FVoteBody(a, k, q);
  // xGMI: the records are in every rank's table once all ranks arrived (one rank: nothing to wait for)
  if (a.xg && FXPeers(a)) FXArrive(a, kFXVote, FXTag(a, xep + 1u));
}

__device__ void FVoteBody(const FArgs& a, int k, int q) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int F = a.F, K = a.vote_k, t = threadIdx.x;
  const int c = FPairChild(a, k, q);
  double* s_gain = reinterpret_cast<double*>(smem);
  int* s_cnt = reinterpret_cast<int*>(s_gain + F);
  __shared__ int s_n[kVoteThreads / 64];
  int nv = 0;
  for (int f = t; f < F; f += blockDim.x) {
    const size_t o = static_cast<size_t>(q) * F + f;
    const SplitKey kk = a.ckey[o];
    const bool valid = c >= 0 && kk.feature >= 0;
    s_gain[f] = valid ? kk.gain : kMinScore;
    s_cnt[f] = valid ? a.cinfo[o].left_count + a.cinfo[o].right_count : -1;
    nv += valid ? 1 : 0;
  }
  const int nvalid = BlockSumInt(nv, s_n);  // (barrier inside: the LDS arrays are complete)
  // (xGMI: the records go to row `rank` of every rank's table)
  const int npeer = a.xg ? a.xc->P : 1;
  const size_t roff = (static_cast<size_t>(a.vote_rank) * 2 * a.kmax + q) * K;
  // rank of feature f = the valid features ordered before it; one wave per feature, its lanes
  // comparing 64 features at a time (ballot + popcount), stopping once the rank reaches K. (A lane
  // per feature scanning all F serially kept every wave holding a top-K feature in a full F-long
  // loop: 132 us per round at F = 500, GOSS 3M x 500.)
  const int lane = t & 63, wv = t >> 6, nw = static_cast<int>(blockDim.x) >> 6;
  for (int f = wv; f < F; f += nw) {
    if (s_cnt[f] < 0) continue;  // (wave-uniform)
    const double g = s_gain[f];
    int rank = 0;
    for (int j0 = 0; j0 < F && rank < K; j0 += 64) {
      const int j = j0 + lane;
      const bool better = j < F && s_cnt[j] >= 0 && FVoteBetter(s_gain[j], j, g, f);
      rank += __popcll(__ballot(better));
    }
    if (rank < K && lane < npeer) {
      VoteRec r;
      r.gain = g;
      r.feature = f;
      r.count = s_cnt[f];
      if (!a.xg) a.vrec[roff + rank] = r;
      else FXStoreRec(reinterpret_cast<VoteRec*>(a.xc->peer[lane] + a.xc->o_vrec) + roff + rank, r);
    }
  }
  for (int i = nvalid + t; i < K; i += blockDim.x) {
    VoteRec r;
    r.gain = kMinScore;
    r.feature = -1;
    r.count = 0;
    if (!a.xg) a.vrec[roff + i] = r;
    for (int p = 0; a.xg && p < npeer; ++p) FXStoreRec(reinterpret_cast<VoteRec*>(a.xc->peer[p] + a.xc->o_vrec) + roff + i, r);
  }
  // the local candidates are consumed: the global pass fills the elected features' entries
  for (int f = t; f < F; f += blockDim.x) {
    SplitKey& kk = a.ckey[static_cast<size_t>(q) * F + f];
    kk.feature = -1;
    kk.gain = kMinScore;
  }
  if (t == 0 && (q & 1) == 0) {
    a.ltot[2 * (q >> 1)] = 0ull;  // (the round's local totals are consumed: zero for the next round)
    a.ltot[2 * (q >> 1) + 1] = 0ull;
  }
}

// GlobalVoting of one child over the gathered records (identical on every rank): s_list[0, n)
// the elected features ascending; returns n
__device__ int FElect(const FArgs& a, int q, int c, double* s_w, int* s_f, int* s_flag, int* s_tmp, int* s_list) {
  const int K = a.vote_k, P = a.vote_P, R = P * K, t = threadIdx.x;
  // mean child rows per rank in float, as the reference's mean_num_data
  const float mean = static_cast<float>(a.nodes[c].gcount) / static_cast<float>(P);
  for (int i = t; i < R; i += blockDim.x) {
    const int r = i / K, j = i - r * K;
    const VoteRec* vp = a.vrec + (static_cast<size_t>(r) * 2 * a.kmax + q) * K + j;
    const VoteRec v = a.xg ? FXLoadRec(vp) : *vp;
    const double w = v.gain * v.count / static_cast<double>(mean);
    const bool valid = v.feature >= 0 && w > kMinScore;
    s_w[i] = w;
    s_f[i] = valid ? v.feature : -1;
  }
  __syncthreads();
  // the best record of each feature (first in gather order on equal weighted gain)
  for (int i = t; i < R; i += blockDim.x) {
    int best = s_f[i] >= 0 ? 1 : 0;
    for (int j = 0; j < R && best; ++j) {
      if (j != i && s_f[j] == s_f[i] && (s_w[j] > s_w[i] || (s_w[j] == s_w[i] && j < i))) best = 0;
    }
    s_flag[i] = best;
  }
  __syncthreads();
  int ne = 0;
  for (int i = t; i < R; i += blockDim.x) {
    int el = 0;
    if (s_flag[i]) {
      int rank = 0;
      for (int j = 0; j < R && rank < K; ++j) rank += (s_flag[j] && FVoteBetter(s_w[j], s_f[j], s_w[i], s_f[i])) ? 1 : 0;
      el = rank < K ? 1 : 0;
    }
    ne += el;
    s_tmp[i] = el;
  }
  __syncthreads();
  for (int i = t; i < R; i += blockDim.x) s_flag[i] = s_tmp[i];
  const int n = BlockSumInt(ne, s_tmp + R);
  for (int i = t; i < R; i += blockDim.x) {
    if (!s_flag[i]) continue;
    int pos = 0;
    for (int j = 0; j < R; ++j) pos += (s_flag[j] && s_f[j] < s_f[i]) ? 1 : 0;
    s_list[pos] = s_f[i];
  }
  __syncthreads();
  return n;
}

__device__ void FElectBody(const FArgs& a, int k, int q);

__global__ __launch_bounds__(kVoteThreads) void k_f_elect(FArgs a) {
  const FState* stp = a.st;
  const unsigned xep = a.xg ? *a.xc->ep : 0u;
  if (stp->done) return;
  const int k = stp->k, q = blockIdx.x;
  if ((q >> 1) < k) FElectBody(a, k, q);
  // xGMI: every rank's rows are summed into every rank's row block once all ranks arrived
  if (a.xg && FXPeers(a)) FXArrive(a, kFXVRows, FXTag(a, xep + 1u));
}

__device__ void FElectBody(const FArgs& a, int k, int q) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int K = a.vote_k, R = a.vote_P * K, t = threadIdx.x;
  const int c = FPairChild(a, k, q);
  int* el = a.velect + static_cast<size_t>(q) * (K + 1);
  if (q == 0 && a.exps[0].parent < 0 && t == 0) {
    // the root round: the root's GLOBAL output (the local pass computed local ones only)
    const double2 sm = a.lsum[0];
    SplitParams p0 = a.sp;
    p0.path_smooth = 0.0;
    a.lout[0] = LeafOutputRaw(sm.x, sm.y, p0, a.nodes[0].gcount, 0.0);
  }
  if (c < 0) {
    if (t == 0) el[0] = 0;
    return;
  }
  double* s_w = reinterpret_cast<double*>(smem);
  int* s_f = reinterpret_cast<int*>(s_w + R);
  int* s_flag = s_f + R;
  int* s_tmp = s_flag + R;                     // R + kVoteThreads / 64
  int* s_list = s_tmp + R + kVoteThreads / 64;  // [K]
  const int n = FElect(a, q, c, s_w, s_f, s_flag, s_tmp, s_list);
  if (t == 0) el[0] = n;
  for (int j = t; j < n; j += blockDim.x) el[1 + j] = s_list[j];
  // this rank's local rows of the elected features: the child's local fp64 histogram (its node
  // slot) back at the fixed-point scale (the smaller child's slot holds exact integers)
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  double sg = ldexp(1.0, EG), sh = ldexp(1.0, EH);
  if (a.quant) {
    double gs, hs;
    QuantScales(a, &gs, &hs);
    sg = 1.0 / gs;
    sh = 1.0 / hs;
  }
  const size_t row = 2 * static_cast<size_t>(a.max_bin);
  const double* slot = a.slots + static_cast<size_t>(c) * 2 * a.TB;
  for (int j = 0; j < n; ++j) {
    const DevFeature fi = a.feat[s_list[j]];
    const size_t o = (static_cast<size_t>(q) * K + j) * row;
    const double* src = slot + 2 * static_cast<size_t>(fi.hist_offset);
    for (int v = t; v < 2 * (fi.num_bin - 1); v += blockDim.x) {
      const unsigned long long x = static_cast<unsigned long long>(__double2ll_rn(src[v] * ((v & 1) ? sh : sg)));
      if (!a.xg) {
        a.vrows[o + v] = x;  // (summed over ranks in place by the all-reduce)
      } else if (x != 0ull) {
        // xGMI: added into every rank's row block (exact integers; k_f_vote_scan re-zeroes its own)
        for (int p = 0; p < a.xc->P; ++p) FXAdd(reinterpret_cast<unsigned long long*>(a.xc->peer[p] + a.xc->o_vrows) + o + v, x);
      }
    }
  }
}

// one wave per (pair, elected slot)
__global__ __launch_bounds__(64) void k_f_vote_scan(FArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const FState* stp = a.st;
  if (stp->done) return;
  const int K = a.vote_k, k = stp->k, F = a.F, lane = threadIdx.x;
  const int q = blockIdx.x / K, j = blockIdx.x - q * K;
  if ((q >> 1) >= k) return;
  const int c = FPairChild(a, k, q);
  if (c < 0) return;
  const int* el = a.velect + static_cast<size_t>(q) * (K + 1);
  if (j >= el[0]) return;
  const int f = el[1 + j];
  const DevFeature fi = a.feat[f];
  int EG, EH;
  GlobalScaleExp(a, &EG, &EH);
  double inv_g = ldexp(1.0, -EG), inv_h = ldexp(1.0, -EH);
  if (a.quant) QuantScales(a, &inv_g, &inv_h);
  double* H = reinterpret_cast<double*>(smem);                                   // [2 max_bin]
  int* order = reinterpret_cast<int*>(H + 2 * a.max_bin);                         // [cat_p2] (+ pad)
  double* ckey = reinterpret_cast<double*>(order + 2 * a.cat_p2);                 // [cat_p2], 8-byte aligned
  __shared__ __align__(8) unsigned char s_out_raw[sizeof(SplitInfo)];
  SplitInfo* out = reinterpret_cast<SplitInfo*>(s_out_raw);
  const unsigned long long* rows = a.vrows + (static_cast<size_t>(q) * K + j) * 2 * a.max_bin;
  const double2 sums = a.lsum[c];
  const int n = a.nodes[c].gcount;
  double sgs = 0.0, shs = 0.0;
  for (int v = lane; v < 2 * (fi.num_bin - 1); v += 64) {
    const unsigned long long rv = a.xg ? FXLoad64(rows + v) : rows[v];
    const double x = static_cast<double>(static_cast<long long>(rv)) * ((v & 1) ? inv_h : inv_g);
    if (a.xg) FXStore64(const_cast<unsigned long long*>(rows) + v, 0ull);  // (xGMI: the next round adds into it)
    const int kb = v >> 1;
    const int b = kb < fi.mfb ? kb : kb + 1;
    H[2 * b + (v & 1)] = x;
    if (v & 1) shs += x;
    else sgs += x;
  }
  sgs = WaveSum(sgs);
  shs = WaveSum(shs);
  if (lane == 0) {
    H[2 * fi.mfb] = sums.x - sgs;
    H[2 * fi.mfb + 1] = sums.y - shs;
    out->Reset();
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const FNode nd = a.nodes[c];
  double po;
  if (nd.parent < 0) {
    SplitParams p0 = a.sp;
    p0.path_smooth = 0.0;
    po = LeafOutputRaw(sums.x, sums.y, p0, n, 0.0);
  } else {
    po = a.lout[c];
  }
  const LeafBounds bounds = a.bounds[c];
  // extra trees (numerical data, one expansion per round): feature f's stream drew for both children
  // in the local pass; the global pass draws for the smaller child's elected features, then the
  // larger's (host FindBestSplitsFromHistograms order). Both children's items read the stream as
  // the local pass left it: the larger's item replays the smaller's draw first when f was elected
  // for both, and only the item that draws last stores the state back.
  int rt = 0;
  if (a.xrng != nullptr && fi.bin_type == 0) {
    const int sel = q & 1, other = q ^ 1;
    bool both = false;
    if (FPairChild(a, k, other) >= 0) {
      const int* eo = a.velect + static_cast<size_t>(other) * (K + 1);
      for (int i = 0; i < eo[0]; ++i) both = both || eo[1 + i] == f;
    }
    unsigned x = a.xrng[f];
    if (fi.num_bin - 2 > 0) {
      if (sel == 1 && both) (void)LcgNext(&x);
      rt = RandNextInt(&x, 0, fi.num_bin - 2);
    }
    if (lane == 0 && (sel == 1 || !both)) a.xrng[f] = x;
  }
  bool spl;
  if (fi.bin_type == 0) {
    spl = ScanNumericalWave(a.sp, fi, H, sums.x, sums.y, n, po, bounds, rt, out);
  } else {
    FeatureScanMeta m;
    m.num_bin = fi.num_bin;
    m.default_bin = static_cast<uint32_t>(fi.default_bin);
    m.missing_type = fi.missing;
    m.bin_type = fi.bin_type;
    m.monotone = fi.monotone;
    m.penalty = fi.penalty;
    m.rand_threshold = 0;
    spl = ScanCategoricalWave(a.sp, m, H, sums.x, sums.y, n, po, bounds, a.cat_p2, order, ckey, out);
  }
  if (lane == 0) {
    if (!spl || (a.max_depth > 0 && nd.depth >= a.max_depth)) {
      out->Reset();
    } else {
      out->feature = f;
      // CEGB split penalty at the leaf's global count (reference ComputeBestSplitForFeature with
      // GetGlobalDataCountInLeaf), then the monotone penalty
      if (a.cegb_split > 0.0) out->gain -= a.cegb_split * n;
      if (out->monotone_type != 0) out->gain *= MonotonePenaltyAt(a.monotone_penalty, nd.depth);
      if (a.ic && !FIcAllows(a, c, f)) out->Reset();
    }
    SplitKey kk;
    kk.feature = out->feature;
    kk.gain = SafeGain(*out);
    kk.threshold = out->threshold;
    kk.group = fi.group;
    kk.offset = fi.offset;
    kk.num_bin = fi.num_bin;
    kk.mfb = fi.mfb;
    kk.default_bin = fi.default_bin;
    kk.missing = fi.missing;
    kk.default_left = out->default_left;
    kk.is_cat = fi.bin_type != 0 ? 1 : 0;
    kk.pad0 = 0;
    kk.pos = f;
    kk.pad2 = 0;
    a.ckey[static_cast<size_t>(q) * F + f] = kk;
  }
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (int i = lane; i < kInfoWords; i += 64) {
    reinterpret_cast<uint32_t*>(a.cinfo + static_cast<size_t>(q) * F + f)[i] = reinterpret_cast<const uint32_t*>(out)[i];
  }
}

// ---------------------------------------------------------------------------
// Feature parallel: one wave per child pair. k_f_pair_best: this rank's best over its owned
// features' candidates -> fpb[rank]; after the all-gather the select's phase A takes the best over
// the ranks' records (gain desc, then feature asc: the order of the sequential select, so the tree
// equals the one-rank tree).
__global__ __launch_bounds__(64) void k_f_pair_best(FArgs a) {
  const FState* stp = a.st;
  if (stp->done) return;
  const int k = stp->k, q = blockIdx.x, F = a.F, lane = threadIdx.x;
  if ((q >> 1) >= k) return;
  const int c = FPairChild(a, k, q);
  double bg = kMinScore;
  int bf = 0x7fffffff, bp = -1;
  for (int f = lane; f < F && c >= 0; f += 64) {
    // (candidates of features this rank does not own are stale: their items never ran)
    if (a.fowned != nullptr && !a.fowned[f]) continue;
    const SplitKey& kk = a.ckey[static_cast<size_t>(q) * F + f];
    if (kk.feature < 0) continue;
    if (FBetter(kk.gain, kk.feature, 0, bg, bf, 0)) {
      bg = kk.gain;
      bf = kk.feature;
      bp = f;
    }
  }
  const int src = WaveArgBestLane(bg, bf, 0);
  bp = ReadLane(bp, src);
  FPairBest* out = a.fpb + static_cast<size_t>(a.vote_rank) * 2 * a.kmax + q;
  constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  if (bp < 0) {
    if (lane == 0) {
      out->key.feature = -1;
      out->key.gain = kMinScore;
    }
    return;
  }
  const size_t o = static_cast<size_t>(q) * F + bp;
  for (int i = lane; i < kKeyWords + kInfoWords; i += 64) {
    if (i < kKeyWords) reinterpret_cast<uint32_t*>(&out->key)[i] = reinterpret_cast<const uint32_t*>(a.ckey + o)[i];
    else reinterpret_cast<uint32_t*>(&out->info)[i - kKeyWords] = reinterpret_cast<const uint32_t*>(a.cinfo + o)[i - kKeyWords];
  }
}

// xGMI root exchange (one block, once per tree, after k_f_init_root): this rank's root sums and
// gradient bounds -> row `rank` of every peer's root table, the handshake, then every rank folds
// the P rows in rank order (sums: the same fp64 result on every rank; bounds: max, as the
// all-reduces this replaces).
__global__ __launch_bounds__(64) void k_fx_root(FArgs a, unsigned* __restrict__ ghmax) {
  const unsigned xep = *a.xc->ep;
  if (threadIdx.x < a.xc->P) {
    FXRoot mine;
    const double2 s = a.lsum[0];
    mine.g = s.x;
    mine.h = s.y;
    for (int i = 0; i < 4; ++i) mine.m[i] = ghmax[i];
    FXStoreRec(reinterpret_cast<FXRoot*>(a.xc->peer[threadIdx.x] + a.xc->o_root) + a.xc->rank, mine);
  }
  if (FXPeers(a)) FXArrive(a, kFXRoot, FXTag(a, xep + 1u));
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const FXRoot* rows = reinterpret_cast<const FXRoot*>(a.xc->peer[a.xc->rank] + a.xc->o_root);
    double g = 0.0, h = 0.0;
    unsigned m[4] = {0u, 0u, 0u, 0u};
    for (int q = 0; q < a.xc->P; ++q) {
      const FXRoot x = FXLoadRec(rows + q);
      g += x.g;
      h += x.h;
      for (int i = 0; i < 4; ++i) m[i] = max(m[i], x.m[i]);
    }
    a.lsum[0] = make_double2(g, h);
    for (int i = 0; i < 4; ++i) ghmax[i] = m[i];
  }
}

// Set-up self-test of the transport (session 0): round r, every rank adds rank + 1 + r into
// words [half, half + n) of every peer's receive chunk and stores a pattern word into its fpb row
// there; after the handshake k_fx_check verifies its own chunk (sum over ranks) and clears it.
// Halves (of the chunk and of the pattern words) alternate by round, so a rank already pushing
// round r + 1 never touches what a slower peer still checks.
__global__ __launch_bounds__(256) void k_fx_push(FArgs a, int round, int n) {
  const int half = (round & 1) * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    for (int q = 0; q < a.xc->P; ++q) {
      FXAdd(reinterpret_cast<unsigned long long*>(a.xc->peer[q] + a.xc->o_recv) + half + i,
            static_cast<unsigned long long>(a.xc->rank + 1 + round));
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < a.xc->P) {
    FXStore(reinterpret_cast<uint32_t*>(a.xc->peer[threadIdx.x] + a.xc->o_fpb) + (round & 1) * kMaxXRanks + a.xc->rank,
            0xA5000000u + 256u * round + a.xc->rank);
  }
  FXArrive(a, kFXTest, FXTag(a, static_cast<unsigned>(round + 1)));
}
__global__ __launch_bounds__(256) void k_fx_check(FArgs a, int round, int n, unsigned* err) {
  const int half = (round & 1) * n;
  const unsigned long long want =
      static_cast<unsigned long long>(a.xc->P) * (a.xc->P + 1) / 2 + static_cast<unsigned long long>(a.xc->P) * round;
  unsigned long long* rx = reinterpret_cast<unsigned long long*>(a.xc->peer[a.xc->rank] + a.xc->o_recv);
  unsigned bad = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    bad += FXLoad64(rx + half + i) != want ? 1u : 0u;
    FXStore64(rx + half + i, 0ull);
  }
  if (blockIdx.x == 0 && threadIdx.x < a.xc->P) {
    const unsigned v = FXLoad(reinterpret_cast<const uint32_t*>(a.xc->peer[a.xc->rank] + a.xc->o_fpb) + (round & 1) * kMaxXRanks + threadIdx.x);
    bad += v != 0xA5000000u + 256u * round + threadIdx.x ? 1u : 0u;
  }
  if (bad) atomicAdd(err, bad);
}

}  // namespace

// ---------------------------------------------------------------------------
// k_f_results: the replay's state (and, once the tree is done, its split records and leaf
// ranges) into the host-visible results buffer
__global__ __launch_bounds__(1024) void k_f_results(FArgs a, char* out) {
  FResultHdr* h = reinterpret_cast<FResultHdr*>(out);
  const FState st = *a.st;
  const int t = threadIdx.x;
  if (t == 0) {
    h->st = st;
    for (int i = 0; i < 4; ++i) h->bar[i] = a.bar[i];
    h->lout0 = a.lout[0];
  }
  if (t < kFrontierRoundCap) h->kused[t] = a.kused != nullptr ? a.kused[t] : 0;
  if (!st.done) return;
  // the committed splits' records: (leaf, cid) from the selects, SplitInfo and children counts
  // gathered here, into the device records (later device consumers) and the pinned copy
  constexpr int kRecWords = static_cast<int>(sizeof(SplitRec) / 4);
  const int nrec = kRecWords * st.num_splits;
  uint32_t* rec = reinterpret_cast<uint32_t*>(out + FrontierResultRecOffset());
  for (int i = t; i < nrec; i += blockDim.x) {
    const int k = i / kRecWords, j = i - k * kRecWords;
    const int c1 = a.rec[k].pad;
    const int c = c1 >= 0 ? c1 : ~c1;
    uint32_t v;
    if (j == 0) {
      v = static_cast<uint32_t>(a.rec[k].leaf);
    } else if (j == 1 || j == 2) {
      v = static_cast<uint32_t>(a.nodes[a.nodes[c].left + (j - 1)].gcount);
    } else if (j == 3) {
      v = 0u;
    } else {
      v = reinterpret_cast<const uint32_t*>(c1 >= 0 ? a.best + c1 : a.fbest + c)[j - 4];
    }
    rec[i] = v;
    if (j != 0 && j != 3) reinterpret_cast<uint32_t*>(a.rec)[i] = v;  // (leaf / cid words stay)
  }
  const int nrange = static_cast<int>(sizeof(LeafRange) / 4) * st.num_leaves;
  uint32_t* rng = reinterpret_cast<uint32_t*>(out + FrontierResultRangeOffset(a.L));
  for (int i = t; i < nrange; i += blockDim.x) rng[i] = reinterpret_cast<const uint32_t*>(a.range_out)[i];
}

// ---------------------------------------------------------------------------
// launchers

// ---------------------------------------------------------------------------
// CEGB lazy penalties (host CegbPenalty::DeltaGain / OnSplit): per-row feature marks.
// k_f_lazy: block (chunk, e) counts, per feature, the rows of expansion e's smaller child not
// marked for it (earlier trees' marks, and the child's path features counted as marked), and
// writes both children's path masks. k_f_lazy_mark (after a tree): every final leaf's rows
// get the features on its path.
constexpr int kLazyChunks = 64;

__global__ __launch_bounds__(256) void k_f_lazy(FArgs a) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const FState* sp = a.st;
  if (sp->done) return;
  const int e = blockIdx.y;
  if (e >= sp->k) return;
  const FExp x = a.exps[e];
  const int lw = a.lazy_words, F = a.F, t = threadIdx.x;
  uint32_t* s_mask = reinterpret_cast<uint32_t*>(lds_raw);
  int* s_cnt = reinterpret_cast<int*>(s_mask + lw);
  for (int i = t; i < lw; i += blockDim.x) {
    uint32_t m = x.parent >= 0 ? a.npath[static_cast<size_t>(x.parent) * lw + i] : 0u;
    if (x.feature >= 0 && (x.feature >> 5) == i) m |= 1u << (x.feature & 31);
    if (i == lw - 1 && (F & 31) != 0) m |= ~0u << (F & 31);  // bits past F: never counted
    s_mask[i] = m;
    if (blockIdx.x == 0) {
      a.npath[static_cast<size_t>(x.smaller) * lw + i] = m;
      if (x.larger >= 0) a.npath[static_cast<size_t>(x.larger) * lw + i] = m;
    }
  }
  // (children of a skipped expansion cannot split: their path masks are all they need, for
  // the marks after the tree)
  if (x.skip) return;
  for (int f = t; f < F; f += blockDim.x) s_cnt[f] = 0;
  __syncthreads();
  const int n = x.h_count;
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int rb = blockIdx.x * chunk, re = min(n, rb + chunk);
  for (int p = rb + t; p < re; p += blockDim.x) {
    const int row = FRowAt(a, x.h_buf, x.h_start + p);
    const uint32_t* bits = a.lazy_bits + static_cast<size_t>(row) * lw;
    for (int i = 0; i < lw; ++i) {
      uint32_t u = ~(bits[i] | s_mask[i]);
      while (u) {
        const int b = __ffs(u) - 1;
        atomicAdd(&s_cnt[(i << 5) + b], 1);
        u &= u - 1u;
      }
    }
  }
  __syncthreads();
  for (int f = t; f < F; f += blockDim.x) {
    if (s_cnt[f]) atomicAdd(&a.lazy_acc[static_cast<size_t>(e) * F + f], s_cnt[f]);
  }
}

__global__ __launch_bounds__(256) void k_f_lazy_mark(FArgs a) {
  const int l = blockIdx.y;
  if (!a.st->done || l >= a.st->num_leaves) return;
  const int c = a.leaf_cid[l];
  const LeafRange r = a.range_out[l];
  const int lw = a.lazy_words;
  const uint32_t* m = a.npath + static_cast<size_t>(c) * lw;
  const int chunk = (r.count + gridDim.x - 1) / gridDim.x;
  const int rb = blockIdx.x * chunk, re = min(r.count, rb + chunk);
  for (int p = rb + threadIdx.x; p < re; p += blockDim.x) {
    const int row = FRowAt(a, r.buf, r.start + p);
    uint32_t* bits = a.lazy_bits + static_cast<size_t>(row) * lw;
    for (int i = 0; i < lw; ++i) bits[i] |= m[i];
  }
}

void LaunchFrontierResults(const FArgs& a, void* host_out, hipStream_t s) {
  k_f_results<<<1, 1024, 0, s>>>(a, static_cast<char*>(host_out));  // (gathers the tree's records)
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierLazyCounts(const FArgs& a, hipStream_t s) {
  const size_t lds = sizeof(uint32_t) * a.lazy_words + sizeof(int) * a.F;
  k_f_lazy<<<dim3(kLazyChunks, a.kmax), 256, lds, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierLazyMark(const FArgs& a, hipStream_t s) {
  k_f_lazy_mark<<<dim3(16, a.L), 256, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierInitRoot(const FArgs& a, const double* root_part, int nblocks, unsigned* ghmax, hipStream_t s) {
  k_f_init_root<<<1, 256, 0, s>>>(a, root_part, nblocks, ghmax);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierInit(const FArgs& a, hipStream_t s) {
  k_f_init<<<1, 256, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

template <int THREADS>
void LaunchHistT(const FArgs& a, size_t lds, hipStream_t s) {
  // working blocks <= max(hist_grid, ceil(hist_grid / 2) + ke): see the chunking in k_f_hist
  const dim3 grid(FrontierHistRows(a.hist_grid, a.kmax), a.num_tiles);
  if (a.hist_nib) {
    // 4-bit rows (every group <= 16 bins, one LDS tile)
    if (a.quant && a.qsub > 0) k_f_hist<0, 3, THREADS><<<grid, THREADS, lds, s>>>(a);
    else if (a.quant) k_f_hist<0, 2, THREADS><<<grid, THREADS, lds, s>>>(a);
    else if (a.use_dp) k_f_hist<0, 1, THREADS><<<grid, THREADS, lds, s>>>(a);
    else k_f_hist<0, 0, THREADS><<<grid, THREADS, lds, s>>>(a);
  } else if (a.quant && a.qsub > 0) {
    if (a.width == 1) k_f_hist<1, 3, THREADS><<<grid, THREADS, lds, s>>>(a);
    else k_f_hist<2, 3, THREADS><<<grid, THREADS, lds, s>>>(a);
  } else if (a.quant) {
    if (a.width == 1) k_f_hist<1, 2, THREADS><<<grid, THREADS, lds, s>>>(a);
    else k_f_hist<2, 2, THREADS><<<grid, THREADS, lds, s>>>(a);
  } else if (a.use_dp) {
    if (a.width == 1) k_f_hist<1, 1, THREADS><<<grid, THREADS, lds, s>>>(a);
    else k_f_hist<2, 1, THREADS><<<grid, THREADS, lds, s>>>(a);
  } else {
    if (a.width == 1) k_f_hist<1, 0, THREADS><<<grid, THREADS, lds, s>>>(a);
    else k_f_hist<2, 0, THREADS><<<grid, THREADS, lds, s>>>(a);
  }
  HIP_CHECK(hipGetLastError());
}

// the histograms' slab rows: one per block of k_f_hist's grid
int FrontierHistRows(int hist_grid, int kmax) { return std::max(hist_grid, hist_grid / 2 + hist_grid % 2 + kmax); }

void LaunchFrontierHist(const FArgs& a, size_t lds, hipStream_t s) {
  if (a.hist_threads == 1024) LaunchHistT<1024>(a, lds, s);
  else LaunchHistT<512>(a, lds, s);
  // the partial rows' reduction (same MODE precedence as the histogram: quantized levels, then
  // gpu_use_dp's 64-bit pairs, then the fixed-point packed words)
  const int grid = std::max(1, std::min(a.red_grid, 4096));
  const bool xg = a.xg && a.own;
  if (a.quant) xg ? k_f_reduce<2, true><<<grid, kRedThreads, 0, s>>>(a) : k_f_reduce<2, false><<<grid, kRedThreads, 0, s>>>(a);
  else if (a.use_dp) xg ? k_f_reduce<1, true><<<grid, kRedThreads, 0, s>>>(a) : k_f_reduce<1, false><<<grid, kRedThreads, 0, s>>>(a);
  else xg ? k_f_reduce<0, true><<<grid, kRedThreads, 0, s>>>(a) : k_f_reduce<0, false><<<grid, kRedThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierScan(const FArgs& a, size_t lds, hipStream_t s) {
  const bool ext = a.voting || a.xrng != nullptr || a.fowned != nullptr || a.mono_inter;
  // (the wave kernel also runs voting's local pass: numerical features, no forced splits; the
  // intermediate-monotone rescans run on the block kernel)
  if (a.scan_wave && (!ext || (a.voting && a.xrng == nullptr && a.fowned == nullptr)) && a.num_forced == 0) {
    // one wave per item, items grid-strided over the RESIDENT blocks: a grid sized for the widest
    // round (up to 2048 blocks) left most blocks without an item in a typical round, dispatched
    // after the resident ones finished (the partition's tail, profiles/r05/ab_notes.md)
    const size_t lds = kFScanWaves * FrontierScanWaveBytes(a.max_bin, a.cat_p2);
    static thread_local size_t cached_lds = 0;
    static thread_local int cached_resident = 0;
    if (cached_lds != lds || cached_resident <= 0) {
      int per_cu = 0, dev = 0, cus = 0;
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_f_scan_w),
                                                             kFScanWaves * 64, lds));
      HIP_CHECK(hipGetDevice(&dev));
      HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      cached_lds = lds;
      cached_resident = std::max(1, per_cu) * std::max(1, cus);
    }
    const int grid = std::max(1, std::min({(a.kmax * a.F + kFScanWaves - 1) / kFScanWaves, 2048, cached_resident}));
    k_f_scan_w<<<grid, kFScanWaves * 64, lds, s>>>(a);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const int grid = std::max(1, std::min(a.kmax * a.F, a.scan_grid > 0 ? a.scan_grid : 4096));
  if (ext) k_f_scan<true><<<grid, kFScanThreads, lds, s>>>(a);
  else k_f_scan<false><<<grid, kFScanThreads, lds, s>>>(a);
  HIP_CHECK(hipGetLastError());
}


void LaunchFrontierSelect(const FArgs& a, hipStream_t s) {
  const size_t lds = FrontierSelectLds(a.C, a.L);
  const bool wide = a.F > 64 || (a.fpb != nullptr && a.vote_P > 64);
  if (a.cegb_raw) {
    k_f_select<true, false, false, false><<<1, kFSelThreads, lds + (a.byn_draw != nullptr ? 2 : 1) * (a.F + 16), s>>>(a);
  } else if (a.mono_inter) {
    const size_t ml = lds + FrontierSelectMonoLds(a.C, a.L, a.F);
    wide ? k_f_select<false, true, false, true><<<1, kFSelThreads, ml, s>>>(a) : k_f_select<false, false, false, true><<<1, kFSelThreads, ml, s>>>(a);
  } else if (a.xg) {
    wide ? k_f_select<false, true, true, false><<<1, kFSelThreads, lds, s>>>(a) : k_f_select<false, false, true, false><<<1, kFSelThreads, lds, s>>>(a);
  } else if (wide) {
    k_f_select<false, true, false, false><<<1, kFSelThreads, lds, s>>>(a);
  } else {
    k_f_select<false, false, false, false><<<1, kFSelThreads, lds, s>>>(a);
  }
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierVote(const FArgs& a, hipStream_t s) {
  const size_t lds = static_cast<size_t>(a.F) * (sizeof(double) + sizeof(int));
  k_f_vote<<<2 * a.kmax, kVoteThreads, lds, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierElect(const FArgs& a, hipStream_t s) {
  const size_t R = static_cast<size_t>(a.vote_P) * a.vote_k;
  const size_t lds = R * (sizeof(double) + 3 * sizeof(int)) + sizeof(int) * (kVoteThreads / 64) + sizeof(int) * a.vote_k + 16;
  k_f_elect<<<2 * a.kmax, kVoteThreads, lds, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierVoteScan(const FArgs& a, size_t lds, hipStream_t s) {
  k_f_vote_scan<<<2 * a.kmax * a.vote_k, 64, lds, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierPairBest(const FArgs& a, hipStream_t s) {
  k_f_pair_best<<<2 * a.kmax, 64, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierXRoot(const FArgs& a, unsigned* ghmax, hipStream_t s) {
  if (a.xc->P > 64) std::abort();  // (kMaxXRanks <= 64: one lane per peer)
  k_fx_root<<<1, 64, 0, s>>>(a, ghmax);
  HIP_CHECK(hipGetLastError());
}

void LaunchFrontierXSelfTest(const FArgs& a, int round, int nvals, unsigned* err, hipStream_t s) {
  k_fx_push<<<4, 256, 0, s>>>(a, round, nvals);
  k_fx_check<<<4, 256, 0, s>>>(a, round, nvals, err);
  HIP_CHECK(hipGetLastError());
}


// resident k_f_partition blocks per CU (occupancy of the instantiation the learner launches)
int FrontierPartitionBlocksPerCU(int iters) {
  int per_cu = 0;
  const void* fn = iters == 4    ? reinterpret_cast<const void*>(k_f_partition<4, 1>)
                   : iters == 16 ? reinterpret_cast<const void*>(k_f_partition<16, 1>)
                                 : reinterpret_cast<const void*>(k_f_partition<8, 1>);
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kFPartThreads, 0));
  return per_cu;
}

// one block per tile (A/B of the tile shapes at 1.25M / 10M rows: 1024-row tiles 884-886 it/s vs
// 855 for two per block, 4096-row tiles at 10M 397.7 vs 394.3 for two 2048-row tiles per block)
void LaunchFrontierPartition(const FArgs& a, int iters, int grid, hipStream_t s) {
  if (iters == 4) k_f_partition<4, 1><<<grid, kFPartThreads, 0, s>>>(a);
  else if (iters == 16) k_f_partition<16, 1><<<grid, kFPartThreads, 0, s>>>(a);
  else k_f_partition<8, 1><<<grid, kFPartThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}


void FrontierSetLds(size_t hist_lds, size_t scan_lds, bool use_dp, int width) {
  (void)use_dp;
  (void)width;
  if (hist_lds > 64 * 1024) {
    const void* fns[24] = {
        reinterpret_cast<const void*>(k_f_hist<0, 0, 512>),  reinterpret_cast<const void*>(k_f_hist<0, 1, 512>),
        reinterpret_cast<const void*>(k_f_hist<0, 2, 512>),  reinterpret_cast<const void*>(k_f_hist<0, 3, 512>),
        reinterpret_cast<const void*>(k_f_hist<0, 0, 1024>), reinterpret_cast<const void*>(k_f_hist<0, 1, 1024>),
        reinterpret_cast<const void*>(k_f_hist<0, 2, 1024>), reinterpret_cast<const void*>(k_f_hist<0, 3, 1024>),
        reinterpret_cast<const void*>(k_f_hist<1, 3, 512>),  reinterpret_cast<const void*>(k_f_hist<2, 3, 512>),
        reinterpret_cast<const void*>(k_f_hist<1, 3, 1024>), reinterpret_cast<const void*>(k_f_hist<2, 3, 1024>),
        reinterpret_cast<const void*>(k_f_hist<1, 0, 512>),  reinterpret_cast<const void*>(k_f_hist<2, 0, 512>),
        reinterpret_cast<const void*>(k_f_hist<1, 1, 512>),  reinterpret_cast<const void*>(k_f_hist<2, 1, 512>),
        reinterpret_cast<const void*>(k_f_hist<1, 2, 512>),  reinterpret_cast<const void*>(k_f_hist<2, 2, 512>),
        reinterpret_cast<const void*>(k_f_hist<1, 0, 1024>), reinterpret_cast<const void*>(k_f_hist<2, 0, 1024>),
        reinterpret_cast<const void*>(k_f_hist<1, 1, 1024>), reinterpret_cast<const void*>(k_f_hist<2, 1, 1024>),
        reinterpret_cast<const void*>(k_f_hist<1, 2, 1024>), reinterpret_cast<const void*>(k_f_hist<2, 2, 1024>)};
    for (const void* fn : fns) {
      HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(hist_lds)));
    }
  }
  if (scan_lds > 64 * 1024) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_f_scan<false>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(scan_lds)));
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_f_scan<true>), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  static_cast<int>(scan_lds)));
  }
  // (the wave kernel: four waves' histograms; the learner uses it only when they fit 150 KB)
  HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_f_scan_w), hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(std::min<size_t>(150 * 1024, 4 * scan_lds))));
}

}  // namespace device
}  // namespace lgap
