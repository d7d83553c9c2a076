// Device row sampling (see sample_kernels.h). Host twin and reference:
// src/boosting/sample_strategy.cpp, ref:src/boosting/bagging.hpp:230-270,
// ref:src/boosting/goss.hpp:118-167.
//
// One 256-thread workgroup per 4096-row tile, 16 rows per thread in registers:
//   k_sample_count    per-tile decision (bagging draws / GOSS radix selects) and kept count
//   k_sample_scatter  tile prefix from the counts, stable ballot compaction of the kept
//                     rows, GOSS scaling of the sampled rows, bagging stream advance
// Two launches over the rows and no host round trip besides the final count.
#include "device/sample_kernels.h"

#include <vector>

#include "device/hip_common.h"
#include "lgap/device_api.h"
#include "lgap/random.h"

namespace lgap {
namespace device {

namespace {

constexpr int kThreads = 256;
constexpr int kPer = kSampleTile / kThreads;  // rows per thread
constexpr int kWaves = kThreads / kWave;

// Bagging decision of row i: SampleStrategy::BagBlock's draw, jumped to directly.
__device__ __forceinline__ bool BagKeep(const SampleArgs& a, int i) {
  // by query: every row of query u shares the query's draw (u-th unit of the streams)
  if (a.mode == 4) i = a.row_unit[i];
  const unsigned s = a.rng[i / kSampleRandBlock];
  const uint2 j = a.jump[i % kSampleRandBlock];
  const unsigned x = j.x * s + j.y;
  // float draw compared in double, exactly as the host (float r < double fraction)
  const double r = static_cast<double>(static_cast<float>((x >> 16) & 0x7FFFu) / 32768.0f);
  if (a.mode == 2) return a.label[i] > 0.f ? r < a.pos_fraction : r < a.neg_fraction;
  return r < a.fraction;
}

__device__ __forceinline__ float GossImportance(const SampleArgs& a, int i) {
  float s = 0.f;
  for (int k = 0; k < a.K; ++k) {
    const float2 v = a.gh[static_cast<size_t>(k) * a.N + i];
    s += fabsf(v.x * v.y);
  }
  return s;
}

__device__ int BlockSum(int v, int* sh) {
  v = WaveSum(v);
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) sh[threadIdx.x / kWave] = v;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) s += sh[w];
  return s;
}

// k-th largest (largest) or k-th smallest value among the flagged entries of the
// tile (16 per thread): MSB-first radix select over four 8-bit digits with an LDS
// digit histogram; wave 0 locates the digit with a wave scan. 1 <= k <= #flagged.
__device__ uint32_t TileSelect(const uint32_t (&v)[kPer], uint32_t flags, int k, bool largest, int* hist, int* sh) {
  uint32_t prefix = 0u, pmask = 0u;
  const int t = threadIdx.x;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[t] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      if (((flags >> q) & 1u) && (v[q] & pmask) == prefix) atomicAdd(&hist[(v[q] >> shift) & 255u], 1);
    }
    __syncthreads();
    if (t < kWave) {
      int c[4], s = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        c[q] = hist[largest ? 255 - (4 * t + q) : 4 * t + q];
        s += c[q];
      }
      const int incl = WaveInclusiveScan(s);
      const unsigned long long m = __ballot(incl >= k);
      const int first = __ffsll(static_cast<unsigned long long>(m)) - 1;
      if (t == first) {
        int acc = incl - s;
        for (int q = 0; q < 4; ++q) {
          if (acc + c[q] >= k) {
            sh[0] = largest ? 255 - (4 * t + q) : 4 * t + q;
            sh[1] = k - acc;
            break;
          }
          acc += c[q];
        }
      }
    }
    __syncthreads();
    prefix |= static_cast<uint32_t>(sh[0]) << shift;
    pmask |= 255u << shift;
    k = sh[1];
    __syncthreads();
  }
  return prefix;
}

// GOSS key modes of a tile
constexpr unsigned kKeyNone = 0u, kKeyAll = 1u, kKeyThreshold = 2u;

__global__ __launch_bounds__(kThreads) void k_sample_count(SampleArgs a) {
  __shared__ int hist[256];
  __shared__ int sh[kWaves > 2 ? kWaves : 2];
  const int t = threadIdx.x;
  const int base = blockIdx.x * kSampleTile;
  const int cnt = min(kSampleTile, a.N - base);
  int keep = 0;
  if (a.mode != 3) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = base + q * kThreads + t;
      if (i < a.N && BagKeep(a, i)) ++keep;
    }
    keep = BlockSum(keep, sh);
    if (t == 0) a.tile_cnt[blockIdx.x] = keep;
    return;
  }
  uint32_t v[kPer];
  uint32_t valid = 0u;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int i = base + q * kThreads + t;
    v[q] = 0u;
    if (i < a.N) {
      v[q] = __float_as_uint(GossImportance(a, i));  // non-negative floats order as their bits
      valid |= 1u << q;
    }
  }
  const int top_k = max(1, static_cast<int>(cnt * a.top_rate));
  const int other_k = static_cast<int>(cnt * a.other_rate);
  const uint32_t thr = TileSelect(v, valid, top_k, true, hist, sh);
  int big = 0;
  uint32_t rest_flags = 0u;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (!((valid >> q) & 1u)) continue;
    if (v[q] >= thr) ++big;
    else rest_flags |= 1u << q;
  }
  big = BlockSum(big, sh);
  const int rest = cnt - big;
  unsigned mode = kKeyNone, kthr = 0u;
  int sampled = 0;
  if (other_k > 0 && rest > 0) {
    if (other_k >= rest) {
      mode = kKeyAll;
      sampled = rest;
    } else {
      uint32_t key[kPer];
#pragma unroll
      for (int q = 0; q < kPer; ++q) key[q] = Hash32(a.seed, static_cast<uint32_t>(base + q * kThreads + t));
      kthr = TileSelect(key, rest_flags, other_k, false, hist, sh);
      mode = kKeyThreshold;
      int s = 0;
#pragma unroll
      for (int q = 0; q < kPer; ++q) s += (((rest_flags >> q) & 1u) && key[q] <= kthr) ? 1 : 0;
      sampled = BlockSum(s, sh);
    }
  }
  if (t == 0) {
    a.tile_cnt[blockIdx.x] = big + sampled;
    unsigned* sel = a.tile_sel + 4 * static_cast<size_t>(blockIdx.x);
    sel[0] = thr;
    sel[1] = kthr;
    sel[2] = mode;
    const float mul = other_k > 0 ? static_cast<float>(cnt - top_k) / other_k : 1.0f;
    sel[3] = __float_as_uint(mul);
  }
}

__global__ __launch_bounds__(kThreads) void k_sample_scatter(SampleArgs a, int ntiles) {
  __shared__ int sh[kWaves > 2 ? kWaves : 2];
  __shared__ int s_w[kPer][kWaves];
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
  const int tile = blockIdx.x;
  const int base = tile * kSampleTile;
  int pre = 0;
  for (int i = t; i < tile; i += kThreads) pre += a.tile_cnt[i];
  pre = BlockSum(pre, sh);
  if (tile == ntiles - 1 && t == 0) *a.total = pre + a.tile_cnt[tile];
  bool keep[kPer], samp[kPer];
  if (a.mode != 3) {
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = base + q * kThreads + t;
      keep[q] = i < a.N && BagKeep(a, i);
      samp[q] = false;
    }
  } else {
    const unsigned* sel = a.tile_sel + 4 * static_cast<size_t>(tile);
    const uint32_t thr = sel[0], kthr = sel[1], mode = sel[2];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int i = base + q * kThreads + t;
      keep[q] = samp[q] = false;
      if (i >= a.N) continue;
      if (__float_as_uint(GossImportance(a, i)) >= thr) {
        keep[q] = true;
      } else if (mode == kKeyAll || (mode == kKeyThreshold && Hash32(a.seed, static_cast<uint32_t>(i)) <= kthr)) {
        keep[q] = samp[q] = true;
      }
    }
  }
  // stable order = ascending row = q-major, then thread
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (kWave - lane));
  unsigned long long mk[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    mk[q] = __ballot(keep[q]);
    if (lane == 0) s_w[q][w] = __popcll(mk[q]);
  }
  __syncthreads();
  int off = pre;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
      before += k < w ? s_w[q][k] : 0;
      all += s_w[q][k];
    }
    const int i = base + q * kThreads + t, kb = off + before + __popcll(mk[q] & lt);  // kept rows before i
    if (keep[q]) a.out[kb] = i;
    else if (a.oob != nullptr && i < a.N) a.oob[i - kb] = i;
    off += all;
  }
  if (a.mode == 3) {
    const float mul = __uint_as_float(a.tile_sel[4 * static_cast<size_t>(tile) + 3]);
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      if (!samp[q]) continue;
      const int i = base + q * kThreads + t;
      for (int k = 0; k < a.K; ++k) {
        float2& v = a.gh[static_cast<size_t>(k) * a.N + i];
        v.x *= mul;
        v.y *= mul;
      }
    }
  } else if (a.mode != 4) {
    // every draw of this tile's streams is consumed: advance them (this block alone owns them)
    __syncthreads();
    constexpr int kStreams = kSampleTile / kSampleRandBlock;
    if (t < kStreams) {
      const int b = tile * kStreams + t;
      const int rows = min(kSampleRandBlock, a.N - b * kSampleRandBlock);
      if (rows > 0) {
        const uint2 j = a.jump[rows - 1];
        a.rng[b] = j.x * a.rng[b] + j.y;
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_sample_advance_units(SampleArgs a) {
  const int b = blockIdx.x * kThreads + threadIdx.x;
  const int units = min(kSampleRandBlock, a.num_units - b * kSampleRandBlock);
  if (units > 0) {
    const uint2 j = a.jump[units - 1];
    a.rng[b] = j.x * a.rng[b] + j.y;
  }
}

}  // namespace

void LaunchSampleAdvanceUnits(const SampleArgs& a, hipStream_t s) {
  const int streams = (a.num_units + kSampleRandBlock - 1) / kSampleRandBlock;
  if (streams <= 0) return;
  k_sample_advance_units<<<(streams + kThreads - 1) / kThreads, kThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchSampleCount(const SampleArgs& a, hipStream_t s) {
  const int nt = SampleTiles(a.N);
  if (nt == 0) return;
  k_sample_count<<<nt, kThreads, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

void LaunchSampleScatter(const SampleArgs& a, hipStream_t s) {
  const int nt = SampleTiles(a.N);
  if (nt == 0) return;
  k_sample_scatter<<<nt, kThreads, 0, s>>>(a, nt);
  HIP_CHECK(hipGetLastError());
}

int SampleRowsOnDevice(int mode, int num_rows, int num_class, float* grad, float* hess, const float* label,
                       double fraction, double pos_fraction, double neg_fraction, double top_rate, double other_rate,
                       int bagging_seed, uint32_t goss_seed, int rounds, int* out_rows) {
  if (mode < 1 || mode > 3) Log::Fatal("SampleRowsOnDevice: mode must be 1, 2 or 3");
  if (num_rows <= 0) return 0;
  const size_t n = static_cast<size_t>(num_rows), nk = n * std::max(1, num_class);
  const int nt = SampleTiles(num_rows);
  std::vector<float2> gh(nk);
  for (size_t i = 0; i < nk; ++i) gh[i] = make_float2(grad ? grad[i] : 0.f, hess ? hess[i] : 0.f);
  std::vector<uint2> jt(kSampleRandBlock);
  BuildLcgJumpTable(jt.data());
  std::vector<unsigned> st((n + kSampleRandBlock - 1) / kSampleRandBlock);
  for (size_t b = 0; b < st.size(); ++b) st[b] = static_cast<unsigned>(bagging_seed + static_cast<int>(b));
  DevBuf<float2> d_gh;
  DevBuf<uint2> d_jump;
  DevBuf<unsigned> d_rng, d_sel(4 * static_cast<size_t>(nt));
  DevBuf<int> d_cnt(nt), d_out(n), d_total(1);
  DevBuf<float> d_label;
  d_gh.Upload(gh);
  d_jump.Upload(jt);
  d_rng.Upload(st);
  if (mode == 2) {
    if (!label) Log::Fatal("SampleRowsOnDevice: balanced bagging needs labels");
    d_label.Upload(label, n);
  }
  SampleArgs a;
  a.mode = mode;
  a.N = num_rows;
  a.K = std::max(1, num_class);
  a.fraction = fraction;
  a.pos_fraction = pos_fraction;
  a.neg_fraction = neg_fraction;
  a.top_rate = top_rate;
  a.other_rate = other_rate;
  a.seed = goss_seed;
  a.label = d_label.get();
  a.gh = d_gh.get();
  a.rng = d_rng.get();
  a.jump = d_jump.get();
  a.tile_cnt = d_cnt.get();
  a.tile_sel = d_sel.get();
  a.out = d_out.get();
  a.total = d_total.get();
  for (int r = 0; r < std::max(1, rounds); ++r) {
    LaunchSampleCount(a, 0);
    LaunchSampleScatter(a, 0);
  }
  int total = 0;
  d_total.Download(&total, 1);
  HIP_CHECK(hipDeviceSynchronize());
  if (total < 0 || total > num_rows) Log::Fatal("SampleRowsOnDevice: invalid count %d", total);
  d_out.Download(out_rows, total);
  d_gh.Download(gh.data(), nk);
  HIP_CHECK(hipDeviceSynchronize());
  for (size_t i = 0; i < nk; ++i) {
    if (grad) grad[i] = gh[i].x;
    if (hess) hess[i] = gh[i].y;
  }
  return total;
}

void BuildLcgJumpTable(uint2* out) {
  uint32_t A = 1u, C = 0u;
  for (int j = 0; j < kSampleRandBlock; ++j) {
    A = 214013u * A;
    C = 214013u * C + 2531011u;
    out[j] = make_uint2(A, C);
  }
}

}  // namespace device
}  // namespace lgap
