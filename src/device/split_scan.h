// Device-side split finding shared by the HIP learners (device_learner.hip: sequential
// per-split chain; frontier_kernels.hip: batched frontier rounds): split predicates on
// packed group bins, wave-parallel numerical / categorical threshold scans over a full
// feature histogram in LDS, and small wave/block helpers.
//
// Reference semantics: feature_histogram.hpp:830-1057 (numerical scans, missing
// handling, tie rules), feature_histogram.cpp:144-739 (categorical one-hot and
// ctr-sorted scans); the host oracle of the same math is lgap/split_math.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "device/hip_common.h"
#include "device/tree_kernels.h"
#include "lgap/split_math.h"

namespace lgap {
namespace device {
namespace {

#ifndef LGAP_SCAN_K
#define LGAP_SCAN_K 2
#endif
constexpr int kScanK = LGAP_SCAN_K;  // consecutive bins per lane in the numerical threshold scan

__device__ __forceinline__ uint32_t DecodeBin(int offset, int num_bin, int mfb, uint32_t gb) {
  const int local = static_cast<int>(gb) - offset;
  if (local < 0 || local >= num_bin - 1) return static_cast<uint32_t>(mfb);
  return static_cast<uint32_t>(local < mfb ? local : local + 1);
}

struct SplitDesc {
  int group, offset, num_bin, mfb, default_bin, missing, thr, default_left, is_cat;
  uint32_t bits[kMaxCatWords];
};

__device__ __forceinline__ bool GoLeft(const SplitDesc& d, uint32_t gb) {
  const uint32_t b = DecodeBin(d.offset, d.num_bin, d.mfb, gb);
  if (d.is_cat) {
    const uint32_t w = b >> 5;
    return w < static_cast<uint32_t>(kMaxCatWords) && ((d.bits[w] >> (b & 31u)) & 1u);
  }
  if ((d.missing == 1 && b == static_cast<uint32_t>(d.default_bin)) ||
      (d.missing == 2 && b == static_cast<uint32_t>(d.num_bin - 1))) {
    return d.default_left != 0;
  }
  return b <= static_cast<uint32_t>(d.thr);
}

// block = 256 threads: sum of an int
__device__ int BlockSumInt(int v, int* sh) {
  v = WaveSum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  int s = 0;
  for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) s += sh[i];
  return s;
}

__device__ __forceinline__ double SafeGain(const SplitInfo& s) {
  double g = s.gain;
  if (g != g) g = kMinScore;
  return s.feature < 0 ? kMinScore : g;
}

__device__ __forceinline__ unsigned LcgNext(unsigned* x) {
  *x = 214013u * *x + 2531011u;
  return *x;
}
__device__ __forceinline__ int RandNextInt(unsigned* x, int lo, int hi) {
  const int v = static_cast<int>(LcgNext(x) & 0x7FFFFFFFu);
  return v % (hi - lo) + lo;
}

__device__ double MonotonePenaltyAt(double pen, int depth) {
  if (pen >= depth + 1.0) return kEpsilon;
  if (pen <= 1.0) return 1.0 - pen / pow(2.0, static_cast<double>(depth)) + kEpsilon;
  return 1.0 - pow(2.0, pen - 1.0 - depth) + kEpsilon;
}

// largest power of two <= x (x > 0)
__device__ __forceinline__ double Pow2AtMost(double x) {
  int e;
  (void)frexp(x, &e);  // x = m * 2^e, m in [0.5, 1)
  return ldexp(1.0, e - 1);
}

struct Cand {
  double gain, lg, lh;
  int lc, thr;
};

// wave argmax; prefer_high: ties go to the larger threshold
__device__ __forceinline__ Cand WaveBest(Cand c, bool prefer_high) {
  const int src = WaveArgBestLane(c.gain, prefer_high ? -c.thr : c.thr, 0);
  Cand r;
  r.gain = ReadLane(c.gain, src);
  r.thr = ReadLane(c.thr, src);
  r.lg = ReadLane(c.lg, src);
  r.lh = ReadLane(c.lh, src);
  r.lc = ReadLane(c.lc, src);
  return r;
}

// Numerical threshold search of one wave over a FULL feature histogram H
// (LDS, num_bin (g, h) pairs, most-frequent bin included). Same semantics as
// FindBestNumerical (split_math.h / feature_histogram.hpp:830-1057): reverse
// pass (right side grows from the top bin) and, with missing values, the
// forward pass; SKIP_DEFAULT_BIN / NA_AS_MISSING as masks; first-max tie rules.
// Returns splittable; lane 0's `out` holds the result.
__device__ bool ScanNumericalWave(const SplitParams& p, const DevFeature& fi, const double* H, double sg, double sh_raw,
                                  int n, double po, const LeafBounds& bounds, int rand_thr, SplitInfo* out) {
  const int lane = threadIdx.x & 63;
  const double sum_h = sh_raw + 2 * kEpsilon;
  const double cnt_factor = n / sum_h;
  const double shift = LeafGain(sg, sum_h, p, n, po) + p.min_gain_to_split;
  const int nb = fi.num_bin;
  const bool two_dir = nb > 2 && fi.missing != 0;
  const bool skip_def = two_dir && fi.missing == 1;
  const bool na = two_dir && fi.missing == 2;
  const int top = nb - 1 - (na ? 1 : 0);
  const bool use_rand = p.extra_trees != 0;
  const int8_t mono = fi.monotone;
  // Each lane owns kScanK consecutive positions of a 64 * kScanK chunk: a serial
  // prefix over its own bins, ONE wave scan of the lane totals per chunk, then the
  // kScanK thresholds are evaluated independently (one 256-bin chunk covers max_bin
  // 255: one wave scan per pass instead of four). Position order = scan order; within
  // a lane the first (strict >) best is kept, across lanes WaveBest applies the same
  // tie rule, so the winner is the scan's first maximum as in the host scan.
  constexpr int K = kScanK;
  Cand rb;
  rb.gain = kMinScore;
  rb.thr = -1;
  rb.lg = rb.lh = 0.0;
  rb.lc = 0;
  bool sp = false;
  double cg = 0.0, ch = 0.0;
  int cc = 0;
  // An empty bin leaves the prefix unchanged: the threshold after it has the same partition
  // and gain as the one before, and the host scan keeps the first of such exact ties. The
  // parallel prefix may round the two positions differently, so empty-bin positions after
  // the first evaluated one are skipped (the host rule, independent of summation order).
  // (extra trees evaluate ONE threshold, the random one: an empty bin there is still a split,
  // so nothing is skipped)
  const int first_rev = use_rand ? -1 : (skip_def && top == fi.default_bin) ? top - 1 : top;
  const int first_fwd = use_rand ? 0x7fffffff : (skip_def && fi.default_bin == 0) ? 1 : 0;
  // reverse pass: position i <-> bin nb - 1 - i (the right side grows from the top bin)
  for (int base = 0; base < nb; base += 64 * K) {
    double pg[K], ph[K];
    int pc[K];
    bool empty[K];
    double tg = 0.0, th = 0.0;
    int tc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int b = nb - 1 - (base + lane * K + k);
      double g = 0.0, h = 0.0;
      int c = 0;
      if (b >= 0 && !(skip_def && b == fi.default_bin) && !(na && b == nb - 1)) {
        g = H[2 * b];
        h = H[2 * b + 1];
        c = RoundCount(h * cnt_factor);
      }
      empty[k] = g == 0.0 && h == 0.0;
      tg += g;
      th += h;
      tc += c;
      pg[k] = tg;
      ph[k] = th;
      pc[k] = tc;
    }
    const double ig = WaveInclusiveSumDpp(tg), ih = WaveInclusiveSumDpp(th);
    const int ic = WaveInclusiveSumDpp(tc);
    const double eg = cg + ig - tg, eh = ch + ih - th;
    const int ec = cc + ic - tc;
    cg += ReadLane(ig, 63);
    ch += ReadLane(ih, 63);
    cc += ReadLane(ic, 63);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int b = nb - 1 - (base + lane * K + k);
      if (b >= 1 && b <= top && !(skip_def && b == fi.default_bin) && !(b < first_rev && empty[k])) {
        const int thr = b - 1;
        const double rg = eg + pg[k];
        const double rh = kEpsilon + eh + ph[k];
        const int rc = ec + pc[k];
        const int lc = n - rc;
        const double lh = sum_h - rh;
        if (rc >= p.min_data_in_leaf && rh >= p.min_sum_hessian_in_leaf && lc >= p.min_data_in_leaf &&
            lh >= p.min_sum_hessian_in_leaf && (!use_rand || thr == rand_thr)) {
          const double lg = sg - rg;
          const double gain = SplitGain(lg, lh, rg, rh, p, mono, lc, rc, po, bounds);
          if (gain > shift) {
            sp = true;
            if (gain > rb.gain) {
              rb.gain = gain;
              rb.thr = thr;
              rb.lg = lg;
              rb.lh = lh;
              rb.lc = lc;
            }
          }
        }
      }
    }
  }
  Cand fb;
  fb.gain = kMinScore;
  fb.thr = 0x7fffffff;
  fb.lg = fb.lh = 0.0;
  fb.lc = 0;
  if (two_dir) {
    // forward pass: position i <-> bin i (the left side grows from bin 0)
    cg = ch = 0.0;
    cc = 0;
    for (int base = 0; base < nb; base += 64 * K) {
      double pg[K], ph[K];
      int pc[K];
      bool empty[K];
      double tg = 0.0, th = 0.0;
      int tc = 0;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int b = base + lane * K + k;
        double g = 0.0, h = 0.0;
        int c = 0;
        if (b < nb && !(skip_def && b == fi.default_bin)) {
          g = H[2 * b];
          h = H[2 * b + 1];
          c = RoundCount(h * cnt_factor);
        }
        empty[k] = g == 0.0 && h == 0.0;
        tg += g;
        th += h;
        tc += c;
        pg[k] = tg;
        ph[k] = th;
        pc[k] = tc;
      }
      const double ig = WaveInclusiveSumDpp(tg), ih = WaveInclusiveSumDpp(th);
      const int ic = WaveInclusiveSumDpp(tc);
      const double eg = cg + ig - tg, eh = ch + ih - th;
      const int ec = cc + ic - tc;
      cg += ReadLane(ig, 63);
      ch += ReadLane(ih, 63);
      cc += ReadLane(ic, 63);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int b = base + lane * K + k;
        if (b <= nb - 2 && !(skip_def && b == fi.default_bin) && !(b > first_fwd && empty[k])) {
          const int thr = b;
          const double lg = eg + pg[k];
          const double lh = kEpsilon + eh + ph[k];
          const int lc = ec + pc[k];
          const int rc = n - lc;
          const double rh = sum_h - lh;
          if (lc >= p.min_data_in_leaf && lh >= p.min_sum_hessian_in_leaf && rc >= p.min_data_in_leaf &&
              rh >= p.min_sum_hessian_in_leaf && (!use_rand || thr == rand_thr)) {
            const double rg = sg - lg;
            const double gain = SplitGain(lg, lh, rg, rh, p, mono, lc, rc, po, bounds);
            if (gain > shift) {
              sp = true;
              if (gain > fb.gain) {
                fb.gain = gain;
                fb.thr = thr;
                fb.lg = lg;
                fb.lh = lh;
                fb.lc = lc;
              }
            }
          }
        }
      }
    }
  }
  const bool any = __any(sp) != 0;
  const Cand r = WaveBest(rb, true);
  const Cand f = two_dir ? WaveBest(fb, false) : fb;
  if (lane == 0) {
    out->Reset();
    out->monotone_type = fi.monotone;
    out->default_left = 1;
    if (any) {
      Cand w = r;
      int dl = 1;
      if (two_dir && f.gain > r.gain) {
        w = f;
        dl = 0;
      }
      if (w.gain > kMinScore) {
        out->threshold = static_cast<uint32_t>(w.thr);
        out->left_output = LeafOutput(w.lg, w.lh, p, w.lc, po, bounds);
        out->left_count = w.lc;
        out->left_sum_gradient = w.lg;
        out->left_sum_hessian = w.lh - kEpsilon;
        out->right_output = LeafOutput(sg - w.lg, sum_h - w.lh, p, n - w.lc, po, bounds);
        out->right_count = n - w.lc;
        out->right_sum_gradient = sg - w.lg;
        out->right_sum_hessian = sum_h - w.lh - kEpsilon;
        out->gain = (w.gain - shift) * fi.penalty;
        out->default_left = dl;
      }
    }
    if (!two_dir && fi.missing == 2) out->default_left = 0;
  }
  return any;
}

// Wave-parallel FindBestCategorical (split_math.h:262-386, the host oracle; reference
// cuda_best_split_finder.cu:639 sorts the categories in-block): the one-hot candidates are
// evaluated one bin per lane with a wave arg-max (first maximum in bin order), and the
// many-vs-many path compacts the used bins with a ballot scan, bitonic-sorts them in LDS by
// (ctr, bin) — the order of the host's stable insertion sort — and lane 0 walks the at most
// max_cat_threshold prefix positions of both directions. `order` / `key` hold cat_p2 entries.
__device__ bool ScanCategoricalWave(const SplitParams& p_in, const FeatureScanMeta& m, const double* H, double sum_g,
                                    double sum_h_raw, int n, double po, const LeafBounds& bounds, int cat_p2,
                                    int* order, double* key, SplitInfo* out) {
  const int lane = threadIdx.x & 63;
  const double sum_h = sum_h_raw + 2 * kEpsilon;
  SplitParams p = p_in;  // monotone bounds clamp categorical outputs too (type 0: no order check)
  double gain_shift;
  if (p.path_smooth > kEpsilon) {
    gain_shift = LeafGainGivenOutput(sum_g, sum_h, p, po);
  } else {
    SplitParams q = p;
    q.path_smooth = 0.0;
    gain_shift = LeafGain(sum_g, sum_h, q, n, 0.0);
  }
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const double cnt_factor = n / sum_h;
  const bool use_rand = p.extra_trees != 0;
  bool sp = false;
  double best_gain = kMinScore, best_lg = 0.0, best_lh = 0.0;
  int best_lc = 0, best_t = -1, best_dir = 1, used = 0;
  const bool onehot = m.num_bin <= p.max_cat_to_onehot;
  if (onehot) {
    double lg = kMinScore, llg = 0.0, llh = 0.0;
    int lt = 0x7fffffff, llc = 0;
    bool lsp = false;
    for (int t = 1 + lane; t < m.num_bin; t += 64) {
      const double g = H[2 * t], h = H[2 * t + 1];
      const int c = RoundCount(h * cnt_factor);
      if (c < p.min_data_in_leaf || h < p.min_sum_hessian_in_leaf) continue;
      const int oc = n - c;
      if (oc < p.min_data_in_leaf) continue;
      const double oh = sum_h - h - kEpsilon;
      if (oh < p.min_sum_hessian_in_leaf) continue;
      const double og = sum_g - g;
      if (use_rand && t != m.rand_threshold) continue;
      const double gain = SplitGain(og, oh, g, h + kEpsilon, p, 0, oc, c, po, bounds);
      if (gain <= min_gain_shift) continue;
      lsp = true;
      if (gain > lg) {
        lg = gain;
        lt = t;
        llg = g;
        llh = h + kEpsilon;
        llc = c;
      }
    }
    sp = __any(lsp) != 0;
    const int src = WaveArgBestLane(lg, lt, 0);
    best_gain = ReadLane(lg, src);
    best_t = ReadLane(lt, src);
    best_lg = ReadLane(llg, src);
    best_lh = ReadLane(llh, src);
    best_lc = ReadLane(llc, src);
  } else {
    // used bins in ascending order (ballot compaction)
    const unsigned long long lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int base = 0; base < m.num_bin; base += 64) {
      const int i = base + lane;
      const bool v = i >= 1 && i < m.num_bin && RoundCount(H[2 * i + 1] * cnt_factor) >= p.cat_smooth;
      const unsigned long long b = __ballot(v);
      if (v) order[used + __popcll(b & lt_mask)] = i;
      used += __popcll(b);
    }
    int P2 = 1;
    while (P2 < used) P2 <<= 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int j = lane; j < P2; j += 64) {
      if (j < used) {
        const int b = order[j];
        key[j] = H[2 * b] / (H[2 * b + 1] + p.cat_smooth);
      } else {
        key[j] = INFINITY;
        order[j] = 0x7fffffff;
      }
    }
    // bitonic sort ascending by (ctr, bin): the stable order of the host's insertion sort
    for (int k = 2; k <= P2; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int i = lane; i < P2; i += 64) {
          const int l = i ^ jj;
          if (l <= i) continue;
          const double ka = key[i], kb = key[l];
          const int ba = order[i], bb = order[l];
          const bool a_gt = ka != kb ? ka > kb : ba > bb;
          if (a_gt == ((i & k) == 0)) {
            key[i] = kb;
            key[l] = ka;
            order[i] = bb;
            order[l] = ba;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    p.lambda_l2 += p.cat_l2;
    if (lane == 0) {
      const int max_num_cat = p.max_cat_threshold < (used + 1) / 2 ? p.max_cat_threshold : (used + 1) / 2;
      for (int dir_i = 0; dir_i < 2; ++dir_i) {
        const int dir = dir_i == 0 ? 1 : -1;
        int pos = dir_i == 0 ? 0 : used - 1;
        int cur_group = 0, lc = 0;
        double lg = 0.0, lh = kEpsilon;
        for (int i = 0; i < used && i < max_num_cat; ++i) {
          const int t = order[pos];
          pos += dir;
          const double g = H[2 * t], h = H[2 * t + 1];
          const int c = RoundCount(h * cnt_factor);
          lg += g;
          lh += h;
          lc += c;
          cur_group += c;
          if (lc < p.min_data_in_leaf || lh < p.min_sum_hessian_in_leaf) continue;
          const int rc = n - lc;
          if (rc < p.min_data_in_leaf || rc < p.min_data_per_group) break;
          const double rh = sum_h - lh;
          if (rh < p.min_sum_hessian_in_leaf) break;
          if (cur_group < p.min_data_per_group) continue;
          cur_group = 0;
          const double rg = sum_g - lg;
          if (use_rand && i != m.rand_threshold) continue;
          const double gain = SplitGain(lg, lh, rg, rh, p, 0, lc, rc, po, bounds);
          if (gain <= min_gain_shift) continue;
          sp = true;
          if (gain > best_gain) {
            best_lc = lc;
            best_lg = lg;
            best_lh = lh;
            best_t = i;
            best_gain = gain;
            best_dir = dir;
          }
        }
      }
    }
    sp = __shfl(sp ? 1 : 0, 0, kWave) != 0;
  }
  if (lane == 0) {
    out->Reset();
    out->default_left = 0;
    if (sp) {
      out->left_output = LeafOutput(best_lg, best_lh, p, best_lc, po, bounds);
      out->left_count = best_lc;
      out->left_sum_gradient = best_lg;
      out->left_sum_hessian = best_lh - kEpsilon;
      out->right_output = LeafOutput(sum_g - best_lg, sum_h - best_lh, p, n - best_lc, po, bounds);
      out->right_count = n - best_lc;
      out->right_sum_gradient = sum_g - best_lg;
      out->right_sum_hessian = sum_h - best_lh - kEpsilon;
      out->gain = (best_gain - min_gain_shift) * m.penalty;
      for (int w = 0; w < kMaxCatWords; ++w) out->cat_bitset[w] = 0u;
      if (onehot) {
        out->num_cat_threshold = 1;
        out->cat_bitset[best_t / 32] |= (1u << (best_t % 32));
      } else {
        out->num_cat_threshold = static_cast<int16_t>(best_t + 1);
        for (int i = 0; i <= best_t; ++i) {
          const int b = best_dir == 1 ? order[i] : order[used - 1 - i];
          out->cat_bitset[b / 32] |= (1u << (b % 32));
        }
      }
      out->monotone_type = 0;
    }
  }
  return sp;
}

}  // namespace
}  // namespace device
}  // namespace lgap
