// Split gain / leaf output math and the per-feature threshold scans, shared
// verbatim by the CPU oracle learner and the HIP device learner (LGAP_HD).
// Formulas: reference feature_histogram.hpp:711-828; numerical scan
// :830-1057 (reverse / forward passes, SKIP_DEFAULT_BIN, NA_AS_MISSING);
// categorical one-hot and ctr-sorted many-vs-many: feature_histogram.cpp:144-382.
//
// Histograms handed to these scans are *full* per-feature histograms: entry b
// holds (sum_grad, sum_hess) of bin b for every b in [0, num_bin), the
// most-frequent bin having been reconstructed by the caller.
#pragma once

#include <cmath>
#include <cstdint>

#include "lgap/meta.h"

namespace lgap {

constexpr int kMaxCatWords = 32;  // categorical bitset capacity: 1024 bins

struct SplitParams {
  double lambda_l1 = 0.0;
  double lambda_l2 = 0.0;
  double max_delta_step = 0.0;
  double path_smooth = 0.0;
  double min_gain_to_split = 0.0;
  double min_sum_hessian_in_leaf = 1e-3;
  double cat_smooth = 10.0;
  double cat_l2 = 10.0;
  int min_data_in_leaf = 20;
  int max_cat_threshold = 32;
  int max_cat_to_onehot = 4;
  int min_data_per_group = 100;
  int extra_trees = 0;
  int use_monotone = 0;
};

struct FeatureScanMeta {
  int num_bin = 0;
  uint32_t default_bin = 0;
  int8_t missing_type = 0;  // MissingType
  int8_t bin_type = 0;      // BinType
  int8_t monotone = 0;
  double penalty = 1.0;
  int rand_threshold = 0;   // extra_trees: pre-drawn threshold
};

// Output bounds of a leaf (basic monotone constraints).
struct LeafBounds {
  double min = -INFINITY;
  double max = INFINITY;
};

// Threshold-dependent bounds of one feature of one leaf (the "advanced" monotone
// method, reference monotone_constraints.hpp:145-257 CumulativeFeatureConstraint).
// Arrays of num_bin entries: for a reverse-pass threshold whose right side starts
// at bin t, the left child is bounded by [lmin[t], lmax[t]] (extremes over bins
// < t) and the right child by [rmin[t], rmax[t]] (extremes over bins >= t). The
// forward pass keeps the reference's fixed cursor: left bounded by bin 0's
// constraint (lmin[1], lmax[1]), right by the whole feature's (rmin[0], rmax[0]).
struct ThresholdBounds {
  const double* lmin;
  const double* lmax;
  const double* rmin;
  const double* rmax;
};

// Fixed-size POD split record; also the on-wire record of the parallel learners
// (reference split_info.hpp:22-294 / LightSplitInfo).
struct SplitInfo {
  int feature = -1;           // inner feature index, -1 = no split
  uint32_t threshold = 0;     // bin threshold (numerical)
  int left_count = 0;
  int right_count = 0;
  double gain = kMinScore;
  double left_output = 0.0;
  double right_output = 0.0;
  double left_sum_gradient = 0.0;
  double left_sum_hessian = 0.0;
  double right_sum_gradient = 0.0;
  double right_sum_hessian = 0.0;
  int8_t default_left = 1;
  int8_t monotone_type = 0;
  int16_t num_cat_threshold = 0;  // number of categories going left (0 = numerical)
  uint32_t cat_bitset[kMaxCatWords];  // bins going left (categorical)

  LGAP_HD void Reset() {
    feature = -1;
    gain = kMinScore;
    num_cat_threshold = 0;
    default_left = 1;
  }
  // Higher gain wins; ties go to the smaller feature index (split_info.hpp:138-165).
  LGAP_HD bool BetterThan(const SplitInfo& o) const {
    double a = gain, b = o.gain;
    if (a != a) a = kMinScore;
    if (b != b) b = kMinScore;
    if (a != b) return a > b;
    int fa = feature < 0 ? 0x7fffffff : feature;
    int fb = o.feature < 0 ? 0x7fffffff : o.feature;
    return fa < fb;
  }
};

// ----------------------------------------------------------------------------
LGAP_HD inline double ThresholdL1(double s, double l1) {
  const double r = fabs(s) - l1;
  const double reg = r > 0.0 ? r : 0.0;
  return (s > 0.0 ? 1.0 : (s < 0.0 ? -1.0 : 0.0)) * reg;
}

LGAP_HD inline double LeafOutputRaw(double g, double h, const SplitParams& p, data_size_t cnt, double parent_output) {
  double ret = p.lambda_l1 > 0.0 ? -ThresholdL1(g, p.lambda_l1) / (h + p.lambda_l2) : -g / (h + p.lambda_l2);
  if (p.max_delta_step > 0.0 && fabs(ret) > p.max_delta_step) ret = (ret > 0.0 ? 1.0 : -1.0) * p.max_delta_step;
  if (p.path_smooth > kEpsilon) {
    const double n = cnt / p.path_smooth;
    ret = ret * n / (n + 1.0) + parent_output / (n + 1.0);
  }
  return ret;
}

LGAP_HD inline double LeafOutput(double g, double h, const SplitParams& p, data_size_t cnt, double parent_output,
                                 const LeafBounds& b) {
  double ret = LeafOutputRaw(g, h, p, cnt, parent_output);
  if (p.use_monotone) {
    if (ret < b.min) ret = b.min;
    else if (ret > b.max) ret = b.max;
  }
  return ret;
}

LGAP_HD inline double LeafGainGivenOutput(double g, double h, const SplitParams& p, double out) {
  const double sg = p.lambda_l1 > 0.0 ? ThresholdL1(g, p.lambda_l1) : g;
  return -(2.0 * sg * out + (h + p.lambda_l2) * out * out);
}

LGAP_HD inline double LeafGain(double g, double h, const SplitParams& p, data_size_t cnt, double parent_output) {
  if (!(p.max_delta_step > 0.0) && !(p.path_smooth > kEpsilon)) {
    const double sg = p.lambda_l1 > 0.0 ? ThresholdL1(g, p.lambda_l1) : g;
    return (sg * sg) / (h + p.lambda_l2);
  }
  const double out = LeafOutputRaw(g, h, p, cnt, parent_output);
  return LeafGainGivenOutput(g, h, p, out);
}

// Gain of a split whose children are bounded by `lb` / `rb` (feature_histogram.hpp:755-796).
LGAP_HD inline double SplitGain2(double lg, double lh, double rg, double rh, const SplitParams& p, int8_t monotone,
                                 data_size_t lc, data_size_t rc, double parent_output, const LeafBounds& lb,
                                 const LeafBounds& rb) {
  if (!p.use_monotone) {
    return LeafGain(lg, lh, p, lc, parent_output) + LeafGain(rg, rh, p, rc, parent_output);
  }
  const double lo = LeafOutput(lg, lh, p, lc, parent_output, lb);
  const double ro = LeafOutput(rg, rh, p, rc, parent_output, rb);
  if ((monotone > 0 && lo > ro) || (monotone < 0 && lo < ro)) return 0.0;
  return LeafGainGivenOutput(lg, lh, p, lo) + LeafGainGivenOutput(rg, rh, p, ro);
}

LGAP_HD inline double SplitGain(double lg, double lh, double rg, double rh, const SplitParams& p, int8_t monotone,
                                data_size_t lc, data_size_t rc, double parent_output, const LeafBounds& b) {
  return SplitGain2(lg, lh, rg, rh, p, monotone, lc, rc, parent_output, b, b);
}

LGAP_HD inline int RoundCount(double x) { return static_cast<int>(x + 0.5f); }

// ----------------------------------------------------------------------------
// Sequential numerical scan over one full feature histogram (`hist` = 2*num_bin doubles).
// `out` must be Reset by the caller; the best of REVERSE / forward passes is kept.
// `tb` (advanced monotone) replaces `bounds` with per-threshold child bounds.
LGAP_HD inline void ScanNumericalPass(const double* hist, const FeatureScanMeta& m, const SplitParams& p,
                                      double sum_g, double sum_h, data_size_t num_data, double min_gain_shift,
                                      double parent_output, const LeafBounds& bounds, bool reverse, bool skip_default,
                                      bool na_as_missing, bool* splittable, SplitInfo* out,
                                      const ThresholdBounds* tb = nullptr) {
  const double cnt_factor = num_data / sum_h;
  double best_lg = NAN, best_lh = NAN, best_gain = kMinScore;
  data_size_t best_lc = 0;
  uint32_t best_t = static_cast<uint32_t>(m.num_bin);
  const bool use_rand = p.extra_trees != 0;
  LeafBounds lb = bounds, rb = bounds, best_lb = bounds, best_rb = bounds;
  if (tb != nullptr && !reverse) {
    lb.min = tb->lmin[1];
    lb.max = tb->lmax[1];
    rb.min = tb->rmin[0];
    rb.max = tb->rmax[0];
  }
  if (reverse) {
    double rg = 0.0, rh = kEpsilon;
    data_size_t rc = 0;
    for (int t = m.num_bin - 1 - (na_as_missing ? 1 : 0); t >= 1; --t) {
      if (skip_default && t == static_cast<int>(m.default_bin)) continue;
      const double g = hist[2 * t], h = hist[2 * t + 1];
      rg += g;
      rh += h;
      rc += RoundCount(h * cnt_factor);
      if (rc < p.min_data_in_leaf || rh < p.min_sum_hessian_in_leaf) continue;
      const data_size_t lc = num_data - rc;
      if (lc < p.min_data_in_leaf) break;
      const double lh = sum_h - rh;
      if (lh < p.min_sum_hessian_in_leaf) break;
      const double lg = sum_g - rg;
      if (use_rand && t - 1 != m.rand_threshold) continue;
      if (tb != nullptr) {
        lb.min = tb->lmin[t];
        lb.max = tb->lmax[t];
        rb.min = tb->rmin[t];
        rb.max = tb->rmax[t];
      }
      const double gain = SplitGain2(lg, lh, rg, rh, p, m.monotone, lc, rc, parent_output, lb, rb);
      if (gain <= min_gain_shift) continue;
      *splittable = true;
      if (gain > best_gain) {
        // a threshold whose child bounds cross cannot be taken (feature_histogram.hpp:920-926)
        if (p.use_monotone && (lb.min > lb.max || rb.min > rb.max)) continue;
        best_lb = lb;
        best_rb = rb;
        best_lc = lc;
        best_lg = lg;
        best_lh = lh;
        best_t = static_cast<uint32_t>(t - 1);
        best_gain = gain;
      }
    }
  } else {
    double lg = 0.0, lh = kEpsilon;
    data_size_t lc = 0;
    const int t_end = m.num_bin - 2;
    for (int t = 0; t <= t_end; ++t) {
      if (skip_default && t == static_cast<int>(m.default_bin)) continue;
      const double g = hist[2 * t], h = hist[2 * t + 1];
      lg += g;
      lh += h;
      lc += RoundCount(h * cnt_factor);
      if (lc < p.min_data_in_leaf || lh < p.min_sum_hessian_in_leaf) continue;
      const data_size_t rc = num_data - lc;
      if (rc < p.min_data_in_leaf) break;
      const double rh = sum_h - lh;
      if (rh < p.min_sum_hessian_in_leaf) break;
      const double rg = sum_g - lg;
      if (use_rand && t != m.rand_threshold) continue;
      const double gain = SplitGain2(lg, lh, rg, rh, p, m.monotone, lc, rc, parent_output, lb, rb);
      if (gain <= min_gain_shift) continue;
      *splittable = true;
      if (gain > best_gain) {
        if (p.use_monotone && (lb.min > lb.max || rb.min > rb.max)) continue;
        best_lb = lb;
        best_rb = rb;
        best_lc = lc;
        best_lg = lg;
        best_lh = lh;
        best_t = static_cast<uint32_t>(t);
        best_gain = gain;
      }
    }
  }
  if (*splittable && best_gain > out->gain + min_gain_shift) {
    out->threshold = best_t;
    out->left_output = LeafOutput(best_lg, best_lh, p, best_lc, parent_output, best_lb);
    out->left_count = best_lc;
    out->left_sum_gradient = best_lg;
    out->left_sum_hessian = best_lh - kEpsilon;
    out->right_output = LeafOutput(sum_g - best_lg, sum_h - best_lh, p, num_data - best_lc, parent_output, best_rb);
    out->right_count = num_data - best_lc;
    out->right_sum_gradient = sum_g - best_lg;
    out->right_sum_hessian = sum_h - best_lh - kEpsilon;
    out->gain = best_gain - min_gain_shift;
    out->default_left = reverse ? 1 : 0;
  }
}

// Best numerical threshold for one feature (FindBestThreshold + FuncForNumrical dispatch).
// sum_h must already include the +2*kEpsilon of the reference (caller passes raw sums).
LGAP_HD inline bool FindBestNumerical(const double* hist, const FeatureScanMeta& m, const SplitParams& p,
                                      double sum_g, double sum_h_raw, data_size_t num_data, double parent_output,
                                      const LeafBounds& bounds, SplitInfo* out, const ThresholdBounds* tb = nullptr) {
  const double sum_h = sum_h_raw + 2 * kEpsilon;
  out->default_left = 1;
  out->gain = kMinScore;
  out->monotone_type = m.monotone;
  const double min_gain_shift = LeafGain(sum_g, sum_h, p, num_data, parent_output) + p.min_gain_to_split;
  bool splittable = false;
  const int8_t mt = m.missing_type;
  if (m.num_bin > 2 && mt != static_cast<int8_t>(MissingType::None)) {
    if (mt == static_cast<int8_t>(MissingType::Zero)) {
      ScanNumericalPass(hist, m, p, sum_g, sum_h, num_data, min_gain_shift, parent_output, bounds, true, true, false,
                        &splittable, out, tb);
      ScanNumericalPass(hist, m, p, sum_g, sum_h, num_data, min_gain_shift, parent_output, bounds, false, true, false,
                        &splittable, out, tb);
    } else {
      ScanNumericalPass(hist, m, p, sum_g, sum_h, num_data, min_gain_shift, parent_output, bounds, true, false, true,
                        &splittable, out, tb);
      ScanNumericalPass(hist, m, p, sum_g, sum_h, num_data, min_gain_shift, parent_output, bounds, false, false, true,
                        &splittable, out, tb);
    }
  } else {
    ScanNumericalPass(hist, m, p, sum_g, sum_h, num_data, min_gain_shift, parent_output, bounds, true, false, false,
                      &splittable, out, tb);
    if (mt == static_cast<int8_t>(MissingType::NaN)) out->default_left = 0;
  }
  out->gain *= m.penalty;
  return splittable;
}

// Categorical split (one-hot or ctr-sorted many-vs-many). `order` is scratch of num_bin ints.
LGAP_HD inline bool FindBestCategorical(const double* hist, const FeatureScanMeta& m, const SplitParams& p_in,
                                        double sum_g, double sum_h_raw, data_size_t num_data, double parent_output,
                                        const LeafBounds& bounds, int* order, SplitInfo* out) {
  const double sum_h = sum_h_raw + 2 * kEpsilon;
  out->default_left = 0;
  out->gain = kMinScore;
  // monotone bounds still clamp the outputs (monotone type 0: no order check),
  // feature_histogram.cpp:195-199
  SplitParams p = p_in;
  double gain_shift;
  if (p.path_smooth > kEpsilon) {
    gain_shift = LeafGainGivenOutput(sum_g, sum_h, p, parent_output);
  } else {
    SplitParams q = p;
    q.path_smooth = 0.0;
    gain_shift = LeafGain(sum_g, sum_h, q, num_data, 0.0);
  }
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const double cnt_factor = num_data / sum_h;
  bool splittable = false;
  double best_gain = kMinScore, best_lg = 0.0, best_lh = 0.0;
  data_size_t best_lc = 0;
  int best_t = -1, best_dir = 1, used_bin = 0;
  const bool onehot = m.num_bin <= p.max_cat_to_onehot;
  const bool use_rand = p.extra_trees != 0;
  if (onehot) {
    for (int t = 1; t < m.num_bin; ++t) {
      const double g = hist[2 * t], h = hist[2 * t + 1];
      const data_size_t c = RoundCount(h * cnt_factor);
      if (c < p.min_data_in_leaf || h < p.min_sum_hessian_in_leaf) continue;
      const data_size_t oc = num_data - c;
      if (oc < p.min_data_in_leaf) continue;
      const double oh = sum_h - h - kEpsilon;
      if (oh < p.min_sum_hessian_in_leaf) continue;
      const double og = sum_g - g;
      if (use_rand && t != m.rand_threshold) continue;
      const double gain = SplitGain(og, oh, g, h + kEpsilon, p, 0, oc, c, parent_output, bounds);
      if (gain <= min_gain_shift) continue;
      splittable = true;
      if (gain > best_gain) {
        best_t = t;
        best_lg = g;
        best_lh = h + kEpsilon;
        best_lc = c;
        best_gain = gain;
      }
    }
  } else {
    for (int i = 1; i < m.num_bin; ++i) {
      if (RoundCount(hist[2 * i + 1] * cnt_factor) >= p.cat_smooth) order[used_bin++] = i;
    }
    p.lambda_l2 += p.cat_l2;
    // stable insertion sort by ctr = g / (h + cat_smooth)
    for (int i = 1; i < used_bin; ++i) {
      const int v = order[i];
      const double cv = hist[2 * v] / (hist[2 * v + 1] + p.cat_smooth);
      int j = i - 1;
      while (j >= 0 && hist[2 * order[j]] / (hist[2 * order[j] + 1] + p.cat_smooth) > cv) {
        order[j + 1] = order[j];
        --j;
      }
      order[j + 1] = v;
    }
    const int max_num_cat = p.max_cat_threshold < (used_bin + 1) / 2 ? p.max_cat_threshold : (used_bin + 1) / 2;
    for (int dir_i = 0; dir_i < 2; ++dir_i) {
      const int dir = dir_i == 0 ? 1 : -1;
      int pos = dir_i == 0 ? 0 : used_bin - 1;
      data_size_t cur_group = 0, lc = 0;
      double lg = 0.0, lh = kEpsilon;
      for (int i = 0; i < used_bin && i < max_num_cat; ++i) {
        const int t = order[pos];
        pos += dir;
        const double g = hist[2 * t], h = hist[2 * t + 1];
        const data_size_t c = RoundCount(h * cnt_factor);
        lg += g;
        lh += h;
        lc += c;
        cur_group += c;
        if (lc < p.min_data_in_leaf || lh < p.min_sum_hessian_in_leaf) continue;
        const data_size_t rc = num_data - lc;
        if (rc < p.min_data_in_leaf || rc < p.min_data_per_group) break;
        const double rh = sum_h - lh;
        if (rh < p.min_sum_hessian_in_leaf) break;
        if (cur_group < p.min_data_per_group) continue;
        cur_group = 0;
        const double rg = sum_g - lg;
        if (use_rand && i != m.rand_threshold) continue;
        const double gain = SplitGain(lg, lh, rg, rh, p, 0, lc, rc, parent_output, bounds);
        if (gain <= min_gain_shift) continue;
        splittable = true;
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
  if (splittable) {
    out->left_output = LeafOutput(best_lg, best_lh, p, best_lc, parent_output, bounds);
    out->left_count = best_lc;
    out->left_sum_gradient = best_lg;
    out->left_sum_hessian = best_lh - kEpsilon;
    out->right_output = LeafOutput(sum_g - best_lg, sum_h - best_lh, p, num_data - best_lc, parent_output, bounds);
    out->right_count = num_data - best_lc;
    out->right_sum_gradient = sum_g - best_lg;
    out->right_sum_hessian = sum_h - best_lh - kEpsilon;
    out->gain = (best_gain - min_gain_shift) * m.penalty;
    for (int w = 0; w < kMaxCatWords; ++w) out->cat_bitset[w] = 0u;
    if (onehot) {
      out->num_cat_threshold = 1;
      if (best_t < kMaxCatWords * 32) out->cat_bitset[best_t / 32] |= (1u << (best_t % 32));
    } else {
      out->num_cat_threshold = static_cast<int16_t>(best_t + 1);
      for (int i = 0; i <= best_t; ++i) {
        const int b = best_dir == 1 ? order[i] : order[used_bin - 1 - i];
        if (b < kMaxCatWords * 32) out->cat_bitset[b / 32] |= (1u << (b % 32));
      }
    }
    out->monotone_type = 0;
  }
  return splittable;
}

}  // namespace lgap
