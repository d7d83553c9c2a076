// LambdaRank pair weighting for the 18 `lambdarank_target`s of the fork
// (reference rank_objective.hpp:182-201 target map, :303-351 pair ranges,
// :357-380 binary-target filter, :397-489 delta_pair). Shared by the host
// objective and the HIP per-query lambda kernel.
#pragma once

#include <cmath>

#include "lgap/meta.h"

namespace lgap {

enum LambdaTarget : int {
  kTgtNdcg = 0,
  kTgtLambdalossNdcg,
  kTgtLambdalossNdcgPP,
  kTgtBndcg,
  kTgtLambdalossBndcg,
  kTgtLambdalossBndcgPP,
  kTgtPrecision,
  kTgtArpK,
  kTgtLambdalossArp1,
  kTgtLambdalossArp2,
  kTgtRanknet,
  kTgtBinRanknet,
  kTgtGapS,
  kTgtGapX,
  kTgtGapSPlus,
  kTgtGapXPlus,
  kTgtGapSPlusPlus,
  kTgtGapXPlusPlus,
  kNumLambdaTargets
};

LGAP_HD inline double RankDiscount(int r) { return 1.0 / log2(2.0 + r); }

// Targets that rank by sorted score (all except the order-free ones).
LGAP_HD inline bool TargetNeedsFullSort(int t) {
  return !(t == kTgtBinRanknet || t == kTgtRanknet || t == kTgtLambdalossArp1 || t == kTgtLambdalossArp2 ||
           t == kTgtPrecision);
}

// Outer loop bound on rank i.
LGAP_HD inline int TargetIEnd(int t, int cnt, int k) {
  switch (t) {
    case kTgtNdcg:
    case kTgtLambdalossNdcg:
    case kTgtLambdalossNdcgPP:
    case kTgtBndcg:
    case kTgtLambdalossBndcg:
    case kTgtLambdalossBndcgPP:
    case kTgtPrecision:
      return (cnt - 1) < k ? (cnt - 1) : k;
    default:
      return cnt - 1;
  }
}

// Inner [start, end) range of rank j for a given i.
LGAP_HD inline void TargetJRange(int t, int i, int cnt, int k, int* start, int* end) {
  switch (t) {
    case kTgtPrecision:
      *start = k;
      *end = cnt;
      break;
    case kTgtArpK:
    case kTgtGapSPlus:
    case kTgtGapXPlus:
    case kTgtGapSPlusPlus:
    case kTgtGapXPlusPlus:
      *start = (i + 1) > k ? (i + 1) : k;
      *end = cnt;
      break;
    case kTgtGapS:
      *start = i + k;
      *end = (*start + 1) < cnt ? (*start + 1) : cnt;
      break;
    case kTgtGapX:
      *start = i + k;
      *end = cnt;
      break;
    default:
      *start = i + 1;
      *end = cnt;
  }
}

// Binary targets skip pairs where both labels are relevant.
LGAP_HD inline bool TargetIsBinary(int t) {
  return t == kTgtPrecision || t == kTgtBndcg || t == kTgtLambdalossBndcg || t == kTgtLambdalossBndcgPP ||
         t == kTgtArpK || t == kTgtBinRanknet || t == kTgtGapS || t == kTgtGapX || t == kTgtGapSPlus ||
         t == kTgtGapXPlus || t == kTgtGapSPlusPlus || t == kTgtGapXPlusPlus;
}

// RankDiscount evaluated directly (the host objective; queries too long for a table)
struct RankDiscountFn {
  LGAP_HD double operator()(int r) const { return RankDiscount(r); }
};

// delta_pair for ranks (i, j) (i < j), with high/low = the better/worse labelled doc.
// `RankDiscount` is the discount source: RankDiscountFn, or a per-query table of the same
// values (the HIP kernel keeps one in LDS: two double log2 per pair were most of its work).
template <typename Disc>
LGAP_HD inline double TargetDeltaPairD(int t, int i, int j, int high_rank, int low_rank, double high_gain,
                                       double low_gain, double high_label, double low_label, double inv_max_dcg,
                                       double inv_max_bdcg, int k, double w, const Disc& RankDiscount) {
  switch (t) {
    case kTgtNdcg:
      return (high_gain - low_gain) * fabs(RankDiscount(high_rank) - RankDiscount(low_rank)) * inv_max_dcg;
    case kTgtLambdalossNdcg:
      return (high_gain - low_gain) * (RankDiscount(j - i) - RankDiscount(j - i + 1)) * inv_max_dcg;
    case kTgtLambdalossNdcgPP:
      return (high_gain - low_gain) *
             (fabs(RankDiscount(high_rank) - RankDiscount(low_rank)) +
              w * (RankDiscount(j - i) - RankDiscount(j - i + 1))) *
             inv_max_dcg;
    case kTgtBndcg:
      return fabs(RankDiscount(high_rank) - RankDiscount(low_rank)) * inv_max_bdcg;
    case kTgtLambdalossBndcg:
      return (RankDiscount(j - i) - RankDiscount(j - i + 1)) * inv_max_bdcg;
    case kTgtLambdalossBndcgPP:
      return (fabs(RankDiscount(high_rank) - RankDiscount(low_rank)) +
              w * (RankDiscount(j - i) - RankDiscount(j - i + 1))) *
             inv_max_bdcg;
    case kTgtPrecision:
    case kTgtGapS:
    case kTgtGapX:
    case kTgtBinRanknet:
    case kTgtRanknet:
      return 1.0;
    case kTgtGapSPlus:
      return (j - i == k) * w + (i < k);
    case kTgtGapXPlus:
      return (j - i >= k) * w + (i < k);
    case kTgtGapSPlusPlus:
      return (j - i == k) * w + (j + 1 - k) - (i >= k) * (i + 1 - k);
    case kTgtGapXPlusPlus:
      return (j - i >= k) * w + (j + 1 - k) - (i >= k) * (i + 1 - k);
    case kTgtArpK:
      return static_cast<double>((j + 1 - k) - (i >= k) * (i + 1 - k));
    case kTgtLambdalossArp1:
      return high_label;
    case kTgtLambdalossArp2:
      return high_label - low_label;
  }
  return 0.0;
}

LGAP_HD inline double TargetDeltaPair(int t, int i, int j, int high_rank, int low_rank, double high_gain,
                                      double low_gain, double high_label, double low_label, double inv_max_dcg,
                                      double inv_max_bdcg, int k, double w) {
  return TargetDeltaPairD(t, i, j, high_rank, low_rank, high_gain, low_gain, high_label, low_label, inv_max_dcg,
                          inv_max_bdcg, k, w, RankDiscountFn());
}

}  // namespace lgap
