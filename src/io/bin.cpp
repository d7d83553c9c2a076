// BinMapper::FindBin — numerical (greedy equal-frequency with a dedicated zero
// bin, optional NaN bin, forced bounds) and categorical (frequency ordered,
// 99% coverage) binning. Reference semantics: src/io/bin.cpp:78-508.
#include "lgap/bin.h"
#include "lgap/split_math.h"

#include <algorithm>
#include <cstring>
#include <iomanip>
#include <limits>
#include <sstream>

#include "lgap/common.h"
#include "lgap/log.h"

namespace lgap {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

// Equal-frequency partition of (distinct value, count) pairs into <= max_bin bins.
std::vector<double> GreedyBins(const double* vals, const int* cnts, int n, int max_bin, size_t total,
                               int min_data_in_bin) {
  std::vector<double> bounds;
  LGAP_CHECK_GT(max_bin, 0);
  if (n <= max_bin) {
    int in_bin = 0;
    for (int i = 0; i + 1 < n; ++i) {
      in_bin += cnts[i];
      if (in_bin >= min_data_in_bin) {
        double ub = common::GetDoubleUpperBound((vals[i] + vals[i + 1]) / 2.0);
        if (bounds.empty() || !common::CheckDoubleEqualOrdered(bounds.back(), ub)) {
          bounds.push_back(ub);
          in_bin = 0;
        }
      }
    }
    bounds.push_back(kInf);
    return bounds;
  }
  if (min_data_in_bin > 0) {
    max_bin = std::max(1, std::min(max_bin, static_cast<int>(total / min_data_in_bin)));
  }
  double mean_size = static_cast<double>(total) / max_bin;
  int rest_bins = max_bin;
  int rest_cnt = static_cast<int>(total);
  std::vector<char> big(n, 0);
  for (int i = 0; i < n; ++i) {
    if (cnts[i] >= mean_size) {
      big[i] = 1;
      --rest_bins;
      rest_cnt -= cnts[i];
    }
  }
  mean_size = static_cast<double>(rest_cnt) / rest_bins;
  std::vector<double> upper(max_bin, kInf), lower(max_bin, kInf);
  int nb = 0;
  lower[0] = vals[0];
  int in_bin = 0;
  for (int i = 0; i + 1 < n; ++i) {
    if (!big[i]) rest_cnt -= cnts[i];
    in_bin += cnts[i];
    bool cut = big[i] || in_bin >= mean_size || (big[i + 1] && in_bin >= std::max(1.0, mean_size * 0.5f));
    if (!cut) continue;
    upper[nb] = vals[i];
    ++nb;
    lower[nb] = vals[i + 1];
    if (nb >= max_bin - 1) break;
    in_bin = 0;
    if (!big[i]) {
      --rest_bins;
      mean_size = rest_cnt / static_cast<double>(rest_bins);
    }
  }
  ++nb;
  for (int i = 0; i + 1 < nb; ++i) {
    double ub = common::GetDoubleUpperBound((upper[i] + lower[i + 1]) / 2.0);
    if (bounds.empty() || !common::CheckDoubleEqualOrdered(bounds.back(), ub)) bounds.push_back(ub);
  }
  bounds.push_back(kInf);
  return bounds;
}

// Negatives / zero / positives are binned separately so that zero is its own bin.
std::vector<double> ZeroSeparatedBins(const double* vals, const int* cnts, int n, int max_bin, size_t total,
                                      int min_data_in_bin) {
  std::vector<double> bounds;
  int neg_cnt = 0, zero_cnt = 0, pos_cnt = 0;
  for (int i = 0; i < n; ++i) {
    if (vals[i] <= -kZeroThreshold) neg_cnt += cnts[i];
    else if (vals[i] > kZeroThreshold) pos_cnt += cnts[i];
    else zero_cnt += cnts[i];
  }
  int n_neg = n;
  for (int i = 0; i < n; ++i) {
    if (vals[i] > -kZeroThreshold) { n_neg = i; break; }
  }
  if (n_neg > 0 && max_bin > 1) {
    int neg_bins = static_cast<int>(static_cast<double>(neg_cnt) / (total - zero_cnt) * (max_bin - 1));
    neg_bins = std::max(1, neg_bins);
    bounds = GreedyBins(vals, cnts, n_neg, neg_bins, neg_cnt, min_data_in_bin);
    if (!bounds.empty()) bounds.back() = -kZeroThreshold;
  }
  int pos_start = -1;
  for (int i = n_neg; i < n; ++i) {
    if (vals[i] > kZeroThreshold) { pos_start = i; break; }
  }
  int pos_bins = max_bin - 1 - static_cast<int>(bounds.size());
  if (pos_start >= 0 && pos_bins > 0) {
    auto pb = GreedyBins(vals + pos_start, cnts + pos_start, n - pos_start, pos_bins, pos_cnt, min_data_in_bin);
    bounds.push_back(kZeroThreshold);
    bounds.insert(bounds.end(), pb.begin(), pb.end());
  } else {
    bounds.push_back(kInf);
  }
  LGAP_CHECK_LE(bounds.size(), static_cast<size_t>(max_bin));
  return bounds;
}

std::vector<double> ForcedBins(const double* vals, const int* cnts, int n, int max_bin, size_t total,
                               int min_data_in_bin, const std::vector<double>& forced) {
  std::vector<double> bounds;
  int n_neg = n;
  for (int i = 0; i < n; ++i) if (vals[i] > -kZeroThreshold) { n_neg = i; break; }
  int pos_start = -1;
  for (int i = n_neg; i < n; ++i) if (vals[i] > kZeroThreshold) { pos_start = i; break; }
  if (max_bin == 2) {
    bounds.push_back(n_neg == 0 ? kZeroThreshold : -kZeroThreshold);
  } else if (max_bin >= 3) {
    if (n_neg > 0) bounds.push_back(-kZeroThreshold);
    if (pos_start >= 0) bounds.push_back(kZeroThreshold);
  }
  bounds.push_back(kInf);
  int room = max_bin - static_cast<int>(bounds.size());
  int inserted = 0;
  for (double f : forced) {
    if (inserted >= room) break;
    if (std::fabs(f) > kZeroThreshold) { bounds.push_back(f); ++inserted; }
  }
  std::stable_sort(bounds.begin(), bounds.end());
  int free_bins = max_bin - static_cast<int>(bounds.size());
  std::vector<double> extra;
  int vi = 0;
  for (size_t i = 0; i < bounds.size(); ++i) {
    int cnt_in = 0, distinct_in = 0, start = vi;
    while (vi < n && vals[vi] < bounds[i]) { cnt_in += cnts[vi]; ++distinct_in; ++vi; }
    int remaining = max_bin - static_cast<int>(bounds.size()) - static_cast<int>(extra.size());
    int sub = static_cast<int>(std::lround(static_cast<double>(cnt_in) * free_bins / total));
    sub = std::min(sub, remaining) + 1;
    if (i + 1 == bounds.size()) sub = remaining + 1;
    auto nb = GreedyBins(vals + start, cnts + start, distinct_in, sub, cnt_in, min_data_in_bin);
    extra.insert(extra.end(), nb.begin(), nb.end() - 1);
  }
  bounds.insert(bounds.end(), extra.begin(), extra.end());
  std::stable_sort(bounds.begin(), bounds.end());
  return bounds;
}

std::vector<double> NumericalBounds(const double* vals, const int* cnts, int n, int max_bin, size_t total,
                                    int min_data_in_bin, const std::vector<double>& forced) {
  if (forced.empty()) return ZeroSeparatedBins(vals, cnts, n, max_bin, total, min_data_in_bin);
  return ForcedBins(vals, cnts, n, max_bin, total, min_data_in_bin, forced);
}

// True if no threshold leaves >= filter_cnt rows on both sides (feature_pre_filter).
bool Unsplittable(const std::vector<int>& cnt_in_bin, int total, int filter_cnt, BinType type) {
  if (type == BinType::Numerical) {
    int left = 0;
    for (size_t i = 0; i + 1 < cnt_in_bin.size(); ++i) {
      left += cnt_in_bin[i];
      if (left >= filter_cnt && total - left >= filter_cnt) return false;
    }
    return true;
  }
  if (cnt_in_bin.size() <= 2) {
    for (size_t i = 0; i + 1 < cnt_in_bin.size(); ++i) {
      int left = cnt_in_bin[i];
      if (left >= filter_cnt && total - left >= filter_cnt) return false;
    }
    return true;
  }
  return false;
}

}  // namespace

void BinMapper::FindBin(double* values, int num_values, size_t total_sample_cnt, int max_bin,
                        int min_data_in_bin, int min_split_data, bool pre_filter, BinType bin_type,
                        bool use_missing, bool zero_as_missing, const std::vector<double>& forced) {
  // compact non-NaN values to the front
  int non_na = 0;
  for (int i = 0; i < num_values; ++i) {
    if (!std::isnan(values[i])) values[non_na++] = values[i];
  }
  int na_cnt = 0;
  if (!use_missing) {
    missing_type_ = MissingType::None;
  } else if (zero_as_missing) {
    missing_type_ = MissingType::Zero;
  } else if (non_na == num_values) {
    missing_type_ = MissingType::None;
  } else {
    missing_type_ = MissingType::NaN;
    na_cnt = num_values - non_na;
  }
  num_values = non_na;
  bin_type_ = bin_type;
  default_bin_ = 0;
  const int zero_cnt = static_cast<int>(total_sample_cnt - num_values - na_cnt);

  // distinct values with counts; zero is injected at its sorted position
  std::stable_sort(values, values + num_values);
  std::vector<double> dv;
  std::vector<int> dc;
  if (num_values == 0 || (values[0] > 0.0 && zero_cnt > 0)) {
    dv.push_back(0.0);
    dc.push_back(zero_cnt);
  }
  if (num_values > 0) {
    dv.push_back(values[0]);
    dc.push_back(1);
  }
  for (int i = 1; i < num_values; ++i) {
    if (!common::CheckDoubleEqualOrdered(values[i - 1], values[i])) {
      if (values[i - 1] < 0.0 && values[i] > 0.0) {
        dv.push_back(0.0);
        dc.push_back(zero_cnt);
      }
      dv.push_back(values[i]);
      dc.push_back(1);
    } else {
      dv.back() = values[i];
      ++dc.back();
    }
  }
  if (num_values > 0 && values[num_values - 1] < 0.0 && zero_cnt > 0) {
    dv.push_back(0.0);
    dc.push_back(zero_cnt);
  }
  min_val_ = dv.front();
  max_val_ = dv.back();
  const int nd = static_cast<int>(dv.size());
  std::vector<int> cnt_in_bin;

  if (bin_type_ == BinType::Numerical) {
    if (missing_type_ == MissingType::NaN) {
      upper_bounds_ = NumericalBounds(dv.data(), dc.data(), nd, max_bin - 1, total_sample_cnt - na_cnt,
                                      min_data_in_bin, forced);
      upper_bounds_.push_back(std::numeric_limits<double>::quiet_NaN());
    } else {
      upper_bounds_ = NumericalBounds(dv.data(), dc.data(), nd, max_bin, total_sample_cnt, min_data_in_bin, forced);
      if (missing_type_ == MissingType::Zero && upper_bounds_.size() == 2) missing_type_ = MissingType::None;
    }
    num_bin_ = static_cast<int>(upper_bounds_.size());
    cnt_in_bin.assign(num_bin_, 0);
    int b = 0;
    for (int i = 0; i < nd; ++i) {
      while (dv[i] > upper_bounds_[b] && b < num_bin_ - 1) ++b;
      cnt_in_bin[b] += dc[i];
    }
    if (missing_type_ == MissingType::NaN) cnt_in_bin[num_bin_ - 1] = na_cnt;
    LGAP_CHECK_LE(num_bin_, max_bin);
  } else {
    // categorical: integer categories, negatives are treated as NaN
    std::vector<int> iv, ic;
    for (int i = 0; i < nd; ++i) {
      int v = static_cast<int>(dv[i]);
      if (v < 0) {
        na_cnt += dc[i];
        continue;
      }
      if (iv.empty() || v != iv.back()) {
        iv.push_back(v);
        ic.push_back(dc[i]);
      } else {
        ic.back() += dc[i];
      }
    }
    bin_2_cat_.clear();
    cat_2_bin_.clear();
    int rest = static_cast<int>(total_sample_cnt - na_cnt);
    if (rest > 0) {
      // sort categories by count (descending, stable on value)
      std::vector<int> order(iv.size());
      for (size_t i = 0; i < order.size(); ++i) order[i] = static_cast<int>(i);
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return ic[a] > ic[b]; });
      const int cut_cnt = common::RoundInt((total_sample_cnt - na_cnt) * 0.99f);
      int distinct = static_cast<int>(iv.size()) + (na_cnt > 0 ? 1 : 0);
      max_bin = std::min(distinct, max_bin);
      bin_2_cat_.push_back(-1);
      cat_2_bin_[-1] = 0;
      cnt_in_bin.push_back(0);
      num_bin_ = 1;
      int used = 0;
      size_t k = 0;
      // categorical splits carry their left-bin set as a kMaxCatWords-word bitset (host and
      // device share SplitInfo): at most 1024 category bins; rarer categories fold into bin 0
      // (the reference has no cap; it only binds for > 1024 frequent categories)
      constexpr int kMaxCatBins = kMaxCatWords * 32;
      while (k < order.size() && (used < cut_cnt || num_bin_ < max_bin)) {
        if (num_bin_ >= kMaxCatBins) {
          Log::Warning("Categorical feature has more than %d frequent categories; the rarest ones share bin 0",
                       kMaxCatBins - 1);
          break;
        }
        int c = order[k];
        if (ic[c] < min_data_in_bin && k > 1) break;
        bin_2_cat_.push_back(iv[c]);
        cat_2_bin_[iv[c]] = static_cast<unsigned int>(num_bin_);
        used += ic[c];
        cnt_in_bin.push_back(ic[c]);
        ++num_bin_;
        ++k;
      }
      missing_type_ = (k == order.size() && na_cnt == 0) ? MissingType::None : MissingType::NaN;
      cnt_in_bin[0] = static_cast<int>(total_sample_cnt - used);
    } else {
      num_bin_ = 1;
      bin_2_cat_.push_back(-1);
      cat_2_bin_[-1] = 0;
      cnt_in_bin.push_back(static_cast<int>(total_sample_cnt));
    }
  }

  is_trivial_ = num_bin_ <= 1;
  if (!is_trivial_ && pre_filter &&
      Unsplittable(cnt_in_bin, static_cast<int>(total_sample_cnt), min_split_data, bin_type_)) {
    is_trivial_ = true;
  }
  if (!is_trivial_) {
    default_bin_ = ValueToBin(0.0);
    most_freq_bin_ = static_cast<uint32_t>(common::ArgMax(cnt_in_bin));
    double rate = static_cast<double>(cnt_in_bin[most_freq_bin_]) / total_sample_cnt;
    if (most_freq_bin_ != default_bin_ && rate < kSparseThreshold) most_freq_bin_ = default_bin_;
    sparse_rate_ = static_cast<double>(cnt_in_bin[most_freq_bin_]) / total_sample_cnt;
  } else {
    sparse_rate_ = 1.0;
  }
}

std::string BinMapper::bin_info_string() const {
  if (bin_type_ == BinType::Categorical) return common::Join(bin_2_cat_, ":");
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  ss << '[' << min_val_ << ':' << max_val_ << ']';
  return ss.str();
}

bool BinMapper::CheckAlign(const BinMapper& o) const {
  if (num_bin_ != o.num_bin_ || missing_type_ != o.missing_type_ || bin_type_ != o.bin_type_) return false;
  if (bin_type_ == BinType::Numerical) {
    for (int i = 0; i < num_bin_; ++i) {
      double a = upper_bounds_[i], b = o.upper_bounds_[i];
      if (!(a == b || (std::isnan(a) && std::isnan(b)))) return false;
    }
  } else {
    if (bin_2_cat_ != o.bin_2_cat_) return false;
  }
  return true;
}

namespace {
template <typename T>
void Put(std::vector<char>* out, const T& v) {
  const char* p = reinterpret_cast<const char*>(&v);
  out->insert(out->end(), p, p + sizeof(T));
}
template <typename T>
T Get(const char*& p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}
}  // namespace

void BinMapper::Serialize(std::vector<char>* out) const {
  Put(out, num_bin_);
  Put(out, static_cast<int8_t>(missing_type_));
  Put(out, static_cast<int8_t>(is_trivial_));
  Put(out, sparse_rate_);
  Put(out, static_cast<int8_t>(bin_type_));
  Put(out, min_val_);
  Put(out, max_val_);
  Put(out, default_bin_);
  Put(out, most_freq_bin_);
  if (bin_type_ == BinType::Numerical) {
    Put(out, static_cast<int32_t>(upper_bounds_.size()));
    for (double d : upper_bounds_) Put(out, d);
  } else {
    Put(out, static_cast<int32_t>(bin_2_cat_.size()));
    for (int c : bin_2_cat_) Put(out, c);
  }
}

size_t BinMapper::Deserialize(const char* buf) {
  const char* p = buf;
  num_bin_ = Get<int>(p);
  missing_type_ = static_cast<MissingType>(Get<int8_t>(p));
  is_trivial_ = Get<int8_t>(p) != 0;
  sparse_rate_ = Get<double>(p);
  bin_type_ = static_cast<BinType>(Get<int8_t>(p));
  min_val_ = Get<double>(p);
  max_val_ = Get<double>(p);
  default_bin_ = Get<uint32_t>(p);
  most_freq_bin_ = Get<uint32_t>(p);
  int32_t n = Get<int32_t>(p);
  upper_bounds_.clear();
  bin_2_cat_.clear();
  cat_2_bin_.clear();
  if (bin_type_ == BinType::Numerical) {
    for (int i = 0; i < n; ++i) upper_bounds_.push_back(Get<double>(p));
  } else {
    for (int i = 0; i < n; ++i) {
      int c = Get<int>(p);
      bin_2_cat_.push_back(c);
      cat_2_bin_[c] = static_cast<unsigned int>(i);
    }
  }
  return static_cast<size_t>(p - buf);
}

}  // namespace lgap
