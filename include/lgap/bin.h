// Feature discretisation (BinMapper). Semantics follow the reference
// (include/LightGBM/bin.h:85-260, src/io/bin.cpp:78-508): greedy equal-frequency
// numerical bins with zero as its own bin and an optional NaN bin; categorical
// bins sorted by frequency with bin 0 reserved for NaN/"other".
#pragma once

#include <cmath>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgap/meta.h"

namespace lgap {

class BinMapper {
 public:
  BinMapper() { upper_bounds_.push_back(std::numeric_limits<double>::infinity()); }

  // values: non-zero sampled values of this feature (NaN allowed); zeros are implicit
  // (total_sample_cnt - num_values of them).
  void FindBin(double* values, int num_values, size_t total_sample_cnt, int max_bin, int min_data_in_bin,
               int min_split_data, bool pre_filter, BinType bin_type, bool use_missing, bool zero_as_missing,
               const std::vector<double>& forced_upper_bounds);

  inline uint32_t ValueToBin(double value) const;

  int num_bin() const { return num_bin_; }
  bool is_trivial() const { return is_trivial_; }
  MissingType missing_type() const { return missing_type_; }
  BinType bin_type() const { return bin_type_; }
  uint32_t default_bin() const { return default_bin_; }
  uint32_t most_freq_bin() const { return most_freq_bin_; }
  double sparse_rate() const { return sparse_rate_; }
  double min_val() const { return min_val_; }
  double max_val() const { return max_val_; }
  const std::vector<double>& upper_bounds() const { return upper_bounds_; }
  const std::vector<int>& bin_to_category() const { return bin_2_cat_; }

  // Real-valued threshold for numerical bin index (left is bin <= threshold).
  double BinToValue(uint32_t bin) const {
    if (bin_type_ == BinType::Numerical) return upper_bounds_[bin];
    return static_cast<double>(bin_2_cat_[bin]);
  }
  // feature_infos entry of the model file (bin.h:224-233)
  std::string bin_info_string() const;

  // Compact serialisation (dataset binary cache, distributed bin finding).
  void Serialize(std::vector<char>* out) const;
  size_t Deserialize(const char* buf);

  bool CheckAlign(const BinMapper& other) const;
  void set_trivial(bool t) { is_trivial_ = t; }

 private:
  int num_bin_ = 1;
  MissingType missing_type_ = MissingType::None;
  bool is_trivial_ = true;
  double sparse_rate_ = 1.0;
  BinType bin_type_ = BinType::Numerical;
  std::vector<double> upper_bounds_;
  std::vector<int> bin_2_cat_;
  std::unordered_map<int, unsigned int> cat_2_bin_;
  double min_val_ = 0.0;
  double max_val_ = 0.0;
  uint32_t default_bin_ = 0;
  uint32_t most_freq_bin_ = 0;
};

inline uint32_t BinMapper::ValueToBin(double value) const {
  if (std::isnan(value)) {
    if (bin_type_ == BinType::Categorical) return 0;
    if (missing_type_ == MissingType::NaN) return static_cast<uint32_t>(num_bin_ - 1);
    value = 0.0;
  }
  if (bin_type_ == BinType::Numerical) {
    int l = 0;
    int r = num_bin_ - 1;
    if (missing_type_ == MissingType::NaN) r -= 1;
    while (l < r) {
      int m = (r + l - 1) / 2;
      if (value <= upper_bounds_[m]) r = m;
      else l = m + 1;
    }
    return static_cast<uint32_t>(l);
  }
  int iv = static_cast<int>(value);
  if (iv < 0) return 0;
  auto it = cat_2_bin_.find(iv);
  return it == cat_2_bin_.end() ? 0u : it->second;
}

}  // namespace lgap
