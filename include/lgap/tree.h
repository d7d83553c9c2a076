// Leaf-wise binary decision tree stored as flat arrays; node/leaf indexing,
// decision_type bits and the text/JSON formats are compatible with the
// reference (include/LightGBM/tree.h:26-731, src/io/tree.cpp). Internal nodes
// are 0..num_leaves-2 in creation order; children < 0 encode ~leaf.
#pragma once

#include <cmath>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgap/meta.h"

namespace lgap {

class Dataset;

constexpr int8_t kCategoricalMask = 1;
constexpr int8_t kDefaultLeftMask = 2;

class Tree {
 public:
  explicit Tree(int max_leaves = 2, bool track_branch_features = false, bool is_linear = false);
  // Parse one "Tree=" block of the model text format.
  explicit Tree(const char* str, size_t* used_len);

  // Numerical split of `leaf`; returns index of the new (right) leaf.
  int Split(int leaf, int feature_inner, int real_feature, uint32_t threshold_bin, double threshold_double,
            double left_value, double right_value, int left_cnt, int right_cnt, double left_weight,
            double right_weight, float gain, MissingType missing_type, bool default_left);
  // Categorical split; bitsets are over inner bins and raw category values.
  int SplitCategorical(int leaf, int feature_inner, int real_feature, const uint32_t* threshold_bin,
                       int num_threshold_bin, const uint32_t* threshold, int num_threshold, double left_value,
                       double right_value, int left_cnt, int right_cnt, double left_weight, double right_weight,
                       float gain, MissingType missing_type);

  // --- prediction on raw feature values
  inline double Predict(const double* features) const;
  inline int PredictLeafIndex(const double* features) const;
  double PredictByMap(const std::unordered_map<int, double>& features) const;
  int PredictLeafIndexByMap(const std::unordered_map<int, double>& features) const;
  // TreeSHAP contributions; out has num_features+1 entries (last = expected value)
  void PredictContrib(const double* features, int num_features, double* out) const;
  void PredictContribByMap(const std::unordered_map<int, double>& features, int num_features,
                           std::unordered_map<int, double>* out) const;

  // --- prediction on binned data
  int GetLeafByBins(const Dataset& data, data_size_t row) const;
  void AddPredictionToScore(const Dataset& data, data_size_t num_data, double* score) const;
  void AddPredictionToScore(const Dataset& data, const data_size_t* indices, data_size_t n, double* score) const;

  // --- mutation
  void Shrinkage(double rate);
  void AddBias(double val);
  void SetLeafOutput(int leaf, double v) { leaf_value_[leaf] = MaybeRoundToZero(v); }
  // a one-leaf tree holding `count` rows (reference tree.h AsConstantTree)
  void AsConstantTree(double v, int count, bool linear) {
    SetLeafOutput(0, v);
    leaf_count_[0] = count;
    if (linear) {
      is_linear_ = true;
      InitLinear();
      SetLeafConst(0, v);
    }
  }
  void SetShrinkage(double s) { shrinkage_ = s; }
  void RecomputeMaxDepth();
  void RecomputeLeafDepths();

  // --- accessors
  int num_leaves() const { return num_leaves_; }
  int max_leaves() const { return max_leaves_; }
  int num_cat() const { return num_cat_; }
  int split_feature(int node) const { return split_feature_[node]; }
  int split_feature_inner(int node) const { return split_feature_inner_[node]; }
  double split_gain(int node) const { return split_gain_[node]; }
  double threshold(int node) const { return threshold_[node]; }
  uint32_t threshold_in_bin(int node) const { return threshold_in_bin_[node]; }
  int8_t decision_type(int node) const { return decision_type_[node]; }
  int left_child(int node) const { return left_child_[node]; }
  int right_child(int node) const { return right_child_[node]; }
  double LeafOutput(int leaf) const { return leaf_value_[leaf]; }
  double leaf_weight(int leaf) const { return leaf_weight_[leaf]; }
  int leaf_count(int leaf) const { return leaf_count_[leaf]; }
  int leaf_parent(int leaf) const { return leaf_parent_[leaf]; }
  int leaf_depth(int leaf) const { return leaf_depth_[leaf]; }
  double internal_value(int node) const { return internal_value_[node]; }
  double internal_weight(int node) const { return internal_weight_[node]; }
  int internal_count(int node) const { return internal_count_[node]; }
  double shrinkage() const { return shrinkage_; }
  int max_depth() const { return max_depth_; }
  bool is_linear() const { return is_linear_; }
  void SetIsLinear(bool l) { is_linear_ = l; }
  const std::vector<int>& branch_features(int leaf) const { return branch_features_[leaf]; }
  const std::vector<int>& cat_boundaries_inner() const { return cat_boundaries_inner_; }
  const std::vector<uint32_t>& cat_threshold_inner() const { return cat_threshold_inner_; }
  const std::vector<int>& cat_boundaries() const { return cat_boundaries_; }
  const std::vector<uint32_t>& cat_threshold() const { return cat_threshold_; }
  std::vector<double>& leaf_values() { return leaf_value_; }

  // linear leaves
  double LeafConst(int leaf) const { return leaf_const_[leaf]; }
  const std::vector<double>& LeafCoeffs(int leaf) const { return leaf_coeff_[leaf]; }
  const std::vector<int>& LeafFeatures(int leaf) const { return leaf_features_[leaf]; }
  const std::vector<int>& LeafFeaturesInner(int leaf) const { return leaf_features_inner_[leaf]; }
  void SetLeafConst(int leaf, double v) { leaf_const_[leaf] = MaybeRoundToZero(v); }
  void SetLeafCoeffs(int leaf, const std::vector<double>& c);
  void InitLinear() {
    leaf_coeff_.assign(max_leaves_, {});
    leaf_const_.assign(max_leaves_, 0.0);
    leaf_features_.assign(max_leaves_, {});
    leaf_features_inner_.assign(max_leaves_, {});
  }
  void SetLeafFeatures(int leaf, const std::vector<int>& f) { leaf_features_[leaf] = f; }
  void SetLeafFeaturesInner(int leaf, const std::vector<int>& f) { leaf_features_inner_[leaf] = f; }

  std::string ToString() const;
  std::string ToJSON() const;
  std::string ToIfElse(int index, bool predict_leaf_index) const;
  double ExpectedValue() const;

  static bool IsZero(double v) { return v >= -kZeroThreshold && v <= kZeroThreshold; }
  static double MaybeRoundToZero(double v) { return IsZero(v) ? 0.0 : v; }
  static bool GetDecisionType(int8_t dt, int8_t mask) { return (dt & mask) > 0; }
  static int8_t GetMissingType(int8_t dt) { return (dt >> 2) & 3; }

  inline int NumericalDecision(double fval, int node) const;
  inline int CategoricalDecision(double fval, int node) const;
  inline int Decision(double fval, int node) const {
    return GetDecisionType(decision_type_[node], kCategoricalMask) ? CategoricalDecision(fval, node)
                                                                   : NumericalDecision(fval, node);
  }
  inline int GetLeaf(const double* features) const {
    int node = 0;
    if (num_cat_ > 0) {
      while (node >= 0) node = Decision(features[split_feature_[node]], node);
    } else {
      while (node >= 0) node = NumericalDecision(features[split_feature_[node]], node);
    }
    return ~node;
  }

 private:
  double LinearOrConstOutput(const Dataset& data, data_size_t row, int leaf) const;
  void SplitCommon(int leaf, int feature_inner, int real_feature, double left_value, double right_value,
                   int left_cnt, int right_cnt, double left_weight, double right_weight, float gain);
  std::string NodeToJSON(int index) const;
  std::string NodeToIfElse(int index, bool predict_leaf_index) const;
  std::string LinearModelToJSON(int leaf) const;
  int GetLeafByMap(const std::unordered_map<int, double>& f) const;
  // TreeSHAP internals
  struct PathElement {
    int feature_index;
    double zero_fraction;
    double one_fraction;
    double pweight;
  };
  void TreeSHAP(const double* features, double* phi, int node, int unique_depth, PathElement* parent_path,
                double parent_zero_fraction, double parent_one_fraction, int parent_feature_index) const;
  double DataCount(int node) const { return node >= 0 ? internal_count_[node] : leaf_count_[~node]; }

  int max_leaves_;
  int num_leaves_;
  std::vector<int> left_child_, right_child_;
  std::vector<int> split_feature_inner_, split_feature_;
  std::vector<uint32_t> threshold_in_bin_;
  std::vector<double> threshold_;
  int num_cat_ = 0;
  std::vector<int> cat_boundaries_inner_;
  std::vector<uint32_t> cat_threshold_inner_;
  std::vector<int> cat_boundaries_;
  std::vector<uint32_t> cat_threshold_;
  std::vector<int8_t> decision_type_;
  std::vector<float> split_gain_;
  std::vector<int> leaf_parent_;
  std::vector<double> leaf_value_, leaf_weight_;
  std::vector<int> leaf_count_;
  std::vector<double> internal_value_, internal_weight_;
  std::vector<int> internal_count_;
  std::vector<int> leaf_depth_;
  double shrinkage_ = 1.0;
  int max_depth_ = -1;
  bool track_branch_features_ = false;
  std::vector<std::vector<int>> branch_features_;
  bool is_linear_ = false;
  std::vector<std::vector<double>> leaf_coeff_;
  std::vector<double> leaf_const_;
  std::vector<std::vector<int>> leaf_features_, leaf_features_inner_;
};

inline int Tree::NumericalDecision(double fval, int node) const {
  const int8_t mt = GetMissingType(decision_type_[node]);
  if (std::isnan(fval) && mt != static_cast<int8_t>(MissingType::NaN)) fval = 0.0;
  if ((mt == static_cast<int8_t>(MissingType::Zero) && IsZero(fval)) ||
      (mt == static_cast<int8_t>(MissingType::NaN) && std::isnan(fval))) {
    return GetDecisionType(decision_type_[node], kDefaultLeftMask) ? left_child_[node] : right_child_[node];
  }
  return fval <= threshold_[node] ? left_child_[node] : right_child_[node];
}

inline int Tree::CategoricalDecision(double fval, int node) const {
  if (std::isnan(fval)) return right_child_[node];
  int iv = static_cast<int>(fval);
  if (iv < 0) return right_child_[node];
  int ci = static_cast<int>(threshold_[node]);
  int b = cat_boundaries_[ci], e = cat_boundaries_[ci + 1];
  int word = iv / 32;
  if (word >= e - b) return right_child_[node];
  return ((cat_threshold_[b + word] >> (iv % 32)) & 1) ? left_child_[node] : right_child_[node];
}

inline double Tree::Predict(const double* features) const {
  if (is_linear_) {
    int leaf = num_leaves_ > 1 ? GetLeaf(features) : 0;
    double out = leaf_const_[leaf];
    for (size_t i = 0; i < leaf_features_[leaf].size(); ++i) {
      double v = features[leaf_features_[leaf][i]];
      if (std::isnan(v)) return leaf_value_[leaf];
      out += leaf_coeff_[leaf][i] * v;
    }
    return out;
  }
  if (num_leaves_ > 1) return leaf_value_[GetLeaf(features)];
  return leaf_value_[0];
}

inline int Tree::PredictLeafIndex(const double* features) const {
  return num_leaves_ > 1 ? GetLeaf(features) : 0;
}

}  // namespace lgap
