// Tree mutation, binned traversal, TreeSHAP, and the text / JSON / if-else
// serialisations (reference: src/io/tree.cpp:61-1055).
#include "lgap/tree.h"

#include <omp.h>

#include <algorithm>
#include <cstring>
#include <iomanip>
#include <limits>
#include <sstream>
#include <unordered_map>

#include "lgap/common.h"
#include "lgap/dataset.h"
#include "lgap/log.h"

namespace lgap {

Tree::Tree(int max_leaves, bool track_branch_features, bool is_linear)
    : max_leaves_(max_leaves), num_leaves_(1), track_branch_features_(track_branch_features),
      is_linear_(is_linear) {
  const int ni = std::max(max_leaves - 1, 1);
  left_child_.assign(ni, 0);
  right_child_.assign(ni, 0);
  split_feature_inner_.assign(ni, -1);
  split_feature_.assign(ni, -1);
  threshold_in_bin_.assign(ni, 0);
  threshold_.assign(ni, 0.0);
  decision_type_.assign(ni, 0);
  split_gain_.assign(ni, 0.0f);
  internal_value_.assign(ni, 0.0);
  internal_weight_.assign(ni, 0.0);
  internal_count_.assign(ni, 0);
  leaf_parent_.assign(max_leaves, -1);
  leaf_value_.assign(max_leaves, 0.0);
  leaf_weight_.assign(max_leaves, 0.0);
  leaf_count_.assign(max_leaves, 0);
  leaf_depth_.assign(max_leaves, 0);
  if (track_branch_features_) branch_features_.assign(max_leaves, {});
  cat_boundaries_.push_back(0);
  cat_boundaries_inner_.push_back(0);
  if (is_linear_) {
    leaf_coeff_.assign(max_leaves, {});
    leaf_const_.assign(max_leaves, 0.0);
    leaf_features_.assign(max_leaves, {});
    leaf_features_inner_.assign(max_leaves, {});
  }
}

void Tree::SplitCommon(int leaf, int feature_inner, int real_feature, double left_value, double right_value,
                       int left_cnt, int right_cnt, double left_weight, double right_weight, float gain) {
  const int node = num_leaves_ - 1;
  const int parent = leaf_parent_[leaf];
  if (parent >= 0) {
    if (left_child_[parent] == ~leaf) left_child_[parent] = node;
    else right_child_[parent] = node;
  }
  split_feature_inner_[node] = feature_inner;
  split_feature_[node] = real_feature;
  split_gain_[node] = gain;
  left_child_[node] = ~leaf;
  right_child_[node] = ~num_leaves_;
  leaf_parent_[leaf] = node;
  leaf_parent_[num_leaves_] = node;
  internal_weight_[node] = left_weight + right_weight;
  internal_value_[node] = leaf_value_[leaf];
  internal_count_[node] = left_cnt + right_cnt;
  leaf_value_[leaf] = std::isnan(left_value) ? 0.0 : left_value;
  leaf_weight_[leaf] = left_weight;
  leaf_count_[leaf] = left_cnt;
  leaf_value_[num_leaves_] = std::isnan(right_value) ? 0.0 : right_value;
  leaf_weight_[num_leaves_] = right_weight;
  leaf_count_[num_leaves_] = right_cnt;
  leaf_depth_[num_leaves_] = leaf_depth_[leaf] + 1;
  leaf_depth_[leaf]++;
  if (track_branch_features_) {
    branch_features_[num_leaves_] = branch_features_[leaf];
    branch_features_[num_leaves_].push_back(real_feature);
    branch_features_[leaf].push_back(real_feature);
  }
}

int Tree::Split(int leaf, int feature_inner, int real_feature, uint32_t threshold_bin, double threshold_double,
                double left_value, double right_value, int left_cnt, int right_cnt, double left_weight,
                double right_weight, float gain, MissingType missing_type, bool default_left) {
  SplitCommon(leaf, feature_inner, real_feature, left_value, right_value, left_cnt, right_cnt, left_weight,
              right_weight, gain);
  const int node = num_leaves_ - 1;
  int8_t dt = 0;
  if (default_left) dt |= kDefaultLeftMask;
  dt |= static_cast<int8_t>(static_cast<int>(missing_type) << 2);
  decision_type_[node] = dt;
  threshold_in_bin_[node] = threshold_bin;
  threshold_[node] = threshold_double;
  ++num_leaves_;
  return num_leaves_ - 1;
}

int Tree::SplitCategorical(int leaf, int feature_inner, int real_feature, const uint32_t* threshold_bin,
                           int num_threshold_bin, const uint32_t* threshold, int num_threshold, double left_value,
                           double right_value, int left_cnt, int right_cnt, double left_weight, double right_weight,
                           float gain, MissingType missing_type) {
  SplitCommon(leaf, feature_inner, real_feature, left_value, right_value, left_cnt, right_cnt, left_weight,
              right_weight, gain);
  const int node = num_leaves_ - 1;
  int8_t dt = kCategoricalMask;
  dt |= static_cast<int8_t>(static_cast<int>(missing_type) << 2);
  decision_type_[node] = dt;
  threshold_in_bin_[node] = static_cast<uint32_t>(num_cat_);
  threshold_[node] = static_cast<double>(num_cat_);
  ++num_cat_;
  cat_boundaries_.push_back(cat_boundaries_.back() + num_threshold);
  for (int i = 0; i < num_threshold; ++i) cat_threshold_.push_back(threshold[i]);
  cat_boundaries_inner_.push_back(cat_boundaries_inner_.back() + num_threshold_bin);
  for (int i = 0; i < num_threshold_bin; ++i) cat_threshold_inner_.push_back(threshold_bin[i]);
  ++num_leaves_;
  return num_leaves_ - 1;
}

void Tree::Shrinkage(double rate) {
  for (int i = 0; i < num_leaves_; ++i) {
    leaf_value_[i] = MaybeRoundToZero(leaf_value_[i] * rate);
    if (i < num_leaves_ - 1) internal_value_[i] = MaybeRoundToZero(internal_value_[i] * rate);
    if (is_linear_) {
      leaf_const_[i] = MaybeRoundToZero(leaf_const_[i] * rate);
      for (auto& c : leaf_coeff_[i]) c = MaybeRoundToZero(c * rate);
    }
  }
  shrinkage_ *= rate;
}

void Tree::AddBias(double val) {
  for (int i = 0; i < num_leaves_; ++i) {
    leaf_value_[i] = MaybeRoundToZero(leaf_value_[i] + val);
    if (i < num_leaves_ - 1) internal_value_[i] = MaybeRoundToZero(internal_value_[i] + val);
    if (is_linear_) leaf_const_[i] = MaybeRoundToZero(leaf_const_[i] + val);
  }
  shrinkage_ = 1.0;
}

void Tree::SetLeafCoeffs(int leaf, const std::vector<double>& c) {
  leaf_coeff_[leaf].resize(c.size());
  for (size_t i = 0; i < c.size(); ++i) leaf_coeff_[leaf][i] = MaybeRoundToZero(c[i]);
}

void Tree::RecomputeLeafDepths() {
  if (num_leaves_ <= 1) {
    leaf_depth_.assign(std::max(num_leaves_, 1), 0);
    return;
  }
  leaf_depth_.assign(max_leaves_, 0);
  std::vector<std::pair<int, int>> st = {{0, 0}};
  while (!st.empty()) {
    auto [n, d] = st.back();
    st.pop_back();
    for (int c : {left_child_[n], right_child_[n]}) {
      if (c < 0) leaf_depth_[~c] = d + 1;
      else st.push_back({c, d + 1});
    }
  }
}

void Tree::RecomputeMaxDepth() {
  if (num_leaves_ == 1) {
    max_depth_ = 0;
    return;
  }
  RecomputeLeafDepths();
  max_depth_ = 0;
  for (int i = 0; i < num_leaves_; ++i) max_depth_ = std::max(max_depth_, leaf_depth_[i]);
}

// ---------------------------------------------------------------------------
int Tree::GetLeafByBins(const Dataset& data, data_size_t row) const {
  int node = 0;
  while (node >= 0) {
    const int f = split_feature_inner_[node];
    const FeatureInfo& fi = data.feature(f);
    const uint32_t bin = data.FeatureBin(row, f);
    const int8_t dt = decision_type_[node];
    if (GetDecisionType(dt, kCategoricalMask)) {
      int ci = static_cast<int>(threshold_in_bin_[node]);
      int b = cat_boundaries_inner_[ci], e = cat_boundaries_inner_[ci + 1];
      bool left = common::FindInBitset(cat_threshold_inner_.data() + b, e - b, static_cast<int>(bin));
      node = left ? left_child_[node] : right_child_[node];
    } else {
      const int8_t mt = GetMissingType(dt);
      if ((mt == static_cast<int8_t>(MissingType::Zero) && bin == fi.default_bin) ||
          (mt == static_cast<int8_t>(MissingType::NaN) && bin == static_cast<uint32_t>(fi.num_bin - 1))) {
        node = GetDecisionType(dt, kDefaultLeftMask) ? left_child_[node] : right_child_[node];
      } else {
        node = bin <= threshold_in_bin_[node] ? left_child_[node] : right_child_[node];
      }
    }
  }
  return ~node;
}

void Tree::AddPredictionToScore(const Dataset& data, data_size_t num_data, double* score) const {
  if (num_leaves_ <= 1) {
    if (leaf_value_[0] != 0.0) {
#pragma omp parallel for schedule(static)
      for (data_size_t i = 0; i < num_data; ++i) score[i] += leaf_value_[0];
    }
    return;
  }
#pragma omp parallel for schedule(static, 2048)
  for (data_size_t i = 0; i < num_data; ++i) score[i] += LinearOrConstOutput(data, i, GetLeafByBins(data, i));
}

void Tree::AddPredictionToScore(const Dataset& data, const data_size_t* idx, data_size_t n, double* score) const {
  if (num_leaves_ <= 1 && !is_linear_) {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) score[idx[i]] += leaf_value_[0];
    return;
  }
#pragma omp parallel for schedule(static, 2048)
  for (data_size_t i = 0; i < n; ++i) {
    const int leaf = num_leaves_ > 1 ? GetLeafByBins(data, idx[i]) : 0;
    score[idx[i]] += LinearOrConstOutput(data, idx[i], leaf);
  }
}

double Tree::LinearOrConstOutput(const Dataset& data, data_size_t row, int leaf) const {
  if (!is_linear_) return leaf_value_[leaf];
  if (!data.has_raw()) Log::Fatal("Linear trees need raw feature values in the Dataset (linear_tree=true)");
  double v = leaf_const_[leaf];
  const auto& f = leaf_features_inner_[leaf];
  for (size_t k = 0; k < f.size(); ++k) {
    const double x = data.raw(row, f[k]);
    if (std::isnan(x)) return leaf_value_[leaf];
    v += leaf_coeff_[leaf][k] * x;
  }
  return v;
}

// ---------------------------------------------------------------------------
int Tree::GetLeafByMap(const std::unordered_map<int, double>& f) const {
  int node = 0;
  while (node >= 0) {
    auto it = f.find(split_feature_[node]);
    node = Decision(it == f.end() ? 0.0 : it->second, node);
  }
  return ~node;
}

double Tree::PredictByMap(const std::unordered_map<int, double>& f) const {
  if (num_leaves_ <= 1) return leaf_value_[0];
  int leaf = GetLeafByMap(f);
  if (!is_linear_) return leaf_value_[leaf];
  double out = leaf_const_[leaf];
  for (size_t i = 0; i < leaf_features_[leaf].size(); ++i) {
    auto it = f.find(leaf_features_[leaf][i]);
    double v = it == f.end() ? 0.0 : it->second;
    if (std::isnan(v)) return leaf_value_[leaf];
    out += leaf_coeff_[leaf][i] * v;
  }
  return out;
}

int Tree::PredictLeafIndexByMap(const std::unordered_map<int, double>& f) const {
  return num_leaves_ > 1 ? GetLeafByMap(f) : 0;
}

double Tree::ExpectedValue() const {
  if (num_leaves_ == 1) return leaf_value_[0];
  const double total = internal_count_[0];
  double e = 0.0;
  for (int i = 0; i < num_leaves_; ++i) e += (leaf_count_[i] / total) * leaf_value_[i];
  return e;
}

// TreeSHAP (Lundberg et al. 2018, Algorithm 2) over the per-node data counts.
namespace {
struct PE {
  int f;
  double z, o, w;
};
void Extend(PE* p, int d, double z, double o, int f) {
  p[d].f = f;
  p[d].z = z;
  p[d].o = o;
  p[d].w = d == 0 ? 1.0 : 0.0;
  for (int i = d - 1; i >= 0; --i) {
    p[i + 1].w += o * p[i].w * (i + 1) / static_cast<double>(d + 1);
    p[i].w = z * p[i].w * (d - i) / static_cast<double>(d + 1);
  }
}
void Unwind(PE* p, int d, int k) {
  const double o = p[k].o, z = p[k].z;
  double next = p[d].w;
  for (int i = d - 1; i >= 0; --i) {
    if (o != 0) {
      const double t = p[i].w;
      p[i].w = next * (d + 1) / static_cast<double>((i + 1) * o);
      next = t - p[i].w * z * (d - i) / static_cast<double>(d + 1);
    } else {
      p[i].w = p[i].w * (d + 1) / static_cast<double>(z * (d - i));
    }
  }
  for (int i = k; i < d; ++i) {
    p[i].f = p[i + 1].f;
    p[i].z = p[i + 1].z;
    p[i].o = p[i + 1].o;
  }
}
double UnwoundSum(const PE* p, int d, int k) {
  const double o = p[k].o, z = p[k].z;
  double next = p[d].w, total = 0.0;
  for (int i = d - 1; i >= 0; --i) {
    if (o != 0) {
      const double t = next * (d + 1) / static_cast<double>((i + 1) * o);
      total += t;
      next = p[i].w - t * z * ((d - i) / static_cast<double>(d + 1));
    } else {
      total += (p[i].w / z) / ((d - i) / static_cast<double>(d + 1));
    }
  }
  return total;
}
}  // namespace

void Tree::TreeSHAP(const double* x, double* phi, int node, int depth, PathElement* parent_path, double pz, double po,
                    int pf) const {
  PE* parent = reinterpret_cast<PE*>(parent_path);
  PE* path = parent + depth;
  if (depth > 0) std::copy(parent, parent + depth, path);
  Extend(path, depth, pz, po, pf);
  if (node < 0) {
    const double v = leaf_value_[~node];
    for (int i = 1; i <= depth; ++i) {
      const double w = UnwoundSum(path, depth, i);
      phi[path[i].f] += w * (path[i].o - path[i].z) * v;
    }
    return;
  }
  const int hot = Decision(x[split_feature_[node]], node);
  const int cold = hot == left_child_[node] ? right_child_[node] : left_child_[node];
  const double w = DataCount(node);
  const double hz = DataCount(hot) / w, cz = DataCount(cold) / w;
  double iz = 1.0, io = 1.0;
  int k = 0;
  for (; k <= depth; ++k) if (path[k].f == split_feature_[node]) break;
  if (k != depth + 1) {
    iz = path[k].z;
    io = path[k].o;
    Unwind(path, depth, k);
    depth -= 1;
  }
  TreeSHAP(x, phi, hot, depth + 1, reinterpret_cast<PathElement*>(path), hz * iz, io, split_feature_[node]);
  TreeSHAP(x, phi, cold, depth + 1, reinterpret_cast<PathElement*>(path), cz * iz, 0.0, split_feature_[node]);
}

void Tree::PredictContrib(const double* x, int num_features, double* out) const {
  out[num_features] += ExpectedValue();
  if (num_leaves_ > 1) {
    int md = 0;
    for (int i = 0; i < num_leaves_; ++i) md = std::max(md, leaf_depth_[i]);
    if (md == 0) {
      const_cast<Tree*>(this)->RecomputeLeafDepths();
      for (int i = 0; i < num_leaves_; ++i) md = std::max(md, leaf_depth_[i]);
    }
    const int max_path = (md + 2) * (md + 3) / 2 + 4;
    std::vector<PE> buf(max_path);
    TreeSHAP(x, out, 0, 0, reinterpret_cast<PathElement*>(buf.data()), 1.0, 1.0, -1);
  }
}

void Tree::PredictContribByMap(const std::unordered_map<int, double>& f, int num_features,
                               std::unordered_map<int, double>* out) const {
  // densify the touched features and reuse the dense path
  std::vector<double> x(num_features, 0.0);
  for (auto& kv : f) if (kv.first < num_features) x[kv.first] = kv.second;
  std::vector<double> phi(num_features + 1, 0.0);
  PredictContrib(x.data(), num_features, phi.data());
  for (int i = 0; i <= num_features; ++i) {
    if (phi[i] != 0.0) (*out)[i] += phi[i];
  }
}

// ---------------------------------------------------------------------------
std::string Tree::ToString() const {
  using common::ArrayToString;
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  const size_t ni = static_cast<size_t>(num_leaves_ - 1);
  const size_t nl = static_cast<size_t>(num_leaves_);
  ss << "num_leaves=" << num_leaves_ << '\n';
  ss << "num_cat=" << num_cat_ << '\n';
  ss << "split_feature=" << ArrayToString(split_feature_, ni) << '\n';
  ss << "split_gain=" << ArrayToString(split_gain_, ni) << '\n';
  ss << "threshold=" << ArrayToString<true>(threshold_, ni) << '\n';
  std::vector<int> dt(decision_type_.begin(), decision_type_.end());
  ss << "decision_type=" << ArrayToString(dt, ni) << '\n';
  ss << "left_child=" << ArrayToString(left_child_, ni) << '\n';
  ss << "right_child=" << ArrayToString(right_child_, ni) << '\n';
  ss << "leaf_value=" << ArrayToString<true>(leaf_value_, nl) << '\n';
  ss << "leaf_weight=" << ArrayToString<true>(leaf_weight_, nl) << '\n';
  ss << "leaf_count=" << ArrayToString(leaf_count_, nl) << '\n';
  ss << "internal_value=" << ArrayToString(internal_value_, ni) << '\n';
  ss << "internal_weight=" << ArrayToString(internal_weight_, ni) << '\n';
  ss << "internal_count=" << ArrayToString(internal_count_, ni) << '\n';
  if (num_cat_ > 0) {
    ss << "cat_boundaries=" << ArrayToString(cat_boundaries_, num_cat_ + 1) << '\n';
    ss << "cat_threshold=" << ArrayToString(cat_threshold_, cat_threshold_.size()) << '\n';
  }
  ss << "is_linear=" << (is_linear_ ? 1 : 0) << '\n';
  if (is_linear_) {
    ss << "leaf_const=" << ArrayToString<true>(leaf_const_, nl) << '\n';
    std::vector<int> nf(nl);
    for (size_t i = 0; i < nl; ++i) nf[i] = static_cast<int>(leaf_coeff_[i].size());
    ss << "num_features=" << ArrayToString(nf, nl) << '\n';
    ss << "leaf_features=";
    for (size_t i = 0; i < nl; ++i) {
      if (nf[i] > 0) ss << ArrayToString(leaf_features_[i], leaf_features_[i].size()) << ' ';
      ss << ' ';
    }
    ss << '\n';
    ss << "leaf_coeff=";
    for (size_t i = 0; i < nl; ++i) {
      if (nf[i] > 0) ss << ArrayToString<true>(leaf_coeff_[i], leaf_coeff_[i].size()) << ' ';
      ss << ' ';
    }
    ss << '\n';
  }
  ss << "shrinkage=" << common::FormatG(shrinkage_) << '\n';
  ss << '\n';
  return ss.str();
}

Tree::Tree(const char* str, size_t* used_len) {
  // parse "key=value" lines until an empty line / next "Tree=" / "end of trees"
  std::unordered_map<std::string, std::string> kv;
  const char* p = str;
  while (*p) {
    const char* e = p;
    while (*e && *e != '\n' && *e != '\r') ++e;
    std::string line(p, e - p);
    while (*e == '\n' || *e == '\r') ++e;
    if (line.empty()) {
      p = e;
      if (!kv.empty()) break;
      continue;
    }
    if (common::StartsWith(line, "Tree=") || common::StartsWith(line, "end of trees")) {
      if (!kv.empty()) break;
      p = e;
      continue;
    }
    size_t eq = line.find('=');
    if (eq != std::string::npos) kv[line.substr(0, eq)] = line.substr(eq + 1);
    p = e;
  }
  if (used_len) *used_len = static_cast<size_t>(p - str);
  auto need = [&](const char* k) -> const std::string& {
    auto it = kv.find(k);
    if (it == kv.end()) Log::Fatal("Tree model string format error, should contain %s field", k);
    return it->second;
  };
  num_leaves_ = common::AtoiOrDie(need("num_leaves"));
  max_leaves_ = num_leaves_;
  num_cat_ = common::AtoiOrDie(need("num_cat"));
  const size_t ni = static_cast<size_t>(std::max(num_leaves_ - 1, 0));
  leaf_value_ = common::StringToArray<double>(need("leaf_value"), num_leaves_);
  if (num_leaves_ > 1) {
    left_child_ = common::StringToArray<int>(need("left_child"), ni);
    right_child_ = common::StringToArray<int>(need("right_child"), ni);
    split_feature_ = common::StringToArray<int>(need("split_feature"), ni);
    threshold_ = common::StringToArray<double>(need("threshold"), ni);
    auto dt = kv.count("decision_type") ? common::StringToArray<int>(kv["decision_type"], ni) : std::vector<int>(ni, 0);
    decision_type_.assign(dt.begin(), dt.end());
    split_gain_ = kv.count("split_gain") ? common::StringToArray<float>(kv["split_gain"], ni) : std::vector<float>(ni, 0);
    internal_value_ = kv.count("internal_value") ? common::StringToArray<double>(kv["internal_value"], ni)
                                                 : std::vector<double>(ni, 0);
    internal_weight_ = kv.count("internal_weight") ? common::StringToArray<double>(kv["internal_weight"], ni)
                                                   : std::vector<double>(ni, 0);
    internal_count_ = kv.count("internal_count") ? common::StringToArray<int>(kv["internal_count"], ni)
                                                 : std::vector<int>(ni, 0);
  } else {
    left_child_.assign(1, 0);
    right_child_.assign(1, 0);
    split_feature_.assign(1, -1);
    threshold_.assign(1, 0);
    decision_type_.assign(1, 0);
    split_gain_.assign(1, 0);
    internal_value_.assign(1, 0);
    internal_weight_.assign(1, 0);
    internal_count_.assign(1, 0);
  }
  split_feature_inner_ = split_feature_;
  threshold_in_bin_.assign(split_feature_.size(), 0);
  leaf_weight_ = kv.count("leaf_weight") ? common::StringToArray<double>(kv["leaf_weight"], num_leaves_)
                                         : std::vector<double>(num_leaves_, 0);
  leaf_count_ = kv.count("leaf_count") ? common::StringToArray<int>(kv["leaf_count"], num_leaves_)
                                       : std::vector<int>(num_leaves_, 0);
  leaf_parent_.assign(num_leaves_, -1);
  for (size_t n = 0; n < ni; ++n) {
    if (left_child_[n] < 0) leaf_parent_[~left_child_[n]] = static_cast<int>(n);
    if (right_child_[n] < 0) leaf_parent_[~right_child_[n]] = static_cast<int>(n);
  }
  cat_boundaries_ = {0};
  cat_boundaries_inner_ = {0};
  if (num_cat_ > 0) {
    cat_boundaries_ = common::StringToArray<int>(need("cat_boundaries"), num_cat_ + 1);
    cat_threshold_ = common::StringToArray<uint32_t>(need("cat_threshold"), cat_boundaries_.back());
  }
  shrinkage_ = kv.count("shrinkage") ? common::AtofOrDie(kv["shrinkage"]) : 1.0;
  is_linear_ = kv.count("is_linear") && common::AtoiOrDie(kv["is_linear"]) != 0;
  if (is_linear_) {
    leaf_const_ = common::StringToArray<double>(need("leaf_const"), num_leaves_);
    auto nf = common::StringToArray<int>(need("num_features"), num_leaves_);
    auto lf = common::StringToArray<int>(kv["leaf_features"]);
    auto lc = common::StringToArray<double>(kv["leaf_coeff"]);
    leaf_features_.assign(num_leaves_, {});
    leaf_features_inner_.assign(num_leaves_, {});
    leaf_coeff_.assign(num_leaves_, {});
    size_t k = 0;
    for (int i = 0; i < num_leaves_; ++i) {
      for (int j = 0; j < nf[i]; ++j, ++k) {
        leaf_features_[i].push_back(lf[k]);
        leaf_coeff_[i].push_back(lc[k]);
      }
    }
  }
  leaf_depth_.assign(num_leaves_, 0);
  RecomputeLeafDepths();
  max_depth_ = -1;
}

// ---------------------------------------------------------------------------
namespace {
std::string J(double v) {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2) << common::AvoidInf(v);
  return ss.str();
}
}  // namespace

std::string Tree::LinearModelToJSON(int leaf) const {
  std::stringstream ss;
  ss << "\"leaf_const\":" << J(leaf_const_[leaf]) << ",\n";
  ss << "\"leaf_features\":[";
  for (size_t i = 0; i < leaf_features_[leaf].size(); ++i) ss << (i ? ", " : "") << leaf_features_[leaf][i];
  ss << "],\n\"leaf_coeff\":[";
  for (size_t i = 0; i < leaf_coeff_[leaf].size(); ++i) ss << (i ? ", " : "") << J(leaf_coeff_[leaf][i]);
  ss << "]\n";
  return ss.str();
}

std::string Tree::NodeToJSON(int index) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  if (index >= 0) {
    ss << "{\n\"split_index\":" << index << ",\n";
    ss << "\"split_feature\":" << split_feature_[index] << ",\n";
    ss << "\"split_gain\":" << J(split_gain_[index]) << ",\n";
    if (GetDecisionType(decision_type_[index], kCategoricalMask)) {
      int ci = static_cast<int>(threshold_[index]);
      std::vector<int> cats;
      for (int i = cat_boundaries_[ci]; i < cat_boundaries_[ci + 1]; ++i)
        for (int j = 0; j < 32; ++j)
          if ((cat_threshold_[i] >> j) & 1) cats.push_back((i - cat_boundaries_[ci]) * 32 + j);
      ss << "\"threshold\":\"" << common::Join(cats, "||") << "\",\n\"decision_type\":\"==\",\n";
    } else {
      ss << "\"threshold\":" << J(threshold_[index]) << ",\n\"decision_type\":\"<=\",\n";
    }
    ss << "\"default_left\":" << (GetDecisionType(decision_type_[index], kDefaultLeftMask) ? "true" : "false") << ",\n";
    int mt = GetMissingType(decision_type_[index]);
    ss << "\"missing_type\":\"" << (mt == 0 ? "None" : mt == 1 ? "Zero" : "NaN") << "\",\n";
    ss << "\"internal_value\":" << J(internal_value_[index]) << ",\n";
    ss << "\"internal_weight\":" << J(internal_weight_[index]) << ",\n";
    ss << "\"internal_count\":" << internal_count_[index] << ",\n";
    ss << "\"left_child\":" << NodeToJSON(left_child_[index]) << ",\n";
    ss << "\"right_child\":" << NodeToJSON(right_child_[index]) << "\n}";
  } else {
    int l = ~index;
    ss << "{\n\"leaf_index\":" << l << ",\n";
    ss << "\"leaf_value\":" << J(leaf_value_[l]) << ",\n";
    ss << "\"leaf_weight\":" << J(leaf_weight_[l]) << ",\n";
    if (is_linear_) {
      ss << "\"leaf_count\":" << leaf_count_[l] << ",\n" << LinearModelToJSON(l);
    } else {
      ss << "\"leaf_count\":" << leaf_count_[l] << "\n";
    }
    ss << "}";
  }
  return ss.str();
}

std::string Tree::ToJSON() const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << "\"num_leaves\":" << num_leaves_ << ",\n";
  ss << "\"num_cat\":" << num_cat_ << ",\n";
  ss << "\"shrinkage\":" << J(shrinkage_) << ",\n";
  if (num_leaves_ == 1) {
    ss << "\"tree_structure\":{\"leaf_value\":" << J(leaf_value_[0]) << ", \n";
    if (is_linear_) ss << "\"leaf_count\":" << leaf_count_[0] << ", \n" << LinearModelToJSON(0);
    else ss << "\"leaf_count\":" << leaf_count_[0];
    ss << "}\n";
  } else {
    ss << "\"tree_structure\":" << NodeToJSON(0) << "\n";
  }
  return ss.str();
}

std::string Tree::NodeToIfElse(int index, bool predict_leaf_index) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  if (index >= 0) {
    const int f = split_feature_[index];
    ss << "fval = arr[" << f << "];";
    if (GetDecisionType(decision_type_[index], kCategoricalMask)) {
      int ci = static_cast<int>(threshold_[index]);
      ss << "int_fval = static_cast<int>(fval); if (!std::isnan(fval) && int_fval >= 0 && (int_fval / 32) < "
         << (cat_boundaries_[ci + 1] - cat_boundaries_[ci]) << " && ((cat_threshold[" << cat_boundaries_[ci]
         << " + int_fval / 32] >> (int_fval & 31)) & 1)) {";
    } else {
      int mt = GetMissingType(decision_type_[index]);
      bool dl = GetDecisionType(decision_type_[index], kDefaultLeftMask);
      if (mt != 2) ss << "if (std::isnan(fval)) fval = 0.0;";
      if (mt == 1) {
        ss << (dl ? "if ((fval >= -1e-35 && fval <= 1e-35) || fval <= " : "if (!(fval >= -1e-35 && fval <= 1e-35) && fval <= ")
           << threshold_[index] << ") {";
      } else if (mt == 2) {
        ss << (dl ? "if (std::isnan(fval) || fval <= " : "if (!std::isnan(fval) && fval <= ") << threshold_[index]
           << ") {";
      } else {
        ss << "if (fval <= " << threshold_[index] << ") {";
      }
    }
    ss << NodeToIfElse(left_child_[index], predict_leaf_index) << "} else {"
       << NodeToIfElse(right_child_[index], predict_leaf_index) << "}";
  } else {
    if (predict_leaf_index) ss << "return " << ~index << ";";
    else ss << "return " << leaf_value_[~index] << ";";
  }
  return ss.str();
}

std::string Tree::ToIfElse(int index, bool predict_leaf_index) const {
  std::stringstream ss;
  ss.imbue(std::locale::classic());
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  ss << "double PredictTree" << index << (predict_leaf_index ? "Leaf" : "") << "(const double* arr) { ";
  if (num_cat_ > 0) {
    ss << "static const uint32_t cat_threshold[] = {" << common::Join(cat_threshold_, ",") << "}; ";
  }
  if (num_leaves_ <= 1) {
    ss << "return " << (predict_leaf_index ? 0.0 : leaf_value_[0]) << "; }\n";
    return ss.str();
  }
  ss << "double fval = 0.0; int int_fval = 0; (void)int_fval; " << NodeToIfElse(0, predict_leaf_index) << " }\n";
  return ss.str();
}

}  // namespace lgap
