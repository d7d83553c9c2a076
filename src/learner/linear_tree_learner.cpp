// Linear-leaf trees (reference src/treelearner/linear_tree_learner.cpp): grow
// the tree with the serial learner, then fit per leaf a ridge regression
//   min_b sum_i h_i (g_i/h_i + x_i.b)^2 + linear_lambda |b|^2
// on the numerical features used on the leaf's branch (Newton step on the
// second-order approximation), solved by Cholesky.
#include <algorithm>
#include <cmath>
#include <unordered_map>

#include "lgap/log.h"
#include "linear_solve.h"
#include "parallel_tree_learner.h"

namespace lgap {

namespace {

class LinearTreeLearner : public SerialTreeLearner {
 public:
  explicit LinearTreeLearner(const Config* c) : SerialTreeLearner(c) {}

  void Init(const Dataset* train_data, bool is_constant_hessian) override {
    SerialTreeLearner::Init(train_data, is_constant_hessian);
    if (!train_data->has_raw() && train_data->num_features() > 0) {
      Log::Fatal("linear_tree requires the Dataset to keep raw feature values (construct it with linear_tree=true)");
    }
    has_nan_ = false;
    for (data_size_t i = 0; i < train_data->num_data() && !has_nan_; ++i) {
      for (int f = 0; f < train_data->num_features() && !has_nan_; ++f) has_nan_ = std::isnan(train_data->raw(i, f));
    }
  }

  std::unique_ptr<Tree> Train(const score_t* g, const score_t* h, bool first) override {
    auto base = SerialTreeLearner::Train(g, h, first);
    // same structure (inner indices, bin thresholds) plus linear leaf models
    auto tree = std::make_unique<Tree>(*base);
    tree->SetIsLinear(true);
    tree->InitLinear();
    const int nl = tree->num_leaves();
    if (first) {
      // the first tree only carries constants (reference CalculateLinear is_first_tree, :184-189)
      for (int l = 0; l < nl; ++l) tree->SetLeafConst(l, tree->LeafOutput(l));
      return tree;
    }
#pragma omp parallel for schedule(dynamic) if (nl > 1)
    for (int l = 0; l < nl; ++l) {
      const std::vector<int> feats = BranchFeatures(base.get(), l);
      std::vector<double> z;
      if (!SolveLeaf(feats, l, g, h, &z)) {
        tree->SetLeafConst(l, tree->LeafOutput(l));
        continue;
      }
      // coefficients that round to zero are dropped (reference :365-369)
      std::vector<double> coef;
      std::vector<int> inner, real;
      for (size_t j = 0; j < feats.size(); ++j) {
        if (Tree::IsZero(z[j])) continue;
        coef.push_back(z[j]);
        inner.push_back(feats[j]);
        real.push_back(train_data_->feature(feats[j]).real_index);
      }
      tree->SetLeafConst(l, z[feats.size()]);
      tree->SetLeafCoeffs(l, coef);
      tree->SetLeafFeatures(l, real);
      tree->SetLeafFeaturesInner(l, inner);
    }
    return tree;
  }

  // refit: the leaf outputs are refit by the serial learner, then each leaf's linear model
  // is re-solved on the new rows over the features it already uses and blended with
  //   new = decay * old + (1 - decay) * solved * shrinkage
  // (reference FitByExistingTree :136-160 and CalculateLinear is_refit, :330-385). A leaf
  // with too few usable rows keeps zeroed coefficients and blends its constant towards the
  // (already refit) leaf output.
  std::unique_ptr<Tree> FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                          const score_t* g, const score_t* h) override {
    auto tree = SerialTreeLearner::FitByExistingTree(old_tree, leaf_pred, g, h);
    tree->SetIsLinear(true);
    const double decay = config_->refit_decay_rate, shrink = tree->shrinkage();
    const int nl = tree->num_leaves();
#pragma omp parallel for schedule(dynamic) if (nl > 1)
    for (int l = 0; l < nl; ++l) {
      std::vector<int> feats;
      for (int rf : tree->LeafFeatures(l)) {
        const int f = train_data_->InnerIndex(rf);
        if (f >= 0 && train_data_->feature(f).bin_type == BinType::Numerical) feats.push_back(f);
      }
      std::sort(feats.begin(), feats.end());
      feats.erase(std::unique(feats.begin(), feats.end()), feats.end());
      // old coefficients by real feature id (the rebuilt list may drop / reorder features)
      std::unordered_map<int, double> old_by_feature;
      {
        const auto& of = tree->LeafFeatures(l);
        const auto& oc = tree->LeafCoeffs(l);
        for (size_t j = 0; j < of.size() && j < oc.size(); ++j) old_by_feature[of[j]] = oc[j];
      }
      const double old_const = tree->LeafConst(l);
      std::vector<int> real(feats.size());
      for (size_t j = 0; j < feats.size(); ++j) real[j] = train_data_->feature(feats[j]).real_index;
      std::vector<double> z;
      std::vector<double> coef(feats.size(), 0.0);
      if (!SolveLeaf(feats, l, g, h, &z)) {
        tree->SetLeafConst(l, decay * old_const + (1.0 - decay) * tree->LeafOutput(l) * shrink);
      } else {
        for (size_t j = 0; j < feats.size(); ++j) {
          const auto it = old_by_feature.find(real[j]);
          const double o = it != old_by_feature.end() ? it->second : 0.0;
          coef[j] = decay * o + (1.0 - decay) * z[j] * shrink;
        }
        tree->SetLeafConst(l, decay * old_const + (1.0 - decay) * z[feats.size()] * shrink);
      }
      tree->SetLeafCoeffs(l, coef);
      tree->SetLeafFeatures(l, real);
      tree->SetLeafFeaturesInner(l, feats);
    }
    return tree;
  }

  void AddPredictionToScore(const Tree* tree, double* out) const override {
    const Dataset* d = train_data_;
    for (int l = 0; l < tree->num_leaves(); ++l) {
      const data_size_t n = partition_.count(l);
      const data_size_t* idx = partition_.indices(l);
      const auto& feats = tree->LeafFeaturesInner(l);
      const auto& coef = tree->LeafCoeffs(l);
      for (data_size_t i = 0; i < n; ++i) {
        double v = tree->LeafConst(l);
        bool nan = false;
        for (size_t k = 0; k < feats.size(); ++k) {
          const double x = d->raw(idx[i], feats[k]);
          if (std::isnan(x)) {
            nan = true;
            break;
          }
          v += coef[k] * x;
        }
        out[idx[i]] += nan ? tree->LeafOutput(l) : v;
      }
    }
  }

 private:
  // distinct numerical features split on along the leaf's branch, sorted (inner indices)
  std::vector<int> BranchFeatures(const Tree* base, int leaf) const {
    std::vector<int> parent(std::max(1, base->num_leaves() - 1), -1);
    for (int p = 0; p < base->num_leaves() - 1; ++p) {
      if (base->left_child(p) >= 0) parent[base->left_child(p)] = p;
      if (base->right_child(p) >= 0) parent[base->right_child(p)] = p;
    }
    std::vector<int> feats;
    for (int node = base->leaf_parent(leaf); node >= 0; node = parent[node]) {
      const int f = base->split_feature_inner(node);
      if (train_data_->feature(f).bin_type == BinType::Numerical) feats.push_back(f);
    }
    std::sort(feats.begin(), feats.end());
    feats.erase(std::unique(feats.begin(), feats.end()), feats.end());
    return feats;
  }

  // Newton step of the leaf's rows on [x, 1]: z = -(X'HX + lambda I_x)^-1 X'g (reference
  // CalculateLinear :191-356; Eq. 3 of arXiv:1802.05640). Rows with a NaN in any of the
  // features are left out. False when fewer usable rows than unknowns or the system is not
  // positive definite.
  bool SolveLeaf(const std::vector<int>& feats, int leaf, const score_t* g, const score_t* h,
                 std::vector<double>* out) const {
    const int k = static_cast<int>(feats.size()), m = k + 1;
    const data_size_t n = partition_.count(leaf);
    const data_size_t* idx = partition_.indices(leaf);
    std::vector<double> A(static_cast<size_t>(m) * m, 0.0), b(m, 0.0), x(m);
    // "enough data" follows the reference's count (CalculateLinear :266-324): with NaNs in
    // the dataset it counts the non-NaN values read (so a leaf without features never has
    // enough and keeps its constant output), otherwise the leaf's rows
    int64_t usable = has_nan_ ? 0 : n;
    for (data_size_t i = 0; i < n; ++i) {
      bool nan = false;
      for (int j = 0; j < k && !nan; ++j) {
        x[j] = train_data_->raw(idx[i], feats[j]);
        nan = std::isnan(x[j]);
        if (has_nan_ && !nan) ++usable;
      }
      if (nan) continue;
      x[k] = 1.0;
      const double hh = h[idx[i]], gg = g[idx[i]];
      for (int a = 0; a < m; ++a) {
        b[a] -= gg * x[a];
        const double hx = hh * x[a];
        for (int c = 0; c <= a; ++c) A[a * m + c] += hx * x[c];
      }
    }
    return SolveLinearLeaf(std::move(A), b, usable, m, config_->linear_lambda, out);
  }
  bool has_nan_ = false;
};

}  // namespace

std::unique_ptr<TreeLearner> CreateLinearTreeLearner(const Config* config) {
  return std::make_unique<LinearTreeLearner>(config);
}

}  // namespace lgap
