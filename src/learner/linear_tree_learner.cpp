// Linear-leaf trees (reference src/treelearner/linear_tree_learner.cpp): grow
// the tree with the serial learner, then fit per leaf a ridge regression
//   min_b sum_i h_i (g_i/h_i + x_i.b)^2 + linear_lambda |b|^2
// on the numerical features used on the leaf's branch (Newton step on the
// second-order approximation), solved by Cholesky.
#include <cmath>

#include "lgap/log.h"
#include "parallel_tree_learner.h"

namespace lgap {

namespace {

class LinearTreeLearner : public SerialTreeLearner {
 public:
  explicit LinearTreeLearner(const Config* c) : SerialTreeLearner(c) {}

  void Init(const Dataset* train_data, bool is_constant_hessian) override {
    SerialTreeLearner::Init(train_data, is_constant_hessian);
    if (!train_data->has_raw()) {
      Log::Fatal("linear_tree requires the Dataset to keep raw feature values (construct it with linear_tree=true)");
    }
  }

  std::unique_ptr<Tree> Train(const score_t* g, const score_t* h, bool first) override {
    auto base = SerialTreeLearner::Train(g, h, first);
    // same structure (inner indices, bin thresholds) plus linear leaf models
    auto tree = std::make_unique<Tree>(*base);
    tree->SetIsLinear(true);
    tree->InitLinear();
    const int nl = tree->num_leaves();
    for (int l = 0; l < nl; ++l) {
      FitLeaf(tree.get(), base.get(), l, g, h);
    }
    last_ = std::move(tree);
    // keep the inner (binned) structure for score updates
    return std::make_unique<Tree>(*last_);
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
  void FitLeaf(Tree* tree, const Tree* base, int leaf, const score_t* g, const score_t* h) {
    // numerical features on the branch (inner indices)
    std::vector<int> feats;
    int node = base->leaf_parent(leaf);
    while (node >= 0) {
      const int f = base->split_feature_inner(node);
      if (train_data_->feature(f).bin_type == BinType::Numerical &&
          std::find(feats.begin(), feats.end(), f) == feats.end()) {
        feats.push_back(f);
      }
      // walk up
      int parent = -1;
      for (int p = 0; p < base->num_leaves() - 1; ++p) {
        if (base->left_child(p) == node || base->right_child(p) == node) {
          parent = p;
          break;
        }
      }
      node = parent;
    }
    std::sort(feats.begin(), feats.end());
    const int k = static_cast<int>(feats.size());
    const data_size_t n = partition_.count(leaf);
    const data_size_t* idx = partition_.indices(leaf);
    // normal equations of [x, 1]
    const int m = k + 1;
    std::vector<double> A(static_cast<size_t>(m) * m, 0.0), b(m, 0.0);
    std::vector<double> x(m);
    for (data_size_t i = 0; i < n; ++i) {
      bool nan = false;
      for (int j = 0; j < k; ++j) {
        x[j] = train_data_->raw(idx[i], feats[j]);
        if (std::isnan(x[j])) nan = true;
      }
      if (nan) continue;
      x[k] = 1.0;
      const double hh = h[idx[i]], gg = g[idx[i]];
      for (int a = 0; a < m; ++a) {
        b[a] -= gg * x[a];
        for (int c = 0; c < m; ++c) A[a * m + c] += hh * x[a] * x[c];
      }
    }
    for (int j = 0; j < k; ++j) A[j * m + j] += config_->linear_lambda;
    // Cholesky solve (A is SPD after ridge; fall back to constant leaf on failure)
    std::vector<double> L(A.size(), 0.0);
    bool ok = true;
    for (int i = 0; i < m && ok; ++i) {
      for (int j = 0; j <= i; ++j) {
        double s = A[i * m + j];
        for (int t = 0; t < j; ++t) s -= L[i * m + t] * L[j * m + t];
        if (i == j) {
          if (s <= 1e-12) ok = false;
          else L[i * m + i] = std::sqrt(s);
        } else {
          L[i * m + j] = s / L[j * m + j];
        }
      }
    }
    const double shrink = config_->learning_rate;
    if (!ok || n < m) {
      tree->SetLeafConst(leaf, base->LeafOutput(leaf));
      tree->SetLeafCoeffs(leaf, {});
      tree->SetLeafFeatures(leaf, {});
      tree->SetLeafFeaturesInner(leaf, {});
      return;
    }
    std::vector<double> y(m), z(m);
    for (int i = 0; i < m; ++i) {
      double s = b[i];
      for (int t = 0; t < i; ++t) s -= L[i * m + t] * y[t];
      y[i] = s / L[i * m + i];
    }
    for (int i = m - 1; i >= 0; --i) {
      double s = y[i];
      for (int t = i + 1; t < m; ++t) s -= L[t * m + i] * z[t];
      z[i] = s / L[i * m + i];
    }
    (void)shrink;
    std::vector<double> coef(z.begin(), z.begin() + k);
    std::vector<int> real(k);
    for (int j = 0; j < k; ++j) real[j] = train_data_->feature(feats[j]).real_index;
    tree->SetLeafConst(leaf, z[k]);
    tree->SetLeafCoeffs(leaf, coef);
    tree->SetLeafFeatures(leaf, real);
    tree->SetLeafFeaturesInner(leaf, feats);
  }
  std::unique_ptr<Tree> last_;
};

}  // namespace

std::unique_ptr<TreeLearner> CreateLinearTreeLearner(const Config* config) {
  return std::make_unique<LinearTreeLearner>(config);
}

}  // namespace lgap
