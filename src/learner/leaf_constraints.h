// Host-side tree-growth policies that sit beside the split scan:
//  * MonotoneLeafConstraints — the "intermediate" monotone-constraint method
//    (reference src/treelearner/monotone_constraints.hpp:516-856): after each
//    split the constraint intervals of leaves that border the two new leaves
//    across a monotone split are tightened with the new leaves' actual outputs,
//    and those leaves get their best split recomputed; and the "advanced" method
//    (:858-1175): every leaf keeps, per numerical feature, bounds that vary along
//    the feature's bins, rebuilt exactly from the bordering leaves when stale, so
//    a split threshold is only constrained by the leaves its children touch.
//  * CegbPenalty — cost-effective gradient boosting
//    (reference src/treelearner/cost_effective_gradient_boosting.hpp:22-174):
//    split / coupled-feature / lazy per-row feature-acquisition penalties.
//  * GradientQuantizer — quantized-gradient training
//    (reference src/treelearner/gradient_discretizer.cpp:66-160): per-iteration
//    max-abs scaling of (g, h) to num_grad_quant_bins integer levels with
//    stochastic rounding. The host learner feeds the de-scaled integers (exact
//    in fp64) to its histograms, which reproduces integer-histogram semantics.
#pragma once

#include <cstdint>
#include <random>
#include <vector>

#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/split_math.h"
#include "lgap/tree.h"

namespace lgap {

// Piecewise-constant bound over the bins of one feature: val[i] holds on
// [start[i], start[i + 1]) and the last piece runs to the last bin.
struct BinPieces {
  std::vector<uint32_t> start;
  std::vector<double> val;
  void Reset(double v) {
    start.assign(1, 0u);
    val.assign(1, v);
  }
  // raise: v is a lower bound (max with it), else an upper bound (min with it)
  void TightenAll(double v, bool raise);
  // the same on the bins [b, e) only
  void TightenRange(double v, bool raise, uint32_t b, uint32_t e, uint32_t num_bin);
  void Expand(int num_bin, double* out) const;
  size_t size() const { return val.size(); }
  void Fuse();  // merges equal neighbouring pieces
};

class MonotoneLeafConstraints {
 public:
  // advanced: per-leaf, per-feature threshold-dependent bounds on top of the
  // intermediate bookkeeping
  void Init(const Dataset* data, int num_leaves, bool advanced);
  void Reset();
  bool advanced() const { return advanced_; }
  // before tree->Split(leaf): records the parent of the node about to be created
  void BeforeSplit(const Tree* tree, int leaf, int new_leaf, int8_t monotone_type);
  // after tree->Split: tightens bounds of the new leaves and of bordering leaves;
  // returns the leaves (other than the new ones) whose split must be recomputed
  std::vector<int> AfterSplit(const Tree* tree, std::vector<LeafBounds>* bounds, bool numerical, int leaf,
                              int new_leaf, int8_t monotone_type, const SplitInfo& split,
                              const std::vector<SplitInfo>& best_per_leaf);
  // advanced, before scanning numerical feature f of `leaf`: rebuilds a bound
  // flagged stale from the leaves that actually border `leaf` along f, then fills
  // `tb` (4 * num_bin doubles of `scratch`) when the bounds vary with the
  // threshold; otherwise returns false with the feature-wide bounds in `flat`
  bool ThresholdBoundsFor(const Tree* tree, int f, int leaf, std::vector<double>* scratch, ThresholdBounds* tb,
                          LeafBounds* flat);

 private:
  struct PathStep {
    int feature;
    uint32_t threshold;
    bool from_right;
  };
  struct FeatureBounds {
    BinPieces lo, hi;
    bool redo_lo = false, redo_hi = false;
  };
  void Climb(const Tree* tree, int node, std::vector<PathStep>* path, const SplitInfo& split,
             const std::vector<SplitInfo>& best, std::vector<LeafBounds>* bounds);
  void Descend(const Tree* tree, int node, const std::vector<PathStep>& path, bool tighten_max, bool use_left,
               bool use_right, const SplitInfo& split, const std::vector<SplitInfo>& best,
               std::vector<LeafBounds>* bounds);
  void Rebuild(const Tree* tree, int f, int leaf, bool lower, BinPieces* target) const;
  void Collect(const Tree* tree, int f, int root_feature, int node, bool lower, uint32_t b, uint32_t e,
               const std::vector<PathStep>& path, BinPieces* target) const;
  int8_t MonotoneOfNode(const Tree* tree, int node) const;
  static void Borders(const Tree* tree, int node, const std::vector<PathStep>& path, bool* go_left,
                      bool* go_right);
  FeatureBounds& entry(int leaf, int f) { return entries_[static_cast<size_t>(leaf) * nf_ + f]; }

  const Dataset* data_ = nullptr;
  bool advanced_ = false;
  int nf_ = 0;
  std::vector<char> in_monotone_subtree_;
  std::vector<int> node_parent_;
  std::vector<int> to_update_;
  std::vector<FeatureBounds> entries_;  // advanced: [leaf * nf + f]
};

class CegbPenalty {
 public:
  static bool Enabled(const Config* c) {
    return c->cegb_tradeoff < 1.0 || c->cegb_penalty_split > 0.0 || !c->cegb_penalty_feature_coupled.empty() ||
           !c->cegb_penalty_feature_lazy.empty();
  }
  void Init(const Dataset* data, const Config* c);
  void BeforeTree();
  // gain deduction of a candidate split on inner feature `f` of `leaf` (rows = the leaf's rows)
  // n rows of the leaf on this machine (the lazy penalty's on-demand count walks them); split_n:
  // the leaf's GLOBAL count for the split penalty (reference ComputeBestSplitForFeature passes
  // GetGlobalDataCountInLeaf in the data / voting learners), -1: n
  double DeltaGain(int f, int leaf, const data_size_t* rows, data_size_t n, const SplitInfo& candidate,
                   data_size_t split_n = -1);
  // before the chosen split of `best_leaf` is applied (rows = that leaf's rows)
  void OnSplit(int num_leaves, int best_leaf, const SplitInfo& chosen, const data_size_t* rows, data_size_t n,
               std::vector<SplitInfo>* best_per_leaf);

 private:
  const Dataset* data_ = nullptr;
  const Config* cfg_ = nullptr;
  int nf_ = 0;
  bool init_ = false;
  std::vector<SplitInfo> per_leaf_feature_;  // [leaf * nf + f], pre-penalty candidates
  std::vector<char> used_in_split_;          // inner feature already paid (coupled)
  std::vector<uint64_t> used_in_row_;        // bitset [f * num_data + row] (lazy)
};

class GradientQuantizer {
 public:
  void Init(data_size_t num_data, int num_bins, int seed, bool stochastic);
  // quantized (integer * scale) copies of g and h into qg / qh
  void Quantize(const score_t* g, const score_t* h, data_size_t n, bool constant_hessian, score_t* qg, score_t* qh);
  double grad_scale() const { return gscale_; }
  double hess_scale() const { return hscale_; }

 private:
  int bins_ = 4;
  bool stochastic_ = true;
  std::vector<float> rg_, rh_;  // per-row uniform [0,1) draws, reused with a rotating offset
  std::mt19937 offset_eng_;
  double gscale_ = 0.0, hscale_ = 0.0;
};

}  // namespace lgap
