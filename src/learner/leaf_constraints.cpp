// Intermediate monotone constraints, CEGB penalties and gradient quantization
// for the host learners. See leaf_constraints.h for the reference map.
#include "leaf_constraints.h"

#include <algorithm>
#include <cmath>

#include "lgap/log.h"
#include "lgap/network.h"

namespace lgap {

// ============================================================================
// IntermediateMonotone
//
// Bookkeeping: which leaves lie below a monotone split (only those can carry
// constraints) and the parent of every internal node. After leaf L splits into
// (L, N), the walk climbs from the new node to the root. At each ancestor P
// that splits numerically on a monotone feature, the subtree on the other side
// of P holds the leaves that must stay below (or above) the new outputs; the
// descent only enters children whose region can border the new leaves, judged
// by the numerical splits met on the way up (same feature, same side = a gap
// separates them). Leaves whose interval actually tightened are rescanned.
// ============================================================================
void IntermediateMonotone::Init(const Dataset* data, int num_leaves) {
  data_ = data;
  in_monotone_subtree_.assign(num_leaves, 0);
  node_parent_.assign(std::max(1, num_leaves - 1), -1);
  to_update_.reserve(num_leaves);
}

void IntermediateMonotone::Reset() {
  std::fill(in_monotone_subtree_.begin(), in_monotone_subtree_.end(), 0);
  std::fill(node_parent_.begin(), node_parent_.end(), -1);
  to_update_.clear();
}

int8_t IntermediateMonotone::MonotoneOfNode(const Tree* tree, int node) const {
  return data_->feature(tree->split_feature_inner(node)).monotone;
}

void IntermediateMonotone::BeforeSplit(const Tree* tree, int leaf, int new_leaf, int8_t monotone_type) {
  if (monotone_type != 0 || in_monotone_subtree_[leaf]) {
    in_monotone_subtree_[leaf] = 1;
    in_monotone_subtree_[new_leaf] = 1;
  }
  node_parent_[new_leaf - 1] = tree->leaf_parent(leaf);
}

std::vector<int> IntermediateMonotone::AfterSplit(const Tree* tree, std::vector<LeafBounds>* bounds, bool numerical,
                                                  int leaf, int new_leaf, int8_t monotone_type,
                                                  const SplitInfo& split, const std::vector<SplitInfo>& best) {
  to_update_.clear();
  if (!in_monotone_subtree_[leaf]) return {};
  auto& b = *bounds;
  b[new_leaf] = b[leaf];
  if (numerical) {
    // the siblings bound each other by their actual outputs (not the midpoint of the basic method)
    if (monotone_type < 0) {
      b[leaf].min = std::max(b[leaf].min, split.right_output);
      b[new_leaf].max = std::min(b[new_leaf].max, split.left_output);
    } else if (monotone_type > 0) {
      b[leaf].max = std::min(b[leaf].max, split.right_output);
      b[new_leaf].min = std::max(b[new_leaf].min, split.left_output);
    }
  }
  std::vector<PathStep> path;
  path.reserve(tree->leaf_depth(new_leaf));
  Climb(tree, tree->leaf_parent(new_leaf), &path, split, best, bounds);
  return to_update_;
}

void IntermediateMonotone::Climb(const Tree* tree, int node, std::vector<PathStep>* path, const SplitInfo& split,
                                 const std::vector<SplitInfo>& best, std::vector<LeafBounds>* bounds) {
  for (;;) {
    const int parent = node_parent_[node];
    if (parent < 0) return;
    const int f = tree->split_feature_inner(parent);
    const bool from_right = tree->right_child(parent) == node;
    const bool numerical = !Tree::GetDecisionType(tree->decision_type(parent), kCategoricalMask);
    bool borders = numerical;
    for (const PathStep& s : *path) {
      if (s.feature == f && s.from_right == from_right) {
        borders = false;  // an earlier same-side split on f already separates the far side
        break;
      }
    }
    if (borders) {
      const int8_t mono = MonotoneOfNode(tree, parent);
      if (mono != 0) {
        const int far = from_right ? tree->left_child(parent) : tree->right_child(parent);
        // increasing feature: leaves on the low side must not exceed the new outputs
        const bool tighten_max = mono < 0 ? !from_right : from_right;
        Descend(tree, far, *path, tighten_max, true, true, split, best, bounds);
      }
      path->push_back({f, tree->threshold_in_bin(parent), from_right});
    }
    node = parent;
  }
}

void IntermediateMonotone::Descend(const Tree* tree, int node, const std::vector<PathStep>& path, bool tighten_max,
                                   bool use_left, bool use_right, const SplitInfo& split,
                                   const std::vector<SplitInfo>& best, std::vector<LeafBounds>* bounds) {
  if (node < 0) {
    const int leaf = ~node;
    if (best[leaf].gain == kMinScore) return;  // cannot split anyway
    double lo, hi;
    if (use_left && use_right) {
      lo = std::min(split.left_output, split.right_output);
      hi = std::max(split.left_output, split.right_output);
    } else if (use_right) {
      lo = hi = split.right_output;
    } else {
      lo = hi = split.left_output;
    }
    LeafBounds& b = (*bounds)[leaf];
    bool changed = false;
    if (tighten_max) {
      if (lo < b.max) b.max = lo, changed = true;
    } else {
      if (hi > b.min) b.min = hi, changed = true;
    }
    if (changed) to_update_.push_back(leaf);
    return;
  }
  const int f = tree->split_feature_inner(node);
  const uint32_t thr = tree->threshold_in_bin(node);
  const bool numerical = !Tree::GetDecisionType(tree->decision_type(node), kCategoricalMask);
  bool go_left = true, go_right = true;
  if (numerical) {
    for (const PathStep& s : path) {
      if (s.feature != f) continue;
      if (thr >= s.threshold && !s.from_right) go_right = false;
      if (thr <= s.threshold && s.from_right) go_left = false;
    }
  }
  // a split on the new split's own feature decides which of the two new leaves each side borders
  bool left_sees_right = true, right_sees_left = true;
  if (numerical && f == split.feature) {
    if (thr <= split.threshold) left_sees_right = false;
    if (thr >= split.threshold) right_sees_left = false;
  }
  if (go_left) {
    Descend(tree, tree->left_child(node), path, tighten_max, use_left, left_sees_right && use_right, split, best,
            bounds);
  }
  if (go_right) {
    Descend(tree, tree->right_child(node), path, tighten_max, right_sees_left && use_left, use_right, split, best,
            bounds);
  }
}

// ============================================================================
// CegbPenalty
// ============================================================================
void CegbPenalty::Init(const Dataset* data, const Config* c) {
  cfg_ = c;
  const int total = data->num_total_features();
  if (!c->cegb_penalty_feature_coupled.empty() && static_cast<int>(c->cegb_penalty_feature_coupled.size()) != total) {
    Log::Fatal("cegb_penalty_feature_coupled should be the same size as feature number.");
  }
  if (!c->cegb_penalty_feature_lazy.empty() && static_cast<int>(c->cegb_penalty_feature_lazy.size()) != total) {
    Log::Fatal("cegb_penalty_feature_lazy should be the same size as feature number.");
  }
  if (init_ && data == data_) return;  // usage state persists across trees (and ResetConfig)
  data_ = data;
  nf_ = data->num_features();
  per_leaf_feature_.assign(static_cast<size_t>(c->num_leaves) * nf_, SplitInfo());
  used_in_split_.assign(nf_, 0);
  if (!c->cegb_penalty_feature_lazy.empty()) {
    used_in_row_.assign((static_cast<size_t>(nf_) * data->num_data() + 63) / 64, 0);
  }
  init_ = true;
}

void CegbPenalty::BeforeTree() {
  if (per_leaf_feature_.size() < static_cast<size_t>(cfg_->num_leaves) * nf_) {
    per_leaf_feature_.resize(static_cast<size_t>(cfg_->num_leaves) * nf_);
  }
  for (auto& s : per_leaf_feature_) s.Reset();
}

double CegbPenalty::DeltaGain(int f, int leaf, const data_size_t* rows, data_size_t n, const SplitInfo& candidate) {
  const double t = cfg_->cegb_tradeoff;
  const int real = data_->feature(f).real_index;
  double delta = t * cfg_->cegb_penalty_split * n;
  if (!cfg_->cegb_penalty_feature_coupled.empty() && !used_in_split_[f]) {
    delta += t * cfg_->cegb_penalty_feature_coupled[real];
  }
  if (!cfg_->cegb_penalty_feature_lazy.empty()) {
    const double pen = cfg_->cegb_penalty_feature_lazy[real];
    const size_t base = static_cast<size_t>(f) * data_->num_data();
    data_size_t fresh = 0;
    for (data_size_t i = 0; i < n; ++i) {
      const size_t bit = base + rows[i];
      fresh += ((used_in_row_[bit >> 6] >> (bit & 63)) & 1) ? 0 : 1;
    }
    delta += t * pen * fresh;
  }
  per_leaf_feature_[static_cast<size_t>(leaf) * nf_ + f] = candidate;
  return delta;
}

void CegbPenalty::OnSplit(int num_leaves, int best_leaf, const SplitInfo& chosen, const data_size_t* rows,
                          data_size_t n, std::vector<SplitInfo>* best_per_leaf) {
  const int f = chosen.feature;
  if (f < 0) return;
  auto& best = *best_per_leaf;
  if (!cfg_->cegb_penalty_feature_coupled.empty() && !used_in_split_[f]) {
    used_in_split_[f] = 1;
    // the feature is now paid for: other leaves' stored candidates on f are refunded
    const double refund = cfg_->cegb_tradeoff * cfg_->cegb_penalty_feature_coupled[data_->feature(f).real_index];
    for (int l = 0; l < num_leaves; ++l) {
      if (l == best_leaf) continue;
      SplitInfo& s = per_leaf_feature_[static_cast<size_t>(l) * nf_ + f];
      s.gain += refund;
      if (best[l].gain > kMinScore && s.feature >= 0 && s.BetterThan(best[l])) best[l] = s;
    }
  }
  if (!cfg_->cegb_penalty_feature_lazy.empty()) {
    const size_t base = static_cast<size_t>(f) * data_->num_data();
    for (data_size_t i = 0; i < n; ++i) {
      const size_t bit = base + rows[i];
      used_in_row_[bit >> 6] |= uint64_t(1) << (bit & 63);
    }
  }
}

// ============================================================================
// GradientQuantizer
// ============================================================================
void GradientQuantizer::Init(data_size_t num_data, int num_bins, int seed, bool stochastic) {
  bins_ = std::max(2, num_bins);
  stochastic_ = stochastic;
  rg_.resize(num_data);
  rh_.resize(num_data);
  std::mt19937 eng(static_cast<uint32_t>(seed));
  std::uniform_real_distribution<float> u(0.0f, 1.0f);
  for (data_size_t i = 0; i < num_data; ++i) rg_[i] = u(eng);
  for (data_size_t i = 0; i < num_data; ++i) rh_[i] = u(eng);
  offset_eng_.seed(static_cast<uint32_t>(seed) + 1u);
}

void GradientQuantizer::Quantize(const score_t* g, const score_t* h, data_size_t n, bool constant_hessian,
                                 score_t* qg, score_t* qh) {
  if (n <= 0) return;
  double mg = 0.0, mh = 0.0;
#pragma omp parallel for schedule(static) reduction(max : mg, mh)
  for (data_size_t i = 0; i < n; ++i) {
    mg = std::max(mg, static_cast<double>(std::fabs(g[i])));
    mh = std::max(mh, static_cast<double>(std::fabs(h[i])));
  }
  if (Network::num_machines() > 1) {
    mg = Network::GlobalSyncUpByMax(mg);
    mh = Network::GlobalSyncUpByMax(mh);
  }
  gscale_ = mg / (bins_ / 2);
  hscale_ = constant_hessian ? mh : mh / bins_;
  const double ig = gscale_ > 0 ? 1.0 / gscale_ : 0.0;
  const double ih = hscale_ > 0 ? 1.0 / hscale_ : 0.0;
  const data_size_t off =
      stochastic_ ? std::uniform_int_distribution<data_size_t>(0, n)(offset_eng_) : 0;
  const data_size_t nr = static_cast<data_size_t>(rg_.size());
#pragma omp parallel for schedule(static)
  for (data_size_t i = 0; i < n; ++i) {
    const double rg = stochastic_ ? rg_[(static_cast<int64_t>(i) + off) % nr] : 0.5;
    const double rh = stochastic_ ? rh_[(static_cast<int64_t>(i) + off) % nr] : 0.5;
    const double x = g[i] * ig;
    const int qgi = static_cast<int8_t>(g[i] >= 0 ? x + rg : x - rg);  // truncation toward zero
    qg[i] = static_cast<score_t>(qgi * gscale_);
    if (constant_hessian) {
      qh[i] = static_cast<score_t>(hscale_);
    } else {
      const int qhi = static_cast<int8_t>(h[i] * ih + rh);
      qh[i] = static_cast<score_t>(qhi * hscale_);
    }
  }
}

}  // namespace lgap
