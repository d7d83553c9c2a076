// Intermediate monotone constraints, CEGB penalties and gradient quantization
// for the host learners. See leaf_constraints.h for the reference map.
#include "leaf_constraints.h"

#include <algorithm>
#include <cmath>

#include "lgap/log.h"
#include "lgap/network.h"

namespace lgap {

// ============================================================================
// MonotoneLeafConstraints
//
// Bookkeeping: which leaves lie below a monotone split (only those can carry
// constraints) and the parent of every internal node. After leaf L splits into
// (L, N), the walk climbs from the new node to the root. At each ancestor P
// that splits numerically on a monotone feature, the subtree on the other side
// of P holds the leaves that must stay below (or above) the new outputs; the
// descent only enters children whose region can border the new leaves, judged
// by the numerical splits met on the way up (same feature, same side = a gap
// separates them). Leaves whose interval actually tightened are rescanned.
//
// Advanced: each (leaf, feature) also holds a lower and an upper BinPieces. The
// updates above tighten every feature's pieces and mark them stale; before the
// leaf's next scan of a numerical feature f a stale bound is rebuilt from
// scratch by the same climb, descending into the far side of every monotone
// ancestor and tightening only the bin range of f that each bordering leaf
// actually shares with L (reference monotone_constraints.hpp:935-1175).
// ============================================================================
void BinPieces::TightenAll(double v, bool raise) {
  for (double& x : val) x = raise ? std::max(x, v) : std::min(x, v);
  Fuse();
}

void BinPieces::Fuse() {
  size_t w = 0;
  for (size_t i = 1; i < start.size(); ++i) {
    if (val[i] == val[w]) continue;
    ++w;
    start[w] = start[i];
    val[w] = val[i];
  }
  start.resize(w + 1);
  val.resize(w + 1);
}

void BinPieces::TightenRange(double v, bool raise, uint32_t b, uint32_t e, uint32_t num_bin) {
  e = std::min(e, num_bin);
  if (b >= e) return;
  // cut the pieces at b and e, tighten those inside, then fuse equal neighbours
  auto cut = [&](uint32_t x) {
    if (x >= num_bin) return;
    const size_t k = static_cast<size_t>(std::upper_bound(start.begin(), start.end(), x) - start.begin()) - 1;
    if (start[k] == x) return;
    start.insert(start.begin() + k + 1, x);
    val.insert(val.begin() + k + 1, val[k]);
  };
  cut(b);
  cut(e);
  for (size_t i = 0; i < start.size(); ++i) {
    if (start[i] >= b && start[i] < e) val[i] = raise ? std::max(val[i], v) : std::min(val[i], v);
  }
  Fuse();
}

void BinPieces::Expand(int num_bin, double* out) const {
  for (size_t i = 0; i < start.size(); ++i) {
    const int e = i + 1 < start.size() ? std::min<int>(num_bin, static_cast<int>(start[i + 1])) : num_bin;
    for (int t = static_cast<int>(start[i]); t < e; ++t) out[t] = val[i];
  }
}

void MonotoneLeafConstraints::Init(const Dataset* data, int num_leaves, bool advanced) {
  data_ = data;
  advanced_ = advanced;
  nf_ = data->num_features();
  in_monotone_subtree_.assign(num_leaves, 0);
  node_parent_.assign(std::max(1, num_leaves - 1), -1);
  to_update_.reserve(num_leaves);
  entries_.assign(advanced ? static_cast<size_t>(num_leaves) * nf_ : 0, FeatureBounds());
  Reset();
}

void MonotoneLeafConstraints::Reset() {
  std::fill(in_monotone_subtree_.begin(), in_monotone_subtree_.end(), 0);
  std::fill(node_parent_.begin(), node_parent_.end(), -1);
  to_update_.clear();
  for (FeatureBounds& e : entries_) {
    e.lo.Reset(-INFINITY);
    e.hi.Reset(INFINITY);
    e.redo_lo = e.redo_hi = false;
  }
}

int8_t MonotoneLeafConstraints::MonotoneOfNode(const Tree* tree, int node) const {
  return data_->feature(tree->split_feature_inner(node)).monotone;
}

void MonotoneLeafConstraints::BeforeSplit(const Tree* tree, int leaf, int new_leaf, int8_t monotone_type) {
  if (monotone_type != 0 || in_monotone_subtree_[leaf]) {
    in_monotone_subtree_[leaf] = 1;
    in_monotone_subtree_[new_leaf] = 1;
  }
  node_parent_[new_leaf - 1] = tree->leaf_parent(leaf);
}

std::vector<int> MonotoneLeafConstraints::AfterSplit(const Tree* tree, std::vector<LeafBounds>* bounds,
                                                     bool numerical, int leaf, int new_leaf, int8_t monotone_type,
                                                     const SplitInfo& split, const std::vector<SplitInfo>& best) {
  to_update_.clear();
  if (!in_monotone_subtree_[leaf]) return {};
  auto& b = *bounds;
  b[new_leaf] = b[leaf];
  if (advanced_) std::copy_n(&entry(leaf, 0), nf_, &entry(new_leaf, 0));
  if (numerical && monotone_type != 0) {
    // the siblings bound each other by their actual outputs (not the midpoint of the basic method)
    const bool dec = monotone_type < 0;
    if (dec) {
      b[leaf].min = std::max(b[leaf].min, split.right_output);
      b[new_leaf].max = std::min(b[new_leaf].max, split.left_output);
    } else {
      b[leaf].max = std::min(b[leaf].max, split.right_output);
      b[new_leaf].min = std::max(b[new_leaf].min, split.left_output);
    }
    for (int f = 0; advanced_ && f < nf_; ++f) {
      (dec ? entry(leaf, f).lo : entry(leaf, f).hi).TightenAll(split.right_output, dec);
      (dec ? entry(new_leaf, f).hi : entry(new_leaf, f).lo).TightenAll(split.left_output, !dec);
    }
  }
  std::vector<PathStep> path;
  path.reserve(tree->leaf_depth(new_leaf));
  Climb(tree, tree->leaf_parent(new_leaf), &path, split, best, bounds);
  return to_update_;
}

void MonotoneLeafConstraints::Climb(const Tree* tree, int node, std::vector<PathStep>* path, const SplitInfo& split,
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

// which children of `node` can border the original leaf, given the numerical
// splits met on the way up
void MonotoneLeafConstraints::Borders(const Tree* tree, int node, const std::vector<PathStep>& path, bool* go_left,
                                      bool* go_right) {
  *go_left = *go_right = true;
  if (Tree::GetDecisionType(tree->decision_type(node), kCategoricalMask)) return;
  const int f = tree->split_feature_inner(node);
  const uint32_t thr = tree->threshold_in_bin(node);
  for (const PathStep& s : path) {
    if (s.feature != f) continue;
    if (thr >= s.threshold && !s.from_right) *go_right = false;
    if (thr <= s.threshold && s.from_right) *go_left = false;
  }
}

void MonotoneLeafConstraints::Descend(const Tree* tree, int node, const std::vector<PathStep>& path,
                                      bool tighten_max, bool use_left, bool use_right, const SplitInfo& split,
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
    if (advanced_) {
      // every feature's pieces tighten and go stale: the exact per-bin bounds are
      // rebuilt at the next scan, so the leaf is always rescanned
      for (int f = 0; f < nf_; ++f) {
        FeatureBounds& e = entry(leaf, f);
        if (tighten_max) {
          e.hi.TightenAll(lo, false);
          e.redo_hi = true;
        } else {
          e.lo.TightenAll(hi, true);
          e.redo_lo = true;
        }
      }
      changed = true;
    }
    if (changed) to_update_.push_back(leaf);
    return;
  }
  const int f = tree->split_feature_inner(node);
  const uint32_t thr = tree->threshold_in_bin(node);
  const bool numerical = !Tree::GetDecisionType(tree->decision_type(node), kCategoricalMask);
  bool go_left, go_right;
  Borders(tree, node, path, &go_left, &go_right);
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

bool MonotoneLeafConstraints::ThresholdBoundsFor(const Tree* tree, int f, int leaf, std::vector<double>* scratch,
                                                 ThresholdBounds* tb, LeafBounds* flat) {
  FeatureBounds& e = entry(leaf, f);
  if (e.redo_lo || e.redo_hi) {
    // one bound is rebuilt per scan, the lower first (the other keeps its tightened pieces)
    const bool lower = e.redo_lo;
    Rebuild(tree, f, leaf, lower, lower ? &e.lo : &e.hi);
    e.redo_lo = e.redo_hi = false;
  }
  if (e.lo.size() == 1 && e.hi.size() == 1) {
    flat->min = e.lo.val[0];
    flat->max = e.hi.val[0];
    return false;
  }
  const int nb = data_->feature(f).num_bin;
  scratch->resize(6 * static_cast<size_t>(nb));
  double* lo = scratch->data();
  double* hi = lo + nb;
  double* lmin = hi + nb;
  double* lmax = lmin + nb;
  double* rmin = lmax + nb;
  double* rmax = rmin + nb;
  e.lo.Expand(nb, lo);
  e.hi.Expand(nb, hi);
  // lmin/lmax[t]: over bins < t; rmin/rmax[t]: over bins >= t
  lmin[0] = -INFINITY;
  lmax[0] = INFINITY;
  for (int t = 1; t < nb; ++t) {
    lmin[t] = std::max(lmin[t - 1], lo[t - 1]);
    lmax[t] = std::min(lmax[t - 1], hi[t - 1]);
  }
  rmin[nb - 1] = lo[nb - 1];
  rmax[nb - 1] = hi[nb - 1];
  for (int t = nb - 2; t >= 0; --t) {
    rmin[t] = std::max(rmin[t + 1], lo[t]);
    rmax[t] = std::min(rmax[t + 1], hi[t]);
  }
  tb->lmin = lmin;
  tb->lmax = lmax;
  tb->rmin = rmin;
  tb->rmax = rmax;
  return true;
}

// Climb from `leaf` to the root; below every monotone ancestor whose far side can
// border the leaf (and constrains it in the `lower` direction), collect the far
// leaves' outputs into the bin ranges of f they share with the leaf. The leaf's
// own range of f narrows on the way up (right child: from the threshold, as the
// reference does; left child: up to threshold + 1).
void MonotoneLeafConstraints::Rebuild(const Tree* tree, int f, int leaf, bool lower, BinPieces* target) const {
  const uint32_t nb = static_cast<uint32_t>(data_->feature(f).num_bin);
  target->Reset(lower ? -INFINITY : INFINITY);
  std::vector<PathStep> path;
  uint32_t b = 0, e = nb;
  int node = ~leaf;
  for (;;) {
    const int parent = node < 0 ? tree->leaf_parent(~node) : node_parent_[node];
    if (parent < 0) return;
    const int pf = tree->split_feature_inner(parent);
    const bool from_right = tree->right_child(parent) == node;
    const bool numerical = !Tree::GetDecisionType(tree->decision_type(parent), kCategoricalMask);
    const uint32_t thr = tree->threshold_in_bin(parent);
    if (pf == f && numerical) {
      if (from_right) b = std::max(thr, b);
      else e = std::min(thr + 1, e);
    }
    bool borders = numerical;
    for (const PathStep& s : path) {
      if (s.feature == pf && s.from_right == from_right) {
        borders = false;
        break;
      }
    }
    if (borders) {
      const int8_t mono = MonotoneOfNode(tree, parent);
      // increasing: the high side is bounded below by the low side's outputs
      if (mono != 0 && (mono < 0 ? !from_right : from_right) == lower) {
        const int far = from_right ? tree->left_child(parent) : tree->right_child(parent);
        Collect(tree, f, pf, far, lower, b, e, path, target);
      }
      path.push_back({pf, thr, from_right});
    }
    if (parent == 0) return;
    node = parent;
  }
}

void MonotoneLeafConstraints::Collect(const Tree* tree, int f, int root_feature, int node, bool lower, uint32_t b,
                                      uint32_t e, const std::vector<PathStep>& path, BinPieces* target) const {
  if (node < 0) {
    target->TightenRange(tree->LeafOutput(~node), lower, b, e,
                         static_cast<uint32_t>(data_->feature(f).num_bin));
    return;
  }
  bool go_left, go_right;
  Borders(tree, node, path, &go_left, &go_right);
  const int nf = tree->split_feature_inner(node);
  const uint32_t thr = tree->threshold_in_bin(node);
  const bool same = nf == f;
  // below a monotone split only the side with the extreme outputs matters, unless
  // the split cuts f itself inside the leaf's range (then both sides touch it)
  bool need_left = true, need_right = true;
  if (!(same && root_feature != f)) {
    const int8_t mono = MonotoneOfNode(tree, node);
    if (mono != 0) {
      const bool left_side = (mono < 0) == lower;  // decreasing + lower bound: the left (higher) side
      need_left = left_side;
      need_right = !left_side;
    }
  }
  if (go_left && (need_left || !go_right)) {
    Collect(tree, f, root_feature, tree->left_child(node), lower, b, same ? std::min(thr + 1, e) : e, path, target);
  }
  if (go_right && (need_right || !go_left)) {
    Collect(tree, f, root_feature, tree->right_child(node), lower, same ? std::max(thr + 1, b) : b, e, path, target);
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

double CegbPenalty::DeltaGain(int f, int leaf, const data_size_t* rows, data_size_t n, const SplitInfo& candidate,
                              data_size_t split_n) {
  const double t = cfg_->cegb_tradeoff;
  const int real = data_->feature(f).real_index;
  double delta = t * cfg_->cegb_penalty_split * (split_n >= 0 ? split_n : n);
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
