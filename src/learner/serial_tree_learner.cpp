// Host leaf-wise learner (correctness oracle). Behaviour mirrors the
// reference's SerialTreeLearner (serial_tree_learner.cpp:179-1114):
// smaller-child histogram + parent-minus-sibling subtraction, per-feature
// splittable inheritance, basic monotone constraints, extra-trees thresholds,
// feature sampling by tree / node, interaction constraints, forced splits,
// refit and L1/quantile leaf renewal.
#include "serial_tree_learner.h"
#include "forced_splits.h"
#include "lgap/omp_errors.h"

#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fstream>
#include <numeric>
#include <queue>
#include <unordered_set>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/network.h"

namespace lgap {

// ============================================================================
// ColSampler (col_sampler.hpp:20-207)
int ColSampler::GetCnt(size_t total, double fraction) {
  const int mn = std::min(1, static_cast<int>(total));
  const int c = common::RoundInt(total * fraction);
  return std::max(c, mn);
}

void ColSampler::Init(const Dataset* data, const Config* cfg) {
  data_ = data;
  frac_tree_ = cfg->feature_fraction;
  frac_node_ = cfg->feature_fraction_bynode;
  if (seed_ != cfg->feature_fraction_seed) {
    seed_ = cfg->feature_fraction_seed;
    rand_ = Random(seed_);
  }
  valid_.clear();
  for (int f = 0; f < data->num_features(); ++f) valid_.push_back(data->feature(f).real_index);
  used_bytree_.assign(data->num_features(), 1);
  if (frac_tree_ >= 1.0) {
    need_reset_tree_ = false;
    used_cnt_tree_ = static_cast<int>(valid_.size());
  } else {
    need_reset_tree_ = true;
    used_cnt_tree_ = GetCnt(valid_.size(), frac_tree_);
  }
  interaction_.clear();
  for (auto& c : cfg->interaction_constraints_vector) interaction_.emplace_back(c.begin(), c.end());
  ResetByTree();
}

void ColSampler::ResetByTree() {
  if (!need_reset_tree_) return;
  std::fill(used_bytree_.begin(), used_bytree_.end(), 0);
  used_idx_ = rand_.Sample(static_cast<int>(valid_.size()), used_cnt_tree_);
  for (int i : used_idx_) used_bytree_[data_->InnerIndex(valid_[i])] = 1;
}

std::vector<int8_t> ColSampler::GetByNode(const Tree* tree, int leaf) {
  std::unordered_set<int> allowed;
  if (!interaction_.empty()) {
    const auto& bf = tree->branch_features(leaf);
    allowed.insert(bf.begin(), bf.end());
    for (auto& c : interaction_) {
      if (bf.empty()) allowed.insert(c.begin(), c.end());
      int found = 0;
      for (int f : bf) {
        if (c.count(f) == 0) break;
        if (++found == static_cast<int>(bf.size())) {
          allowed.insert(c.begin(), c.end());
          break;
        }
      }
    }
  }
  const int nf = data_->num_features();
  std::vector<int8_t> ret(nf, 0);
  if (frac_node_ >= 1.0) {
    if (interaction_.empty()) return std::vector<int8_t>(nf, 1);
    for (int f : allowed) {
      if (f < data_->num_total_features()) {
        int in = data_->InnerIndex(f);
        if (in >= 0) ret[in] = 1;
      }
    }
    return ret;
  }
  std::vector<int> pool;
  if (need_reset_tree_) {
    for (int i : used_idx_) if (interaction_.empty() || allowed.count(valid_[i])) pool.push_back(i);
  } else {
    for (int i = 0; i < static_cast<int>(valid_.size()); ++i)
      if (interaction_.empty() || allowed.count(valid_[i])) pool.push_back(i);
  }
  int cnt = GetCnt(need_reset_tree_ ? used_idx_.size() : valid_.size(), frac_node_);
  cnt = std::min(cnt, static_cast<int>(pool.size()));
  auto s = rand_.Sample(static_cast<int>(pool.size()), cnt);
  for (int i : s) ret[data_->InnerIndex(valid_[pool[i]])] = 1;
  return ret;
}

std::vector<uint8_t> ColSampler::ByNodeSampleModes(int* cnt, bool* filter_bytree) const {
  *filter_bytree = need_reset_tree_;
  *cnt = GetCnt(need_reset_tree_ ? static_cast<size_t>(used_cnt_tree_) : valid_.size(), frac_node_);
  const int nf = data_->num_features();
  std::vector<uint8_t> m(nf + 1);
  for (int n = 0; n <= nf; ++n) {
    const int k = std::min(*cnt, n);  // (GetByNode: min(cnt, pool size))
    m[n] = static_cast<uint8_t>(k > n || k <= 0 ? 0 : (k == n ? 1 : (k > 1 && k > (n / std::log2(k)) ? 2 : 3)));
  }
  return m;
}

// ============================================================================
// DataPartition
void DataPartition::Init(data_size_t num_data, int num_leaves) {
  num_data_ = num_data;
  indices_.resize(num_data);
  tmp_.resize(num_data);
  begin_.assign(num_leaves, 0);
  count_.assign(num_leaves, 0);
}

void DataPartition::SetUsedIndices(const data_size_t* idx, data_size_t n) {
  if (idx == nullptr) {
    use_bag_ = false;
    used_.clear();
  } else {
    use_bag_ = true;
    used_.assign(idx, idx + n);
  }
  bag_cnt_ = n;
}

void DataPartition::Reset() {
  std::fill(begin_.begin(), begin_.end(), 0);
  std::fill(count_.begin(), count_.end(), 0);
  if (use_bag_) {
    std::copy(used_.begin(), used_.end(), indices_.begin());
    count_[0] = static_cast<data_size_t>(used_.size());
  } else {
    std::iota(indices_.begin(), indices_.end(), 0);
    count_[0] = num_data_;
  }
}

void DataPartition::ResetByLeafPred(const std::vector<int>& leaf_pred, int num_leaves) {
  std::vector<std::vector<data_size_t>> lists(num_leaves);
  for (data_size_t i = 0; i < static_cast<data_size_t>(leaf_pred.size()); ++i) lists[leaf_pred[i]].push_back(i);
  begin_.assign(std::max<size_t>(begin_.size(), num_leaves), 0);
  count_.assign(begin_.size(), 0);
  data_size_t off = 0;
  for (int l = 0; l < num_leaves; ++l) {
    begin_[l] = off;
    count_[l] = static_cast<data_size_t>(lists[l].size());
    std::copy(lists[l].begin(), lists[l].end(), indices_.begin() + off);
    off += count_[l];
  }
}

// ============================================================================
SerialTreeLearner::SerialTreeLearner(const Config* config) : config_(config) {}

void SerialTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  train_data_ = train_data;
  num_data_ = train_data->num_data();
  num_features_ = train_data->num_features();
  is_constant_hessian_ = is_constant_hessian;
  partition_.Init(num_data_, config_->num_leaves);
  col_sampler_.Init(train_data, config_);
  best_split_per_leaf_.assign(config_->num_leaves, SplitInfo());
  ResetHistPool();
  splittable_.assign(config_->num_leaves, std::vector<char>(num_features_, 1));
  bounds_.assign(config_->num_leaves, LeafBounds());
  leaf_count_global_.assign(config_->num_leaves, 0);
  use_monotone_ = !config_->monotone_constraints.empty();
  SetupPolicies();
  extra_rand_ = Random(config_->extra_seed);
  feature_mask_.assign(num_features_, 1);
  hist_begin_ = 0;
  hist_end_ = train_data->num_total_bin();
  if (!config_->forcedsplits_filename.empty()) {
    std::ifstream in(config_->forcedsplits_filename);
    if (in) forced_json_.assign((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    else Log::Warning("Forced splits file %s cannot be opened", config_->forcedsplits_filename.c_str());
    CheckForcedSplitFeatures();
  }
  if (want_device_hist_) hist_backend_ = device::CreateHistogramBackend(config_, train_data);
  SetupResident();
  Log::Info("Number of data points in the train set: %d, number of used features: %d", num_data_, num_features_);
}

void SerialTreeLearner::ResetConfig(const Config* config) {
  config_ = config;
  if (static_cast<int>(best_split_per_leaf_.size()) != config->num_leaves) {
    partition_.Init(num_data_, config->num_leaves);
    best_split_per_leaf_.assign(config->num_leaves, SplitInfo());
    splittable_.assign(config->num_leaves, std::vector<char>(num_features_, 1));
    bounds_.assign(config->num_leaves, LeafBounds());
    leaf_count_global_.assign(config->num_leaves, 0);
  }
  if (train_data_ != nullptr) ResetHistPool();
  if (train_data_ != nullptr) SetupResident();
  col_sampler_.Init(train_data_, config_);
  use_monotone_ = !config_->monotone_constraints.empty();
  SetupPolicies();
}

// Device-resident leaf histograms (EnableDeviceScans): one device slot per leaf, no LRU pool (the
// factory only asks for it when num_leaves slots fit the device's histogram budget). Re-checked on
// every ResetConfig: a reset that turns on extra_trees (random thresholds drawn from the host
// histogram) or forced splits, leaves the intermediate / advanced method, or sets a
// histogram_pool_size the slots exceed hands the scans back to the host.
void SerialTreeLearner::SetupResident() {
  const double slot_mb = 16.0 * std::max(1, train_data_->num_total_bin()) * std::max(2, config_->num_leaves) / (1024.0 * 1024.0);
  const bool serve = want_device_scans_ && !config_->extra_trees && config_->forcedsplits_filename.empty() &&
                     !config_->monotone_constraints.empty() && config_->monotone_constraints_method != "basic" &&
                     (config_->histogram_pool_size <= 0 || slot_mb <= config_->histogram_pool_size);
  resident_ = hist_backend_ && serve && hist_backend_->EnableResidentSlots(config_->num_leaves);
  if (!resident_) return;
  dslot_.resize(config_->num_leaves);
  dvalid_.assign(config_->num_leaves, 0);
}

void SerialTreeLearner::SetupPolicies() {
  intermediate_monotone_ = use_monotone_ && config_->monotone_constraints_method != "basic";
  if (intermediate_monotone_) {
    mono_.Init(train_data_, config_->num_leaves, config_->monotone_constraints_method == "advanced");
  }
  if (CegbPenalty::Enabled(config_)) {
    if (!cegb_) cegb_ = std::make_unique<CegbPenalty>();
    cegb_->Init(train_data_, config_);
  } else {
    cegb_.reset();
  }
  if (config_->use_quantized_grad) {
    quantizer_.Init(num_data_, config_->num_grad_quant_bins, config_->seed, config_->stochastic_rounding);
    qgrad_.resize(num_data_);
    qhess_.resize(num_data_);
  }
}

void SerialTreeLearner::SetBaggingData(const data_size_t* used_indices, data_size_t num_data) {
  partition_.SetUsedIndices(used_indices, num_data);
}

SplitParams SerialTreeLearner::MakeParams() const {
  SplitParams p;
  p.lambda_l1 = config_->lambda_l1;
  p.lambda_l2 = config_->lambda_l2;
  p.max_delta_step = config_->max_delta_step;
  p.path_smooth = config_->path_smooth;
  p.min_gain_to_split = config_->min_gain_to_split;
  p.min_sum_hessian_in_leaf = config_->min_sum_hessian_in_leaf;
  p.cat_smooth = config_->cat_smooth;
  p.cat_l2 = config_->cat_l2;
  p.min_data_in_leaf = config_->min_data_in_leaf;
  p.max_cat_threshold = config_->max_cat_threshold;
  p.max_cat_to_onehot = config_->max_cat_to_onehot;
  p.min_data_per_group = config_->min_data_per_group;
  p.extra_trees = config_->extra_trees ? 1 : 0;
  p.use_monotone = use_monotone_ ? 1 : 0;
  return p;
}

void SerialTreeLearner::ResetHistPool() {
  const int L = config_->num_leaves;
  int cap = L;
  const double pool_mb = config_->histogram_pool_size > 0 ? config_->histogram_pool_size : pool_budget_mb_;
  if (pool_mb > 0) {
    const double per_leaf = 16.0 * train_data_->num_total_bin();  // (grad, hess) doubles per bin
    cap = static_cast<int>(pool_mb * 1024 * 1024 / per_leaf);
  }
  hist_cap_ = std::min(std::max(2, cap), L);
  Log::Debug("Histogram pool: %d of %d leaves", hist_cap_, L);
  hist_.assign(L, {});
  hist_stamp_.assign(L, 0);
  hist_live_ = 0;
}

std::vector<double>& SerialTreeLearner::HistOf(int leaf) {
  auto& h = hist_[leaf];
  const size_t want = static_cast<size_t>(2 * train_data_->num_total_bin());
  if (h.size() == want) return h;
  if (hist_live_ >= hist_cap_) {
    // drop the oldest histogram not in use by the two current leaves
    int victim = -1;
    for (int l = 0; l < static_cast<int>(hist_.size()); ++l) {
      if (l == leaf || l == smaller_.leaf || l == larger_.leaf || hist_[l].size() != want) continue;
      if (victim < 0 || hist_stamp_[l] < hist_stamp_[victim]) victim = l;
    }
    if (victim >= 0) {
      std::vector<double>().swap(hist_[victim]);
      --hist_live_;
    }
  }
  h.assign(want, 0.0);
  ++hist_live_;
  hist_stamp_[leaf] = ++hist_clock_;
  return h;
}

void SerialTreeLearner::ComputeLeafSums(const data_size_t* idx, data_size_t n, double* sg, double* sh) const {
  double g = 0.0, h = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : g, h) if (n >= 4096)
  for (data_size_t i = 0; i < n; ++i) {
    g += gradients_[idx[i]];
    h += hessians_[idx[i]];
  }
  *sg = g;
  *sh = h;
}

// Row-wise histogram over the packed group bins; group bin 0 (all features at
// their most-frequent bin) is never accumulated.
namespace {
template <typename BinT>
void HistRows(const data_size_t* idx, data_size_t i0, data_size_t i1, const uint8_t* bins, int stride, int ng,
              const int* gstart, const uint64_t* sp_ptr, const uint32_t* sp_bin, const score_t* grad,
              const score_t* hess, double* hh) {
  // rows of a deep leaf are scattered: prefetch the bin row and the gradients kPf rows
  // ahead so the misses overlap (reference dense_bin.hpp ConstructHistogram prefetch)
  constexpr data_size_t kPf = 32;
  for (data_size_t i = i0; i < i1; ++i) {
    if (i + kPf < i1) {
      const data_size_t rp = idx[i + kPf];
      __builtin_prefetch(bins + static_cast<size_t>(rp) * stride);
      __builtin_prefetch(grad + rp);
      __builtin_prefetch(hess + rp);
      if (sp_ptr) __builtin_prefetch(sp_ptr + rp);
    }
    const data_size_t r = idx[i];
    const double g = grad[r], h = hess[r];
    const BinT* row = reinterpret_cast<const BinT*>(bins + static_cast<size_t>(r) * stride);
    for (int k = 0; k < ng; ++k) {
      const uint32_t bv = row[k];
      if (bv == 0) continue;
      double* e = hh + 2 * (gstart[k] + static_cast<int>(bv));
      e[0] += g;
      e[1] += h;
    }
    if (sp_ptr) {
      // multi-value sparse groups: only the row's non-zero entries (global bins)
      for (uint64_t k = sp_ptr[r], ke = sp_ptr[r + 1]; k < ke; ++k) {
        double* e = hh + 2 * static_cast<size_t>(sp_bin[k]);
        e[0] += g;
        e[1] += h;
      }
    }
  }
}
}  // namespace

void SerialTreeLearner::BuildHistogram(const data_size_t* idx, data_size_t n, double* hist) const {
  if (hist_backend_) {
    hist_backend_->Histogram(idx, n, hist);
    return;
  }
  if (hist_layout_ == HistLayout::kAuto) {
    if (config_->force_col_wise && config_->force_row_wise) {
      Log::Fatal("Cannot set both `force_col_wise` and `force_row_wise` to `true` at the same time");
    }
    if (config_->force_col_wise) {
      hist_layout_ = HistLayout::kColWise;
    } else if (config_->force_row_wise || train_data_->num_dense_groups() <= 1 || omp_get_max_threads() == 1) {
      hist_layout_ = HistLayout::kRowWise;
    } else {
      // time both on this (root-sized) histogram; the results are identical, keep the faster
      std::vector<double> probe(2 * static_cast<size_t>(train_data_->num_total_bin()));
      const auto t0 = std::chrono::steady_clock::now();
      BuildHistogramRowWise(idx, n, hist);
      const auto t1 = std::chrono::steady_clock::now();
      BuildHistogramColWise(idx, n, probe.data());
      const auto t2 = std::chrono::steady_clock::now();
      const double row_s = std::chrono::duration<double>(t1 - t0).count();
      const double col_s = std::chrono::duration<double>(t2 - t1).count();
      const bool col = col_s < row_s;
      hist_layout_ = col ? HistLayout::kColWise : HistLayout::kRowWise;
      if (!col) std::vector<uint8_t>().swap(colbins_);
      Log::Info("Auto-choosing %s-wise multi-threading, the overhead of testing was %f seconds.\n"
                "You can set `force_%s_wise=true` to remove the overhead.",
                col ? "col" : "row", std::min(row_s, col_s) + (col ? row_s : col_s), col ? "col" : "row");
      if (col) std::memcpy(hist, probe.data(), probe.size() * sizeof(double));
      return;
    }
  }
  if (hist_layout_ == HistLayout::kColWise) BuildHistogramColWise(idx, n, hist);
  else BuildHistogramRowWise(idx, n, hist);
}

namespace {
// rows per histogram thread chunk: shared by both layouts so their sums associate alike
inline int HistChunks(data_size_t n) {
  return static_cast<int>(std::max<data_size_t>(1, std::min<data_size_t>(omp_get_max_threads(), n / 8192)));
}

template <typename BinT>
void HistColumn(const BinT* col, const data_size_t* idx, data_size_t i0, data_size_t i1, const score_t* grad,
                const score_t* hess, double* buf) {
  for (data_size_t i = i0; i < i1; ++i) {
    const data_size_t r = idx[i];
    const uint32_t b = col[r];
    if (b == 0) continue;
    buf[2 * b] += grad[r];
    buf[2 * b + 1] += hess[r];
  }
}
}  // namespace

void SerialTreeLearner::BuildHistogramColWise(const data_size_t* idx, data_size_t n, double* hist) const {
  const Dataset* d = train_data_;
  const int tb = d->num_total_bin();
  const int nd = d->num_dense_groups();
  const int width = d->bin_width();
  const size_t N = static_cast<size_t>(d->num_data());
  if (colbins_.size() != N * nd * width) {
    colbins_.resize(N * nd * width);
#pragma omp parallel for schedule(static)
    for (int g = 0; g < nd; ++g) {
      uint8_t* c = colbins_.data() + static_cast<size_t>(g) * N * width;
      for (size_t i = 0; i < N; ++i) {
        const uint32_t v = d->GroupBin(static_cast<data_size_t>(i), g);
        if (width == 1) c[i] = static_cast<uint8_t>(v);
        else reinterpret_cast<uint16_t*>(c)[i] = static_cast<uint16_t>(v);
      }
    }
  }
  std::memset(hist, 0, sizeof(double) * 2 * tb);
  const int nt = HistChunks(n);
  const data_size_t per = (n + nt - 1) / nt;
  // dense groups: one thread per group, chunk partials folded in chunk order
  OmpErrors errs;
#pragma omp parallel for schedule(dynamic, 1)
  for (int g = 0; g < nd; ++g) {
    errs.Run([&] {
      const FeatureGroup& fg = d->group(g);
      std::vector<double> buf(2 * static_cast<size_t>(fg.num_bin));
      double* out = hist + 2 * static_cast<size_t>(fg.hist_start);
      const uint8_t* c = colbins_.data() + static_cast<size_t>(g) * N * width;
      for (int t = 0; t < nt; ++t) {
        const data_size_t i0 = std::min(n, t * per), i1 = std::min(n, i0 + per);
        std::fill(buf.begin(), buf.end(), 0.0);
        if (width == 1) HistColumn<uint8_t>(c, idx, i0, i1, gradients_, hessians_, buf.data());
        else HistColumn<uint16_t>(reinterpret_cast<const uint16_t*>(c), idx, i0, i1, gradients_, hessians_, buf.data());
        for (int b = 2; b < 2 * fg.num_bin; ++b) out[b] += buf[b];
      }
    });
  }
  errs.Rethrow();
  if (!d->has_sparse()) return;
  // multi-value sparse groups: row chunks over the CSR into the sparse bin range
  const int s0 = d->group(nd).hist_start;
  const size_t sw = 2 * static_cast<size_t>(tb - s0);
  if (static_cast<int>(tls_hist_.size()) < nt) tls_hist_.resize(nt);
  const uint64_t* sp_ptr = d->sp_ptr();
  const uint32_t* sp_bin = d->sp_bins();
#pragma omp parallel for schedule(static, 1) num_threads(nt)
  for (int t = 0; t < nt; ++t) {
    auto& buf = tls_hist_[t];
    buf.assign(sw, 0.0);
    const data_size_t i0 = std::min(n, t * per), i1 = std::min(n, i0 + per);
    for (data_size_t i = i0; i < i1; ++i) {
      const data_size_t r = idx[i];
      const double gr = gradients_[r], hs = hessians_[r];
      for (uint64_t k = sp_ptr[r], ke = sp_ptr[r + 1]; k < ke; ++k) {
        double* e = buf.data() + 2 * (static_cast<size_t>(sp_bin[k]) - s0);
        e[0] += gr;
        e[1] += hs;
      }
    }
  }
  double* out = hist + 2 * static_cast<size_t>(s0);
  for (int t = 0; t < nt; ++t) {
    const double* b = tls_hist_[t].data();
    for (size_t j = 0; j < sw; ++j) out[j] += b[j];
  }
}

void SerialTreeLearner::BuildHistogramRowWise(const data_size_t* idx, data_size_t n, double* hist) const {
  const int tb = train_data_->num_total_bin();
  const int ng = train_data_->num_dense_groups();
  const auto& groups = train_data_->groups();
  std::vector<int> gstart(ng);
  for (int g = 0; g < ng; ++g) gstart[g] = groups[g].hist_start;
  const uint64_t* sp_ptr = train_data_->has_sparse() ? train_data_->sp_ptr() : nullptr;
  const uint32_t* sp_bin = train_data_->sp_bins();
  std::memset(hist, 0, sizeof(double) * 2 * tb);
  // one private histogram per thread above ~8k rows each (kept across calls), folded after
  const int nt = HistChunks(n);
  const uint8_t* bins = train_data_->dense_bins();
  const int stride = train_data_->dense_stride();
  const bool w1 = train_data_->bin_width() == 1;
  auto run = [&](data_size_t i0, data_size_t i1, double* hh) {
    if (w1) HistRows<uint8_t>(idx, i0, i1, bins, stride, ng, gstart.data(), sp_ptr, sp_bin, gradients_, hessians_, hh);
    else HistRows<uint16_t>(idx, i0, i1, bins, stride, ng, gstart.data(), sp_ptr, sp_bin, gradients_, hessians_, hh);
  };
  if (nt == 1) {
    run(0, n, hist);
    return;
  }
  if (static_cast<int>(tls_hist_.size()) < nt) tls_hist_.resize(nt);
  const data_size_t per = (n + nt - 1) / nt;
#pragma omp parallel for schedule(static, 1) num_threads(nt)
  for (int t = 0; t < nt; ++t) {
    auto& buf = tls_hist_[t];
    buf.assign(2 * static_cast<size_t>(tb), 0.0);
    const data_size_t i0 = std::min(n, t * per);
    run(i0, std::min(n, i0 + per), buf.data());
  }
#pragma omp parallel for schedule(static) num_threads(nt) if (2 * tb >= 16384)
  for (int j = 0; j < 2 * tb; ++j) {
    double s = 0.0;
    for (int t = 0; t < nt; ++t) s += tls_hist_[t][j];
    hist[j] = s;
  }
}

void SerialTreeLearner::InitLeafStat(LeafStat* ls, int leaf, double sg, double sh, double output) {
  ls->leaf = leaf;
  ls->sum_g = sg;
  ls->sum_h = sh;
  ls->output = output;
  ls->count = leaf >= 0 ? partition_.count(leaf) : 0;
  ls->global_count = ls->count;
  if (leaf >= 0) leaf_count_global_[leaf] = ls->count;
}

void SerialTreeLearner::BeforeTrain() {
  col_sampler_.ResetByTree();
  partition_.Reset();
  for (auto& s : best_split_per_leaf_) s.Reset();
  for (auto& b : bounds_) b = LeafBounds();
  for (auto& s : splittable_) std::fill(s.begin(), s.end(), 1);
  if (intermediate_monotone_) mono_.Reset();
  if (cegb_) cegb_->BeforeTree();
  if (resident_) {
    for (size_t l = 0; l < dslot_.size(); ++l) dslot_[l] = static_cast<int>(l);
    std::fill(dvalid_.begin(), dvalid_.end(), 0);
  }
  double sg, sh;
  ComputeLeafSums(partition_.indices(0), partition_.count(0), &sg, &sh);
  InitLeafStat(&smaller_, 0, sg, sh, 0.0);
  larger_ = LeafStat();
  has_parent_hist_ = false;
}

double SerialTreeLearner::ParentOutput(const Tree* tree, const LeafStat& ls) const {
  if (tree->num_leaves() == 1) {
    SplitParams p = MakeParams();
    p.path_smooth = 0.0;
    return LeafOutputRaw(ls.sum_g, ls.sum_h, p, ls.global_count, 0.0);
  }
  return ls.output;
}

double SerialTreeLearner::MonotonePenalty(const Tree* tree, int leaf) const {
  const double pen = config_->monotone_penalty;
  const int depth = tree->leaf_depth(leaf);
  if (pen >= depth + 1.0) return kEpsilon;
  if (pen <= 1.0) return 1.0 - pen / std::pow(2.0, depth) + kEpsilon;
  return 1.0 - std::pow(2.0, pen - 1.0 - depth) + kEpsilon;
}

SplitInfo SerialTreeLearner::BestSplitForFeature(const double* group_hist, int f, const LeafStat& leaf,
                                                 double parent_output, const LeafBounds& bounds,
                                                 const ThresholdBounds* tb, bool* splittable) const {
  const FeatureInfo& fi = train_data_->feature(f);
  std::vector<double> full(2 * fi.num_bin);
  train_data_->FeatureHistogram(group_hist, f, leaf.sum_g, leaf.sum_h, full.data());
  FeatureScanMeta m;
  m.num_bin = fi.num_bin;
  m.default_bin = fi.default_bin;
  m.missing_type = static_cast<int8_t>(fi.missing);
  m.bin_type = static_cast<int8_t>(fi.bin_type);
  m.monotone = fi.monotone;
  m.penalty = fi.penalty;
  SplitParams p = MakeParams();
  SplitInfo out;
  out.Reset();
  if (config_->extra_trees) {
    // per-feature RNG stream (feature_histogram.hpp:1450): Random(extra_seed + f)
    Random& r = const_cast<std::vector<Random>&>(extra_rands_)[f];
    if (fi.bin_type == BinType::Numerical) {
      if (fi.num_bin - 2 > 0) m.rand_threshold = r.NextInt(0, fi.num_bin - 2);
    } else if (fi.num_bin <= p.max_cat_to_onehot) {
      if (fi.num_bin - 1 > 0) m.rand_threshold = r.NextInt(1, fi.num_bin);
    } else {
      const double cnt_factor = leaf.global_count / (leaf.sum_h + 2 * kEpsilon);
      int used = 0;
      for (int b = 1; b < fi.num_bin; ++b) used += RoundCount(full[2 * b + 1] * cnt_factor) >= p.cat_smooth;
      const int max_num_cat = std::min(p.max_cat_threshold, (used + 1) / 2);
      const int max_thr = std::max(std::min(max_num_cat, used) - 1, 0);
      if (max_thr > 0) m.rand_threshold = r.NextInt(0, max_thr);
    }
  }
  bool sp;
  if (fi.bin_type == BinType::Numerical) {
    sp = FindBestNumerical(full.data(), m, p, leaf.sum_g, leaf.sum_h, leaf.global_count, parent_output, bounds, &out,
                           tb);
  } else {
    std::vector<int> order(fi.num_bin);
    sp = FindBestCategorical(full.data(), m, p, leaf.sum_g, leaf.sum_h, leaf.global_count, parent_output, bounds,
                             order.data(), &out);
  }
  *splittable = sp;
  out.feature = sp ? f : -1;
  if (!sp) out.gain = kMinScore;
  return out;
}

std::unique_ptr<Tree> SerialTreeLearner::Train(const score_t* gradients, const score_t* hessians, bool) {
  ScopedTimer t("SerialTreeLearner::Train");
  gradients_ = true_gradients_ = gradients;
  hessians_ = true_hessians_ = hessians;
  if (config_->use_quantized_grad) {
    // integer-level (g, h); sums of de-scaled integers are exact in the fp64 histograms
    quantizer_.Quantize(gradients, hessians, num_data_, is_constant_hessian_, qgrad_.data(), qhess_.data());
    gradients_ = qgrad_.data();
    hessians_ = qhess_.data();
  }
  if (hist_backend_) hist_backend_->SetGradients(gradients_, hessians_, num_data_);
  if (extra_rands_.size() != static_cast<size_t>(num_features_)) {
    extra_rands_.clear();
    for (int f = 0; f < num_features_; ++f) extra_rands_.emplace_back(config_->extra_seed + f);
  }
  BeforeTrain();
  const bool track = !config_->interaction_constraints_vector.empty();
  auto tree = std::make_unique<Tree>(config_->num_leaves, track, false);
  {
    SplitParams p = MakeParams();
    p.path_smooth = 0.0;
    tree->SetLeafOutput(0, LeafOutputRaw(smaller_.sum_g, smaller_.sum_h, p, smaller_.global_count, 0.0));
    smaller_.output = tree->LeafOutput(0);
  }
  int left = 0, right = -1;
  forced_rescored_ = false;
  int init_splits = ForceSplits(tree.get(), &left, &right);
  for (int s = init_splits; s < config_->num_leaves - 1; ++s) {
    // after forced splits every leaf already has its best split (ForceSplits rescored them)
    if (forced_rescored_) forced_rescored_ = false;
    else if (BeforeFindBestSplit(tree.get(), left, right)) FindBestSplits(tree.get());
    int best = 0;
    for (int l = 1; l < tree->num_leaves(); ++l) {
      if (best_split_per_leaf_[l].BetterThan(best_split_per_leaf_[best])) best = l;
    }
    const SplitInfo& bs = best_split_per_leaf_[best];
    if (bs.feature < 0 || bs.gain <= 0.0) {
      Log::Debug("No further splits with positive gain, best gain: %f", bs.gain);
      break;
    }
    Split(tree.get(), best, &left, &right);
  }
  if (config_->use_quantized_grad && config_->quant_train_renew_leaf) RenewQuantizedLeaves(tree.get());
  tree->RecomputeMaxDepth();
  return tree;
}

bool SerialTreeLearner::BeforeFindBestSplit(const Tree* tree, int left, int right) {
  if (config_->max_depth > 0 && tree->leaf_depth(left) >= config_->max_depth) {
    best_split_per_leaf_[left].gain = kMinScore;
    best_split_per_leaf_[left].feature = -1;
    if (right >= 0) {
      best_split_per_leaf_[right].gain = kMinScore;
      best_split_per_leaf_[right].feature = -1;
    }
    return false;
  }
  const data_size_t nl = GlobalCount(left), nr = GlobalCount(right);
  if (nr < config_->min_data_in_leaf * 2 && nl < config_->min_data_in_leaf * 2) {
    best_split_per_leaf_[left].gain = kMinScore;
    best_split_per_leaf_[left].feature = -1;
    if (right >= 0) {
      best_split_per_leaf_[right].gain = kMinScore;
      best_split_per_leaf_[right].feature = -1;
    }
    return false;
  }
  has_parent_hist_ = false;
  if (right >= 0) {
    // the parent histogram lives in hist_[left]; hand it to the larger child
    if (larger_.leaf == right) {
      std::swap(hist_[left], hist_[right]);
      std::swap(hist_stamp_[left], hist_stamp_[right]);
      std::swap(splittable_[left], splittable_[right]);
      if (resident_) {
        std::swap(dslot_[left], dslot_[right]);
        std::swap(dvalid_[left], dvalid_[right]);
      }
    }
    hist_stamp_[larger_.leaf] = ++hist_clock_;
    has_parent_hist_ = resident_ ? dvalid_[larger_.leaf] != 0
                                 : hist_[larger_.leaf].size() == static_cast<size_t>(2 * train_data_->num_total_bin());
    // the smaller child inherits the parent's splittable flags too
    splittable_[smaller_.leaf] = splittable_[larger_.leaf];
  }
  return true;
}

void SerialTreeLearner::FindBestSplits(const Tree* tree) {
  ConstructHistograms(has_parent_hist_);
  FindBestSplitsFromHistograms(tree, has_parent_hist_);
}

void SerialTreeLearner::ConstructHistograms(bool use_subtract) {
  ScopedTimer timer("SerialTreeLearner::ConstructHistograms");
  if (resident_) {
    hist_backend_->HistogramToSlot(partition_.indices(smaller_.leaf), partition_.count(smaller_.leaf),
                                   dslot_[smaller_.leaf]);
    dvalid_[smaller_.leaf] = 1;
    if (larger_.leaf >= 0 && !use_subtract) {
      hist_backend_->HistogramToSlot(partition_.indices(larger_.leaf), partition_.count(larger_.leaf),
                                     dslot_[larger_.leaf]);
      dvalid_[larger_.leaf] = 1;
    }
    return;
  }
  BuildHistogram(partition_.indices(smaller_.leaf), partition_.count(smaller_.leaf), HistOf(smaller_.leaf).data());
  if (larger_.leaf >= 0 && !use_subtract) {
    BuildHistogram(partition_.indices(larger_.leaf), partition_.count(larger_.leaf), HistOf(larger_.leaf).data());
  }
}

void SerialTreeLearner::FindBestSplitsFromHistograms(const Tree* tree, bool use_subtract) {
  ScopedTimer timer("SerialTreeLearner::FindBestSplitsFromHistograms");
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  std::vector<int8_t> node_s = col_sampler_.GetByNode(tree, smaller_.leaf);
  std::vector<int8_t> node_l;
  const bool has_larger = larger_.leaf >= 0;
  if (has_larger) node_l = col_sampler_.GetByNode(tree, larger_.leaf);
  const double po_s = ParentOutput(tree, smaller_);
  const double po_l = has_larger ? ParentOutput(tree, larger_) : 0.0;
  if (resident_) {
    // the same flow on the device: subtraction in the larger child's slot, one scan launch for
    // both children, only their per-feature SplitInfo rows come back
    if (use_subtract && has_larger) hist_backend_->SubtractSlots(dslot_[larger_.leaf], dslot_[smaller_.leaf]);
    auto& spl_s = splittable_[smaller_.leaf];
    std::vector<char> en(num_features_);
    for (int f = 0; f < num_features_; ++f) {
      en[f] = bytree[f] && feature_mask_[f] && !(use_subtract && !spl_s[f]);
    }
    std::vector<const LeafStat*> leaves{&smaller_};
    std::vector<double> po{po_s};
    std::vector<const std::vector<char>*> ens{&en};
    if (has_larger) {
      leaves.push_back(&larger_);
      po.push_back(po_l);
      ens.push_back(&en);
    }
    std::vector<SplitInfo> out;
    std::vector<uint8_t> sp;
    DeviceScanLeaves(tree, leaves, po, ens, &out, &sp);
    SplitInfo best_s, best_l;
    best_s.Reset();
    best_l.Reset();
    for (int f = 0; f < num_features_; ++f) {
      if (!en[f]) continue;
      spl_s[f] = sp[f];
      if (node_s[f] && out[f].feature >= 0 && out[f].BetterThan(best_s)) best_s = out[f];
      if (has_larger) {
        const size_t j = static_cast<size_t>(num_features_) + f;
        splittable_[larger_.leaf][f] = sp[j];
        if (node_l[f] && out[j].feature >= 0 && out[j].BetterThan(best_l)) best_l = out[j];
      }
    }
    best_split_per_leaf_[smaller_.leaf] = best_s;
    if (has_larger) best_split_per_leaf_[larger_.leaf] = best_l;
    SyncBestSplits();
    return;
  }
  const double* hs = HistOf(smaller_.leaf).data();
  if (use_subtract && has_larger) {
    double* hl = HistOf(larger_.leaf).data();
    const int j0 = 2 * hist_begin_, j1 = 2 * hist_end_;
#pragma omp parallel for schedule(static) if (j1 - j0 >= 65536)
    for (int j = j0; j < j1; ++j) hl[j] -= hs[j];
  }
  const double* hl = has_larger ? HistOf(larger_.leaf).data() : nullptr;
  std::vector<SplitInfo> bs(num_features_), bl(num_features_);
  auto& spl_s = splittable_[smaller_.leaf];
  std::vector<char>* spl_l = has_larger ? &splittable_[larger_.leaf] : nullptr;
#pragma omp parallel for schedule(dynamic)
  for (int f = 0; f < num_features_; ++f) {
    bs[f].Reset();
    bl[f].Reset();
    if (!bytree[f] || !feature_mask_[f]) continue;
    if (use_subtract && !spl_s[f]) {
      // the parent could not split on f: neither child tries (feature_histogram is_splittable inheritance)
      continue;
    }
    bool sp = false;
    SplitInfo s = ScoreFeature(tree, hs, f, smaller_, po_s, &sp);
    spl_s[f] = sp;
    if (node_s[f]) bs[f] = s;
    if (has_larger) {
      SplitInfo l = ScoreFeature(tree, hl, f, larger_, po_l, &sp);
      (*spl_l)[f] = sp;
      if (node_l[f]) bl[f] = l;
    }
  }
  SplitInfo best_s, best_l;
  best_s.Reset();
  best_l.Reset();
  for (int f = 0; f < num_features_; ++f) {
    if (bs[f].feature >= 0 && bs[f].BetterThan(best_s)) best_s = bs[f];
    if (bl[f].feature >= 0 && bl[f].BetterThan(best_l)) best_l = bl[f];
  }
  best_split_per_leaf_[smaller_.leaf] = best_s;
  if (has_larger) best_split_per_leaf_[larger_.leaf] = best_l;
  SyncBestSplits();
}

SplitInfo SerialTreeLearner::ScoreFeature(const Tree* tree, const double* group_hist, int f, const LeafStat& leaf,
                                          double parent_output, bool* splittable) {
  SplitInfo s;
  if (intermediate_monotone_ && mono_.advanced() && train_data_->feature(f).bin_type == BinType::Numerical) {
    // advanced monotone: the bounds of this feature's thresholds (serial_tree_learner.cpp:970-974)
    std::vector<double> scratch;
    ThresholdBounds tb;
    LeafBounds flat;
    const bool varies = mono_.ThresholdBoundsFor(tree, f, leaf.leaf, &scratch, &tb, &flat);
    s = BestSplitForFeature(group_hist, f, leaf, parent_output, flat, varies ? &tb : nullptr, splittable);
  } else {
    s = BestSplitForFeature(group_hist, f, leaf, parent_output, bounds_[leaf.leaf], nullptr, splittable);
  }
  if (s.feature < 0) return s;
  if (cegb_) {
    s.gain -= cegb_->DeltaGain(f, leaf.leaf, partition_.indices(leaf.leaf), partition_.count(leaf.leaf), s,
                               leaf.global_count);
  }
  if (s.monotone_type != 0) s.gain *= MonotonePenalty(tree, leaf.leaf);
  return s;
}

// reference serial_tree_learner.cpp RecomputeBestSplitForLeaf: the leaf keeps its
// histogram; its statistics come from the pending best split
void SerialTreeLearner::RecomputeBestSplit(const Tree* tree, int leaf) {
  SplitInfo& cur = best_split_per_leaf_[leaf];
  if (resident_ && !dvalid_[leaf]) {
    hist_backend_->HistogramToSlot(partition_.indices(leaf), partition_.count(leaf), dslot_[leaf]);
    dvalid_[leaf] = 1;
  } else if (!resident_ && hist_[leaf].size() != static_cast<size_t>(2 * train_data_->num_total_bin())) {
    // dropped from the histogram pool: rebuilt from the leaf's rows (the reference skips the
    // rescan here, serial_tree_learner.cpp:1025-1031, leaving a split that may break the
    // tightened bounds)
    BuildHistogram(partition_.indices(leaf), partition_.count(leaf), HistOf(leaf).data());
  }
  LeafStat ls;
  ls.leaf = leaf;
  ls.sum_g = cur.left_sum_gradient + cur.right_sum_gradient;
  ls.sum_h = cur.left_sum_hessian + cur.right_sum_hessian;
  ls.count = ls.global_count = cur.left_count + cur.right_count;
  double po = 0.0;
  if (config_->path_smooth > kEpsilon) {
    SplitParams p = MakeParams();
    p.path_smooth = 0.0;
    po = LeafOutputRaw(ls.sum_g, ls.sum_h, p, ls.count, 0.0);
  }
  ls.output = po;
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  // node-level sampling and interaction constraints of this leaf (serial_tree_learner.cpp:1050)
  const std::vector<int8_t> node_used = col_sampler_.GetByNode(tree, leaf);
  SplitInfo best;
  best.Reset();
  if (resident_) {
    std::vector<char> en(num_features_);
    for (int f = 0; f < num_features_; ++f) en[f] = bytree[f] && feature_mask_[f] && splittable_[leaf][f];
    std::vector<SplitInfo> out;
    std::vector<uint8_t> sp;
    DeviceScanLeaves(tree, {&ls}, {po}, {&en}, &out, &sp);
    for (int f = 0; f < num_features_; ++f) {
      if (en[f] && node_used[f] && out[f].feature >= 0 && out[f].BetterThan(best)) best = out[f];
    }
    cur = best;
    return;
  }
  for (int f = 0; f < num_features_; ++f) {
    if (!bytree[f] || !feature_mask_[f] || !splittable_[leaf][f]) continue;
    bool sp;
    SplitInfo s = ScoreFeature(tree, hist_[leaf].data(), f, ls, po, &sp);
    if (node_used[f] && s.feature >= 0 && s.BetterThan(best)) best = s;
  }
  cur = best;
}

void SerialTreeLearner::DeviceScanLeaves(const Tree* tree, const std::vector<const LeafStat*>& leaves,
                                         const std::vector<double>& po,
                                         const std::vector<const std::vector<char>*>& enable,
                                         std::vector<SplitInfo>* out, std::vector<uint8_t>* splittable) {
  ScopedTimer timer("SerialTreeLearner::DeviceScanLeaves");
  const int F = num_features_;
  const int R = static_cast<int>(leaves.size());
  auto& b = scan_batch_;
  b.Clear();
  const bool advanced = intermediate_monotone_ && mono_.advanced();
  std::vector<double> scratch;
  for (int r = 0; r < R; ++r) {
    const LeafStat& ls = *leaves[r];
    b.slot.push_back(dslot_[ls.leaf]);
    b.count.push_back(ls.global_count);
    b.sum_g.push_back(ls.sum_g);
    b.sum_h.push_back(ls.sum_h);
    b.parent_output.push_back(po[r]);
    for (int f = 0; f < F; ++f) {
      const bool en = (*enable[r])[f] != 0;
      b.enable.push_back(en ? 1 : 0);
      long long off = -1;
      LeafBounds lb = bounds_[ls.leaf];
      if (en && advanced && train_data_->feature(f).bin_type == BinType::Numerical) {
        // advanced monotone: the feature's per-threshold child bounds (ScoreFeature's host path)
        ThresholdBounds tb;
        LeafBounds flat;
        if (mono_.ThresholdBoundsFor(tree, f, ls.leaf, &scratch, &tb, &flat)) {
          const int nb = train_data_->feature(f).num_bin;
          off = static_cast<long long>(b.tb.size());
          for (const double* arr : {tb.lmin, tb.lmax, tb.rmin, tb.rmax}) b.tb.insert(b.tb.end(), arr, arr + nb);
        }
        lb = flat;
      }
      b.bmin.push_back(lb.min);
      b.bmax.push_back(lb.max);
      b.tb_off.push_back(off);
    }
  }
  out->assign(static_cast<size_t>(R) * F, SplitInfo());
  splittable->assign(static_cast<size_t>(R) * F, 0);
  hist_backend_->ScanSlots(b, MakeParams(), out->data(), splittable->data());
  // ScoreFeature's adjustments of a found split: CEGB deduction, then the monotone penalty
  for (int r = 0; r < R; ++r) {
    const LeafStat& ls = *leaves[r];
    for (int f = 0; f < F; ++f) {
      SplitInfo& s = (*out)[static_cast<size_t>(r) * F + f];
      if (s.feature < 0) continue;
      if (cegb_) {
        s.gain -= cegb_->DeltaGain(f, ls.leaf, partition_.indices(ls.leaf), partition_.count(ls.leaf), s,
                                   ls.global_count);
      }
      if (s.monotone_type != 0) s.gain *= MonotonePenalty(tree, ls.leaf);
    }
  }
}

void SerialTreeLearner::RenewQuantizedLeaves(Tree* tree) const {
  const int nl = tree->num_leaves();
  std::vector<double> st(2 * nl, 0.0);
  for (int l = 0; l < nl; ++l) {
    const data_size_t n = partition_.count(l);
    const data_size_t* idx = partition_.indices(l);
    double g = 0.0, h = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : g, h) if (n >= 4096)
    for (data_size_t i = 0; i < n; ++i) {
      g += true_gradients_[idx[i]];
      h += true_hessians_[idx[i]];
    }
    st[2 * l] = g;
    st[2 * l + 1] = h;
  }
  const bool global = config_->tree_learner == "data" && Network::num_machines() > 1;
  if (global) Network::GlobalSum(&st);
  SplitParams p = MakeParams();
  p.path_smooth = 0.0;
  for (int l = 0; l < nl; ++l) {
    const data_size_t cnt = global ? GlobalCount(l) : partition_.count(l);
    tree->SetLeafOutput(l, LeafOutputRaw(st[2 * l], st[2 * l + 1], p, cnt, 0.0));
  }
}

void SerialTreeLearner::Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) {
  ScopedTimer timer("SerialTreeLearner::Split");
  if (cegb_) {
    cegb_->OnSplit(tree->num_leaves(), best_leaf, best_split_per_leaf_[best_leaf], partition_.indices(best_leaf),
                   partition_.count(best_leaf), &best_split_per_leaf_);
  }
  SplitInfo info = best_split_per_leaf_[best_leaf];
  const int f = info.feature;
  const FeatureInfo& fi = train_data_->feature(f);
  const BinMapper& mapper = train_data_->inner_mapper(f);
  const int next = tree->num_leaves();
  *left_leaf = best_leaf;
  const Dataset* d = train_data_;
  data_size_t nl;
  if (intermediate_monotone_) mono_.BeforeSplit(tree, best_leaf, next, info.monotone_type);
  if (fi.bin_type == BinType::Numerical) {
    const uint32_t thr = info.threshold;
    const bool dl = info.default_left != 0;
    const MissingType mt = fi.missing;
    const uint32_t nan_bin = static_cast<uint32_t>(fi.num_bin - 1);
    auto pf = [&](data_size_t r) { __builtin_prefetch(d->dense_row(r)); };
    nl = partition_.Split(best_leaf, next, [&](data_size_t r) {
      const uint32_t b = d->FeatureBin(r, f);
      if ((mt == MissingType::Zero && b == fi.default_bin) || (mt == MissingType::NaN && b == nan_bin)) return dl;
      return b <= thr;
    }, pf);
    if (!global_counts_from_split_) {
      info.left_count = nl;
      info.right_count = partition_.count(next);
    }
    *right_leaf = tree->Split(best_leaf, f, fi.real_index, thr, mapper.BinToValue(thr), info.left_output,
                              info.right_output, info.left_count, info.right_count, info.left_sum_hessian,
                              info.right_sum_hessian, static_cast<float>(info.gain + config_->min_gain_to_split),
                              mt, dl);
  } else {
    const uint32_t* bits = info.cat_bitset;
    int nwords = 0;
    std::vector<int> cats;
    for (int w = 0; w < kMaxCatWords; ++w) {
      if (bits[w]) nwords = w + 1;
      for (int j = 0; j < 32; ++j) {
        if ((bits[w] >> j) & 1) cats.push_back(mapper.bin_to_category()[w * 32 + j]);
      }
    }
    std::vector<uint32_t> inner(bits, bits + nwords);
    std::vector<uint32_t> raw = common::ConstructBitset(cats.data(), static_cast<int>(cats.size()));
    nl = partition_.Split(best_leaf, next, [&](data_size_t r) {
      const uint32_t b = d->FeatureBin(r, f);
      return common::FindInBitset(inner.data(), nwords, static_cast<int>(b));
    });
    if (!global_counts_from_split_) {
      info.left_count = nl;
      info.right_count = partition_.count(next);
    }
    *right_leaf = tree->SplitCategorical(best_leaf, f, fi.real_index, inner.data(), nwords, raw.data(),
                                         static_cast<int>(raw.size()), info.left_output, info.right_output,
                                         info.left_count, info.right_count, info.left_sum_hessian,
                                         info.right_sum_hessian,
                                         static_cast<float>(info.gain + config_->min_gain_to_split), fi.missing);
  }
  // children statistics; the smaller (by count) child gets the fresh histogram
  if (info.left_count < info.right_count) {
    InitLeafStat(&smaller_, *left_leaf, info.left_sum_gradient, info.left_sum_hessian, info.left_output);
    InitLeafStat(&larger_, *right_leaf, info.right_sum_gradient, info.right_sum_hessian, info.right_output);
  } else {
    InitLeafStat(&smaller_, *right_leaf, info.right_sum_gradient, info.right_sum_hessian, info.right_output);
    InitLeafStat(&larger_, *left_leaf, info.left_sum_gradient, info.left_sum_hessian, info.left_output);
  }
  if (global_counts_from_split_) {
    leaf_count_global_[*left_leaf] = info.left_count;
    leaf_count_global_[*right_leaf] = info.right_count;
    smaller_.global_count = leaf_count_global_[smaller_.leaf];
    larger_.global_count = leaf_count_global_[larger_.leaf];
  }
  bounds_[next] = bounds_[best_leaf];
  if (intermediate_monotone_) {
    const auto redo = mono_.AfterSplit(tree, &bounds_, fi.bin_type == BinType::Numerical, best_leaf, next,
                                       info.monotone_type, info, best_split_per_leaf_);
    for (int l : redo) RecomputeBestSplit(tree, l);
  } else if (use_monotone_ && fi.bin_type == BinType::Numerical) {
    // basic method: both children bounded by the midpoint of their outputs
    const double mid = (info.left_output + info.right_output) / 2.0f;
    if (info.monotone_type < 0) {
      bounds_[best_leaf].min = std::max(bounds_[best_leaf].min, mid);
      bounds_[next].max = std::min(bounds_[next].max, mid);
    } else if (info.monotone_type > 0) {
      bounds_[best_leaf].max = std::min(bounds_[best_leaf].max, mid);
      bounds_[next].min = std::max(bounds_[next].min, mid);
    }
  }
}

// Forced splits from a JSON file: ForcedNode / ParseForced in learner/forced_splits.h.

// reference gbdt.cpp CheckForcedSplitFeatures: every node's feature must exist in the data
void SerialTreeLearner::CheckForcedSplitFeatures() const {
  if (forced_json_.empty()) return;
  size_t pos = 0;
  auto root = ParseForced(forced_json_, &pos);
  const int max_idx = train_data_->num_total_features() - 1;
  std::queue<const ForcedNode*> q;
  if (root) q.push(root.get());
  while (!q.empty()) {
    const ForcedNode* n = q.front();
    q.pop();
    if (n->feature > max_idx) {
      Log::Fatal("Forced splits file includes feature index %d, but maximum feature index in dataset is %d",
                 n->feature, max_idx);
    }
    if (n->left) q.push(n->left.get());
    if (n->right) q.push(n->right.get());
  }
}

int SerialTreeLearner::ForceSplits(Tree* tree, int* left_leaf, int* right_leaf) {
  if (forced_json_.empty()) return 0;
  size_t pos = 0;
  auto root = ParseForced(forced_json_, &pos);
  if (!root || root->feature < 0) return 0;
  int done = 0;
  std::queue<std::pair<const ForcedNode*, int>> q;
  q.push({root.get(), 0});
  while (!q.empty() && done < config_->num_leaves - 1) {
    auto [node, leaf] = q.front();
    q.pop();
    if (node->feature < 0 || node->feature >= train_data_->num_total_features()) continue;
    const int inner = train_data_->InnerIndex(node->feature);
    if (inner < 0) continue;
    const FeatureInfo& fi = train_data_->feature(inner);
    if (fi.bin_type != BinType::Numerical) continue;
    // statistics of `leaf`: build its histogram directly
    LeafStat ls;
    double sg, sh;
    ComputeLeafSums(partition_.indices(leaf), partition_.count(leaf), &sg, &sh);
    ls.leaf = leaf;
    ls.sum_g = sg;
    ls.sum_h = sh;
    ls.count = ls.global_count = partition_.count(leaf);
    ls.output = tree->LeafOutput(leaf);
    auto& h = HistOf(leaf);
    BuildHistogram(partition_.indices(leaf), partition_.count(leaf), h.data());
    std::vector<double> full(2 * fi.num_bin);
    train_data_->FeatureHistogram(h.data(), inner, sg, sh, full.data());
    const uint32_t thr = train_data_->inner_mapper(inner).ValueToBin(node->threshold);
    // GatherInfoForThresholdNumerical (feature_histogram.hpp:486-588): the right side
    // sums bins above the threshold, skipping the zero bin (MissingType::Zero) and
    // the NaN bin (MissingType::NaN); missing values go left
    const bool na = fi.missing == MissingType::NaN, zero = fi.missing == MissingType::Zero;
    double rg = 0.0, rh = 0.0;
    data_size_t rc = 0;
    const double cf = ls.count / sh;
    for (int b = fi.num_bin - 1 - (na ? 1 : 0); b >= 1; --b) {
      if (static_cast<uint32_t>(b) <= thr) break;
      if (zero && b == static_cast<int>(fi.default_bin)) continue;
      rg += full[2 * b];
      rh += full[2 * b + 1];
      rc += RoundCount(full[2 * b + 1] * cf);
    }
    const double lg = sg - rg, lh = sh - rh;
    const data_size_t lc = ls.count - rc;
    SplitParams p = MakeParams();
    SplitInfo info;
    info.Reset();
    info.feature = inner;
    info.threshold = thr;
    info.default_left = 1;
    info.left_sum_gradient = lg;
    info.left_sum_hessian = lh;
    info.right_sum_gradient = rg;
    info.right_sum_hessian = rh;
    info.left_count = lc;
    info.right_count = rc;
    info.left_output = LeafOutputRaw(lg, lh, p, lc, ls.output);
    info.right_output = LeafOutputRaw(rg, rh, p, rc, ls.output);
    info.gain = SplitGain(lg, lh, rg, rh, p, 0, lc, rc, ls.output, LeafBounds()) -
                LeafGain(sg, sh, p, ls.count, ls.output) - config_->min_gain_to_split;
    if (!(info.gain > 0.0)) {
      Log::Warning("'Forced Split' will be ignored since the gain getting worse.");
      break;
    }
    best_split_per_leaf_[leaf] = info;
    Split(tree, leaf, left_leaf, right_leaf);
    ++done;
    if (node->left) q.push({node->left.get(), *left_leaf});
    if (node->right) q.push({node->right.get(), *right_leaf});
  }
  // fresh start for the regular loop: recompute best splits for all current leaves
  for (int l = 0; l < tree->num_leaves(); ++l) {
    double sg, sh;
    ComputeLeafSums(partition_.indices(l), partition_.count(l), &sg, &sh);
    LeafStat ls;
    InitLeafStat(&ls, l, sg, sh, tree->LeafOutput(l));
    BuildHistogram(partition_.indices(l), partition_.count(l), HistOf(l).data());
    SplitInfo best;
    best.Reset();
    for (int f = 0; f < num_features_; ++f) {
      if (!col_sampler_.is_feature_used_bytree()[f]) continue;
      bool sp;
      SplitInfo s = ScoreFeature(tree, HistOf(l).data(), f, ls, ls.output, &sp);
      if (s.feature >= 0 && s.BetterThan(best)) best = s;
    }
    best_split_per_leaf_[l] = best;
  }
  // the main loop resumes with no pending histograms to build
  forced_rescored_ = true;
  *left_leaf = 0;
  *right_leaf = -1;
  smaller_.leaf = 0;
  larger_.leaf = -1;
  return done;
}

// ----------------------------------------------------------------------------
std::unique_ptr<Tree> SerialTreeLearner::FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                                           const score_t* g, const score_t* h) {
  auto tree = std::make_unique<Tree>(*old_tree);
  partition_.ResetByLeafPred(leaf_pred, tree->num_leaves());
  SplitParams p = MakeParams();
  for (int i = 0; i < tree->num_leaves(); ++i) {
    const data_size_t n = partition_.count(i);
    const data_size_t* idx = partition_.indices(i);
    double sg = 0.0, sh = kEpsilon;
    for (data_size_t j = 0; j < n; ++j) {
      sg += g[idx[j]];
      sh += h[idx[j]];
    }
    double out;
    if (config_->path_smooth > kEpsilon && i > 0) {
      out = LeafOutputRaw(sg, sh, p, n, tree->leaf_parent(i));
    } else {
      SplitParams q = p;
      q.path_smooth = 0.0;
      out = LeafOutputRaw(sg, sh, q, n, 0.0);
    }
    const double old_v = tree->LeafOutput(i);
    const double new_v = out * tree->shrinkage();
    tree->SetLeafOutput(i, config_->refit_decay_rate * old_v + (1.0 - config_->refit_decay_rate) * new_v);
  }
  return tree;
}

void SerialTreeLearner::AddPredictionToScore(const Tree* tree, double* out_score) const {
  if (tree->num_leaves() <= 1) {
    const double v = tree->LeafOutput(0);
    const data_size_t n = partition_.count(0);
    const data_size_t* idx = partition_.indices(0);
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) out_score[idx[i]] += v;
    return;
  }
#pragma omp parallel for schedule(dynamic)
  for (int l = 0; l < tree->num_leaves(); ++l) {
    const double v = tree->LeafOutput(l);
    const data_size_t n = partition_.count(l);
    const data_size_t* idx = partition_.indices(l);
    for (data_size_t i = 0; i < n; ++i) out_score[idx[i]] += v;
  }
}

void SerialTreeLearner::RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj, const double* score, data_size_t,
                                        const data_size_t*, data_size_t) const {
  if (obj == nullptr || !obj->IsRenewTreeOutput()) return;
  const int nl = tree->num_leaves();
  std::vector<double> outs(nl, 0.0);
  std::vector<int> nonzero(nl, 1);
#pragma omp parallel for schedule(dynamic)
  for (int l = 0; l < nl; ++l) {
    const data_size_t n = partition_.count(l);
    if (n > 0) {
      outs[l] = obj->RenewTreeOutput(tree->LeafOutput(l), score, partition_.indices(l), n);
    } else {
      outs[l] = 0.0;
      nonzero[l] = 0;
    }
  }
  if (Network::num_machines() > 1) {
    Network::GlobalSum(&outs);
    Network::GlobalSum(&nonzero);
    for (int l = 0; l < nl; ++l) outs[l] = nonzero[l] > 0 ? outs[l] / nonzero[l] : 0.0;
  }
  for (int l = 0; l < nl; ++l) tree->SetLeafOutput(l, outs[l]);
}

std::string SerialTreeLearner::DeviceName() const {
  if (resident_) return hist_backend_->DeviceName() + " (HIP histograms and split scans, host constraint bookkeeping)";
  return hist_backend_ ? hist_backend_->DeviceName() + " (HIP histograms, host split policy)" : "cpu";
}

std::vector<data_size_t> SerialTreeLearner::LeafIndices(int leaf) const {
  return std::vector<data_size_t>(partition_.indices(leaf), partition_.indices(leaf) + partition_.count(leaf));
}

}  // namespace lgap
