// Host leaf-wise tree learner: the correctness oracle for the HIP learner and
// the device_type=cpu path. Reference: src/treelearner/serial_tree_learner.{h,cpp},
// data_partition.hpp, leaf_splits.hpp, col_sampler.hpp, monotone_constraints.hpp
// (basic method), feature_histogram.hpp (via split_math.h).
#pragma once

#include <omp.h>

#include <memory>
#include <set>
#include <vector>

#include "leaf_constraints.h"
#include "lgap/device_api.h"
#include "lgap/random.h"
#include "lgap/split_math.h"
#include "lgap/tree_learner.h"

namespace lgap {

// Feature sampling by tree / by node and interaction constraints.
class ColSampler {
 public:
  void Init(const Dataset* data, const Config* cfg);
  void ResetByTree();
  std::vector<int8_t> GetByNode(const Tree* tree, int leaf);
  const std::vector<int8_t>& is_feature_used_bytree() const { return used_bytree_; }
  // the node sampler's random state: a device learner that pre-draws a tree's by-node masks
  // rewinds to it and replays only the draws the tree used, so the stream stays the host's
  const Random& rng_state() const { return rand_; }
  void set_rng_state(const Random& r) { rand_ = r; }
  // by-node masks drawn on the device (interaction constraints: each node's pool depends on its
  // path): Random::Sample's branch for a pool of n = 0..num_features features (0 none, 1 all,
  // 2 Bernoulli scan, 3 Floyd), the draw count, and whether the pool keeps only by-tree features
  std::vector<uint8_t> ByNodeSampleModes(int* cnt, bool* filter_bytree) const;

 private:
  static int GetCnt(size_t total, double fraction);
  const Dataset* data_ = nullptr;
  double frac_tree_ = 1.0, frac_node_ = 1.0;
  bool need_reset_tree_ = false;
  int used_cnt_tree_ = 0;
  Random rand_;
  int seed_ = -1;
  std::vector<int> valid_;          // real feature indices of used features
  std::vector<int> used_idx_;       // sampled positions into valid_
  std::vector<int8_t> used_bytree_;
  std::vector<std::set<int>> interaction_;
};

// Contiguous per-leaf index ranges with stable 2-way split.
class DataPartition {
 public:
  void Init(data_size_t num_data, int num_leaves);
  void SetUsedIndices(const data_size_t* idx, data_size_t n);
  void Reset();  // all rows (or the bag) into leaf 0
  // go_left(row) -> bool; returns left count. prefetch(row) is called a few rows ahead of
  // go_left on the same row (the rows of a deep leaf are scattered)
  template <typename F, typename P>
  data_size_t Split(int leaf, int right_leaf, F go_left, P prefetch);
  template <typename F>
  data_size_t Split(int leaf, int right_leaf, F go_left) {
    return Split(leaf, right_leaf, go_left, [](data_size_t) {});
  }
  const data_size_t* indices(int leaf) const { return indices_.data() + begin_[leaf]; }
  data_size_t count(int leaf) const { return count_[leaf]; }
  data_size_t begin(int leaf) const { return begin_[leaf]; }
  void ResetByLeafPred(const std::vector<int>& leaf_pred, int num_leaves);
  int num_leaves() const { return static_cast<int>(begin_.size()); }

 private:
  data_size_t num_data_ = 0;
  std::vector<data_size_t> indices_, tmp_;
  std::vector<data_size_t> begin_, count_;
  std::vector<data_size_t> used_;
  bool use_bag_ = false;
  data_size_t bag_cnt_ = 0;
};

struct LeafStat {
  int leaf = -1;
  double sum_g = 0.0, sum_h = 0.0;
  data_size_t count = 0;         // local rows
  data_size_t global_count = 0;  // all ranks
  double output = 0.0;           // leaf weight (parent output for path smoothing)
};

class SerialTreeLearner : public TreeLearner {
 public:
  explicit SerialTreeLearner(const Config* config);
  void Init(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetConfig(const Config* config) override;
  void SetBaggingData(const data_size_t* used_indices, data_size_t num_data) override;
  std::unique_ptr<Tree> Train(const score_t* gradients, const score_t* hessians, bool is_first_tree) override;
  std::unique_ptr<Tree> FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                          const score_t* gradients, const score_t* hessians) override;
  void AddPredictionToScore(const Tree* tree, double* out_score) const override;
  void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj, const double* score, data_size_t total_num_data,
                       const data_size_t* bag_indices, data_size_t bag_cnt) const override;
  std::vector<data_size_t> LeafIndices(int leaf) const override;
  std::string DeviceName() const override;
  // device_type=gpu with a host split policy: histograms are built by the HIP kernels
  void EnableDeviceHistograms() { want_device_hist_ = true; }
  // ... and, for the monotone intermediate / advanced policies, device-resident leaf histograms
  // with device split scans (HistogramBackend::ScanSlots): the host keeps the tree, the row
  // partition and the constraint bookkeeping only
  void EnableDeviceScans() { want_device_scans_ = true; }
  // bound of the live leaf histograms in MB when histogram_pool_size is unset (<= 0: none)
  void SetHistPoolBudgetMB(double mb) { pool_budget_mb_ = mb; }

 protected:
  // ---- hooks for the parallel learners
  virtual void BeforeTrain();
  virtual bool BeforeFindBestSplit(const Tree* tree, int left_leaf, int right_leaf);
  virtual void FindBestSplits(const Tree* tree);
  virtual void ConstructHistograms(bool use_subtract);
  virtual void FindBestSplitsFromHistograms(const Tree* tree, bool use_subtract);
  virtual void Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf);
  virtual data_size_t GlobalCount(int leaf) const { return leaf < 0 ? 0 : leaf_count_global_[leaf]; }
  // parallel learners: agree on the best split of the two current leaves
  virtual void SyncBestSplits() {}

  void BuildHistogram(const data_size_t* idx, data_size_t n, double* hist) const;
  void BuildHistogramRowWise(const data_size_t* idx, data_size_t n, double* hist) const;
  void BuildHistogramColWise(const data_size_t* idx, data_size_t n, double* hist) const;
  void ComputeLeafSums(const data_size_t* idx, data_size_t n, double* sg, double* sh) const;
  SplitInfo BestSplitForFeature(const double* group_hist, int f, const LeafStat& leaf, double parent_output,
                                const LeafBounds& bounds, const ThresholdBounds* tb, bool* splittable) const;
  double ParentOutput(const Tree* tree, const LeafStat& ls) const;
  double MonotonePenalty(const Tree* tree, int leaf) const;
  void InitLeafStat(LeafStat* ls, int leaf, double sg, double sh, double output);
  SplitParams MakeParams() const;
  std::vector<double>& HistOf(int leaf);
  void ResetHistPool();
  void SetupPolicies();
  void SetupResident();
  int ForceSplits(Tree* tree, int* left_leaf, int* right_leaf);
  void CheckForcedSplitFeatures() const;
  // BestSplitForFeature + CEGB deduction + monotone split penalty (ComputeBestSplitForFeature)
  SplitInfo ScoreFeature(const Tree* tree, const double* group_hist, int f, const LeafStat& leaf,
                         double parent_output, bool* splittable);
  // intermediate monotone: rescan a leaf whose constraint interval tightened
  void RecomputeBestSplit(const Tree* tree, int leaf);
  // quant_train_renew_leaf: leaf outputs from the true (unquantized) gradient sums
  void RenewQuantizedLeaves(Tree* tree) const;
  // device-resident mode (EnableDeviceScans): scans of `leaves` on the device, ScoreFeature's
  // CEGB / monotone-penalty adjustments on the host; out[r * F + f], splittable the same
  void DeviceScanLeaves(const Tree* tree, const std::vector<const LeafStat*>& leaves, const std::vector<double>& po,
                        const std::vector<const std::vector<char>*>& enable, std::vector<SplitInfo>* out,
                        std::vector<uint8_t>* splittable);

  const Config* config_;
  const Dataset* train_data_ = nullptr;
  data_size_t num_data_ = 0;
  int num_features_ = 0;
  const score_t* gradients_ = nullptr;
  const score_t* hessians_ = nullptr;
  bool is_constant_hessian_ = false;
  DataPartition partition_;
  ColSampler col_sampler_;
  std::vector<SplitInfo> best_split_per_leaf_;
  std::vector<std::vector<double>> hist_;            // per leaf, 2*num_total_bin
  mutable std::vector<std::vector<double>> tls_hist_;  // per-thread partial histograms (BuildHistogram)
  // TrainingShareStates analogue (reference dataset.cpp TestMultiThreadingMethod,
  // train_share_states.h): histogram threads split the leaf's ROWS (per-thread histograms,
  // folded) or the feature GROUPS (over a column-major copy of the dense groups). Both sum
  // the same row chunks and fold the chunk partials in the same order, so the choice never
  // changes a model; force_col_wise / force_row_wise pin it, otherwise the first root
  // histogram times both and keeps the faster.
  enum class HistLayout { kAuto, kRowWise, kColWise };
  mutable HistLayout hist_layout_ = HistLayout::kAuto;
  mutable std::vector<uint8_t> colbins_;  // dense groups column-major (col-wise only)
  // histogram_pool_size: at most hist_cap_ leaf histograms live at once; the one
  // produced longest ago is dropped first (reference HistogramPool LRU,
  // feature_histogram.hpp:1367-1594)
  int hist_cap_ = 0, hist_live_ = 0;
  double pool_budget_mb_ = 0.0;
  int64_t hist_clock_ = 0;
  std::vector<int64_t> hist_stamp_;
  std::vector<std::vector<char>> splittable_;        // per leaf, per feature
  std::vector<LeafBounds> bounds_;                   // monotone basic constraints
  std::vector<data_size_t> leaf_count_global_;
  LeafStat smaller_, larger_;
  int parent_leaf_ = -1;  // leaf whose histogram became the larger child's (subtraction source)
  bool has_parent_hist_ = false;
  Random extra_rand_;
  bool use_monotone_ = false;
  bool intermediate_monotone_ = false;
  MonotoneLeafConstraints mono_;
  std::unique_ptr<CegbPenalty> cegb_;
  GradientQuantizer quantizer_;
  std::vector<score_t> qgrad_, qhess_;
  const score_t* true_gradients_ = nullptr;
  const score_t* true_hessians_ = nullptr;
  std::unique_ptr<device::HistogramBackend> hist_backend_;
  bool want_device_hist_ = false;
  bool want_device_scans_ = false;
  bool resident_ = false;           // leaf histograms live in device slots (dslot_)
  std::vector<int> dslot_;          // leaf -> device histogram slot
  std::vector<char> dvalid_;        // leaf's slot holds its histogram
  device::HistogramBackend::ScanBatch scan_batch_;
  std::string forced_json_;
  bool forced_rescored_ = false;  // ForceSplits left every leaf's best split current
  std::vector<Random> extra_rands_;
  // parallel learners
  std::vector<char> feature_mask_;       // features scanned by this rank
  int hist_begin_ = 0, hist_end_ = -1;   // histogram entries (bins) owned by this rank; -1 = all
  bool global_counts_from_split_ = false;
};

// ---------------------------------------------------------------------------
template <typename F, typename P>
data_size_t DataPartition::Split(int leaf, int right_leaf, F go_left, P prefetch) {
  const data_size_t b = begin_[leaf], n = count_[leaf];
  data_size_t* src = indices_.data() + b;
  data_size_t* dst = tmp_.data() + b;
  // Stable partition in one predicate pass (reference data_partition.hpp:104-160 splits the
  // leaf into per-thread blocks the same way): each block writes its lefts forward from its
  // start and its rights backward from its end in `dst`, then every block copies its lefts
  // and (re-reversed) rights to their final offsets in `src`.
  constexpr data_size_t kMinPerBlock = 8192;
  const int nblk = static_cast<int>(std::max<data_size_t>(1, std::min<data_size_t>(
      static_cast<data_size_t>(omp_get_max_threads()), n / kMinPerBlock)));
  const data_size_t per = (n + nblk - 1) / nblk;
  std::vector<data_size_t> lcnt(nblk + 1, 0), rcnt(nblk + 1, 0);
#pragma omp parallel for schedule(static, 1) num_threads(nblk) if (nblk > 1)
  for (int t = 0; t < nblk; ++t) {
    const data_size_t s0 = std::min(n, t * per), s1 = std::min(n, s0 + per);
    data_size_t l = s0, r = s1;
    constexpr data_size_t kPf = 32;
    for (data_size_t i = s0; i < s1; ++i) {
      if (i + kPf < s1) prefetch(src[i + kPf]);
      const data_size_t row = src[i];
      if (go_left(row)) dst[l++] = row;
      else dst[--r] = row;
    }
    lcnt[t + 1] = l - s0;
    rcnt[t + 1] = s1 - r;
  }
  for (int t = 0; t < nblk; ++t) {
    lcnt[t + 1] += lcnt[t];
    rcnt[t + 1] += rcnt[t];
  }
  const data_size_t nl = lcnt[nblk];
#pragma omp parallel for schedule(static, 1) num_threads(nblk) if (nblk > 1)
  for (int t = 0; t < nblk; ++t) {
    const data_size_t s0 = std::min(n, t * per), s1 = std::min(n, s0 + per);
    const data_size_t nlt = lcnt[t + 1] - lcnt[t], nrt = rcnt[t + 1] - rcnt[t];
    std::copy(dst + s0, dst + s0 + nlt, src + lcnt[t]);
    data_size_t* rout = src + nl + rcnt[t];
    for (data_size_t k = 0; k < nrt; ++k) rout[k] = dst[s1 - 1 - k];
  }
  if (right_leaf >= static_cast<int>(begin_.size())) {
    begin_.resize(right_leaf + 1, 0);
    count_.resize(right_leaf + 1, 0);
  }
  count_[leaf] = nl;
  begin_[right_leaf] = b + nl;
  count_[right_leaf] = n - nl;
  return nl;
}

}  // namespace lgap
