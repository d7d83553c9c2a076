// Tree learner interface (reference include/LightGBM/tree_learner.h:27-114,
// factory src/treelearner/tree_learner.cpp:15-57). Host learners: serial
// (correctness oracle), feature/data/voting parallel over Network. Device
// learners (HIP, MI355X) implement the same interface and additionally own the
// device-resident score / gradients (OwnsScore() == true).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/objective.h"
#include "lgap/rank_metric_spec.h"
#include "lgap/tree.h"

namespace lgap {

// What the boosting loop asks a device learner to do with the row sample of
// this iteration (SampleStrategy::PlanDevice).
enum DeviceSamplePlan {
  kSampleHost = -2,      // the host SampleStrategy draws it
  kSampleAll = -1,       // train on all rows
  kSampleKeep = 0,       // keep the current bag
  kSampleBag = 1,        // uniform bagging (bagging_fraction)
  kSampleBalanced = 2,   // balanced bagging (pos/neg_bagging_fraction)
  kSampleGoss = 3,       // GOSS (top_rate / other_rate)
  kSampleBagQuery = 4,   // bagging by query (whole queries kept or dropped)
};

class TreeLearner {
 public:
  virtual ~TreeLearner() = default;
  virtual void Init(const Dataset* train_data, bool is_constant_hessian) = 0;
  virtual void ResetConfig(const Config* config) = 0;
  virtual void ResetIsConstantHessian(bool) {}
  // Bagging: subset of row indices used to grow the next tree (nullptr = all rows).
  virtual void SetBaggingData(const data_size_t* used_indices, data_size_t num_data) = 0;
  virtual std::unique_ptr<Tree> Train(const score_t* gradients, const score_t* hessians, bool is_first_tree) = 0;
  // Refit leaf values of an existing tree structure (uses the leaf partition of leaf_pred).
  virtual std::unique_ptr<Tree> FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                                  const score_t* gradients, const score_t* hessians) = 0;
  // Adds tree outputs to the training score using the learner's leaf partition.
  virtual void AddPredictionToScore(const Tree* tree, double* out_score) const = 0;
  // L1 / quantile / MAPE leaf renewal (serial_tree_learner.cpp:924-962).
  virtual void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj, const double* score,
                               data_size_t total_num_data, const data_size_t* bag_indices, data_size_t bag_cnt) const = 0;
  // Row indices of a leaf of the last trained tree (in original numbering).
  virtual std::vector<data_size_t> LeafIndices(int leaf) const = 0;

  // ---- device-resident boosting (HIP learners)
  virtual bool OwnsScore() const { return false; }
  virtual bool SupportsDeviceGradients(const ObjectiveFunction*) const { return false; }
  virtual void DeviceInitScore(const std::vector<double>& host_score, int num_tree_per_iter) { (void)host_score; (void)num_tree_per_iter; }
  virtual void DeviceComputeGradients(const ObjectiveFunction*) {}
  virtual void DeviceSetGradients(const score_t*, const score_t*, int) {}
  virtual std::unique_ptr<Tree> DeviceTrain(int class_id, bool is_first_tree) { (void)class_id; (void)is_first_tree; return nullptr; }
  virtual void DeviceAddTreeToScore(const Tree*, int class_id) { (void)class_id; }
  // training metric from the device-resident score of class k (false: evaluate on the host)
  virtual bool DeviceEvalPointwise(const PwMetricParams&, int /*k*/, double* /*sum*/) { return false; }
  virtual void DeviceAddConstant(double, int class_id) { (void)class_id; }
  virtual void DeviceGetScore(std::vector<double>*) const {}
  virtual void DeviceGetGradients(std::vector<score_t>*, std::vector<score_t>*) const {}
  // Row sampling drawn on the device from the device-resident gradients.
  // L1 / quantile / MAPE leaf renewal from the device-resident score and partition
  // (false: not handled, the host renews from a downloaded score)
  virtual bool DeviceRenewTreeOutput(Tree*, const ObjectiveFunction*, int /*class_id*/) { return false; }
  // Refit of an existing tree from the device-resident gradients of class k; also updates the
  // device score by the change of the leaf outputs (nullptr: not handled)
  virtual std::unique_ptr<Tree> DeviceFitByExistingTree(const Tree*, const std::vector<int>& /*leaf_pred*/,
                                                        int /*class_id*/) {
    return nullptr;
  }
  // Validation sets scored on the device (training-layout packed rows): returns a handle, or
  // -1 when the learner keeps validation scores on the host.
  virtual int DeviceAddValidSet(const Dataset*, const std::vector<double>& /*init_score*/) { return -1; }
  virtual void DeviceAddTreeToValid(int /*id*/, const Tree*, int /*class_id*/) {}
  virtual void DeviceValidAddConstant(int /*id*/, double, int /*class_id*/) {}
  virtual void DeviceGetValidScore(int /*id*/, std::vector<double>*) {}
  virtual void DeviceSetValidScore(int /*id*/, const std::vector<double>&) {}
  virtual bool DeviceEvalPointwiseValid(int /*id*/, const PwMetricParams&, int /*k*/, double* /*sum*/) { return false; }
  // Ranking / AUC metric of the training set (id < 0) or device validation set `id`, class k,
  // on the device score: raw sums for Metric::FinishRank (false: evaluate on the host)
  virtual bool DeviceEvalRank(int /*id*/, const RankMetricSpec&, int /*k*/, std::vector<double>* /*out*/) { return false; }
  // multiclass metric over the class-major device score of the training set (id < 0) or a
  // device validation set: the weighted loss sum
  virtual bool DeviceEvalMulti(int /*id*/, const MultiMetricParams&, double* /*sum*/) { return false; }
  // auc_mu per-pair accumulators S_ij (pairs i < j in row-major order) on the device score
  virtual bool DeviceEvalAucMu(int /*id*/, const AucMuSpec&, std::vector<double>* /*out*/) { return false; }
  virtual bool SupportsDeviceSampling() const { return false; }
  virtual void DeviceSample(int plan, int iter) { (void)plan; (void)iter; }
  virtual std::string DeviceName() const { return "cpu"; }

  // `train` (optional) lets the factory size the device learner's per-leaf histograms
  // against histogram_pool_size / the device memory before choosing it.
  static std::unique_ptr<TreeLearner> Create(const std::string& learner_type, const std::string& device_type,
                                             bool linear_tree, const Config* config, const Dataset* train = nullptr);
};

}  // namespace lgap
