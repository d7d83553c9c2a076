// Boosting: GBDT loop, DART, random forest, sample strategies (bagging /
// GOSS), model text IO, prediction and feature importance.
// Reference: include/LightGBM/boosting.h:27-321, src/boosting/*.
#pragma once

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/metric.h"
#include "lgap/objective.h"
#include "lgap/random.h"
#include "lgap/tree.h"
#include "lgap/tree_learner.h"

namespace lgap {

// Bagging / GOSS row sampling (bagging.hpp:14-296, goss.hpp:18-170).
class SampleStrategy {
 public:
  SampleStrategy(const Config* cfg, const Dataset* data, const ObjectiveFunction* obj, int num_tree_per_iter);
  void ResetConfig(const Config* cfg);
  // returns true if a new bag was drawn this iteration
  bool Bagging(int iter, score_t* gradients, score_t* hessians);
  // The same decision as Bagging() for a learner that draws the sample on the
  // device: returns a DeviceSamplePlan (kSampleHost when only the host can).
  int PlanDevice(int iter);
  bool is_hessian_change() const { return goss_; }
  bool active() const { return bag_cnt_ < num_data_; }
  data_size_t bag_cnt() const { return bag_cnt_; }
  const std::vector<data_size_t>& bag_indices() const { return bag_; }  // [bag | out-of-bag]
  bool by_query() const { return by_query_; }

 private:
  data_size_t BagBlock(data_size_t start, data_size_t cnt, data_size_t* out, bool balanced);
  data_size_t GossBlock(data_size_t start, data_size_t cnt, data_size_t* out, score_t* g, score_t* h, uint32_t seed);
  const Config* cfg_;
  const Dataset* data_;
  const ObjectiveFunction* obj_;
  int ntpi_;
  data_size_t num_data_;
  bool goss_ = false;
  bool balanced_ = false;
  bool by_query_ = false;
  bool need_rebag_ = false;
  data_size_t bag_cnt_;
  std::vector<data_size_t> bag_;
  std::vector<Random> rands_;
};

class PredictionEarlyStop {
 public:
  PredictionEarlyStop(const std::string& type, int round_period, double margin_threshold);
  bool Check(const double* pred, int n) const;
  int round_period() const { return round_period_; }
  bool enabled() const { return type_ != 0; }

 private:
  int type_ = 0;  // 0 none, 1 binary, 2 multiclass
  int round_period_ = 1 << 30;
  double margin_ = 0.0;
};

class GBDT {
 public:
  GBDT() = default;
  virtual ~GBDT() = default;

  virtual void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
                    const std::vector<const Metric*>& training_metrics);
  void AddValidDataset(const Dataset* valid_data, const std::vector<const Metric*>& valid_metrics);
  void ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                         const std::vector<const Metric*>& training_metrics);
  virtual void ResetConfig(const Config* config);

  // returns true when training cannot continue (no split possible)
  virtual bool TrainOneIter(const score_t* gradients, const score_t* hessians);
  void Train(int snapshot_freq, const std::string& model_output_path);
  virtual void RollbackOneIter();
  bool EvalAndCheckEarlyStopping();
  std::string OutputMetric(int iter);
  std::vector<double> GetEvalAt(int data_idx);
  std::vector<std::string> GetEvalNames() const;
  virtual const double* GetTrainingScore(int64_t* out_len);
  int64_t GetNumPredictAt(int data_idx) const;
  void GetPredictAt(int data_idx, double* out, int64_t* out_len);
  void RefitTree(const std::vector<std::vector<int>>& leaf_preds);
  void MergeFrom(const GBDT* other);
  void ShuffleModels(int start_iter, int end_iter);

  // prediction on raw feature rows
  void PredictRaw(const double* features, double* out, const PredictionEarlyStop* es) const;
  void Predict(const double* features, double* out, const PredictionEarlyStop* es) const;
  void PredictLeafIndex(const double* features, double* out) const;
  void PredictContrib(const double* features, double* out) const;
  void PredictRawByMap(const std::unordered_map<int, double>& f, double* out) const;
  void InitPredict(int start_iteration, int num_iteration, bool is_pred_contrib);
  int NumPredictOneRow(int start_iteration, int num_iteration, bool is_pred_leaf, bool is_pred_contrib) const;

  // model IO
  std::string SaveModelToString(int start_iteration, int num_iteration, int importance_type) const;
  bool SaveModelToFile(int start_iteration, int num_iteration, int importance_type, const std::string& filename) const;
  bool LoadModelFromString(const char* buffer, size_t len);
  std::string DumpModel(int start_iteration, int num_iteration, int importance_type) const;
  std::string ModelToIfElse(int num_iteration) const;
  std::vector<double> FeatureImportance(int num_iteration, int importance_type) const;

  // accessors
  virtual const char* SubModelName() const { return "tree"; }
  int NumberOfTotalModel() const { return static_cast<int>(models_.size()); }
  int NumModelPerIteration() const { return num_tree_per_iteration_; }
  int NumberOfClasses() const { return num_class_; }
  // prediction early stopping applies only when this is false (reference gbdt.h:229-235)
  virtual bool NeedAccuratePrediction() const { return objective() == nullptr || objective()->NeedAccuratePrediction(); }
  int GetCurrentIteration() const { return static_cast<int>(models_.size()) / std::max(1, num_tree_per_iteration_); }
  int MaxFeatureIdx() const { return max_feature_idx_; }
  const std::string& parser_config() const { return parser_config_str_; }
  const std::vector<std::string>& FeatureNames() const { return feature_names_; }
  std::vector<std::string>& MutableFeatureNames() { return feature_names_; }
  double GetLeafValue(int tree, int leaf) const { return models_[tree]->LeafOutput(leaf); }
  void SetLeafValue(int tree, int leaf, double v) { models_[tree]->SetLeafOutput(leaf, v); }
  const Tree* GetTree(int i) const { return models_[i].get(); }
  Tree* MutableTree(int i) { return models_[i].get(); }
  void AddTree(std::unique_ptr<Tree> t) { models_.push_back(std::move(t)); }
  bool average_output() const { return average_output_; }
  const ObjectiveFunction* objective() const { return objective_; }
  void set_objective_for_prediction(std::unique_ptr<ObjectiveFunction> o) { loaded_objective_ = std::move(o); objective_ = loaded_objective_.get(); }
  const std::string& loaded_parameter() const { return loaded_parameter_; }
  TreeLearner* tree_learner() { return learner_.get(); }
  // Gradients / hessians of the last boosting round (downloaded from the device in device mode).
  void GetGradients(std::vector<score_t>* g, std::vector<score_t>* h) const {
    if (device_mode_ && learner_) {
      learner_->DeviceGetGradients(g, h);
    } else {
      *g = gradients_;
      *h = hessians_;
    }
  }
  const Config* config() const { return config_; }
  int best_iteration() const { return best_iter_; }
  std::string parser_config_str_;

 protected:
  virtual double BoostFromAverage(int class_id, bool update_scorer);
  void Boosting();
  void UpdateScore(const Tree* tree, int cur_tree_id);
  void AddScoreConstant(double v, int cur_tree_id);
  void SyncTrainScoreFromDevice();
  void ResetGradientBuffers();
  std::vector<double> EvalTraining(const Metric* m, const double** score);
  // DART drops trees when the training score is first read in an iteration: keep that read
  virtual bool DeviceMetricsAllowed() const { return true; }
  std::vector<double> EvalOne(const Metric* m, const double* score) const;

  const Config* config_ = nullptr;
  const Dataset* train_data_ = nullptr;
  const ObjectiveFunction* objective_ = nullptr;
  std::unique_ptr<ObjectiveFunction> loaded_objective_;
  std::unique_ptr<TreeLearner> learner_;
  std::unique_ptr<SampleStrategy> sampler_;
  std::vector<const Metric*> training_metrics_;
  std::vector<const Dataset*> valid_data_;
  std::vector<std::vector<const Metric*>> valid_metrics_;
  std::vector<std::vector<double>> valid_score_;
  std::vector<int> valid_dev_;     // device handle of each validation set (-1: scored on the host)
  std::vector<char> valid_stale_;  // host copy behind the device score
  const double* ValidScore(size_t d);
  std::vector<double> EvalValid(size_t d, const Metric* m);
  std::vector<double> train_score_;   // [num_tree_per_iteration x num_data]
  bool train_score_stale_ = false;    // device owns the score and the host copy is out of date
  bool device_mode_ = false;
  std::vector<score_t> gradients_, hessians_;
  std::vector<std::unique_ptr<Tree>> models_;
  std::vector<bool> class_need_train_;
  int num_class_ = 1;
  int num_tree_per_iteration_ = 1;
  int num_iteration_for_pred_ = 0;
  int start_iteration_for_pred_ = 0;
  int max_feature_idx_ = 0;
  int label_idx_ = 0;
  data_size_t num_data_ = 0;
  int iter_ = 0;
  int num_init_models_ = 0;  // leading trees merged from an init model (MergeFrom)
  double shrinkage_rate_ = 0.1;
  bool average_output_ = false;
  bool has_init_score_ = false;
  int early_stopping_round_ = 0;
  double es_min_delta_ = 0.0;
  std::vector<std::vector<double>> best_score_;
  std::vector<std::vector<int>> best_iter_vec_;
  std::vector<std::vector<std::string>> best_msg_;
  int best_iter_ = 0;
  std::vector<std::string> feature_names_;
  std::vector<std::string> feature_infos_;
  std::vector<int8_t> monotone_constraints_;
  std::string loaded_parameter_;
};

class DART : public GBDT {
 public:
  void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
            const std::vector<const Metric*>& training_metrics) override;
  bool TrainOneIter(const score_t* gradients, const score_t* hessians) override;
  const double* GetTrainingScore(int64_t* out_len) override;
  bool DeviceMetricsAllowed() const override { return false; }
  const char* SubModelName() const override { return "tree"; }

 private:
  bool updated_cur_iter_ = false;
  void DroppingTrees();
  void Normalize();
  Random random_for_drop_;
  std::vector<double> tree_weight_;
  double sum_weight_ = 0.0;
  std::vector<int> drop_index_;
};

class RF : public GBDT {
 public:
  void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
            const std::vector<const Metric*>& training_metrics) override;
  bool TrainOneIter(const score_t* gradients, const score_t* hessians) override;
  void RollbackOneIter() override;
  bool NeedAccuratePrediction() const override { return true; }  // rf.hpp:224: no early stopping

 private:
  std::vector<double> init_scores_;
  std::vector<score_t> tmp_grad_, tmp_hess_;
};

std::unique_ptr<GBDT> CreateBoosting(const std::string& type, const char* model_filename);

}  // namespace lgap
