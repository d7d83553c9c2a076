// GBDT training loop, DART and RF (reference: src/boosting/gbdt.cpp:27-881,
// dart.hpp, rf.hpp). In device mode (HIP learner owning the score) gradients,
// scores and the tree build stay in HBM; the host only receives each finished
// tree (tens of KB) and syncs the score when a metric or the user asks for it.
#include "lgap/boosting.h"

#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <thread>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/network.h"

namespace lgap {

namespace {
double AutomaticInitScore(const ObjectiveFunction* obj, int class_id) {
  double v = obj ? obj->BoostFromScore(class_id) : 0.0;
  if (Network::num_machines() > 1) v = Network::GlobalSyncUpByMean(v);
  return v;
}
std::unique_ptr<Tree> ConstantTree(double v, data_size_t n, bool linear) {
  auto t = std::make_unique<Tree>(2);
  t->AsConstantTree(v, n, linear);
  return t;
}
}  // namespace

void GBDT::Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
                const std::vector<const Metric*>& training_metrics) {
  config_ = config;
  train_data_ = train_data;
  if (train_data != nullptr && !train_data->parser_config().empty()) parser_config_str_ = train_data->parser_config();
  objective_ = objective;
  iter_ = 0;
  num_class_ = config->num_class;
  num_tree_per_iteration_ = objective ? objective->NumModelPerIteration() : num_class_;
  shrinkage_rate_ = config->learning_rate;
  early_stopping_round_ = config->early_stopping_round;
  es_min_delta_ = config->early_stopping_min_delta;
  average_output_ = config->boosting == "rf";
  num_data_ = train_data->num_data();
  max_feature_idx_ = train_data->num_total_features() - 1;
  feature_names_ = train_data->feature_names();
  feature_infos_ = train_data->feature_infos();
  monotone_constraints_ = config->monotone_constraints;
  learner_ = TreeLearner::Create(config->tree_learner, config->device_type, config->linear_tree, config, train_data);
  learner_->Init(train_data, objective && objective->IsConstantHessian());
  device_mode_ = learner_->OwnsScore();
  sampler_ = std::make_unique<SampleStrategy>(config, train_data, objective, num_tree_per_iteration_);
  training_metrics_ = training_metrics;
  ResetGradientBuffers();
  // initial training score
  const size_t total = static_cast<size_t>(num_tree_per_iteration_) * num_data_;
  train_score_.assign(total, 0.0);
  const auto& md = train_data->metadata();
  has_init_score_ = md.init_score() != nullptr;
  if (has_init_score_) {
    if (md.init_score_size() != total) {
      Log::Fatal("Number of class for initial score error");
    }
    std::copy(md.init_score(), md.init_score() + total, train_score_.begin());
  }
  class_need_train_.assign(num_tree_per_iteration_, true);
  if (objective_ && objective_->SkipEmptyClass()) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) class_need_train_[k] = objective_->ClassNeedTrain(k);
  }
  if (device_mode_) learner_->DeviceInitScore(train_score_, num_tree_per_iteration_);
  best_score_.clear();
  best_iter_vec_.clear();
  best_msg_.clear();
}

void GBDT::ResetGradientBuffers() {
  const size_t total = static_cast<size_t>(num_tree_per_iteration_) * num_data_;
  gradients_.assign(total, 0.0f);
  hessians_.assign(total, 0.0f);
}

void GBDT::AddValidDataset(const Dataset* valid, const std::vector<const Metric*>& metrics) {
  if (!train_data_->CheckAlign(*valid)) {
    Log::Fatal("Cannot add validation data, since it has different bin mappers with training data");
  }
  valid_data_.push_back(valid);
  const size_t total = static_cast<size_t>(num_tree_per_iteration_) * valid->num_data();
  std::vector<double> s(total, 0.0);
  const auto& md = valid->metadata();
  if (md.init_score() != nullptr && md.init_score_size() == total) std::copy(md.init_score(), md.init_score() + total, s.begin());
  // models trained by this booster before the set was added; merged init-model trees reach
  // the set through its init score (reference gbdt.cpp AddValidDataset loops over iter_ only)
  for (size_t i = static_cast<size_t>(num_init_models_); i < models_.size(); ++i) {
    const int k = static_cast<int>(i % num_tree_per_iteration_);
    models_[i]->AddPredictionToScore(*valid, valid->num_data(), s.data() + static_cast<size_t>(k) * valid->num_data());
  }
  valid_score_.push_back(std::move(s));
  // device mode: the set's packed rows and score live on the device; trees are added and
  // pointwise metrics evaluated there, the host copy is refreshed only when read
  int dev = -1;
  const char* ev = std::getenv("LGAP_DEVICE_VALID");  // "0": score validation sets on the host
  if (device_mode_ && DeviceMetricsAllowed() && !(ev && std::strcmp(ev, "0") == 0)) {
    dev = learner_->DeviceAddValidSet(valid, valid_score_.back());
  }
  valid_dev_.push_back(dev);
  valid_stale_.push_back(0);
  valid_metrics_.push_back(metrics);
  best_score_.emplace_back(metrics.size(), kMinScore);
  best_iter_vec_.emplace_back(metrics.size(), 0);
  best_msg_.emplace_back(metrics.size());
}

void GBDT::ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                             const std::vector<const Metric*>& training_metrics) {
  auto models = std::move(models_);
  models_.clear();
  const int iter = iter_;
  // Init builds a new tree learner: validation sets scored on the old learner's device come
  // back to the host first (their device handles die with it), and early-stopping state
  // survives the reset
  for (size_t d = 0; d < valid_dev_.size(); ++d) (void)ValidScore(d);
  auto best_score = std::move(best_score_);
  auto best_iter = std::move(best_iter_vec_);
  auto best_msg = std::move(best_msg_);
  Init(config_, train_data, objective, training_metrics);
  best_score_ = std::move(best_score);
  best_iter_vec_ = std::move(best_iter);
  best_msg_ = std::move(best_msg);
  models_ = std::move(models);
  iter_ = iter;
  // recompute training score from the existing trees
  for (size_t i = 0; i < models_.size(); ++i) {
    const int k = static_cast<int>(i % num_tree_per_iteration_);
    models_[i]->AddPredictionToScore(*train_data_, num_data_, train_score_.data() + static_cast<size_t>(k) * num_data_);
  }
  if (device_mode_) learner_->DeviceInitScore(train_score_, num_tree_per_iteration_);
  // register the validation sets with the new learner (device scoring where it applies)
  const char* ev = std::getenv("LGAP_DEVICE_VALID");
  const bool dev_ok = device_mode_ && DeviceMetricsAllowed() && !(ev && std::strcmp(ev, "0") == 0);
  for (size_t d = 0; d < valid_dev_.size(); ++d) {
    valid_dev_[d] = dev_ok ? learner_->DeviceAddValidSet(valid_data_[d], valid_score_[d]) : -1;
    valid_stale_[d] = 0;
  }
}

void GBDT::ResetConfig(const Config* config) {
  config_ = config;
  shrinkage_rate_ = config->learning_rate;
  early_stopping_round_ = config->early_stopping_round;
  es_min_delta_ = config->early_stopping_min_delta;
  if (learner_) learner_->ResetConfig(config);
  if (sampler_) sampler_->ResetConfig(config);
}

void GBDT::SyncTrainScoreFromDevice() {
  if (device_mode_ && train_score_stale_) {
    learner_->DeviceGetScore(&train_score_);
    train_score_stale_ = false;
  }
}

const double* GBDT::ValidScore(size_t d) {
  if (valid_dev_[d] >= 0 && valid_stale_[d]) {
    learner_->DeviceGetValidScore(valid_dev_[d], &valid_score_[d]);
    valid_stale_[d] = 0;
  }
  return valid_score_[d].data();
}

const double* GBDT::GetTrainingScore(int64_t* out_len) {
  SyncTrainScoreFromDevice();
  *out_len = static_cast<int64_t>(train_score_.size());
  return train_score_.data();
}

void GBDT::AddScoreConstant(double v, int k) {
  if (device_mode_) {
    learner_->DeviceAddConstant(v, k);
    train_score_stale_ = true;
  } else {
    double* s = train_score_.data() + static_cast<size_t>(k) * num_data_;
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) s[i] += v;
  }
  for (size_t d = 0; d < valid_score_.size(); ++d) {
    if (valid_dev_[d] >= 0) {
      learner_->DeviceValidAddConstant(valid_dev_[d], v, k);
      valid_stale_[d] = 1;
      continue;
    }
    const data_size_t n = valid_data_[d]->num_data();
    double* s = valid_score_[d].data() + static_cast<size_t>(k) * n;
    for (data_size_t i = 0; i < n; ++i) s[i] += v;
  }
}

double GBDT::BoostFromAverage(int k, bool update) {
  if (models_.empty() && !has_init_score_ && objective_ != nullptr) {
    if (config_->boost_from_average || train_data_->num_features() == 0) {
      const double init = AutomaticInitScore(objective_, k);
      if (std::fabs(init) > kEpsilon) {
        if (update) AddScoreConstant(init, k);
        Log::Info("Start training from score %lf", init);
        return init;
      }
    } else if (std::string(objective_->GetName()) == "regression_l1" || std::string(objective_->GetName()) == "quantile" ||
               std::string(objective_->GetName()) == "mape") {
      Log::Warning("Disabling boost_from_average in %s may cause the slow convergence", objective_->GetName());
    }
  }
  return 0.0;
}

void GBDT::Boosting() {
  if (objective_ == nullptr) Log::Fatal("No objective function provided");
  if (device_mode_ && learner_->SupportsDeviceGradients(objective_)) {
    ScopedTimer t("GBDT::Boosting(device)");
    learner_->DeviceComputeGradients(objective_);
    return;
  }
  ScopedTimer t("GBDT::Boosting");
  int64_t len;
  const double* score = GetTrainingScore(&len);
  objective_->GetGradients(score, gradients_.data(), hessians_.data());
  if (device_mode_) learner_->DeviceSetGradients(gradients_.data(), hessians_.data(), num_tree_per_iteration_);
}

void GBDT::UpdateScore(const Tree* tree, int k) {
  ScopedTimer t("GBDT::UpdateScore");
  if (device_mode_) {
    learner_->DeviceAddTreeToScore(tree, k);
    train_score_stale_ = true;
  } else {
    double* s = train_score_.data() + static_cast<size_t>(k) * num_data_;
    if (sampler_->active()) {
      learner_->AddPredictionToScore(tree, s);
      const auto& bag = sampler_->bag_indices();
      const data_size_t bc = sampler_->bag_cnt();
      if (num_data_ - bc > 0) tree->AddPredictionToScore(*train_data_, bag.data() + bc, num_data_ - bc, s);
    } else {
      learner_->AddPredictionToScore(tree, s);
    }
  }
  for (size_t d = 0; d < valid_score_.size(); ++d) {
    if (valid_dev_[d] >= 0) {
      learner_->DeviceAddTreeToValid(valid_dev_[d], tree, k);
      valid_stale_[d] = 1;
      continue;
    }
    const data_size_t n = valid_data_[d]->num_data();
    tree->AddPredictionToScore(*valid_data_[d], n, valid_score_[d].data() + static_cast<size_t>(k) * n);
  }
}

// Fault injection for failure-detection tests (no reference counterpart: the
// reference has none). LGAP_FAULT_INJECT="<rank>:<iter>:<mode>"
// makes machine <rank> fail when it starts boosting iteration <iter>:
// mode "exit" ends the process at once (no cleanup, sockets / communicator
// dropped), "hang" stops it in place so its peers' timeouts / the collective
// watchdog must notice, "throw" raises a fatal error through the normal path.
// LGAP_FAULT_INJECT=xgmi is the device learner's: its in-kernel xGMI exchange never signals.
static void MaybeInjectFault(int iter) {
  static const char* spec = std::getenv("LGAP_FAULT_INJECT");
  if (spec == nullptr || *spec == '\0' || std::strcmp(spec, "xgmi") == 0) return;
  int rank = -1, at = -1;
  char mode[16] = {0};
  if (std::sscanf(spec, "%d:%d:%15s", &rank, &at, mode) != 3) Log::Fatal("Malformed LGAP_FAULT_INJECT=%s", spec);
  if (iter != at || rank != std::max(0, Network::rank())) return;
  if (std::strcmp(mode, "exit") == 0) {
    std::fprintf(stderr, "[fault-inject] rank %d exits at iteration %d\n", rank, iter);
    std::fflush(stderr);
    std::_Exit(3);
  } else if (std::strcmp(mode, "hang") == 0) {
    std::fprintf(stderr, "[fault-inject] rank %d hangs at iteration %d\n", rank, iter);
    std::fflush(stderr);
    for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
  } else {
    Log::Fatal("[fault-inject] rank %d fails at iteration %d", rank, iter);
  }
}

bool GBDT::TrainOneIter(const score_t* gradients, const score_t* hessians) {
  ScopedTimer timer("GBDT::TrainOneIter");
  MaybeInjectFault(iter_);
  std::vector<double> init_scores(num_tree_per_iteration_, 0.0);
  const bool custom = gradients != nullptr && hessians != nullptr;
  if (!custom) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) init_scores[k] = BoostFromAverage(k, true);
    Boosting();
  } else {
    if (objective_ != nullptr) Log::Fatal("Cannot use custom gradients with a built-in objective (set objective=custom)");
    std::copy(gradients, gradients + gradients_.size(), gradients_.begin());
    std::copy(hessians, hessians + hessians_.size(), hessians_.begin());
    if (device_mode_) learner_->DeviceSetGradients(gradients_.data(), hessians_.data(), num_tree_per_iteration_);
  }
  // bagging / GOSS: drawn on the device from the device-resident gradients when the
  // learner can; otherwise on the host (GOSS then round-trips the gradients)
  int plan = kSampleHost;
  if (device_mode_ && config_->device_sampling && learner_->SupportsDeviceSampling()) plan = sampler_->PlanDevice(iter_);
  if (plan != kSampleHost) {
    learner_->DeviceSample(plan, iter_);
  } else {
    const bool need_host_grads = sampler_->is_hessian_change() && device_mode_ && !custom &&
                                 learner_->SupportsDeviceGradients(objective_);
    if (need_host_grads) learner_->DeviceGetGradients(&gradients_, &hessians_);
    const bool rebag = sampler_->Bagging(iter_, gradients_.data(), hessians_.data());
    if (rebag) {
      if (sampler_->active()) learner_->SetBaggingData(sampler_->bag_indices().data(), sampler_->bag_cnt());
      else learner_->SetBaggingData(nullptr, num_data_);
    }
    if (sampler_->is_hessian_change() && device_mode_ && sampler_->active()) {
      learner_->DeviceSetGradients(gradients_.data(), hessians_.data(), num_tree_per_iteration_);
    }
  }
  bool should_continue = false;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t off = static_cast<size_t>(k) * num_data_;
    std::unique_ptr<Tree> tree = std::make_unique<Tree>(2);
    if (class_need_train_[k] && train_data_->num_features() > 0) {
      const bool first = models_.size() < static_cast<size_t>(num_tree_per_iteration_);
      if (device_mode_) tree = learner_->DeviceTrain(k, first);
      else tree = learner_->Train(gradients_.data() + off, hessians_.data() + off, first);
    }
    if (tree->num_leaves() > 1) {
      should_continue = true;
      if (objective_ && objective_->IsRenewTreeOutput() &&
          !(device_mode_ && learner_->DeviceRenewTreeOutput(tree.get(), objective_, k))) {
        int64_t len;
        const double* score = GetTrainingScore(&len);
        learner_->RenewTreeOutput(tree.get(), objective_, score + off, num_data_, sampler_->bag_indices().data(),
                                  sampler_->bag_cnt());
      }
      tree->Shrinkage(shrinkage_rate_);
      UpdateScore(tree.get(), k);
      if (std::fabs(init_scores[k]) > kEpsilon) tree->AddBias(init_scores[k]);
    } else {
      if (models_.size() < static_cast<size_t>(num_tree_per_iteration_)) {
        if (objective_ && !config_->boost_from_average && !has_init_score_) {
          init_scores[k] = AutomaticInitScore(objective_, k);
          AddScoreConstant(init_scores[k], k);
        }
        tree = ConstantTree(init_scores[k], num_data_, config_->linear_tree);
      } else {
        tree = ConstantTree(0.0, num_data_, config_->linear_tree);
      }
    }
    models_.push_back(std::move(tree));
  }
  if (!should_continue) {
    Log::Warning("Stopped training because there are no more leaves that meet the split requirements");
    if (models_.size() > static_cast<size_t>(num_tree_per_iteration_)) {
      for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
    }
    return true;
  }
  ++iter_;
  return false;
}

void GBDT::RollbackOneIter() {
  if (iter_ <= 0) return;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t t = models_.size() - num_tree_per_iteration_ + k;
    models_[t]->Shrinkage(-1.0);
    if (device_mode_) {
      learner_->DeviceAddTreeToScore(models_[t].get(), k);
      train_score_stale_ = true;
    } else {
      models_[t]->AddPredictionToScore(*train_data_, num_data_, train_score_.data() + static_cast<size_t>(k) * num_data_);
    }
    for (size_t d = 0; d < valid_score_.size(); ++d) {
      if (valid_dev_[d] >= 0) {
        learner_->DeviceAddTreeToValid(valid_dev_[d], models_[t].get(), k);
        valid_stale_[d] = 1;
        continue;
      }
      const data_size_t n = valid_data_[d]->num_data();
      models_[t]->AddPredictionToScore(*valid_data_[d], n, valid_score_[d].data() + static_cast<size_t>(k) * n);
    }
  }
  for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
  --iter_;
}

std::vector<double> GBDT::EvalOne(const Metric* m, const double* score) const { return m->Eval(score, objective_); }

// Training metrics: pointwise, AUC / average precision and query metrics are evaluated where
// the score lives (the device learner's HBM copy, no N-double download); everything else reads
// the training score on the host. `*score` is fetched lazily and reused.
std::vector<double> GBDT::EvalTraining(const Metric* m, const double** score) {
  PwMetricParams p;
  const char* off = std::getenv("LGAP_DEVICE_METRICS");  // "0": always evaluate on the host (A/B, tests)
  const bool allow = off == nullptr || std::strcmp(off, "0") != 0;
  if (allow && device_mode_ && num_tree_per_iteration_ == 1 && DeviceMetricsAllowed() &&
      m->DevicePointwise(objective_, &p)) {
    double sum = 0.0;
    if (learner_->DeviceEvalPointwise(p, 0, &sum)) return m->FinishSum(sum);
  }
  // ranking / AUC metrics: sorted on the device, only their sums come back
  RankMetricSpec rs;
  if (allow && device_mode_ && num_tree_per_iteration_ == 1 && DeviceMetricsAllowed() && m->DeviceRankSpec(&rs)) {
    std::vector<double> raw;
    if (learner_->DeviceEvalRank(-1, rs, 0, &raw)) return m->FinishRank(raw);
  }
  // multiclass logloss / error: the class-major device score, only the loss sum comes back
  MultiMetricParams mp;
  if (allow && device_mode_ && num_tree_per_iteration_ > 1 && DeviceMetricsAllowed() && m->DeviceMulti(objective_, &mp)) {
    double sum = 0.0;
    if (learner_->DeviceEvalMulti(-1, mp, &sum)) return m->FinishSum(sum);
  }
  AucMuSpec am;
  if (allow && device_mode_ && num_tree_per_iteration_ > 1 && DeviceMetricsAllowed() && m->DeviceAucMu(&am)) {
    std::vector<double> s;
    if (learner_->DeviceEvalAucMu(-1, am, &s)) return m->FinishAucMu(s);
  }
  if (*score == nullptr) {
    int64_t len;
    *score = GetTrainingScore(&len);
  }
  return EvalOne(m, *score);
}

// Validation metrics: pointwise, AUC / average precision and the query metrics (NDCG, MAP,
// precision@k), multiclass logloss / error and auc_mu on the device-resident validation score; the rest on the
// host copy, refreshed once when stale.
std::vector<double> GBDT::EvalValid(size_t d, const Metric* m) {
  PwMetricParams p;
  if (valid_dev_[d] >= 0 && num_tree_per_iteration_ == 1 && m->DevicePointwise(objective_, &p)) {
    double sum = 0.0;
    if (learner_->DeviceEvalPointwiseValid(valid_dev_[d], p, 0, &sum)) return m->FinishSum(sum);
  }
  RankMetricSpec rs;
  const char* off = std::getenv("LGAP_DEVICE_METRICS");
  const bool allow = off == nullptr || std::strcmp(off, "0") != 0;
  if (allow && valid_dev_[d] >= 0 && num_tree_per_iteration_ == 1 && m->DeviceRankSpec(&rs)) {
    std::vector<double> raw;
    if (learner_->DeviceEvalRank(valid_dev_[d], rs, 0, &raw)) return m->FinishRank(raw);
  }
  MultiMetricParams mp;
  if (allow && valid_dev_[d] >= 0 && num_tree_per_iteration_ > 1 && m->DeviceMulti(objective_, &mp)) {
    double sum = 0.0;
    if (learner_->DeviceEvalMulti(valid_dev_[d], mp, &sum)) return m->FinishSum(sum);
  }
  AucMuSpec am;
  if (allow && valid_dev_[d] >= 0 && num_tree_per_iteration_ > 1 && m->DeviceAucMu(&am)) {
    std::vector<double> s;
    if (learner_->DeviceEvalAucMu(valid_dev_[d], am, &s)) return m->FinishAucMu(s);
  }
  return EvalOne(m, ValidScore(d));
}

std::vector<std::string> GBDT::GetEvalNames() const {
  std::vector<std::string> out;
  for (auto* m : training_metrics_) for (auto& n : m->GetName()) out.push_back(n);
  return out;
}

std::string GBDT::OutputMetric(int iter) {
  const bool need_output = (iter % config_->metric_freq) == 0;
  std::string ret;
  std::stringstream msg;
  std::vector<std::pair<size_t, size_t>> improved;
  if (need_output && !training_metrics_.empty()) {
    const double* score = nullptr;
    for (auto* m : training_metrics_) {
      auto names = m->GetName();
      auto vals = EvalTraining(m, &score);
      for (size_t k = 0; k < names.size(); ++k) {
        std::stringstream line;
        line << "Iteration:" << iter << ", training " << names[k] << " : " << vals[k];
        Log::Info("%s", line.str().c_str());
        if (early_stopping_round_ > 0) msg << line.str() << '\n';
      }
    }
  }
  if (need_output || early_stopping_round_ > 0) {
    for (size_t i = 0; i < valid_metrics_.size(); ++i) {
      for (size_t j = 0; j < valid_metrics_[i].size(); ++j) {
        auto vals = EvalValid(i, valid_metrics_[i][j]);
        auto names = valid_metrics_[i][j]->GetName();
        for (size_t k = 0; k < names.size(); ++k) {
          std::stringstream line;
          line << "Iteration:" << iter << ", valid_" << i + 1 << " " << names[k] << " : " << vals[k];
          if (need_output) Log::Info("%s", line.str().c_str());
          if (early_stopping_round_ > 0) msg << line.str() << '\n';
        }
        if (config_->first_metric_only && j > 0) continue;
        if (ret.empty() && early_stopping_round_ > 0) {
          const double cur = valid_metrics_[i][j]->factor_to_bigger_better() * vals.back();
          if (cur - best_score_[i][j] > es_min_delta_) {
            best_score_[i][j] = cur;
            best_iter_vec_[i][j] = iter;
            improved.emplace_back(i, j);
          } else if (iter - best_iter_vec_[i][j] >= early_stopping_round_) {
            ret = best_msg_[i][j];
          }
        }
      }
    }
  }
  for (auto& p : improved) best_msg_[p.first][p.second] = msg.str();
  return ret;
}

bool GBDT::EvalAndCheckEarlyStopping() {
  auto best = OutputMetric(iter_);
  if (best.empty()) return false;
  Log::Info("Early stopping at iteration %d, the best iteration round is %d", iter_, iter_ - early_stopping_round_);
  Log::Info("Output of best iteration round:\n%s", best.c_str());
  best_iter_ = iter_ - early_stopping_round_;
  for (int i = 0; i < early_stopping_round_ * num_tree_per_iteration_; ++i) models_.pop_back();
  return true;
}

std::vector<double> GBDT::GetEvalAt(int data_idx) {
  std::vector<double> ret;
  if (data_idx == 0) {
    const double* score = nullptr;
    for (auto* m : training_metrics_) for (double v : EvalTraining(m, &score)) ret.push_back(v);
  } else {
    const size_t i = static_cast<size_t>(data_idx - 1);
    if (i >= valid_score_.size()) Log::Fatal("Invalid data index %d", data_idx);
    for (auto* m : valid_metrics_[i]) for (double v : EvalValid(i, m)) ret.push_back(v);
  }
  return ret;
}

int64_t GBDT::GetNumPredictAt(int data_idx) const {
  const data_size_t n = data_idx == 0 ? num_data_ : valid_data_[data_idx - 1]->num_data();
  return static_cast<int64_t>(n) * num_class_;
}

void GBDT::GetPredictAt(int data_idx, double* out, int64_t* out_len) {
  const double* raw;
  data_size_t n;
  if (data_idx == 0) {
    int64_t len;
    raw = GetTrainingScore(&len);
    n = num_data_;
  } else {
    raw = ValidScore(static_cast<size_t>(data_idx - 1));
    n = valid_data_[data_idx - 1]->num_data();
  }
  *out_len = static_cast<int64_t>(n) * num_class_;
  if (objective_ != nullptr) {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) {
      std::vector<double> in(num_tree_per_iteration_), o(num_class_);
      for (int k = 0; k < num_tree_per_iteration_; ++k) in[k] = raw[static_cast<size_t>(k) * n + i];
      objective_->ConvertOutput(in.data(), o.data());
      for (int k = 0; k < num_class_; ++k) out[static_cast<size_t>(k) * n + i] = o[k];
    }
  } else {
    std::copy(raw, raw + *out_len, out);
  }
}

void GBDT::Train(int snapshot_freq, const std::string& model_output_path) {
  bool finished = false;
  auto start = std::chrono::steady_clock::now();
  for (int iter = 0; iter < config_->num_iterations && !finished; ++iter) {
    finished = TrainOneIter(nullptr, nullptr);
    if (!finished) finished = EvalAndCheckEarlyStopping();
    auto now = std::chrono::steady_clock::now();
    Log::Info("%f seconds elapsed, finished iteration %d", std::chrono::duration<double>(now - start).count(), iter + 1);
    if (snapshot_freq > 0 && (iter + 1) % snapshot_freq == 0) {
      SaveModelToFile(0, -1, config_->saved_feature_importance_type,
                      model_output_path + ".snapshot_iter_" + std::to_string(iter + 1));
    }
  }
}

void GBDT::RefitTree(const std::vector<std::vector<int>>& leaf_preds) {
  if (leaf_preds.empty()) return;
  const int num_iter = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  std::vector<int> leaf_pred(num_data_);
  for (int it = 0; it < num_iter; ++it) {
    Boosting();
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      const int m = it * num_tree_per_iteration_ + k;
      for (data_size_t i = 0; i < num_data_; ++i) leaf_pred[i] = leaf_preds[i][m];
      const size_t off = static_cast<size_t>(k) * num_data_;
      if (device_mode_) {
        // device-resident gradients and score (Boosting() left the gradients on the device)
        auto nt = learner_->DeviceFitByExistingTree(models_[m].get(), leaf_pred, k);
        if (nt) {
          models_[m] = std::move(nt);
          train_score_stale_ = true;
          continue;
        }
        learner_->DeviceGetGradients(&gradients_, &hessians_);
      }
      auto nt = learner_->FitByExistingTree(models_[m].get(), leaf_pred, gradients_.data() + off, hessians_.data() + off);
      // The refit booster's training score starts from the init score alone (MergeFrom adds
      // no score), so each refit tree is added on top of the refit trees before it
      // (reference gbdt.cpp RefitTree:293-294, AddScore of the new tree only).
      if (device_mode_) {
        learner_->DeviceAddTreeToScore(nt.get(), k);
        train_score_stale_ = true;
      } else {
        learner_->AddPredictionToScore(nt.get(), train_score_.data() + off);
      }
      models_[m] = std::move(nt);
    }
  }
}

void GBDT::MergeFrom(const GBDT* other) {
  std::vector<std::unique_ptr<Tree>> merged;
  for (auto& t : other->models_) merged.push_back(std::make_unique<Tree>(*t));
  for (auto& t : models_) merged.push_back(std::move(t));
  models_ = std::move(merged);
  num_init_models_ += static_cast<int>(other->models_.size());
}

void GBDT::ShuffleModels(int start_iter, int end_iter) {
  const int total = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  start_iter = std::max(0, start_iter);
  if (end_iter <= 0) end_iter = total;
  end_iter = std::min(total, end_iter);
  std::vector<int> idx;
  for (int i = start_iter; i < end_iter; ++i) idx.push_back(i);
  Random r(config_ ? config_->seed : 0);
  for (int i = 0; i + 1 < static_cast<int>(idx.size()); ++i) {
    int j = r.NextShort(i + 1, static_cast<int>(idx.size()));
    std::swap(idx[i], idx[j]);
  }
  std::vector<std::unique_ptr<Tree>> nm;
  for (int i = 0; i < start_iter * num_tree_per_iteration_; ++i) nm.push_back(std::move(models_[i]));
  for (int it : idx)
    for (int k = 0; k < num_tree_per_iteration_; ++k) nm.push_back(std::move(models_[it * num_tree_per_iteration_ + k]));
  for (size_t i = static_cast<size_t>(end_iter) * num_tree_per_iteration_; i < models_.size(); ++i) nm.push_back(std::move(models_[i]));
  models_ = std::move(nm);
}

// ============================================================================
// DART (dart.hpp)
void DART::Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
                const std::vector<const Metric*>& training_metrics) {
  GBDT::Init(config, train_data, objective, training_metrics);
  random_for_drop_ = Random(config->drop_seed);
  sum_weight_ = 0.0;
  tree_weight_.clear();
  if (device_mode_) {
    // DART rewrites old trees' contributions every iteration: keep the score on host.
    device_mode_ = false;
  }
}

void DART::DroppingTrees() {
  drop_index_.clear();
  // only this session's iterations are dropped; merged init-model trees stay fixed
  // (dart.hpp DroppingTrees: num_init_iteration_ + i)
  const int init_iter = num_init_models_ / num_tree_per_iteration_;
  const bool skip = random_for_drop_.NextFloat() < config_->skip_drop;
  if (!skip) {
    double rate = config_->drop_rate;
    if (!config_->uniform_drop) {
      const double inv_avg = static_cast<double>(tree_weight_.size()) / sum_weight_;
      if (config_->max_drop > 0) rate = std::min(rate, config_->max_drop * inv_avg / sum_weight_);
      const int n = std::min(iter_, static_cast<int>(tree_weight_.size()));
      for (int i = 0; i < n; ++i) {
        if (random_for_drop_.NextFloat() < rate * tree_weight_[i] * inv_avg) {
          drop_index_.push_back(init_iter + i);
          if (drop_index_.size() >= static_cast<size_t>(config_->max_drop)) break;
        }
      }
    } else {
      if (config_->max_drop > 0) rate = std::min(rate, config_->max_drop / static_cast<double>(iter_));
      for (int i = 0; i < iter_; ++i) {
        if (random_for_drop_.NextFloat() < rate) {
          drop_index_.push_back(init_iter + i);
          if (drop_index_.size() >= static_cast<size_t>(config_->max_drop)) break;
        }
      }
    }
  }
  for (int i : drop_index_) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      Tree* t = models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k].get();
      t->Shrinkage(-1.0);
      t->AddPredictionToScore(*train_data_, num_data_, train_score_.data() + static_cast<size_t>(k) * num_data_);
    }
  }
  if (!config_->xgboost_dart_mode) {
    shrinkage_rate_ = config_->learning_rate / (1.0 + static_cast<double>(drop_index_.size()));
  } else {
    shrinkage_rate_ = drop_index_.empty() ? config_->learning_rate
                                          : config_->learning_rate / (config_->learning_rate + drop_index_.size());
  }
}

void DART::Normalize() {
  const double k = static_cast<double>(drop_index_.size());
  for (int i : drop_index_) {
    for (int c = 0; c < num_tree_per_iteration_; ++c) {
      Tree* t = models_[static_cast<size_t>(i) * num_tree_per_iteration_ + c].get();
      if (!config_->xgboost_dart_mode) {
        t->Shrinkage(1.0 / (k + 1.0));
      } else {
        t->Shrinkage(shrinkage_rate_);
      }
      for (size_t d = 0; d < valid_score_.size(); ++d) {
        const data_size_t n = valid_data_[d]->num_data();
        t->AddPredictionToScore(*valid_data_[d], n, valid_score_[d].data() + static_cast<size_t>(c) * n);
      }
      t->Shrinkage(!config_->xgboost_dart_mode ? -k : -k / config_->learning_rate);
      t->AddPredictionToScore(*train_data_, num_data_, train_score_.data() + static_cast<size_t>(c) * num_data_);
    }
    if (!config_->uniform_drop) {
      const int w = i - num_init_models_ / num_tree_per_iteration_;
      if (!config_->xgboost_dart_mode) {
        sum_weight_ -= tree_weight_[w] * (1.0 / (k + 1.0));
        tree_weight_[w] *= (k / (k + 1.0));
      } else {
        sum_weight_ -= tree_weight_[w] * (1.0 / (k + config_->learning_rate));
        tree_weight_[w] *= (k / (k + config_->learning_rate));
      }
    }
  }
}

const double* DART::GetTrainingScore(int64_t* out_len) {
  // dropping happens when the score is first read in an iteration (dart.hpp GetTrainingScore)
  if (!updated_cur_iter_) {
    DroppingTrees();
    updated_cur_iter_ = true;
  }
  return GBDT::GetTrainingScore(out_len);
}

bool DART::TrainOneIter(const score_t* gradients, const score_t* hessians) {
  if (gradients != nullptr && !updated_cur_iter_) {
    int64_t len;
    GetTrainingScore(&len);
  }
  const bool ret = GBDT::TrainOneIter(gradients, hessians);
  updated_cur_iter_ = false;
  if (ret) return ret;
  Normalize();
  if (!config_->uniform_drop) {
    tree_weight_.push_back(shrinkage_rate_);
    sum_weight_ += shrinkage_rate_;
  }
  return false;
}

// ============================================================================
// RF (rf.hpp)
void RF::Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
              const std::vector<const Metric*>& training_metrics) {
  if (config->data_sample_strategy == "bagging") {
    if (!((config->bagging_freq > 0 && config->bagging_fraction < 1.0 && config->bagging_fraction > 0.0) ||
          (config->feature_fraction < 1.0 && config->feature_fraction > 0.0))) {
      Log::Fatal("Cannot use RF without bagging or feature subsampling");
    }
  }
  GBDT::Init(config, train_data, objective, training_metrics);
  device_mode_ = false;  // RF averages scores on host
  average_output_ = true;
  shrinkage_rate_ = 1.0;
  if (objective_ == nullptr) Log::Fatal("RF mode do not support custom objective function, please use built-in objectives.");
  init_scores_.assign(num_tree_per_iteration_, 0.0);
  for (int k = 0; k < num_tree_per_iteration_; ++k) init_scores_[k] = BoostFromAverage(k, false);
  std::vector<double> tmp(static_cast<size_t>(num_data_) * num_tree_per_iteration_);
  for (int k = 0; k < num_tree_per_iteration_; ++k)
    std::fill(tmp.begin() + static_cast<size_t>(k) * num_data_, tmp.begin() + static_cast<size_t>(k + 1) * num_data_,
              init_scores_[k]);
  objective_->GetGradients(tmp.data(), gradients_.data(), hessians_.data());
}

bool RF::TrainOneIter(const score_t*, const score_t*) {
  const bool rebag = sampler_->Bagging(iter_, gradients_.data(), hessians_.data());
  if (rebag) {
    if (sampler_->active()) learner_->SetBaggingData(sampler_->bag_indices().data(), sampler_->bag_cnt());
    else learner_->SetBaggingData(nullptr, num_data_);
  }
  auto mult = [&](int k, double v) {
    double* s = train_score_.data() + static_cast<size_t>(k) * num_data_;
    for (data_size_t i = 0; i < num_data_; ++i) s[i] *= v;
    for (size_t d = 0; d < valid_score_.size(); ++d) {
      const data_size_t n = valid_data_[d]->num_data();
      double* vs = valid_score_[d].data() + static_cast<size_t>(k) * n;
      for (data_size_t i = 0; i < n; ++i) vs[i] *= v;
    }
  };
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t off = static_cast<size_t>(k) * num_data_;
    std::unique_ptr<Tree> tree = std::make_unique<Tree>(2);
    if (class_need_train_[k]) tree = learner_->Train(gradients_.data() + off, hessians_.data() + off, false);
    if (tree->num_leaves() > 1) {
      if (objective_->IsRenewTreeOutput()) {
        std::vector<double> pred(num_data_, init_scores_[k]);
        learner_->RenewTreeOutput(tree.get(), objective_, pred.data(), num_data_, sampler_->bag_indices().data(),
                                  sampler_->bag_cnt());
      }
      if (std::fabs(init_scores_[k]) > kEpsilon) tree->AddBias(init_scores_[k]);
      mult(k, iter_);
      UpdateScore(tree.get(), k);
      mult(k, 1.0 / (iter_ + 1));
    } else if (models_.size() < static_cast<size_t>(num_tree_per_iteration_)) {
      double out = 0.0;
      if (!class_need_train_[k]) out = objective_->BoostFromScore(k);
      tree = ConstantTree(out, num_data_, config_->linear_tree);
      mult(k, iter_);
      UpdateScore(tree.get(), k);
      mult(k, 1.0 / (iter_ + 1));
    }
    models_.push_back(std::move(tree));
  }
  ++iter_;
  return false;
}

void RF::RollbackOneIter() {
  if (iter_ <= 0) return;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t t = static_cast<size_t>(iter_ - 1) * num_tree_per_iteration_ + k;
    models_[t]->Shrinkage(-1.0);
    double* s = train_score_.data() + static_cast<size_t>(k) * num_data_;
    for (data_size_t i = 0; i < num_data_; ++i) s[i] *= iter_;
    models_[t]->AddPredictionToScore(*train_data_, num_data_, s);
    if (iter_ > 1)
      for (data_size_t i = 0; i < num_data_; ++i) s[i] /= (iter_ - 1);
  }
  for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
  --iter_;
}

std::unique_ptr<GBDT> CreateBoosting(const std::string& type, const char* model_filename) {
  std::unique_ptr<GBDT> b;
  if (type == "gbdt" || type == "goss") b = std::make_unique<GBDT>();
  else if (type == "dart") b = std::make_unique<DART>();
  else if (type == "rf") b = std::make_unique<RF>();
  else Log::Fatal("Unknown boosting type %s", type.c_str());
  if (model_filename != nullptr && model_filename[0] != '\0') {
    std::ifstream in(model_filename, std::ios::binary);
    if (!in) Log::Fatal("Model file %s is not available", model_filename);
    std::string s((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    if (!b->LoadModelFromString(s.data(), s.size())) Log::Fatal("Failed to load model from %s", model_filename);
  }
  return b;
}

}  // namespace lgap
