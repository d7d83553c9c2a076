// Evaluation metrics (reference: include/LightGBM/metric.h:24-149,
// factory src/metric/metric.cpp:20-139) and the DCG helper used by ranking
// objectives/metrics, including the fork's binarized ideal DCG.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/meta.h"
#include "lgap/objective.h"
#include "lgap/pointwise_metric.h"
#include "lgap/rank_metric_spec.h"

namespace lgap {

class Metric {
 public:
  virtual ~Metric() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  virtual const std::vector<std::string>& GetName() const = 0;
  // +1 if bigger is better, -1 otherwise
  virtual double factor_to_bigger_better() const = 0;
  // score: raw scores [num_class x num_data] class-major
  virtual std::vector<double> Eval(const double* score, const ObjectiveFunction* objective) const = 0;
  static std::unique_ptr<Metric> Create(const std::string& type, const Config& config);
  // Pointwise metrics that a device learner can evaluate from its device-resident
  // score: fill the row-loss description (objective output transform included)
  // and turn the device's weighted loss sum into the metric value.
  virtual bool DevicePointwise(const ObjectiveFunction*, PwMetricParams*) const { return false; }
  virtual std::vector<double> FinishSum(double) const { return {}; }
  // Ranking / AUC metrics a device learner evaluates from its device-resident score: the
  // description (lgap/rank_metric_spec.h), and the values from the device's raw sums.
  virtual bool DeviceRankSpec(RankMetricSpec*) const { return false; }
  virtual std::vector<double> FinishRank(const std::vector<double>&) const { return {}; }
  // Multiclass metrics over the device-resident class-major score (lgap/pointwise_metric.h)
  virtual bool DeviceMulti(const ObjectiveFunction*, MultiMetricParams*) const { return false; }
  // auc_mu: the per-pair accumulators the device computes (lgap/rank_metric_spec.h) -> value
  virtual bool DeviceAucMu(AucMuSpec*) const { return false; }
  virtual std::vector<double> FinishAucMu(const std::vector<double>&) const { return {}; }
};

class DCGCalculator {
 public:
  static void DefaultEvalAt(std::vector<int>* eval_at);
  static void DefaultLabelGain(std::vector<double>* label_gain);
  static void Init(const std::vector<double>& label_gain);
  static double CalMaxDCGAtK(data_size_t k, const label_t* label, data_size_t n);
  // fork: ideal DCG when every relevant (label > 0) document has gain 1
  static double CalMaxBDCGAtK(data_size_t k, const label_t* label, data_size_t n);
  static void CalMaxDCG(const std::vector<data_size_t>& ks, const label_t* label, data_size_t n, std::vector<double>* out);
  static void CalDCG(const std::vector<data_size_t>& ks, const label_t* label, const double* score, data_size_t n,
                     std::vector<double>* out);
  static void CheckLabel(const label_t* label, data_size_t n);
  static void CheckMetadata(const Metadata& md, data_size_t num_queries);
  static double GetDiscount(data_size_t k) { return discount_[k]; }
  static const std::vector<double>& label_gain() { return label_gain_; }
  static constexpr data_size_t kMaxPosition = 10000;

 private:
  static std::vector<double> label_gain_;
  static std::vector<double> discount_;
};

}  // namespace lgap
