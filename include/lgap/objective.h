// Objective functions (reference: include/LightGBM/objective_function.h:18-126,
// factory src/objective/objective_function.cpp:20-150). Each objective has a
// host implementation (the correctness oracle / CPU path); the hot ones also
// expose a device kernel via DeviceObjective (device/objectives.hip).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/dataset.h"
#include "lgap/meta.h"
#include "lgap/pointwise.h"
#include "lgap/pointwise_metric.h"

namespace lgap {

// How the device learner obtains gradients for an objective.
enum class DeviceGradKind : int { kHostOnly = 0, kPointwise = 1, kSoftmax = 2, kOVA = 3, kLambdarank = 4, kXendcg = 5 };

class ObjectiveFunction {
 public:
  virtual ~ObjectiveFunction() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  // score: [num_class x num_data] class-major; gradients/hessians same layout.
  virtual void GetGradients(const double* score, score_t* gradients, score_t* hessians) const = 0;
  virtual const char* GetName() const = 0;
  virtual std::string ToString() const { return GetName(); }
  virtual bool IsConstantHessian() const { return false; }
  virtual bool IsRenewTreeOutput() const { return false; }
  // Leaf value renewal from residuals (L1 / quantile / MAPE): rows are data indices of the leaf.
  virtual double RenewTreeOutput(double ori_output, const double* score, const data_size_t* rows,
                                 data_size_t n) const {
    (void)score; (void)rows; (void)n;
    return ori_output;
  }
  virtual double BoostFromScore(int /*class_id*/) const { return 0.0; }
  virtual bool ClassNeedTrain(int /*class_id*/) const { return true; }
  virtual bool SkipEmptyClass() const { return false; }
  virtual int NumModelPerIteration() const { return 1; }
  virtual int NumPredictOneRow() const { return 1; }
  virtual bool NeedAccuratePrediction() const { return true; }
  virtual void ConvertOutput(const double* input, double* output) const { output[0] = input[0]; }
  virtual data_size_t NumPositiveData() const { return 0; }
  virtual bool IsRanking() const { return false; }
  virtual DeviceGradKind device_kind() const { return DeviceGradKind::kHostOnly; }
  // pointwise objectives: formula parameters, (possibly transformed) labels, MAPE label weights
  virtual const PointwiseParams* pointwise() const { return nullptr; }
  // per-class pointwise parameters (multiclassova: class k's binary objective)
  virtual const PointwiseParams* pointwise_class(int k) const { return k == 0 ? pointwise() : nullptr; }
  virtual const label_t* effective_label() const { return nullptr; }
  virtual const label_t* aux_weight() const { return nullptr; }
  virtual int num_class() const { return 1; }
  virtual double sigmoid() const { return 1.0; }

  static std::unique_ptr<ObjectiveFunction> Create(const std::string& type, const Config& config);
  // From the "objective=" line of a saved model.
  static std::unique_ptr<ObjectiveFunction> CreateFromString(const std::string& str);
};

// Percentile helpers shared by objectives and metrics.
// Lookup tables of a lambdarank objective, consumed by the device gradient kernel.
struct LambdarankTables {
  int target, k, norm;
  double sigmoid, gap_weight, tmin, tmax, tfactor;
  const std::vector<double>* label_gain;
  const std::vector<double>* inv_max_dcg;
  const std::vector<double>* inv_max_bdcg;
  const std::vector<double>* table;
  double pos_lr, pos_reg;  // position-bias Newton step (learning_rate, lambdarank_position_bias_regularization)
};
bool GetLambdarankTables(const ObjectiveFunction* obj, LambdarankTables* out);
// objective_seed of a rank_xendcg objective (its per-query Random streams start at seed + q)
bool GetXendcgSeed(const ObjectiveFunction* obj, int* seed);
// output transform of a pointwise objective as a PwOutput code (lgap/pointwise_metric.h);
// false for objectives whose ConvertOutput is not pointwise
bool PointwiseOutputTransform(const ObjectiveFunction* obj, int* output, double* sigmoid);

double Percentile(std::vector<double> v, double alpha);
double WeightedPercentile(const std::vector<double>& v, const std::vector<double>& w, double alpha);

}  // namespace lgap
