// Pointwise objectives (regression family, binary, cross-entropy), multiclass
// softmax / one-vs-all and the objective factory. Reference:
// src/objective/{regression,binary,multiclass,xentropy}_objective.hpp and
// objective_function.cpp:20-150. The per-row math lives in pointwise.h and is
// shared with the HIP gradient kernel.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <numeric>
#include <sstream>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/network.h"
#include "lgap/objective.h"

namespace lgap {

std::unique_ptr<ObjectiveFunction> CreateRankObjective(const std::string& type, const Config& config);
std::unique_ptr<ObjectiveFunction> CreateRankObjectiveFromString(const std::string& type,
                                                                 const std::vector<std::string>& strs);

// ---------------------------------------------------------------------------
double Percentile(std::vector<double> v, double alpha) {
  const data_size_t n = static_cast<data_size_t>(v.size());
  if (n <= 1) return n == 1 ? v[0] : 0.0;
  const double float_pos = static_cast<double>(n - 1) * (1.0 - alpha);
  const data_size_t pos = static_cast<data_size_t>(float_pos) + 1;
  if (pos < 1) return *std::max_element(v.begin(), v.end());
  if (pos >= n) return *std::min_element(v.begin(), v.end());
  const double bias = float_pos - (pos - 1);
  std::sort(v.begin(), v.end(), std::greater<double>());
  const double v1 = v[pos - 1], v2 = v[pos];
  return v1 - (v1 - v2) * bias;
}

double WeightedPercentile(const std::vector<double>& v, const std::vector<double>& w, double alpha) {
  const data_size_t n = static_cast<data_size_t>(v.size());
  if (n <= 1) return n == 1 ? v[0] : 0.0;
  std::vector<data_size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](data_size_t a, data_size_t b) { return v[a] < v[b]; });
  std::vector<double> cdf(n);
  cdf[0] = w[idx[0]];
  for (data_size_t i = 1; i < n; ++i) cdf[i] = cdf[i - 1] + w[idx[i]];
  const double thr = cdf[n - 1] * alpha;
  size_t pos = std::upper_bound(cdf.begin(), cdf.end(), thr) - cdf.begin();
  pos = std::min(pos, static_cast<size_t>(n - 1));
  if (pos == 0 || pos == static_cast<size_t>(n - 1)) return v[idx[pos]];
  const double v1 = v[idx[pos - 1]], v2 = v[idx[pos]];
  if (cdf[pos + 1] - cdf[pos] >= 1.0f) return (thr - cdf[pos]) / (cdf[pos + 1] - cdf[pos]) * (v2 - v1) + v1;
  return v2;
}

namespace {

// All pointwise objectives share one implementation parameterised by kind.
class PointwiseObjective : public ObjectiveFunction {
 public:
  PointwiseObjective(int kind, const Config& c) {
    p_.kind = kind;
    deterministic_ = c.deterministic;
    sqrt_ = c.reg_sqrt && kind == kPwL2;
    if (c.reg_sqrt && kind != kPwL2 && kind != kPwL1 && kind != kPwFair && kind != kPwQuantile && kind != kPwMape) {
      Log::Warning("Cannot use sqrt transform in %s Regression, will auto disable it", NameOf(kind));
    }
    if (c.reg_sqrt && (kind == kPwL1 || kind == kPwFair || kind == kPwQuantile || kind == kPwMape)) sqrt_ = true;
    p_.alpha = kind == kPwQuantile ? static_cast<double>(static_cast<float>(c.alpha)) : c.alpha;
    p_.fair_c = c.fair_c;
    p_.exp_max_delta = std::exp(c.poisson_max_delta_step);
    p_.rho = c.tweedie_variance_power;
    p_.sigmoid = c.sigmoid;
    if (kind == kPwQuantile && !(p_.alpha > 0 && p_.alpha < 1)) Log::Fatal("alpha should be in (0, 1) for quantile");
    if (kind == kPwBinary) {
      if (p_.sigmoid <= 0.0) Log::Fatal("Sigmoid parameter %f should be greater than zero", p_.sigmoid);
      is_unbalance_ = c.is_unbalance;
      scale_pos_weight_ = c.scale_pos_weight;
      if (is_unbalance_ && std::fabs(scale_pos_weight_ - 1.0) > 1e-6) {
        Log::Fatal("Cannot set is_unbalance and scale_pos_weight at the same time");
      }
    }
  }
  PointwiseObjective(int kind, const std::vector<std::string>& strs) {
    p_.kind = kind;
    for (auto& s : strs) {
      if (s == "sqrt") sqrt_ = true;
      auto kv = common::Split(s, ':');
      if (kv.size() == 2 && kv[0] == "sigmoid") p_.sigmoid = common::AtofOrDie(kv[1]);
    }
    if (kind == kPwBinary && p_.sigmoid <= 0.0) Log::Fatal("Sigmoid parameter should be greater than zero");
  }

  static const char* NameOf(int k) {
    static const char* n[] = {"regression", "regression_l1", "huber", "fair", "poisson", "quantile",
                              "mape", "gamma", "tweedie", "binary", "cross_entropy", "cross_entropy_lambda"};
    return n[k];
  }

  void Init(const Metadata& md, data_size_t num_data) override {
    num_data_ = num_data;
    label_ = md.label();
    weights_ = md.weights();
    if (sqrt_) {
      tlabel_.resize(num_data);
      for (data_size_t i = 0; i < num_data; ++i) tlabel_[i] = static_cast<label_t>(common::Sign(label_[i]) * std::sqrt(std::fabs(label_[i])));
      label_ = tlabel_.data();
    }
    const int k = p_.kind;
    if (k == kPwPoisson || k == kPwGamma || k == kPwTweedie) {
      double sum = 0.0;
      label_t mn = label_[0];
      for (data_size_t i = 0; i < num_data; ++i) {
        sum += label_[i];
        mn = std::min(mn, label_[i]);
      }
      if (mn < 0.0f) Log::Fatal("[%s]: at least one target label is negative", GetName());
      if (sum == 0.0) Log::Fatal("[%s]: sum of labels is zero", GetName());
    }
    if (k == kPwXent || k == kPwXentLambda) {
      for (data_size_t i = 0; i < num_data; ++i) {
        if (label_[i] < 0.0f || label_[i] > 1.0f) Log::Fatal("[%s]: label must be in [0, 1]", GetName());
      }
    }
    if (k == kPwMape) {
      aux_.resize(num_data);
      for (data_size_t i = 0; i < num_data; ++i) {
        aux_[i] = 1.0f / std::max(1.0f, std::fabs(label_[i]));
        if (weights_) aux_[i] *= weights_[i];
      }
    }
    if (k == kPwBinary) {
      data_size_t pos = 0, neg = 0;
      for (data_size_t i = 0; i < num_data; ++i) (label_[i] > 0 ? pos : neg)++;
      num_pos_ = pos;
      if (Network::num_machines() > 1) {
        pos = Network::GlobalSyncUpBySum(pos);
        neg = Network::GlobalSyncUpBySum(neg);
      }
      need_train_ = true;
      if (pos == 0 || neg == 0) {
        Log::Warning("Contains only one class");
        need_train_ = false;
      }
      Log::Info("Number of positive: %d, number of negative: %d", pos, neg);
      p_.label_weight_neg = 1.0;
      p_.label_weight_pos = 1.0;
      if (is_unbalance_ && pos > 0 && neg > 0) {
        if (pos > neg) p_.label_weight_neg = static_cast<double>(pos) / neg;
        else p_.label_weight_pos = static_cast<double>(neg) / pos;
      }
      p_.label_weight_pos *= scale_pos_weight_;
    }
  }

  void GetGradients(const double* score, score_t* g, score_t* h) const override {
    if (p_.kind == kPwBinary && !need_train_) return;
    const bool weighted = weights_ != nullptr;
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weighted ? weights_[i] : 1.0;
      PointwiseGradient(p_, score[i], label_[i], w, weighted, aux_.empty() ? 0.0 : aux_[i], &g[i], &h[i]);
    }
  }

  const char* GetName() const override { return NameOf(p_.kind); }
  std::string ToString() const override {
    std::stringstream ss;
    ss << GetName();
    if (p_.kind == kPwBinary) ss << " sigmoid:" << common::FormatG(p_.sigmoid);
    if (sqrt_) ss << " sqrt";
    return ss.str();
  }
  bool IsConstantHessian() const override {
    const int k = p_.kind;
    if (k == kPwMape) return true;
    if (k == kPwL2 || k == kPwL1 || k == kPwHuber || k == kPwQuantile) return weights_ == nullptr;
    return false;
  }
  bool IsRenewTreeOutput() const override { return p_.kind == kPwL1 || p_.kind == kPwQuantile || p_.kind == kPwMape; }

  double RenewTreeOutput(double, const double* score, const data_size_t* rows, data_size_t n) const override {
    std::vector<double> r(n);
    for (data_size_t i = 0; i < n; ++i) r[i] = static_cast<double>(label_[rows[i]]) - score[rows[i]];
    const double alpha = p_.kind == kPwQuantile ? p_.alpha : 0.5;
    if (p_.kind == kPwMape) {
      std::vector<double> w(n);
      for (data_size_t i = 0; i < n; ++i) w[i] = aux_[rows[i]];
      return WeightedPercentile(r, w, alpha);
    }
    if (weights_ == nullptr) return Percentile(r, alpha);
    std::vector<double> w(n);
    for (data_size_t i = 0; i < n; ++i) w[i] = weights_[rows[i]];
    return WeightedPercentile(r, w, alpha);
  }

  double BoostFromScore(int) const override {
    const int k = p_.kind;
    auto mean = [&](bool binary) {
      double suml = 0.0, sumw = 0.0;
      if (weights_) {
        for (data_size_t i = 0; i < num_data_; ++i) {
          suml += (binary ? (label_[i] > 0 ? 1.0 : 0.0) : static_cast<double>(label_[i])) * weights_[i];
          sumw += weights_[i];
        }
      } else {
        sumw = num_data_;
        for (data_size_t i = 0; i < num_data_; ++i) suml += binary ? (label_[i] > 0 ? 1.0 : 0.0) : label_[i];
      }
      if (Network::num_machines() > 1 && binary) {
        suml = Network::GlobalSyncUpBySum(suml);
        sumw = Network::GlobalSyncUpBySum(sumw);
      }
      return suml / sumw;
    };
    auto labels = [&]() { return std::vector<double>(label_, label_ + num_data_); };
    switch (k) {
      case kPwL2:
      case kPwHuber:
      case kPwFair:
        return mean(false);
      case kPwL1:
      case kPwQuantile: {
        const double a = k == kPwQuantile ? p_.alpha : 0.5;
        if (weights_) return WeightedPercentile(labels(), std::vector<double>(weights_, weights_ + num_data_), a);
        return Percentile(labels(), a);
      }
      case kPwMape:
        return WeightedPercentile(labels(), std::vector<double>(aux_.begin(), aux_.end()), 0.5);
      case kPwPoisson:
      case kPwGamma:
      case kPwTweedie: {
        const double m = mean(false);
        return m <= 0 ? -std::numeric_limits<double>::infinity() : std::log(m);
      }
      case kPwBinary: {
        double pavg = mean(true);
        pavg = std::min(pavg, 1.0 - kEpsilon);
        pavg = std::max(pavg, kEpsilon);
        const double init = std::log(pavg / (1.0 - pavg)) / p_.sigmoid;
        Log::Info("[binary:BoostFromScore]: pavg=%f -> initscore=%f", pavg, init);
        return init;
      }
      case kPwXent: {
        double pavg = mean(false);
        pavg = std::min(pavg, 1.0 - kEpsilon);
        pavg = std::max(pavg, kEpsilon);
        return std::log(pavg / (1.0 - pavg));
      }
      case kPwXentLambda:
        return std::log(std::expm1(mean(false)));
    }
    return 0.0;
  }

  bool ClassNeedTrain(int) const override { return p_.kind != kPwBinary || need_train_; }
  bool SkipEmptyClass() const override { return p_.kind == kPwBinary; }
  bool NeedAccuratePrediction() const override { return p_.kind != kPwBinary; }
  data_size_t NumPositiveData() const override { return num_pos_; }

  void ConvertOutput(const double* in, double* out) const override {
    switch (p_.kind) {
      case kPwPoisson:
      case kPwGamma:
      case kPwTweedie:
        out[0] = std::exp(in[0]);
        break;
      case kPwBinary:
        out[0] = 1.0f / (1.0f + std::exp(-p_.sigmoid * in[0]));
        break;
      case kPwXent:
        out[0] = 1.0f / (1.0f + std::exp(-in[0]));
        break;
      case kPwXentLambda:
        out[0] = std::log1p(std::exp(in[0]));
        break;
      default:
        out[0] = sqrt_ ? common::Sign(in[0]) * in[0] * in[0] : in[0];
    }
  }

  DeviceGradKind device_kind() const override { return DeviceGradKind::kPointwise; }
  const PointwiseParams* pointwise() const override { return &p_; }
  // ConvertOutput above as a PwOutput code (device metrics)
  int OutputTransform(double* sigmoid) const {
    *sigmoid = p_.sigmoid;
    switch (p_.kind) {
      case kPwPoisson:
      case kPwGamma:
      case kPwTweedie:
        return kOutExp;
      case kPwBinary:
        return kOutSigmoid;
      case kPwXent:
        *sigmoid = 1.0;
        return kOutSigmoid;
      case kPwXentLambda:
        return kOutLog1pExp;
      default:
        return sqrt_ ? kOutSignedSquare : kOutIdentity;
    }
  }
  const label_t* effective_label() const override { return label_; }
  const label_t* aux_weight() const override { return aux_.empty() ? nullptr : aux_.data(); }
  double sigmoid() const override { return p_.sigmoid; }

 private:
  PointwiseParams p_;
  bool sqrt_ = false;
  bool deterministic_ = false;
  bool is_unbalance_ = false;
  double scale_pos_weight_ = 1.0;
  bool need_train_ = true;
  data_size_t num_pos_ = 0;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  std::vector<label_t> tlabel_;
  std::vector<label_t> aux_;
};

class MulticlassSoftmax : public ObjectiveFunction {
 public:
  explicit MulticlassSoftmax(int num_class) : num_class_(num_class) {
    factor_ = static_cast<double>(num_class_) / (num_class_ - 1.0f);
  }
  void Init(const Metadata& md, data_size_t num_data) override {
    num_data_ = num_data;
    label_ = md.label();
    weights_ = md.weights();
    label_int_.resize(num_data);
    probs_.assign(num_class_, 0.0);
    double sw = 0.0;
    for (data_size_t i = 0; i < num_data; ++i) {
      label_int_[i] = static_cast<int>(label_[i]);
      if (label_int_[i] < 0 || label_int_[i] >= num_class_) {
        Log::Fatal("Label must be in [0, %d), but found %d in label", num_class_, label_int_[i]);
      }
      const double w = weights_ ? weights_[i] : 1.0;
      probs_[label_int_[i]] += w;
      sw += w;
    }
    if (Network::num_machines() > 1) {
      sw = Network::GlobalSyncUpBySum(sw);
      for (auto& p : probs_) p = Network::GlobalSyncUpBySum(p);
    }
    for (auto& p : probs_) p /= sw;
  }
  void GetGradients(const double* score, score_t* g, score_t* h) const override {
#pragma omp parallel
    {
      std::vector<double> rec(num_class_);
#pragma omp for schedule(static)
      for (data_size_t i = 0; i < num_data_; ++i) {
        for (int k = 0; k < num_class_; ++k) rec[k] = score[static_cast<size_t>(num_data_) * k + i];
        common::Softmax(&rec);
        const double w = weights_ ? weights_[i] : 1.0;
        for (int k = 0; k < num_class_; ++k) {
          const double p = rec[k];
          const size_t idx = static_cast<size_t>(num_data_) * k + i;
          if (weights_) {
            g[idx] = static_cast<score_t>((label_int_[i] == k ? p - 1.0f : p) * w);
            h[idx] = static_cast<score_t>(factor_ * p * (1.0f - p) * w);
          } else {
            g[idx] = static_cast<score_t>(label_int_[i] == k ? p - 1.0f : p);
            h[idx] = static_cast<score_t>(factor_ * p * (1.0f - p));
          }
        }
      }
    }
  }
  void ConvertOutput(const double* in, double* out) const override { common::Softmax(in, out, num_class_); }
  const char* GetName() const override { return "multiclass"; }
  std::string ToString() const override { return "multiclass num_class:" + std::to_string(num_class_); }
  bool SkipEmptyClass() const override { return true; }
  int NumModelPerIteration() const override { return num_class_; }
  int NumPredictOneRow() const override { return num_class_; }
  bool NeedAccuratePrediction() const override { return false; }
  double BoostFromScore(int k) const override { return std::log(std::max<double>(kEpsilon, probs_[k])); }
  bool ClassNeedTrain(int k) const override {
    return !(std::fabs(probs_[k]) <= kEpsilon || std::fabs(probs_[k]) >= 1.0 - kEpsilon);
  }
  DeviceGradKind device_kind() const override { return DeviceGradKind::kSoftmax; }
  int num_class() const override { return num_class_; }
  const label_t* effective_label() const override { return label_; }

 private:
  int num_class_;
  double factor_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  std::vector<int> label_int_;
  std::vector<double> probs_;
};

class MulticlassOVA : public ObjectiveFunction {
 public:
  MulticlassOVA(int num_class, double sigmoid, const Config* c) : num_class_(num_class), sigmoid_(sigmoid) {
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid parameter %f should be greater than zero", sigmoid_);
    if (c) cfg_ = *c;
    cfg_.sigmoid = sigmoid;
  }
  void Init(const Metadata& md, data_size_t num_data) override {
    num_data_ = num_data;
    label_ = md.label();
    bin_.clear();
    onehot_.assign(num_class_, std::vector<label_t>(num_data));
    for (int k = 0; k < num_class_; ++k) {
      for (data_size_t i = 0; i < num_data; ++i) onehot_[k][i] = static_cast<int>(md.label()[i]) == k ? 1.0f : 0.0f;
      Metadata m2 = md;
      m2.SetLabel(onehot_[k].data(), num_data);
      mds_.push_back(m2);
    }
    for (int k = 0; k < num_class_; ++k) {
      bin_.emplace_back(new PointwiseObjective(kPwBinary, cfg_));
      bin_.back()->Init(mds_[k], num_data);
    }
  }
  void GetGradients(const double* score, score_t* g, score_t* h) const override {
    for (int k = 0; k < num_class_; ++k) {
      const size_t off = static_cast<size_t>(num_data_) * k;
      bin_[k]->GetGradients(score + off, g + off, h + off);
    }
  }
  const char* GetName() const override { return "multiclassova"; }
  std::string ToString() const override {
    return "multiclassova num_class:" + std::to_string(num_class_) + " sigmoid:" + common::FormatG(sigmoid_);
  }
  void ConvertOutput(const double* in, double* out) const override {
    for (int k = 0; k < num_class_; ++k) out[k] = 1.0f / (1.0f + std::exp(-sigmoid_ * in[k]));
  }
  bool SkipEmptyClass() const override { return true; }
  int NumModelPerIteration() const override { return num_class_; }
  int NumPredictOneRow() const override { return num_class_; }
  bool NeedAccuratePrediction() const override { return false; }
  double BoostFromScore(int k) const override { return bin_[k]->BoostFromScore(0); }
  bool ClassNeedTrain(int k) const override { return bin_[k]->ClassNeedTrain(0); }
  int num_class() const override { return num_class_; }
  double sigmoid() const override { return sigmoid_; }
  // device: one binary kernel pass per class over the original labels (label == k)
  DeviceGradKind device_kind() const override { return DeviceGradKind::kOVA; }
  const PointwiseParams* pointwise_class(int k) const override {
    return k >= 0 && k < static_cast<int>(bin_.size()) ? bin_[k]->pointwise() : nullptr;
  }
  const label_t* effective_label() const override { return label_; }

 private:
  int num_class_;
  double sigmoid_;
  const label_t* label_ = nullptr;
  Config cfg_;
  data_size_t num_data_ = 0;
  std::vector<std::unique_ptr<PointwiseObjective>> bin_;
  std::vector<std::vector<label_t>> onehot_;
  std::vector<Metadata> mds_;
};

int PointwiseKindOf(const std::string& t) {
  static const std::pair<const char*, int> m[] = {
      {"regression", kPwL2}, {"regression_l1", kPwL1}, {"huber", kPwHuber}, {"fair", kPwFair},
      {"poisson", kPwPoisson}, {"quantile", kPwQuantile}, {"mape", kPwMape}, {"gamma", kPwGamma},
      {"tweedie", kPwTweedie}, {"binary", kPwBinary}, {"cross_entropy", kPwXent},
      {"cross_entropy_lambda", kPwXentLambda}};
  for (auto& kv : m) if (t == kv.first) return kv.second;
  return -1;
}

}  // namespace

std::unique_ptr<ObjectiveFunction> ObjectiveFunction::Create(const std::string& type, const Config& config) {
  if (type == "custom" || type.empty()) return nullptr;
  int k = PointwiseKindOf(type);
  if (k >= 0) return std::make_unique<PointwiseObjective>(k, config);
  if (type == "multiclass") return std::make_unique<MulticlassSoftmax>(config.num_class);
  if (type == "multiclassova") return std::make_unique<MulticlassOVA>(config.num_class, config.sigmoid, &config);
  if (type == "lambdarank" || type == "rank_xendcg") return CreateRankObjective(type, config);
  Log::Fatal("Unknown objective type name: %s", type.c_str());
}

std::unique_ptr<ObjectiveFunction> ObjectiveFunction::CreateFromString(const std::string& str) {
  auto strs = common::Split(str, ' ');
  if (strs.empty()) return nullptr;
  const std::string& type = strs[0];
  if (type == "custom") return nullptr;
  int k = PointwiseKindOf(type);
  if (k >= 0) return std::make_unique<PointwiseObjective>(k, strs);
  int num_class = -1;
  double sigmoid = -1;
  for (auto& s : strs) {
    auto kv = common::Split(s, ':');
    if (kv.size() == 2 && kv[0] == "num_class") num_class = common::AtoiOrDie(kv[1]);
    if (kv.size() == 2 && kv[0] == "sigmoid") sigmoid = common::AtofOrDie(kv[1]);
  }
  if (type == "multiclass") {
    if (num_class < 0) Log::Fatal("Objective should contain num_class field");
    return std::make_unique<MulticlassSoftmax>(num_class);
  }
  if (type == "multiclassova") {
    if (num_class < 0) Log::Fatal("Objective should contain num_class field");
    return std::make_unique<MulticlassOVA>(num_class, sigmoid, nullptr);
  }
  if (type == "lambdarank" || type == "rank_xendcg") return CreateRankObjectiveFromString(type, strs);
  Log::Fatal("Unknown objective type name: %s", type.c_str());
}

bool PointwiseOutputTransform(const ObjectiveFunction* obj, int* output, double* sigmoid) {
  auto* p = dynamic_cast<const PointwiseObjective*>(obj);
  if (p == nullptr) return false;
  *output = p->OutputTransform(sigmoid);
  return true;
}

}  // namespace lgap
