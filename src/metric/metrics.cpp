// All evaluation metrics + the DCG calculator. Reference: src/metric/*.hpp,
// factory metric.cpp:20-139, dcg_calculator.cpp:14-189 (incl. the fork's
// CalMaxBDCGAtK :82-96 and precision@k metric precision_metric.hpp:16-141).
//
// precision@k keeps the reference's denominator min(k, n - prev_k)
// (precision_metric.hpp:81) where it is well defined; when that denominator
// would be <= 0 (undefined in the reference) min(k, n) is used instead.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/metric.h"
#include "lgap/parallel_sort.h"
#include "lgap/pointwise_metric.h"

namespace lgap {

std::vector<double> DCGCalculator::label_gain_;
std::vector<double> DCGCalculator::discount_;

void DCGCalculator::DefaultEvalAt(std::vector<int>* eval_at) {
  if (eval_at->empty()) {
    for (int i = 1; i <= 5; ++i) eval_at->push_back(i);
  } else {
    for (int k : *eval_at) LGAP_CHECK_GT(k, 0);
  }
}

void DCGCalculator::DefaultLabelGain(std::vector<double>* g) {
  if (!g->empty()) return;
  g->push_back(0.0);
  for (int i = 1; i < 31; ++i) g->push_back(static_cast<double>((1 << i) - 1));
}

void DCGCalculator::Init(const std::vector<double>& g) {
  label_gain_ = g;
  discount_.resize(kMaxPosition);
  for (data_size_t i = 0; i < kMaxPosition; ++i) discount_[i] = 1.0 / std::log2(2.0 + i);
}

double DCGCalculator::CalMaxDCGAtK(data_size_t k, const label_t* label, data_size_t n) {
  std::vector<data_size_t> cnt(label_gain_.size(), 0);
  for (data_size_t i = 0; i < n; ++i) ++cnt[static_cast<int>(label[i])];
  int top = static_cast<int>(label_gain_.size()) - 1;
  k = std::min(k, n);
  double ret = 0.0;
  for (data_size_t j = 0; j < k; ++j) {
    while (top > 0 && cnt[top] <= 0) --top;
    if (top < 0) break;
    ret += discount_[j] * label_gain_[top];
    --cnt[top];
  }
  return ret;
}

double DCGCalculator::CalMaxBDCGAtK(data_size_t k, const label_t* label, data_size_t n) {
  int rel = 0;
  for (data_size_t i = 0; i < n; ++i) rel += label[i] > 0;
  k = std::min(std::min(k, n), rel);
  double ret = 0.0;
  for (data_size_t j = 0; j < k; ++j) ret += discount_[j];
  return ret;
}

void DCGCalculator::CalMaxDCG(const std::vector<data_size_t>& ks, const label_t* label, data_size_t n,
                              std::vector<double>* out) {
  std::vector<data_size_t> cnt(label_gain_.size(), 0);
  for (data_size_t i = 0; i < n; ++i) ++cnt[static_cast<int>(label[i])];
  double cur = 0.0;
  data_size_t left = 0;
  int top = static_cast<int>(label_gain_.size()) - 1;
  for (size_t i = 0; i < ks.size(); ++i) {
    data_size_t k = std::min(ks[i], n);
    for (data_size_t j = left; j < k; ++j) {
      while (top > 0 && cnt[top] <= 0) --top;
      if (top < 0) break;
      cur += discount_[j] * label_gain_[top];
      --cnt[top];
    }
    (*out)[i] = cur;
    left = k;
  }
}

void DCGCalculator::CalDCG(const std::vector<data_size_t>& ks, const label_t* label, const double* score,
                           data_size_t n, std::vector<double>* out) {
  std::vector<data_size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
  double cur = 0.0;
  data_size_t left = 0;
  for (size_t i = 0; i < ks.size(); ++i) {
    data_size_t k = std::min(ks[i], n);
    for (data_size_t j = left; j < k; ++j) cur += label_gain_[static_cast<int>(label[idx[j]])] * discount_[j];
    (*out)[i] = cur;
    left = k;
  }
}

void DCGCalculator::CheckLabel(const label_t* label, data_size_t n) {
  for (data_size_t i = 0; i < n; ++i) {
    label_t d = std::fabs(label[i] - static_cast<int>(label[i]));
    if (d > kEpsilon) Log::Fatal("label should be int type (met %f) for ranking task", label[i]);
    if (label[i] < 0) Log::Fatal("Label should be non-negative (met %f) for ranking task", label[i]);
    if (label[i] >= static_cast<label_t>(label_gain_.size())) {
      Log::Fatal("Label %zu is not less than the number of label mappings (%zu)", static_cast<size_t>(label[i]),
                 label_gain_.size());
    }
  }
}

void DCGCalculator::CheckMetadata(const Metadata& md, data_size_t nq) {
  const data_size_t* qb = md.query_boundaries();
  if (nq > 0 && qb != nullptr) {
    for (data_size_t i = 0; i < nq; ++i) {
      if (qb[i + 1] - qb[i] > kMaxPosition) {
        Log::Fatal("Number of rows %i exceeds upper limit of %i for a query", qb[i + 1] - qb[i], kMaxPosition);
      }
    }
  }
}

namespace {

// ---------------------------------------------------------------------------
class PointwiseMetric : public Metric {
 public:
  enum Kind { L2, RMSE, L1, QUANTILE, HUBER, FAIR, POISSON, MAPE, GAMMA, GAMMA_DEV, TWEEDIE, BIN_LOGLOSS, BIN_ERROR,
              XENT, XENT_LAMBDA, KLDIV };
  PointwiseMetric(Kind k, const Config& c) : k_(k), cfg_(c) {
    pm_.kind = static_cast<int>(k);  // Kind and PwMetricKind list the metrics in the same order
    pm_.alpha = c.alpha;
    pm_.fair_c = c.fair_c;
    pm_.tweedie_rho = c.tweedie_variance_power;
    static const char* names[] = {"l2", "rmse", "l1", "quantile", "huber", "fair", "poisson", "mape", "gamma",
                                  "gamma_deviance", "tweedie", "binary_logloss", "binary_error", "cross_entropy",
                                  "cross_entropy_lambda", "kullback_leibler"};
    name_.push_back(names[k]);
  }
  void Init(const Metadata& md, data_size_t n) override {
    n_ = n;
    label_ = md.label();
    w_ = md.weights();
    sumw_ = 0.0;
    if (w_) for (data_size_t i = 0; i < n; ++i) sumw_ += w_[i];
    else sumw_ = n;
    if (k_ == GAMMA || k_ == GAMMA_DEV) {
      for (data_size_t i = 0; i < n; ++i) if (!(label_[i] > 0)) Log::Fatal("[%s]: label should be positive", name_[0].c_str());
    }
    if (k_ == KLDIV) {
      ent_ = 0.0;
      for (data_size_t i = 0; i < n; ++i) ent_ += Yent(label_[i]) * (w_ ? w_[i] : 1.0);
      ent_ /= sumw_;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return -1.0; }

  static double Yent(double p) {
    double h = 0.0;
    if (p > 0) h += p * std::log(p);
    double q = 1.0f - p;
    if (q > 0) h += q * std::log(q);
    return h;
  }

  // the row loss is shared with the device metric kernel (lgap/pointwise_metric.h)
  double Loss(label_t y, double s, double w) const { return PmLoss(pm_, y, s, w); }

  bool DevicePointwise(const ObjectiveFunction* obj, PwMetricParams* out) const override {
    PwMetricParams p = pm_;
    if (obj == nullptr) {
      p.output = k_ == XENT_LAMBDA ? kOutLog1pExp : kOutIdentity;
    } else if (!PointwiseOutputTransform(obj, &p.output, &p.sigmoid)) {
      return false;
    }
    *out = p;
    return true;
  }

  std::vector<double> FinishSum(double sum) const override {
    double v;
    if (k_ == RMSE) v = std::sqrt(sum / sumw_);
    else if (k_ == GAMMA_DEV) v = sum * 2;
    else if (k_ == XENT_LAMBDA) v = sum / static_cast<double>(n_);
    else if (k_ == KLDIV) v = ent_ + sum / sumw_;
    else v = sum / sumw_;
    return {v};
  }

  std::vector<double> Eval(const double* score, const ObjectiveFunction* obj) const override {
    double sum = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : sum)
    for (data_size_t i = 0; i < n_; ++i) {
      double s = score[i];
      if (k_ == XENT_LAMBDA) {
        if (obj) obj->ConvertOutput(&score[i], &s);
        else s = std::log1p(std::exp(score[i]));
        sum += Loss(label_[i], s, w_ ? w_[i] : 1.0);
        continue;
      }
      if (obj) obj->ConvertOutput(&score[i], &s);
      sum += w_ ? Loss(label_[i], s, 1.0) * w_[i] : Loss(label_[i], s, 1.0);
    }
    return FinishSum(sum);
  }

 private:
  Kind k_;
  Config cfg_;
  std::vector<std::string> name_;
  data_size_t n_ = 0;
  const label_t* label_ = nullptr;
  const label_t* w_ = nullptr;
  double sumw_ = 0.0, ent_ = 0.0;
  PwMetricParams pm_;
};

// AUC with tied-score groups (binary_metric.hpp:194-251).
class AUCMetric : public Metric {
 public:
  explicit AUCMetric(bool ap) : ap_(ap) { name_.push_back(ap ? "average_precision" : "auc"); }
  void Init(const Metadata& md, data_size_t n) override {
    n_ = n;
    label_ = md.label();
    w_ = md.weights();
    sumw_ = 0.0;
    if (w_) for (data_size_t i = 0; i < n; ++i) sumw_ += w_[i];
    else sumw_ = n;
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  bool DeviceRankSpec(RankMetricSpec* out) const override {
    out->kind = ap_ ? RankMetricSpec::kAveragePrecision : RankMetricSpec::kAUC;
    out->owner = this;
    out->num_data = n_;
    out->label = label_;
    out->weights = w_;
    return true;
  }
  // device sums {accumulator, positive weight} -> the value, as the end of Eval below
  std::vector<double> FinishRank(const std::vector<double>& v) const override {
    const double accum = v[0], sum_pos = v[1];
    double r = 1.0;
    if (ap_) {
      if (sum_pos > 0.0 && sum_pos != sumw_) r = accum / sum_pos;
    } else if (sum_pos > 0.0 && sum_pos != sumw_) {
      r = accum / (sum_pos * (sumw_ - sum_pos));
    }
    return {r};
  }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    if (n_ == 0) return {1.0};
    std::vector<data_size_t> idx(n_);
    std::iota(idx.begin(), idx.end(), 0);
    // tied scores form one group below, so their order is free: an unstable parallel sort
    // (reference binary_metric.hpp:200 Common::ParallelSort)
    common::ParallelSort(&idx, [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
    double cur_pos = 0, sum_pos = 0, accum = 0, cur_neg = 0;
    double sum_pred_pos = 0, accum_prec = 1.0;
    double thr = score[idx[0]];
    for (data_size_t i = 0; i < n_; ++i) {
      const label_t y = label_[idx[i]];
      const double s = score[idx[i]];
      const double w = w_ ? w_[idx[i]] : 1.0;
      if (s != thr) {
        thr = s;
        if (ap_) {
          sum_pos += cur_pos;
          sum_pred_pos += cur_pos + cur_neg;
          accum_prec = sum_pos / sum_pred_pos;
          accum += cur_pos * accum_prec;
        } else {
          accum += cur_neg * (cur_pos * 0.5f + sum_pos);
          sum_pos += cur_pos;
        }
        cur_neg = cur_pos = 0.0;
      }
      cur_neg += (y <= 0) * w;
      cur_pos += (y > 0) * w;
    }
    if (ap_) {
      sum_pos += cur_pos;
      sum_pred_pos += cur_pos + cur_neg;
      accum_prec = sum_pos / sum_pred_pos;
      accum += cur_pos * accum_prec;
      double v = 1.0;
      if (sum_pos > 0.0 && sum_pos != sumw_) v = accum / sum_pos;
      return {v};
    }
    accum += cur_neg * (cur_pos * 0.5f + sum_pos);
    sum_pos += cur_pos;
    double auc = 1.0;
    if (sum_pos > 0.0 && sum_pos != sumw_) auc = accum / (sum_pos * (sumw_ - sum_pos));
    return {auc};
  }

 private:
  bool ap_;
  std::vector<std::string> name_;
  data_size_t n_ = 0;
  const label_t* label_ = nullptr;
  const label_t* w_ = nullptr;
  double sumw_ = 0.0;
};

class MulticlassMetric : public Metric {
 public:
  MulticlassMetric(bool error, const Config& c) : error_(error), cfg_(c), num_class_(c.num_class) {
    if (error) name_.push_back(c.multi_error_top_k == 1 ? "multi_error" : "multi_error@" + std::to_string(c.multi_error_top_k));
    else name_.push_back("multi_logloss");
  }
  void Init(const Metadata& md, data_size_t n) override {
    n_ = n;
    label_ = md.label();
    w_ = md.weights();
    sumw_ = 0.0;
    if (w_) for (data_size_t i = 0; i < n; ++i) sumw_ += w_[i];
    else sumw_ = n;
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return -1.0; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction* obj) const override {
    const int ntree = obj ? obj->NumModelPerIteration() : num_class_;
    const int npred = obj ? obj->NumPredictOneRow() : num_class_;
    double sum = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : sum)
    for (data_size_t i = 0; i < n_; ++i) {
      std::vector<double> raw(ntree), rec(npred);
      for (int k = 0; k < ntree; ++k) raw[k] = score[static_cast<size_t>(n_) * k + i];
      if (obj) obj->ConvertOutput(raw.data(), rec.data());
      else rec = raw;
      const size_t y = static_cast<size_t>(label_[i]);
      double l;
      if (error_) {
        int larger = 0;
        l = 0.0;
        for (size_t k = 0; k < rec.size(); ++k) {
          if (rec[k] >= rec[y]) ++larger;
          if (larger > cfg_.multi_error_top_k) {
            l = 1.0;
            break;
          }
        }
      } else {
        l = rec[y] > kEpsilon ? -std::log(rec[y]) : -std::log(kEpsilon);
      }
      sum += w_ ? l * w_[i] : l;
    }
    return {sum / sumw_};
  }
  bool DeviceMulti(const ObjectiveFunction* obj, MultiMetricParams* out) const override {
    MultiMetricParams p;
    if (obj == nullptr) {
      p.output = 0;
    } else if (std::strcmp(obj->GetName(), "multiclass") == 0) {
      p.output = 1;
    } else if (std::strcmp(obj->GetName(), "multiclassova") == 0) {
      p.output = 2;
      p.sigmoid = obj->sigmoid();
    } else {
      return false;
    }
    if (obj != nullptr && (obj->NumModelPerIteration() != num_class_ || obj->NumPredictOneRow() != num_class_)) return false;
    p.error = error_ ? 1 : 0;
    p.top_k = cfg_.multi_error_top_k;
    p.num_class = num_class_;
    *out = p;
    return true;
  }
  std::vector<double> FinishSum(double sum) const override { return {sum / sumw_}; }

 private:
  bool error_;
  Config cfg_;
  int num_class_;
  std::vector<std::string> name_;
  data_size_t n_ = 0;
  const label_t* label_ = nullptr;
  const label_t* w_ = nullptr;
  double sumw_ = 0.0;
};

class AucMuMetric : public Metric {
 public:
  explicit AucMuMetric(const Config& c) : num_class_(c.num_class), cw_(c.auc_mu_weights_matrix) { name_.push_back("auc_mu"); }
  void Init(const Metadata& md, data_size_t n) override {
    n_ = n;
    label_ = md.label();
    w_ = md.weights();
    sorted_.resize(n);
    std::iota(sorted_.begin(), sorted_.end(), 0);
    std::stable_sort(sorted_.begin(), sorted_.end(), [this](data_size_t a, data_size_t b) { return label_[a] < label_[b]; });
    sizes_.assign(num_class_, 0);
    cls_w_.assign(num_class_, 0.0);
    for (data_size_t i = 0; i < n; ++i) {
      ++sizes_[static_cast<int>(label_[i])];
      if (w_) cls_w_[static_cast<int>(label_[i])] += w_[i];
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    std::vector<std::vector<double>> S(num_class_, std::vector<double>(num_class_, 0.0));
    int istart = 0;
    for (int i = 0; i < num_class_; ++i) {
      int jstart = istart + sizes_[i];
      for (int j = i + 1; j < num_class_; ++j) {
        std::vector<double> v(num_class_);
        for (int k = 0; k < num_class_; ++k) v[k] = cw_[i][k] - cw_[j][k];
        const double t1 = v[i] - v[j];
        std::vector<std::pair<data_size_t, double>> dist;
        auto add = [&](int b, int c) {
          for (int q = b; q < b + c; ++q) {
            data_size_t a = sorted_[q];
            double va = 0;
            for (int m = 0; m < num_class_; ++m) va += v[m] * score[static_cast<size_t>(n_) * m + a];
            dist.emplace_back(a, t1 * va);
          }
        };
        add(istart, sizes_[i]);
        add(jstart, sizes_[j]);
        std::stable_sort(dist.begin(), dist.end(), [this](const std::pair<data_size_t, double>& a,
                                                          const std::pair<data_size_t, double>& b) {
          if (std::fabs(a.second - b.second) < kEpsilon) return label_[a.first] > label_[b.first];
          return a.second < b.second;
        });
        double num_j = 0, last = 0, cur_j = 0;
        for (auto& d : dist) {
          const double w = w_ ? w_[d.first] : 1.0;
          if (label_[d.first] == i) {
            S[i][j] += w * (std::fabs(d.second - last) < kEpsilon ? num_j - 0.5 * cur_j : num_j);
          } else {
            num_j += w;
            if (std::fabs(d.second - last) < kEpsilon) {
              cur_j += w;
            } else {
              last = d.second;
              cur_j = w;
            }
          }
        }
        jstart += sizes_[j];
      }
      istart += sizes_[i];
    }
    std::vector<double> flat;
    for (int i = 0; i < num_class_; ++i)
      for (int j = i + 1; j < num_class_; ++j) flat.push_back(S[i][j]);
    return FinishAucMu(flat);
  }
  bool DeviceAucMu(AucMuSpec* out) const override {
    if (num_class_ < 2 || num_class_ > AucMuSpec::kMaxClass) return false;
    out->owner = this;
    out->num_data = n_;
    out->label = label_;
    out->weights = w_;
    out->num_class = num_class_;
    out->sorted = &sorted_;
    out->sizes = &sizes_;
    out->cw = &cw_;
    return true;
  }
  std::vector<double> FinishAucMu(const std::vector<double>& S) const override {
    double ans = 0;
    size_t q = 0;
    for (int i = 0; i < num_class_; ++i)
      for (int j = i + 1; j < num_class_; ++j, ++q)
        ans += w_ ? (S[q] / cls_w_[i]) / cls_w_[j] : (S[q] / sizes_[i]) / sizes_[j];
    ans = (2.0 * ans / num_class_) / (num_class_ - 1);
    return {ans};
  }

 private:
  int num_class_;
  std::vector<std::vector<double>> cw_;
  std::vector<std::string> name_;
  data_size_t n_ = 0;
  const label_t* label_ = nullptr;
  const label_t* w_ = nullptr;
  std::vector<data_size_t> sorted_;
  std::vector<int> sizes_;
  std::vector<double> cls_w_;
};

// ndcg@k / map@k / precision@k over queries.
class QueryMetric : public Metric {
 public:
  enum Kind { NDCG, MAP, PRECISION };
  QueryMetric(Kind k, const Config& c) : k_(k) {
    eval_at_ = c.eval_at;
    DCGCalculator::DefaultEvalAt(&eval_at_);
    const char* prefix = k == NDCG ? "ndcg@" : k == MAP ? "map@" : "precision@";
    for (int e : eval_at_) name_.push_back(prefix + std::to_string(e));
    if (k == NDCG) {
      std::vector<double> g = c.label_gain;
      DCGCalculator::DefaultLabelGain(&g);
      DCGCalculator::Init(g);
    }
  }
  void Init(const Metadata& md, data_size_t n) override {
    n_ = n;
    label_ = md.label();
    qb_ = md.query_boundaries();
    if (qb_ == nullptr) Log::Fatal("The %s metric requires query information", name_[0].c_str());
    nq_ = md.num_queries();
    qw_ = md.query_weights();
    sumqw_ = 0.0;
    if (qw_) for (data_size_t q = 0; q < nq_; ++q) sumqw_ += qw_[q];
    else sumqw_ = nq_;
    if (k_ == NDCG) {
      DCGCalculator::CheckLabel(label_, n);
      inv_max_.assign(nq_, std::vector<double>(eval_at_.size()));
      std::vector<data_size_t> ks(eval_at_.begin(), eval_at_.end());
      for (data_size_t q = 0; q < nq_; ++q) {
        DCGCalculator::CalMaxDCG(ks, label_ + qb_[q], qb_[q + 1] - qb_[q], &inv_max_[q]);
        for (auto& v : inv_max_[q]) v = v > 0.0 ? 1.0 / v : -1.0;
      }
    } else if (k_ == MAP) {
      npos_.assign(nq_, 0);
      for (data_size_t q = 0; q < nq_; ++q)
        for (data_size_t i = qb_[q]; i < qb_[q + 1]; ++i) npos_[q] += label_[i] > 0.5f;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  bool DeviceRankSpec(RankMetricSpec* out) const override {
    if (eval_at_.empty() || eval_at_.size() > static_cast<size_t>(RankMetricSpec::kMaxEvalAt)) return false;
    out->kind = k_ == NDCG ? RankMetricSpec::kNDCG : (k_ == MAP ? RankMetricSpec::kMAP : RankMetricSpec::kPrecision);
    out->owner = this;
    out->num_data = n_;
    out->label = label_;
    out->num_queries = nq_;
    out->query_boundaries = qb_;
    out->query_weights = qw_;
    out->eval_at = eval_at_;
    if (k_ == NDCG) {
      out->label_gain = DCGCalculator::label_gain();
      out->inv_max.clear();
      for (const auto& v : inv_max_) out->inv_max.insert(out->inv_max.end(), v.begin(), v.end());
    } else if (k_ == MAP) {
      out->npos.assign(npos_.begin(), npos_.end());
    }
    return true;
  }
  std::vector<double> FinishRank(const std::vector<double>& v) const override {
    std::vector<double> r(v);
    for (auto& x : r) x /= sumqw_;
    return r;
  }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    const size_t ne = eval_at_.size();
    std::vector<double> result(ne, 0.0);
    std::vector<data_size_t> ks(eval_at_.begin(), eval_at_.end());
#pragma omp parallel
    {
      std::vector<double> local(ne, 0.0), tmp(ne, 0.0);
#pragma omp for schedule(guided)
      for (data_size_t q = 0; q < nq_; ++q) {
        const data_size_t b = qb_[q], n = qb_[q + 1] - qb_[q];
        const double qw = qw_ ? qw_[q] : 1.0;
        if (k_ == NDCG) {
          if (inv_max_[q][0] <= 0.0) {
            for (size_t j = 0; j < ne; ++j) local[j] += qw;
            continue;
          }
          DCGCalculator::CalDCG(ks, label_ + b, score + b, n, &tmp);
          for (size_t j = 0; j < ne; ++j) local[j] += tmp[j] * inv_max_[q][j] * qw;
        } else {
          std::vector<data_size_t> idx(n);
          std::iota(idx.begin(), idx.end(), 0);
          std::stable_sort(idx.begin(), idx.end(), [&](data_size_t a, data_size_t c) { return score[b + a] > score[b + c]; });
          int hit = 0;
          double sum_ap = 0.0;
          data_size_t left = 0;
          for (size_t e = 0; e < ne; ++e) {
            data_size_t k = ks[e];
            if (k_ == MAP) {
              k = std::min(k, n);
              for (data_size_t j = left; j < k; ++j) {
                if (label_[b + idx[j]] > 0.5f) {
                  ++hit;
                  sum_ap += static_cast<double>(hit) / (j + 1.0f);
                }
              }
              tmp[e] = npos_[q] > 0 ? sum_ap / std::min(npos_[q], k) : 1.0;
              left = k;
            } else {
              for (data_size_t j = left; j < k && j < n; ++j) hit += label_[b + idx[j]] > 0.5f;
              data_size_t den = std::min(k, n - left);
              if (den <= 0) den = std::min(k, n);
              tmp[e] = den > 0 ? static_cast<double>(hit) / den : 0.0;
              left = k;
            }
          }
          for (size_t j = 0; j < ne; ++j) local[j] += tmp[j] * qw;
        }
      }
#pragma omp critical
      for (size_t j = 0; j < ne; ++j) result[j] += local[j];
    }
    for (auto& r : result) r /= sumqw_;
    return result;
  }

 private:
  Kind k_;
  std::vector<int> eval_at_;
  std::vector<std::string> name_;
  data_size_t n_ = 0, nq_ = 0;
  const label_t* label_ = nullptr;
  const data_size_t* qb_ = nullptr;
  const label_t* qw_ = nullptr;
  double sumqw_ = 0.0;
  std::vector<std::vector<double>> inv_max_;
  std::vector<data_size_t> npos_;
};

}  // namespace

std::unique_ptr<Metric> Metric::Create(const std::string& type, const Config& c) {
  using P = PointwiseMetric;
  static const std::pair<const char*, P::Kind> pw[] = {
      {"l2", P::L2}, {"rmse", P::RMSE}, {"l1", P::L1}, {"quantile", P::QUANTILE}, {"huber", P::HUBER},
      {"fair", P::FAIR}, {"poisson", P::POISSON}, {"mape", P::MAPE}, {"gamma", P::GAMMA},
      {"gamma_deviance", P::GAMMA_DEV}, {"tweedie", P::TWEEDIE}, {"binary_logloss", P::BIN_LOGLOSS},
      {"binary_error", P::BIN_ERROR}, {"cross_entropy", P::XENT}, {"cross_entropy_lambda", P::XENT_LAMBDA},
      {"kullback_leibler", P::KLDIV}};
  for (auto& kv : pw) if (type == kv.first) return std::make_unique<PointwiseMetric>(kv.second, c);
  if (type == "auc") return std::make_unique<AUCMetric>(false);
  if (type == "average_precision") return std::make_unique<AUCMetric>(true);
  if (type == "auc_mu") return std::make_unique<AucMuMetric>(c);
  if (type == "multi_logloss") return std::make_unique<MulticlassMetric>(false, c);
  if (type == "multi_error") return std::make_unique<MulticlassMetric>(true, c);
  if (type == "ndcg") return std::make_unique<QueryMetric>(QueryMetric::NDCG, c);
  if (type == "map") return std::make_unique<QueryMetric>(QueryMetric::MAP, c);
  if (type == "precision") return std::make_unique<QueryMetric>(QueryMetric::PRECISION, c);
  if (type == "custom" || type == "none" || type.empty()) return nullptr;
  Log::Warning("Unknown metric type name: %s", type.c_str());
  return nullptr;
}

}  // namespace lgap
