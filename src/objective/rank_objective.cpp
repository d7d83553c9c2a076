// Ranking objectives: LambdaRank with the fork's 18 `lambdarank_target`s and
// `lambdagap_weight`, position-bias Newton updates (unbiased LTR), and
// RankXENDCG. Reference: src/objective/rank_objective.hpp:44-728.
//
// Deliberate fix vs. the reference: for target `precision` the reference calls
// nth_element at truncation_level-1 even when k > cnt (undefined behaviour,
// rank_objective.hpp:268-276); here k is clamped to the query size.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <numeric>

#include "lgap/omp_errors.h"
#include "lgap/common.h"
#include "lgap/log.h"
#include "lgap/metric.h"
#include "lgap/objective.h"
#include "lgap/random.h"
#include "lgap/rank_math.h"

namespace lgap {

namespace {

int ParseTarget(const std::string& s) {
  static const std::map<std::string, int> m = {
      {"ndcg", kTgtNdcg},
      {"lambdaloss-ndcg", kTgtLambdalossNdcg},
      {"lambdaloss-ndcg-plus-plus", kTgtLambdalossNdcgPP},
      {"bndcg", kTgtBndcg},
      {"lambdaloss-bndcg", kTgtLambdalossBndcg},
      {"lambdaloss-bndcg-plus-plus", kTgtLambdalossBndcgPP},
      {"precision", kTgtPrecision},
      {"arpk", kTgtArpK},
      {"lambdaloss-arp1", kTgtLambdalossArp1},
      {"lambdaloss-arp2", kTgtLambdalossArp2},
      {"ranknet", kTgtRanknet},
      {"bin-ranknet", kTgtBinRanknet},
      {"lambdagap-s", kTgtGapS},
      {"lambdagap-x", kTgtGapX},
      {"lambdagap-s-plus", kTgtGapSPlus},
      {"lambdagap-x-plus", kTgtGapXPlus},
      {"lambdagap-s-plus-plus", kTgtGapSPlusPlus},
      {"lambdagap-x-plus-plus", kTgtGapXPlusPlus}};
  auto it = m.find(s);
  if (it == m.end()) Log::Fatal("Unknown lambdarank target '%s'", s.c_str());
  return it->second;
}

class RankingBase : public ObjectiveFunction {
 public:
  explicit RankingBase(const Config* c) {
    if (c) {
      seed_ = c->objective_seed;
      learning_rate_ = c->learning_rate;
      pos_reg_ = c->lambdarank_position_bias_regularization;
    }
  }
  void Init(const Metadata& md, data_size_t num_data) override {
    num_data_ = num_data;
    label_ = md.label();
    weights_ = md.weights();
    positions_ = md.positions();
    num_position_ids_ = md.num_position_ids();
    position_ids_ = md.position_ids();
    qb_ = md.query_boundaries();
    if (qb_ == nullptr) Log::Fatal("Ranking tasks require query information");
    num_queries_ = md.num_queries();
    pos_biases_.assign(num_position_ids_, 0.0f);
    effective_pairs_.assign(num_queries_, 0.0);
  }
  void GetGradients(const double* score, score_t* g, score_t* h) const override {
    OmpErrors errs;  // label / target checks inside OneQuery raise
#pragma omp parallel for schedule(guided)
    for (data_size_t q = 0; q < num_queries_; ++q) {
      errs.Run([&] {
        const data_size_t start = qb_[q];
        const data_size_t cnt = qb_[q + 1] - qb_[q];
        std::vector<double> adj;
        const double* s = score + start;
        if (num_position_ids_ > 0) {
          adj.resize(cnt);
          for (data_size_t j = 0; j < cnt; ++j) adj[j] = score[start + j] + pos_biases_[positions_[start + j]];
          s = adj.data();
        }
        OneQuery(q, cnt, label_ + start, s, g + start, h + start);
        if (weights_) {
          for (data_size_t j = 0; j < cnt; ++j) {
            g[start + j] = static_cast<score_t>(g[start + j] * weights_[start + j]);
            h[start + j] = static_cast<score_t>(h[start + j] * weights_[start + j]);
          }
        }
      });
    }
    errs.Rethrow();
    if (Log::Level() >= LogLevel::Debug) {
      double avg = 0.0;
      for (auto e : effective_pairs_) if (!std::isnan(e)) avg += e;
      Log::Debug("Average effective pairs per query: %.4f%%", 100.0 * avg / std::max(1, num_queries_));
    }
    if (num_position_ids_ > 0) UpdatePositionBias(g, h);
    ++iter_;
  }
  virtual void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* g,
                        score_t* h) const = 0;
  bool NeedAccuratePrediction() const override { return false; }
  bool IsRanking() const override { return true; }
  const std::vector<label_t>& position_biases() const { return pos_biases_; }
  double position_learning_rate() const { return learning_rate_; }
  double position_regularization() const { return pos_reg_; }
  const std::vector<double>& effective_pairs() const { return effective_pairs_; }

 protected:
  void UpdatePositionBias(const score_t* g, const score_t* h) const {
    std::vector<double> d1(num_position_ids_, 0.0), d2(num_position_ids_, 0.0);
    std::vector<int> cnt(num_position_ids_, 0);
    for (data_size_t i = 0; i < num_data_; ++i) {
      d1[positions_[i]] -= g[i];
      d2[positions_[i]] -= h[i];
      cnt[positions_[i]]++;
    }
    for (int p = 0; p < num_position_ids_; ++p) {
      double a = d1[p] - pos_biases_[p] * pos_reg_ * cnt[p];
      double b = d2[p] - pos_reg_ * cnt[p];
      pos_biases_[p] += static_cast<label_t>(learning_rate_ * a / (std::abs(b) + 0.001));
    }
  }

  int seed_ = 0;
  double learning_rate_ = 0.1;
  double pos_reg_ = 0.0;
  data_size_t num_data_ = 0;
  data_size_t num_queries_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  const int32_t* positions_ = nullptr;
  int num_position_ids_ = 0;
  std::vector<std::string> position_ids_;
  const data_size_t* qb_ = nullptr;
  mutable std::vector<label_t> pos_biases_;
  mutable std::vector<double> effective_pairs_;
  mutable int iter_ = 0;
};

class LambdarankObjective : public RankingBase {
 public:
  explicit LambdarankObjective(const Config& c)
      : RankingBase(&c), sigmoid_(c.sigmoid), norm_(c.lambdarank_norm), k_(c.lambdarank_truncation_level),
        gap_weight_(c.lambdagap_weight) {
    target_ = ParseTarget(c.lambdarank_target);
    target_name_ = c.lambdarank_target;
    label_gain_ = c.label_gain;
    DCGCalculator::DefaultLabelGain(&label_gain_);
    DCGCalculator::Init(label_gain_);
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid param %f should be greater than zero", sigmoid_);
    Log::Info("Using lambdarank objective with target '%s'", target_name_.c_str());
  }
  explicit LambdarankObjective(const std::vector<std::string>&) : RankingBase(nullptr) {}

  void Init(const Metadata& md, data_size_t num_data) override {
    RankingBase::Init(md, num_data);
    DCGCalculator::CheckMetadata(md, num_queries_);
    DCGCalculator::CheckLabel(label_, num_data_);
    inv_max_dcg_.resize(num_queries_);
    inv_max_bdcg_.resize(num_queries_);
#pragma omp parallel for schedule(static)
    for (data_size_t q = 0; q < num_queries_; ++q) {
      const data_size_t n = qb_[q + 1] - qb_[q];
      double v = DCGCalculator::CalMaxDCGAtK(k_, label_ + qb_[q], n);
      inv_max_dcg_[q] = v > 0.0 ? 1.0f / v : v;
      double b = DCGCalculator::CalMaxBDCGAtK(k_, label_ + qb_[q], n);
      inv_max_bdcg_[q] = b > 0.0 ? 1.0f / b : b;
    }
    BuildSigmoidTable();
  }

  void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* lambdas,
                score_t* hessians) const override {
    for (data_size_t i = 0; i < cnt; ++i) {
      lambdas[i] = 0.0f;
      hessians[i] = 0.0f;
    }
    if (cnt <= 1) {
      effective_pairs_[q] = NAN;
      return;
    }
    std::vector<data_size_t> idx(cnt);
    std::iota(idx.begin(), idx.end(), 0);
    double best, worst;
    if (target_ == kTgtPrecision) {
      const data_size_t kk = std::min<data_size_t>(k_, cnt);
      // top-k by score with ties to the lower index: a deterministic choice of
      // the reference's nth_element set (ties there are implementation-defined),
      // identical to the device kernel's stable-sorted prefix
      std::nth_element(idx.begin(), idx.begin() + (kk - 1), idx.end(), [score](data_size_t a, data_size_t b) {
        return score[a] > score[b] || (score[a] == score[b] && a < b);
      });
      auto mm = std::minmax_element(score, score + cnt);
      worst = *mm.first;
      best = *mm.second;
    } else if (!TargetNeedsFullSort(target_)) {
      auto mm = std::minmax_element(score, score + cnt);
      worst = *mm.first;
      best = *mm.second;
    } else {
      std::stable_sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
      best = score[idx[0]];
      data_size_t wi = cnt - 1;
      if (wi > 0 && score[idx[wi]] == kMinScore) wi -= 1;
      worst = score[idx[wi]];
    }
    double sum_lambdas = 0.0;
    int count = 0;
    const int i_end = TargetIEnd(target_, cnt, k_);
    const bool binary = TargetIsBinary(target_);
    for (int i = 0; i < i_end; ++i) {
      if (score[idx[i]] == kMinScore) continue;
      int js, je;
      TargetJRange(target_, i, cnt, k_, &js, &je);
      for (int j = js; j < je; ++j) {
        if (score[idx[j]] == kMinScore) continue;
        const score_t li = label[idx[i]], lj = label[idx[j]];
        if (li == lj) continue;
        if (binary && li > 0 && lj > 0) continue;
        int hr, lr;
        if (li > lj) {
          hr = i;
          lr = j;
        } else {
          hr = j;
          lr = i;
        }
        const data_size_t high = idx[hr], low = idx[lr];
        const double ds = score[high] - score[low];
        const int hl = static_cast<int>(label[high]), ll = static_cast<int>(label[low]);
        double dp = TargetDeltaPair(target_, i, j, hr, lr, label_gain_[hl], label_gain_[ll], label[high], label[low],
                                    inv_max_dcg_[q], inv_max_bdcg_[q], k_, gap_weight_);
        if (dp == 0) continue;
        if (norm_ && best != worst) dp /= (0.01f + std::fabs(ds));
        double pl = Sigmoid(ds);
        double ph = pl * (1.0f - pl);
        pl *= -sigmoid_ * dp;
        ph *= sigmoid_ * sigmoid_ * dp;
        lambdas[low] -= static_cast<score_t>(pl);
        hessians[low] += static_cast<score_t>(ph);
        lambdas[high] += static_cast<score_t>(pl);
        hessians[high] += static_cast<score_t>(ph);
        sum_lambdas -= 2 * pl;
        ++count;
      }
    }
    if (norm_ && sum_lambdas > 0) {
      const double f = std::log2(1 + sum_lambdas) / sum_lambdas;
      for (data_size_t i = 0; i < cnt; ++i) {
        lambdas[i] = static_cast<score_t>(lambdas[i] * f);
        hessians[i] = static_cast<score_t>(hessians[i] * f);
      }
    }
    effective_pairs_[q] = 2.0 * count / (static_cast<double>(cnt) * (cnt - 1));
  }

  inline double Sigmoid(double s) const {
    if (s <= min_in_) return table_[0];
    if (s >= max_in_) return table_[kBins - 1];
    return table_[static_cast<size_t>((s - min_in_) * idx_factor_)];
  }

  const char* GetName() const override { return "lambdarank"; }
  std::string ToString() const override { return "lambdarank"; }
  DeviceGradKind device_kind() const override { return DeviceGradKind::kLambdarank; }
  double sigmoid() const override { return sigmoid_; }

  // exposed to the device kernel
  int target() const { return target_; }
  int truncation() const { return k_; }
  bool norm() const { return norm_; }
  double gap_weight() const { return gap_weight_; }
  const std::vector<double>& label_gain() const { return label_gain_; }
  const std::vector<double>& inv_max_dcg() const { return inv_max_dcg_; }
  const std::vector<double>& inv_max_bdcg() const { return inv_max_bdcg_; }
  const std::vector<double>& sigmoid_table() const { return table_; }
  double table_min() const { return min_in_; }
  double table_max() const { return max_in_; }
  double table_factor() const { return idx_factor_; }

 private:
  void BuildSigmoidTable() {
    min_in_ = -50.0 / sigmoid_ / 2;
    max_in_ = -min_in_;
    table_.resize(kBins);
    idx_factor_ = kBins / (max_in_ - min_in_);
    for (size_t i = 0; i < kBins; ++i) {
      const double s = i / idx_factor_ + min_in_;
      table_[i] = 1.0f / (1.0f + std::exp(s * sigmoid_));
    }
  }
  static constexpr size_t kBins = 1024 * 1024;
  double sigmoid_ = 1.0;
  bool norm_ = true;
  int k_ = 30;
  double gap_weight_ = 1.0;
  int target_ = kTgtNdcg;
  std::string target_name_ = "ndcg";
  std::vector<double> label_gain_;
  std::vector<double> inv_max_dcg_, inv_max_bdcg_;
  std::vector<double> table_;
  double min_in_ = -50, max_in_ = 50, idx_factor_ = 1;
};

class RankXENDCG : public RankingBase {
 public:
  explicit RankXENDCG(const Config& c) : RankingBase(&c) {}
  explicit RankXENDCG(const std::vector<std::string>&) : RankingBase(nullptr) {}
  void Init(const Metadata& md, data_size_t num_data) override {
    RankingBase::Init(md, num_data);
    rands_.clear();
    for (data_size_t q = 0; q < num_queries_; ++q) rands_.emplace_back(seed_ + q);
  }
  void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* lambdas,
                score_t* hessians) const override {
    if (cnt <= 1) {
      for (data_size_t i = 0; i < cnt; ++i) lambdas[i] = hessians[i] = 0.0f;
      return;
    }
    std::vector<double> rho(cnt), params(cnt);
    common::Softmax(score, rho.data(), cnt);
    double inv_den = 0.0;
    for (data_size_t i = 0; i < cnt; ++i) {
      params[i] = std::pow(2.0, static_cast<int>(label[i])) - rands_[q].NextFloat();
      inv_den += params[i];
    }
    inv_den = 1. / std::max<double>(kEpsilon, inv_den);
    double sum_l1 = 0.0;
    for (data_size_t i = 0; i < cnt; ++i) {
      const double term = -params[i] * inv_den + rho[i];
      lambdas[i] = static_cast<score_t>(term);
      params[i] = term / (1. - rho[i]);
      sum_l1 += params[i];
    }
    double sum_l2 = 0.0;
    for (data_size_t i = 0; i < cnt; ++i) {
      const double term = rho[i] * (sum_l1 - params[i]);
      lambdas[i] += static_cast<score_t>(term);
      params[i] = term / (1. - rho[i]);
      sum_l2 += params[i];
    }
    for (data_size_t i = 0; i < cnt; ++i) {
      lambdas[i] += static_cast<score_t>(rho[i] * (sum_l2 - params[i]));
      hessians[i] = static_cast<score_t>(rho[i] * (1.0 - rho[i]));
    }
  }
  const char* GetName() const override { return "rank_xendcg"; }
  DeviceGradKind device_kind() const override { return DeviceGradKind::kXendcg; }
  int objective_seed() const { return seed_; }

 private:
  mutable std::vector<Random> rands_;
};

}  // namespace

std::unique_ptr<ObjectiveFunction> CreateRankObjective(const std::string& type, const Config& config) {
  if (type == "lambdarank") return std::make_unique<LambdarankObjective>(config);
  return std::make_unique<RankXENDCG>(config);
}

std::unique_ptr<ObjectiveFunction> CreateRankObjectiveFromString(const std::string& type,
                                                                 const std::vector<std::string>& strs) {
  if (type == "lambdarank") return std::make_unique<LambdarankObjective>(strs);
  return std::make_unique<RankXENDCG>(strs);
}

// Device learners need the lambdarank tables; expose a narrow accessor.
bool GetXendcgSeed(const ObjectiveFunction* obj, int* seed) {
  auto* x = dynamic_cast<const RankXENDCG*>(obj);
  if (!x) return false;
  *seed = x->objective_seed();
  return true;
}

bool GetLambdarankTables(const ObjectiveFunction* obj, LambdarankTables* out) {
  auto* l = dynamic_cast<const LambdarankObjective*>(obj);
  if (!l) return false;
  out->target = l->target();
  out->k = l->truncation();
  out->norm = l->norm() ? 1 : 0;
  out->sigmoid = l->sigmoid();
  out->gap_weight = l->gap_weight();
  out->tmin = l->table_min();
  out->tmax = l->table_max();
  out->tfactor = l->table_factor();
  out->label_gain = &l->label_gain();
  out->inv_max_dcg = &l->inv_max_dcg();
  out->inv_max_bdcg = &l->inv_max_bdcg();
  out->table = &l->sigmoid_table();
  out->pos_lr = l->position_learning_rate();
  out->pos_reg = l->position_regularization();
  return true;
}

}  // namespace lgap
