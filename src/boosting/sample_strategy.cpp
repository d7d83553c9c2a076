// Row sampling: bagging (uniform, balanced pos/neg, by query) and GOSS.
// Reference: src/boosting/bagging.hpp:14-296, goss.hpp:18-170. One
// Random(bagging_seed + block) stream per 1024-row block, so the bag does not
// depend on the thread count.
#include <omp.h>

#include <algorithm>
#include <cmath>

#include "lgap/boosting.h"
#include "lgap/log.h"

namespace lgap {

namespace {
constexpr data_size_t kRandBlock = 1024;
}

SampleStrategy::SampleStrategy(const Config* cfg, const Dataset* data, const ObjectiveFunction* obj, int ntpi)
    : cfg_(cfg), data_(data), obj_(obj), ntpi_(ntpi), num_data_(data->num_data()) {
  bag_cnt_ = num_data_;
  ResetConfig(cfg);
}

void SampleStrategy::ResetConfig(const Config* cfg) {
  cfg_ = cfg;
  goss_ = cfg->data_sample_strategy == "goss";
  by_query_ = cfg->bagging_by_query;
  if (goss_) {
    if (!(cfg->top_rate + cfg->other_rate <= 1.0)) Log::Fatal("top_rate + other_rate should be <= 1 for GOSS");
    if (!(cfg->top_rate > 0.0 && cfg->other_rate > 0.0)) Log::Fatal("top_rate and other_rate should be > 0 for GOSS");
    if (cfg->bagging_freq > 0 && cfg->bagging_fraction != 1.0) Log::Fatal("Cannot use bagging in GOSS");
    Log::Info("Using GOSS");
  }
  balanced_ = (cfg->pos_bagging_fraction < 1.0 || cfg->neg_bagging_fraction < 1.0) && cfg->bagging_freq > 0;
  const bool bagging = cfg->bagging_freq > 0 && (cfg->bagging_fraction < 1.0 || balanced_);
  bag_.resize(num_data_);
  rands_.clear();
  const data_size_t units = by_query_ ? data_->metadata().num_queries() : num_data_;
  for (data_size_t b = 0; b < (units + kRandBlock - 1) / kRandBlock; ++b) rands_.emplace_back(cfg->bagging_seed + b);
  need_rebag_ = bagging;
  if (!bagging && !goss_) bag_cnt_ = num_data_;
  if (balanced_) Log::Info("Using balanced bagging");
}

data_size_t SampleStrategy::BagBlock(data_size_t start, data_size_t cnt, data_size_t* out, bool balanced) {
  const label_t* label = data_->metadata().label();
  data_size_t nl = 0;
  for (data_size_t i = 0; i < cnt; ++i) {
    const data_size_t idx = start + i;
    const float r = rands_[idx / kRandBlock].NextFloat();
    bool keep;
    if (balanced) keep = label[idx] > 0 ? r < cfg_->pos_bagging_fraction : r < cfg_->neg_bagging_fraction;
    else keep = r < cfg_->bagging_fraction;
    if (keep) out[nl++] = idx;
  }
  return nl;
}

// One GOSS tile (goss.hpp:118-167 Helper): keep every row whose sum_k |g_k h_k| reaches the
// top_k-th largest, sample other_k of the rest and scale their (g, h) by (cnt - top_k) / other_k.
// Deliberate difference from the reference: the reference's blocks are one per thread and it
// draws the rest with a sequential adaptive-probability scan of per-1024-row LCG streams, so
// its bag depends on the thread count. Here tiles are fixed (kGossTile rows) and the rest
// sample is the other_k smallest Hash32(seed, row) keys (an exact-size uniform sample): the
// bag depends only on the data, the seed and the iteration, and the HIP sampler
// (src/device/sample_kernels.hip) draws the identical bag.
data_size_t SampleStrategy::GossBlock(data_size_t start, data_size_t cnt, data_size_t* out, score_t* g, score_t* h,
                                      uint32_t seed) {
  if (cnt <= 0) return 0;
  std::vector<score_t> imp(cnt, 0.0f);
  for (data_size_t i = 0; i < cnt; ++i)
    for (int k = 0; k < ntpi_; ++k) {
      const size_t idx = static_cast<size_t>(k) * num_data_ + start + i;
      imp[i] += std::fabs(g[idx] * h[idx]);
    }
  const data_size_t top_k = std::max<data_size_t>(1, static_cast<data_size_t>(cnt * cfg_->top_rate));
  const data_size_t other_k = static_cast<data_size_t>(cnt * cfg_->other_rate);
  std::vector<score_t> sorted = imp;
  std::nth_element(sorted.begin(), sorted.begin() + (top_k - 1), sorted.end(), std::greater<score_t>());
  const score_t threshold = sorted[top_k - 1];
  std::vector<uint32_t> keys;
  for (data_size_t i = 0; i < cnt; ++i) {
    if (!(imp[i] >= threshold)) keys.push_back(Hash32(seed, static_cast<uint32_t>(start + i)));
  }
  const data_size_t rest = static_cast<data_size_t>(keys.size());
  // 0: sample none, 1: all of the rest, 2: keys <= kthr
  int mode = 0;
  uint32_t kthr = 0;
  if (other_k > 0 && rest > 0) {
    if (other_k >= rest) {
      mode = 1;
    } else {
      std::nth_element(keys.begin(), keys.begin() + (other_k - 1), keys.end());
      kthr = keys[other_k - 1];
      mode = 2;
    }
  }
  const score_t multiply = other_k > 0 ? static_cast<score_t>(cnt - top_k) / other_k : 1.0f;
  data_size_t nl = 0;
  for (data_size_t i = 0; i < cnt; ++i) {
    const data_size_t idx = start + i;
    if (imp[i] >= threshold) {
      out[nl++] = idx;
    } else if (mode == 1 || (mode == 2 && Hash32(seed, static_cast<uint32_t>(idx)) <= kthr)) {
      out[nl++] = idx;
      for (int k = 0; k < ntpi_; ++k) {
        const size_t j = static_cast<size_t>(k) * num_data_ + idx;
        g[j] *= multiply;
        h[j] *= multiply;
      }
    }
  }
  return nl;
}

int SampleStrategy::PlanDevice(int iter) {
  if (goss_) {
    if (iter < static_cast<int>(1.0f / cfg_->learning_rate)) return iter == 0 ? kSampleAll : kSampleKeep;
    return kSampleGoss;
  }
  const bool bagging = cfg_->bagging_freq > 0 && (cfg_->bagging_fraction < 1.0 || balanced_);
  if (!bagging) return kSampleKeep;
  if (!(need_rebag_ || iter % cfg_->bagging_freq == 0)) return kSampleKeep;
  need_rebag_ = false;
  if (by_query_) return kSampleBagQuery;
  return balanced_ ? kSampleBalanced : kSampleBag;
}

bool SampleStrategy::Bagging(int iter, score_t* g, score_t* h) {
  if (goss_) {
    bag_cnt_ = num_data_;
    if (iter < static_cast<int>(1.0f / cfg_->learning_rate)) {
      return iter == 0;
    }
    // fixed tiles: the bag does not depend on the thread count (see GossBlock)
    const data_size_t block = kGossTile;
    const int nb = static_cast<int>((num_data_ + block - 1) / block);
    const uint32_t seed = GossSeed(cfg_->bagging_seed, iter);
    std::vector<std::vector<data_size_t>> left(nb);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nb; ++b) {
      const data_size_t s = b * block, c = std::min(block, num_data_ - s);
      left[b].resize(c);
      left[b].resize(GossBlock(s, c, left[b].data(), g, h, seed));
    }
    std::vector<char> in(num_data_, 0);
    data_size_t p = 0;
    for (auto& l : left)
      for (data_size_t i : l) {
        bag_[p++] = i;
        in[i] = 1;
      }
    bag_cnt_ = p;
    for (data_size_t i = 0; i < num_data_; ++i) if (!in[i]) bag_[p++] = i;
    return true;
  }
  const bool bagging = cfg_->bagging_freq > 0 && (cfg_->bagging_fraction < 1.0 || balanced_);
  if (!bagging) return false;
  if (!(need_rebag_ || iter % cfg_->bagging_freq == 0)) return false;
  need_rebag_ = false;
  std::vector<char> in(num_data_, 0);
  data_size_t p = 0;
  if (!by_query_) {
    const int nb = static_cast<int>((num_data_ + kRandBlock - 1) / kRandBlock);
    std::vector<std::vector<data_size_t>> left(nb);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < nb; ++b) {
      const data_size_t s = b * kRandBlock, c = std::min(kRandBlock, num_data_ - s);
      left[b].resize(c);
      left[b].resize(BagBlock(s, c, left[b].data(), balanced_));
    }
    for (auto& l : left)
      for (data_size_t i : l) {
        bag_[p++] = i;
        in[i] = 1;
      }
  } else {
    const auto& md = data_->metadata();
    const data_size_t nq = md.num_queries();
    const data_size_t* qb = md.query_boundaries();
    for (data_size_t q = 0; q < nq; ++q) {
      if (rands_[q / kRandBlock].NextFloat() < cfg_->bagging_fraction) {
        for (data_size_t i = qb[q]; i < qb[q + 1]; ++i) {
          bag_[p++] = i;
          in[i] = 1;
        }
      }
    }
  }
  bag_cnt_ = p;
  for (data_size_t i = 0; i < num_data_; ++i) if (!in[i]) bag_[p++] = i;
  Log::Debug("Re-bagging, using %d data to train", bag_cnt_);
  return true;
}

}  // namespace lgap
