#include "parallel_tree_learner.h"

#include <algorithm>
#include <cstring>
#include <numeric>

#include "lgap/log.h"
#include "lgap/network.h"

namespace lgap {

SplitInfo AllgatherBestSplit(const SplitInfo& mine) {
  const int n = Network::num_machines();
  if (n <= 1) return mine;
  std::vector<SplitInfo> all(n);
  SplitInfo m = mine;
  Network::Allgather(reinterpret_cast<char*>(&m), sizeof(SplitInfo), reinterpret_cast<char*>(all.data()));
  SplitInfo best = all[0];
  for (int i = 1; i < n; ++i) {
    if (all[i].feature >= 0 && (best.feature < 0 || all[i].BetterThan(best))) best = all[i];
  }
  return best;
}

// ============================================================================
void FeatureParallelTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  const int n = Network::num_machines(), r = Network::rank();
  // bin-balanced greedy assignment of features to ranks
  std::vector<long long> load(n, 0);
  for (int f = 0; f < num_features_; ++f) {
    const int owner = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
    load[owner] += train_data->feature(f).num_bin;
    feature_mask_[f] = owner == r;
  }
}

void FeatureParallelTreeLearner::SyncBestSplits() {
  best_split_per_leaf_[smaller_.leaf] = AllgatherBestSplit(best_split_per_leaf_[smaller_.leaf]);
  if (larger_.leaf >= 0) best_split_per_leaf_[larger_.leaf] = AllgatherBestSplit(best_split_per_leaf_[larger_.leaf]);
}

// ============================================================================
void DataParallelTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  global_counts_from_split_ = true;
  const int n = Network::num_machines(), r = Network::rank();
  const int total = train_data->num_total_bin();
  // contiguous group ranges with ~equal bins per rank (owner computes the scan)
  std::vector<int> owner(train_data->num_groups());
  for (int g = 0; g < train_data->num_groups(); ++g) {
    const auto& grp = train_data->group(g);
    const long long mid = grp.hist_start + grp.num_bin / 2;
    owner[g] = std::min(n - 1, static_cast<int>(mid * n / std::max(1, total)));
  }
  block_start_.assign(n, 0);
  block_len_.assign(n, 0);
  std::vector<int> bstart(n, total), bend(n, 0);
  for (int g = 0; g < train_data->num_groups(); ++g) {
    const auto& grp = train_data->group(g);
    bstart[owner[g]] = std::min(bstart[owner[g]], grp.hist_start);
    bend[owner[g]] = std::max(bend[owner[g]], grp.hist_start + grp.num_bin);
  }
  // make ranges contiguous and covering [0, total)
  int cur = 0;
  for (int i = 0; i < n; ++i) {
    int e = bend[i] > 0 ? std::max(bend[i], cur) : cur;
    block_start_[i] = static_cast<comm_size_t>(cur) * 2 * sizeof(double);
    block_len_[i] = static_cast<comm_size_t>(e - cur) * 2 * sizeof(double);
    if (i == r) {
      hist_begin_ = cur;
      hist_end_ = e;
    }
    cur = e;
  }
  // last rank absorbs any tail
  if (cur < total) {
    block_len_[n - 1] += static_cast<comm_size_t>(total - cur) * 2 * sizeof(double);
    if (r == n - 1) hist_end_ = total;
  }
  for (int f = 0; f < num_features_; ++f) feature_mask_[f] = owner[train_data->feature(f).group] == r;
}

void DataParallelTreeLearner::BeforeTrain() {
  SerialTreeLearner::BeforeTrain();
  double buf[3] = {static_cast<double>(smaller_.count), smaller_.sum_g, smaller_.sum_h};
  double out[3];
  Network::Allreduce(reinterpret_cast<char*>(buf), sizeof(buf), sizeof(double), reinterpret_cast<char*>(out),
                     Network::SumReducer<double>());
  smaller_.global_count = static_cast<data_size_t>(out[0] + 0.5);
  smaller_.sum_g = out[1];
  smaller_.sum_h = out[2];
  leaf_count_global_[0] = smaller_.global_count;
}

void DataParallelTreeLearner::ConstructHistograms(bool use_subtract) {
  const int total = train_data_->num_total_bin();
  std::vector<double> local(2 * static_cast<size_t>(total));
  auto reduce_into = [&](int leaf) {
    BuildHistogram(partition_.indices(leaf), partition_.count(leaf), local.data());
    auto& h = HistOf(leaf);
    const int r = Network::rank();
    Network::ReduceScatter(reinterpret_cast<char*>(local.data()), static_cast<comm_size_t>(local.size() * sizeof(double)),
                           sizeof(double), block_start_.data(), block_len_.data(),
                           reinterpret_cast<char*>(h.data() + 2 * static_cast<size_t>(hist_begin_)), block_len_[r],
                           Network::SumReducer<double>());
  };
  reduce_into(smaller_.leaf);
  if (larger_.leaf >= 0 && !use_subtract) reduce_into(larger_.leaf);
}

void DataParallelTreeLearner::SyncBestSplits() {
  best_split_per_leaf_[smaller_.leaf] = AllgatherBestSplit(best_split_per_leaf_[smaller_.leaf]);
  if (larger_.leaf >= 0) best_split_per_leaf_[larger_.leaf] = AllgatherBestSplit(best_split_per_leaf_[larger_.leaf]);
}

// ============================================================================
void VotingParallelTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  global_counts_from_split_ = true;
}

void VotingParallelTreeLearner::BeforeTrain() {
  SerialTreeLearner::BeforeTrain();
  double buf[3] = {static_cast<double>(smaller_.count), smaller_.sum_g, smaller_.sum_h};
  double out[3];
  Network::Allreduce(reinterpret_cast<char*>(buf), sizeof(buf), sizeof(double), reinterpret_cast<char*>(out),
                     Network::SumReducer<double>());
  smaller_.global_count = static_cast<data_size_t>(out[0] + 0.5);
  smaller_.sum_g = out[1];
  smaller_.sum_h = out[2];
  leaf_count_global_[0] = smaller_.global_count;
}

std::vector<int> VotingParallelTreeLearner::Vote(const std::vector<SplitInfo>& local_best, int top_k) {
  // local top-k features by gain
  std::vector<int> order(num_features_);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return local_best[a].BetterThan(local_best[b]); });
  struct Cand {
    int feature;
    double gain;
  };
  std::vector<Cand> mine(top_k, Cand{-1, kMinScore});
  for (int i = 0; i < top_k && i < num_features_; ++i) {
    if (local_best[order[i]].feature >= 0) mine[i] = {order[i], local_best[order[i]].gain};
  }
  const int n = Network::num_machines();
  std::vector<Cand> all(static_cast<size_t>(top_k) * n);
  Network::Allgather(reinterpret_cast<char*>(mine.data()), static_cast<comm_size_t>(sizeof(Cand) * top_k),
                     reinterpret_cast<char*>(all.data()));
  // global voting: number of votes, ties broken by summed gain then feature index
  std::vector<double> votes(num_features_, 0.0), gains(num_features_, 0.0);
  for (auto& c : all) {
    if (c.feature < 0) continue;
    votes[c.feature] += 1.0;
    gains[c.feature] += c.gain;
  }
  std::vector<int> cand;
  for (int f = 0; f < num_features_; ++f) if (votes[f] > 0) cand.push_back(f);
  std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) {
    if (votes[a] != votes[b]) return votes[a] > votes[b];
    if (gains[a] != gains[b]) return gains[a] > gains[b];
    return a < b;
  });
  if (static_cast<int>(cand.size()) > 2 * top_k) cand.resize(2 * top_k);
  std::sort(cand.begin(), cand.end());
  return cand;
}

void VotingParallelTreeLearner::ReduceGroups(const std::vector<int>& features, int leaf) {
  // sum the groups of the elected features across ranks (in place in hist_[leaf])
  std::vector<int> groups;
  for (int f : features) groups.push_back(train_data_->feature(f).group);
  std::sort(groups.begin(), groups.end());
  groups.erase(std::unique(groups.begin(), groups.end()), groups.end());
  auto& h = HistOf(leaf);
  std::vector<double> buf;
  for (int g : groups) {
    const auto& grp = train_data_->group(g);
    buf.insert(buf.end(), h.begin() + 2 * grp.hist_start, h.begin() + 2 * (grp.hist_start + grp.num_bin));
  }
  if (buf.empty()) return;
  std::vector<double> out(buf.size());
  Network::Allreduce(reinterpret_cast<char*>(buf.data()), static_cast<comm_size_t>(buf.size() * sizeof(double)),
                     sizeof(double), reinterpret_cast<char*>(out.data()), Network::SumReducer<double>());
  size_t p = 0;
  for (int g : groups) {
    const auto& grp = train_data_->group(g);
    std::copy(out.begin() + p, out.begin() + p + 2 * grp.num_bin, h.begin() + 2 * grp.hist_start);
    p += 2 * grp.num_bin;
  }
}

void VotingParallelTreeLearner::FindBestSplitsFromHistograms(const Tree* tree, bool use_subtract) {
  const int n = Network::num_machines();
  const bool has_larger = larger_.leaf >= 0;
  // histograms in hist_ are LOCAL here; keep local copies, reduce elected groups into scratch
  const double* hs = HistOf(smaller_.leaf).data();
  if (use_subtract && has_larger) {
    double* hl = HistOf(larger_.leaf).data();
    for (size_t j = 0; j < hist_[larger_.leaf].size(); ++j) hl[j] -= hs[j];
  }
  // local leaf statistics
  auto local_stat = [&](const LeafStat& g) {
    LeafStat l = g;
    ComputeLeafSums(partition_.indices(g.leaf), partition_.count(g.leaf), &l.sum_g, &l.sum_h);
    l.count = l.global_count = partition_.count(g.leaf);
    return l;
  };
  LeafStat ls = local_stat(smaller_);
  LeafStat ll = has_larger ? local_stat(larger_) : LeafStat();
  // local scan with min_data / min_hessian scaled by 1/num_machines
  Config local_cfg = *config_;
  local_cfg.min_data_in_leaf = std::max(1, config_->min_data_in_leaf / n);
  local_cfg.min_sum_hessian_in_leaf = config_->min_sum_hessian_in_leaf / n;
  const Config* saved = config_;
  config_ = &local_cfg;
  std::vector<SplitInfo> bs(num_features_), bl(num_features_);
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  for (int f = 0; f < num_features_; ++f) {
    bs[f].Reset();
    bl[f].Reset();
    if (!bytree[f]) continue;
    bool sp;
    bs[f] = BestSplitForFeature(hs, f, ls, ParentOutput(tree, smaller_), bounds_[smaller_.leaf], &sp);
    if (has_larger) bl[f] = BestSplitForFeature(HistOf(larger_.leaf).data(), f, ll, ParentOutput(tree, larger_),
                                                bounds_[larger_.leaf], &sp);
  }
  config_ = saved;
  const int top_k = std::min(config_->top_k, num_features_);
  std::vector<int> elected_s = Vote(bs, top_k);
  std::vector<int> elected_l = has_larger ? Vote(bl, top_k) : std::vector<int>();
  // global histograms of the elected features only (copies, local ones stay for subtraction)
  std::vector<double> local_s = hist_[smaller_.leaf];
  std::vector<double> local_l = has_larger ? hist_[larger_.leaf] : std::vector<double>();
  ReduceGroups(elected_s, smaller_.leaf);
  if (has_larger) ReduceGroups(elected_l, larger_.leaf);
  SplitInfo best_s, best_l;
  best_s.Reset();
  best_l.Reset();
  std::vector<int8_t> node_s = col_sampler_.GetByNode(tree, smaller_.leaf);
  for (int f : elected_s) {
    bool sp;
    SplitInfo s = BestSplitForFeature(HistOf(smaller_.leaf).data(), f, smaller_, ParentOutput(tree, smaller_),
                                      bounds_[smaller_.leaf], &sp);
    if (node_s[f] && s.feature >= 0 && s.BetterThan(best_s)) best_s = s;
  }
  if (has_larger) {
    std::vector<int8_t> node_l = col_sampler_.GetByNode(tree, larger_.leaf);
    for (int f : elected_l) {
      bool sp;
      SplitInfo s = BestSplitForFeature(HistOf(larger_.leaf).data(), f, larger_, ParentOutput(tree, larger_),
                                        bounds_[larger_.leaf], &sp);
      if (node_l[f] && s.feature >= 0 && s.BetterThan(best_l)) best_l = s;
    }
  }
  // restore local histograms for future subtraction
  hist_[smaller_.leaf] = std::move(local_s);
  if (has_larger) hist_[larger_.leaf] = std::move(local_l);
  best_split_per_leaf_[smaller_.leaf] = AllgatherBestSplit(best_s);
  if (has_larger) best_split_per_leaf_[larger_.leaf] = AllgatherBestSplit(best_l);
}

std::unique_ptr<TreeLearner> CreateLinearTreeLearner(const Config* config);

}  // namespace lgap
