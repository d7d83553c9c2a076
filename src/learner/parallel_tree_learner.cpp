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
// Global voting of voting_parallel_tree_learner.cpp:150-181 (GlobalVoting): every rank's
// local top-k records are weighted by (left + right count) / (global leaf count / P); each
// feature keeps its best weighted record (first in gather order on ties); the top_k
// features by (weighted gain desc, feature asc) are elected. Returned sorted by feature.
// Shared with the device learner, which evaluates the same rule in k_vote_pack.
std::vector<int> ElectFeatures(const VoteRecord* recs, int num_recs, int top_k, data_size_t global_count,
                               int num_machines) {
  const float mean = static_cast<float>(global_count) / static_cast<float>(num_machines);
  std::vector<std::pair<double, int>> best;  // (weighted gain, feature), first-seen order
  for (int i = 0; i < num_recs; ++i) {
    const VoteRecord& r = recs[i];
    if (r.feature < 0) continue;
    const double w = r.gain * r.count / mean;
    auto it = std::find_if(best.begin(), best.end(), [&](const std::pair<double, int>& b) { return b.second == r.feature; });
    if (it == best.end()) {
      if (w > kMinScore) best.emplace_back(w, r.feature);
    } else if (w > it->first) {
      it->first = w;
    }
  }
  std::stable_sort(best.begin(), best.end(), [](const std::pair<double, int>& a, const std::pair<double, int>& b) {
    if (a.first != b.first) return a.first > b.first;
    return a.second < b.second;
  });
  std::vector<int> out;
  for (size_t i = 0; i < best.size() && static_cast<int>(i) < top_k; ++i) out.push_back(best[i].second);
  std::sort(out.begin(), out.end());
  return out;
}

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

std::vector<int> VotingParallelTreeLearner::Vote(const std::vector<SplitInfo>& local_best, int top_k,
                                                data_size_t global_count) {
  const int n = Network::num_machines();
  // local top-k by (gain desc, feature asc): ArrayArgs::MaxK of voting_parallel_tree_learner.cpp:354
  std::vector<int> order(num_features_);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return local_best[a].BetterThan(local_best[b]); });
  std::vector<VoteRecord> mine(top_k);
  for (int i = 0; i < top_k; ++i) {
    const SplitInfo& s = local_best[order[i]];
    if (s.feature >= 0) mine[i] = VoteRecord{s.gain, s.feature, s.left_count + s.right_count, 0};
  }
  std::vector<VoteRecord> all(static_cast<size_t>(top_k) * n);
  Network::Allgather(reinterpret_cast<char*>(mine.data()), static_cast<comm_size_t>(sizeof(VoteRecord) * top_k),
                     reinterpret_cast<char*>(all.data()));
  return ElectFeatures(all.data(), static_cast<int>(all.size()), top_k, global_count, n);
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
  // local scan with min_data / min_hessian divided by num_machines (voting_parallel_tree_learner.cpp:61-63;
  // integer division as in the reference); no split penalties in the local pass
  Config local_cfg = *config_;
  local_cfg.min_data_in_leaf = config_->min_data_in_leaf / n;
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
    bs[f] = BestSplitForFeature(hs, f, ls, ParentOutput(tree, ls), bounds_[smaller_.leaf], nullptr, &sp);
    if (has_larger) bl[f] = BestSplitForFeature(HistOf(larger_.leaf).data(), f, ll, ParentOutput(tree, ll),
                                                bounds_[larger_.leaf], nullptr, &sp);
  }
  config_ = saved;
  const int top_k = std::min(config_->top_k, num_features_);
  std::vector<int> elected_s = Vote(bs, top_k, smaller_.global_count);
  std::vector<int> elected_l = has_larger ? Vote(bl, top_k, larger_.global_count) : std::vector<int>();
  // global histograms of the elected features only (copies, local ones stay for subtraction)
  std::vector<double> local_s = hist_[smaller_.leaf];
  std::vector<double> local_l = has_larger ? hist_[larger_.leaf] : std::vector<double>();
  ReduceGroups(elected_s, smaller_.leaf);
  if (has_larger) ReduceGroups(elected_l, larger_.leaf);
  SplitInfo best_s, best_l;
  best_s.Reset();
  best_l.Reset();
  std::vector<int8_t> node_s = col_sampler_.GetByNode(tree, smaller_.leaf);
  // global pass over the elected features: global sums and counts, split penalties applied
  // (FindBestSplitsFromHistograms of the reference's voting learner)
  for (int f : elected_s) {
    bool sp;
    SplitInfo s = ScoreFeature(tree, HistOf(smaller_.leaf).data(), f, smaller_, ParentOutput(tree, smaller_), &sp);
    if (node_s[f] && s.feature >= 0 && s.BetterThan(best_s)) best_s = s;
  }
  if (has_larger) {
    std::vector<int8_t> node_l = col_sampler_.GetByNode(tree, larger_.leaf);
    for (int f : elected_l) {
      bool sp;
      SplitInfo s = ScoreFeature(tree, HistOf(larger_.leaf).data(), f, larger_, ParentOutput(tree, larger_), &sp);
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
