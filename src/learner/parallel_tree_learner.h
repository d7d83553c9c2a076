// Host parallel tree learners over the Network collectives (reference:
// feature_parallel_tree_learner.cpp, data_parallel_tree_learner.cpp,
// voting_parallel_tree_learner.cpp, parallel_tree_learner.h:209-232).
#pragma once

#include <memory>
#include <vector>

#include "serial_tree_learner.h"

namespace lgap {

// Every rank holds all rows; features are split across ranks; the global best
// split is agreed with an allgather of SplitInfo records.
class FeatureParallelTreeLearner : public SerialTreeLearner {
 public:
  explicit FeatureParallelTreeLearner(const Config* config) : SerialTreeLearner(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;

 protected:
  void SyncBestSplits() override;
};

// Rows sharded across ranks. Root sums are allreduced; the smaller leaf's
// histogram is reduce-scattered by (bin-balanced, contiguous) feature-group
// ownership; each rank scans the groups it owns; the best split is agreed
// with an allgather of SplitInfo; child counts are global.
class DataParallelTreeLearner : public SerialTreeLearner {
 public:
  explicit DataParallelTreeLearner(const Config* config) : SerialTreeLearner(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;

 protected:
  void BeforeTrain() override;
  void ConstructHistograms(bool use_subtract) override;
  void SyncBestSplits() override;
  std::vector<comm_size_t> block_start_, block_len_;  // bytes, per rank
};

// PV-Tree: local top-k voting, then only the elected features' histograms are
// reduced (voting_parallel_tree_learner.cpp:22-514).
class VotingParallelTreeLearner : public SerialTreeLearner {
 public:
  explicit VotingParallelTreeLearner(const Config* config) : SerialTreeLearner(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;

 protected:
  void BeforeTrain() override;
  void FindBestSplitsFromHistograms(const Tree* tree, bool use_subtract) override;
  std::vector<int> Vote(const std::vector<SplitInfo>& local_best, int top_k, data_size_t global_count);
  void ReduceGroups(const std::vector<int>& features, int leaf);
};

// One rank's local top-k candidate of the voting learner (LightSplitInfo analogue,
// split_info.hpp:199-262): gain and left + right count of a feature's best local split.
struct VoteRecord {
  double gain = kMinScore;
  int feature = -1;
  int count = 0;
  int pad = 0;
};
std::vector<int> ElectFeatures(const VoteRecord* recs, int num_recs, int top_k, data_size_t global_count,
                               int num_machines);

// Piecewise-linear leaves (linear_tree_learner.cpp): serial tree structure,
// then a ridge fit of each leaf on its branch's numerical features.
std::unique_ptr<TreeLearner> CreateLinearTreeLearner(const Config* config);

// Helper shared by the parallel learners: allgather one SplitInfo per rank and
// return the best (higher gain, then smaller feature index).
SplitInfo AllgatherBestSplit(const SplitInfo& mine);

}  // namespace lgap
