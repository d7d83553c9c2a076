// TreeLearner factory (reference src/treelearner/tree_learner.cpp:15-57).
// device_type=cpu -> host learners; device_type=gpu|cuda -> the HIP learner
// (fails loudly when no MI355X is visible: no silent CPU fallback).
#include "lgap/tree_learner.h"

#include "lgap/device_api.h"
#include "lgap/log.h"
#include "parallel_tree_learner.h"
#include "serial_tree_learner.h"

namespace lgap {

std::unique_ptr<TreeLearner> TreeLearner::Create(const std::string& learner_type, const std::string& device_type,
                                                 bool linear_tree, const Config* config) {
  if (device_type == "gpu" || device_type == "cuda") {
    if (device::DeviceCount() <= 0) {
      Log::Fatal("device_type=%s requested but no AMD GPU (gfx950) is visible to HIP", device_type.c_str());
    }
    if (linear_tree) Log::Fatal("linear_tree is not supported by the HIP learner yet; use device_type=cpu");
    return device::CreateDeviceTreeLearner(config, learner_type);
  }
  if (device_type != "cpu") Log::Fatal("Unknown device type %s", device_type.c_str());
  if (linear_tree) return CreateLinearTreeLearner(config);
  if (learner_type == "serial") return std::make_unique<SerialTreeLearner>(config);
  if (learner_type == "feature") return std::make_unique<FeatureParallelTreeLearner>(config);
  if (learner_type == "data") return std::make_unique<DataParallelTreeLearner>(config);
  if (learner_type == "voting") return std::make_unique<VotingParallelTreeLearner>(config);
  Log::Fatal("Unknown tree learner type %s", learner_type.c_str());
}

}  // namespace lgap
