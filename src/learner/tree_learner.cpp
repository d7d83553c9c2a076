// TreeLearner factory (reference src/treelearner/tree_learner.cpp:15-57).
// device_type=cpu -> host learners. device_type=gpu|cuda -> the device-resident
// HIP learner, or — when a split policy only the host learners implement is
// requested — the host learner of that type with HIP histograms (the
// reference's GPUTreeLearner arrangement). Fails loudly when no MI355X is
// visible: no silent CPU fallback.
#include "lgap/tree_learner.h"

#include <cstdlib>

#include "lgap/device_api.h"
#include "lgap/log.h"
#include "parallel_tree_learner.h"
#include "serial_tree_learner.h"

namespace lgap {

namespace {

std::unique_ptr<TreeLearner> CreateHost(const std::string& learner_type, bool linear_tree, const Config* config) {
  if (linear_tree) return CreateLinearTreeLearner(config);
  if (learner_type == "serial") return std::make_unique<SerialTreeLearner>(config);
  if (learner_type == "feature") return std::make_unique<FeatureParallelTreeLearner>(config);
  if (learner_type == "data") return std::make_unique<DataParallelTreeLearner>(config);
  if (learner_type == "voting") return std::make_unique<VotingParallelTreeLearner>(config);
  Log::Fatal("Unknown tree learner type %s", learner_type.c_str());
  return nullptr;
}

// The device learner keeps one fp64 (g, h) histogram per open leaf (2 x 8 bytes per bin,
// device_learner.hip slots; the frontier engine adds its speculation slots inside an 8 GiB
// cap). When num_leaves of them exceed half of the device memory, training takes the host
// learner, whose LRU pool bounds the live histograms and rebuilds evicted ones from rows
// (reference feature_histogram.hpp HistogramPool), with the histograms still built by the HIP
// kernels. histogram_pool_size stays what it is in the reference, a bound on the HOST cache: it
// does not move device training to the host policy (288 GB of HBM per MI355X hold the device
// histograms of any realistic num_leaves).
bool DeviceHistogramsExceedPool(const Config* c, const Dataset* train) {
  if (train == nullptr) return false;
  const double per_leaf = 16.0 * static_cast<double>(std::max(1, train->num_total_bin()));
  const double need = per_leaf * std::max(2, c->num_leaves);
  double budget = 0.5 * static_cast<double>(device::DeviceTotalMemory());
  // LGAP_DEVICE_HIST_BUDGET_MB: a smaller device budget (tests of the pooled route)
  if (const char* e = std::getenv("LGAP_DEVICE_HIST_BUDGET_MB")) budget = std::atof(e) * 1024.0 * 1024.0;
  return budget > 0 && need > budget;
}

// Why the device-resident learner cannot serve `config` (nullptr = it can).
const char* HostPolicyReason(const std::string& learner_type, bool linear_tree, const Config* c,
                             const Dataset* train) {
  if (DeviceHistogramsExceedPool(c, train)) return "per-leaf device histograms above the histogram pool";
  // linear leaves: on the device (MFMA Gram systems) within its shape, else the host learner
  if (linear_tree && !device::LinearOnDevice(c, train, learner_type)) return "linear_tree";
  // voting with extra trees on the device: the global pass redraws each elected feature's threshold
  // from the per-feature streams, which stay identical on every rank only when no draw depends on
  // local data (categorical draws count the local histogram's used bins)
  if (learner_type == "voting" && c->extra_trees) {
    // the frontier's global-pass redraws run over the in-kernel xGMI exchange only (the
    // host-staged / RCCL collectives path of this combination is not tree-equal to the host)
    const char* t = std::getenv("LGAP_DP_TRANSPORT");
    const char* h = std::getenv("LGAP_DEVICE_DP_TRANSPORT");
    if ((t != nullptr && std::string(t) != "auto" && std::string(t) != "xgmi") ||
        (h != nullptr && std::string(h) == "host" && !(t != nullptr && std::string(t) == "xgmi"))) {
      return "voting-parallel with extra_trees over collectives";
    }
    // (with the CEGB split penalty as well the device and host voting learners part after a few
    // trees: not verified tree-equal, so the host policy keeps it)
    if (CegbPenalty::Enabled(c)) return "voting-parallel with extra_trees and CEGB";
  }
  if (learner_type == "voting" && c->extra_trees && train != nullptr) {
    for (int f = 0; f < train->num_features(); ++f) {
      if (train->feature(f).bin_type != BinType::Numerical) return "voting-parallel with extra_trees and categorical features";
    }
  }
  // CEGB: the split penalty runs in the device scans, the coupled and lazy feature penalties
  // in the frontier engine (serial learner: the select's replay refunds leaves and voids
  // speculation on a feature's first use; per-row marks count each node's unmarked rows).
  // Forced splits also run on the frontier only. Both route by the frontier's own shape
  // predicate (device::FrontierServes: the select / scan LDS and node capacity), so a
  // configuration the frontier cannot hold trains under the host policy instead of failing.
  const bool feature_pens = !c->cegb_penalty_feature_coupled.empty() || !c->cegb_penalty_feature_lazy.empty();
  const bool needs_frontier = feature_pens || !c->forcedsplits_filename.empty();
  const bool frontier_ok = needs_frontier && device::FrontierServes(c, train, learner_type) &&
                           (!feature_pens || ((train == nullptr || train->num_features() <= 8192) &&
                                              c->interaction_constraints_vector.empty()));
  if (feature_pens && !frontier_ok) {
    return "cost-effective gradient boosting (feature penalties)";
  }
  if (!c->forcedsplits_filename.empty() && !frontier_ok) return "forced splits";
  // intermediate monotone constraints: the frontier select walks the constraints and re-scans the
  // leaves they tighten (device::FrontierServesMonoInter); advanced keeps the host walk
  if (!c->monotone_constraints.empty() && c->monotone_constraints_method != "basic" &&
      (linear_tree || !device::FrontierServesMonoInter(c, train, learner_type))) {
    return "intermediate/advanced monotone constraints (device scans, host constraint walk)";
  }
  // (more than 64 sets: the frontier's multi-word masks, up to 256; the sequential chain holds 64.
  // By-node sampling: the frontier's select draws each node's mask over its own allowed pool)
  if (!c->interaction_constraints_vector.empty() &&
      ((c->feature_fraction_bynode < 1.0 && !device::FrontierServesByNode(c, train, learner_type)) ||
       (c->interaction_constraints_vector.size() > 64 && !device::FrontierServes(c, train, learner_type)))) {
    return "interaction constraints with by-node sampling / more than 64 sets off the frontier";
  }
  return nullptr;
}

// Intermediate / advanced monotone constraints keep the leaves' histograms on the device and scan
// them there (SerialTreeLearner::EnableDeviceScans, device/policy_scan.h): the serial learner's
// constraint walk runs on the host between device launches. Extra-trees draws (which read the
// host histogram) and forced splits keep the host scans.
bool DeviceScansServe(const std::string& learner_type, bool linear_tree, const Config* c, const Dataset* train) {
  return learner_type == "serial" && !linear_tree && !c->monotone_constraints.empty() &&
         c->monotone_constraints_method != "basic" && !c->extra_trees && c->forcedsplits_filename.empty() &&
         !DeviceHistogramsExceedPool(c, train);
}

}  // namespace

std::unique_ptr<TreeLearner> TreeLearner::Create(const std::string& learner_type, const std::string& device_type,
                                                 bool linear_tree, const Config* config, const Dataset* train) {
  if (device_type == "gpu" || device_type == "cuda") {
    if (device::DeviceCount() <= 0) {
      Log::Fatal("device_type=%s requested but no AMD GPU (gfx950) is visible to HIP", device_type.c_str());
    }
    const char* why = HostPolicyReason(learner_type, linear_tree, config, train);
    if (why == nullptr) return device::CreateDeviceTreeLearner(config, learner_type);
    Log::Info("%s: host split policy over HIP histograms", why);
    auto learner = CreateHost(learner_type, linear_tree, config);
    auto* serial = static_cast<SerialTreeLearner*>(learner.get());
    serial->EnableDeviceHistograms();
    if (DeviceScansServe(learner_type, linear_tree, config, train)) serial->EnableDeviceScans();
    // routed here by the histogram bound: keep the host pool within the same budget
    if (DeviceHistogramsExceedPool(config, train) && config->histogram_pool_size <= 0) {
      double mb = 0.5 * static_cast<double>(device::DeviceTotalMemory()) / (1024.0 * 1024.0);
      if (const char* e = std::getenv("LGAP_DEVICE_HIST_BUDGET_MB")) mb = std::atof(e);
      serial->SetHistPoolBudgetMB(mb);
    }
    return learner;
  }
  if (device_type != "cpu") Log::Fatal("Unknown device type %s", device_type.c_str());
  return CreateHost(learner_type, linear_tree, config);
}

}  // namespace lgap
