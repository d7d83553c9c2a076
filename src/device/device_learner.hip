// HIP leaf-wise tree learner for MI355X (gfx950).
//
// Data layout (device-resident for the whole training run):
//   rowbins  N x stride dwords   packed group bins of a row (histogram input:
//                                one lane per dword, so a wave reads a
//                                contiguous 256 B run of consecutive rows)
//   colbins  G x N               group-major copy (partition decisions and the
//                                split column are 1 byte/row streams)
//   gh       K x N float2        (gradient, hessian), class-major
//   idx[0/1] N ints              ping-pong row-index buffers (stable partition)
//   idx[2]   bag list            root rows when bagging
//   idx[3/4] N ints              frontier engine: depth-indexed buffers 2 and 3
//
// Two growth engines share the data layout, the split scan (split_scan.h) and the
// tree-building / score-update tail:
//
// FRONTIER engine (default for serial training; frontier.h, frontier_kernels.hip).
// A tree grows in batched ROUNDS; one round is four launches:
//   partition  stable partition of up to kFrontierKmax expansions at once (one
//              grid, decoupled look-back over 4096-row tiles, children written to
//              depth-indexed row buffers so a speculative expansion never
//              overwrites rows a committed node still owns)
//   hist       LDS fixed-point histograms of every expansion's smaller child,
//              flushed with int64 atomics at one global scale per tree
//   scan       larger = parent - smaller, best split of both children per feature
//   select     one block replays sequential best-first order EXACTLY (gain desc,
//              feature asc, leaf asc) over every computed node, commits what the
//              replay reaches, and picks the next round's expansions: the replay's
//              blocking leaf plus speculative candidates ranked by gain (adaptive
//              depth alpha from the rows the previous tree wasted)
// The result is bit-identical in structure to sequential growth; a tree takes
// ~log2(num_leaves)+a few rounds instead of num_leaves-1 split steps. The rounds
// are captured into hipGraphs (main graph for the predicted round count plus a
// 4-round continuation graph replayed until the tree is done).
//
// SEQUENTIAL engine (configurations the frontier does not hold: histogram budgets its select
// cannot hold in LDS, the distributed learners with extra trees or by-node sampling): a FIXED
// kernel sequence per split (kernels: seq_kernels.h, seq_{hist,scan,vote,partition}_kernels.hip):
//   partition  best-leaf select from the candidate table, stable partition of the
//              parent range (decoupled look-back), post-split bookkeeping: ranges,
//              sums, depth, monotone bounds, smaller / larger child, slot handoff
//   hist       LDS fixed-point histograms of the smaller child into per-block slab rows
//   scan       one workgroup per feature: slab fold (or the owner rows), parent -
//              smaller subtraction, mfb reconstruction, threshold / categorical scans
// Every launch has a fixed grid and exits early when the tree is done, so the
// sequence is captured once into a hipGraph and replayed per tree. Its distributed modes
// exchange through collectives (RCCL or the host-staged rehearsal transport).
//
// Distributed frontier modes (one rank per GPU). Default transport: the in-kernel xGMI exchange
// (FArgs::xg: pushes into the peers' IPC-mapped exchange buffers, flag handshakes in the
// producing launches' last blocks, no collective or extra launch per round); collectives
// (RCCL / host-staged) when LGAP_DP_TRANSPORT=collective or the set-up self-test fails:
//   data     owner-computes: every rank partitions / histograms its own rows, k_f_reduce adds
//            each bin into its owner's receive chunk (collectives: one exact reduce-scatter),
//            owners scan their features, the select pushes per-child bests and merges the
//            ranks' records (collectives: k_f_pair_best + all-gather). Configurations that need
//            every feature's candidates on every rank all-reduce the round's accumulators and
//            scan redundantly (LGAP_DP_PIPELINE=1 splits that all-reduce on a comm stream)
//   voting   the local pass (local sums / counts / config), the round's top-k votes exchanged,
//            the election, the elected rows summed exactly over ranks, and the global pass
//            over them (PV-Tree per round)
//   feature  every rank holds all rows and grows the same partition; each scans the
//            features of the groups it owns and the per-child bests are exchanged
//
// By-node sampling and extra trees also run on the frontier (masks / random thresholds drawn
// in the host learner's order); linear_tree leaves are fitted after the structure (fp64 MFMA
// Gram systems, linear_kernels.hip).
//
// After either engine: leaf outputs / renew (leaf_kernels.hip), then the score
// update walks the new tree in group-bin space (traverse_kernels.hip).
//
// Reference parity: serial_tree_learner.cpp:170-680 (growth loop, smaller /
// larger handling, BeforeFindBestSplit), feature_histogram.hpp:830-1057
// (threshold scans), cuda_best_split_finder.cu / cuda_histogram_constructor.cu
// (the reference's GPU learner, whose role this file fills).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "device/grad_kernels.h"
#include "device/hip_common.h"
#include "device/leaf_kernels.h"
#include "device/metric_kernels.h"
#include "device/linear_kernels.h"
#include "device/runtime_internal.h"
#include "device/frontier.h"
#include "device/policy_scan.h"
#include "device/traverse_kernels.h"
#include "device/sample_kernels.h"
#include "device/seq_kernels.h"
#include "device/split_scan.h"
#include "device/tree_kernels.h"
#include "learner/forced_splits.h"
#include "learner/linear_solve.h"
#include "learner/parallel_tree_learner.h"
#include "learner/serial_tree_learner.h"
#include "lgap/common.h"
#include "lgap/device_api.h"
#include "lgap/network.h"
#include "lgap/objective.h"
#include "lgap/rank_math.h"
#include "lgap/metric.h"
#include "lgap/split_math.h"

namespace lgap {
namespace device {
namespace {

// Kernel-variant overrides for the coverage tests and A/B runs, all in one knob:
// LGAP_KERNEL="key=value,key=value" with the keys fhist_threads (512 | 1024), hist_lds_kb (LDS
// tile budget), quant_lds32 (0 | 1), part_iters (4 | 8 | 16), hist_il (0 | 1), nibble (0: 8-bit
// rows), quant_hist (off: float histograms under quantized training), scan_global (1), scan_wave
// (1: the wave-per-item scan below its 64-feature threshold), oob_rows (2 | 4 | 8: rows per
// thread of the out-of-bag walk). Returns
// the key's value, nullptr when it is not set. Read at each use: tests change the environment
// between trainings in one process. Each key's value has its own storage (a caller may hold the
// values of several keys at once); empty items (a trailing comma) are skipped.
const char* KernelOverride(const char* key) {
  static const char* const kKeys[] = {"fhist_threads", "hist_lds_kb", "quant_lds32", "part_iters",
                                      "hist_il",       "nibble",      "quant_hist",  "scan_global",
                                      "scan_wave",     "oob_rows",    "select_merge"};
  constexpr int kNumKeys = static_cast<int>(sizeof(kKeys) / sizeof(kKeys[0]));
  thread_local std::string vals[kNumKeys];
  const char* e = std::getenv("LGAP_KERNEL");
  if (e == nullptr) return nullptr;
  const std::string s(e);
  const char* found = nullptr;
  for (size_t p = 0; p < s.size();) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    const std::string item = s.substr(p, q - p);
    p = q + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    const std::string k = item.substr(0, eq);
    int idx = -1;
    for (int i = 0; i < kNumKeys; ++i) idx = k == kKeys[i] ? i : idx;
    if (idx < 0) Log::Fatal("LGAP_KERNEL: unknown key '%s'", k.c_str());
    if (k == key) {
      vals[idx] = eq == std::string::npos ? "1" : item.substr(eq + 1);
      found = vals[idx].c_str();
    }
  }
  return found;
}


using namespace seq;  // NOLINT: the sequential chain's kernels and argument block

template <typename T>
class PinnedBuf {
 public:
  ~PinnedBuf() {
    if (p_) (void)hipHostFree(p_);
  }
  T* Get(size_t n) {
    if (n > n_) {
      if (p_) HIP_CHECK(hipHostFree(p_));
      HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_), std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault));
      n_ = n;
    }
    return p_;
  }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

// Parallel modes of the device learner (tree_learner=serial|data|feature|voting).
enum class DevParallel { kSerial, kData, kFeature, kVoting };

// Computed-node capacity of one frontier tree: every committed node (2 L - 1) plus room for
// speculation (8 L + 2 kmax, fewer when the per-node fp64 histograms would exceed ~8 GiB).
int FrontierCapacityFor(int L, int TB) {
  const long long lo = 4LL * L + 2 * kFrontierKmax, hi = 8LL * L + 2 * kFrontierKmax;
  const long long slot_bytes = 16LL * std::max(TB, 1);
  const long long fit = (8LL << 30) / slot_bytes;
  const long long c = std::max(lo, std::min({hi, fit, static_cast<long long>(kFrontierMaxNodes)}));
  return static_cast<int>(c);
}

// LDS of the frontier's k_f_scan: two full fp64 (g, h) histograms of the widest feature plus
// the categorical sort arrays (index, ctr) of both scanning waves.
size_t FrontierScanLds(int max_bin, int max_cat_bin) {
  int cat_p2 = 1;
  while (cat_p2 < max_cat_bin) cat_p2 <<= 1;
  return static_cast<size_t>(max_bin) * 4 * sizeof(double) + static_cast<size_t>(cat_p2) * 2 * (sizeof(int) + sizeof(double));
}

// Whether a tree of L leaves over TB total bins / F features fits the frontier engine's fixed
// resources: the select's LDS image of the computed nodes (plus the CEGB used flags), the node
// capacity, and the scan's LDS. LGAP_FRONTIER=0 forces the sequential chain (A/B runs). The
// learner factory routes with the same predicate (FrontierServes), so a configuration the
// frontier cannot hold takes the host split policy instead of failing at allocation.
bool FrontierShapeFits(int L, int TB, int F, int max_bin, int max_cat_bin, bool cegb_raw, bool mono_inter) {
  const char* e = std::getenv("LGAP_FRONTIER");
  if (e != nullptr && e[0] == '0') return false;
  const int C = FrontierCapacityFor(std::max(2, L), TB);
  if (C > kFrontierMaxNodes || F <= 0) return false;
  if (FrontierScanLds(max_bin, max_cat_bin) > 150 * 1024) return false;
  // (raw candidates: the CEGB used-feature flags and the by-node draws' scratch, F bytes each)
  return FrontierSelectLds(C, std::max(2, L)) + (cegb_raw ? 2 * (F + 16) : 0) +
             (mono_inter ? FrontierSelectMonoLds(C, std::max(2, L), F) : 0) <=
         150 * 1024;
}

class DeviceTreeLearner : public TreeLearner {
 public:
  DeviceTreeLearner(const Config* config, DevParallel mode)
      : config_(config), mode_(mode), data_parallel_(mode == DevParallel::kData) {}

  ~DeviceTreeLearner() override {
    if (fres_host_) (void)hipHostFree(fres_host_);
    for (auto& ev : tree_evt_) {
      if (ev) (void)hipEventDestroy(ev);
    }
    if (graph_exec_) (void)hipGraphExecDestroy(graph_exec_);
    for (auto& kv : fgraphs_) (void)hipGraphExecDestroy(kv.second);
    if (fcont_) (void)hipGraphExecDestroy(fcont_);
    if (!fx_peers_.empty()) XgmiClose(fx_local_, &fx_peers_);
    if (fx_local_) (void)hipFree(fx_local_);
    for (auto& ev : pipe_ev_) {
      if (ev) (void)hipEventDestroy(ev);
    }
    if (comm_stream_) (void)hipStreamDestroy(comm_stream_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  void Init(const Dataset* train, bool is_constant_hessian) override {
    is_const_hess_ = is_constant_hessian;
    data_ = train;
    N_ = train->num_data();
    F_ = train->num_features();
    G_ = train->num_groups();
    TB_ = train->num_total_bin();
    width_ = train->bin_width();
    stride_dw_ = train->row_stride() / 4;
    tstride_dw_ = stride_dw_;
    const bool parallel = mode_ != DevParallel::kSerial;
    if (parallel && !CommActive() && !HostStagedDP() && Network::num_machines() > 1) {
      Log::Fatal("Parallel HIP training needs an RCCL communicator (LGBM_DeviceCommInit)");
    }
    // LGAP_FORCE_DEVICE_DP=1 (or =voting) routes a single-rank run through the data-parallel (or
    // voting-parallel) path on a one-rank communicator: the configuration sets tree_learner to
    // serial for one machine, as the reference does, so a 1-GPU box needs this to run either path.
    const char* force_dp = std::getenv("LGAP_FORCE_DEVICE_DP");
    const bool force_vote = force_dp != nullptr && std::strcmp(force_dp, "voting") == 0;
    const bool forced = CommExists() && force_dp != nullptr && (force_dp[0] == '1' || force_vote);
    if (forced && mode_ == DevParallel::kSerial) {
      mode_ = force_vote ? DevParallel::kVoting : DevParallel::kData;
      data_parallel_ = !force_vote;
    }
    const bool multi = CommActive() || HostStagedDP() || forced;
    // voting: a one-rank communicator also runs the voting path (single-GPU rehearsal)
    voting_ = mode_ == DevParallel::kVoting && (multi || CommExists());
    owner_scan_ = (mode_ == DevParallel::kData || mode_ == DevParallel::kFeature) && multi;
    distributed_ = (owner_scan_ && data_parallel_) || voting_;
    device_id_ = CommExists() ? CommDevice() : std::max(0, config_->gpu_device_id);
    HIP_CHECK(hipSetDevice(device_id_));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device_id_));
    device_name_ = std::string(prop.name[0] ? prop.name : "AMD GPU") + " (" + prop.gcnArchName + ")";
    num_cu_ = prop.multiProcessorCount;
    if (!stream_) HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));

    use_dp_ = config_->gpu_use_dp;
    UploadData();
    linear_ = config_->linear_tree;
    if (linear_) {
      // linear leaves read the raw feature values (Dataset constructed with linear_tree=true)
      if (!train->has_raw() && F_ > 0) {
        Log::Fatal("linear_tree requires the Dataset to keep raw feature values (construct it with linear_tree=true)");
      }
      const auto& raw = train->raw_values();
      lin_has_nan_ = false;
      for (float v : raw) {
        if (std::isnan(v)) {
          lin_has_nan_ = true;
          break;
        }
      }
      if (!raw.empty()) lin_raw_.Upload(raw, stream_);
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    SetupOwnership();
    ResetConfig(config_);
    SetupTransport();
    Log::Info("HIP tree learner on %s: %d rows, %d features, %d groups, %d bins%s", device_name_.c_str(), N_, F_, G_,
              TB_, (owner_scan_ || voting_) ? (" (" + ParallelDesc() + ")").c_str() : "");
  }

  // Feature-group ownership of the owner-computes modes: contiguous group ranges with
  // ~equal bins per rank (the host DataParallelTreeLearner's assignment), so rank r's
  // block of the histogram is the contiguous bin range [bin_lo[r], bin_lo[r + 1]).
  void SetupOwnership() {
    P_ = (owner_scan_ || voting_) ? DpSize() : 1;
    rank_ = (owner_scan_ || voting_) ? DpRank() : 0;
    h_bin_lo_.assign(P_ + 1, TB_);
    std::vector<int> owner(G_);
    for (int g = 0; g < G_; ++g) {
      const auto& grp = data_->group(g);
      const long long mid = grp.hist_start + grp.num_bin / 2;
      owner[g] = std::min(P_ - 1, static_cast<int>(mid * P_ / std::max(1, TB_)));
    }
    // owners are non-decreasing in g: rank r owns groups [first_r, first_{r+1})
    for (int r = P_ - 1; r >= 0; --r) {
      int lo = h_bin_lo_[r + 1];
      for (int g = 0; g < G_; ++g) {
        if (owner[g] == r) {
          lo = data_->group(g).hist_start;
          break;
        }
      }
      h_bin_lo_[r] = std::min(lo, h_bin_lo_[r + 1]);
    }
    h_bin_lo_[0] = 0;
    bbin_ = 1;
    for (int r = 0; r < P_; ++r) bbin_ = std::max(bbin_, h_bin_lo_[r + 1] - h_bin_lo_[r]);
    std::vector<int> cnt(P_, 0);
    h_own_feat_.clear();
    for (int f = 0; f < F_; ++f) {
      const int r = owner_scan_ ? owner[data_->feature(f).group] : 0;
      ++cnt[r];
      if (r == rank_) h_own_feat_.push_back(f);
    }
    Fmax_ = 1;
    for (int r = 0; r < P_; ++r) Fmax_ = std::max(Fmax_, cnt[r]);
    if (!owner_scan_) Fmax_ = std::max(1, F_);
    h_own_feat_.resize(Fmax_, -1);
    const size_t kb = Round256(2 * static_cast<size_t>(Fmax_) * sizeof(SplitKey));
    const size_t ib = Round256(2 * static_cast<size_t>(Fmax_) * sizeof(SplitInfo));
    cand_key_bytes_ = static_cast<int>(kb);
    cand_stride_ = static_cast<int>(kb + ib);
    if (voting_) SetupVoting();
  }

  static size_t Round256(size_t x) { return (x + 255) & ~static_cast<size_t>(255); }

  // Voting: top-k width, the packed elected-histogram row, and the global candidate table
  // (one row of 2 x top_k positions). The xGMI exchange buffer reuses the histogram receive
  // rows (P x vcap values) and the candidate region (P x 2 top_k VoteRecs).
  void SetupVoting() {
    topk_ = std::max(1, std::min(config_->top_k, F_));
    if (topk_ > 1024 || F_ > 12000) {
      Log::Fatal("The HIP voting-parallel learner supports top_k <= 1024 and up to 12000 features "
                 "(top_k=%d, %d features); use device_type=cpu", config_->top_k, F_);
    }
    vcap_ = 2 * topk_ * 2 * std::max(1, max_bin_ - 1);
    bbin_ = vcap_ / 2;
    vcand_key_bytes_ = static_cast<int>(Round256(2 * static_cast<size_t>(topk_) * sizeof(SplitKey)));
    vcand_stride_ = vcand_key_bytes_ + static_cast<int>(Round256(2 * static_cast<size_t>(topk_) * sizeof(SplitInfo)));
    if (static_cast<size_t>(cand_stride_) < 2 * static_cast<size_t>(topk_) * sizeof(VoteRec)) {
      cand_stride_ = static_cast<int>(Round256(2 * static_cast<size_t>(topk_) * sizeof(VoteRec)));
    }
  }

  // Transport of the distributed exchanges. LGAP_DP_TRANSPORT = auto (default: the frontier's
  // xGMI in-kernel exchange when every rank maps every peer and the self-test passes, else
  // collectives) | xgmi | collective | allreduce.
  void SetupTransport() {
    if (!owner_scan_ && !voting_) return;
    const char* e = std::getenv("LGAP_DP_TRANSPORT");
    const std::string want = e ? e : "auto";
    if (want != "auto" && want != "xgmi" && want != "collective" && want != "allreduce") {
      Log::Fatal("LGAP_DP_TRANSPORT=%s: expected auto|xgmi|collective|allreduce", want.c_str());
    }
    // the distributed frontier engine: the in-kernel xGMI exchange (auto / xgmi) where its
    // exchanges are the owner histogram chunks and the per-child bests (owner-computes data
    // parallel, feature parallel); collectives otherwise (collective, allreduce, voting, raw
    // per-feature candidates)
    if (frontier_) {
      if ((want == "auto" || want == "xgmi") && (fowner_ || ffeature_ || fvoting_) && P_ <= kMaxXRanks) {
        SetupFrontierXgmi(want == "xgmi");
      }
      else if (want == "xgmi") Log::Warning("xGMI transport: this frontier configuration exchanges through collectives");
      // (TreeLearner::Create routes voting + extra trees over collectives to the host policy: the
      // frontier's global-pass redraws are verified over the in-kernel exchange only)
      if (fvoting_ && config_->extra_trees && !FrontierXg()) {
        Log::Fatal("voting-parallel with extra_trees on the device needs the xGMI transport (set up failed)");
      }
      return;
    }
    // the sequential chain (configurations the frontier does not hold) exchanges through collectives
    if (want == "xgmi") Log::Warning("xGMI transport: the sequential chain exchanges through collectives");
  }

  // The distributed frontier's in-kernel exchange (FArgs::xg): one uncached exchange buffer per
  // rank at identical offsets -- [receive chunk: kmax x owned bins x 2 words][per-child best
  // records: P x 2 kmax][root rows: P][flags: kinds x P] -- IPC-mapped by every peer, then a
  // self-test of remote atomics, stores and the handshake on every rank. Any failure on any rank
  // keeps the collectives on all ranks (fatal when LGAP_DP_TRANSPORT=xgmi asked for it).
  // Reference: data_parallel_tree_learner.cpp:284-298 (ReduceScatter of the histograms by owner),
  // :443 (SyncUpGlobalBestSplit); here both are pushes from the producing kernels.
  void SetupFrontierXgmi(bool required) {
    const size_t recv_words = std::max<size_t>(static_cast<size_t>(kFrontierKmax) * bbin_ * 2, 8192);
    ArenaLayout lay;
    fxo_recv_ = static_cast<unsigned>(lay.Add<unsigned long long>(recv_words));
    fxo_fpb_ = static_cast<unsigned>(lay.Add<FPairBest>(static_cast<size_t>(P_) * 2 * kFrontierKmax));
    fxo_root_ = static_cast<unsigned>(lay.Add<FXRoot>(kMaxXRanks));
    fxo_flag_ = static_cast<unsigned>(lay.Add<unsigned long long>(static_cast<size_t>(kFXKinds) * kMaxXRanks));
    fxo_vrec_ = fxo_vrows_ = 0;
    if (fvoting_) {
      // voting: every rank's top-k records per child, the elected rows summed over ranks
      fxo_vrec_ = lay.Add<VoteRec>(static_cast<size_t>(P_) * 2 * kFrontierKmax * topk_);
      fxo_vrows_ = lay.Add<unsigned long long>(2 * static_cast<size_t>(kFrontierKmax) * topk_ * 2 * max_bin_);
    }
    const size_t bytes = lay.bytes();
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      p = nullptr;
    }
    int ok = p != nullptr ? 1 : 0;
    if (ok) HIP_CHECK(hipMemset(p, 0, bytes));
    if (P_ > 1) ok = Network::GlobalSyncUpByMin(ok);
    auto fail = [&](const char* why) {
      if (p) (void)hipFree(p);
      fx_local_ = nullptr;
      if (required) Log::Fatal("xGMI transport: %s", why);
      Log::Warning("xGMI transport unavailable (%s); using collectives", why);
    };
    if (!ok) return fail("cannot allocate the uncached exchange buffer");
    fx_local_ = static_cast<char*>(p);
    if (!XgmiOpen(fx_local_, &fx_peers_)) return fail("peer exchange buffers could not be mapped");
    fxep_.Resize(1);
    fxep_.Zero(stream_);
    fxcnt_.Resize(kFXKinds);
    fxcnt_.Zero(stream_);
    {
      FXConf c;
      std::memset(&c, 0, sizeof(c));
      for (int q = 0; q < P_; ++q) c.peer[q] = fx_peers_[q];
      c.o_recv = fxo_recv_;
      c.o_fpb = fxo_fpb_;
      c.o_root = fxo_root_;
      c.o_flag = fxo_flag_;
      c.o_vrec = fxo_vrec_;
      c.o_vrows = fxo_vrows_;
      c.ep = fxep_.get();
      c.cnt = fxcnt_.get();
      c.timeout = static_cast<unsigned long long>(100e6 * XTimeoutSeconds());
      c.P = P_;
      c.rank = rank_;
      c.fault = std::getenv("LGAP_FAULT_INJECT") != nullptr && std::strcmp(std::getenv("LGAP_FAULT_INJECT"), "xgmi") == 0;
      fxconf_.Resize(1);
      fxconf_.Upload(&c, 1, stream_);
    }
    fxg_ = true;
    // self-test (session-0 tags, below every training tag)
    FArgs a = MakeFArgs();
    a.xsession = 0;
    DevBuf<unsigned> err(1);
    err.Zero(stream_);
    const int nvals = static_cast<int>(std::min<size_t>(recv_words / 2, 4096));
    for (int round = 0; round < 4; ++round) LaunchFrontierXSelfTest(a, round, nvals, err.get(), stream_);
    unsigned h = 0;
    err.Download(&h, 1, stream_);
    unsigned* hb = pin_bar_.Get(4);
    HIP_CHECK(hipMemcpyAsync(hb, bar_.get(), 4 * sizeof(unsigned), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    int good = h == 0u && hb[3] == 0u ? 1 : 0;
    if (!good) Log::Warning("frontier xGMI self-test on rank %d: %u wrong values, wait status %u", rank_, h, hb[3]);
    if (P_ > 1) good = Network::GlobalSyncUpByMin(good);
    if (!good) {
      fxg_ = false;
      bar_.Zero(stream_);
      HIP_CHECK(hipStreamSynchronize(stream_));
      XgmiClose(fx_local_, &fx_peers_);
      return fail("self-test failed");
    }
    InvalidateGraph();
  }

  std::string ParallelDesc() const {
    std::string m = mode_ == DevParallel::kFeature ? "feature-parallel"
                                                   : (voting_ ? "voting-parallel" : "data-parallel");
    m += ", " + std::to_string(P_) + " ranks, ";
    if (frontier_) {
      const std::string via = HostStagedDP() ? "host-staged collectives" : "RCCL";
      if (FrontierXg() && fowner_) return m + "frontier engine, owner histogram chunks + best-split push per round (xGMI in-kernel exchange)";
      if (FrontierXg() && fvoting_) return m + "frontier engine, top-k votes + elected rows per round (xGMI in-kernel exchange)";
      if (FrontierXg()) return m + "frontier engine, best-split push per round (xGMI in-kernel exchange)";
      if (fowner_) return m + "frontier engine, owner reduce-scatter + best-split all-gather per round (" + via + ")";
      if (ffeature_ || fvoting_) return m + "frontier engine, " + via;
      return m + "frontier engine, all-reduce per round (" + via + ")";
    }
    if (HostStagedDP()) return m + "host-staged collectives";
    return m + "RCCL reduce-scatter/all-gather";
  }

  void ResetConfig(const Config* config) override {
    config_ = config;
    col_sampler_.Init(data_, config_);
    L_ = std::max(2, config_->num_leaves);
    AllocState();
    InvalidateGraph();
  }

  void SetBaggingData(const data_size_t* used, data_size_t n) override {
    if (used == nullptr || n >= N_) {
      bag_cnt_ = N_;
      use_bag_ = false;
    } else {
      bag_cnt_ = n;
      use_bag_ = true;
      idx_[2].Upload(used, n, stream_);
    }
    oob_ok_ = false;  // (a host bag: no out-of-bag list, the score update walks every row)
  }

  // ---- row sampling on the device (sample_kernels.hip): the bag goes straight into idx_[2]
  bool SupportsDeviceSampling() const override { return true; }

  void DeviceSample(int plan, int iter) override {
    ScopedTimer timer("Device::Sample");
    if (plan == kSampleKeep) return;
    if (plan == kSampleAll) {
      SetBaggingData(nullptr, N_);
      return;
    }
    const int nt = SampleTiles(N_);
    if (samp_jump_.size() == 0) {
      std::vector<uint2> jt(kSampleRandBlock);
      BuildLcgJumpTable(jt.data());
      samp_jump_.Upload(jt, stream_);
      // Random(bagging_seed + block) per 1024-unit block (rows, or queries when bagging
      // by query), as SampleStrategy seeds them
      const int units = plan == kSampleBagQuery ? data_->metadata().num_queries() : N_;
      std::vector<unsigned> st(std::max(1, DivUp(units, kSampleRandBlock)));
      for (size_t b = 0; b < st.size(); ++b) st[b] = static_cast<unsigned>(config_->bagging_seed + static_cast<int>(b));
      samp_rng_.Upload(st, stream_);
      samp_cnt_.Resize(std::max(nt, 1));
      samp_sel_.Resize(4 * static_cast<size_t>(std::max(nt, 1)));
      samp_total_.Resize(1);
    }
    SampleArgs a;
    a.mode = plan == kSampleGoss ? 3 : (plan == kSampleBalanced ? 2 : (plan == kSampleBagQuery ? 4 : 1));
    if (a.mode == 4) {
      const Metadata& md = data_->metadata();
      if (row_query_.size() == 0) {
        std::vector<int> rq(std::max(N_, 1));
        const data_size_t* qb = md.query_boundaries();
        for (data_size_t q = 0; q < md.num_queries(); ++q)
          for (data_size_t i = qb[q]; i < qb[q + 1]; ++i) rq[i] = q;
        row_query_.Upload(rq, stream_);
      }
      a.row_unit = row_query_.get();
      a.num_units = md.num_queries();
    }
    a.N = N_;
    a.K = K_;
    a.fraction = config_->bagging_fraction;
    a.pos_fraction = config_->pos_bagging_fraction;
    a.neg_fraction = config_->neg_bagging_fraction;
    a.top_rate = config_->top_rate;
    a.other_rate = config_->other_rate;
    a.seed = GossSeed(config_->bagging_seed, iter);  // the host sampler's seed: identical GOSS bags
    if (a.mode == 2) {
      if (bag_label_.size() == 0) bag_label_.Upload(data_->metadata().label(), N_, stream_);
      a.label = bag_label_.get();
    }
    a.gh = gh_.get();
    a.rng = samp_rng_.get();
    a.jump = samp_jump_.get();
    a.tile_cnt = samp_cnt_.get();
    a.tile_sel = samp_sel_.get();
    a.out = idx_[2].get();
    // the frontier's score update walks only the out-of-bag rows (LeafMapScore)
    if (frontier_ && width_ >= 1 && width_ <= 2) {
      if (oob_.size() < static_cast<size_t>(N_)) oob_.Resize(std::max(N_, 1));
      a.oob = oob_.get();
    }
    a.total = samp_total_.get();
    LaunchSampleCount(a, stream_);
    LaunchSampleScatter(a, stream_);
    if (a.mode == 4) LaunchSampleAdvanceUnits(a, stream_);
    int* cnt = pin_cnt_.Get(1);
    samp_total_.Download(cnt, 1, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    if (*cnt < 0 || *cnt > N_) Log::Fatal("device sampling: invalid bag size %d", *cnt);
    bag_cnt_ = *cnt;
    use_bag_ = bag_cnt_ < N_;
    if (!use_bag_) bag_cnt_ = N_;
    oob_ok_ = a.oob != nullptr;
    Log::Debug("Device %s, using %d data to train", a.mode == 3 ? "GOSS" : "bagging", bag_cnt_);
  }

  std::unique_ptr<Tree> Train(const score_t* g, const score_t* h, bool is_first_tree) override {
    DeviceSetGradients(g, h, 1);
    return DeviceTrain(0, is_first_tree);
  }

  std::unique_ptr<Tree> FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred, const score_t* g,
                                          const score_t* h) override {
    // refit is a one-off host pass over leaf assignments; the host learner computes it (linear
    // trees: the host linear learner, which re-solves the leaf models)
    if (linear_) {
      auto host = CreateLinearTreeLearner(config_);
      host->Init(data_, false);
      return host->FitByExistingTree(old_tree, leaf_pred, g, h);
    }
    SerialTreeLearner host(config_);
    host.Init(data_, false);
    return host.FitByExistingTree(old_tree, leaf_pred, g, h);
  }

  // Refit on the device (reference cuda_single_gpu_tree_learner.cu:19-78): leaf sums of the
  // device gradients over the leaf assignment, the host's output formula, and the new
  // outputs added to the device score.
  std::unique_ptr<Tree> DeviceFitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                                int class_id) override {
    ScopedTimer timer("Device::Refit");
    if (static_cast<data_size_t>(leaf_pred.size()) != N_ || gh_.size() < static_cast<size_t>(class_id + 1) * N_ ||
        old_tree->is_linear()) {
      return nullptr;  // (linear trees: the host linear learner's refit, FitByExistingTree)
    }
    const int L = old_tree->num_leaves();
    leaf_pred_dev_.Upload(leaf_pred, stream_);
    refit_partial_.Resize(static_cast<size_t>(RefitPartialBlocks(N_)) * 3 * L);
    refit_sums_.Resize(3 * static_cast<size_t>(L));
    LaunchRefitLeafSums(gh_.get() + static_cast<size_t>(class_id) * N_, leaf_pred_dev_.get(), N_, L,
                        refit_partial_.get(), refit_sums_.get(), stream_);
    std::vector<double> sums(3 * static_cast<size_t>(L));
    refit_sums_.Download(sums.data(), sums.size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    auto tree = std::make_unique<Tree>(*old_tree);
    SplitParams p = MakeArgs().sp;
    std::vector<double> delta(L);
    for (int i = 0; i < L; ++i) {
      const double sg = sums[3 * i], sh = kEpsilon + sums[3 * i + 1];
      const data_size_t n = static_cast<data_size_t>(sums[3 * i + 2] + 0.5);
      double out;
      if (config_->path_smooth > kEpsilon && i > 0) {
        out = LeafOutputRaw(sg, sh, p, n, tree->leaf_parent(i));  // (the reference passes leaf_parent)
      } else {
        SplitParams q = p;
        q.path_smooth = 0.0;
        out = LeafOutputRaw(sg, sh, q, n, 0.0);
      }
      const double old_v = tree->LeafOutput(i);
      const double new_v = config_->refit_decay_rate * old_v + (1.0 - config_->refit_decay_rate) * out * tree->shrinkage();
      tree->SetLeafOutput(i, new_v);
      delta[i] = new_v;  // the refit score holds only the refit trees so far (GBDT::RefitTree)
    }
    refit_delta_.Upload(delta, stream_);
    FlushScore();
    LaunchAddLeafDelta(score_.get() + static_cast<size_t>(class_id) * N_, leaf_pred_dev_.get(), refit_delta_.get(), N_,
                       stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    return tree;
  }

  // L1 / quantile / MAPE leaf renewal on the device: residual percentiles over the final leaf
  // ranges of the tree just grown (bagged rows only, as the partition holds them).
  bool DeviceRenewTreeOutput(Tree* tree, const ObjectiveFunction* obj, int class_id) override {
    if (obj == nullptr || !obj->IsRenewTreeOutput()) return true;
    const PointwiseParams* pp = obj->pointwise();
    const int nl = tree->num_leaves();
    if (pp == nullptr || obj->effective_label() == nullptr || static_cast<int>(h_range_.size()) != nl) return false;
    ScopedTimer timer("Device::RenewTreeOutput");
    PrepareObjective(obj);
    std::vector<LeafSeg> segs(nl);
    std::vector<int> off(nl + 1, 0);
    for (int l = 0; l < nl; ++l) {
      segs[l].buf = h_range_[l].buf;
      segs[l].start = h_range_[l].start;
      segs[l].count = h_range_[l].count;
      segs[l].pad = 0;
      off[l + 1] = off[l] + h_range_[l].count;
    }
    const int total = off[nl];
    renew_segs_.Upload(segs, stream_);
    renew_off_.Upload(off, stream_);
    RenewArgs ra;
    FlushScore();
    ra.score = score_.get() + static_cast<size_t>(class_id) * N_;
    ra.label = label_.get();
    ra.weight = pp->kind == kPwMape ? aux_.get() : (weight_.size() ? weight_.get() : nullptr);
    for (int i = 0; i < kLeafIdxBufs; ++i) ra.idx[i] = i < kFrontierIdx ? idx_[i].get() : nullptr;
    ra.segs = renew_segs_.get();
    ra.seg_off = renew_off_.get();
    ra.num_leaves = nl;
    ra.alpha = pp->kind == kPwQuantile ? pp->alpha : 0.5;
    const size_t bytes = RenewScratchBytes(total, nl);
    if (renew_scratch_.size() < bytes) renew_scratch_.Resize(bytes);
    renew_out_.Resize(std::max<size_t>(renew_out_.size(), nl));
    renew_nz_.Resize(std::max<size_t>(renew_nz_.size(), nl));
    LaunchRenewLeaves(ra, total, renew_scratch_.get(), renew_scratch_.size(), renew_out_.get(), renew_nz_.get(),
                      stream_);
    std::vector<double> outs(nl);
    std::vector<int> nonzero(nl);
    renew_out_.Download(outs.data(), nl, stream_);
    renew_nz_.Download(nonzero.data(), nl, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int l = 0; l < nl; ++l) {
      if (!nonzero[l]) outs[l] = 0.0;
    }
    if (Network::num_machines() > 1) {
      // the reference averages the per-machine renewed outputs (serial_tree_learner.cpp:947-960)
      Network::GlobalSum(&outs);
      Network::GlobalSum(&nonzero);
      for (int l = 0; l < nl; ++l) outs[l] = nonzero[l] > 0 ? outs[l] / nonzero[l] : 0.0;
    }
    for (int l = 0; l < nl; ++l) tree->SetLeafOutput(l, outs[l]);
    return true;
  }

  void AddPredictionToScore(const Tree* tree, double* out_score) const override {
    tree->AddPredictionToScore(*data_, N_, out_score);
  }

  void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj, const double* score, data_size_t,
                       const data_size_t*, data_size_t) const override {
    if (obj == nullptr || !obj->IsRenewTreeOutput()) return;
    const int nl = tree->num_leaves();
    std::vector<double> outs(nl, 0.0);
    std::vector<int> nonzero(nl, 1);
    for (int l = 0; l < nl; ++l) {
      auto rows = LeafIndices(l);
      if (!rows.empty()) outs[l] = obj->RenewTreeOutput(tree->LeafOutput(l), score, rows.data(), static_cast<data_size_t>(rows.size()));
      else nonzero[l] = 0;
    }
    if (Network::num_machines() > 1) {
      Network::GlobalSum(&outs);
      Network::GlobalSum(&nonzero);
      for (int l = 0; l < nl; ++l) outs[l] = nonzero[l] > 0 ? outs[l] / nonzero[l] : 0.0;
    }
    for (int l = 0; l < nl; ++l) tree->SetLeafOutput(l, outs[l]);
  }

  std::vector<data_size_t> LeafIndices(int leaf) const override {
    if (leaf < 0 || leaf >= static_cast<int>(h_range_.size())) return {};
    const LeafRange r = h_range_[leaf];
    std::vector<data_size_t> out(r.count);
    if (r.count == 0) return out;
    if (r.buf < 0) {
      for (int i = 0; i < r.count; ++i) out[i] = r.start + i;
    } else {
      HIP_CHECK(hipMemcpyAsync(out.data(), idx_[r.buf].get() + r.start, sizeof(int) * r.count, hipMemcpyDeviceToHost,
                               stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    return out;
  }

  // ---- device-resident boosting
  bool OwnsScore() const override { return true; }

  bool SupportsDeviceGradients(const ObjectiveFunction* obj) const override {
    if (obj == nullptr) return false;
    switch (obj->device_kind()) {
      case DeviceGradKind::kPointwise:
        return obj->pointwise() != nullptr && obj->effective_label() != nullptr;
      case DeviceGradKind::kSoftmax:
        return obj->effective_label() != nullptr;
      case DeviceGradKind::kOVA:
        return obj->effective_label() != nullptr && obj->pointwise_class(0) != nullptr;
      case DeviceGradKind::kLambdarank:
        // any query length (long queries in global scratch), position bias included
        return data_->metadata().num_queries() > 0;
      case DeviceGradKind::kXendcg:
        // (position-biased rank_xendcg stays on the host)
        return data_->metadata().num_queries() > 0 && data_->metadata().positions() == nullptr;
      default:
        return false;
    }
  }

  void DeviceInitScore(const std::vector<double>& host_score, int num_tree_per_iter) override {
    pend_.on = false;  // (the uploaded score replaces everything)
    K_ = num_tree_per_iter;
    score_.Resize(static_cast<size_t>(K_) * N_);
    score_.Upload(host_score, stream_);
    gh_.Resize(static_cast<size_t>(K_) * N_);
    if (graph_exec_) InvalidateGraph();
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void DeviceComputeGradients(const ObjectiveFunction* obj) override {
    ScopedTimer timer("Device::ComputeGradients");
    PrepareObjective(obj);
    if (pend_.on && pend_.k == 0 && K_ == 1 && obj->device_kind() == DeviceGradKind::kPointwise) {
      // the deferred leaf add of the last tree, fused with this gradient pass
      pend_.on = false;
      LaunchLeafMapAddGrad(leaf_map_.get(), pend_lv_.get(), pend_.nl, N_, score_.get(), *obj->pointwise(), label_.get(),
                           weight_.size() ? weight_.get() : nullptr, aux_.size() ? aux_.get() : nullptr, gh_.get(),
                           num_cu_, stream_);
      return;
    }
    FlushScore();
    switch (obj->device_kind()) {
      case DeviceGradKind::kPointwise:
        LaunchPointwiseGrad(*obj->pointwise(), score_.get(), label_.get(), weight_.size() ? weight_.get() : nullptr,
                            aux_.size() ? aux_.get() : nullptr, N_, gh_.get(), stream_);
        break;
      case DeviceGradKind::kSoftmax:
        LaunchSoftmaxGrad(K_, static_cast<double>(K_) / (K_ - 1.0), score_.get(), label_.get(),
                          weight_.size() ? weight_.get() : nullptr, N_, gh_.get(), stream_);
        break;
      case DeviceGradKind::kOVA:
        LaunchOvaGrad(K_, ova_params_.get(), score_.get(), label_.get(), weight_.size() ? weight_.get() : nullptr, N_,
                      gh_.get(), stream_);
        break;
      case DeviceGradKind::kLambdarank: {
        RankKernelArgs ra = rank_args_;
        ra.score = score_.get();
        ra.gh = gh_.get();
        LaunchLambdarankGrad(ra, stream_);
        if (ra.positions) {
          LaunchPositionBiasUpdate(gh_.get(), ra.positions, N_, num_pos_ids_, pos_lr_, pos_reg_, pos_acc_.get(),
                                   pos_bias_.get(), stream_);
        }
        break;
      }
      case DeviceGradKind::kXendcg: {
        XendcgArgs xa = xendcg_args_;
        xa.score = score_.get();
        xa.gh = gh_.get();
        LaunchXendcgGrad(xa, stream_);
        break;
      }
      default:
        Log::Fatal("Objective %s has no device gradient kernel", obj->GetName());
    }
  }

  void DeviceSetGradients(const score_t* g, const score_t* h, int num_class) override {
    const size_t n = static_cast<size_t>(num_class) * N_;
    if (gh_.size() < n) gh_.Resize(n);
    float2* p = pin_gh_.Get(n);
    for (size_t i = 0; i < n; ++i) p[i] = make_float2(g[i], h[i]);
    HIP_CHECK(hipMemcpyAsync(gh_.get(), p, n * sizeof(float2), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void DeviceGetGradients(std::vector<score_t>* g, std::vector<score_t>* h) const override {
    const size_t n = static_cast<size_t>(K_) * N_;
    std::vector<float2> tmp(n);
    HIP_CHECK(hipMemcpyAsync(tmp.data(), gh_.get(), n * sizeof(float2), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    g->resize(n);
    h->resize(n);
    for (size_t i = 0; i < n; ++i) {
      (*g)[i] = tmp[i].x;
      (*h)[i] = tmp[i].y;
    }
  }

  void DeviceGetScore(std::vector<double>* out) const override {
    FlushScore();
    out->resize(static_cast<size_t>(K_) * N_);
    score_.Download(out->data(), out->size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void DeviceAddConstant(double v, int k) override {
    FlushScore();
    LaunchAddConstant(score_.get() + static_cast<size_t>(k) * N_, N_, v, stream_);
  }

  bool DeviceEvalPointwise(const PwMetricParams& p, int k, double* sum) override {
    if (score_.size() < static_cast<size_t>(k + 1) * N_ || N_ <= 0) return false;
    ScopedTimer timer("Device::EvalMetric");
    FlushScore();
    EnsureMetricLabels();
    LaunchPointwiseMetric(p, score_.get() + static_cast<size_t>(k) * N_, metric_label_.get(),
                          metric_weight_.size() ? metric_weight_.get() : nullptr, N_, metric_partial_.get(),
                          kMetricBlocks, metric_partial_.get() + kMetricBlocks, stream_);
    double* h = pin_lout_.Get(1);
    HIP_CHECK(hipMemcpyAsync(h, metric_partial_.get() + kMetricBlocks, sizeof(double), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    *sum = h[0];
    return true;
  }

  void DeviceAddTreeToScore(const Tree* tree, int k) override {
    ScopedTimer timer("Device::AddTreeToScore");
    FlushScore();
    double* s = score_.get() + static_cast<size_t>(k) * N_;
    if (tree->num_leaves() <= 1) {
      if (tree->LeafOutput(0) != 0.0) LaunchAddConstant(s, N_, tree->LeafOutput(0), stream_);
      return;
    }
    if (tree->is_linear()) {
      TraverseLinear(tree, s);
      return;
    }
    const bool fresh = tree == last_trained_;
    last_trained_ = nullptr;
    if (fresh && frontier_ && (!use_bag_ || oob_ok_) && LeafMapScore(tree, k)) return;
    TraverseTree(tree, rowbins_.get(), N_, s);
  }

  // Score update from the leaf ranges of the frontier tree just grown (traverse_kernels.h
  // LaunchLeafMap): every trained row sits in exactly one leaf's index segment, so the rows'
  // leaves come from those segments instead of a walk of the tree over the packed rows. A
  // bagged / GOSS tree (reference gbdt.cpp:495-516) adds the out-of-bag list the device sampler
  // wrote (oob_) as one more segment, and only those rows walk the tree (LaunchLeafMapList).
  // The map is built here; the add itself is deferred (pend_) into the next pointwise
  // gradient pass, or flushed by the first reader of the score (FlushScore). Uploads go
  // through the traversal's staging ring (no host wait).
  bool LeafMapScore(const Tree* tree, int k) {
    const int nl = tree->num_leaves();
    const bool bag = use_bag_;
    const int nseg = nl + (bag ? 1 : 0);  // (bag: the out-of-bag rows, placeholder leaf nl)
    if (nl != static_cast<int>(h_range_.size()) || nseg > kLMMaxLeaves) return false;
    long long total = 0;
    for (const auto& r : h_range_) {
      if (r.buf < 0 || r.buf >= kFrontierIdx) return false;  // (a partitioned leaf: an index buffer)
      total += r.count;
    }
    if (total != (bag ? bag_cnt_ : N_)) return false;
    const size_t seg_bytes = Round256(sizeof(LeafSeg) * nseg), off_bytes = Round256(sizeof(int) * (nseg + 1));
    const size_t map_part = Round256(seg_bytes + off_bytes + sizeof(double) * nseg);
    const CompactLayout z = bag ? CompactTreeLayout(tree) : CompactLayout{0, 0, 0, 0};
    const size_t bytes = map_part + z.total;
    const int slot = tree_slot_++ & 1;
    if (tree_evt_[slot] == nullptr) HIP_CHECK(hipEventCreateWithFlags(&tree_evt_[slot], hipEventDisableTiming));
    else HIP_CHECK(hipEventSynchronize(tree_evt_[slot]));
    char* hp = pin_tree_ring_[slot].Get(bytes);
    LeafSeg* segs = reinterpret_cast<LeafSeg*>(hp);
    int* off = reinterpret_cast<int*>(hp + seg_bytes);
    double* lv = reinterpret_cast<double*>(hp + seg_bytes + off_bytes);
    // the frontier partition writes a right child's rows from its range's end: a leaf's rows
    // descend when it lies right of an odd number of its ancestors' splits (LeafMapArgs::segs)
    leaf_desc_.assign(nl, 0);
    std::vector<std::pair<int, int>>& stack = leaf_walk_;
    stack.assign(1, {0, 0});
    while (!stack.empty()) {
      const auto [node, par] = stack.back();
      stack.pop_back();
      const int ch[2] = {tree->left_child(node), tree->right_child(node)};
      for (int side = 0; side < 2; ++side) {
        if (ch[side] < 0) leaf_desc_[~ch[side]] = static_cast<uint8_t>(par ^ side);
        else stack.push_back({ch[side], par ^ side});
      }
    }
    off[0] = 0;
    for (int l = 0; l < nl; ++l) {
      segs[l].buf = h_range_[l].buf;
      segs[l].start = h_range_[l].start;
      segs[l].count = h_range_[l].count;
      segs[l].pad = leaf_desc_[l];
      off[l + 1] = off[l] + h_range_[l].count;
      lv[l] = tree->LeafOutput(l);
    }
    if (bag) {
      segs[nl].buf = kLeafOobBuf;
      segs[nl].start = 0;
      segs[nl].count = N_ - bag_cnt_;
      segs[nl].pad = 0;  // (ascending)
      off[nl + 1] = N_;
      lv[nl] = 0.0;
      PackCompactTree(tree, hp + map_part, z);
    }
    if (ttree_buf_.size() < bytes) {
      HIP_CHECK(hipStreamSynchronize(stream_));  // queued score updates still read the old buffer
      ttree_buf_.Resize(bytes);
    }
    HIP_CHECK(hipMemcpyAsync(ttree_buf_.get(), hp, bytes, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipEventRecord(tree_evt_[slot], stream_));
    const size_t bound_ints = LeafTileBoundsInts(N_, nseg);
    const size_t map_bytes = Round256(static_cast<size_t>(N_) * (nseg > 256 ? 2 : 1));
    if (leaf_bounds_.size() < bound_ints || leaf_map_.size() < map_bytes || pend_lv_.size() < static_cast<size_t>(kLMMaxLeaves)) {
      HIP_CHECK(hipStreamSynchronize(stream_));
      leaf_bounds_.Resize(std::max(leaf_bounds_.size(), bound_ints));
      leaf_map_.Resize(std::max(leaf_map_.size(), map_bytes));
      pend_lv_.Resize(kLMMaxLeaves);
    }
    LeafMapArgs la;
    for (int i = 0; i < kLeafIdxBufs; ++i) la.idx[i] = i < kFrontierIdx ? idx_[i].get() : nullptr;
    static_assert(kFrontierIdx <= kLeafOobBuf, "the out-of-bag list's index-buffer id");
    la.idx[kLeafOobBuf] = bag ? oob_.get() : nullptr;
    const char* db = ttree_buf_.get();
    la.segs = reinterpret_cast<const LeafSeg*>(db);
    la.seg_off = reinterpret_cast<const int*>(db + seg_bytes);
    la.leaf_value = reinterpret_cast<const double*>(db + seg_bytes + off_bytes);
    la.num_leaves = nseg;
    la.n = N_;
    LaunchLeafMap(la, leaf_bounds_.get(), leaf_map_.get(), pend_lv_.get(), stream_);
    if (bag) {
      const char* dt = db + map_part;
      const bool cols = stride_dw_ > 16 && colbins_.size() >= static_cast<size_t>(G_) * N_ * width_;
      LaunchLeafMapList(cols ? colbins_.get() : nullptr, rowbins_.get(), stride_dw_, width_, N_, oob_.get(),
                        N_ - bag_cnt_, reinterpret_cast<const TNode*>(dt), nl - 1,
                        reinterpret_cast<const TCat*>(dt + z.cat), reinterpret_cast<const uint32_t*>(dt + z.bit), nseg,
                        leaf_map_.get(), KernelOverride("oob_rows") ? std::atoi(KernelOverride("oob_rows")) : 4,
                        num_cu_, stream_);
    }
    pend_.on = true;
    pend_.k = k;
    pend_.nl = nseg;
    return true;
  }

  // the deferred leaf add of LeafMapScore, before anything reads (or adds to) the score
  void FlushScore() const {
    if (!pend_.on) return;
    pend_.on = false;
    LaunchLeafMapAdd(leaf_map_.get(), pend_lv_.get(), pend_.nl, N_, score_.get() + static_cast<size_t>(pend_.k) * N_,
                     num_cu_, stream_);
  }

  // score[i] += tree(row i) over packed rows of the training layout (training or validation set)
  void TraverseTree(const Tree* tree, const uint32_t* rowbins, int n, double* s) {
    if (tree->num_leaves() <= 1) {
      if (tree->LeafOutput(0) != 0.0) LaunchAddConstant(s, n, tree->LeafOutput(0), stream_);
      return;
    }
    if (tree->num_leaves() <= 32767) {
      TraverseTreeCompact(tree, rowbins, n, s);
      return;
    }
    const int nn = tree->num_leaves() - 1;
    const auto& cb = tree->cat_boundaries_inner();
    const auto& ct = tree->cat_threshold_inner();
    // pack nodes + leaf values + categorical words into one pinned upload
    const size_t node_bytes = sizeof(DevNode) * nn;
    const size_t leaf_bytes = sizeof(double) * tree->num_leaves();
    const size_t cat_bytes = sizeof(uint32_t) * std::max<size_t>(1, ct.size());
    const size_t total = node_bytes + leaf_bytes + cat_bytes;
    char* hp = pin_tree_.Get(total);
    DevNode* nodes = reinterpret_cast<DevNode*>(hp);
    for (int i = 0; i < nn; ++i) {
      const FeatureInfo& fi = data_->feature(tree->split_feature_inner(i));
      DevNode& d = nodes[i];
      d.group = fi.group;
      d.offset = fi.offset;
      d.num_bin = fi.num_bin;
      d.mfb = static_cast<int>(fi.mfb);
      d.default_bin = static_cast<int>(fi.default_bin);
      const int8_t dt = tree->decision_type(i);
      d.missing = Tree::GetMissingType(dt);
      d.decision = (Tree::GetDecisionType(dt, kCategoricalMask) ? 1 : 0) | (Tree::GetDecisionType(dt, kDefaultLeftMask) ? 2 : 0);
      d.left = tree->left_child(i);
      d.right = tree->right_child(i);
      if (d.decision & 1) {
        const int ci = static_cast<int>(tree->threshold_in_bin(i));
        d.cat_begin = cb[ci];
        d.cat_nwords = cb[ci + 1] - cb[ci];
        d.threshold = 0;
      } else {
        d.threshold = static_cast<int>(tree->threshold_in_bin(i));
        d.cat_begin = 0;
        d.cat_nwords = 0;
      }
    }
    double* lv = reinterpret_cast<double*>(hp + node_bytes);
    for (int l = 0; l < tree->num_leaves(); ++l) lv[l] = tree->LeafOutput(l);
    uint32_t* cw = reinterpret_cast<uint32_t*>(hp + node_bytes + leaf_bytes);
    for (size_t i = 0; i < ct.size(); ++i) cw[i] = ct[i];
    tree_buf_.Resize(std::max(tree_buf_.size(), total));
    HIP_CHECK(hipMemcpyAsync(tree_buf_.get(), hp, total, hipMemcpyHostToDevice, stream_));
    const DevNode* dn = reinterpret_cast<const DevNode*>(tree_buf_.get());
    const double* dl = reinterpret_cast<const double*>(tree_buf_.get() + node_bytes);
    const uint32_t* dc = reinterpret_cast<const uint32_t*>(tree_buf_.get() + node_bytes + leaf_bytes);
    const int grid = std::min(DivUp(n, kTraverseThreads), num_cu_ * 8);
    const int sdw = StrideOf(rowbins);
    const size_t lds = node_bytes + (sdw <= kTraverseMaxDw ? sizeof(uint32_t) * kTraverseThreads * sdw : 0);
    k_add_tree<<<std::max(grid, 1), kTraverseThreads, lds, stream_>>>(rowbins, sdw, width_, n, dn, nn, dc, dl, s);
    HIP_CHECK(hipGetLastError());
    // the pinned staging buffer is reused by the next call: wait for the copy
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  // Compact tree staging (traverse_kernels.h TNode / TCat): offsets of the nodes, the
  // categorical node data, the leaf values and the categorical words in one upload
  struct CompactLayout {
    size_t cat, leaf, bit, total;
  };
  static CompactLayout CompactTreeLayout(const Tree* tree) {
    const int nn = tree->num_leaves() - 1, nl = tree->num_leaves();
    const size_t node_bytes = Round256(sizeof(TNode) * nn), cat_bytes = Round256(sizeof(TCat) * nn);
    const size_t leaf_bytes = Round256(sizeof(double) * nl);
    const size_t bit_bytes = sizeof(uint32_t) * std::max<size_t>(1, tree->cat_threshold_inner().size());
    CompactLayout z;
    z.cat = node_bytes;
    z.leaf = z.cat + cat_bytes;
    z.bit = z.leaf + leaf_bytes;
    z.total = z.bit + bit_bytes;
    return z;
  }
  void PackCompactTree(const Tree* tree, char* hp, const CompactLayout& z) const {
    const int nn = tree->num_leaves() - 1, nl = tree->num_leaves();
    const auto& cb = tree->cat_boundaries_inner();
    const auto& ct = tree->cat_threshold_inner();
    TNode* nodes = reinterpret_cast<TNode*>(hp);
    TCat* cats = reinterpret_cast<TCat*>(hp + z.cat);
    for (int i = 0; i < nn; ++i) {
      const FeatureInfo& fi = data_->feature(tree->split_feature_inner(i));
      const int8_t dt = tree->decision_type(i);
      const int missing = Tree::GetMissingType(dt);
      const bool dleft = Tree::GetDecisionType(dt, kDefaultLeftMask);
      const int offset = fi.offset, nb = fi.num_bin, mfb = static_cast<int>(fi.mfb);
      TNode& d = nodes[i];
      std::memset(&d, 0, sizeof(d));
      d.group = static_cast<uint16_t>(fi.group);
      d.left = static_cast<int16_t>(tree->left_child(i));
      d.right = static_cast<int16_t>(tree->right_child(i));
      d.gmiss = -1;
      if (Tree::GetDecisionType(dt, kCategoricalMask)) {
        const int ci = static_cast<int>(tree->threshold_in_bin(i));
        d.flags = kTCat;
        TCat& c = cats[i];
        c.offset = offset;
        c.num_bin = nb;
        c.mfb = mfb;
        c.begin = cb[ci];
        c.nwords = cb[ci + 1] - cb[ci];
        c.pad = 0;
        continue;
      }
      const int thr = static_cast<int>(tree->threshold_in_bin(i));
      const int bmiss = missing == 1 ? static_cast<int>(fi.default_bin) : (missing == 2 ? nb - 1 : -1);
      // stored feature bins k = 0 .. nb - 2 sit at group bins offset + k (the mfb is implicit)
      d.lo = static_cast<uint16_t>(offset);
      d.hi = static_cast<uint16_t>(offset + nb - 2);
      const bool out_left = bmiss == mfb ? dleft : (mfb <= thr);
      if (bmiss >= 0 && bmiss != mfb) d.gmiss = static_cast<int16_t>(offset + (bmiss < mfb ? bmiss : bmiss - 1));
      // last group bin whose feature bin is <= thr; below `offset` (thr == mfb == 0) no stored bin
      // goes left, and tg = 0 makes `gb <= tg` false for every in-range bin (offset >= 1)
      const int tg = offset + (thr < mfb ? thr : thr - 1);
      d.tg = static_cast<uint16_t>(tg < offset ? 0 : tg);
      d.flags = static_cast<uint8_t>((out_left ? kTOutLeft : 0) | (dleft ? kTDefaultLeft : 0));
    }
    double* lv = reinterpret_cast<double*>(hp + z.leaf);
    for (int l = 0; l < nl; ++l) lv[l] = tree->LeafOutput(l);
    uint32_t* cw = reinterpret_cast<uint32_t*>(hp + z.bit);
    for (size_t i = 0; i < ct.size(); ++i) cw[i] = ct[i];
  }

  // Compact traversal (traverse_kernels.h): node predicates precomputed in group-bin space.
  void TraverseTreeCompact(const Tree* tree, const uint32_t* rowbins, int n, double* s) {
    const int nn = tree->num_leaves() - 1, nl = tree->num_leaves();
    const CompactLayout z = CompactTreeLayout(tree);
    const size_t node_bytes = z.cat, cat_bytes = z.leaf - z.cat, leaf_bytes = z.bit - z.leaf, total = z.total;
    // staging ring: the host fills one pinned buffer while the copy out of the other may still
    // be queued, so the score update returns without waiting for the GPU (the next iteration's
    // launches queue behind the traversal instead of after a host round trip)
    const int slot = tree_slot_++ & 1;
    if (tree_evt_[slot] == nullptr) HIP_CHECK(hipEventCreateWithFlags(&tree_evt_[slot], hipEventDisableTiming));
    else HIP_CHECK(hipEventSynchronize(tree_evt_[slot]));
    char* hp = pin_tree_ring_[slot].Get(total);
    PackCompactTree(tree, hp, z);
    if (ttree_buf_.size() < total) {
      HIP_CHECK(hipStreamSynchronize(stream_));  // queued traversals still read the old buffer
      ttree_buf_.Resize(total);
    }
    HIP_CHECK(hipMemcpyAsync(ttree_buf_.get(), hp, total, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipEventRecord(tree_evt_[slot], stream_));
    const char* db = ttree_buf_.get();
    if (lin_pending_ != nullptr) {
      LaunchTraverseLinear(rowbins, StrideOf(rowbins), width_, n, reinterpret_cast<const TNode*>(db), nn,
                           reinterpret_cast<const TCat*>(db + node_bytes),
                           reinterpret_cast<const uint32_t*>(db + node_bytes + cat_bytes + leaf_bytes),
                           reinterpret_cast<const double*>(db + node_bytes + cat_bytes), nl, *lin_pending_, s, num_cu_,
                           stream_);
      return;
    }
    if (rowbins == rowbins_.get() && n == N_ && stride_dw_ > 16 && colbins_.size() >= static_cast<size_t>(G_) * N_ * width_) {
      LaunchTraverseCols(colbins_.get(), width_, n, reinterpret_cast<const TNode*>(db), nn,
                         reinterpret_cast<const TCat*>(db + node_bytes),
                         reinterpret_cast<const uint32_t*>(db + node_bytes + cat_bytes + leaf_bytes),
                         reinterpret_cast<const double*>(db + node_bytes + cat_bytes), nl, s, num_cu_, stream_);
      return;
    }
    if (nib_ && rowbins == rowbins_.get() && n == N_) {
      LaunchTraverse(rowbins4_.get(), stride4_dw_, 0, n, reinterpret_cast<const TNode*>(db), nn,
                     reinterpret_cast<const TCat*>(db + node_bytes), reinterpret_cast<const uint32_t*>(db + node_bytes + cat_bytes + leaf_bytes),
                     reinterpret_cast<const double*>(db + node_bytes + cat_bytes), nl, s, num_cu_, stream_);
      return;
    }
    LaunchTraverse(rowbins, StrideOf(rowbins), width_, n, reinterpret_cast<const TNode*>(db), nn,
                   reinterpret_cast<const TCat*>(db + node_bytes), reinterpret_cast<const uint32_t*>(db + node_bytes + cat_bytes + leaf_bytes),
                   reinterpret_cast<const double*>(db + node_bytes + cat_bytes), nl, s, num_cu_, stream_);
  }

  // ---- validation sets on the device: packed rows (training layout), score, labels / weights
  int DeviceAddValidSet(const Dataset* v, const std::vector<double>& score) override {
    if (linear_) return -1;  // linear leaves need the set's raw values: validation scored on the host
    if (v->row_stride() != data_->row_stride() || v->bin_width() != width_ || v->num_data() <= 0) return -1;
    ScopedTimer timer("Device::AddValidSet");
    auto dv = std::make_unique<DevValid>();
    dv->n = v->num_data();
    std::vector<uint8_t> full;  // a sparse-stored set is materialized to full rows for the upload
    dv->rowbins.Upload(reinterpret_cast<const uint32_t*>(v->RowsForDevice(&full)), static_cast<size_t>(dv->n) * stride_dw_,
                       stream_);
    if (!full.empty()) HIP_CHECK(hipStreamSynchronize(stream_));  // the scratch dies here
    dv->score.Upload(score, stream_);
    const Metadata& md = v->metadata();
    if (md.label()) dv->label.Upload(md.label(), dv->n, stream_);
    if (md.weights()) dv->weight.Upload(md.weights(), dv->n, stream_);
    dv->host_label = md.label();
    HIP_CHECK(hipStreamSynchronize(stream_));
    valid_.push_back(std::move(dv));
    return static_cast<int>(valid_.size()) - 1;
  }
  void DeviceAddTreeToValid(int id, const Tree* tree, int k) override {
    ScopedTimer timer("Device::AddTreeToValid");
    DevValid& v = *valid_[id];
    TraverseTree(tree, v.rowbins.get(), v.n, v.score.get() + static_cast<size_t>(k) * v.n);
  }
  void DeviceValidAddConstant(int id, double c, int k) override {
    DevValid& v = *valid_[id];
    LaunchAddConstant(v.score.get() + static_cast<size_t>(k) * v.n, v.n, c, stream_);
  }
  void DeviceGetValidScore(int id, std::vector<double>* out) override {
    DevValid& v = *valid_[id];
    out->resize(v.score.size());
    v.score.Download(out->data(), out->size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  void DeviceSetValidScore(int id, const std::vector<double>& in) override {
    valid_[id]->score.Upload(in, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  bool DeviceEvalPointwiseValid(int id, const PwMetricParams& p, int k, double* sum) override {
    DevValid& v = *valid_[id];
    if (v.label.size() == 0) return false;
    ScopedTimer timer("Device::EvalValid");
    if (metric_partial_.size() < static_cast<size_t>(kMetricBlocks + 1)) metric_partial_.Resize(kMetricBlocks + 1);
    LaunchPointwiseMetric(p, v.score.get() + static_cast<size_t>(k) * v.n, v.label.get(),
                          v.weight.size() ? v.weight.get() : nullptr, v.n, metric_partial_.get(), kMetricBlocks,
                          metric_partial_.get() + kMetricBlocks, stream_);
    double* h = pin_lout_.Get(1);
    HIP_CHECK(hipMemcpyAsync(h, metric_partial_.get() + kMetricBlocks, sizeof(double), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    *sum = h[0];
    return true;
  }

  bool DeviceEvalMulti(int id, const MultiMetricParams& p, double* sum) override {
    const double* score = nullptr;
    const float* label = nullptr;
    const float* weight = nullptr;
    int n = 0;
    if (id < 0) {
      FlushScore();
      n = N_;
      if (n <= 0 || score_.size() < static_cast<size_t>(p.num_class) * N_) return false;
      EnsureMetricLabels();
      score = score_.get();
      label = metric_label_.get();
      weight = metric_weight_.size() ? metric_weight_.get() : nullptr;
    } else {
      if (id >= static_cast<int>(valid_.size())) return false;
      DevValid& v = *valid_[id];
      n = v.n;
      if (v.label.size() == 0 || n <= 0 || v.score.size() < static_cast<size_t>(p.num_class) * n) return false;
      score = v.score.get();
      label = v.label.get();
      weight = v.weight.size() ? v.weight.get() : nullptr;
    }
    ScopedTimer timer("Device::EvalMultiMetric");
    if (metric_partial_.size() < static_cast<size_t>(kMetricBlocks + 1)) metric_partial_.Resize(kMetricBlocks + 1);
    LaunchMultiMetric(p, score, label, weight, n, metric_partial_.get(), kMetricBlocks, metric_partial_.get() + kMetricBlocks,
                      stream_);
    double* h = pin_lout_.Get(1);
    HIP_CHECK(hipMemcpyAsync(h, metric_partial_.get() + kMetricBlocks, sizeof(double), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    *sum = h[0];
    return true;
  }

  bool DeviceEvalAucMu(int id, const AucMuSpec& spec, std::vector<double>* out) override {
    const int K = spec.num_class;
    if (K < 2 || K > kAucMuMaxClass || spec.sorted == nullptr || spec.sizes == nullptr || spec.cw == nullptr) return false;
    const double* score = nullptr;
    const float* weight = nullptr;
    const void* host_label = nullptr;
    int n = 0;
    if (id < 0) {
      FlushScore();
      n = N_;
      if (n <= 0 || score_.size() < static_cast<size_t>(K) * N_) return false;
      EnsureMetricLabels();
      score = score_.get();
      weight = metric_weight_.size() ? metric_weight_.get() : nullptr;
      host_label = data_->metadata().label();
    } else {
      if (id >= static_cast<int>(valid_.size())) return false;
      DevValid& v = *valid_[id];
      n = v.n;
      if (v.label.size() == 0 || n <= 0 || v.score.size() < static_cast<size_t>(K) * n) return false;
      score = v.score.get();
      weight = v.weight.size() ? v.weight.get() : nullptr;
      host_label = v.host_label;
    }
    if (spec.num_data != n || spec.label != host_label || (spec.weights != nullptr) != (weight != nullptr)) return false;
    if (static_cast<int>(spec.sorted->size()) != n || static_cast<int>(spec.sizes->size()) != K) return false;
    ScopedTimer timer("Device::EvalAucMu");
    auto& slot = aucmu_states_[spec.owner];
    const int npairs = K * (K - 1) / 2;
    int maxpair = 0;
    for (int i = 0; i < K; ++i)
      for (int j = i + 1; j < K; ++j) maxpair = std::max(maxpair, (*spec.sizes)[i] + (*spec.sizes)[j]);
    if (!slot || slot->n != n || slot->host_label != host_label) {
      slot = std::make_unique<AucMuState>();
      slot->n = n;
      slot->host_label = host_label;
      std::vector<int> idx(spec.sorted->begin(), spec.sorted->end());
      slot->idx.Upload(idx, stream_);
      HIP_CHECK(hipStreamSynchronize(stream_));  // (idx is a local staging vector)
      slot->dist.Resize(std::max(maxpair, 1));
      slot->lab.Resize(std::max(maxpair, 1));
      slot->w.Resize(std::max(maxpair, 1));
      slot->scratch.Resize(AucScratchBytes(std::max(maxpair, 1)));
      slot->out.Resize(2 * static_cast<size_t>(npairs));
    }
    AucMuState& st = *slot;
    AucMuPairArgs pa;
    pa.score = score;
    pa.n = n;
    pa.K = K;
    pa.idx = st.idx.get();
    pa.weight = weight;
    pa.out_score = st.dist.get();
    pa.out_label = st.lab.get();
    pa.out_w = st.w.get();
    const auto& cw = *spec.cw;
    int istart = 0, q = 0;
    for (int i = 0; i < K; ++i) {
      int jstart = istart + (*spec.sizes)[i];
      for (int j = i + 1; j < K; ++j, ++q) {
        for (int c = 0; c < K; ++c) pa.v[c] = cw[i][c] - cw[j][c];
        pa.t1 = pa.v[i] - pa.v[j];
        pa.istart = istart;
        pa.ni = (*spec.sizes)[i];
        pa.jstart = jstart;
        pa.nj = (*spec.sizes)[j];
        LaunchAucMuPair(pa, stream_);
        LaunchAucMetric(false, st.dist.get(), st.lab.get(), weight != nullptr ? st.w.get() : nullptr, pa.ni + pa.nj,
                        st.scratch.get(), st.scratch.size(), st.out.get() + 2 * q, stream_);
        jstart += (*spec.sizes)[j];
      }
      istart += (*spec.sizes)[i];
    }
    std::vector<double> h(2 * static_cast<size_t>(npairs));
    st.out.Download(h.data(), h.size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    out->assign(npairs, 0.0);
    for (int p = 0; p < npairs; ++p) (*out)[p] = h[2 * p];
    return true;
  }

  // Ranking / AUC metrics on the device score (metric_kernels.h): the training set (id < 0)
  // or a device validation set. The metric's per-query tables are uploaded once per metric;
  // only the metric's raw sums come back (no score download).
  bool DeviceEvalRank(int id, const RankMetricSpec& spec, int k, std::vector<double>* out) override {
    const double* score = nullptr;
    const float* label = nullptr;
    const float* weight = nullptr;
    const void* host_label = nullptr;
    int n = 0;
    if (id < 0) {
      FlushScore();
      n = N_;
      if (n <= 0 || score_.size() < static_cast<size_t>(k + 1) * N_) return false;
      EnsureMetricLabels();
      score = score_.get() + static_cast<size_t>(k) * N_;
      label = metric_label_.get();
      weight = metric_weight_.size() ? metric_weight_.get() : nullptr;
      host_label = data_->metadata().label();
    } else {
      if (id >= static_cast<int>(valid_.size())) return false;
      DevValid& v = *valid_[id];
      if (v.label.size() == 0) return false;
      n = v.n;
      score = v.score.get() + static_cast<size_t>(k) * n;
      label = v.label.get();
      weight = v.weight.size() ? v.weight.get() : nullptr;
      host_label = v.host_label;
    }
    if (spec.num_data != n || spec.label != host_label) return false;
    if ((spec.weights != nullptr) != (weight != nullptr)) return false;
    const bool query = spec.kind >= RankMetricSpec::kNDCG;
    if (query && (spec.num_queries <= 0 || spec.query_boundaries == nullptr || spec.eval_at.empty() ||
                  spec.eval_at.size() > static_cast<size_t>(RankMetricSpec::kMaxEvalAt))) {
      return false;
    }
    ScopedTimer timer("Device::EvalRankMetric");
    auto& slot = rank_states_[spec.owner];
    if (!slot || slot->kind != spec.kind || slot->n != n || slot->nq != spec.num_queries || slot->host_label != host_label ||
        slot->host_qb != static_cast<const void*>(spec.query_boundaries) || slot->ks != spec.eval_at) {
      // built aside and installed only when complete: a rejected spec leaves no half-built
      // state behind a matching key
      auto fresh = std::make_unique<RankEvalState>();
      RankEvalState& r = *fresh;
      r.kind = spec.kind;
      r.n = n;
      r.nq = spec.num_queries;
      r.host_label = host_label;
      r.host_qb = spec.query_boundaries;
      r.ks = spec.eval_at;
      if (query) {
        const int nq = spec.num_queries, ne = static_cast<int>(spec.eval_at.size());
        std::vector<int> qb(spec.query_boundaries, spec.query_boundaries + nq + 1);
        int maxq = 1;
        for (int q = 0; q < nq; ++q) maxq = std::max(maxq, qb[q + 1] - qb[q]);
        r.qb.Upload(qb, stream_);
        if (spec.query_weights) r.qw.Upload(spec.query_weights, nq, stream_);
        r.ks_dev.Upload(spec.eval_at, stream_);
        if (spec.kind == RankMetricSpec::kNDCG) {
          if (spec.inv_max.size() != static_cast<size_t>(nq) * ne || spec.label_gain.empty()) return false;
          r.inv_max.Upload(spec.inv_max, stream_);
          r.gain.Upload(spec.label_gain, stream_);
          std::vector<double> disc(maxq);  // DCGCalculator::Init's discount table
          for (int i = 0; i < maxq; ++i) disc[i] = 1.0 / std::log2(2.0 + i);
          r.disc.Upload(disc, stream_);
        } else if (spec.kind == RankMetricSpec::kMAP) {
          if (spec.npos.size() != static_cast<size_t>(nq)) return false;
          r.npos.Upload(spec.npos, stream_);
        }
        r.scratch.Resize(QueryMetricScratchBytes(n, nq, ne));
      } else {
        r.scratch.Resize(AucScratchBytes(n));
      }
      r.out.Resize(RankMetricSpec::kMaxEvalAt);
      // the uploads' host sources (qb, disc, ...) are locals of this scope
      HIP_CHECK(hipStreamSynchronize(stream_));
      slot = std::move(fresh);
    }
    RankEvalState& r = *slot;
    int nout = 2;
    if (query) {
      QueryMetricArgs qa;
      qa.kind = spec.kind;
      qa.qb = r.qb.get();
      qa.nq = r.nq;
      qa.qw = r.qw.size() ? r.qw.get() : nullptr;
      qa.inv_max = r.inv_max.size() ? r.inv_max.get() : nullptr;
      qa.npos = r.npos.size() ? r.npos.get() : nullptr;
      qa.ks = r.ks_dev.get();
      qa.ne = static_cast<int>(r.ks.size());
      qa.gain = r.gain.size() ? r.gain.get() : nullptr;
      qa.ngain = static_cast<int>(r.gain.size());
      qa.disc = r.disc.size() ? r.disc.get() : nullptr;
      LaunchQueryMetric(qa, score, label, n, r.scratch.get(), r.scratch.size(), r.out.get(), stream_);
      nout = qa.ne;
    } else {
      LaunchAucMetric(spec.kind == RankMetricSpec::kAveragePrecision, score, label, weight, n, r.scratch.get(),
                      r.scratch.size(), r.out.get(), stream_);
    }
    double* h = pin_metric_.Get(RankMetricSpec::kMaxEvalAt);
    HIP_CHECK(hipMemcpyAsync(h, r.out.get(), sizeof(double) * nout, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    out->assign(h, h + nout);
    return true;
  }

  // ---- linear-leaf trees (linear_tree=true; reference linear_tree_learner.cpp:180-360)
  // The structure comes from the frontier / sequential chain as for any tree; each leaf's
  // Gram system over the numerical features on its branch is accumulated by the fp64 MFMA
  // kernel over the leaf's rows (linear_kernels.hip) and solved on the host (linear_solve.h),
  // as LinearTreeLearner::Train does on the host. The first tree keeps constant leaves.
  void FitLinearLeaves(Tree* tree, bool is_first_tree, int class_id) {
    ScopedTimer timer("Device::LinearLeaves");
    tree->SetIsLinear(true);
    tree->InitLinear();
    const int nl = tree->num_leaves();
    if (is_first_tree || nl <= 1) {
      for (int l = 0; l < nl; ++l) tree->SetLeafConst(l, tree->LeafOutput(l));
      return;
    }
    if (static_cast<int>(h_range_.size()) != nl) Log::Fatal("linear leaves: %d leaf ranges for %d leaves", static_cast<int>(h_range_.size()), nl);
    // distinct numerical features split on along each leaf's branch, sorted (inner indices)
    std::vector<int> parent(std::max(1, nl - 1), -1);
    for (int p = 0; p < nl - 1; ++p) {
      if (tree->left_child(p) >= 0) parent[tree->left_child(p)] = p;
      if (tree->right_child(p) >= 0) parent[tree->right_child(p)] = p;
    }
    std::vector<std::vector<int>> feats(nl);
    std::vector<int> off(nl + 1, 0), flat;
    int max_m = 1, max_cnt = 1;
    for (int l = 0; l < nl; ++l) {
      for (int node = tree->leaf_parent(l); node >= 0; node = parent[node]) {
        const int f = tree->split_feature_inner(node);
        if (data_->feature(f).bin_type == BinType::Numerical) feats[l].push_back(f);
      }
      std::sort(feats[l].begin(), feats[l].end());
      feats[l].erase(std::unique(feats[l].begin(), feats[l].end()), feats[l].end());
      off[l + 1] = off[l] + static_cast<int>(feats[l].size());
      flat.insert(flat.end(), feats[l].begin(), feats[l].end());
      max_m = std::max(max_m, static_cast<int>(feats[l].size()) + 1);
      max_cnt = std::max(max_cnt, h_range_[l].count);
    }
    if (max_m > kLinMaxM) Log::Fatal("linear leaves on the device: %d branch features (at most %d)", max_m - 1, kLinMaxM - 1);
    std::vector<LeafSeg> segs(nl);
    for (int l = 0; l < nl; ++l) {
      segs[l].buf = h_range_[l].buf;
      segs[l].start = h_range_[l].start;
      segs[l].count = h_range_[l].count;
      segs[l].pad = 0;
    }
    lin_segs_.Upload(segs, stream_);
    lin_off_.Upload(off, stream_);
    if (flat.empty()) flat.push_back(0);
    lin_feats_.Upload(flat, stream_);
    LinearGramArgs ga;
    ga.raw = lin_raw_.get();
    ga.F = F_;
    ga.gh = gh_.get() + static_cast<size_t>(class_id) * N_;
    for (int i = 0; i < kLeafIdxBufs; ++i) ga.idx[i] = i < kFrontierIdx ? idx_[i].get() : nullptr;
    ga.segs = lin_segs_.get();
    ga.feat_off = lin_off_.get();
    ga.feats = lin_feats_.get();
    ga.num_leaves = nl;
    // row chunks per leaf: enough blocks to cover the CUs, a few thousand rows each
    ga.chunks = std::max(1, std::min(std::max(1, 2 * num_cu_ / nl), DivUp(max_cnt, 4096)));
    lin_partial_.Resize(std::max(lin_partial_.size(), LinearGramPartialDoubles(nl, ga.chunks)));
    lin_out_.Resize(std::max(lin_out_.size(), static_cast<size_t>(nl) * kLinDim * kLinDim));
    lin_usable_.Resize(std::max(lin_usable_.size(), static_cast<size_t>(nl)));
    LaunchLinearGram(ga, max_m, lin_partial_.get(), lin_out_.get(), lin_usable_.get(), stream_);
    std::vector<double> gram(static_cast<size_t>(nl) * kLinDim * kLinDim);
    std::vector<long long> usable(nl);
    lin_out_.Download(gram.data(), gram.size(), stream_);
    lin_usable_.Download(usable.data(), nl, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int l = 0; l < nl; ++l) {
      const int k = static_cast<int>(feats[l].size()), m = k + 1;
      const double* G = gram.data() + static_cast<size_t>(l) * kLinDim * kLinDim;
      std::vector<double> A(static_cast<size_t>(m) * m), b(m), z;
      for (int i = 0; i < m; ++i) {
        for (int j = 0; j < m; ++j) A[static_cast<size_t>(i) * m + j] = G[i * kLinDim + j];
        b[i] = -G[i * kLinDim + m];
      }
      const int64_t use = lin_has_nan_ ? usable[l] : h_range_[l].count;
      if (!SolveLinearLeaf(std::move(A), b, use, m, config_->linear_lambda, &z)) {
        tree->SetLeafConst(l, tree->LeafOutput(l));
        continue;
      }
      // coefficients that round to zero are dropped (reference :365-369)
      std::vector<double> coef;
      std::vector<int> inner, real;
      for (int j = 0; j < k; ++j) {
        if (Tree::IsZero(z[j])) continue;
        coef.push_back(z[j]);
        inner.push_back(feats[l][j]);
        real.push_back(data_->feature(feats[l][j]).real_index);
      }
      tree->SetLeafConst(l, z[k]);
      tree->SetLeafCoeffs(l, coef);
      tree->SetLeafFeatures(l, real);
      tree->SetLeafFeaturesInner(l, inner);
    }
  }

  // score update of a linear-leaf tree: the traversal evaluates the leaf's model at the row's
  // raw values (8- / 16-bit training rows)
  void TraverseLinear(const Tree* tree, double* s) {
    const int nl = tree->num_leaves();
    std::vector<int> off(nl + 1, 0), feat;
    std::vector<double> coef, cnst(nl);
    for (int l = 0; l < nl; ++l) {
      const auto& fi = tree->LeafFeaturesInner(l);
      const auto& c = tree->LeafCoeffs(l);
      for (size_t j = 0; j < fi.size() && j < c.size(); ++j) {
        feat.push_back(fi[j]);
        coef.push_back(c[j]);
      }
      off[l + 1] = static_cast<int>(feat.size());
      cnst[l] = tree->LeafConst(l);
    }
    if (feat.empty()) {
      feat.push_back(0);
      coef.push_back(0.0);
    }
    HIP_CHECK(hipStreamSynchronize(stream_));  // (the previous tree's linear arrays may still be read)
    lin_toff_.Upload(off, stream_);
    lin_tfeat_.Upload(feat, stream_);
    lin_tcoef_.Upload(coef, stream_);
    lin_tcnst_.Upload(cnst, stream_);
    LinearLeaves lin;
    lin.raw = lin_raw_.get();
    lin.F = F_;
    lin.off = lin_toff_.get();
    lin.feat = lin_tfeat_.get();
    lin.coef = lin_tcoef_.get();
    lin.cnst = lin_tcnst_.get();
    lin_pending_ = &lin;
    TraverseTreeCompact(tree, rowbins_.get(), N_, s);
    lin_pending_ = nullptr;
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void EnsureMetricLabels() {
    if (metric_label_.size() != 0) return;
    const Metadata& md = data_->metadata();
    metric_label_.Upload(md.label(), N_, stream_);  // the raw labels (objectives may relabel theirs)
    if (md.weights()) metric_weight_.Upload(md.weights(), N_, stream_);
    metric_partial_.Resize(kMetricBlocks + 1);
  }

  std::unique_ptr<Tree> DeviceTrain(int class_id, bool is_first_tree) override {
    (void)is_first_tree;
    ScopedTimer timer("DeviceTreeLearner::Train");
    // per-tree inputs: root rows, class, feature sampling
    TreeParams* tp = pin_tp_.Get(1);
    tp->root_buf = use_bag_ ? 2 : -1;
    tp->root_count = use_bag_ ? bag_cnt_ : N_;
    tp->cls = class_id;
    int gcount = tp->root_count;
    if (distributed_) {
      // the global root count changes only with the bag: one host collective per new bag
      if (gcount != cached_gcount_local_) {
        cached_gcount_local_ = gcount;
        cached_gcount_ = Network::num_machines() > 1 ? Network::GlobalSyncUpBySum(gcount) : gcount;
      }
      gcount = cached_gcount_;
    }
    tp->root_gcount = gcount;
    const bool tune = frontier_ && stune_.on;
    tp->spec_alpha = static_cast<float>(tune ? stune_.Alpha() : fspec_alpha_);
    tp->byn_rng = 0;
    tp->pad[0] = tp->pad[1] = 0;
    HIP_CHECK(hipMemcpyAsync(tparams_.get(), tp, sizeof(TreeParams), hipMemcpyHostToDevice, stream_));
    const auto t_tree0 = std::chrono::steady_clock::now();
    if (config_->use_quantized_grad) QuantizeGradients(class_id);
    col_sampler_.ResetByTree();
    const auto& used = col_sampler_.is_feature_used_bytree();
    uint8_t* um = pin_mask_.Get(static_cast<size_t>(F_) * (1 + 2 * L_) + 8);
    for (int f = 0; f < F_; ++f) um[f] = used[f] ? 1 : 0;
    HIP_CHECK(hipMemcpyAsync(used_bytree_.get(), um, F_, hipMemcpyHostToDevice, stream_));
    Random byn_state;
    const bool byn_dev = use_bynode_ && frontier_ && ByNodeOnDevice();
    if (use_bynode_ && !frontier_ && ByNodeOnDevice()) {
      Log::Fatal("feature_fraction_bynode with interaction constraints needs the frontier engine (shape / node capacity)");
    }
    if (use_bynode_) {
      // the tree's masks in the host's draw order (root, then smaller / larger child of each
      // scanned split); the stream is rewound below to the draws the tree actually used. Under
      // interaction constraints only the root's: the select draws the rest from its state on
      byn_state = col_sampler_.rng_state();
      Tree dummy(2, true);  // (the root: no branch features; GetByNode reads them under constraints)
      uint8_t* bm = um + F_;
      const int rows = byn_dev ? 1 : 2 * L_;
      for (int r = 0; r < rows; ++r) {
        auto m = col_sampler_.GetByNode(&dummy, 0);
        for (int f = 0; f < F_; ++f) bm[static_cast<size_t>(r) * F_ + f] = m[f] ? 1 : 0;
      }
      HIP_CHECK(hipMemcpyAsync(bynode_.get(), bm, static_cast<size_t>(rows) * F_, hipMemcpyHostToDevice, stream_));
      if (byn_dev) {
        const unsigned st = col_sampler_.rng_state().state();
        uint8_t* w = um + static_cast<size_t>(F_) * (1 + 2 * L_);
        std::memcpy(w, &st, sizeof(st));
        HIP_CHECK(hipMemcpyAsync(reinterpret_cast<char*>(tparams_.get()) + offsetof(TreeParams, byn_rng), w, sizeof(st),
                                 hipMemcpyHostToDevice, stream_));
      }
    }
    SplitRec* hr = pin_rec_.Get(L_);
    LeafRange* hrange = pin_range_.Get(L_);
    double* hlo = pin_lout_.Get(1);
    int num_splits = 0, num_leaves = 1;
    bynode_draws_ = 0;
    if (frontier_) {
      FrontierGrow(&num_splits, &num_leaves, hr, hrange, hlo);
      if (tune) stune_.Record(std::chrono::duration<double>(std::chrono::steady_clock::now() - t_tree0).count());
    } else {
      SequentialGrow(&num_splits, &num_leaves, hr, hrange, hlo);
    }
    if (byn_dev) {
      col_sampler_.set_rng_state(Random(static_cast<int>(bynode_rng_)));  // (the select's draws)
    } else if (use_bynode_) {
      col_sampler_.set_rng_state(byn_state);
      Tree dummy(2);
      for (int r = 0; r < std::min(bynode_draws_, 2 * L_); ++r) (void)col_sampler_.GetByNode(&dummy, 0);
    }
    auto tree = std::make_unique<Tree>(L_, false, false);
    tree->SetLeafOutput(0, hlo[0]);
    if (num_splits < 0 || num_splits > L_ - 1) Log::Fatal("device tree: invalid split count %d", num_splits);
    for (int s = 0; s < num_splits; ++s) {
      const SplitRec& r = hr[s];
      const SplitInfo& info = r.info;
      if (r.leaf < 0 || r.leaf > s || info.feature < 0 || info.feature >= F_) {
        Log::Fatal("device tree: invalid split record %d (leaf %d, feature %d)", s, r.leaf, info.feature);
      }
      const FeatureInfo& fi = data_->feature(info.feature);
      const BinMapper& mapper = data_->inner_mapper(info.feature);
      if (fi.bin_type == BinType::Numerical && info.threshold >= static_cast<uint32_t>(std::max(1, fi.num_bin))) {
        Log::Fatal("device tree: invalid split record %d (feature %d, threshold %u of %d bins)", s, info.feature,
                   info.threshold, fi.num_bin);
      }
      const float gain = static_cast<float>(info.gain + config_->min_gain_to_split);
      if (fi.bin_type == BinType::Numerical) {
        tree->Split(r.leaf, info.feature, fi.real_index, info.threshold, mapper.BinToValue(info.threshold),
                    info.left_output, info.right_output, r.left_count, r.right_count, info.left_sum_hessian,
                    info.right_sum_hessian, gain, fi.missing, info.default_left != 0);
      } else {
        int nwords = 0;
        std::vector<int> cats;
        for (int w = 0; w < kMaxCatWords; ++w) {
          if (info.cat_bitset[w]) nwords = w + 1;
          for (int j = 0; j < 32; ++j) {
            if ((info.cat_bitset[w] >> j) & 1) cats.push_back(mapper.bin_to_category()[w * 32 + j]);
          }
        }
        std::vector<uint32_t> inner(info.cat_bitset, info.cat_bitset + nwords);
        std::vector<uint32_t> raw = common::ConstructBitset(cats.data(), static_cast<int>(cats.size()));
        tree->SplitCategorical(r.leaf, info.feature, fi.real_index, inner.data(), nwords, raw.data(),
                               static_cast<int>(raw.size()), info.left_output, info.right_output, r.left_count,
                               r.right_count, info.left_sum_hessian, info.right_sum_hessian, gain, fi.missing);
      }
    }
    h_range_.assign(hrange, hrange + num_leaves);
    if (config_->use_quantized_grad && config_->quant_train_renew_leaf) RenewQuantizedLeaves(tree.get());
    if (linear_) FitLinearLeaves(tree.get(), is_first_tree, class_id);
    if (stamps_.size() && !frontier_ && ++stamp_trees_ == 3) ReportStamps(num_splits);
    tree->RecomputeMaxDepth();
    last_trained_ = tree.get();
    return tree;
  }

  // ---- frontier tree growth (frontier.h): batched rounds, replayed best-first order

  // The frontier engine covers the single-device learner; bynode sampling and extra-trees
  // draw per split in sequential order, the global-memory scan has no frontier variant, and
  // the computed-node image of the select must fit its LDS. LGAP_FRONTIER=0 forces the
  // sequential chain (A/B runs).
  bool FrontierEligible() const {
    if (!FrontierSerial() && !FrontierDP() && !FrontierVoting() && !FrontierFeature()) return false;
    // extra trees: the single-device frontier and the voting frontier on numerical data (one
    // expansion per round: FArgs::xrng; the global pass redraws in the host's order, k_f_vote_scan)
    if (config_->extra_trees && !FrontierSerial() && !(FrontierVoting() && !has_cat_)) return false;
    // by-node sampling: the single-device frontier (masks in the host's draw order, FArgs::bynode;
    // under interaction constraints drawn in the select, FArgs::byn_draw)
    if (use_bynode_ && !FrontierSerial()) return false;
    if (MonoInter() && (!FrontierSerial() || RawCands() || config_->extra_trees || fnum_forced_ > 0 ||
                        !config_->forcedsplits_filename.empty()))
      return false;
    return FrontierShapeFits(L_, TB_, F_, max_bin_, max_cat_bin_, RawCands(), MonoInter());
  }
  // per-node raw candidates of every feature (FArgs::cegb_raw): CEGB feature penalties, and
  // by-node sampling (a node is scored once its mask is known)
  bool RawCands() const { return CegbRaw() || use_bynode_; }
  // intermediate monotone constraints in the frontier select (FArgs::mono_inter; the serial
  // frontier only: TreeLearner::Create routes the other learners to the host policy)
  bool MonoInter() const {
    return !config_->monotone_constraints.empty() && config_->monotone_constraints_method == "intermediate";
  }
  // by-node masks drawn in the select: each node's pool follows its interaction constraints
  bool ByNodeOnDevice() const { return use_bynode_ && !config_->interaction_constraints_vector.empty(); }
  // CEGB feature penalties in the frontier select: coupled (FArgs::cegb_coupled: refunds on a
  // feature's first use) and lazy (FArgs::cegb_lazy: per-row marks, unmarked-row counts per
  // node). Either makes the scans publish raw gains (FArgs::cegb_raw).
  bool CegbCoupled() const { return !config_->cegb_penalty_feature_coupled.empty(); }
  bool CegbLazy() const { return !config_->cegb_penalty_feature_lazy.empty(); }
  bool CegbRaw() const { return CegbCoupled() || CegbLazy(); }
  bool FrontierSerial() const {
    return mode_ == DevParallel::kSerial && !owner_scan_ && !voting_ && !distributed_;
  }
  // the frontier's exchanges run in-kernel over xGMI (SetupFrontierXgmi; FArgs::xg)
  bool FrontierXg() const { return fxg_ && frontier_ && (fowner_ || ffeature_ || fvoting_); }
  // Data-parallel frontier: every rank partitions / builds histograms of its own rows, the
  // round's fixed-point accumulators are summed over ranks (one exact integer all-reduce per
  // round, RCCL or the host-staged rehearsal transport), and every rank scans and selects
  // redundantly: the select is deterministic in the summed histograms, so all ranks grow the
  // same tree with no further exchange. Children's counts come from the summed histograms
  // (the split record), row ranges from the local partition. LGAP_FRONTIER_DP=0: the
  // sequential owner-scan chain instead. Reference: data_parallel_tree_learner.cpp:148-297.
  // The exchanges: the owner-computes rounds below (FrontierOwner) over the in-kernel xGMI
  // transport (FrontierXg, the default where every rank maps every peer) or RCCL / the host-staged
  // rehearsal collectives; the per-round all-reduce for configurations that need every feature.
  bool FrontierDP() const {
    const char* e = std::getenv("LGAP_FRONTIER_DP");
    if (e != nullptr && e[0] == '0') return false;
    return mode_ == DevParallel::kData && data_parallel_ && owner_scan_ && distributed_ && !voting_ &&
           (CommExists() || HostStagedDP());
  }
  // Owner-computes data-parallel rounds (the default data-parallel frontier): the round's
  // fixed-point accumulators are REDUCE-SCATTERED by feature-group ownership (SetupOwnership:
  // contiguous, bin-balanced group ranges), so each rank receives only the summed bins of its own
  // features (half the bytes of the all-reduce) and scans only those (1/P of the scan work); each
  // child's best over the owned features is all-gathered and the best over ranks becomes the
  // child's candidate (the feature-parallel exchange: k_f_pair_best, then the select's phase A); every rank
  // then selects redundantly from identical candidates. Reference:
  // data_parallel_tree_learner.cpp:284-297 (ReduceScatter of the smaller leaf's histograms by
  // feature ownership), :305-450 (owner scans, SyncUpGlobalBestSplit). Raw per-feature candidates
  // (CEGB penalties, by-node sampling) and forced splits need every feature's scan on every rank:
  // they keep the all-reduce, as does LGAP_DP_TRANSPORT=allreduce (A/B).
  bool FrontierOwner() const {
    if (!FrontierDP() || RawCands() || !config_->forcedsplits_filename.empty() || config_->extra_trees) return false;
    const char* t = std::getenv("LGAP_DP_TRANSPORT");
    return !(t != nullptr && std::strcmp(t, "allreduce") == 0);
  }
  // Voting-parallel frontier (PV-Tree per round): the local pass of every expansion's children,
  // one all-gather of the round's top-k vote records, the election, one exact integer
  // all-reduce of only the elected features' rows, and the global pass over them; every rank
  // then selects redundantly, as the data-parallel frontier does. Over xGMI the records and the
  // elected rows are pushed in-kernel (FArgs::xg). Reference: voting_parallel_tree_learner.cpp:243-399.
  bool FrontierVoting() const {
    return mode_ == DevParallel::kVoting && voting_ && distributed_ && (CommExists() || HostStagedDP());
  }
  // Feature-parallel frontier: every rank holds all rows and grows the same partition and
  // histograms; the scans cover this rank's features (the groups it owns), each child's best is
  // exchanged (pushed over xGMI, or all-gathered) and the best over ranks is the child's candidate.
  // Reference: feature_parallel_tree_learner.cpp:23-80.
  bool FrontierFeature() const {
    return mode_ == DevParallel::kFeature && owner_scan_ && !distributed_ && (CommExists() || HostStagedDP());
  }
  int FrontierKmax() const {
    return std::max(1, std::min(kFrontierKmax, L_ - 1));
  }
  // computed nodes of one tree: every committed node (2 L - 1) plus room for speculation
  // (8 L + 2 kmax, fewer when the per-node fp64 histograms would exceed ~8 GiB)
  int FrontierCapacity() const { return FrontierCapacityFor(L_, TB_); }

  // forcedsplits_filename -> the FForced list the frontier select applies first (the host
  // learner's order and skips: learner/forced_splits.h)
  void UploadForcedSplits() {
    fnum_forced_ = 0;
    if (config_->forcedsplits_filename.empty()) return;
    std::ifstream in(config_->forcedsplits_filename);
    if (!in) {
      Log::Warning("Forced splits file %s cannot be opened", config_->forcedsplits_filename.c_str());
      return;
    }
    const std::string js((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    size_t pos = 0;
    auto root = ParseForced(js, &pos);
    const auto flat = FlattenForced(root.get(), [&](int f) {
      if (f < 0 || f >= data_->num_total_features()) return false;
      const int inner = data_->InnerIndex(f);
      return inner >= 0 && data_->feature(inner).bin_type == BinType::Numerical;
    });
    std::vector<FForced> h(flat.size());
    for (size_t i = 0; i < flat.size(); ++i) {
      const int inner = data_->InnerIndex(flat[i].feature);
      h[i].feature = inner;
      h[i].threshold = static_cast<int>(data_->inner_mapper(inner).ValueToBin(flat[i].threshold));
      h[i].left = flat[i].left;
      h[i].right = flat[i].right;
    }
    fforced_.Resize(std::max<size_t>(1, h.size()));
    if (!h.empty()) fforced_.Upload(h.data(), h.size(), stream_);
    fnum_forced_ = static_cast<int>(h.size());
  }

  void AllocFrontier() {
    frontier_ = FrontierEligible();
    if (!frontier_ && !config_->forcedsplits_filename.empty()) {
      // (TreeLearner::Create routes these by FrontierServes: reaching here is a routing bug)
      Log::Fatal("forced splits on the device need the frontier engine (serial learner, no "
                 "feature_fraction_bynode / extra_trees, frontier LDS shape)");
    }
    if (!frontier_ && config_->interaction_constraints_vector.size() > 64) {
      // (TreeLearner::Create routes these by FrontierServes: reaching here is a routing bug)
      Log::Fatal("more than 64 interaction constraint sets on the device need the frontier engine");
    }
    if (!frontier_ && MonoInter()) {
      // (TreeLearner::Create routes these by FrontierServesMonoInter: reaching here is a routing bug)
      Log::Fatal("intermediate monotone constraints on the device need the serial frontier engine");
    }
    if (!frontier_ && CegbRaw()) {
      Log::Fatal("cegb_penalty_feature_coupled / _lazy on the device need the frontier engine (serial learner, "
                 "no feature_fraction_bynode / extra_trees, frontier LDS shape)");
    }
    if (!frontier_) return;
    fkmax_ = FrontierKmax();
    fC_ = FrontierCapacity();
    const size_t C = fC_, K = fkmax_, F = std::max(F_, 1);
    ArenaLayout lay;
    const size_t o_st = lay.Add<FState>(1), o_nodes = lay.Add<FNode>(C), o_exps = lay.Add<FExp>(K),
                 o_bits = lay.Add<uint32_t>(K * kMaxCatWords), o_lsum = lay.Add<double2>(C), o_lout = lay.Add<double>(C),
                 o_bounds = lay.Add<LeafBounds>(C), o_key = lay.Add<SplitKey>(C), o_best = lay.Add<SplitInfo>(C),
                 o_spl = lay.Add<uint8_t>(C * F), o_ic = lay.Add<unsigned long long>(C * kFrontierIcWords), o_nst = lay.Add<uint8_t>(C),
                 o_lcid = lay.Add<int>(L_), o_ckey = lay.Add<SplitKey>(K * 2 * F), o_cinfo = lay.Add<SplitInfo>(K * 2 * F),
                 o_fbest = lay.Add<SplitInfo>(C), o_fkey = lay.Add<SplitKey>(C),
                 o_cbnd = lay.Add<LeafBounds>(MonoInter() ? C : 1), o_sal = lay.Add<int>(C);
    farena_.Resize(lay.bytes());
    farena_.Zero(stream_);
    char* b = farena_.get();
    fst_ = reinterpret_cast<FState*>(b + o_st);
    fnodes_ = reinterpret_cast<FNode*>(b + o_nodes);
    fexps_ = reinterpret_cast<FExp*>(b + o_exps);
    fbits_ = reinterpret_cast<uint32_t*>(b + o_bits);
    flsum_ = reinterpret_cast<double2*>(b + o_lsum);
    flout_ = reinterpret_cast<double*>(b + o_lout);
    fbounds_ = reinterpret_cast<LeafBounds*>(b + o_bounds);
    fkey_ = reinterpret_cast<SplitKey*>(b + o_key);
    fbest_ = reinterpret_cast<SplitInfo*>(b + o_best);
    fspl_ = reinterpret_cast<uint8_t*>(b + o_spl);
    fic_ = reinterpret_cast<unsigned long long*>(b + o_ic);
    fnst_ = reinterpret_cast<uint8_t*>(b + o_nst);
    flcid_ = reinterpret_cast<int*>(b + o_lcid);
    fckey_ = reinterpret_cast<SplitKey*>(b + o_ckey);
    fcinfo_ = reinterpret_cast<SplitInfo*>(b + o_cinfo);
    ffbest_ = reinterpret_cast<SplitInfo*>(b + o_fbest);
    ffkey_ = reinterpret_cast<SplitKey*>(b + o_fkey);
    fcbnd_ = MonoInter() ? reinterpret_cast<LeafBounds*>(b + o_cbnd) : nullptr;
    fsal_ = reinterpret_cast<int*>(b + o_sal);
    UploadForcedSplits();
    if (RawCands()) {
      fnkey_.Resize(C * F);
      fninfo_.Resize(C * F);
      fnuep_.Resize(C);
      fnuep_.Zero(stream_);
    }
    if (CegbCoupled()) {
      // tradeoff x coupled penalty per inner feature; used flags and the event count persist
      // over the trees of this training set (host CegbPenalty::Init)
      const auto& cp = config_->cegb_penalty_feature_coupled;
      if (static_cast<int>(cp.size()) != data_->num_total_features()) {
        Log::Fatal("cegb_penalty_feature_coupled should be the same size as feature number.");
      }
      std::vector<double> h(F_);
      for (int f = 0; f < F_; ++f) h[f] = config_->cegb_tradeoff * cp[data_->feature(f).real_index];
      cegb_coupled_.Resize(F_);
      cegb_coupled_.Upload(h.data(), h.size(), stream_);
      // the used flags survive ResetConfig on the same training set (host CegbPenalty::Init)
      const bool fresh = cegb_data_ != data_ || cegb_used_.size() != static_cast<size_t>(F_);
      cegb_used_.Resize(F_);
      cegb_epoch_.Resize(1);
      if (fresh) {
        cegb_used_.Zero(stream_);
        cegb_epoch_.Zero(stream_);
      }
    }
    if (CegbLazy()) {
      // tradeoff x lazy penalty per inner feature; per-row marks persist over the trees
      const auto& lp = config_->cegb_penalty_feature_lazy;
      if (static_cast<int>(lp.size()) != data_->num_total_features()) {
        Log::Fatal("cegb_penalty_feature_lazy should be the same size as feature number.");
      }
      std::vector<double> h(F_);
      for (int f = 0; f < F_; ++f) h[f] = config_->cegb_tradeoff * lp[data_->feature(f).real_index];
      cegb_lazy_.Resize(F_);
      cegb_lazy_.Upload(h.data(), h.size(), stream_);
      lazy_words_ = (F_ + 31) / 32;
      const size_t nbits = static_cast<size_t>(std::max(N_, 1)) * lazy_words_;
      const bool fresh = cegb_data_ != data_ || lazy_bits_.size() != nbits;
      lazy_bits_.Resize(nbits);
      if (fresh) lazy_bits_.Zero(stream_);  // per-row marks survive ResetConfig on the same data
      lazy_acc_.Resize(K * F);
      lazy_acc_.Zero(stream_);
      fnlazy_.Resize(C * F);
      fnpath_.Resize(C * lazy_words_);
    }
    cegb_data_ = data_;
    // replay results: coherent pinned host memory the results kernel writes directly
    const size_t rbytes = FrontierResultBytes(L_);
    if (rbytes > fres_bytes_) {
      if (fres_host_) HIP_CHECK(hipHostFree(fres_host_));
      void* hp = nullptr;
      HIP_CHECK(hipHostMalloc(&hp, rbytes, hipHostMallocMapped | hipHostMallocCoherent));
      fres_host_ = static_cast<char*>(hp);
      HIP_CHECK(hipHostGetDevicePointer(&fres_dev_, hp, 0));
      fres_bytes_ = rbytes;
    }
    fslots_.Resize(C * 2 * static_cast<size_t>(TB_));
    // global row count (data parallel: the packed quantized accumulators must hold every
    // rank's level sums)
    fglobal_rows_ = static_cast<double>(N_);
    if (distributed_) {
      DevBuf<double> gr(1);
      const double nloc = static_cast<double>(N_);
      gr.Upload(&nloc, 1, stream_);
      AllreduceSumF64(gr.get(), 1, stream_);
      HIP_CHECK(hipMemcpyAsync(&fglobal_rows_, gr.get(), sizeof(double), hipMemcpyDeviceToHost, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    facc_.Resize(K * 2 * static_cast<size_t>(TB_));
    facc_.Zero(stream_);  // the scan re-zeroes what it consumes: zero between rounds from here on
    // partial-histogram slab: one row of TB words (gpu_use_dp: 2 TB) per histogram block
    {
      const int rows = FrontierHistRows(FrontierHistBlocks(), K);
      fhslab_stride_ = static_cast<size_t>(TB_) * (use_dp_ && !QuantHist() ? 2 : 1);
      fhslab_.Resize(static_cast<size_t>(rows) * fhslab_stride_);
      fhmeta_.Resize(rows);

      if (num_tiles_ > 256) Log::Fatal("frontier histograms: %d LDS tiles (at most 256)", num_tiles_);
    }
    ffeature_ = FrontierFeature();
    fowner_ = FrontierOwner();
    if (ffeature_ || fowner_) {
      std::vector<uint8_t> own(F_, 0);
      std::vector<int> list;
      for (int f : h_own_feat_) {
        if (f >= 0) {
          own[f] = 1;
          list.push_back(f);
        }
      }
      ffowned_.Upload(own, stream_);
      fown_n_ = static_cast<int>(list.size());
      fown_list_.Resize(std::max<size_t>(1, list.size()));
      if (!list.empty()) fown_list_.Upload(list.data(), list.size(), stream_);
      ffpb_.Resize(static_cast<size_t>(P_) * 2 * K);
    }
    if (fowner_) {
      // send layout [rank][kmax][widest owner's bins] (>= the plain layout), receive [kmax][own bins]
      fown_b0_.Upload(h_bin_lo_, stream_);
      const size_t send = static_cast<size_t>(P_) * K * bbin_ * 2;
      if (facc_.size() < send) facc_.Resize(send);
      facc_.Zero(stream_);
      facc_recv_.Resize(static_cast<size_t>(K) * bbin_ * 2);
    }
    if (ByNodeOnDevice()) {
      bool filt = false;
      const std::vector<uint8_t> m = col_sampler_.ByNodeSampleModes(&fbyn_cnt_, &filt);
      fbyn_reset_ = filt ? 1 : 0;
      fbyn_mode_.Resize(m.size());
      fbyn_mode_.Upload(m.data(), m.size(), stream_);
    }
    fvoting_ = FrontierVoting();
    if (fvoting_) {
      // voting's local pass: min_data / min_hessian divided by the ranks (reference :61-63, integer division)
      SplitParams sl = MakeArgs().sp;
      sl.min_data_in_leaf = config_->min_data_in_leaf / P_;
      sl.min_sum_hessian_in_leaf = config_->min_sum_hessian_in_leaf / P_;
      fsp_local_.Resize(1);
      fsp_local_.Upload(&sl, 1, stream_);
      flsum_loc_.Resize(C);
      fltot_.Resize(2 * K);
      fltot_.Zero(stream_);  // k_f_vote re-zeroes what the round consumed
      fvrec_.Resize(static_cast<size_t>(P_) * 2 * K * topk_);
      fvelect_.Resize(2 * K * static_cast<size_t>(topk_ + 1));
      fvrows_.Resize(2 * K * static_cast<size_t>(topk_) * 2 * max_bin_);
    }
    // frontier tile rows: the chain's rows per thread (8192-row tiles were an A/B loss: 10M 400.9
    // vs 408.9 it/s, 1.25M 746 vs 878; profiles/r05/ab_partition_8192_tiles.log)
    fpart_iters_ = part_iters_;
    fpart_tile_ = kPartThreads * fpart_iters_;
    ftile_cap_ = DivUp(N_, fpart_tile_) + fkmax_ + 1;
    ftile_pub_.Resize(ftile_cap_);
    ftile_pub_.Zero(stream_);
    for (int i = 3; i < kFrontierIdx; ++i) idx_[i].Resize(std::max(N_, 1));
    // partition grid: the resident blocks (at most one per tile of the tile capacity); a block
    // takes tiles b, b + G, ... in passes and only waits on lower tiles. A grid of the full tile
    // capacity (2.4K blocks at 10M) left ~1.2K blocks with no tile in a typical round, dispatched
    // behind the working ones: each still read the round state before exiting, at the kernel's tail.
    {
      const int per_cu = std::max(1, FrontierPartitionBlocksPerCU(fpart_iters_));
      fpart_grid_ = std::max(1, std::min(ftile_cap_, per_cu * num_cu_));
    }
    fscan_lds_ = FrontierScanLds(max_bin_, has_cat_ ? max_cat_bin_ : 1);
    FrontierSetLds(FrontierHistLds(), fscan_lds_, use_dp_, width_);
    fspec_cap_ = 0;
    // 512 / 1024 threads per histogram block. Round 3 (after the grid cap at 7/8 of the CUs),
    // paired on one box: single-tile rows at 10M 370.6 / 368.9 (1024) vs 363.6 / 365.4 (512),
    // quantized 405.6 vs 398.3; at 1.25M mixed (737.9 / 778.4 vs 779.2 / 770.0). Multi-tile rows
    // keep 512 (two resident 56 KB blocks per CU); 150 KB tiles hold one block per CU.
    fhist_threads_ = big_tiles_ || (num_tiles_ == 1 && N_ >= 4000000) ? 1024 : 512;
    if (const char* e = KernelOverride("fhist_threads")) fhist_threads_ = std::atoi(e) == 1024 ? 1024 : 512;
    fpolicy_ = 1;
    // speculation budget: every eligible node within the remaining splits (alpha 1). One knob,
    // LGAP_FRONTIER_SPEC, picks another budget for A/B: "fixed" (alpha 1, no tuner), a number
    // (that fixed alpha) or "adapt". The
    // waste-driven throttle ("adapt": alpha x0.75 while > 12% of the partitioned
    // rows go to never-committed expansions) trades rows for rounds and loses where rounds cost
    // more than rows: 255 leaves x 500 iterations at 10M, 93.5 it/s adaptive vs 141.4 fixed
    // (139 vs 76 rounds per tree); 1.25M x 150 iterations, 2.07 vs 1.73 ms per iteration
    fspec_alpha_ = 1.0;
    const char* spec_env = std::getenv("LGAP_FRONTIER_SPEC");
    const std::string spec = spec_env != nullptr ? spec_env : "";
    fspec_fixed_ = spec != "adapt";
    if (!spec.empty() && spec != "adapt" && spec != "fixed") {  // a fixed speculation depth (A/B)
      char* end = nullptr;
      const double alpha = std::strtod(spec.c_str(), &end);
      if (end == spec.c_str() || *end != '\0') Log::Fatal("LGAP_FRONTIER_SPEC=%s: expected fixed|adapt|<alpha>", spec.c_str());
      fspec_alpha_ = std::max(0.01, std::min(4.0, alpha));
    }
    // timed speculation tuner: one process, >= 128 leaves, no other budget requested
    {
      stune_ = SpecTuner();
      // (not with raw CEGB candidates or forced splits: there the select's replay of speculated
      // expansions depends on what was speculated, and the budget must not follow wall-clock time)
      // Below 128 leaves the early trees are near-balanced and alpha 1 is their optimum (30-step
      // A/B, profiles/r06/ab_notes.md); later trees grow chain-like and gain from deeper
      // speculation (10M x 28 / 63 leaves over 500 iterations: 358 it/s at alpha 1, 377 at 1.5,
      // 385 tuned). There the tuner starts probing after the first 64 trees. LGAP_SPEC_TUNE=0:
      // off below 128 leaves; 1: probing from the first tree.
      const char* te = std::getenv("LGAP_SPEC_TUNE");
      const bool tune_small = te == nullptr || te[0] != '0';
      stune_.on = !distributed_ && (L_ >= 128 || tune_small) && !RawCands() && fnum_forced_ == 0 &&
                  spec.empty();
      if (L_ < 128 && te == nullptr) stune_.rest = 64;
    }
    if (std::getenv("LGAP_FSTAMPS")) {
      fstamps_.Resize(256 * 4 * kFStampSlots);
      fstamps_.Zero(stream_);
    }
    for (auto& kv : fgraphs_) (void)hipGraphExecDestroy(kv.second);
    fgraphs_.clear();
    if (fcont_) (void)hipGraphExecDestroy(fcont_);
    fcont_ = nullptr;
  }

  FArgs MakeFArgs() const {
    FArgs a;
    std::memset(&a, 0, sizeof(a));
    a.rowbins = rowbins_.get();
    a.colbins = colbins_.get();
    a.gh = gh_.get();
    for (int i = 0; i < kFrontierIdx; ++i) a.idx[i] = idx_[i].get();
    a.N = N_;
    a.stride_dw = tstride_dw_;
    a.width = width_;
    a.num_groups = G_;
    a.TB = TB_;
    a.F = F_;
    a.L = L_;
    a.C = fC_;
    a.kmax = fkmax_;
    a.gstart = gstart_.get();
    a.feat = feat_.get();
    a.tiles = tiles_.get();
    a.num_tiles = num_tiles_;
    a.used_bytree = used_bytree_.get();
    a.tp = tparams_.get();
    a.st = fst_;
    a.nodes = fnodes_;
    a.exps = fexps_;
    a.exp_bits = fbits_;
    a.lsum = flsum_;
    a.lout = flout_;
    a.bounds = fbounds_;
    a.key = fkey_;
    a.best = fbest_;
    a.spl = fspl_;
    a.ic = use_ic_ ? fic_ : nullptr;
    a.ic_feat = use_ic_ ? fic_feat_.get() : nullptr;
    a.ic_words = ic_words_;
    a.nstate = fnst_;
    a.leaf_cid = flcid_;
    a.rec = rec_.get();
    a.range_out = range_.get();
    a.slots = fslots_.get();
    a.acc = reinterpret_cast<unsigned long long*>(facc_.get());
    a.hslab = fhslab_.get();
    a.hslab_stride = fhslab_stride_;
    a.hmeta = fhmeta_.get();
    a.red_grid = (num_tiles_ > 1 ? 4 : 2) * num_cu_;  // (wide data: many reduce items per round)
    a.ghmax = ghmax_.get();
    a.sum_mult = distributed_ && !ffeature_ ? std::max(1, P_) : 1;  // (max-reduced local sums)
    {
      const char* e = std::getenv("LGAP_FIXED_SUMBOUND");
      a.sum_bound = e == nullptr || std::atoi(e) != 0;
    }
    a.forced = fnum_forced_ > 0 ? fforced_.get() : nullptr;
    a.num_forced = fnum_forced_;
    a.fbest = ffbest_;
    a.fkey = ffkey_;
    a.ckey = fckey_;
    a.cinfo = fcinfo_;
    a.tile_pub = ftile_pub_.get();
    a.bar = bar_.get();
    a.hist_min_rows = HistMinRows();
    a.hist_grid = FrontierHistBlocks();
    a.hist_threads = fhist_threads_;
    if (nib_) {
      a.rowbins = rowbins4_.get();
      a.stride_dw = stride4_dw_;
      a.tiles = ntile_.get();
      a.hist_nib = 1;
    }
    a.part_tile = fpart_tile_;
    a.max_depth = config_->max_depth;
    a.use_monotone = config_->monotone_constraints.empty() ? 0 : 1;
    a.mono_inter = fcbnd_ != nullptr ? 1 : 0;
    a.cbnd = fcbnd_;
    // LGAP_KERNEL=select_merge=0: the select re-sorts the alive list every round (A/B)
    const char* sm = KernelOverride("select_merge");
    a.salive = sm != nullptr && sm[0] == '0' ? nullptr : fsal_;
    a.monotone_penalty = config_->monotone_penalty;
    a.cegb_split = CegbPenalty::Enabled(config_) ? config_->cegb_tradeoff * config_->cegb_penalty_split : 0.0;
    a.max_bin = max_bin_;
    a.cat_p2 = cat_p2_;
    a.use_dp = use_dp_ ? 1 : 0;
    a.ghq = ghq_.get();
    a.qmax = qmax_.get();
    a.quant = QuantHist() && ghq_.size() >= static_cast<size_t>(K_) * N_ ? 1 : 0;
    a.qbins = std::max(2, config_->num_grad_quant_bins);
    a.qconst = is_const_hess_ ? 1 : 0;
    {
      // one packed g32|h32 word per bin when no expansion's level sums can leave 32 bits
      const double rows = static_cast<double>(N_);
      const double gl = a.qbins / 2, hl = a.qconst ? 1 : a.qbins;
      a.qpack = rows * gl < 2147483647.0 && rows * hl < 4294967295.0 ? 1 : 0;
      // g16|h16 LDS bins: a sub-chunk's per-bin level sums stay within the 16-bit fields
      const int sub = static_cast<int>(std::min(32767.0 / gl, 65535.0 / hl));
      const char* e = KernelOverride("quant_lds32");  // A/B knob: 0 keeps the 64-bit LDS bins
      // single-tile data only: the 1.5x LDS would drop multi-tile grids (several blocks per
      // CU) to one resident block (A/B, 12.5M x 500 GOSS: 87.7 it/s with 64-bit bins, 80.0)
      const bool want = e != nullptr ? e[0] != '0' : num_tiles_ == 1;
      a.qsub = a.quant && !use_dp_ && sub >= 2048 && want ? sub : 0;
    }
    a.hist_il = !use_dp_ && a.qsub == 0 ? HistInterleave() : 0;
    {
      // one wave per scan item on wide data (F >= 64, numerical features only)
      const bool fits = kFScanWaves * FrontierScanWaveBytes(max_bin_, cat_p2_) <= 150 * 1024;
      const char* sw = KernelOverride("scan_wave");  // coverage knob: the wave scan on narrow data
      a.scan_wave = fits && !has_cat_ && !a.mono_inter && (F_ >= 64 || (sw != nullptr && sw[0] == '1')) ? 1 : 0;
      // (block scan grid cap: 512 blocks loop over a large round's items instead of 4096
      // mostly-idle blocks being dispatched every round; A/B 10M 2.850 vs 2.875, 1.25M 1.331 vs 1.341)
      a.scan_grid = 512;
    }
    a.e_lo = 0;
    a.e_hi = kFrontierKmax;
    if (RawCands() && fnuep_.size() > 0) {
      a.cegb_raw = 1;
      a.cegb_tradeoff = config_->cegb_tradeoff;
      a.nkey = fnkey_.get();
      a.ninfo = fninfo_.get();
      a.nuep = fnuep_.get();
      if (CegbCoupled()) {
        a.cegb_coupled = cegb_coupled_.get();
        a.cegb_used = cegb_used_.get();
        a.cegb_epoch = cegb_epoch_.get();
      }
      if (CegbLazy()) {
        a.cegb_lazy = cegb_lazy_.get();
        a.lazy_bits = lazy_bits_.get();
        a.lazy_words = lazy_words_;
        a.lazy_acc = lazy_acc_.get();
        a.nlazy = fnlazy_.get();
        a.npath = fnpath_.get();
      }
    }
    a.spec_cap = fspec_cap_;
    a.policy = fpolicy_;
    a.stamps = fstamps_.size() ? fstamps_.get() : nullptr;
    a.distributed = distributed_ ? 1 : 0;
    a.kcap = fcaps_on_ ? fkcap_.get() : nullptr;
    a.kused = distributed_ ? fkused_.get() : nullptr;
    if (distributed_) {
      // the all-reduced level sums of every rank: packed only when the GLOBAL rows fit
      const double gl = a.qbins / 2, hl = a.qconst ? 1 : a.qbins;
      a.qpack = fglobal_rows_ * gl < 2147483647.0 && fglobal_rows_ * hl < 4294967295.0 ? 1 : 0;
    }
    a.sp = MakeArgs().sp;
    a.bynode = use_bynode_ ? bynode_.get() : nullptr;
    a.byn_draw = frontier_ && ByNodeOnDevice() ? bynode_.get() : nullptr;
    a.byn_mode = fbyn_mode_.size() ? fbyn_mode_.get() : nullptr;
    a.byn_cnt = fbyn_cnt_;
    a.byn_reset = fbyn_reset_;
    a.xrng = config_->extra_trees ? rng_.get() : nullptr;
    if (ffeature_ || fowner_) {
      a.fowned = ffowned_.get();
      a.fpb = ffpb_.get();
      a.vote_P = P_;
      a.vote_rank = rank_;
      a.fown_list = fown_list_.get();
      a.fown_n = fown_n_;
    }
    a.xkb = fkmax_;
    if (fowner_) {
      a.own = 1;
      a.own_P = P_;
      a.own_rank = rank_;
      a.own_w = bbin_;
      a.own_b0 = fown_b0_.get();
      a.acc_recv = facc_recv_.get();
    }
    if (FrontierXg()) {
      // in-kernel exchange: the owner's receive chunk and the per-child best rows live in this
      // rank's exchange buffer; the chunk stride covers every expansion a round can hold
      a.xg = 1;
      a.xsession = 1;
      a.xc = fxconf_.get();
      if (fowner_ || ffeature_) a.fpb = reinterpret_cast<FPairBest*>(fx_local_ + fxo_fpb_);
      if (fowner_) a.acc_recv = reinterpret_cast<unsigned long long*>(fx_local_ + fxo_recv_);
    }
    if (fvoting_) {
      a.voting = 1;
      a.vote_k = topk_;
      a.vote_P = P_;
      a.vote_rank = rank_;
      a.sp_local = fsp_local_.get();
      a.lsum_loc = flsum_loc_.get();
      a.ltot = fltot_.get();
      a.vrec = fvrec_.get();
      a.velect = fvelect_.get();
      a.vrows = reinterpret_cast<unsigned long long*>(fvrows_.get());
      if (FrontierXg()) {
        // (xGMI: the records and rows every rank pushes land in this rank's exchange buffer)
        a.vrec = reinterpret_cast<VoteRec*>(fx_local_ + fxo_vrec_);
        a.vrows = reinterpret_cast<unsigned long long*>(fx_local_ + fxo_vrows_);
      }
    }
    return a;
  }

  // accumulator words per histogram bin of the frontier (k_f_hist): 1 with packed quantized
  // level sums (qpack), else 2
  int AccWordsPerBin() const {
    const FArgs fa = MakeFArgs();
    return fa.quant && fa.qpack ? 1 : 2;
  }

  // Data-parallel frontier: sum the round's accumulators of the first `kb` expansions over
  // the ranks (the rest are zero on every rank).
  void FrontierExchange(int kb) {
    if (!distributed_ || fvoting_ || fowner_) return;
    AllreduceSumU64(reinterpret_cast<unsigned long long*>(facc_.get()),
                    static_cast<size_t>(std::max(1, std::min(kb, fkmax_))) * AccWordsPerBin() * TB_, stream_);
  }

  // Data-parallel rounds with at least two expansions pipeline the exchange with histogram
  // and scan work (RCCL only: the host-staged rehearsal transport synchronises anyway):
  //
  //   compute: partition | hist A | hist B |  wait  | scan A |  wait  | scan B | select
  //   comm:                       | wait A | all-reduce A | wait B | all-reduce B |
  //
  // A / B are the first / second half of the round's expansions (their accumulator rows are
  // contiguous), so half A's all-reduce overlaps half B's histograms and half B's overlaps
  // half A's scans. The histogram grid stops short of the CU count (7/8), which leaves the
  // RCCL kernel CUs of its own. Opt-in (LGAP_DP_PIPELINE=1): on a one-rank communicator the
  // extra launches and the two cross-stream event waits per round cost more than an
  // all-reduce of a round's accumulators (1.25M rows: 529.6 it/s pipelined vs 754.5 serial;
  // 10M: 289.2 vs 361.0; profiles/r03/dp_pipeline_ab.txt), so the serial order is the default
  // until a multi-GPU node shows the overlap paying for them.
  bool FrontierPipelined(int kb) const {
    if (!distributed_ || HostStagedDP() || !CommExists() || kb < 2) return false;
    const char* e = std::getenv("LGAP_DP_PIPELINE");
    return e != nullptr && e[0] == '1';
  }

  void EnsureCommStream() {
    if (comm_stream_ != nullptr) return;
    HIP_CHECK(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking));
    for (auto& ev : pipe_ev_) HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }

  // One round: partition -> histograms -> [all-reduce] -> scans -> select. `kb` bounds the
  // round's expansion count (round r >= 1 of a tree has at most 2^(r-1) open nodes to expand).
  // Voting: after the round's local-pass scan, the vote all-gather, the election, the exact
  // all-reduce of the elected rows (kb expansions' worth), the global pass.
  void FrontierVoteExchange(const FArgs& fa, int kb) {
    if (fa.xg) {
      // xGMI: the records and the elected rows are pushed in-kernel (k_f_vote, k_f_elect)
      LaunchFrontierVote(fa, stream_);
      LaunchFrontierElect(fa, stream_);
      LaunchFrontierVoteScan(fa, FrontierVoteScanLds(), stream_);
      return;
    }
    LaunchFrontierVote(fa, stream_);
    AllGatherInPlace(fvrec_.get(), sizeof(VoteRec) * 2 * static_cast<size_t>(fkmax_) * topk_, stream_);
    LaunchFrontierElect(fa, stream_);
    const size_t rows = 2 * static_cast<size_t>(std::max(1, std::min(kb, fkmax_))) * topk_ * 2 * max_bin_;
    AllreduceSumU64(reinterpret_cast<unsigned long long*>(fvrows_.get()), rows, stream_);
    LaunchFrontierVoteScan(fa, FrontierVoteScanLds(), stream_);
  }
  size_t FrontierVoteScanLds() const {
    return static_cast<size_t>(max_bin_) * 2 * sizeof(double) + static_cast<size_t>(cat_p2_) * (2 * sizeof(int) + sizeof(double));
  }

  // Owner-computes data-parallel round (FrontierOwner): histograms + reduce into the per-rank
  // chunks, the reduce-scatter, owner-only scans, the per-child bests exchanged. `kb` = the
  // round's expansion bound (the chunk stride the reduce and the reduce-scatter agree on).
  void FrontierOwnerRound(const FArgs& fa, int kb) {
    if (fa.xg) {
      // xGMI: k_f_reduce adds into the owners' chunks and completes the exchange in-kernel;
      // the owner scans its features; k_f_pair_best pushes the per-child bests to every rank
      LaunchFrontierHist(fa, FrontierHistLds(), stream_);
      LaunchFrontierScan(fa, fscan_lds_, stream_);
      return;  // (the select pushes the per-child bests and merges the ranks' records)
    }
    FArgs fr = fa;
    fr.xkb = std::max(1, std::min(kb, fkmax_));
    LaunchFrontierHist(fr, FrontierHistLds(), stream_);
    if (fr.cegb_lazy != nullptr) LaunchFrontierLazyCounts(fr, stream_);
    ReduceScatterSumU64(reinterpret_cast<unsigned long long*>(facc_.get()), facc_recv_.get(),
                        static_cast<size_t>(fr.xkb) * bbin_ * AccWordsPerBin(), stream_);
    LaunchFrontierScan(fr, fscan_lds_, stream_);
    FrontierFeatureExchange(fr);
  }

  // Feature parallel: this rank's per-child bests all-gathered (the select takes the best over
  // ranks in its phase A: no merge launch). CEGB's raw per-feature candidates would need every
  // feature's scan on every rank: those configurations never reach these modes (FrontierOwner,
  // the factory's FrontierServes).
  void FrontierFeatureExchange(const FArgs& fa) {
    if (fa.cegb_raw) Log::Fatal("frontier feature exchange: raw CEGB candidates are not exchanged");
    if (fa.xg) return;  // (xGMI: the select pushes the per-child bests and merges the ranks' records)
    LaunchFrontierPairBest(fa, stream_);
    AllGatherInPlace(ffpb_.get(), sizeof(FPairBest) * 2 * static_cast<size_t>(fkmax_), stream_);
  }

  void EnqueueFrontierRound(const FArgs& fa, int kb) {
    LaunchFrontierPartition(fa, fpart_iters_, fpart_grid_, stream_);
    if (fowner_) {
      FrontierOwnerRound(fa, kb);
      LaunchFrontierSelect(fa, stream_);
      return;
    }
    if (fa.cegb_lazy != nullptr) LaunchFrontierLazyCounts(fa, stream_);
    if (ffeature_) {
      LaunchFrontierHist(fa, FrontierHistLds(), stream_);
      LaunchFrontierScan(fa, fscan_lds_, stream_);
      FrontierFeatureExchange(fa);
    } else if (fvoting_) {
      LaunchFrontierHist(fa, FrontierHistLds(), stream_);
      LaunchFrontierScan(fa, fscan_lds_, stream_);
      FrontierVoteExchange(fa, kb);
    } else if (!FrontierPipelined(kb)) {
      LaunchFrontierHist(fa, FrontierHistLds(), stream_);
      FrontierExchange(kb);
      LaunchFrontierScan(fa, fscan_lds_, stream_);
    } else {
      EnsureCommStream();
      kb = std::min(kb, fkmax_);
      const int kh = (kb + 1) / 2;
      FArgs fa_a = fa, fa_b = fa;
      fa_a.e_hi = kh;
      fa_b.e_lo = kh;
      auto* acc = reinterpret_cast<unsigned long long*>(facc_.get());
      const size_t row = static_cast<size_t>(AccWordsPerBin()) * TB_;
      LaunchFrontierHist(fa_a, FrontierHistLds(), stream_);
      HIP_CHECK(hipEventRecord(pipe_ev_[0], stream_));
      LaunchFrontierHist(fa_b, FrontierHistLds(), stream_);
      HIP_CHECK(hipEventRecord(pipe_ev_[1], stream_));
      HIP_CHECK(hipStreamWaitEvent(comm_stream_, pipe_ev_[0], 0));
      AllreduceSumU64(acc, static_cast<size_t>(kh) * row, comm_stream_);
      HIP_CHECK(hipEventRecord(pipe_ev_[2], comm_stream_));
      HIP_CHECK(hipStreamWaitEvent(comm_stream_, pipe_ev_[1], 0));
      AllreduceSumU64(acc + static_cast<size_t>(kh) * row, static_cast<size_t>(kb - kh) * row, comm_stream_);
      HIP_CHECK(hipEventRecord(pipe_ev_[3], comm_stream_));
      HIP_CHECK(hipStreamWaitEvent(stream_, pipe_ev_[2], 0));
      LaunchFrontierScan(fa_a, fscan_lds_, stream_);
      HIP_CHECK(hipStreamWaitEvent(stream_, pipe_ev_[3], 0));
      LaunchFrontierScan(fa_b, fscan_lds_, stream_);
      ++fstat_pipelined_;
    }
    LaunchFrontierSelect(fa, stream_);
  }

  // The root round (setup, root sums, root histogram and scan, first select), then `rounds`
  // rounds; a finished tree turns the remaining launches into early exits.
  void EnqueueFrontier(int rounds, bool prologue) {
    const FArgs fa = MakeFArgs();
    if (prologue) {
      Args ra = MakeArgs(0);
      ra.lsum = flsum_;  // root sums -> the root node; ghmax -> the fixed-point scales
      const int root_blocks = RootBlocks();
      k_root_sums<<<root_blocks, kRootThreads, 0, stream_>>>(ra);
      HIP_CHECK(hipGetLastError());
      // the tree setup and k_root_final's fold of the partials in one launch
      LaunchFrontierInitRoot(fa, ra.root_part, root_blocks, ghmax_.get(), stream_);
      if (distributed_ && fa.xg) {
        // global root sums and gradient maxima, exchanged in-kernel (xGMI transport)
        LaunchFrontierXRoot(fa, ghmax_.get(), stream_);
      } else if (distributed_) {
        // global root sums and gradient maxima (the fixed-point scales must agree on all ranks)
        AllreduceSumF64(reinterpret_cast<double*>(flsum_), 2, stream_);
        AllreduceMaxU32(ghmax_.get(), 4, stream_);
      }
      if (fowner_) {
        FrontierOwnerRound(fa, 1);
      } else {
        LaunchFrontierHist(fa, FrontierHistLds(), stream_);
        if (fa.cegb_lazy != nullptr) LaunchFrontierLazyCounts(fa, stream_);
        FrontierExchange(1);
        LaunchFrontierScan(fa, fscan_lds_, stream_);
        if (fvoting_) FrontierVoteExchange(fa, 1);
        if (ffeature_) FrontierFeatureExchange(fa);
      }
      LaunchFrontierSelect(fa, stream_);
    }
    for (int r = 0; r < rounds; ++r) {
      // round r + 1 of the tree (main replay) has at most 2^r open nodes, and at most its cap
      int kb = prologue && r < 7 ? (1 << r) : fkmax_;
      if (prologue && fcaps_on_ && r + 1 < kFrontierRoundCap) kb = std::min(kb, fcap_host_[r + 1]);
      fstat_ar_exps_ += distributed_ ? std::max(1, std::min(kb, fkmax_)) : 0;
      EnqueueFrontierRound(fa, kb);
    }
  }

  // Data-parallel: expansions round r (>= 1) may take: the bound 2^(r-1), tightened to 1.5x the
  // most any of the last 4 trees took in that round (+1, at least 2). Identical on every rank
  // (the history comes from the replicated select), so every rank sizes its all-reduces alike.
  int FrontierRoundCap(int r) const {
    int c = std::min(fkmax_, r - 1 < 7 ? (1 << (r - 1)) : fkmax_);
    if (fkused_trees_ > 0) {
      int m = 0;
      for (int t = 0; t < std::min(fkused_trees_, 4); ++t) m = std::max(m, fkused_hist_[t][r]);
      c = std::min(c, std::max(2, (3 * m + 1) / 2 + 1));
    }
    return std::max(1, c);
  }

  hipGraphExec_t CaptureFrontier(int rounds, bool prologue) {
    hipGraph_t g;
    hipGraphExec_t ex = nullptr;
    HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    EnqueueFrontier(rounds, prologue);
    HIP_CHECK(hipStreamEndCapture(stream_, &g));
    HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    return ex;
  }

  // Grow one tree: the root round plus a predicted number of rounds (the previous trees'
  // count) in one replay; if the tree is not finished, continuation replays of a few rounds
  // each until it is. Results: the committed splits, the final leaf ranges, the root output.
  // a stream carrying RCCL collectives: a lost peer must not hang the process
  void FrontierSync() {
    if ((distributed_ || ffeature_) && !HostStagedDP() && !FrontierXg()) {
      WatchedStreamSync(stream_, CommTimeoutSeconds(config_->time_out), "frontier tree growth (RCCL all-reduce)");
    } else {
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
  }

  void FrontierGrow(int* num_splits, int* num_leaves, SplitRec* hr, LeafRange* hrange, double* hlo) {
    // collectives: RCCL calls replay from the graph only on request (LGAP_DP_GRAPH=1, as in the
    // sequential chain); the host-staged rehearsal transport synchronises inside its exchange
    // (feature parallel exchanges candidates over collectives too, without distributed rows)
    // (the xGMI transport keeps every exchange inside the kernels: a tree replays as one graph)
    const bool comm = (distributed_ || ffeature_) && !FrontierXg();
    const bool use_graph = config_->device_use_graph && (!comm || (DPGraphEnabled() && !HostStagedDP()));
    if (use_graph && comm && !fgraphs_.empty() && graph_comm_ != ActiveComm()) InvalidateGraph();
    if (use_graph && comm) graph_comm_ = ActiveComm();
    // per-round caps need the eager enqueue (the all-reduce sizes change from tree to tree)
    fcaps_on_ = distributed_ && !use_graph && !FrontierXg();
    if (distributed_) {
      if (fkused_.size() < static_cast<size_t>(kFrontierRoundCap)) {
        fkused_.Resize(kFrontierRoundCap);
        fkcap_.Resize(kFrontierRoundCap);
      }
      fkused_.Zero(stream_);
      if (fcaps_on_) {
        const int pr = std::max(1, std::min(fpred_rounds_, L_));
        int* hc = pin_kcap_.Get(kFrontierRoundCap);
        for (int r = 0; r < kFrontierRoundCap; ++r) {
          fcap_host_[r] = r == 0 ? 1 : (r <= pr ? FrontierRoundCap(r) : fkmax_);
          hc[r] = fcap_host_[r];
        }
        HIP_CHECK(hipMemcpyAsync(fkcap_.get(), hc, sizeof(int) * kFrontierRoundCap, hipMemcpyHostToDevice, stream_));
      }
    }
    const int pred = std::max(1, std::min(fpred_rounds_, L_));
    const FResultHdr* hh = reinterpret_cast<const FResultHdr*>(fres_host_);
    const FState* hs = &hh->st;
    const FArgs fa_res = MakeFArgs();
    if (fgraph_gh_ != gh_.get()) {  // captured launches hold the gradient buffer's address
      InvalidateGraph();
      fgraph_gh_ = gh_.get();
    }
    if (use_graph) {
      auto it = fgraphs_.find(pred);
      if (it == fgraphs_.end()) it = fgraphs_.emplace(pred, CaptureFrontier(pred, true)).first;
      HIP_CHECK(hipGraphLaunch(it->second, stream_));
    } else {
      EnqueueFrontier(pred, true);
    }
    constexpr int kCont = 4;
    int launched = pred;
    for (;;) {
      LaunchFrontierResults(fa_res, fres_dev_, stream_);
      FrontierSync();
      if (hs->done) {
        // CEGB lazy: the final leaves' rows are marked for their paths' features (stream order:
        // before the next tree's replay)
        if (fa_res.cegb_lazy != nullptr) LaunchFrontierLazyMark(fa_res, stream_);
        break;
      }
      // (intermediate monotone: a split may wait on a round of rescans and one of expansion)
      // (a bound against a replay that stops advancing; each split needs at most an expansion, a
      // rescan and a re-expansion round, several per split when its speculation is voided)
      if (launched > (MonoInter() ? 6 : 1) * L_ + 2 * kCont) Log::Fatal("frontier tree: not finished after %d rounds", launched);
      if (use_graph) {
        if (!fcont_) fcont_ = CaptureFrontier(kCont, false);
        HIP_CHECK(hipGraphLaunch(fcont_, stream_));
      } else {
        EnqueueFrontier(kCont, false);
      }
      launched += kCont;
    }
    // speculation feedback: the fraction of partitioned rows spent on expansions the tree never
    // committed steers the next tree's speculation depth (deep, chain-like trees waste more)
    const double rows_all = static_cast<double>(hs->used_rows + hs->waste_rows);
    if (rows_all > 0 && !fspec_fixed_) {
      const double waste = static_cast<double>(hs->waste_rows) / rows_all;
      if (waste > 0.12) fspec_alpha_ = std::max(0.15, fspec_alpha_ * 0.75);
      else if (waste < 0.04) fspec_alpha_ = std::min(1.0, fspec_alpha_ * 1.2);
    }
    fstat_waste_ += rows_all > 0 ? static_cast<double>(hs->waste_rows) / rows_all : 0.0;
    // rounds the tree needed (selects run after the root's) -> next tree's replay length
    const int used = std::max(1, hs->round - 1);
    frounds_hist_[frounds_pos_++ % 4] = used;
    int mx = 1;
    for (int v : frounds_hist_) mx = std::max(mx, v);
    fpred_rounds_ = mx;
    fstat_rounds_ += used;
    fstat_spec_ += hs->spec;
    fstat_trees_ += 1;
    *num_splits = hs->num_splits;
    *num_leaves = hs->num_leaves;
    bynode_draws_ = hs->byn;
    bynode_rng_ = hs->byn_rng;
    // (k_f_results already wrote the records, ranges, root output and flags with the state)
    if (*num_splits > 0) std::memcpy(hr, fres_host_ + FrontierResultRecOffset(), sizeof(SplitRec) * *num_splits);
    std::memcpy(hrange, fres_host_ + FrontierResultRangeOffset(L_), sizeof(LeafRange) * *num_leaves);
    *hlo = hh->lout0;
    unsigned hbar[4];
    std::memcpy(hbar, hh->bar, sizeof(hbar));
    if (hbar[3] != 0u) {
      static const char* const kinds[kFXKinds] = {"histogram", "split candidates", "root sums", "self-test"};
      Log::Fatal("xGMI exchange (%s) timed out on rank %d after %.0f s: a peer stopped training",
                 kinds[std::min<unsigned>(hbar[3] - 1u, kFXKinds - 1)], rank_, XTimeoutSeconds());
    }
    if (distributed_) {
      std::memcpy(fkused_hist_[fkused_trees_ % 4], hh->kused, sizeof(int) * kFrontierRoundCap);
      ++fkused_trees_;
    }
    if (fstamps_.size() && fstat_trees_ == 3) ReportFrontierStamps(hs->round);
    if (fstamps_.size() && fstat_trees_ % 10 == 0) {  // (LGAP_FSTAMPS: stamps and round statistics)
      std::fprintf(stderr, "frontier: %d trees, %.2f rounds/tree, %.2f expansions/tree (%d leaves max), wasted rows %.1f%%, "
                   "alpha %.3f, all-reduced expansion slots/tree %.1f, pipelined rounds/tree %.2f\n", fstat_trees_,
                   static_cast<double>(fstat_rounds_) / fstat_trees_, static_cast<double>(fstat_spec_) / fstat_trees_, L_,
                   100.0 * fstat_waste_ / fstat_trees_, stune_.on ? stune_.lo : fspec_alpha_, fstat_ar_exps_ / fstat_trees_,
                   static_cast<double>(fstat_pipelined_) / fstat_trees_);
    }
  }

  // Mean phase offsets (us from each kernel's block-0 start) over the rounds of the last
  // tree, and the round chain: select -> partition -> hist -> scan -> next select.
  void ReportFrontierStamps(int rounds) {
    std::vector<unsigned long long> h(fstamps_.size());
    fstamps_.Download(h.data(), h.size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    static const char* names[4] = {"partition", "hist", "scan", "select"};
    auto at = [&](int r, int k, int i) { return h[(static_cast<size_t>(r) * 4 + k) * kFStampSlots + i]; };
    for (int k = 0; k < 4; ++k) {
      double acc[kFStampSlots] = {0};
      int cnt = 0;
      for (int r = 0; r < std::min(rounds + 1, 256); ++r) {
        const unsigned long long s0 = at(r, k, 0);
        if (!s0) continue;
        ++cnt;
        for (int i = 1; i < kFStampSlots; ++i) {
          const unsigned long long v = at(r, k, i);
          if (v >= s0) acc[i] += (v - s0) * 0.01;
        }
      }
      if (!cnt) continue;
      std::string line;
      for (int i = 1; i < kFStampSlots; ++i) {
        if (acc[i] > 0) line += " t" + std::to_string(i) + "=" + common::FormatG(acc[i] / cnt);
      }
      std::fprintf(stderr, "fstamps %s (%d rounds, us from block-0 start; t7 = last block exit):%s\n", names[k], cnt,
                   line.c_str());
      if (at(0, k, 0)) {
        // the root round alone (the largest histogram / partition of the tree)
        std::string root;
        for (int i = 1; i < kFStampSlots; ++i) {
          const unsigned long long v = at(0, k, i);
          if (v >= at(0, k, 0) && v) root += " t" + std::to_string(i) + "=" + common::FormatG((v - at(0, k, 0)) * 0.01);
        }
        std::fprintf(stderr, "fstamps %s root round:%s\n", names[k], root.c_str());
      }
    }
    double gap[4] = {0};
    int cnt = 0;
    for (int r = 1; r + 1 < std::min(rounds, 255); ++r) {
      const unsigned long long P = at(r, 0, 0), H = at(r, 1, 0), S = at(r, 2, 0), Q = at(r, 3, 0), P2 = at(r + 1, 0, 0);
      if (!P || !H || !S || !Q || !P2 || !(P < H && H < S && S < Q && Q < P2)) continue;
      gap[0] += (H - P) * 0.01;
      gap[1] += (S - H) * 0.01;
      gap[2] += (Q - S) * 0.01;
      gap[3] += (P2 - Q) * 0.01;
      ++cnt;
    }
    if (cnt) {
      std::fprintf(stderr, "fstamps chain (%d rounds, start to start, us): partition->hist %.2f hist->scan %.2f "
                   "scan->select %.2f select->partition %.2f\n", cnt, gap[0] / cnt, gap[1] / cnt, gap[2] / cnt, gap[3] / cnt);
    }
  }

  // The one-split-at-a-time device tree (one fixed kernel chain per split, replayed from a
  // hipGraph): the path of the distributed learners and of the options the frontier engine
  // does not cover (feature_fraction_bynode, extra_trees, global-memory scans).
  void SequentialGrow(int* num_splits, int* num_leaves, SplitRec* hr, LeafRange* hrange, double* hlo) {
    // LGAP_DP_GRAPH=1 also captures the RCCL data-parallel tree (the per-split ncclAllReduce
    // calls replay from the graph). Off by default: on a one-rank communicator it measured
    // 358 it/s captured vs 368 eager at 1.25M rows (profiles/README.md), and the eager host
    // enqueue stays ahead of the ~40 us splits. The host-staged rehearsal transport
    // synchronises inside its all-reduce and is never captured.
    // the xGMI transport keeps every exchange inside the kernels: the tree replays as one graph
    const bool collectives = owner_scan_ || voting_;
    const bool use_graph = config_->device_use_graph && (!collectives || (DPGraphEnabled() && !HostStagedDP()));
    if (use_graph) {
      if (graph_exec_ && distributed_ && graph_comm_ != ActiveComm()) InvalidateGraph();
      if (!graph_exec_) CaptureGraph();
      HIP_CHECK(hipGraphLaunch(graph_exec_, stream_));
    } else {
      EnqueueTree();
    }
    // results
    Ctl* hc2 = pin_ctl_.Get(2);
    HIP_CHECK(hipMemcpyAsync(hc2, ctl_.get(), 2 * sizeof(Ctl), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(hr, rec_.get(), sizeof(SplitRec) * (L_ - 1), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(hrange, range_.get(), sizeof(LeafRange) * L_, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(hlo, lout_.get(), sizeof(double), hipMemcpyDeviceToHost, stream_));
    unsigned* hbar = pin_bar_.Get(4);
    HIP_CHECK(hipMemcpyAsync(hbar, bar_.get(), 4 * sizeof(unsigned), hipMemcpyDeviceToHost, stream_));
    if (collectives && !HostStagedDP()) {
      // the tree's collectives ride on this stream: a lost peer must not hang us
      static const double timeout_s = CommTimeoutSeconds(config_->time_out);
      WatchedStreamSync(stream_, timeout_s, "device tree growth (RCCL histogram reduce-scatter)");
    } else {
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
    if (hbar[2] != 0u) Log::Fatal("k_partition: a wait on published tile counts timed out (blocks not co-resident?)");
    // the control buffer written last holds the final tree state
    const Ctl* hc = hc2[1].num_splits > hc2[0].num_splits ? &hc2[1] : &hc2[0];
    bynode_draws_ = 1 + 2 * hc->scan_round;  // the root's mask, two per scanned split
    *num_splits = hc->num_splits;
    *num_leaves = hc->num_leaves;
  }

  std::string DeviceName() const override {
    if (!owner_scan_ && !voting_) {
      if (!FrontierEligible()) return device_name_;
      if (MonoInter()) return device_name_ + " [frontier engine, intermediate monotone walk + rescans]";
      return device_name_ + (QuantHist() ? " [frontier engine, int8-level histograms]" : " [frontier engine]");
    }
    return device_name_ + " [" + ParallelDesc() + "]";
  }

  void ReportStamps(int nsplits) {
    std::vector<unsigned long long> h(stamps_.size());
    stamps_.Download(h.data(), h.size(), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    static const char* names[5] = {"part_count", "part_scatter", "hist", "reduce_scan", "post"};
    auto at = [&](int k, int sp, int b, int i) { return h[((static_cast<size_t>(k) * 256 + sp) * 2 + b) * 8 + i]; };
    {
      // start-to-start of block 0 along the per-split chain hist(j) -> scan(j) -> partition(j) -> hist(j+1)
      double hs = 0, sp_ = 0, ph = 0;
      int cnt = 0;
      for (int j = 1; j + 1 < std::min(nsplits, 255); ++j) {
        const unsigned long long H = at(2, j, 0, 0), S = at(3, j, 0, 0), P = at(0, j, 0, 0), H2 = at(2, j + 1, 0, 0);
        if (!H || !S || !P || !H2 || !(H < S && S < P && P < H2)) continue;
        hs += (S - H) * 0.01;
        sp_ += (P - S) * 0.01;
        ph += (H2 - P) * 0.01;
        ++cnt;
      }
      double e_h = 0, e_s = 0, e_p = 0;
      int ce = 0;
      for (int j = 1; j + 1 < std::min(nsplits, 255); ++j) {
        const unsigned long long H = at(2, j, 0, 0), S = at(3, j, 0, 0), P = at(0, j, 0, 0), H2 = at(2, j + 1, 0, 0);
        const unsigned long long He = at(2, j, 0, 7), Se = at(3, j, 0, 7), Pe = at(0, j, 0, 7);
        if (!H || !S || !P || !H2 || !He || !Se || !Pe) continue;
        e_h += (static_cast<double>(He) - H) * 0.01;
        e_s += (static_cast<double>(Se) - S) * 0.01;
        e_p += (static_cast<double>(Pe) - P) * 0.01;
        ++ce;
      }
      if (ce) {
        std::fprintf(stderr, "stamps kernel spans (%d splits, block-0 start to last block exit, us): hist %.2f scan %.2f "
                     "partition %.2f\n", ce, e_h / ce, e_s / ce, e_p / ce);
      }
      if (cnt) {
        std::fprintf(stderr, "stamps chain (%d splits, block-0 start to start, us): hist->scan %.2f scan->partition %.2f "
                     "partition->hist %.2f\n", cnt, hs / cnt, sp_ / cnt, ph / cnt);
      }
    }
    for (int k = 0; k < 5; ++k) {
      for (int b = 0; b < 2; ++b) {
        double acc[8] = {0};
        int cnt = 0;
        for (int sp = 1; sp < std::min(nsplits, 255); ++sp) {
          const unsigned long long* st = &h[((static_cast<size_t>(k) * 256 + sp) * 2 + b) * 8];
          if (st[0] == 0) continue;
          ++cnt;
          for (int i = 1; i < 8; ++i) {
            if (st[i] >= st[0]) acc[i] += (st[i] - st[0]) * 0.01;  // 100 MHz -> us
          }
        }
        if (!cnt) continue;
        std::string line;
        for (int i = 1; i < 8; ++i) {
          if (acc[i] > 0) line += " t" + std::to_string(i) + "=" + common::FormatG(acc[i] / cnt);
        }
        std::fprintf(stderr, "stamps %s block %d (%d splits, us from kernel start):%s\n", names[k], b, cnt, line.c_str());
      }
    }
  }

  void QuantizeGradients(int class_id) {
    float2* gh = gh_.get() + static_cast<size_t>(class_id) * N_;
    const bool renew = config_->quant_train_renew_leaf;
    if (renew && gh_true_.size() < static_cast<size_t>(N_)) gh_true_.Resize(N_);
    qmax_.Zero(stream_);
    const int grid = std::max(1, std::min(DivUp(N_, 256), num_cu_ * 4));
    k_qmax<<<grid, 256, 0, stream_>>>(gh, N_, qmax_.get());
    HIP_CHECK(hipGetLastError());
    if (Network::num_machines() > 1) {
      unsigned* hm = pin_max_.Get(2);
      qmax_.Download(hm, 2, stream_);
      HIP_CHECK(hipStreamSynchronize(stream_));
      float v[2];
      std::memcpy(v, hm, 8);
      v[0] = static_cast<float>(Network::GlobalSyncUpByMax(static_cast<double>(v[0])));
      v[1] = static_cast<float>(Network::GlobalSyncUpByMax(static_cast<double>(v[1])));
      std::memcpy(hm, v, 8);
      HIP_CHECK(hipMemcpyAsync(qmax_.get(), hm, 8, hipMemcpyHostToDevice, stream_));
    }
    const uint32_t seed = static_cast<uint32_t>(config_->seed) * 0x9E3779B9u + (quant_round_++);
    uint16_t* ghq = nullptr;
    if (QuantHist()) {
      if (ghq_.size() < static_cast<size_t>(K_) * N_) {
        ghq_.Resize(static_cast<size_t>(K_) * N_);
        InvalidateGraph();  // captured frontier rounds hold the buffer's address
      }
      ghq = ghq_.get() + static_cast<size_t>(class_id) * N_;
    }
    k_quantize<<<grid, 256, 0, stream_>>>(gh, renew ? gh_true_.get() : nullptr, ghq, N_, qmax_.get(),
                                          std::max(2, config_->num_grad_quant_bins), is_const_hess_ ? 1 : 0, seed,
                                          config_->stochastic_rounding ? 1 : 0);
    HIP_CHECK(hipGetLastError());
  }

  // the frontier histogram's dynamic LDS: the tile plan's, plus the 32-bit bins of hist MODE 3
  size_t FrontierHistLds() const {
    const FArgs fa = MakeFArgs();
    // (the interleaved slots' reserve only where k_f_hist can use them: fixed-point and MODE 2)
    const size_t plan = use_dp_ || fa.qsub > 0 ? hist_lds_plain_ : hist_lds_bytes_;
    const size_t b = use_dp_ || !QuantHist() || fa.qsub == 0 ? plan : plan * 3 / 2 + 64;
    return b;
  }

  // Integer-level histograms for quantized training (frontier hist MODE 2): int8 g and
  // uint8 h levels, i.e. num_grad_quant_bins <= 254.
  bool QuantHist() const {
    return config_->use_quantized_grad && std::max(2, config_->num_grad_quant_bins) <= 254 &&
           KernelOverride("quant_hist") == nullptr;  // LGAP_KERNEL=quant_hist=off: A/B against float histograms
  }

  void RenewQuantizedLeaves(Tree* tree) {
    const int nl = tree->num_leaves();
    const Args args = MakeArgs();
    k_leaf_true_sums<<<nl, kNodeThreads, 0, stream_>>>(args, gh_true_.get(), nl, true_sums_.get());
    HIP_CHECK(hipGetLastError());
    std::vector<double2> st(nl);
    true_sums_.Download(st.data(), nl, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    std::vector<double> flat(2 * nl);
    for (int l = 0; l < nl; ++l) flat[2 * l] = st[l].x, flat[2 * l + 1] = st[l].y;
    if (distributed_) Network::GlobalSum(&flat);
    SplitParams p = MakeArgs().sp;
    p.path_smooth = 0.0;
    for (int l = 0; l < nl; ++l) {
      tree->SetLeafOutput(l, LeafOutputRaw(flat[2 * l], flat[2 * l + 1], p, tree->leaf_count(l), 0.0));
    }
  }

  // ---- histogram engine for the host learners (HistogramBackend)
  void BackendSetGradients(const float* g, const float* h, int n) {
    if (n != N_) Log::Fatal("HistogramBackend: %d gradients for %d rows", n, N_);
    K_ = 1;
    if (gh_.size() < static_cast<size_t>(N_)) gh_.Resize(static_cast<size_t>(N_));
    DeviceSetGradients(g, h, 1);
    float mg = 0.f, mh = 0.f;
    for (int i = 0; i < N_; ++i) {
      mg = std::max(mg, std::fabs(g[i]));
      mh = std::max(mh, std::fabs(h[i]));
    }
    unsigned* hm = pin_max_.Get(2);
    std::memcpy(&hm[0], &mg, 4);
    std::memcpy(&hm[1], &mh, 4);
    HIP_CHECK(hipMemcpyAsync(ghmax_.get(), hm, 8, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void BackendHistogram(const int* rows, int n, double* out) {
    if (n == 0) {
      std::memset(out, 0, sizeof(double) * 2 * static_cast<size_t>(TB_));
      return;
    }
    BackendHistogramStaging(rows, n);
    staging_.Download(out, 2 * static_cast<size_t>(TB_), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  // the same histogram left on the device, in `dst` (2 * TB doubles)
  void BackendHistogramDevice(const int* rows, int n, double* dst) {
    if (n == 0) {
      HIP_CHECK(hipMemsetAsync(dst, 0, sizeof(double) * 2 * static_cast<size_t>(TB_), stream_));
      return;
    }
    BackendHistogramStaging(rows, n);
    HIP_CHECK(hipMemcpyAsync(dst, staging_.get(), sizeof(double) * 2 * static_cast<size_t>(TB_),
                             hipMemcpyDeviceToDevice, stream_));
    // (the row upload below reuses idx_[2] and the pinned control records: one histogram in flight)
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  hipStream_t BackendStream() const { return stream_; }

  void BackendHistogramStaging(const int* rows, int n) {
    // a full row set is order-free for a histogram: skip the index upload
    const bool all = rows == nullptr || n == N_;
    if (!all) idx_[2].Upload(rows, n, stream_);
    Ctl* hc = pin_ctl_.Get(1);
    std::memset(hc, 0, sizeof(Ctl));
    hc->num_leaves = 1;
    hc->larger = -1;
    LeafRange* hr = pin_range_.Get(L_);
    hr[0].buf = all ? -1 : 2;
    hr[0].start = 0;
    hr[0].count = all ? N_ : n;
    hr[0].pad = 0;
    HIP_CHECK(hipMemcpyAsync(ctl_.get(), hc, sizeof(Ctl), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(range_.get(), hr, sizeof(LeafRange), hipMemcpyHostToDevice, stream_));
    staging_.Zero(stream_);
    const Args args = MakeArgs();
    LaunchHist(args, /*collective=*/false);
    LaunchHistReduce(args);
  }

  // One histogram of (g, h) over `rows` (identity when null) into `out` (2 * TB doubles).
  // ---- direct tests of the frontier's production kernels (tests/test_frontier_kernels.py)

  // The root round's k_f_scan (init, root sums, k_f_hist, k_f_scan over all rows) -> out[F][8]
  // per feature: gain, threshold, left count, default_left, left sum g, left sum h, valid,
  // categorical thresholds; ref[F][8] the host's split_math.h scan of the exact fp64 histogram
  // of the same rows (FindBestNumerical / FindBestCategorical with the learner's SplitParams).
  void TestFrontierScan(const float* g, const float* h, double* out, double* ref) {
    if (!frontier_) Log::Fatal("TestFrontierScan: the frontier engine is not enabled for this configuration");
    K_ = 1;
    DeviceSetGradients(g, h, 1);
    TreeParams* tp = pin_tp_.Get(1);
    std::memset(tp, 0, sizeof(TreeParams));
    tp->root_buf = -1;
    tp->root_count = tp->root_gcount = N_;
    tp->spec_alpha = 1.f;
    HIP_CHECK(hipMemcpyAsync(tparams_.get(), tp, sizeof(TreeParams), hipMemcpyHostToDevice, stream_));
    if (config_->use_quantized_grad) QuantizeGradients(0);
    {
      uint8_t* um = pin_mask_.Get(static_cast<size_t>(F_));
      std::memset(um, 1, static_cast<size_t>(F_));  // every feature in use (no feature_fraction)
      HIP_CHECK(hipMemcpyAsync(used_bytree_.get(), um, F_, hipMemcpyHostToDevice, stream_));
    }
    const FArgs fa = MakeFArgs();
    LaunchFrontierInit(fa, stream_);
    Args ra = MakeArgs(0);
    ra.lsum = flsum_;
    const int root_blocks = RootBlocks();
    k_root_sums<<<root_blocks, kRootThreads, 0, stream_>>>(ra);
    k_root_final<<<1, kRootThreads, 0, stream_>>>(ra, root_blocks);
    HIP_CHECK(hipGetLastError());
    facc_.Zero(stream_);
    LaunchFrontierHist(fa, FrontierHistLds(), stream_);
    LaunchFrontierScan(fa, fscan_lds_, stream_);
    std::vector<SplitInfo> dev(F_);
    double2 root_sum;
    HIP_CHECK(hipMemcpyAsync(dev.data(), fcinfo_, sizeof(SplitInfo) * F_, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(&root_sum, flsum_, sizeof(double2), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    facc_.Zero(stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    auto put = [](double* o, const SplitInfo& si) {
      o[0] = si.gain;
      o[1] = static_cast<double>(si.threshold);
      o[2] = static_cast<double>(si.left_count);
      o[3] = si.default_left ? 1.0 : 0.0;
      o[4] = si.left_sum_gradient;
      o[5] = si.left_sum_hessian;
      o[6] = si.feature >= 0 ? 1.0 : 0.0;
      o[7] = static_cast<double>(si.num_cat_threshold);
    };
    for (int f = 0; f < F_; ++f) put(out + 8 * static_cast<size_t>(f), dev[f]);
    // host oracle: the same rows' exact fp64 histogram and the split_math.h scans, over the
    // device's own (g, h) (quantized training: the de-quantized levels k_quantize left in gh)
    std::vector<float2> ghd(N_);
    HIP_CHECK(hipMemcpy(ghd.data(), gh_.get(), sizeof(float2) * N_, hipMemcpyDeviceToHost));
    std::vector<double> hg(N_), hh(N_);
    for (int i = 0; i < N_; ++i) {
      hg[i] = ghd[i].x;
      hh[i] = ghd[i].y;
    }
    double sg = 0.0, sh = 0.0;
    for (int i = 0; i < N_; ++i) {
      sg += hg[i];
      sh += hh[i];
    }
    const SplitParams sp = fa.sp;
    SplitParams p0 = sp;
    p0.path_smooth = 0.0;
    const double po = LeafOutputRaw(root_sum.x, root_sum.y, p0, N_, 0.0);
    for (int f = 0; f < F_; ++f) {
      const FeatureInfo& fi = data_->feature(f);
      std::vector<double> full(2 * static_cast<size_t>(fi.num_bin), 0.0);
      for (int i = 0; i < N_; ++i) {
        const uint32_t b = data_->FeatureBin(i, f);
        full[2 * b] += hg[i];
        full[2 * b + 1] += hh[i];
      }
      FeatureScanMeta m;
      m.num_bin = fi.num_bin;
      m.default_bin = fi.default_bin;
      m.missing_type = static_cast<int8_t>(fi.missing);
      m.bin_type = static_cast<int8_t>(fi.bin_type);
      m.monotone = fi.monotone;
      m.penalty = fi.penalty;
      SplitInfo r;
      r.Reset();
      bool ok;
      if (fi.bin_type == BinType::Numerical) {
        ok = FindBestNumerical(full.data(), m, sp, sg, sh, N_, po, LeafBounds(), &r);
      } else {
        std::vector<int> order(fi.num_bin);
        ok = FindBestCategorical(full.data(), m, sp, sg, sh, N_, po, LeafBounds(), order.data(), &r);
      }
      r.feature = ok ? f : -1;
      if (!ok) r.gain = kMinScore;
      put(ref + 8 * static_cast<size_t>(f), r);
    }
  }

  // k_f_hist over k row subsets at once (one expansion each, as a round of the frontier):
  // out[k][TB][2] = the accumulators at the tree's global fixed-point scale (quantized
  // training: the integer level sums), levels[N] = the quantized levels (g << 8 | h).
  void TestFrontierHist(const float* g, const float* h, const int* rows, const int* offsets, int k, double* out,
                        uint16_t* levels) {
    if (!frontier_) Log::Fatal("TestFrontierHist: the frontier engine is not enabled for this configuration");
    if (k < 1 || k > fkmax_) Log::Fatal("TestFrontierHist: %d subsets (1..%d)", k, fkmax_);
    const int total = offsets[k];
    if (idx_[3].size() < static_cast<size_t>(total)) idx_[3].Resize(total);  // (subsets may overlap)
    K_ = 1;
    DeviceSetGradients(g, h, 1);
    TreeParams* tp = pin_tp_.Get(1);
    std::memset(tp, 0, sizeof(TreeParams));
    tp->root_buf = -1;
    tp->root_count = tp->root_gcount = N_;
    tp->spec_alpha = 1.f;
    HIP_CHECK(hipMemcpyAsync(tparams_.get(), tp, sizeof(TreeParams), hipMemcpyHostToDevice, stream_));
    // the scale bounds of k_root_final: max |value| and sum |value| (rounded up)
    float bnd[4] = {0.f, 0.f, 0.f, 0.f};
    double sg = 0.0, sh = 0.0;
    for (int i = 0; i < N_; ++i) {
      bnd[0] = std::max(bnd[0], std::fabs(g[i]));
      bnd[1] = std::max(bnd[1], std::fabs(h[i]));
      sg += std::fabs(static_cast<double>(g[i]));
      sh += std::fabs(static_cast<double>(h[i]));
    }
    bnd[2] = std::nextafter(static_cast<float>(sg * (1.0 + 0x1p-20)), INFINITY);
    bnd[3] = std::nextafter(static_cast<float>(sh * (1.0 + 0x1p-20)), INFINITY);
    unsigned* hm = pin_max_.Get(4);
    std::memcpy(hm, bnd, 16);
    HIP_CHECK(hipMemcpyAsync(ghmax_.get(), hm, 16, hipMemcpyHostToDevice, stream_));
    if (config_->use_quantized_grad) QuantizeGradients(0);
    idx_[3].Upload(rows, total, stream_);
    FState st;
    std::memset(&st, 0, sizeof(st));
    st.round = 1;
    st.k = k;
    st.kx = k;
    st.num_leaves = 1;
    std::vector<FExp> ex(k);
    for (int e = 0; e < k; ++e) {
      std::memset(&ex[e], 0, sizeof(FExp));
      ex[e].h_buf = 3;
      ex[e].h_start = offsets[e];
      ex[e].h_count = offsets[e + 1] - offsets[e];
      ex[e].forced = -1;
    }
    HIP_CHECK(hipMemcpyAsync(fst_, &st, sizeof(FState), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(fexps_, ex.data(), sizeof(FExp) * k, hipMemcpyHostToDevice, stream_));
    facc_.Zero(stream_);
    FArgs fa = MakeFArgs();
    LaunchFrontierHist(fa, FrontierHistLds(), stream_);
    const int pw = fa.quant && fa.qpack ? 1 : 2;
    std::vector<unsigned long long> acc(static_cast<size_t>(k) * pw * TB_);
    HIP_CHECK(hipMemcpyAsync(acc.data(), facc_.get(), acc.size() * 8, hipMemcpyDeviceToHost, stream_));
    if (fa.quant && levels != nullptr) HIP_CHECK(hipMemcpyAsync(levels, ghq_.get(), sizeof(uint16_t) * N_, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    facc_.Zero(stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    // the kernel's global scale (frontier_kernels.hip GlobalScaleExp)
    constexpr double k62 = 4611686018427387904.0;
    const float sb2 = fa.sum_bound ? bnd[2] : INFINITY, sb3 = fa.sum_bound ? bnd[3] : INFINITY;
    const double ig = fa.quant ? 1.0 : std::ldexp(1.0, -FixedPointExp(k62, N_, bnd[0], sb2));
    const double ih = fa.quant ? 1.0 : std::ldexp(1.0, -FixedPointExp(k62, N_, bnd[1], sb3));
    for (int e = 0; e < k; ++e) {
      for (int b = 0; b < TB_; ++b) {
        const size_t o = (static_cast<size_t>(e) * TB_ + b) * pw;
        long long qg, qh;
        if (pw == 1) {
          const unsigned long long hs = acc[o] & 0xFFFFFFFFull;
          qg = static_cast<long long>(acc[o] - hs) >> 32;
          qh = static_cast<long long>(hs);
        } else {
          qg = static_cast<long long>(acc[o]);
          qh = static_cast<long long>(acc[o + 1]);
        }
        out[(static_cast<size_t>(e) * TB_ + b) * 2] = static_cast<double>(qg) * ig;
        out[(static_cast<size_t>(e) * TB_ + b) * 2 + 1] = static_cast<double>(qh) * ih;
      }
    }
  }

  // k_f_partition of k parents at once (row subsets, split by inner feature feats[e] at
  // threshold bin thr[e] / the categorical bins of catbits[e]): out_rows = the device's
  // children lists (lefts in order, then rights), out_left = left counts; exp_rows / exp_left =
  // the host learner's partition (SerialTreeLearner::Split's predicate, stable).
  void TestFrontierPartition(const int* rows, const int* offsets, int k, const int* feats, const int* thr,
                             const int* dleft, const uint32_t* catbits, int* out_rows, int* out_left, int* exp_rows,
                             int* exp_left) {
    if (!frontier_) Log::Fatal("TestFrontierPartition: the frontier engine is not enabled for this configuration");
    if (k < 1 || k > fkmax_ || 3 * k > fC_) Log::Fatal("TestFrontierPartition: %d parents (1..%d)", k, fkmax_);
    const int total = offsets[k];
    if (total > N_) Log::Fatal("TestFrontierPartition: %d rows over the subsets (at most %d)", total, N_);
    FState st;
    HIP_CHECK(hipMemcpyAsync(&st, fst_, sizeof(FState), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    idx_[0].Upload(rows, total, stream_);
    std::vector<FExp> ex(k);
    std::vector<uint32_t> bits(static_cast<size_t>(fkmax_) * kMaxCatWords, 0u);
    int tiles = 0;
    for (int e = 0; e < k; ++e) {
      const int f = feats[e];
      if (f < 0 || f >= F_) Log::Fatal("TestFrontierPartition: feature %d", f);
      const FeatureInfo& fi = data_->feature(f);
      FExp& x = ex[e];
      std::memset(&x, 0, sizeof(FExp));
      x.parent = e;
      x.left = k + 2 * e;
      x.count = offsets[e + 1] - offsets[e];
      x.start = offsets[e];
      x.src_buf = 0;
      x.dst_buf = 1;
      x.ntiles = std::max(1, DivUp(x.count, fpart_tile_));
      x.tile0 = tiles;
      tiles += x.ntiles;
      x.group = fi.group;
      x.offset = fi.offset;
      x.num_bin = fi.num_bin;
      x.mfb = static_cast<int>(fi.mfb);
      x.default_bin = static_cast<int>(fi.default_bin);
      x.missing = static_cast<int>(fi.missing);
      x.thr = thr[e];
      x.default_left = dleft[e];
      x.is_cat = fi.bin_type == BinType::Categorical ? 1 : 0;
      x.forced = -1;
      x.feature = f;
      for (int w = 0; w < kMaxCatWords; ++w) bits[static_cast<size_t>(e) * kMaxCatWords + w] = catbits[static_cast<size_t>(e) * kMaxCatWords + w];
      // host oracle: the serial learner's predicate, stable
      std::vector<int> l, r;
      const uint32_t nan_bin = static_cast<uint32_t>(fi.num_bin - 1);
      for (int i = 0; i < x.count; ++i) {
        const int row = rows[x.start + i];
        const uint32_t b = data_->FeatureBin(row, f);
        bool go;
        if (x.is_cat) {
          go = b < 32u * kMaxCatWords && ((catbits[static_cast<size_t>(e) * kMaxCatWords + (b >> 5)] >> (b & 31u)) & 1u);
        } else if ((fi.missing == MissingType::Zero && b == fi.default_bin) || (fi.missing == MissingType::NaN && b == nan_bin)) {
          go = dleft[e] != 0;
        } else {
          go = b <= static_cast<uint32_t>(thr[e]);
        }
        (go ? l : r).push_back(row);
      }
      exp_left[e] = static_cast<int>(l.size());
      std::copy(l.begin(), l.end(), exp_rows + x.start);
      std::copy(r.begin(), r.end(), exp_rows + x.start + l.size());
    }
    if (tiles > ftile_cap_) Log::Fatal("TestFrontierPartition: %d tiles (capacity %d)", tiles, ftile_cap_);
    st.round = 1;
    st.k = k;
    st.kx = k;
    st.total_tiles = tiles;
    st.done = 0;
    st.epoch = st.epoch + 1u;
    HIP_CHECK(hipMemcpyAsync(fst_, &st, sizeof(FState), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(fexps_, ex.data(), sizeof(FExp) * k, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(fbits_, bits.data(), sizeof(uint32_t) * bits.size(), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(fbest_, 0, sizeof(SplitInfo) * k, stream_));
    FArgs fa = MakeFArgs();
    LaunchFrontierPartition(fa, fpart_iters_, fpart_grid_, stream_);
    HIP_CHECK(hipMemcpyAsync(out_rows, idx_[1].get(), sizeof(int) * total, hipMemcpyDeviceToHost, stream_));
    std::vector<FNode> nodes(3 * static_cast<size_t>(k));
    HIP_CHECK(hipMemcpyAsync(nodes.data(), fnodes_, sizeof(FNode) * nodes.size(), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int e = 0; e < k; ++e) out_left[e] = nodes[k + 2 * e].count;
    // the look-back's fallback (a predecessor's block not resident: the waiting thread counts the
    // tile itself) must place every row exactly where the published counts do: the same launch
    // again with every look-back self-counted
    st.epoch = st.epoch + 1u;
    HIP_CHECK(hipMemcpyAsync(fst_, &st, sizeof(FState), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(fexps_, ex.data(), sizeof(FExp) * k, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemsetAsync(idx_[1].get(), 0xff, sizeof(int) * total, stream_));
    fa.part_selfcount = 1;
    LaunchFrontierPartition(fa, fpart_iters_, fpart_grid_, stream_);
    std::vector<int> rows2(total);
    HIP_CHECK(hipMemcpyAsync(rows2.data(), idx_[1].get(), sizeof(int) * total, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(nodes.data(), fnodes_, sizeof(FNode) * nodes.size(), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    for (int e = 0; e < k; ++e) {
      if (nodes[k + 2 * e].count != out_left[e]) Log::Fatal("TestFrontierPartition: self-counted look-back, parent %d: left count differs", e);
    }
    if (!std::equal(rows2.begin(), rows2.end(), out_rows)) Log::Fatal("TestFrontierPartition: self-counted look-back places rows differently");
  }

  void TestHistogram(const float* g, const float* h, const int* rows, int n, double* out) {
    K_ = 1;
    gh_.Resize(static_cast<size_t>(N_));
    DeviceSetGradients(g, h, 1);
    if (rows) idx_[2].Upload(rows, n, stream_);
    Ctl* hc = pin_ctl_.Get(1);
    std::memset(hc, 0, sizeof(Ctl));
    hc->num_leaves = 1;
    hc->larger = -1;
    LeafRange* hr = pin_range_.Get(L_);
    hr[0].buf = rows ? 2 : -1;
    hr[0].start = 0;
    hr[0].count = rows ? n : N_;
    hr[0].pad = 0;
    HIP_CHECK(hipMemcpyAsync(ctl_.get(), hc, sizeof(Ctl), hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(range_.get(), hr, sizeof(LeafRange), hipMemcpyHostToDevice, stream_));
    float mg = 0.f, mh = 0.f;
    for (int i = 0; i < (rows ? n : N_); ++i) {
      const int r = rows ? rows[i] : i;
      mg = std::max(mg, std::fabs(g[r]));
      mh = std::max(mh, std::fabs(h[r]));
    }
    unsigned* hm = pin_max_.Get(2);
    std::memcpy(&hm[0], &mg, 4);
    std::memcpy(&hm[1], &mh, 4);
    HIP_CHECK(hipMemcpyAsync(ghmax_.get(), hm, 8, hipMemcpyHostToDevice, stream_));
    staging_.Zero(stream_);
    const Args args = MakeArgs();
    LaunchHist(args, /*collective=*/false);
    LaunchHistReduce(args);
    staging_.Download(out, 2 * static_cast<size_t>(TB_), stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    staging_.Zero(stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

 private:
  // Fused-partition tile: 8 rows per thread from 8M rows per GPU up, 4 below (A/B:
  // 10M 227 it/s at 8 vs 225 at 4 vs 214 at 16; 5M 3.42 ms/iter at 4 vs 3.48 at 8;
  // 2.5M 2.83 vs 2.92; 1.25M 390 it/s at 4 vs 368 at 8 vs 330 at 16).
  // LGAP_KERNEL=part_iters=4 / 8 / 16 overrides.
  int PartIters() const {
    if (const char* e = KernelOverride("part_iters")) {
      const int v = std::atoi(e);
      if (v == 4 || v == 8 || v == 16) return v;
    }
    // (frontier A/B: 4096-row tiles at 10M, 1024-row tiles at 1.25M; the sequential chain's
    // partition uses the same rows per thread)
    return N_ >= 8000000 ? 16 : 4;
  }

  typedef void (*PartitionFn)(Args);
  PartitionFn PartitionKernel() const {
    return part_iters_ == 16 ? k_partition<16> : (part_iters_ == 8 ? k_partition<8> : k_partition<4>);
  }

  int HistMinRows() const {
    if (config_->device_hist_min_rows > 0) return config_->device_hist_min_rows;
    return kHistMinRows;
  }

  int RootBlocks() const { return std::max(1, std::min(DivUp(N_, kRootThreads), 4 * num_cu_)); }

  int HistBlocks() const {
    // one block per CU: A/B on MI355X (10M rows) 256 blocks 4.68-4.74 ms/iter vs 512: 4.85,
    // 384: 4.85, 320: 4.91, 768: 4.93 (fewer slab rows for the scan to fold; an uneven
    // multiple of the CU count leaves a tail); 1.25M rows: flat within 0.6%
    // Wide data (many LDS feature tiles): the grid is row blocks x tiles, so fewer row blocks
    // still fill the chip while the slab rows the scan folds (each one 8 B x all bins) shrink:
    // LambdaRank 1M x 300 (11 tiles) 17.7 -> 16.4 ms/iter at 46 row blocks instead of 256.
    // (multi-tile: as many row blocks per tile as the CUs hold at once over all tiles -- two
    // blocks per CU when the tile's LDS allows, one for 150 KB tiles. Every row block flushes
    // its whole tile with global atomics: LambdaRank 2M x 300 moved 130 MB of atomics per
    // histogram launch with 102 row blocks x 5 tiles of 128 KB, twice the resident blocks)
    const int bpc = std::max(1, std::min(2, static_cast<int>((160 * 1024) / std::max<size_t>(hist_lds_bytes_, 1))));
    const int want = config_->device_hist_blocks > 0 ? config_->device_hist_blocks
                                                     : std::min(num_cu_, std::max(1, bpc * num_cu_ / std::max(1, num_tiles_)));
    // partial-histogram slab: one row of 2 * TB accumulators per block, capped at 4 GiB
    const size_t row_bytes = 2 * static_cast<size_t>(TB_) * (use_dp_ ? 8 : 4);
    const int mem_cap = static_cast<int>(std::max<size_t>(1, (size_t(4) << 30) / std::max<size_t>(row_bytes, 1)));
    return std::max(1, std::min({want, DivUp(N_, HistMinRows()), mem_cap}));
  }

  // Frontier histogram grid: every working block on its own CU (k_f_hist caps the chunk
  // count at the grid), 7/8 of the CUs: A/B at 10M rows 224 blocks 363 it/s, 192: 361,
  // 256: 355, 384: 346, 512: 327 (the per-block flush of a full LDS tile is the fixed cost)
  int FrontierHistBlocks() const {
    if (config_->device_hist_blocks > 0) return HistBlocks();
    // several LDS tiles: the grid is row blocks x tiles, ~2 blocks per CU in all
    if (num_tiles_ > 1) return HistBlocks();
    return std::max(1, HistBlocks() * 7 / 8);
  }

  void LaunchHist(const Args& a, bool collective = true) {
    const dim3 hgrid(HistBlocks(), num_tiles_);
    if (use_dp_) {
      if (width_ == 1) k_hist<1, 1><<<hgrid, kHistThreads, hist_lds_bytes_, stream_>>>(a);
      else k_hist<2, 1><<<hgrid, kHistThreads, hist_lds_bytes_, stream_>>>(a);
    } else {
      if (width_ == 1) k_hist<1, 0><<<hgrid, kHistThreads, hist_lds_bytes_, stream_>>>(a);
      else k_hist<2, 0><<<hgrid, kHistThreads, hist_lds_bytes_, stream_>>>(a);
    }
    HIP_CHECK(hipGetLastError());
    if (owner_scan_ && data_parallel_ && collective) {
      // owner reduce-scatter of the smaller child's histogram (xGMI: inside k_hist_owner)
      const int ogrid = DivUp(static_cast<long long>(P_) * 2 * bbin_, 64);
      if (use_dp_) {
        k_hist_owner<double><<<ogrid, 1024, 0, stream_>>>(a, HistBlocks(), reinterpret_cast<double*>(stage_.get()));
      } else {
        k_hist_owner<float><<<ogrid, 1024, 0, stream_>>>(a, HistBlocks(), reinterpret_cast<float*>(stage_.get()));
      }
      HIP_CHECK(hipGetLastError());
      ReduceScatterSum(stage_.get(), rx_.get(), 2 * static_cast<size_t>(bbin_), use_dp_, stream_);
    }
  }

  // rank-local fp64 histogram into `staging` (kernel test hooks, host split policies)
  void LaunchHistReduce(const Args& a) {
    const int rgrid = DivUp(2 * static_cast<long long>(TB_), 64);
    if (use_dp_) k_hist_reduce<double, double><<<rgrid, 1024, 0, stream_>>>(a, HistBlocks(), staging_.get());
    else k_hist_reduce<float, double><<<rgrid, 1024, 0, stream_>>>(a, HistBlocks(), staging_.get());
    HIP_CHECK(hipGetLastError());
  }

  void LaunchScan(const Args& a) {
    if (voting_) {
      LaunchVoting(a);
      return;
    }
    LaunchReduceScan(a, Fmax_);
    HIP_CHECK(hipGetLastError());
    // complete the candidate table (xGMI: inside k_reduce_scan)
    if (owner_scan_ && P_ > 1) AllGatherInPlace(cand_.get(), cand_stride_, stream_);
  }

  void LaunchReduceScan(const Args& a0, int grid) {
    const int hg = HistBlocks();
    Args a = a0;
    // slab rows folded by fold_chunks_ blocks per feature (single GPU / feature parallel /
    // voting local pass); the exchange transport counts its blocks, so it keeps one per feature
    if (fold_chunks_ > 1 && a.scan_src == 0 && !scan_global_ && a.fold_cnt) {
      a.fold_chunks = fold_chunks_;
      a.fold_feats = grid;
      grid = (grid * fold_chunks_ + 7) & ~7;
    }
    if (use_dp_) {
      if (scan_global_) k_reduce_scan<double, true><<<grid, kScanThreads, 0, stream_>>>(a, hg);
      else k_reduce_scan<double, false><<<grid, kScanThreads, scan_lds_bytes_, stream_>>>(a, hg);
    } else {
      if (scan_global_) k_reduce_scan<float, true><<<grid, kScanThreads, 0, stream_>>>(a, hg);
      else k_reduce_scan<float, false><<<grid, kScanThreads, scan_lds_bytes_, stream_>>>(a, hg);
    }
    HIP_CHECK(hipGetLastError());
  }

  // The voting learner's per-split chain after k_hist (see k_vote_local).
  void LaunchVoting(const Args& a) {
    Args al = a;  // local pass: every feature, local sums / counts, divided thresholds, local table
    al.vote = 1;
    al.cand = cand_.get();
    al.Fmax = F_;
    al.cand_rows = 1;
    al.cand_key_bytes = cand_key_bytes_;
    al.cand_stride = cand_stride_;
    al.rank = 0;
    al.P = 1;
    al.own_feat = nullptr;
    al.sp.min_data_in_leaf = config_->min_data_in_leaf / P_;  // integer division (reference :61-63)
    al.sp.min_sum_hessian_in_leaf = config_->min_sum_hessian_in_leaf / P_;
    LaunchReduceScan(al, F_);
    HIP_CHECK(hipGetLastError());
    k_vote_local<<<1, kVoteThreads, vote_local_lds_, stream_>>>(a);
    HIP_CHECK(hipGetLastError());
    AllGatherInPlace(vrec_.get(), 2 * static_cast<size_t>(topk_) * sizeof(VoteRec), stream_);
    if (use_dp_) k_vote_pack<double><<<2 * topk_, kVoteThreads, vote_pack_lds_, stream_>>>(a);
    else k_vote_pack<float><<<2 * topk_, kVoteThreads, vote_pack_lds_, stream_>>>(a);
    HIP_CHECK(hipGetLastError());
    if (use_dp_) AllreduceSumF64(reinterpret_cast<double*>(vhist_.get()), static_cast<size_t>(vcap_), stream_);
    else AllreduceSumF32(reinterpret_cast<float*>(vhist_.get()), static_cast<size_t>(vcap_), stream_);
    const size_t vlds = scan_global_ ? 0 : vote_scan_lds_;
    if (use_dp_) {
      if (scan_global_) k_vote_scan<double, true><<<topk_, 128, 0, stream_>>>(a);
      else k_vote_scan<double, false><<<topk_, 128, vlds, stream_>>>(a);
    } else {
      if (scan_global_) k_vote_scan<float, true><<<topk_, 128, 0, stream_>>>(a);
      else k_vote_scan<float, false><<<topk_, 128, vlds, stream_>>>(a);
    }
    HIP_CHECK(hipGetLastError());
  }

  // dword stride of a packed-row buffer: the training rows may be padded (RowAlign), validation
  // rows keep the dataset's stride
  int StrideOf(const uint32_t* rb) const { return rb == rowbins_.get() ? tstride_dw_ : stride_dw_; }

  // bank-interleaved LDS histograms (frontier MODE 0 / 2; LGAP_KERNEL=hist_il=0: packed bins)
  // (1: the root round's contiguous rows only, 2: every round; default 1 from 4M rows: A/B one
  // box, 10M 2.864 / 2.885 / 2.875 ms for 1 / 2 / 0, 1.25M 1.358 / 1.375 / 1.341)
  int HistInterleave() const {
    const char* e = KernelOverride("hist_il");
    return e != nullptr ? std::atoi(e) : (N_ >= (4 << 20) ? 1 : 0);
  }

  // Wide rows in several LDS tiles: tiles cut at multiples of RowAlign() dwords and the training
  // rows padded to a multiple of it, so every tile's slice of a row is whole aligned 32 / 64 /
  // 128-byte sectors instead of straddling them (LGAP_ROW_ALIGN_DW: 0 off, 8, 16 or 32)
  int RowAlign() const {
    // (default 16: A/B on one box, GOSS 5M x 500 quantized 10.95 -> 10.40 ms/iter, LambdaRank
    // 3M x 300 9.52 -> 9.30)
    return 16;
  }

  void PadTrainingRows(int align) {
    const int pad = DivUp(stride_dw_, align) * align;
    if (pad == stride_dw_ || N_ <= 0) return;
    uint32_t* p = nullptr;
    const size_t n = static_cast<size_t>(N_) * pad;
    HIP_CHECK(hipMalloc(&p, n * sizeof(uint32_t)));
    HIP_CHECK(hipMemsetAsync(p, 0, n * sizeof(uint32_t), stream_));
    HIP_CHECK(hipMemcpy2DAsync(p, pad * sizeof(uint32_t), rowbins_.get(), stride_dw_ * sizeof(uint32_t),
                               stride_dw_ * sizeof(uint32_t), N_, hipMemcpyDeviceToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    rowbins_.Adopt(p, n);
    tstride_dw_ = pad;
    Log::Debug("HIP learner: training rows padded from %d to %d dwords (tiles aligned to %d)", stride_dw_, pad, align);
  }

  static double XTimeoutSeconds() {
    static const double t = [] {
      const char* e = std::getenv("LGAP_XGMI_TIMEOUT_S");
      return e != nullptr && *e ? std::max(0.1, std::atof(e)) : 60.0;
    }();
    return t;
  }

  void UploadData() {
    // packed rows
    const size_t rb = static_cast<size_t>(N_) * stride_dw_;
    // rows binned on the device (bin_kernels.hip) are adopted instead of uploaded again
    void* adopted = rb > 0 ? TakeDeviceRows(data_, rb * sizeof(uint32_t)) : nullptr;
    if (adopted != nullptr) {
      rowbins_.Adopt(static_cast<uint32_t*>(adopted), rb);
      Log::Debug("HIP learner: adopted the device-binned rows (%zu bytes)", rb * sizeof(uint32_t));
    } else {
      rowbins_.Resize(std::max<size_t>(rb, 1));
      std::vector<uint8_t> full;  // a sparse-stored (host-constructed) set becomes full rows
      rowbins_.Upload(reinterpret_cast<const uint32_t*>(data_->RowsForDevice(&full)), rb, stream_);
      if (!full.empty()) HIP_CHECK(hipStreamSynchronize(stream_));
    }
    // group-major copy, transposed on the device from the packed rows
    const size_t cb = static_cast<size_t>(G_) * N_ * width_;
    colbins_.Resize(std::max<size_t>(cb, 1));
    if (cb > 0) {
      const int grid = std::max(1, std::min(DivUp(static_cast<long long>(G_) * N_, 256), 65536));
      if (width_ == 1) k_transpose_bins<uint8_t><<<grid, 256, 0, stream_>>>(rowbins_.get(), stride_dw_, N_, G_, colbins_.get());
      else k_transpose_bins<uint16_t><<<grid, 256, 0, stream_>>>(rowbins_.get(), stride_dw_, N_, G_, colbins_.get());
      HIP_CHECK(hipGetLastError());
    }
    // features / groups
    std::vector<DevFeature> feats(std::max(F_, 1));
    max_cat_bin_ = 1;
    has_cat_ = false;
    for (int f = 0; f < F_; ++f) {
      const FeatureInfo& fi = data_->feature(f);
      DevFeature& d = feats[f];
      std::memset(&d, 0, sizeof(d));
      d.group = fi.group;
      d.offset = fi.offset;
      d.num_bin = fi.num_bin;
      d.mfb = static_cast<int>(fi.mfb);
      d.default_bin = static_cast<int>(fi.default_bin);
      d.hist_offset = fi.hist_offset;
      d.missing = static_cast<int8_t>(fi.missing);
      d.bin_type = static_cast<int8_t>(fi.bin_type);
      d.monotone = fi.monotone;
      d.penalty = fi.penalty;
      if (fi.bin_type == BinType::Categorical) {
        has_cat_ = true;
        max_cat_bin_ = std::max(max_cat_bin_, fi.num_bin);
      }
    }
    h_feats_ = feats;
    max_bin_ = 2;
    for (int f = 0; f < F_; ++f) max_bin_ = std::max(max_bin_, data_->feature(f).num_bin);
    // k_reduce_scan: two full histograms + 16x64 partials + 2 categorical sort arrays (bin, ctr)
    cat_p2_ = 1;
    if (has_cat_) {
      while (cat_p2_ < max_cat_bin_) cat_p2_ <<= 1;
    }
    scan_lds_bytes_ = static_cast<size_t>(max_bin_) * 4 * sizeof(double) + 16 * 64 * sizeof(double) +
                      static_cast<size_t>(cat_p2_) * 2 * (sizeof(int) + sizeof(double));
    // wider than the LDS budget: the scan kernels work in global scratch (one slice per block)
    scan_global_ = scan_lds_bytes_ > 150 * 1024 || KernelOverride("scan_global") != nullptr;
    scan_scratch_stride_ = Round256(scan_lds_bytes_);
    if (scan_global_) {
      scan_scratch_.Resize(scan_scratch_stride_ * static_cast<size_t>(std::max(F_, 1)));
      Log::Debug("HIP split scan: %d-bin features use %zu bytes of global scratch per block", max_bin_,
                 scan_scratch_stride_);
    } else if (scan_lds_bytes_ > 64 * 1024) {
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_reduce_scan<float, false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(scan_lds_bytes_)));
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_reduce_scan<double, false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(scan_lds_bytes_)));
    }
    std::vector<int> gs(std::max(G_, 1));
    for (int g = 0; g < G_; ++g) gs[g] = data_->group(g).hist_start;
    h_gstart_ = gs;
    BuildTiles();
    BuildNibbleRows();
    // labels / weights for the device objectives are uploaded lazily
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  void BuildTiles() {
    row_align_ = RowAlign();
    const int env_kb = [] {
      const char* e = KernelOverride("hist_lds_kb");  // A/B / test knob: LDS tile budget
      return e ? std::max(16, std::min(150, std::atoi(e))) : 0;
    }();
    big_tiles_ = false;
    PlanTiles(env_kb > 0 ? env_kb * 1024 : kHistLdsBytes);
    // Wide rows split into narrow tiles (< 16 dwords = 64 B of a row per pass) re-gather a
    // partial cache line of every row once per tile: serial training then plans tiles for one
    // 150 KB block per CU (1024 threads in the frontier). A/B, LambdaRank 5M x 300 (255 bins,
    // 11 tiles of 7 dwords at 56 KB): 79.8 -> 92.2 it/s; GOSS 12.5M x 500 (63 bins, 5 tiles
    // of 28 dwords) keeps 56 KB (150 KB measured 76.8 -> 61.8).
    if (env_kb == 0 && mode_ == DevParallel::kSerial && num_tiles_ > 1 && min_tile_dw_ < 16) {
      big_tiles_ = true;
      PlanTiles(150 * 1024);
    }
    if (num_tiles_ > 1 && row_align_ > 0) PadTrainingRows(row_align_);
    // single-tile rows padded to whole 32-byte sectors from 4M rows (LGAP_ROW_PAD_SINGLE=0/8/16):
    // 28-byte rows -> 32 bytes, so a gathered row never straddles two sectors (A/B 10M 2.838 vs
    // 2.874 ms/iter; 1.25M flat)
    if (num_tiles_ == 1) {
      if (N_ >= (4 << 20) && stride_dw_ > 4 && stride_dw_ < 8) PadTrainingRows(8);
    }
  }

  // 4-bit rows for the frontier histograms and the training score update: 8-bit data whose
  // every group has <= 16 bins (max_bin <= 15, no wide bundles) in one LDS tile. The 8-bit
  // rows stay for everything else (validation sets, the sequential chain, device binning).
  void BuildNibbleRows() {
    nib_ = false;
    const char* e = KernelOverride("nibble");  // A/B knob: 0 keeps 8-bit rows
    if (e != nullptr && e[0] == '0') return;
    if (width_ != 1 || num_tiles_ != 1 || G_ <= 0 || N_ <= 0 || h_tiles_.empty() || h_tiles_[0].direct) return;
    for (int g = 0; g < G_; ++g) {
      if (data_->group(g).num_bin > 16) return;
    }
    stride4_dw_ = DivUp(G_, 8);
    rowbins4_.Resize(static_cast<size_t>(N_) * stride4_dw_);
    LaunchPackNibbles(rowbins_.get(), tstride_dw_, N_, G_, rowbins4_.get(), stride4_dw_, stream_);
    HistTile t = h_tiles_[0];
    t.d0 = 0;
    t.d1 = stride4_dw_;
    ntile_.Resize(1);
    ntile_.Upload(&t, 1, stream_);
    HIP_CHECK(hipStreamSynchronize(stream_));
    nib_ = true;
    Log::Debug("HIP learner: 4-bit rows (%d dwords per row instead of %d)", stride4_dw_, stride_dw_);
  }

  void PlanTiles(int lds_budget) {
    const int per = 4 / width_;
    const size_t acc = use_dp_ ? 16 : 8;  // LDS bytes per bin (grad + hess)
    const int max_bins = static_cast<int>(lds_budget / acc) - 64;
    const int max_dw = kHistThreads / 2;
    std::vector<HistTile> tiles;
    hist_lds_bytes_ = 16;
    hist_lds_plain_ = 16;
    int d = 0;
    const int nd = DivUp(G_, per);
    while (d < nd) {
      HistTile t;
      t.d0 = d;
      t.g0 = d * per;
      t.bin0 = data_->group(t.g0).hist_start;
      int bins = 0;
      int e = d;
      while (e < nd && e - d < max_dw) {
        int wb = 0;
        for (int g = e * per; g < std::min(G_, (e + 1) * per); ++g) wb += data_->group(g).num_bin;
        if (bins + wb > max_bins && e > d) break;
        bins += wb;
        ++e;
      }
      if (row_align_ > 0 && e < nd && e - d >= row_align_ && (e - d) % row_align_ != 0) {
        // cut at the alignment (the rows are padded to it when there are several tiles)
        const int ea = d + (e - d) / row_align_ * row_align_;
        for (int x = ea; x < e; ++x) {
          for (int g = x * per; g < std::min(G_, (x + 1) * per); ++g) bins -= data_->group(g).num_bin;
        }
        e = ea;
      }
      t.d1 = e;
      t.g1 = std::min(G_, e * per);
      t.nbins = bins;
      // a single dword of huge bundles that cannot fit: accumulate straight into global memory
      t.direct = bins > max_bins ? 1 : 0;
      // bank-interleaved LDS slots (k_f_hist il): (largest group's bins) x (groups rounded up to
      // 16), when that stays within 1.25x of the packed tile and the 150 KB block budget
      t.pad = 0;
      if (!t.direct && HistInterleave() > 0) {
        int maxb = 0;
        for (int g = t.g0; g < t.g1; ++g) maxb = std::max(maxb, data_->group(g).num_bin);
        // (plus the packed image the interleaved slots are transposed into before the flush)
        const size_t il = static_cast<size_t>(maxb) * ((t.g1 - t.g0 + 15) & ~15) * 8;
        const size_t need = il + sizeof(int) * ((t.g1 - t.g0 + 1) & ~1) + static_cast<size_t>(bins) * 8 + 16;
        if (il <= static_cast<size_t>(bins) * 8 * 5 / 4 + 4096 && need <= 150 * 1024) {
          t.pad = maxb;
          hist_lds_bytes_ = std::max(hist_lds_bytes_, need);
        }
      }
      tiles.push_back(t);
      const size_t plain = t.direct ? sizeof(int) * (t.g1 - t.g0) + 16
                                    : static_cast<size_t>(bins) * acc + sizeof(int) * (t.g1 - t.g0) + 16;
      hist_lds_bytes_ = std::max(hist_lds_bytes_, plain);
      hist_lds_plain_ = std::max(hist_lds_plain_, plain);
      d = e;
    }
    if (hist_lds_bytes_ > 64 * 1024) {
      const void* fn = use_dp_ ? (width_ == 1 ? reinterpret_cast<const void*>(k_hist<1, 1>)
                                              : reinterpret_cast<const void*>(k_hist<2, 1>))
                               : (width_ == 1 ? reinterpret_cast<const void*>(k_hist<1, 0>)
                                              : reinterpret_cast<const void*>(k_hist<2, 0>));
      HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(hist_lds_bytes_)));
    }
    num_tiles_ = static_cast<int>(tiles.size());
    nib_ = false;
    min_tile_dw_ = 1 << 30;
    for (size_t i = 0; i + 1 < tiles.size(); ++i) min_tile_dw_ = std::min(min_tile_dw_, tiles[i].d1 - tiles[i].d0);
    h_tiles_ = tiles;
  }

  void AllocState() {
    const size_t L = L_;
    part_iters_ = PartIters();
    // tile bookkeeping sized for the smaller of the fused (256 * part_iters_) and
    // two-kernel (kTileRows) tiles
    max_tiles_ = std::max(1, DivUp(N_, kPartThreads * std::min(part_iters_, kPartIters)));
    fused_blocks_ = 0;
    // optionally the histogram rides in the partition kernel (one LDS tile, packed
    // fixed point). Measured slower than k_hist (whole-row threads, half the lanes
    // idle on the larger child, 2 blocks/CU): off by default, kept for A/B runs.
    if (config_->device_fused_partition) {
      // k_partition waits on other blocks' published counts: every block must be resident at once
      int per_cu = 0;
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, PartitionKernel(), kPartThreads, 0));
      // the occupancy API can overstate residency by one block per CU (MI355X_MICROARCH.md): keep a margin
      per_cu = std::max(1, per_cu - 1);
      fused_blocks_ = std::min({max_tiles_ + 1, 4 * num_cu_, per_cu * num_cu_});
    }
    use_bynode_ = config_->feature_fraction_bynode < 1.0;
    // every small per-tree structure + the static feature metadata in one allocation
    ArenaLayout lay;
    const size_t o_tp = lay.Add<TreeParams>(1), o_ctl = lay.Add<Ctl>(2), o_range = lay.Add<LeafRange>(L),
                 o_lsum = lay.Add<double2>(L), o_lout = lay.Add<double>(L), o_gcount = lay.Add<int>(L),
                 o_depth = lay.Add<int>(L), o_slot = lay.Add<int>(L), o_bounds = lay.Add<LeafBounds>(L),
                 o_best = lay.Add<SplitInfo>(L), o_rec = lay.Add<SplitRec>(L), o_ghmax = lay.Add<unsigned>(4),
                 o_spl = lay.Add<uint8_t>(L * F_), o_tcnt = lay.Add<int>(max_tiles_), o_toff = lay.Add<int>(max_tiles_),
                 o_used = lay.Add<uint8_t>(std::max(F_, 1)), o_byn = lay.Add<uint8_t>(use_bynode_ ? 2 * L * F_ : 1),
                 o_rng = lay.Add<unsigned>(std::max(F_, 1)), o_feat = lay.Add<DevFeature>(h_feats_.size()),
                 o_gst = lay.Add<int>(h_gstart_.size()), o_tiles = lay.Add<HistTile>(h_tiles_.size()),
                 o_icf = lay.Add<unsigned long long>(std::max(F_, 1)), o_icl = lay.Add<unsigned long long>(L),
                 o_qmax = lay.Add<unsigned>(2), o_tsum = lay.Add<double2>(L),
                 o_rpart = lay.Add<double>(6 * static_cast<size_t>(std::max(1, 4 * num_cu_))),
                 o_bar = lay.Add<unsigned>(4), o_lkey = lay.Add<SplitKey>(L),
                 o_tpub = lay.Add<unsigned long long>(max_tiles_), o_xcnt = lay.Add<unsigned>(4),
                 o_own = lay.Add<int>(Fmax_), o_binlo = lay.Add<int>(P_ + 1);
    arena_.Resize(std::max<size_t>(lay.bytes(), size_t(2) << 20));
    char* base = arena_.get();
    tparams_.Attach(reinterpret_cast<TreeParams*>(base + o_tp), 1);
    ctl_.Attach(reinterpret_cast<Ctl*>(base + o_ctl), 2);
    range_.Attach(reinterpret_cast<LeafRange*>(base + o_range), L);
    lsum_.Attach(reinterpret_cast<double2*>(base + o_lsum), L);
    lout_.Attach(reinterpret_cast<double*>(base + o_lout), L);
    gcount_.Attach(reinterpret_cast<int*>(base + o_gcount), L);
    depth_.Attach(reinterpret_cast<int*>(base + o_depth), L);
    slot_.Attach(reinterpret_cast<int*>(base + o_slot), L);
    bounds_.Attach(reinterpret_cast<LeafBounds*>(base + o_bounds), L);
    best_.Attach(reinterpret_cast<SplitInfo*>(base + o_best), L);
    rec_.Attach(reinterpret_cast<SplitRec*>(base + o_rec), L);
    ghmax_.Attach(reinterpret_cast<unsigned*>(base + o_ghmax), 4);
    splittable_.Attach(reinterpret_cast<uint8_t*>(base + o_spl), L * F_);
    tile_cnt_.Attach(reinterpret_cast<int*>(base + o_tcnt), max_tiles_);
    tile_off_.Attach(reinterpret_cast<int*>(base + o_toff), max_tiles_);
    used_bytree_.Attach(reinterpret_cast<uint8_t*>(base + o_used), std::max(F_, 1));
    bynode_.Attach(reinterpret_cast<uint8_t*>(base + o_byn), use_bynode_ ? 2 * L * F_ : 1);
    rng_.Attach(reinterpret_cast<unsigned*>(base + o_rng), std::max(F_, 1));
    feat_.Attach(reinterpret_cast<DevFeature*>(base + o_feat), h_feats_.size());
    gstart_.Attach(reinterpret_cast<int*>(base + o_gst), h_gstart_.size());
    tiles_.Attach(reinterpret_cast<HistTile*>(base + o_tiles), h_tiles_.size());
    ic_feat_.Attach(reinterpret_cast<unsigned long long*>(base + o_icf), std::max(F_, 1));
    ic_leaf_.Attach(reinterpret_cast<unsigned long long*>(base + o_icl), L);
    qmax_.Attach(reinterpret_cast<unsigned*>(base + o_qmax), 2);
    true_sums_.Attach(reinterpret_cast<double2*>(base + o_tsum), L);
    root_part_.Attach(reinterpret_cast<double*>(base + o_rpart), 6 * static_cast<size_t>(std::max(1, 4 * num_cu_)));
    bar_.Attach(reinterpret_cast<unsigned*>(base + o_bar), 4);
    leaf_key_.Attach(reinterpret_cast<SplitKey*>(base + o_lkey), L);
    tile_pub_.Attach(reinterpret_cast<unsigned long long*>(base + o_tpub), max_tiles_);
    xcnt_.Attach(reinterpret_cast<unsigned*>(base + o_xcnt), 4);
    own_feat_.Attach(reinterpret_cast<int*>(base + o_own), Fmax_);
    bin_lo_.Attach(reinterpret_cast<int*>(base + o_binlo), P_ + 1);
    arena_.Zero(stream_);
    own_feat_.Upload(h_own_feat_, stream_);
    bin_lo_.Upload(h_bin_lo_, stream_);
    // candidate table: P blocks (a local copy; the xGMI transport uses the table inside
    // the exchange buffer that the peers push into)
    cand_.Resize(static_cast<size_t>(P_) * cand_stride_);
    cand_.Zero(stream_);
    if (voting_) {
      const size_t es = use_dp_ ? 8 : 4;
      vcand_.Resize(static_cast<size_t>(vcand_stride_));
      vcand_.Zero(stream_);
      vrec_.Resize(static_cast<size_t>(P_) * 2 * topk_);
      vhist_.Resize(static_cast<size_t>(vcap_) * es);
      vhist_.Zero(stream_);
      elect_.Resize(2 * static_cast<size_t>(topk_ + 2));
      elect_.Zero(stream_);
      hsum_part_.Resize(static_cast<size_t>(std::max(1, HistBlocks())));
      lsum_loc_.Resize(L);
      const int R = P_ * topk_;
      vote_local_lds_ = static_cast<size_t>(F_) * (sizeof(double) + sizeof(int));
      vote_pack_lds_ = static_cast<size_t>(R) * (sizeof(double) + 3 * sizeof(int)) + sizeof(int) * (kVoteThreads / 64) +
                       2 * sizeof(int) * topk_;
      vote_scan_lds_ = static_cast<size_t>(max_bin_) * 4 * sizeof(double) +
                       static_cast<size_t>(cat_p2_) * 2 * (sizeof(int) + sizeof(double));
      auto big = [](const void* fn, size_t bytes) {
        if (bytes > 64 * 1024) {
          HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes)));
        }
      };
      if (vote_local_lds_ > 150 * 1024 || vote_pack_lds_ > 150 * 1024) {
        Log::Fatal("HIP voting learner: %d features x top_k %d x %d ranks exceed the LDS budget; use device_type=cpu",
                   F_, topk_, P_);
      }
      big(reinterpret_cast<const void*>(k_vote_local), vote_local_lds_);
      big(reinterpret_cast<const void*>(k_vote_pack<float>), vote_pack_lds_);
      big(reinterpret_cast<const void*>(k_vote_pack<double>), vote_pack_lds_);
      if (!scan_global_) {
        big(reinterpret_cast<const void*>(k_vote_scan<float, false>), vote_scan_lds_);
        big(reinterpret_cast<const void*>(k_vote_scan<double, false>), vote_scan_lds_);
      }
    }
    rx_.Resize(std::max<size_t>(1, 2 * static_cast<size_t>(bbin_) * (use_dp_ ? 8 : 4)));
    stage_.Resize(owner_scan_ ? static_cast<size_t>(P_) * 2 * bbin_ * (use_dp_ ? 8 : 4) : 1);
    use_ic_ = !config_->interaction_constraints_vector.empty();
    if (use_ic_) {
      const auto& sets = config_->interaction_constraints_vector;
      // the frontier holds up to 256 sets (words of 64); the sequential chain's one word, 64
      // (TreeLearner::Create routes more than 64 sets to the frontier or the host policy)
      if (sets.size() > 64 * static_cast<size_t>(kFrontierIcWords)) {
        Log::Fatal("The HIP learner holds at most %d interaction constraint sets", 64 * kFrontierIcWords);
      }
      ic_words_ = static_cast<int>((sets.size() + 63) / 64);
      std::vector<unsigned long long> m(std::max(F_, 1), 0ull);
      std::vector<unsigned long long> mw(static_cast<size_t>(std::max(F_, 1)) * ic_words_, 0ull);
      for (int f = 0; f < F_; ++f) {
        const int real = data_->feature(f).real_index;
        for (size_t k = 0; k < sets.size(); ++k) {
          if (std::find(sets[k].begin(), sets[k].end(), real) == sets[k].end()) continue;
          if (k < 64) m[f] |= 1ull << k;
          mw[static_cast<size_t>(f) * ic_words_ + k / 64] |= 1ull << (k % 64);
        }
      }
      ic_feat_.Upload(m, stream_);
      fic_feat_.Upload(mw, stream_);
    }
    feat_.Upload(h_feats_, stream_);
    gstart_.Upload(h_gstart_, stream_);
    tiles_.Upload(h_tiles_, stream_);
    // extra-trees streams: Random(extra_seed + f) per feature, persistent across trees
    std::vector<unsigned> rs(std::max(F_, 1));
    for (int f = 0; f < F_; ++f) rs[f] = static_cast<unsigned>(config_->extra_seed + f);
    rng_.Upload(rs, stream_);
    // large buffers keep their own allocations
    slots_.Resize(L * 2 * static_cast<size_t>(TB_));
    staging_.Resize(2 * static_cast<size_t>(TB_));
    staging_.Zero(stream_);
    staging_f_.Resize(2 * static_cast<size_t>(TB_));
    hist_slab_.Resize(static_cast<size_t>(HistBlocks()) * 2 * TB_ * (use_dp_ ? 8 : 4));
    // split slab fold (LGAP_SCAN_CHUNKS=C: C blocks per feature, in-launch combine). Off: A/B on
    // MI355X, 10M rows C=8 222 it/s, C=4 229, C=1 232; 1.25M C=8 348, C=1 386 -- the release /
    // ticket / acquire hand-off costs more than the shorter fold saves
    fold_chunks_ = 1;
#if LGAP_SCAN_FOLD == 2
    fold_chunks_ = 1;
#endif
    if (fold_chunks_ > 1) {
      fold_part_.Resize(static_cast<size_t>(fold_chunks_) * 2 * TB_);
      fold_cnt_.Resize(std::max(F_, 1));
      fold_cnt_.Zero(stream_);
    }
    // all three index buffers hold N rows up front: a captured graph keeps their
    // addresses, so a later bag (host upload or device draw) must not reallocate
    for (int i = 0; i < 3; ++i) idx_[i].Resize(std::max(N_, 1));
    if (bag_cnt_ == 0) bag_cnt_ = N_;
    AllocFrontier();
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  // Args of a launch in split round `it`: the partition of round it reads control
  // buffer it % 2 and writes the other; the histogram / scan after it read the new one.
  Args MakeArgs(int it = 0) const {
    Args a;
    std::memset(&a, 0, sizeof(a));
    a.rowbins = rowbins_.get();
    a.colbins = colbins_.get();
    a.gh = gh_.get();
    for (int i = 0; i < 5; ++i) a.idx[i] = idx_[i].get();
    a.N = N_;
    a.stride_dw = tstride_dw_;
    a.width = width_;
    a.num_groups = G_;
    a.TB = TB_;
    a.F = F_;
    a.L = L_;
    a.max_tiles = max_tiles_;
    a.gstart = gstart_.get();
    a.feat = feat_.get();
    a.tiles = tiles_.get();
    a.used_bytree = used_bytree_.get();
    a.bynode = use_bynode_ ? bynode_.get() : nullptr;
    a.tp = tparams_.get();
    a.ctl = ctl_.get() + (it & 1);
    a.ctl_next = ctl_.get() + ((it + 1) & 1);
    a.range = range_.get();
    a.lsum = lsum_.get();
    a.lout = lout_.get();
    a.gcount = gcount_.get();
    a.depth = depth_.get();
    a.slot = slot_.get();
    a.bounds = bounds_.get();
    a.best = best_.get();
    a.rec = rec_.get();
    a.slots = slots_.get();
    a.staging = staging_.get();
    a.staging_f = staging_f_.get();
    a.hist_slab = hist_slab_.get();
    a.ghmax = ghmax_.get();
    a.splittable = splittable_.get();
    a.tile_cnt = tile_cnt_.get();
    a.tile_off = tile_off_.get();
    a.rng = rng_.get();
    a.max_cat_bin = max_cat_bin_;
    a.max_bin = max_bin_;
    a.cat_p2 = cat_p2_;
    a.scan_scratch = scan_global_ ? scan_scratch_.get() : nullptr;
    a.fold_chunks = 1;  // LaunchReduceScan splits the fold where it applies
    a.fold_part = fold_chunks_ > 1 ? fold_part_.get() : nullptr;
    a.fold_cnt = fold_chunks_ > 1 ? fold_cnt_.get() : nullptr;
    a.scan_scratch_stride = scan_scratch_stride_;
    a.max_depth = config_->max_depth;
    // 0: separate k_post kernel, 1: block 0 after its tiles, 2: first spare block
    a.fuse_post = config_->device_post_mode;
    a.stamps = stamps_.size() ? stamps_.get() : nullptr;
    a.distributed = distributed_ ? 1 : 0;
    a.use_monotone = config_->monotone_constraints.empty() ? 0 : 1;
    a.monotone_penalty = config_->monotone_penalty;
    a.cegb_split = CegbPenalty::Enabled(config_) ? config_->cegb_tradeoff * config_->cegb_penalty_split : 0.0;
    a.ic_feat = use_ic_ ? ic_feat_.get() : nullptr;
    a.ic_leaf = use_ic_ ? ic_leaf_.get() : nullptr;
    a.root_part = root_part_.get();
    a.bar = bar_.get();
    a.leaf_key = leaf_key_.get();
    a.tile_pub = tile_pub_.get();
    a.hist_min_rows = HistMinRows();
    a.P = P_;
    a.rank = rank_;
    a.Fmax = Fmax_;
    a.cand_rows = owner_scan_ ? P_ : 1;
    a.own_feat = owner_scan_ ? own_feat_.get() : nullptr;
    a.cand = cand_.get();
    a.cand_stride = cand_stride_;
    a.cand_key_bytes = cand_key_bytes_;
    if (voting_) {
      // the partition's select and k_vote_scan use the global (elected) table
      a.cand = vcand_.get();
      a.Fmax = topk_;
      a.cand_stride = vcand_stride_;
      a.cand_key_bytes = vcand_key_bytes_;
      a.hsum_part = hsum_part_.get();
      a.lsum_loc = lsum_loc_.get();
      a.topk = topk_;
      a.lcand = cand_.get();
      a.lcand_key_bytes = cand_key_bytes_;
      a.vrec = vrec_.get();
      a.vhist = vhist_.get();
      a.vcap = vcap_;
      a.elect = elect_.get();
    }
    // data parallel: the scan reads the reduce-scattered owner row; single GPU / feature parallel:
    // the local slab rows
    a.scan_src = (owner_scan_ && data_parallel_) ? 1 : 0;
    a.rx = rx_.get();
    a.own_bin0 = h_bin_lo_.empty() ? 0 : h_bin_lo_[rank_];
    a.bbin = bbin_;
    a.bin_lo = bin_lo_.get();
    SplitParams& p = a.sp;
    p.lambda_l1 = config_->lambda_l1;
    p.lambda_l2 = config_->lambda_l2;
    p.max_delta_step = config_->max_delta_step;
    p.path_smooth = config_->path_smooth;
    p.min_gain_to_split = config_->min_gain_to_split;
    p.min_sum_hessian_in_leaf = config_->min_sum_hessian_in_leaf;
    p.cat_smooth = config_->cat_smooth;
    p.cat_l2 = config_->cat_l2;
    p.min_data_in_leaf = config_->min_data_in_leaf;
    p.max_cat_threshold = config_->max_cat_threshold;
    p.max_cat_to_onehot = config_->max_cat_to_onehot;
    p.min_data_per_group = config_->min_data_per_group;
    p.extra_trees = config_->extra_trees ? 1 : 0;
    p.use_monotone = a.use_monotone;
    return a;
  }

  // The whole growth of one tree; fixed launch shapes, data-dependent work read on device.
  void EnqueueTree() {
    const Args a = MakeArgs(0);
    hipStream_t s = stream_;
    const int part_blocks = std::max(1, std::min(max_tiles_, 4 * num_cu_));
    k_init_tree<<<1, kNodeThreads, 0, s>>>(a);
    const int root_blocks = RootBlocks();
    k_root_sums<<<root_blocks, kRootThreads, 0, s>>>(a);
    k_root_final<<<1, kRootThreads, 0, s>>>(a, root_blocks);
    if (distributed_) AllreduceSumF64(reinterpret_cast<double*>(lsum_.get()), 2, s);
    LaunchHist(a);
    LaunchScan(a);
    for (int it = 0; it < L_ - 1; ++it) {
      const Args ap = MakeArgs(it);
      if (fused_blocks_ > 0) {
        hipLaunchKernelGGL(PartitionKernel(), dim3(fused_blocks_), dim3(kPartThreads), 0, s, ap);
      } else {
        k_part_count<<<part_blocks, kPartThreads, 0, s>>>(ap);
        k_part_scatter<<<part_blocks, kPartThreads, 0, s>>>(ap);
        if (!ap.fuse_post) k_post<<<1, kPartThreads, 0, s>>>(ap);
      }
      if (it < L_ - 2) {
        const Args an = MakeArgs(it + 1);
        LaunchHist(an);
        LaunchScan(an);
      }
    }
    HIP_CHECK(hipGetLastError());
  }

  void CaptureGraph() {
    InvalidateGraph();
    hipGraph_t g;
    HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    EnqueueTree();
    HIP_CHECK(hipStreamEndCapture(stream_, &g));
    HIP_CHECK(hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    graph_comm_ = distributed_ ? ActiveComm() : nullptr;  // the captured collectives' communicator
  }

  static bool DPGraphEnabled() {
    return false;
  }

  void InvalidateGraph() {
    if (graph_exec_) {
      (void)hipGraphExecDestroy(graph_exec_);
      graph_exec_ = nullptr;
    }
    for (auto& kv : fgraphs_) (void)hipGraphExecDestroy(kv.second);
    fgraphs_.clear();
    if (fcont_) (void)hipGraphExecDestroy(fcont_);
    fcont_ = nullptr;
  }

  // Queries longer than kMaxDeviceQuery: their list and per-query slices of global scratch.
  void SetupLongQueries(const Metadata& md, bool xendcg, int* num, const int** list, const long long** off,
                        char** scratch) {
    std::vector<int> lq;
    std::vector<long long> lo;
    long long bytes = 0;
    const data_size_t* qb = md.query_boundaries();
    for (data_size_t q = 0; q < md.num_queries(); ++q) {
      const int cnt = qb[q + 1] - qb[q];
      if (cnt <= kMaxDeviceQuery) continue;
      lq.push_back(q);
      lo.push_back(bytes);
      bytes += static_cast<long long>(xendcg ? XendcgGlobalBytes(cnt) : RankGlobalBytes(cnt));
    }
    *num = static_cast<int>(lq.size());
    *list = nullptr;
    *off = nullptr;
    *scratch = nullptr;
    if (lq.empty()) return;
    long_q_.Upload(lq, stream_);
    long_off_.Upload(lo, stream_);
    long_scratch_.Resize(static_cast<size_t>(bytes));
    *list = long_q_.get();
    *off = long_off_.get();
    *scratch = long_scratch_.get();
    Log::Debug("HIP %s: %d queries longer than %d documents use %lld bytes of global scratch",
               xendcg ? "rank_xendcg" : "lambdarank", *num, kMaxDeviceQuery, bytes);
  }

  void PrepareObjective(const ObjectiveFunction* obj) {
    if (obj == prepared_obj_) return;
    prepared_obj_ = obj;
    const Metadata& md = data_->metadata();
    const label_t* lab = obj->effective_label() ? obj->effective_label() : md.label();
    label_.Upload(lab, N_, stream_);
    if (md.weights()) weight_.Upload(md.weights(), N_, stream_);
    else weight_.Free();
    if (obj->aux_weight()) aux_.Upload(obj->aux_weight(), N_, stream_);
    else aux_.Free();
    if (obj->device_kind() == DeviceGradKind::kOVA) {
      std::vector<PointwiseParams> pp(std::max(1, obj->num_class()));
      for (int k = 0; k < obj->num_class(); ++k) pp[k] = *obj->pointwise_class(k);
      ova_params_.Upload(pp, stream_);
    }
    if (obj->device_kind() == DeviceGradKind::kLambdarank) {
      LambdarankTables t;
      if (!GetLambdarankTables(obj, &t)) Log::Fatal("lambdarank tables unavailable");
      rank_gain_.Upload(*t.label_gain, stream_);
      rank_inv_dcg_.Upload(*t.inv_max_dcg, stream_);
      rank_inv_bdcg_.Upload(*t.inv_max_bdcg, stream_);
      rank_qb_.Upload(md.query_boundaries_vec(), stream_);
      RankKernelArgs& r = rank_args_;
      r.target = t.target;
      r.k = t.k;
      r.norm = t.norm;
      r.sigmoid = t.sigmoid;
      r.gap_weight = t.gap_weight;
      r.tmin = t.tmin;
      r.tmax = t.tmax;
      r.tfactor = t.tfactor;
      r.table_size = static_cast<int>(t.table->size());  // (the kernel evaluates the bins itself)
      r.label_gain = rank_gain_.get();
      r.num_label_gain = static_cast<int>(t.label_gain->size());
      r.inv_max_dcg = rank_inv_dcg_.get();
      r.inv_max_bdcg = rank_inv_bdcg_.get();
      r.qb = rank_qb_.get();
      r.num_queries = md.num_queries();
      r.max_query = 1;
      for (data_size_t q = 0; q < md.num_queries(); ++q) {
        r.max_query = std::max(r.max_query, md.query_boundaries()[q + 1] - md.query_boundaries()[q]);
      }
      {
        // 1 / log2(2 + r) for every rank of the longest query (the host objective's values)
        std::vector<double> disc(static_cast<size_t>(std::max(r.max_query, 2)) + 1);
        for (size_t i = 0; i < disc.size(); ++i) disc[i] = RankDiscount(static_cast<int>(i));
        rank_disc_.Upload(disc, stream_);
        HIP_CHECK(hipStreamSynchronize(stream_));  // (the host vector dies here)
        r.disc = rank_disc_.get();
      }
      r.label = label_.get();
      r.weight = weight_.size() ? weight_.get() : nullptr;
      // unbiased LTR: positions and the learned biases live on the device
      r.positions = nullptr;
      r.pos_bias = nullptr;
      if (md.positions() != nullptr && md.num_position_ids() > 0) {
        num_pos_ids_ = md.num_position_ids();
        pos_lr_ = t.pos_lr;
        pos_reg_ = t.pos_reg;
        std::vector<int> pos(md.positions(), md.positions() + N_);
        positions_.Upload(pos, stream_);
        pos_bias_.Resize(num_pos_ids_);
        pos_bias_.Zero(stream_);
        pos_acc_.Resize(3 * static_cast<size_t>(num_pos_ids_));
        pos_acc_.Zero(stream_);
        r.positions = positions_.get();
        r.pos_bias = pos_bias_.get();
      }
      SetupLongQueries(md, /*xendcg=*/false, &r.num_large, &r.large_q, &r.large_off, &r.large_scratch);
    }
    if (obj->device_kind() == DeviceGradKind::kXendcg) {
      int seed = 0;
      if (!GetXendcgSeed(obj, &seed)) Log::Fatal("rank_xendcg state unavailable");
      const int nq = md.num_queries();
      std::vector<unsigned> st(std::max(nq, 1));
      for (int q = 0; q < nq; ++q) st[q] = static_cast<unsigned>(seed + q);  // Random(seed + q)
      xendcg_state_.Upload(st, stream_);
      rank_qb_.Upload(md.query_boundaries_vec(), stream_);
      XendcgArgs& x = xendcg_args_;
      x.qb = rank_qb_.get();
      x.num_queries = nq;
      x.label = label_.get();
      x.weight = weight_.size() ? weight_.get() : nullptr;
      x.state = xendcg_state_.get();
      SetupLongQueries(md, /*xendcg=*/true, &x.num_large, &x.large_q, &x.large_off, &x.large_scratch);
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
  }

  // frontier engine (frontier.h)
  bool frontier_ = false;
  int fhist_threads_ = 512;
  bool nib_ = false;             // 4-bit rows built (BuildNibbleRows)
  int stride4_dw_ = 0;
  DevBuf<uint32_t> rowbins4_;
  DevBuf<HistTile> ntile_;
  bool big_tiles_ = false;  // BuildTiles chose 150 KB LDS tiles (wide rows)
  int min_tile_dw_ = 0;
  int fC_ = 0, fkmax_ = 1, fpart_tile_ = 2048, ftile_cap_ = 1, fpart_grid_ = 1, fspec_cap_ = 0, fpolicy_ = 1;
  size_t fscan_lds_ = 0;
  DevBuf<char> farena_;
  // score update fused with the next pointwise gradients (DeviceAddTreeToScore)
  // linear-leaf trees (FitLinearLeaves / TraverseLinear)
  bool linear_ = false, lin_has_nan_ = false;
  DevBuf<float> lin_raw_;
  DevBuf<LeafSeg> lin_segs_;
  DevBuf<int> lin_off_, lin_feats_, lin_toff_, lin_tfeat_;
  DevBuf<double> lin_partial_, lin_out_, lin_tcoef_, lin_tcnst_;
  DevBuf<long long> lin_usable_;
  const LinearLeaves* lin_pending_ = nullptr;  // set around TraverseLinear's traversal
  // feature-parallel frontier (FrontierFeature)
  bool ffeature_ = false;
  bool fowner_ = false;  // data-parallel owner-computes rounds (FrontierOwner)
  int fown_n_ = 0;
  DevBuf<int> fown_list_, fown_b0_;
  DevBuf<unsigned long long> facc_recv_;
  DevBuf<uint8_t> ffowned_;
  DevBuf<FPairBest> ffpb_;
  // voting-parallel frontier (FrontierVoting)
  bool fvoting_ = false;
  DevBuf<double2> flsum_loc_;
  DevBuf<unsigned long long> fltot_;
  DevBuf<VoteRec> fvrec_;
  DevBuf<int> fvelect_;
  DevBuf<unsigned long long> fvrows_;
  FState* fst_ = nullptr;
  FNode* fnodes_ = nullptr;
  FExp* fexps_ = nullptr;
  uint32_t* fbits_ = nullptr;
  double2* flsum_ = nullptr;
  double* flout_ = nullptr;
  LeafBounds* fbounds_ = nullptr;
  LeafBounds* fcbnd_ = nullptr;  // intermediate monotone: the committed leaves' current bounds
  int* fsal_ = nullptr;          // the select's alive order, carried to the next round
  SplitKey* fkey_ = nullptr;
  SplitInfo* fbest_ = nullptr;
  uint8_t* fspl_ = nullptr;
  unsigned long long* fic_ = nullptr;
  uint8_t* fnst_ = nullptr;
  int* flcid_ = nullptr;
  SplitKey* fckey_ = nullptr;
  SplitInfo* fcinfo_ = nullptr;
  DevBuf<double> fslots_;
  DevBuf<unsigned long long> facc_;
  DevBuf<unsigned long long> fhslab_;  // k_f_hist partial rows
  size_t fhslab_stride_ = 0;
  DevBuf<long long> fhmeta_;           // per row: bh << 32 | bg

  DevBuf<unsigned long long> ftile_pub_;
  std::map<int, hipGraphExec_t> fgraphs_;
  hipGraphExec_t fcont_ = nullptr;
  int fpred_rounds_ = 16, frounds_hist_[4] = {1, 1, 1, 1}, frounds_pos_ = 0;
  // data-parallel per-round expansion caps (= all-reduce sizes) from the last trees' rounds
  DevBuf<FForced> fforced_;
  // CEGB coupled penalties (frontier select): penalties, used flags, event count, per-node
  // raw candidates and the event count each node's best was scored at
  DevBuf<double> cegb_coupled_;
  DevBuf<uint8_t> cegb_used_;
  DevBuf<unsigned> cegb_epoch_;
  DevBuf<SplitKey> fnkey_;
  DevBuf<SplitInfo> fninfo_;
  DevBuf<int> fnuep_;
  // CEGB lazy penalties: penalties, per-row marks, round counts, per-node counts and paths
  DevBuf<double> cegb_lazy_;
  DevBuf<uint32_t> lazy_bits_;
  DevBuf<int> lazy_acc_;
  DevBuf<int> fnlazy_;
  DevBuf<uint32_t> fnpath_;
  int lazy_words_ = 0;
  const Dataset* cegb_data_ = nullptr;  // training set the CEGB usage state belongs to
  int fnum_forced_ = 0;
  SplitInfo* ffbest_ = nullptr;
  SplitKey* ffkey_ = nullptr;
  char* fres_host_ = nullptr;  // FResultHdr + records + ranges (coherent pinned host memory)
  void* fres_dev_ = nullptr;
  size_t fres_bytes_ = 0;
  bool fcaps_on_ = false;
  int fcap_host_[kFrontierRoundCap] = {};
  int fkused_hist_[4][kFrontierRoundCap] = {};
  int fkused_trees_ = 0;
  double fstat_ar_exps_ = 0.0;
  long long fstat_pipelined_ = 0;
  double fglobal_rows_ = 0.0;  // rows over all ranks (qpack bound of the data-parallel frontier)
  // data-parallel pipeline: the comm stream and its fork / join events (EnqueueFrontierRound)
  hipStream_t comm_stream_ = nullptr;
  hipEvent_t pipe_ev_[4] = {nullptr, nullptr, nullptr, nullptr};
  DevBuf<int> fkcap_, fkused_;
  PinnedBuf<int> pin_kcap_;
  long long fstat_rounds_ = 0, fstat_spec_ = 0;
  double fstat_waste_ = 0.0, fspec_alpha_ = 1.0;
  bool fspec_fixed_ = false;
  // Speculation budget tuned on measured tree times (trees share the exact split sequence
  // whatever the budget, so only the time changes): pairs of consecutive trees at alpha and
  // 1.5 alpha, six pairs per decision; a budget that is >= 2% faster on average becomes the
  // base, a >= 2% slower one sends the base down (floor 1), otherwise the base rests 48 trees
  struct SpecTuner {
    bool on = false;
    double lo = 1.0, t_lo = 0.0, dsum = 0.0;
    int phase = 0, pairs = 0, rest = 0;
    double Alpha() const { return rest > 0 || phase == 0 ? lo : std::min(4.0, lo * 1.5); }
    void Record(double dt) {
      if (rest > 0) {
        --rest;
        return;
      }
      if (phase == 0) {
        t_lo = dt;
        phase = 1;
        return;
      }
      phase = 0;
      dsum += t_lo > 0.0 ? (dt - t_lo) / t_lo : 0.0;
      if (++pairs < 6) return;
      const double m = dsum / pairs;
      pairs = 0;
      dsum = 0.0;
      if (m < -0.02 && lo < 4.0) {
        lo = std::min(4.0, lo * 1.5);
      } else if (m > 0.02 && lo > 1.0) {
        lo = std::max(1.0, lo / 1.5);
      } else {
        rest = 48;
      }
    }
  };
  SpecTuner stune_;
  int fstat_trees_ = 0;
  DevBuf<unsigned long long> fstamps_;
  const float2* fgraph_gh_ = nullptr;
  const Config* config_;
  bool data_parallel_ = false;
  bool distributed_ = false;
  const Dataset* data_ = nullptr;
  int N_ = 0, F_ = 0, G_ = 0, TB_ = 0, width_ = 1, stride_dw_ = 1, L_ = 2, K_ = 1;
  int row_align_ = 0;     // tile / padded-row alignment in dwords (RowAlign), 0: none
  int tstride_dw_ = 1;   // row stride of the TRAINING rows (rowbins_): stride_dw_, or padded (RowAlign)
  int device_id_ = 0, num_cu_ = 256, num_tiles_ = 0, max_tiles_ = 1, max_cat_bin_ = 1;
  bool has_cat_ = false, use_bag_ = false, use_bynode_ = false, use_dp_ = false;
  int bynode_draws_ = 0;  // by-node masks the last tree used (the host sampler's GetByNode calls)
  data_size_t bag_cnt_ = 0;
  size_t hist_lds_bytes_ = 0, scan_lds_bytes_ = 0;
  size_t hist_lds_plain_ = 0;  // the tile plan's LDS without the interleaved slots' reserve
  int max_bin_ = 2, cat_p2_ = 1;
  bool scan_global_ = false;
  size_t scan_scratch_stride_ = 0;
  DevBuf<char> scan_scratch_;
  int fold_chunks_ = 1;
  DevBuf<double> fold_part_;
  DevBuf<unsigned> fold_cnt_;
  std::string device_name_;
  hipStream_t stream_ = nullptr;
  hipGraphExec_t graph_exec_ = nullptr;
  ncclComm_t graph_comm_ = nullptr;
  ColSampler col_sampler_;
  const ObjectiveFunction* prepared_obj_ = nullptr;
  std::vector<LeafRange> h_range_;

  DevBuf<uint32_t> rowbins_;
  DevBuf<uint8_t> colbins_;
  DevBuf<float2> gh_;
  DevBuf<double> score_;
  DevBuf<float> label_, weight_, aux_;
  static_assert(kFrontierIdx <= kLeafIdxBufs, "leaf renewal addresses every index buffer");
  DevBuf<int> idx_[kFrontierIdx];
  DevBuf<DevFeature> feat_;
  DevBuf<int> gstart_;
  DevBuf<HistTile> tiles_;
  DevBuf<TreeParams> tparams_;
  DevBuf<Ctl> ctl_;
  DevBuf<LeafRange> range_;
  DevBuf<double2> lsum_;
  DevBuf<double> lout_;
  DevBuf<int> gcount_, depth_, slot_;
  DevBuf<LeafBounds> bounds_;
  DevBuf<SplitInfo> best_;
  DevBuf<SplitRec> rec_;
  DevBuf<double> slots_, staging_;
  DevBuf<float> staging_f_;
  DevBuf<char> hist_slab_, arena_;
  DevBuf<unsigned long long> stamps_;
  int stamp_trees_ = 0;
  std::vector<DevFeature> h_feats_;
  std::vector<int> h_gstart_;
  std::vector<HistTile> h_tiles_;
  DevBuf<unsigned> ghmax_;
  DevBuf<uint8_t> splittable_;
  DevBuf<int> tile_cnt_, tile_off_;
  DevBuf<uint8_t> used_bytree_, bynode_;
  DevBuf<unsigned long long> ic_feat_, ic_leaf_;
  DevBuf<unsigned long long> fic_feat_;  // [F][ic_words_] (the frontier's interaction-constraint words)
  int ic_words_ = 1;
  DevBuf<unsigned> qmax_;
  DevBuf<double2> true_sums_;
  DevBuf<double> root_part_;
  DevBuf<unsigned> bar_;
  DevBuf<SplitKey> leaf_key_;
  // owner-computes parallel modes
  DevParallel mode_ = DevParallel::kSerial;
  bool owner_scan_ = false;
  int P_ = 1, rank_ = 0, Fmax_ = 1, bbin_ = 1, cand_stride_ = 0, cand_key_bytes_ = 0;
  std::vector<int> h_bin_lo_, h_own_feat_;
  DevBuf<int> own_feat_, bin_lo_;
  DevBuf<char> cand_, rx_, stage_;
  DevBuf<unsigned> xcnt_;
  // voting parallel
  bool voting_ = false;
  int topk_ = 1, vcap_ = 2, vcand_key_bytes_ = 0, vcand_stride_ = 0;
  size_t vote_local_lds_ = 0, vote_pack_lds_ = 0, vote_scan_lds_ = 0;
  DevBuf<char> vcand_, vhist_;
  DevBuf<VoteRec> vrec_;
  DevBuf<int> elect_;
  DevBuf<double2> hsum_part_, lsum_loc_;
  // frontier xGMI transport (SetupFrontierXgmi; FArgs::xg)
  bool fxg_ = false;
  char* fx_local_ = nullptr;
  std::vector<char*> fx_peers_;
  unsigned fxo_recv_ = 0, fxo_fpb_ = 0, fxo_root_ = 0, fxo_flag_ = 0;
  size_t fxo_vrec_ = 0, fxo_vrows_ = 0;
  DevBuf<unsigned> fxep_, fxcnt_;
  DevBuf<FXConf> fxconf_;          // FArgs::xc
  DevBuf<SplitParams> fsp_local_;  // FArgs::sp_local (voting's local pass)
  DevBuf<uint8_t> fbyn_mode_;      // FArgs::byn_mode (by-node draws in the select)
  int fbyn_cnt_ = 0, fbyn_reset_ = 0;
  unsigned bynode_rng_ = 0;        // the select's sampler state after the last tree (FState::byn_rng)
  int cached_gcount_ = -1, cached_gcount_local_ = -1;
  DevBuf<unsigned long long> tile_pub_;
  PinnedBuf<unsigned> pin_bar_;
  int fused_blocks_ = 0;  // k_partition grid (0: two-kernel partition)
  int part_iters_ = 8;    // rows per thread of the fused partition (PartIters())
  int fpart_iters_ = 8;   // rows per thread of the frontier partition
  const Tree* last_trained_ = nullptr;  // DeviceTrain's tree: its leaf ranges are still on the device
  DevBuf<float2> gh_true_;
  DevBuf<uint16_t> ghq_;  // quantized levels for the frontier's integer histograms
  bool use_ic_ = false, is_const_hess_ = false;
  unsigned quant_round_ = 0;
  DevBuf<unsigned> rng_;
  DevBuf<char> tree_buf_;
  // lambdarank tables
  DevBuf<double> rank_disc_, rank_gain_, rank_inv_dcg_, rank_inv_bdcg_;
  DevBuf<int> rank_qb_;
  RankKernelArgs rank_args_;
  DevBuf<unsigned> xendcg_state_;
  DevBuf<int> row_query_;  // bagging by query: query of each row
  struct DevValid {
    int n = 0;
    DevBuf<uint32_t> rowbins;
    DevBuf<double> score;
    DevBuf<float> label, weight;
    const float* host_label = nullptr;  // the dataset's labels (identity check of metric specs)
  };
  // per-metric device tables of the ranking / AUC metrics (DeviceEvalRank), keyed by the metric
  struct RankEvalState {
    int kind = -1, n = 0, nq = 0;
    const void* host_label = nullptr;
    const void* host_qb = nullptr;
    std::vector<int> ks;
    DevBuf<int> qb, npos, ks_dev;
    DevBuf<float> qw;
    DevBuf<double> inv_max, gain, disc, out;
    DevBuf<char> scratch;
  };
  std::map<const void*, std::unique_ptr<RankEvalState>> rank_states_;
  // auc_mu tables per metric: the class-ordered row index, one pair's scored rows, the pairs' sums
  struct AucMuState {
    int n = 0;
    const void* host_label = nullptr;
    DevBuf<int> idx;
    DevBuf<double> dist, out;
    DevBuf<float> lab, w;
    DevBuf<char> scratch;
  };
  std::map<const void*, std::unique_ptr<AucMuState>> aucmu_states_;
  PinnedBuf<double> pin_metric_;
  std::vector<std::unique_ptr<DevValid>> valid_;
  // refit / leaf renewal
  DevBuf<int> leaf_pred_dev_, renew_off_, renew_nz_;
  DevBuf<double> refit_partial_, refit_sums_, refit_delta_, renew_out_;
  DevBuf<LeafSeg> renew_segs_;
  DevBuf<int> leaf_bounds_;  // LeafMapScore: per-leaf tile bounds
  DevBuf<uint8_t> leaf_map_;  // LeafMapScore: leaf of every row (uint8 / uint16)
  DevBuf<double> pend_lv_;    // LeafMapScore: the pending add's leaf values
  DevBuf<int> oob_;           // DeviceSample: the out-of-bag rows, ascending (LeafMapScore)
  bool oob_ok_ = false;       // oob_ holds the current bag's complement
  struct PendingAdd {
    bool on = false;
    int k = 0, nl = 0;
  };
  mutable PendingAdd pend_;  // a tree's leaf add not yet applied to score_ (FlushScore)
  std::vector<uint8_t> leaf_desc_;  // LeafMapScore: per-leaf row direction
  std::vector<std::pair<int, int>> leaf_walk_;
  DevBuf<char> renew_scratch_;
  // multiclassova / unbiased LTR / long queries
  DevBuf<PointwiseParams> ova_params_;
  DevBuf<int> positions_, long_q_;
  DevBuf<double> pos_bias_;
  DevBuf<long long> pos_acc_, long_off_;
  DevBuf<char> long_scratch_;
  int num_pos_ids_ = 0;
  double pos_lr_ = 0.0, pos_reg_ = 0.0;
  // device training metrics
  static constexpr int kMetricBlocks = 1024;
  DevBuf<float> metric_label_, metric_weight_;
  DevBuf<double> metric_partial_;
  XendcgArgs xendcg_args_;
  // pinned staging
  PinnedBuf<TreeParams> pin_tp_;
  PinnedBuf<uint8_t> pin_mask_;
  PinnedBuf<Ctl> pin_ctl_;
  PinnedBuf<SplitRec> pin_rec_;
  PinnedBuf<LeafRange> pin_range_;
  PinnedBuf<double> pin_lout_;
  PinnedBuf<float2> pin_gh_;
  PinnedBuf<char> pin_tree_;
  PinnedBuf<char> pin_tree_ring_[2];  // TraverseTreeCompact staging (see there)
  DevBuf<char> ttree_buf_;             // its device copy (stream-ordered reuse)
  hipEvent_t tree_evt_[2] = {nullptr, nullptr};
  unsigned tree_slot_ = 0;
  PinnedBuf<unsigned> pin_max_;
  // device row sampling
  DevBuf<uint2> samp_jump_;
  DevBuf<unsigned> samp_rng_, samp_sel_;
  DevBuf<int> samp_cnt_, samp_total_;
  DevBuf<float> bag_label_;
  PinnedBuf<int> pin_cnt_;
};

}  // namespace

std::unique_ptr<TreeLearner> CreateDeviceTreeLearner(const Config* config, const std::string& parallel_mode) {
  if (parallel_mode == "serial") return std::make_unique<DeviceTreeLearner>(config, DevParallel::kSerial);
  if (parallel_mode == "data") return std::make_unique<DeviceTreeLearner>(config, DevParallel::kData);
  if (parallel_mode == "feature") return std::make_unique<DeviceTreeLearner>(config, DevParallel::kFeature);
  if (parallel_mode == "voting") return std::make_unique<DeviceTreeLearner>(config, DevParallel::kVoting);
  Log::Fatal("Unknown tree learner type %s", parallel_mode.c_str());
  return nullptr;
}

bool LinearOnDevice(const Config* config, const Dataset* train, const std::string& learner_type) {
  if (learner_type != "serial" || config->use_quantized_grad || train == nullptr || !train->has_raw()) return false;
  // the Gram tile holds <= kLinMaxM - 1 branch features: bounded by the features, the leaves
  // and the depth
  long long k = std::min<long long>(train->num_features(), std::max(1, config->num_leaves) - 1);
  if (config->max_depth > 0) k = std::min<long long>(k, config->max_depth);
  return k + 1 <= kLinMaxM;
}

namespace {
bool FrontierShapeFor(const Config* config, const Dataset* train, bool raw, bool mono_inter = false) {
  if (config->interaction_constraints_vector.size() > 64 * static_cast<size_t>(kFrontierIcWords)) return false;
  if (train == nullptr) return config->num_leaves <= 256;  // (no data yet: a conservative shape)
  int max_bin = 2, max_cat_bin = 1;
  for (int f = 0; f < train->num_features(); ++f) {
    const FeatureInfo& fi = train->feature(f);
    max_bin = std::max(max_bin, fi.num_bin);
    if (fi.bin_type == BinType::Categorical) max_cat_bin = std::max(max_cat_bin, fi.num_bin);
  }
  return FrontierShapeFits(std::max(2, config->num_leaves), train->num_total_bin(), train->num_features(), max_bin,
                           max_cat_bin, raw, mono_inter);
}
}  // namespace

bool FrontierServes(const Config* config, const Dataset* train, const std::string& learner_type) {
  if (learner_type != "serial" || config->feature_fraction_bynode < 1.0 || config->extra_trees) return false;
  const bool cegb_raw = !config->cegb_penalty_feature_coupled.empty() || !config->cegb_penalty_feature_lazy.empty();
  return FrontierShapeFor(config, train, cegb_raw);
}

bool FrontierServesMonoInter(const Config* config, const Dataset* train, const std::string& learner_type) {
  if (learner_type != "serial" || config->feature_fraction_bynode < 1.0 || config->extra_trees) return false;
  if (!config->forcedsplits_filename.empty() || CegbPenalty::Enabled(config)) return false;
  if (config->monotone_constraints_method != "intermediate") return false;
  return FrontierShapeFor(config, train, false, true);
}

bool FrontierServesByNode(const Config* config, const Dataset* train, const std::string& learner_type) {
  if (learner_type != "serial" || config->extra_trees) return false;
  return FrontierShapeFor(config, train, true);  // (by-node sampling keeps raw candidates)
}

namespace {
class DeviceHistogramBackend final : public HistogramBackend {
 public:
  DeviceHistogramBackend(const Config* user, const Dataset* data) {
    // private config: only the knobs the histogram kernels read
    cfg_.num_leaves = 2;
    cfg_.verbosity = user->verbosity;
    cfg_.gpu_use_dp = user->gpu_use_dp;
    cfg_.gpu_device_id = user->gpu_device_id;
    cfg_.device_hist_blocks = user->device_hist_blocks;
    learner_ = std::make_unique<DeviceTreeLearner>(&cfg_, DevParallel::kSerial);
    learner_->Init(data, false);
    data_ = data;
  }
  void SetGradients(const float* g, const float* h, int n) override { learner_->BackendSetGradients(g, h, n); }
  void Histogram(const int* rows, int n, double* out) override { learner_->BackendHistogram(rows, n, out); }
  std::string DeviceName() const override { return learner_->DeviceName(); }

  // ---- resident slots + device scans (policy_scan.h)
  bool EnableResidentSlots(int num_slots) override {
    int max_bin = 2;
    std::vector<PolicyFeat> feats(data_->num_features());
    for (int f = 0; f < data_->num_features(); ++f) {
      const FeatureInfo& fi = data_->feature(f);
      PolicyFeat& p = feats[f];
      p.hist_offset = fi.hist_offset;
      p.num_bin = fi.num_bin;
      p.mfb = static_cast<int>(fi.mfb);
      p.default_bin = static_cast<int>(fi.default_bin);
      p.missing = static_cast<int8_t>(fi.missing);
      p.bin_type = static_cast<int8_t>(fi.bin_type);
      p.monotone = fi.monotone;
      p.pad = 0;
      p.penalty = fi.penalty;
      max_bin = std::max(max_bin, fi.num_bin);
    }
    // the scan's LDS holds one full feature histogram and its sort order (<= 64 KiB)
    if (static_cast<size_t>(max_bin) * (2 * sizeof(double) + sizeof(int)) > 64 * 1024) return false;
    max_bin_ = max_bin;
    stride_ = 2 * static_cast<size_t>(data_->num_total_bin());
    slots_.Resize(static_cast<size_t>(std::max(1, num_slots)) * stride_);
    feat_.Upload(feats, learner_->BackendStream());
    HIP_CHECK(hipStreamSynchronize(learner_->BackendStream()));
    num_slots_ = num_slots;
    return true;
  }
  void HistogramToSlot(const int* rows, int n, int slot) override {
    CheckSlot(slot);
    learner_->BackendHistogramDevice(rows, n, slots_.get() + static_cast<size_t>(slot) * stride_);
  }
  void SubtractSlots(int larger, int smaller) override {
    CheckSlot(larger);
    CheckSlot(smaller);
    LaunchPolicySubtract(slots_.get() + static_cast<size_t>(larger) * stride_,
                         slots_.get() + static_cast<size_t>(smaller) * stride_, stride_, learner_->BackendStream());
  }
  void ScanSlots(const ScanBatch& b, const SplitParams& params, SplitInfo* out, uint8_t* splittable) override {
    const int R = static_cast<int>(b.slot.size());
    const int F = data_->num_features();
    if (R == 0 || F == 0) return;
    hipStream_t s = learner_->BackendStream();
    std::vector<PolicyReq> req(R);
    for (int r = 0; r < R; ++r) {
      CheckSlot(b.slot[r]);
      req[r].slot = b.slot[r];
      req[r].count = b.count[r];
      req[r].sum_g = b.sum_g[r];
      req[r].sum_h = b.sum_h[r];
      req[r].parent_output = b.parent_output[r];
    }
    const size_t items = static_cast<size_t>(R) * F;
    if (b.enable.size() != items || b.bmin.size() != items || b.bmax.size() != items || b.tb_off.size() != items) {
      Log::Fatal("HIP policy scan: batch of %d leaves x %d features is malformed", R, F);
    }
    std::vector<PolicyBound> bnd(items);
    for (size_t i = 0; i < items; ++i) {
      bnd[i].min = b.bmin[i];
      bnd[i].max = b.bmax[i];
      bnd[i].tb_off = b.tb_off[i];
      const int nb = data_->feature(static_cast<int>(i % F)).num_bin;
      if (b.tb_off[i] >= 0 && static_cast<size_t>(b.tb_off[i]) + 4 * static_cast<size_t>(nb) > b.tb.size()) {
        Log::Fatal("HIP policy scan: threshold bounds offset %lld outside %zu values", b.tb_off[i], b.tb.size());
      }
    }
    req_.Upload(req, s);
    bnd_.Upload(bnd, s);
    en_.Upload(b.enable, s);
    if (!b.tb.empty()) tb_.Upload(b.tb, s);
    if (out_.size() < items) out_.Resize(items);
    if (sp_.size() < items) sp_.Resize(items);
    PolicyScanArgs a;
    a.slots = slots_.get();
    a.slot_stride = stride_;
    a.feat = feat_.get();
    a.F = F;
    a.R = R;
    a.max_bin = max_bin_;
    a.req = req_.get();
    a.bnd = bnd_.get();
    a.enable = en_.get();
    a.tb = b.tb.empty() ? nullptr : tb_.get();
    a.p = params;
    a.out = out_.get();
    a.splittable = sp_.get();
    LaunchPolicyScan(a, s);
    out_.Download(out, items, s);
    sp_.Download(splittable, items, s);
    HIP_CHECK(hipStreamSynchronize(s));
  }

 private:
  void CheckSlot(int slot) const {
    if (slot < 0 || slot >= num_slots_) Log::Fatal("HIP histogram slot %d outside [0, %d)", slot, num_slots_);
  }
  Config cfg_;
  std::unique_ptr<DeviceTreeLearner> learner_;
  const Dataset* data_ = nullptr;
  int max_bin_ = 2, num_slots_ = 0;
  size_t stride_ = 0;
  DevBuf<double> slots_, tb_;
  DevBuf<PolicyFeat> feat_;
  DevBuf<PolicyReq> req_;
  DevBuf<PolicyBound> bnd_;
  DevBuf<uint8_t> en_, sp_;
  DevBuf<SplitInfo> out_;
};
}  // namespace

std::unique_ptr<HistogramBackend> CreateHistogramBackend(const Config* config, const Dataset* data) {
  if (DeviceCount() <= 0) Log::Fatal("HIP histogram backend: no AMD GPU visible to HIP");
  return std::make_unique<DeviceHistogramBackend>(config, data);
}

void TestFrontierHist(const Dataset* data, const Config& config, const float* grad, const float* hess, const int* rows,
                      const int* offsets, int k, double* out, uint16_t* levels) {
  if (DeviceCount() <= 0) Log::Fatal("TestFrontierHist: no AMD GPU visible to HIP");
  DeviceTreeLearner learner(&config, DevParallel::kSerial);
  learner.Init(data, false);
  learner.TestFrontierHist(grad, hess, rows, offsets, k, out, levels);
}

void TestFrontierScan(const Dataset* data, const Config& config, const float* grad, const float* hess, double* out,
                      double* ref) {
  if (DeviceCount() <= 0) Log::Fatal("TestFrontierScan: no AMD GPU visible to HIP");
  DeviceTreeLearner learner(&config, DevParallel::kSerial);
  learner.Init(data, false);
  learner.TestFrontierScan(grad, hess, out, ref);
}

void TestFrontierPartition(const Dataset* data, const Config& config, const int* rows, const int* offsets, int k,
                           const int* feats, const int* thr, const int* dleft, const uint32_t* catbits, int* out_rows,
                           int* out_left, int* exp_rows, int* exp_left) {
  if (DeviceCount() <= 0) Log::Fatal("TestFrontierPartition: no AMD GPU visible to HIP");
  DeviceTreeLearner learner(&config, DevParallel::kSerial);
  learner.Init(data, false);
  learner.TestFrontierPartition(rows, offsets, k, feats, thr, dleft, catbits, out_rows, out_left, exp_rows, exp_left);
}

void DeviceHistogram(const Dataset* data, const float* grad, const float* hess, const int* rows, int num_rows,
                     double* out) {
  if (DeviceCount() <= 0) Log::Fatal("DeviceHistogram: no AMD GPU visible to HIP");
  Config cfg;
  cfg.num_leaves = 2;
  cfg.verbosity = -1;
  DeviceTreeLearner learner(&cfg, DevParallel::kSerial);
  learner.Init(data, false);
  learner.TestHistogram(grad, hess, rows, num_rows, out);
}

}  // namespace device
}  // namespace lgap
