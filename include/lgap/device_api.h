// Host-callable entry points of the HIP device layer (src/device/*.hip).
// Kept free of HIP headers so plain C++ translation units can include it.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "lgap/config.h"
#include "lgap/split_math.h"
#include "lgap/tree_learner.h"

namespace lgap {
namespace device {

// Number of visible MI355X (gfx950) devices; 0 when no GPU / no driver.
int DeviceCount();
// hipDeviceSynchronize on the current device (no-op without a GPU).
void DeviceSynchronize();
// Total memory of the current device in bytes (0 without a GPU).
size_t DeviceTotalMemory();
// RCCL communicator over xGMI for the multi-GPU learners.
std::string CommGetUniqueId();
void CommInit(const std::string& unique_id, int num_ranks, int rank, int device_id);
void CommFree();
int CommRank();
int CommSize();
bool CommActive();

// Single-process HIP tree learner (device_type=gpu|cuda) and its data-parallel
// variant (tree_learner=data|voting|feature with an RCCL communicator).
std::unique_ptr<TreeLearner> CreateDeviceTreeLearner(const Config* config, const std::string& parallel_mode);
// Whether the device learner's frontier engine can grow `config`'s trees on `train` (learner
// type, sampling options and the engine's fixed LDS / node-capacity shape). The options only
// the frontier implements on the device (forced splits, CEGB feature penalties) route to the
// host split policy when it cannot.
bool FrontierServes(const Config* config, const Dataset* train, const std::string& learner_type);
// The same for feature_fraction_bynode under interaction constraints: the frontier's select
// draws each node's mask over the features its constraints allow (serial learner only).
bool FrontierServesByNode(const Config* config, const Dataset* train, const std::string& learner_type);
// intermediate monotone constraints in the serial frontier's select (FArgs::mono_inter): no by-node
// sampling, extra trees, forced splits or CEGB, and the select's extra LDS fits
bool FrontierServesMonoInter(const Config* config, const Dataset* train, const std::string& learner_type);
// Whether the device learner fits linear_tree leaves itself (fp64 MFMA Gram systems): serial
// learner, float gradients, raw values kept, and at most 30 branch features per leaf.
bool LinearOnDevice(const Config* config, const Dataset* train, const std::string& learner_type);

// GPU histogram engine for the host learners (the reference's GPUTreeLearner
// split, src/treelearner/gpu_tree_learner.cpp: histograms on the device, split
// policy on the host). Used when a host-side policy (CEGB, forced splits,
// intermediate/advanced monotone, linear leaves, voting/feature parallel) is
// requested with device_type=gpu. Gradients are uploaded once per tree.
class HistogramBackend {
 public:
  virtual ~HistogramBackend() = default;
  virtual void SetGradients(const float* grad, const float* hess, int num_data) = 0;
  // out: 2 * num_total_bin doubles (group bin 0 left zero, as the host builder)
  virtual void Histogram(const int* rows, int num_rows, double* out) = 0;
  virtual std::string DeviceName() const = 0;

  // ---- device-resident histograms and device split scans (intermediate / advanced monotone
  // constraints: src/device/policy_scan.h). The host keeps only the tree, the row partition and
  // the constraint bookkeeping; histograms never leave the device, scans return SplitInfo rows.
  // Allocates `num_slots` histogram slots of 2 * num_total_bin doubles; false: not available.
  virtual bool EnableResidentSlots(int num_slots) { (void)num_slots; return false; }
  // slot <- histogram of `rows` (all rows when null)
  virtual void HistogramToSlot(const int* rows, int num_rows, int slot) { (void)rows; (void)num_rows; (void)slot; }
  // larger <- larger - smaller (the parent's histogram held by the larger child's slot)
  virtual void SubtractSlots(int larger, int smaller) { (void)larger; (void)smaller; }
  // Scans the batch's leaves over every feature. Per leaf r: slot, row count, sums, parent output;
  // per (r, f): enable flag, flat bounds and (advanced) the offset of lmin / lmax / rmin / rmax
  // (num_bin doubles each) in `tb`, or -1. Returns out[r * F + f] (feature -1 when the feature
  // cannot split) and splittable[r * F + f].
  struct ScanBatch {
    std::vector<int> slot, count;
    std::vector<double> sum_g, sum_h, parent_output;
    std::vector<uint8_t> enable;
    std::vector<double> bmin, bmax;
    std::vector<long long> tb_off;
    std::vector<double> tb;
    void Clear() {
      slot.clear(); count.clear(); sum_g.clear(); sum_h.clear(); parent_output.clear();
      enable.clear(); bmin.clear(); bmax.clear(); tb_off.clear(); tb.clear();
    }
  };
  virtual void ScanSlots(const ScanBatch& batch, const SplitParams& params, SplitInfo* out, uint8_t* splittable) {
    (void)batch; (void)params; (void)out; (void)splittable;
  }
};
std::unique_ptr<HistogramBackend> CreateHistogramBackend(const Config* config, const Dataset* data);

// Histogram of (grad, hess) over `rows` (all rows when null) with the HIP
// histogram kernel; out has 2 * num_total_bin doubles.
void DeviceHistogram(const Dataset* data, const float* grad, const float* hess, const int* rows, int num_rows,
                     double* out);

// Direct tests of the frontier's production kernels (tests/test_frontier_kernels.py):
// k_f_hist over k row subsets (rows concatenated, offsets[k + 1]) -> out[k][num_total_bin][2]
// at the kernel's fixed-point scale (quantized training: integer level sums; levels[N] the
// quantized g << 8 | h levels); k_f_partition of k parents split by (inner feature, threshold
// bin / categorical bin set, default_left) -> the device's children lists and left counts, and
// the host learner's stable partition of the same split.
void TestFrontierHist(const Dataset* data, const Config& config, const float* grad, const float* hess, const int* rows,
                      const int* offsets, int k, double* out, uint16_t* levels);
// k_f_scan of the root round over all rows -> out[F][8] (gain, threshold, left count, default_left,
// left sum g, left sum h, valid, categorical thresholds), ref[F][8] the host split_math.h scan
void TestFrontierScan(const Dataset* data, const Config& config, const float* grad, const float* hess, double* out,
                      double* ref);
void TestFrontierPartition(const Dataset* data, const Config& config, const int* rows, const int* offsets, int k,
                           const int* feats, const int* thr, const int* dleft, const uint32_t* catbits, int* out_rows,
                           int* out_left, int* exp_rows, int* exp_left);

// One pass of the device row-sampling kernels over host arrays (LGBM_DeviceSampleRows):
// returns the kept-row count, rows in out_rows, GOSS scaling applied to grad / hess.
int SampleRowsOnDevice(int mode, int num_rows, int num_class, float* grad, float* hess, const float* label,
                       double fraction, double pos_fraction, double neg_fraction, double top_rate, double other_rate,
                       int bagging_seed, uint32_t goss_seed, int rounds, int* out_rows);

// Feature binning on the device (bin_kernels.hip): packs `nrow` rows of a dense row-major
// matrix (fp32 / fp64) into `ds`'s packed group-bin layout (its mappers and EFB groups),
// writing host_out (nrow x row_stride bytes). With keep_device_copy the device rows stay
// registered for the HIP learner of `ds` (TakeDeviceRows). False: not supported here (the
// caller bins on the host).
bool DevicePackDense(const Dataset& ds, const void* data, bool f64, int nrow, int ncol, uint8_t* host_out,
                     bool keep_device_copy);
// the device copy of `ds`'s packed rows (ownership moves to the caller; hipFree), or nullptr
// when none matches `bytes`
void* TakeDeviceRows(const Dataset* ds, size_t bytes);
void ReleaseDeviceRows(const Dataset* ds);

}  // namespace device
}  // namespace lgap
