// Host-callable entry points of the HIP device layer (src/device/*.hip).
// Kept free of HIP headers so plain C++ translation units can include it.
#pragma once

#include <memory>
#include <string>

#include "lgap/config.h"
#include "lgap/tree_learner.h"

namespace lgap {
namespace device {

// Number of visible MI355X (gfx950) devices; 0 when no GPU / no driver.
int DeviceCount();
// hipDeviceSynchronize on the current device (no-op without a GPU).
void DeviceSynchronize();
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

// Histogram of (grad, hess) over `rows` (all rows when null) with the HIP
// histogram kernel; out has 2 * num_total_bin doubles.
void DeviceHistogram(const Dataset* data, const float* grad, const float* hess, const int* rows, int num_rows,
                     double* out);

}  // namespace device
}  // namespace lgap
