// Internal accessors of the device runtime shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>

namespace lgap {
namespace device {

ncclComm_t ActiveComm();
int CommDevice();
// communicator present (CommActive() additionally requires more than one rank)
bool CommExists();
// LGAP_DEVICE_DP_TRANSPORT=host with a multi-rank host Network and no RCCL
// communicator: the device data-parallel learner stages its collectives through
// host memory (lets several ranks share one GPU to rehearse the multi-rank path).
bool HostStagedDP();
// In-place sum all-reduce of device doubles on `stream` (no-op without a communicator).
void AllreduceSumF64(double* dev_ptr, size_t count, hipStream_t stream);
void AllreduceSumF32(float* dev_ptr, size_t count, hipStream_t stream);
// hipStreamSynchronize for streams carrying collectives: polls the communicator's
// async error and aborts it after timeout_s (<= 0: no limit), raising a fatal error.
void WatchedStreamSync(hipStream_t stream, double timeout_s, const char* what);
// collective timeout: LGAP_COMM_TIMEOUT_S, else the `time_out` parameter (minutes)
double CommTimeoutSeconds(int time_out_minutes);

}  // namespace device
}  // namespace lgap
