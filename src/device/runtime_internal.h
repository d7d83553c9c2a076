// Internal accessors of the device runtime shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <vector>

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
// exact integer sums (fixed-point histograms: two's complement wraps like int64 addition)
void AllreduceSumU64(unsigned long long* dev_ptr, size_t count, hipStream_t stream);
// in-place max of device uint32 values (e.g. the float bits of non-negative maxima)
void AllreduceMaxU32(unsigned* dev_ptr, size_t count, hipStream_t stream);
// hipStreamSynchronize for streams carrying collectives: polls the communicator's
// async error and aborts it after timeout_s (<= 0: no limit), raising a fatal error.
void WatchedStreamSync(hipStream_t stream, double timeout_s, const char* what);
// collective timeout: LGAP_COMM_TIMEOUT_S, else the `time_out` parameter (minutes)
double CommTimeoutSeconds(int time_out_minutes);

// ---- owner-computes data parallelism (device learner)
// ranks / this rank of the data-parallel group (host Network when it spans several
// processes, else the RCCL communicator)
int DpSize();
int DpRank();
// `send`: DpSize() blocks of `count` fp32 (fp64 with f64) values; recv: this rank's block
// summed over ranks (ncclReduceScatter, or host-staged for the rehearsal transport)
void ReduceScatterSum(const void* send, void* recv, size_t count, bool f64, hipStream_t stream);
void ReduceScatterSumU64(const unsigned long long* send, unsigned long long* recv, size_t count, hipStream_t stream);
// in-place allgather of DpSize() blocks of `bytes` (this rank's block filled)
void AllGatherInPlace(void* buf, size_t bytes, hipStream_t stream);
// map every rank's exchange buffer (same size / layout on all ranks) into this process
// over IPC (xGMI transport); collective; false on every rank if any rank failed
bool XgmiOpen(char* local, std::vector<char*>* peers);
void XgmiClose(char* local, std::vector<char*>* peers);

}  // namespace device
}  // namespace lgap
