// Device runtime: device discovery and the RCCL communicator (one process per
// GPU, xGMI transport). The communicator is bootstrapped from an ncclUniqueId
// that the launcher (torch.distributed / the CLI's socket network) broadcasts.
//
// Besides the device learners' histogram all-reduce, the same communicator
// backs the host collective layer (Network) when no socket mesh is configured:
// allgather of host bytes goes through a device staging buffer and
// ncclAllGather (Network derives reduce-scatter from it), so scalar syncs (boost_from_average, distributed bin
// finding, metric sums) need no second transport.
// Reference counterpart: src/network/network.cpp:30-75 (external functions).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "device/hip_common.h"
#include "device/runtime_internal.h"
#include "lgap/device_api.h"
#include "lgap/network.h"

namespace lgap {
namespace device {

namespace {

struct CommState {
  ncclComm_t comm = nullptr;
  int rank = 0;
  int size = 1;
  int device = 0;
  hipStream_t stream = nullptr;
  char* dev_buf = nullptr;
  size_t dev_cap = 0;
  std::mutex mu;
};

CommState& S() {
  static CommState s;
  return s;
}

void NcclCheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) Log::Fatal("RCCL error in %s: %s", what, ncclGetErrorString(r));
}

char* Staging(size_t bytes) {
  auto& s = S();
  if (bytes > s.dev_cap) {
    if (s.dev_buf) HIP_CHECK(hipFree(s.dev_buf));
    s.dev_cap = std::max<size_t>(bytes, 1 << 20);
    HIP_CHECK(hipMalloc(&s.dev_buf, s.dev_cap));
  }
  return s.dev_buf;
}

// Equal-size allgather of `bytes` per rank from host memory into host memory.
void HostAllgatherEqual(const char* in, size_t bytes, char* out) {
  auto& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  HIP_CHECK(hipSetDevice(s.device));
  char* d = Staging(bytes * (s.size + 1));
  char* d_in = d + bytes * s.size;
  HIP_CHECK(hipMemcpyAsync(d_in, in, bytes, hipMemcpyHostToDevice, s.stream));
  NcclCheck(ncclAllGather(d_in, d, bytes, ncclChar, s.comm, s.stream), "ncclAllGather");
  HIP_CHECK(hipMemcpyAsync(out, d, bytes * s.size, hipMemcpyDeviceToHost, s.stream));
  HIP_CHECK(hipStreamSynchronize(s.stream));
}

// Network external allgather: variable blocks, padded to the largest block.
void RcclAllgather(char* input, comm_size_t input_size, const comm_size_t* block_start, const comm_size_t* block_len,
                   int num_block, char* output, comm_size_t output_size) {
  (void)input_size;
  (void)output_size;
  comm_size_t mx = 0;
  for (int i = 0; i < num_block; ++i) mx = std::max(mx, block_len[i]);
  if (mx == 0) return;
  std::vector<char> pad(mx, 0), all(static_cast<size_t>(mx) * num_block);
  std::memcpy(pad.data(), input, block_len[S().rank]);
  HostAllgatherEqual(pad.data(), mx, all.data());
  for (int i = 0; i < num_block; ++i) {
    std::memcpy(output + block_start[i], all.data() + static_cast<size_t>(i) * mx, block_len[i]);
  }
}

std::string ToHex(const char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = d[(static_cast<unsigned char>(p[i]) >> 4) & 15];
    s[2 * i + 1] = d[static_cast<unsigned char>(p[i]) & 15];
  }
  return s;
}

int HexVal(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  Log::Fatal("Invalid hex digit in RCCL unique id");
  return 0;
}

}  // namespace

int DeviceCount() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

size_t DeviceTotalMemory() {
  if (DeviceCount() <= 0) return 0;
  size_t free_b = 0, total_b = 0;
  HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
  return total_b;
}

void DeviceSynchronize() {
  if (DeviceCount() > 0) HIP_CHECK(hipDeviceSynchronize());
}

std::string CommGetUniqueId() {
  ncclUniqueId id;
  NcclCheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return ToHex(id.internal, sizeof(id.internal));
}

void CommInit(const std::string& unique_id, int num_ranks, int rank, int device_id) {
  auto& s = S();
  if (s.comm) CommFree();
  if (unique_id.size() != 2 * sizeof(ncclUniqueId().internal)) Log::Fatal("Malformed RCCL unique id");
  ncclUniqueId id;
  for (size_t i = 0; i < sizeof(id.internal); ++i) {
    id.internal[i] = static_cast<char>(HexVal(unique_id[2 * i]) * 16 + HexVal(unique_id[2 * i + 1]));
  }
  s.device = device_id;
  HIP_CHECK(hipSetDevice(device_id));
  HIP_CHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  NcclCheck(ncclCommInitRank(&s.comm, num_ranks, id, rank), "ncclCommInitRank");
  s.rank = rank;
  s.size = num_ranks;
  // host collectives ride on the same communicator unless a socket mesh exists
  if (Network::num_machines() <= 1 && num_ranks > 1) {
    // allgather only: Network derives reduce-scatter from it (the path the torch.distributed
    // transport exercises in the multi-rank CPU tests)
    Network::Init(num_ranks, rank, nullptr, RcclAllgather);
  }
  Log::Info("RCCL communicator ready: rank %d / %d on device %d", rank, num_ranks, device_id);
}

void CommFree() {
  auto& s = S();
  if (s.comm) {
    (void)ncclCommDestroy(s.comm);
    s.comm = nullptr;
  }
  if (s.stream) {
    (void)hipStreamDestroy(s.stream);
    s.stream = nullptr;
  }
  if (s.dev_buf) {
    (void)hipFree(s.dev_buf);
    s.dev_buf = nullptr;
    s.dev_cap = 0;
  }
  s.rank = 0;
  s.size = 1;
}

int CommRank() { return S().rank; }
int CommSize() { return S().size; }
bool CommActive() { return S().comm != nullptr && S().size > 1; }
bool CommExists() { return S().comm != nullptr; }
ncclComm_t ActiveComm() { return S().comm; }
int CommDevice() { return S().device; }

bool HostStagedDP() {
  static const bool on = [] {
    const char* e = std::getenv("LGAP_DEVICE_DP_TRANSPORT");
    return e != nullptr && std::strcmp(e, "host") == 0;
  }();
  return on && S().comm == nullptr && Network::num_machines() > 1;
}

template <typename T>
void AllreduceSum(T* dev_ptr, size_t count, hipStream_t stream, ncclDataType_t type) {
  if (count == 0) return;
  if (HostStagedDP()) {
    // Rehearsal transport (several ranks sharing one GPU, host Network underneath):
    // device -> pinned host -> Network allreduce -> device. Not for production runs.
    thread_local std::vector<T> h;
    h.resize(count);
    HIP_CHECK(hipMemcpyAsync(h.data(), dev_ptr, count * sizeof(T), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    Network::Allreduce(reinterpret_cast<char*>(h.data()), static_cast<comm_size_t>(count * sizeof(T)), sizeof(T),
                       reinterpret_cast<char*>(h.data()), Network::SumReducer<T>());
    HIP_CHECK(hipMemcpyAsync(dev_ptr, h.data(), count * sizeof(T), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  // a one-rank communicator still runs the collective (single-GPU rehearsal of the DP path)
  if (!CommExists()) return;
  NcclCheck(ncclAllReduce(dev_ptr, dev_ptr, count, type, ncclSum, S().comm, stream), "ncclAllReduce");
}

void AllreduceSumF64(double* dev_ptr, size_t count, hipStream_t stream) {
  AllreduceSum(dev_ptr, count, stream, ncclFloat64);
}

void AllreduceSumF32(float* dev_ptr, size_t count, hipStream_t stream) {
  AllreduceSum(dev_ptr, count, stream, ncclFloat32);
}

void AllreduceSumU64(unsigned long long* dev_ptr, size_t count, hipStream_t stream) {
  AllreduceSum(dev_ptr, count, stream, ncclUint64);
}

void AllreduceMaxU32(unsigned* dev_ptr, size_t count, hipStream_t stream) {
  if (count == 0) return;
  if (HostStagedDP()) {
    std::vector<unsigned> h(count);
    HIP_CHECK(hipMemcpyAsync(h.data(), dev_ptr, count * sizeof(unsigned), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    for (auto& v : h) v = static_cast<unsigned>(Network::GlobalSyncUpByMax(static_cast<double>(v)));
    HIP_CHECK(hipMemcpyAsync(dev_ptr, h.data(), count * sizeof(unsigned), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  if (!CommExists()) return;
  NcclCheck(ncclAllReduce(dev_ptr, dev_ptr, count, ncclUint32, ncclMax, S().comm, stream), "ncclAllReduce(max)");
}

int DpSize() { return Network::num_machines() > 1 ? Network::num_machines() : std::max(1, S().size); }
int DpRank() { return Network::num_machines() > 1 ? Network::rank() : S().rank; }

// Owner reduce-scatter of the data-parallel histogram: `send` holds DpSize() blocks of
// `count` elements (block r = the bins rank r owns); `recv` gets this rank's block summed
// over ranks (reference data_parallel_tree_learner.cpp:284-297, HistogramSumReducer).
void ReduceScatterSum(const void* send, void* recv, size_t count, bool f64, hipStream_t stream) {
  if (count == 0) return;
  const size_t es = f64 ? sizeof(double) : sizeof(float);
  if (HostStagedDP()) {
    const int n = Network::num_machines();
    thread_local std::vector<char> h, o;
    h.resize(es * count * n);
    o.resize(es * count);
    HIP_CHECK(hipMemcpyAsync(h.data(), send, h.size(), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    std::vector<comm_size_t> start(n), len(n, static_cast<comm_size_t>(es * count));
    for (int i = 0; i < n; ++i) start[i] = static_cast<comm_size_t>(es * count * i);
    Network::ReduceScatter(h.data(), static_cast<comm_size_t>(h.size()), static_cast<int>(es), start.data(),
                           len.data(), o.data(), static_cast<comm_size_t>(o.size()),
                           f64 ? Network::SumReducer<double>() : Network::SumReducer<float>());
    HIP_CHECK(hipMemcpyAsync(recv, o.data(), o.size(), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  if (!CommExists()) {
    HIP_CHECK(hipMemcpyAsync(recv, send, es * count, hipMemcpyDeviceToDevice, stream));
    return;
  }
  NcclCheck(ncclReduceScatter(send, recv, count, f64 ? ncclFloat64 : ncclFloat32, ncclSum, S().comm, stream),
            "ncclReduceScatter");
}

// Reduce-scatter of exact 64-bit integer sums (the data-parallel frontier's fixed-point
// accumulators): `send` = DpSize() chunks of `count` words, `recv` = this rank's chunk summed.
void ReduceScatterSumU64(const unsigned long long* send, unsigned long long* recv, size_t count, hipStream_t stream) {
  if (count == 0) return;
  if (HostStagedDP()) {
    const int n = Network::num_machines();
    thread_local std::vector<char> h, o;
    h.resize(sizeof(uint64_t) * count * n);
    o.resize(sizeof(uint64_t) * count);
    HIP_CHECK(hipMemcpyAsync(h.data(), send, h.size(), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    std::vector<comm_size_t> start(n), len(n, static_cast<comm_size_t>(sizeof(uint64_t) * count));
    for (int i = 0; i < n; ++i) start[i] = static_cast<comm_size_t>(sizeof(uint64_t) * count * i);
    Network::ReduceScatter(h.data(), static_cast<comm_size_t>(h.size()), static_cast<int>(sizeof(uint64_t)), start.data(),
                           len.data(), o.data(), static_cast<comm_size_t>(o.size()), Network::SumReducer<uint64_t>());
    HIP_CHECK(hipMemcpyAsync(recv, o.data(), o.size(), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  if (!CommExists()) {
    HIP_CHECK(hipMemcpyAsync(recv, send, sizeof(uint64_t) * count, hipMemcpyDeviceToDevice, stream));
    return;
  }
  NcclCheck(ncclReduceScatter(send, recv, count, ncclUint64, ncclSum, S().comm, stream), "ncclReduceScatter(u64)");
}

// In-place allgather: `buf` holds DpSize() blocks of `bytes` each, this rank's block filled.
void AllGatherInPlace(void* buf, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return;
  if (HostStagedDP()) {
    const int n = Network::num_machines(), r = Network::rank();
    thread_local std::vector<char> h;
    h.resize(bytes * n);
    char* mine = h.data() + bytes * r;
    HIP_CHECK(hipMemcpyAsync(mine, static_cast<char*>(buf) + bytes * r, bytes, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    std::vector<char> in(mine, mine + bytes);
    Network::Allgather(in.data(), static_cast<comm_size_t>(bytes), h.data());
    HIP_CHECK(hipMemcpyAsync(buf, h.data(), h.size(), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  if (!CommExists() || S().size <= 1) return;
  char* base = static_cast<char*>(buf);
  NcclCheck(ncclAllGather(base + bytes * S().rank, base, bytes, ncclChar, S().comm, stream), "ncclAllGather");
}

// xGMI peer mapping (collective over the DpSize() ranks): every rank exports `local`
// (one allocation of identical size and layout on every rank) with hipIpcGetMemHandle,
// the handles are all-gathered over the host collectives, and each rank maps its peers'
// buffers. Returns false on every rank when any rank failed (the caller then keeps the
// collective transport); no HIP error is fatal here.
bool XgmiOpen(char* local, std::vector<char*>* peers) {
  const int n = DpSize(), r = DpRank();
  struct Rec {
    int ok, pad;
    hipIpcMemHandle_t h;
  };
  Rec mine;
  std::memset(&mine, 0, sizeof(mine));
  mine.ok = hipIpcGetMemHandle(&mine.h, local) == hipSuccess ? 1 : 0;
  if (!mine.ok) (void)hipGetLastError();
  std::vector<Rec> all(n);
  if (n > 1) {
    Network::Allgather(reinterpret_cast<char*>(&mine), sizeof(Rec), reinterpret_cast<char*>(all.data()));
  } else {
    all[0] = mine;
  }
  int ok = 1;
  for (const Rec& x : all) ok &= x.ok;
  peers->assign(n, nullptr);
  for (int q = 0; q < n && ok; ++q) {
    if (q == r) {
      (*peers)[q] = local;
      continue;
    }
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, all[q].h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      ok = 0;
    } else {
      (*peers)[q] = static_cast<char*>(p);
    }
  }
  if (n > 1) ok = Network::GlobalSyncUpByMin(ok);
  if (!ok) XgmiClose(local, peers);
  return ok != 0;
}

void XgmiClose(char* local, std::vector<char*>* peers) {
  for (char* p : *peers) {
    if (p != nullptr && p != local) (void)hipIpcCloseMemHandle(p);
  }
  peers->clear();
}

// Collective watchdog (the reference only has socket timeouts; a lost
// worker hangs its peers). Waits for `stream` while polling the communicator's
// asynchronous error state; on an RCCL error, or when the wait outlives
// `timeout_s` (a peer stopped joining the collectives, so the RCCL kernels on
// this stream wait forever), the communicator is aborted — which releases
// those kernels — and the failure is raised as a fatal error on this rank.
void WatchedStreamSync(hipStream_t stream, double timeout_s, const char* what) {
  auto& s = S();
  if (s.comm == nullptr) {  // (a one-rank communicator is watched too: the rehearsal path)
    HIP_CHECK(hipStreamSynchronize(stream));
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (long long polls = 0;; ++polls) {
    const hipError_t r = hipStreamQuery(stream);
    if (r == hipSuccess) return;
    if (r != hipErrorNotReady) HIP_CHECK(r);
    ncclResult_t ae = ncclSuccess;
    if (ncclCommGetAsyncError(s.comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      (void)ncclCommAbort(s.comm);
      s.comm = nullptr;
      Log::Fatal("RCCL asynchronous error during %s on rank %d: %s", what, s.rank, ncclGetErrorString(ae));
    }
    if ((polls & 255) == 0 && timeout_s > 0) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) {
        (void)ncclCommAbort(s.comm);
        s.comm = nullptr;
        Log::Fatal("%s did not finish within %.1f s on rank %d: a peer stopped joining the collectives; "
                   "RCCL communicator aborted",
                   what, timeout_s, s.rank);
      }
    }
    // spin for the first milliseconds (a tree takes a few), then back off
    if (polls > 4096) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

double CommTimeoutSeconds(int time_out_minutes) {
  const char* e = std::getenv("LGAP_COMM_TIMEOUT_S");
  if (e != nullptr && *e != '\0') return std::atof(e);
  return 60.0 * std::max(1, time_out_minutes);
}

}  // namespace device
}  // namespace lgap
